"""Metric CSVs with the reference's exact headers (``Main/main.py:656-682``;
``main_result/additional_param.csv`` and ``crossFold_additional_param.csv``),
plus a machine-readable ``metrics.jsonl`` per run.

The reference appends a header + rows on every run and, by bug, writes LR's
train/test time into the DT and RF rows (``main.py:665,668``) and labels the CV
rows with the non-CV model uids (``:677,680``).  Here each row carries its own
model's numbers; ``append=True`` reproduces the append-with-header behaviour.
"""
from __future__ import annotations

import csv
import json
import os
from typing import Dict, List

PLAIN_FIELDS = ['Classifier', 'Count Total', 'Correct', 'Wrong', 'Ratio Wrong', 'Ratio Correct', 'F1 Score',
                'Training Time', 'Testing Time', 'Accuracy']
CV_FIELDS = ['Classifier', 'Count Total', 'Correct', 'Wrong', 'Ratio Wrong', 'Ratio Correct', 'F1 Score',
             'Cross Validation Training Time', 'Cross Validation Testing Time', 'Cross Fold Accuracy']


def plain_row(name: str, r, train_s: float, test_s: float) -> Dict:
    return {'Classifier': name, 'Count Total': r.count_total, 'Correct': r.correct, 'Wrong': r.wrong,
            'Ratio Wrong': r.ratio_wrong, 'Ratio Correct': r.ratio_correct, 'F1 Score': r.f1,
            'Training Time': train_s, 'Testing Time': test_s, 'Accuracy': r.accuracy}


def cv_row(name: str, r, train_s: float, test_s: float) -> Dict:
    return {'Classifier': name, 'Count Total': r.count_total, 'Correct': r.correct, 'Wrong': r.wrong,
            'Ratio Wrong': r.ratio_wrong, 'Ratio Correct': r.ratio_correct, 'F1 Score': r.f1,
            'Cross Validation Training Time': train_s, 'Cross Validation Testing Time': test_s,
            'Cross Fold Accuracy': r.accuracy}


def write_rows(path: str, fields: List[str], rows: List[Dict], append: bool = False):
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    with open(path, "a" if append else "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=fields)
        w.writeheader()
        for r in rows:
            w.writerow(r)


def append_jsonl(path: str, record: Dict):
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    with open(path, "a") as f:
        f.write(json.dumps(record) + "\n")
