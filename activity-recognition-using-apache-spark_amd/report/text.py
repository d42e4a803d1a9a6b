"""``result.txt`` writer in the reference's section format.

The reference redirects ``sys.stdout`` to ``main_result/result.txt`` and prints
banner-separated sections (``Main/main.py:11-12, 27-43, 49-100, 133-195`` and the
five evaluation copies; the committed log is ``result.txt``).  ``RunLog`` keeps
the same banners and line formats (``%g`` numbers) so existing tooling that
parses the log keeps working.  Differences, on purpose: the "Mean Squared Error"
line prints the MSE (the reference prints the RMSE twice, ``main.py:171``), and the
"Prediction made in" time is real device-synchronized inference time (the
reference times Spark's lazy plan construction, ``main.py:121-123``).
"""
from __future__ import annotations

import io
import sys
from typing import Optional, TextIO

from ..evaluation.evaluators import MetricsRecord

BANNER_PIPELINE = "\n===========================MODELING PIPELINE==============================\n"
BANNER_TRAIN = "\n===========================TRAINING AND TESTING==============================\n"
BANNER_CLASSIFY = "============================CLASSIFICATION AND EVALUATION============================"


class RunLog:
    """Tee of everything the run prints: the result file and (optionally) stdout."""

    def __init__(self, path: Optional[str] = None, echo: bool = False):
        self.path = path
        self.buf = io.StringIO()
        self.echo = echo
        self._f: Optional[TextIO] = open(path, "w") if path else None

    def print(self, *args, **kw):
        s = io.StringIO()
        print(*args, file=s, **kw)
        txt = s.getvalue()
        self.buf.write(txt)
        if self._f:
            self._f.write(txt)
            self._f.flush()
        if self.echo:
            sys.stdout.write(txt)

    def close(self):
        if self._f:
            self._f.close()
            self._f = None

    def text(self) -> str:
        return self.buf.getvalue()


# dash counts of the reference's banners (main.py:27,29,34,42,74,76)
_DASHES = {"Activity Count": 58, "Summary": 63}


def section(log: RunLog, title: str):
    log.print(title + "-" * _DASHES.get(title, 60))


def model_header(log: RunLog, model_str: str, train_s: float, predict_s: float):
    log.print(model_str)
    log.print("Classifier trained in %g seconds" % train_s)
    log.print("Prediction made in %g seconds" % predict_s)


def evaluation_block(log: RunLog, r: MetricsRecord):
    log.print("\n-----------Binary Classification Evaluator-------------\n")
    log.print("Binary Classifier Raw Prediction ------------: %g" % r.raw_prediction)
    log.print("Binary Clasifier Area Under PR --------------: %g" % r.area_under_pr)
    log.print("Binary Clasifier Area Under ROC -------------: %g" % r.area_under_roc)
    log.print("\n-----------MultiClass Classification Evaluaton---------\n")
    log.print("MultiClass F1 -------------------------------: %g" % r.f1)
    log.print("MultiClass Weighted Precision ---------------: %g" % r.weighted_precision)
    log.print("MultiClass Weighted Recall ------------------: %g" % r.weighted_recall)
    log.print("MultiClass Accuracy -------------------------: %g" % r.accuracy)
    log.print("\n----------------Regression Evaluator-------------------\n")
    log.print("Root Mean Squared Error (RMSE) on test data -: %g" % r.rmse)
    log.print("Mean Squared Error on test data -------------: %g" % r.mse)
    log.print("R^2 metric on test data ---------------------: %g" % r.r2)
    log.print("Mean Absolute Error on test data ------------: %g" % r.mae)
    log.print("\n------------------Additional Factors--------------------\n")
    log.print("Total Count          = %g" % r.count_total)
    log.print("Total Correct        = %g" % r.correct)
    log.print("Total Wrong          = %g" % r.wrong)
    log.print("Wrong Ratio          = %g" % r.ratio_wrong)
    log.print("Right Ratio          = %g" % r.ratio_correct)
    log.print("\n*********************************************************\n")
