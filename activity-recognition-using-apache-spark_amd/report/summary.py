"""Run summary: the reference's hand-curated results, generated.

The reference's authors copied one run's numbers by hand into Excel
(``Main/wisdm_main_ver_0.0/main_result/Results.xls``: per classifier the count,
correct / wrong predictions, their ratios, F1, accuracy, training and "testing"
time, plus an LR vs LR+CV table), charted them in ``Graph.xlsx`` / ``Graph.pdf``
(PREDICTION, PREDICTION RATIO, ACCURACY, LR vs LR-CV, pie charts of training and
testing time) and published the notebook as a static page (``docs/index.html``)
— SURVEY.md C30/C31.  ``write_report`` produces all of that from the
``main.py`` records of one run:

* ``Results.csv`` / ``Results.md`` — the Results.xls table (one row per model);
* ``LR_vs_LRCV.csv`` — the comparison block, when both models ran;
* ``prediction.png``, ``prediction_ratio.png``, ``accuracy.png``,
  ``lr_vs_lrcv.png``, ``training_time.png``, ``testing_time.png`` — the Graph.pdf
  charts (Agg backend, no display needed);
* ``index.html`` — one self-contained page (charts inlined as base64 PNG) with the
  table, the charts, the per-phase timings and the full ``result.txt`` log.
"""
from __future__ import annotations

import base64
import csv
import html
import io
import os
from typing import Dict, List

DISPLAY = {"lr": "Logistic Regression", "lrcv": "Logistic Regression (5-fold CV)", "dt": "Decision Tree",
           "dtcv": "Decision Tree (5-fold CV)", "rf": "Random Forest", "rfcv": "Random Forest (5-fold CV)",
           "nb": "Naive Bayes", "mlp": "Multilayer Perceptron"}
COLUMNS = ["Classifier", "Count", "Correct", "Wrong", "Correct Ratio", "Wrong Ratio", "F1 Score", "Accuracy",
           "Training Time (s)", "Testing Time (s)"]


def results_rows(summary: Dict) -> List[Dict]:
    rows = []
    for name, r in summary["models"].items():
        rows.append({"Classifier": DISPLAY.get(name, name), "Count": r["count_total"], "Correct": r["correct"],
                     "Wrong": r["wrong"], "Correct Ratio": r["ratio_correct"], "Wrong Ratio": r["ratio_wrong"],
                     "F1 Score": r["f1"], "Accuracy": r["accuracy"], "Training Time (s)": r["train_s"],
                     "Testing Time (s)": r["predict_s"], "_key": name})
    return rows


def _fmt(v):
    return f"{v:.6g}" if isinstance(v, float) else str(v)


def _markdown(rows: List[Dict]) -> str:
    out = ["| " + " | ".join(COLUMNS) + " |", "|" + "---|" * len(COLUMNS)]
    for r in rows:
        out.append("| " + " | ".join(_fmt(r[c]) for c in COLUMNS) + " |")
    return "\n".join(out) + "\n"


def _charts(rows: List[Dict], summary: Dict) -> Dict[str, bytes]:
    import matplotlib

    matplotlib.use("Agg")
    import matplotlib.pyplot as plt

    names = [r["Classifier"] for r in rows]
    figs = {}

    def save(name, fig):
        buf = io.BytesIO()
        fig.tight_layout()
        fig.savefig(buf, format="png", dpi=90)
        plt.close(fig)
        figs[name] = buf.getvalue()

    x = list(range(len(rows)))
    fig, ax = plt.subplots(figsize=(8, 4))
    ax.bar([i - 0.2 for i in x], [r["Correct"] for r in rows], 0.4, label="Correct")
    ax.bar([i + 0.2 for i in x], [r["Wrong"] for r in rows], 0.4, label="Wrong")
    ax.set_xticks(x, names, rotation=20, ha="right", fontsize=8)
    ax.set_title("PREDICTION")
    ax.legend()
    save("prediction.png", fig)

    fig, ax = plt.subplots(figsize=(8, 4))
    ax.bar([i - 0.2 for i in x], [r["Correct Ratio"] for r in rows], 0.4, label="Correct ratio")
    ax.bar([i + 0.2 for i in x], [r["Wrong Ratio"] for r in rows], 0.4, label="Wrong ratio")
    ax.set_xticks(x, names, rotation=20, ha="right", fontsize=8)
    ax.set_title("PREDICTION RATIO")
    ax.legend()
    save("prediction_ratio.png", fig)

    fig, ax = plt.subplots(figsize=(8, 4))
    ax.bar([i - 0.2 for i in x], [r["Accuracy"] for r in rows], 0.4, label="Accuracy")
    ax.bar([i + 0.2 for i in x], [r["F1 Score"] for r in rows], 0.4, label="Weighted F1")
    ax.set_xticks(x, names, rotation=20, ha="right", fontsize=8)
    ax.set_ylim(0, 1)
    ax.set_title("ACCURACY")
    ax.legend()
    save("accuracy.png", fig)

    keys = {r["_key"]: r for r in rows}
    if "lr" in keys and "lrcv" in keys:
        fig, ax = plt.subplots(figsize=(6, 4))
        mets = ["Accuracy", "F1 Score", "Correct Ratio"]
        for j, k in enumerate(("lr", "lrcv")):
            ax.bar([i + (j - 0.5) * 0.4 for i in range(len(mets))], [keys[k][m] for m in mets], 0.4,
                   label=keys[k]["Classifier"])
        ax.set_xticks(range(len(mets)), mets)
        ax.set_ylim(0, 1)
        ax.set_title("LR vs LR-CV")
        ax.legend(fontsize=8)
        save("lr_vs_lrcv.png", fig)

    for col, fname, title in (("Training Time (s)", "training_time.png", "TRAINING TIME"),
                              ("Testing Time (s)", "testing_time.png", "TESTING TIME")):
        vals = [max(float(r[col]), 0.0) for r in rows]
        if sum(vals) <= 0:
            continue
        fig, ax = plt.subplots(figsize=(6, 5))
        ax.pie(vals, labels=names, autopct="%1.1f%%", textprops={"fontsize": 7})
        ax.set_title(title)
        save(fname, fig)
    return figs


def write_report(summary: Dict, out_dir: str, result_txt: str = "") -> List[str]:
    """Write the Results table, the charts and ``index.html`` into ``out_dir``."""
    os.makedirs(out_dir, exist_ok=True)
    rows = results_rows(summary)
    written = []
    p = os.path.join(out_dir, "Results.csv")
    with open(p, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=COLUMNS, extrasaction="ignore")
        w.writeheader()
        w.writerows(rows)
    written.append(p)
    md = _markdown(rows)
    p = os.path.join(out_dir, "Results.md")
    with open(p, "w") as f:
        f.write(md)
    written.append(p)
    keys = {r["_key"]: r for r in rows}
    if "lr" in keys and "lrcv" in keys:
        p = os.path.join(out_dir, "LR_vs_LRCV.csv")
        with open(p, "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["Metric", keys["lr"]["Classifier"], keys["lrcv"]["Classifier"]])
            for m in ("Accuracy", "F1 Score", "Correct", "Wrong", "Training Time (s)", "Testing Time (s)"):
                w.writerow([m, keys["lr"][m], keys["lrcv"][m]])
        written.append(p)
    figs = _charts(rows, summary) if rows else {}
    for name, data in figs.items():
        p = os.path.join(out_dir, name)
        with open(p, "wb") as f:
            f.write(data)
        written.append(p)
    # self-contained page (the docs/index.html analogue)
    table = ["<table><tr>" + "".join(f"<th>{html.escape(c)}</th>" for c in COLUMNS) + "</tr>"]
    for r in rows:
        table.append("<tr>" + "".join(f"<td>{html.escape(_fmt(r[c]))}</td>" for c in COLUMNS) + "</tr>")
    table.append("</table>")
    imgs = "".join(f'<figure><img src="data:image/png;base64,{base64.b64encode(d).decode()}" alt="{n}">'
                   f"<figcaption>{html.escape(n)}</figcaption></figure>" for n, d in figs.items())
    phases = "".join(f"<tr><td>{html.escape(k)}</td><td>{v:.6f}</td></tr>"
                     for k, v in summary.get("phases_s", {}).items())
    page = f"""<!DOCTYPE html>
<html><head><meta charset="utf-8"><title>Human Activity Recognition — run report</title>
<style>body{{font-family:sans-serif;margin:2em;max-width:1100px}} table{{border-collapse:collapse}}
td,th{{border:1px solid #bbb;padding:3px 8px;font-size:13px}} figure{{display:inline-block;margin:6px}}
pre{{background:#f5f5f5;padding:1em;font-size:11px;overflow-x:auto}}</style></head><body>
<h1>Human Activity Recognition on WISDM — run report</h1>
<p>Device <b>{html.escape(str(summary.get('device')))}</b>, world size {summary.get('world_size', 1)},
encoding <b>{html.escape(str(summary.get('encoding')))}</b>, {summary.get('n_train')} training /
{summary.get('n_test')} test windows, seed {summary.get('seed')}.</p>
<h2>Results</h2>{''.join(table)}
<h2>Charts</h2>{imgs}
<h2>Phase timings (s, device-synchronized)</h2><table>{phases}</table>
<h2>Run log (result.txt)</h2><pre>{html.escape(result_txt)}</pre>
</body></html>
"""
    p = os.path.join(out_dir, "index.html")
    with open(p, "w") as f:
        f.write(page)
    written.append(p)
    return written
