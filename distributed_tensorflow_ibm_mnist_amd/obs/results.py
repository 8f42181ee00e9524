"""Classification result writer — replacement for DLI's
``inference_helper.writeClassificationResult`` (``inference.py:103-110``; the
module is not in the repository [DLI]).

Two call forms, as at the reference call sites:
* validate mode: ``writeClassificationResult(path, imagenames, prediction,
  ground_truth=labels)`` → per-image top-1 + correctness, overall accuracy;
* prediction mode: ``writeClassificationResult(path, imagenames, prediction,
  prob_thresh=0.5, label_file=...)`` → per-image classes whose probability is
  ≥ ``prob_thresh`` (always at least the top-1), named via ``label_file``.

Output: ``path`` as JSON (``.json`` or no extension) plus a sibling ``.csv``.
"""
from __future__ import annotations

import csv
import json
import os
from typing import List, Optional, Sequence

import numpy as np


def read_label_file(path: Optional[str], n: int) -> List[str]:
    if path and os.path.exists(path):
        names = [l.strip() for l in open(path) if l.strip()]
        if len(names) >= n:
            return names[:n]
    return [str(i) for i in range(n)]


def writeClassificationResult(path: str, imagenames: Sequence, prediction: np.ndarray, ground_truth=None,
                              prob_thresh: float = 0.5, label_file: Optional[str] = None) -> dict:
    prediction = np.asarray(prediction, dtype=np.float64)
    n, k = prediction.shape if prediction.ndim == 2 else (0, 10)
    names = read_label_file(label_file, k)
    top = prediction.argmax(1) if n else np.zeros(0, dtype=int)
    rows = []
    for i in range(n):
        name = imagenames[i]
        name = name.decode() if isinstance(name, bytes) else str(name)
        r = {"image": name, "prediction": int(top[i]), "label": names[int(top[i])],
             "probability": float(prediction[i, top[i]])}
        if ground_truth is not None:
            gt = int(ground_truth[i])
            r["ground_truth"] = gt
            r["correct"] = bool(gt == int(top[i]))
        else:
            keep = [j for j in np.argsort(-prediction[i]) if prediction[i, j] >= prob_thresh] or [int(top[i])]
            r["classes"] = [{"label": names[j], "index": int(j), "probability": float(prediction[i, j])}
                            for j in keep]
        rows.append(r)
    summary = {"count": n}
    if ground_truth is not None and n:
        summary["accuracy"] = float(np.mean([r["correct"] for r in rows]))
    out = {"summary": summary, "results": rows}
    os.makedirs(os.path.dirname(os.path.abspath(path)) or ".", exist_ok=True)
    jpath = path if path.endswith(".json") else path + ".json" if not os.path.splitext(path)[1] else path
    with open(jpath, "w") as f:
        json.dump(out, f, indent=1)
    with open(os.path.splitext(jpath)[0] + ".csv", "w", newline="") as f:
        w = csv.writer(f)
        hdr = ["image", "prediction", "label", "probability"] + (["ground_truth", "correct"]
                                                                if ground_truth is not None else [])
        w.writerow(hdr)
        for r in rows:
            w.writerow([r[h] for h in hdr])
    return out
