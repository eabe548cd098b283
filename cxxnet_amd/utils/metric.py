"""MetricSet over the native metrics (reference src/utils/metric.h:182-236)."""
from __future__ import annotations

from typing import Dict, List

import numpy as np

from .. import native


class MetricSet:
    def __init__(self):
        self.evals = []
        self.fields: List[str] = []

    def add_metric(self, name: str, field: str = "label"):
        self.evals.append(native.rt().Metric(name))
        self.fields.append(field)

    def clear(self):
        for e in self.evals:
            e.clear()

    def __len__(self):
        return len(self.evals)

    def add_eval(self, preds: List[np.ndarray], label_fields: Dict[str, np.ndarray]):
        if len(preds) != len(self.evals):
            raise ValueError("Metric: Number of predict scores and number of metrics should be equal.")
        for e, f, p in zip(self.evals, self.fields, preds):
            if f not in label_fields:
                raise ValueError(f"Metric: unknown target = {f}")
            lab = label_fields[f]
            p = np.ascontiguousarray(p, dtype=np.float32).reshape(p.shape[0], -1)
            lab = np.ascontiguousarray(lab, dtype=np.float32).reshape(lab.shape[0], -1)
            e.add_eval(p, lab)

    def print(self, evname: str) -> str:
        out = []
        for e, f in zip(self.evals, self.fields):
            s = f"\t{evname}-{e.name}"
            if f != "label":
                s += f"[{f}]"
            out.append(f"{s}:{e.get():g}")
        return "".join(out)
