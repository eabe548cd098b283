"""MetricSet over the native metrics (reference src/utils/metric.h:182-236)."""
from __future__ import annotations

from typing import Dict, List

import numpy as np
import torch

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


class DeviceMetricSet:
    """Training / evaluation metrics accumulated ON THE DEVICE (reference semantics of
    src/utils/metric.h:20-236: error = first-max argmax != label[0] (a 1-wide score is
    thresholded at 0), logloss = -log(clamp(p[label], 1e-15, 1-1e-15)) (binary form for a
    1-wide score), rmse = mean over instances of the squared-error SUM (no sqrt, as the
    reference), rec@n = fraction of an instance's labels found in its top-n scores).

    Every add_eval enqueues a few tiny kernels on the current stream and adds into a float64
    accumulator; nothing is copied to the host until print(), which (under data
    parallelism) all-reduces the sums and counts once.  The reference instead copies every
    eval node to the host every step and reduces there (nnet_impl-inl.hpp:174-180).
    Deviation: rec@n breaks exact score ties by the lowest index (kernel and fallback alike)
    where the reference shuffles before sorting; ties between float softmax scores are
    measure-zero."""

    KINDS = ("error", "logloss", "rmse")

    def __init__(self):
        self.names: List[str] = []
        self.fields: List[str] = []
        self._sum = None
        self._cnt = None

    def add_metric(self, name: str, field: str = "label"):
        if name not in self.KINDS and not name.startswith("rec@"):
            raise ValueError(f"unknown metric type {name}")
        if name.startswith("rec@"):
            int(name[4:])
        self.names.append(name)
        self.fields.append(field)

    def __len__(self):
        return len(self.names)

    def _acc(self, device):
        if self._sum is None or self._sum.device != device:
            self._sum = torch.zeros(len(self.names), dtype=torch.float64, device=device)
            self._cnt = [0] * len(self.names)  # instance counts are known on the host
        return self._sum, self._cnt

    def clear(self):
        if self._sum is not None:
            self._sum.zero_()
            self._cnt = [0] * len(self.names)

    _KIND = {"error": 0, "logloss": 1}

    def _kernel_ok(self, i) -> bool:
        n = self.names[i]
        return n in self._KIND or n.startswith("rec@")

    def _run_kernel(self, lo, hi, p, lab, b):
        """metrics lo..hi-1 share scores p and labels lab: one metric_rows + one
        metric_accum launch (csrc/kernels/nn_kernels.hip) add their sums into the float64
        accumulator."""
        import ctypes
        from .. import native
        from ..ops.gemm import _stream
        nm = hi - lo
        kinds = (ctypes.c_int * nm)(*[self._KIND.get(n, 2) for n in self.names[lo:hi]])
        args = (ctypes.c_int * nm)(*[int(n[4:]) if n.startswith("rec@") else 0 for n in self.names[lo:hi]])
        K = p.shape[1]
        for n in self.names[lo:hi]:
            if n.startswith("rec@") and K < int(n[4:]):
                raise ValueError(f"it is meaningless to take rec@n for list shorter than n, evaluating {n}, "
                                 f"list={K}")
        if getattr(self, "_part", None) is None or self._part.device != p.device:
            self._part = torch.empty(256 * 8, dtype=torch.float32, device=p.device)
        native.check(native.kernels().cxn_metric_eval(
            p.data_ptr(), p.stride(0), lab.data_ptr(), lab.stride(0), lab.shape[1], b, K, nm, kinds, args,
            self._sum.data_ptr() + 8 * lo, self._part.data_ptr(), _stream()), "metric_eval")

    @staticmethod
    def _one(name: str, p: torch.Tensor, lab: torch.Tensor) -> torch.Tensor:
        K = p.shape[1]
        if name == "error":
            idx = p.argmax(1) if K != 1 else (p[:, 0] > 0).long()
            return (idx != lab[:, 0].long()).sum()
        if name == "logloss":
            if K != 1:
                v = p.gather(1, lab[:, :1].long()).clamp(1e-15, 1.0 - 1e-15)
                return -v.log().sum()
            py = p[:, 0].clamp(1e-15, 1.0 - 1e-15)
            y = lab[:, 0]
            return -(y * py.log() + (1.0 - y) * (1.0 - py).log()).sum()
        if name == "rmse":
            if lab.shape[1] != K:
                raise ValueError("Metric: In RMSE metric, the size of prediction and label must be same.")
            return ((p - lab) ** 2).sum()
        n = int(name[4:])
        if K < n:
            raise ValueError(f"it is meaningless to take rec@n for list shorter than n, evaluating rec@{n}, "
                             f"list={K}")
        # rank of each distinct label: scores larger, or equal at a lower index (the kernel's
        # tie rule, so at most n labels hit); hit if rank < n
        L = lab.long()
        valid = (L >= 0) & (L < K)
        Lc = L.clamp(0, K - 1)
        s = p.gather(1, Lc)                                              # (B, lw)
        idx = torch.arange(K, device=p.device).view(1, 1, K)
        pe = p.unsqueeze(1)                                              # (B, 1, K)
        rank = ((pe > s.unsqueeze(2)) | ((pe == s.unsqueeze(2)) & (idx < Lc.unsqueeze(2)))).sum(2)
        first = torch.ones_like(valid)
        for c in range(1, L.shape[1]):                                   # duplicates count once
            first[:, c] = (L[:, :c] != L[:, c:c + 1]).all(1)
        hit = (rank < n) & valid & first
        return hit.float().sum() / lab.shape[1]

    def add_eval(self, preds: List[torch.Tensor], label_fields: Dict[str, torch.Tensor], rows: int = None):
        """preds[i]: (B, K) scores of metric i's node (device tensor); label_fields: device
        label slices; rows: only the first `rows` instances count (padded batch tail)."""
        if len(preds) != len(self.names):
            raise ValueError("Metric: Number of predict scores and number of metrics should be equal.")
        if not preds:
            return
        acc, cnt = self._acc(preds[0].device)
        i, nm = 0, len(self.names)
        while i < nm:
            f = self.fields[i]
            if f not in label_fields:
                raise ValueError(f"Metric: unknown target = {f}")
            lab = label_fields[f]
            p = preds[i].reshape(preds[i].shape[0], -1)
            lab = lab.reshape(lab.shape[0], -1)
            b = p.shape[0] if rows is None else max(0, min(rows, p.shape[0]))
            # a run of metrics on the same scores and labels
            j = i + 1
            while j < nm and j - i < 8 and preds[j] is preds[i] and self.fields[j] == f:
                j += 1
            if p.is_cuda and p.dtype == torch.float32 and lab.dtype == torch.float32 and \
                    all(self._kernel_ok(q) for q in range(i, j)) and p.stride(1) == 1 and lab.stride(1) == 1:
                if b:
                    self._run_kernel(i, j, p, lab, b)
            else:
                for q in range(i, j):
                    if b:
                        acc[q:q + 1].add_(self._one(self.names[q], p[:b].float(), lab[:b].float()).double())
            for q in range(i, j):
                cnt[q] += b
            i = j

    def values(self, group_reduce=None) -> List[float]:
        if self._sum is None:
            return [float("nan")] * len(self.names)
        both = torch.cat([self._sum, torch.tensor(self._cnt, dtype=torch.float64).to(self._sum.device)])
        if group_reduce is not None:
            both = group_reduce(both)
        both = both.cpu()
        n = len(self.names)
        return [(both[i] / both[n + i]).item() if both[n + i] > 0 else float("nan") for i in range(n)]

    def print(self, evname: str, group_reduce=None) -> str:
        out = []
        for name, f, v in zip(self.names, self.fields, self.values(group_reduce)):
            s = f"\t{evname}-{name}"
            if f != "label":
                s += f"[{f}]"
            out.append(f"{s}:{v:g}")
        return "".join(out)
