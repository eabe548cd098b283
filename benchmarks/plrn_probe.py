"""Fused max-pool -> LRN kernels (ops.pool_lrn_forward / lrn_pool_backward) against the separate
pool + LRN kernels on AlexNet's pool1 / pool2 shapes: median kernel time of each arm (CUDA
events, back-to-back launches).  One JSON line per (shape, arm).
    python benchmarks/plrn_probe.py [--batch 256] [--reps 20]"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cxxnet_amd import ops  # noqa: E402


def timeit(fn, reps):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for _ in range(reps):
        s.record()
        fn()
        e.record()
        e.synchronize()
        ts.append(s.elapsed_time(e) * 1e3)
    return sorted(ts)[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--arms", default="", help="only these arms (comma list)")
    a = ap.parse_args()
    n, alpha, beta, k = 5, 1e-4, 0.75, 1.0
    for name, H, C in (("pool1", 55, 96), ("pool2", 27, 256)):
        N = a.batch
        x = torch.randn(N, H, H, C, device="cuda").clamp_min(0).to(torch.bfloat16)
        Ho = (H - 3) // 2 + 1
        P = torch.empty(N, Ho, Ho, C, device="cuda", dtype=torch.bfloat16)
        st = torch.empty(N, Ho, Ho, C, device="cuda", dtype=torch.uint8)
        Y = torch.empty_like(P)
        dY = torch.randn_like(Y)
        dP = torch.empty_like(P)
        dx = torch.empty_like(x)
        db = torch.zeros(C, device="cuda")
        rows = ops.lrn_pool_backward_rows(x.shape, P.shape, n)
        part = torch.empty(rows, C, device="cuda")
        arms = {
            "fused_fwd": lambda: ops.pool_lrn_forward(x, P, st, Y, 6, n, alpha, beta, k),
            "sep_pool_fwd": lambda: ops.pool_forward(x, P, st, 3, 3, 2, 0, "max", relu=False, mark_mask=True),
            "sep_lrn_fwd": lambda: ops.lrn_forward(P, Y, n, alpha, beta, k),
            "fused_bwd": lambda: ops.lrn_pool_backward(P, dY, st, dx, 1, n, alpha, beta, k),
            "fused_bwd_db": lambda: ops.lrn_pool_backward(P, dY, st, dx, 1, n, alpha, beta, k, dbias=db, part=part),
            "sep_lrn_bwd": lambda: ops.lrn_backward(P, dY, dP, n, alpha, beta, k),
            "sep_pool_bwd": lambda: ops.pool_backward(x, st, dP, dx, 3, 3, 2, 0, "max", relu=2, dbias=db),
        }
        for arm, fn in arms.items():
            if a.arms and arm not in a.arms.split(","):
                continue
            rec = {"shape": name, "arm": arm, "us": round(timeit(fn, a.reps), 1)}
            if os.environ.get("CXN_LRN_POOL_R"):
                rec["R"] = int(os.environ["CXN_LRN_POOL_R"])
            print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
