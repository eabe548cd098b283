"""Interleaved timing of conv weight-gradient paths on model layer shapes, in ONE process: the
shipped path (split-K GEMMs / halo tiles, CXXNET_WGRAD_DIRECT=0 behaviour) against the direct
small-map kernel (ops.gemm.conv_wgrad_direct), each checked against fp32 torch.

  python benchmarks/wgrad_probe.py [--layers alexnet] [--batch 256] [--rounds 7]
"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cxxnet_amd.ops import gemm as G  # noqa: E402
from cxxnet_amd.ops.gemm import ConvGeom  # noqa: E402

# name: (H, W, C, Cout, K, pad, groups)
LAYERS = {
    "alexnet": {"conv3": (13, 13, 256, 384, 3, 1, 1), "conv4": (13, 13, 384, 384, 3, 1, 2),
                "conv5": (13, 13, 384, 256, 3, 1, 2), "conv2": (27, 27, 96, 256, 5, 2, 2)},
}


def _time(fn, iters):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters * 1000.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layers", default="alexnet")
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--splits", default="0", help="split counts of the direct kernel to time (0 = its default)")
    ap.add_argument("--only", default="", help="comma list of layers to run")
    ap.add_argument("--arms", default="", help="comma list of arms to time (shipped, direct_s0, ...)")
    a = ap.parse_args()
    N = a.batch
    for name, (H, W, C, Cout, K, pad, grp) in LAYERS[a.layers].items():
        if a.only and name not in a.only.split(","):
            continue
        g = ConvGeom(N, H, W, C, H, W, Cout, K, K, 1, pad, pad, grp)
        x = torch.randn(N, H, W, C, device="cuda").to(torch.bfloat16)
        dy = torch.randn(N, H, W, Cout, device="cuda").to(torch.bfloat16)
        ref = torch.nn.grad.conv2d_weight(x.float().permute(0, 3, 1, 2), (Cout, C // grp, K, K),
                                          dy.float().permute(0, 3, 1, 2), stride=1, padding=pad, groups=grp)
        flops = 2.0 * N * H * W * Cout * (C // grp) * K * K
        dw = torch.zeros(Cout, K, K, C // grp, device="cuda")

        def shipped():
            G._WGD = "0"
            try:
                G.conv_backward_weight(x, dy, dw, g)
            finally:
                G._WGD = "auto"
        arms = {"shipped": shipped}
        for sp in [int(v) for v in a.splits.split(",")]:
            arms[f"direct_s{sp}"] = (lambda sp=sp: G.conv_wgrad_direct(x, dy, dw, g, splits=sp))
        if a.arms:
            arms = {k: v for k, v in arms.items() if k in a.arms.split(",")}
        errs, ok = {}, {}
        for k, fn in arms.items():
            dw.zero_()
            r = fn()
            torch.cuda.synchronize()
            if r is False:
                ok[k] = False
                continue
            ok[k] = True
            errs[k] = ((dw.permute(0, 3, 1, 2) - ref).norm() / ref.norm()).item()
        times = {k: [] for k in arms if ok[k]}
        for _ in range(a.rounds):
            for k in times:
                times[k].append(_time(arms[k], a.iters))
        rec = {"layer": name, "batch": N, "gflop": flops / 1e9}
        for k in times:
            us = statistics.median(times[k])
            rec[k] = {"us": round(us, 1), "tflops": round(flops / us / 1e6, 1), "rel_err": errs[k]}
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
