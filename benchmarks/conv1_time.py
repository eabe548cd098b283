"""Time AlexNet conv1 forward (3-channel 228-pixel-row input, b256) on the direct row-run
kernel (conv_rowrun.hip), median of rounds.  python benchmarks/conv1_time.py [--rounds 9]"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=9)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--arms", default="new", help="comma list of arms (new: conv_rowrun.hip)")
    a = ap.parse_args()
    from cxxnet_amd import native
    from cxxnet_amd.ops import gemm as G
    N, H, W, C, Cout, K, S = a.batch, 227, 228, 3, 96, 11, 4
    Ho, Wo = 55, 55
    x = torch.randn(N, H, W, C, device="cuda").to(torch.bfloat16)
    w = (torch.randn(Cout, K, K, C, device="cuda") * 0.05).to(torch.bfloat16)
    b = torch.randn(Cout, device="cuda")
    g = G.ConvGeom(N, H, W, C, Ho, Wo, Cout, K, K, S, 0, 0, 1)
    wp, lp = G._row_padded_weights(w, g)
    y = torch.empty(N, Ho, Wo, Cout, device="cuda", dtype=torch.bfloat16)
    k = native.kernels()

    def run(fn):
        rc = fn(x.data_ptr(), x.numel() * 2, wp.data_ptr(), b.data_ptr(), y.data_ptr(), N, H, W, C,
                                   Ho, Wo, Cout, K, lp, S, Cout, 1, torch.cuda.current_stream().cuda_stream)
        assert rc == 0, rc
    fns = {"new": k.cxn_conv_rowrun_fwd}
    arms = a.arms.split(",")
    outs = {}
    for arm in arms:
        run(fns[arm])
        torch.cuda.synchronize()
        outs[arm] = y.float().clone()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = {arm: [] for arm in arms}
    for _ in range(a.rounds):
        for arm in arms:
            s.record()
            for _ in range(a.iters):
                run(fns[arm])
            e.record()
            e.synchronize()
            ts[arm].append(s.elapsed_time(e) / a.iters * 1000)
    flops = 2.0 * N * Ho * Wo * Cout * K * K * C
    rec = {"op": "conv1_rowrun_fwd", "batch": N}
    for arm in arms:
        us = statistics.median(ts[arm])
        rec[f"{arm}_us"] = round(us, 1)
        rec[f"{arm}_tflops"] = round(flops / us / 1e6, 1)
    if len(arms) > 1:
        rec["max_abs_diff"] = (outs[arms[0]] - outs[arms[1]]).abs().max().item()
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
