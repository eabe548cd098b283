"""Interleaved A/B of GEMM tiles on chosen shapes, in ONE process (cdna guide rule 24): each
round times every tile once, the median over rounds is reported, and every tile's output is
checked against the register-staged kernel.  For square shapes hipBLASLt (torch.mm, same
operands) is timed in the same rounds.

  python benchmarks/gemm_tile_probe.py --ops sq8192_fwd,vgg.c4_2_fwd --tiles 21,34,90,91 [--rounds 7]
"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from gemm_glds_bench import make  # noqa: E402
from cxxnet_amd.ops import gemm as G  # noqa: E402


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
    ap.add_argument("--ops", default="sq8192_fwd")
    ap.add_argument("--tiles", default="21,90,91", help="tile ids; -1 = the shipped table's choice")
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--groups", default="0", help="tile-order groups to A/B (ops.gemm.set_tile_group), e.g. 0,8")
    a = ap.parse_args()
    tiles = [int(t) for t in a.tiles.split(",")]
    for name in a.ops.split(","):
        run, out, flops = make(name)
        G.set_glds(False)
        run()
        torch.cuda.synchronize()
        ref = out.float().clone()
        arms = {}
        errs = {}
        groups = [int(x) for x in a.groups.split(",")]
        for t in tiles:
            for gi in groups:
                G.set_glds(True, t)
                G.set_tile_group(gi)
                out.zero_()
                run()
                torch.cuda.synchronize()
                tag = (f"t{t}" if t >= 0 else "tdef") + (f"g{gi}" if len(groups) > 1 else "")
                errs[tag] = ((out.float() - ref).norm() / ref.norm().clamp_min(1e-6)).item()
                arms[tag] = (lambda t=t, gi=gi: (G.set_glds(True, t), G.set_tile_group(gi), run()))
        if name.startswith("sq"):
            n = int(name[2:].split("_")[0])
            g = torch.Generator(device="cuda").manual_seed(1)
            x = torch.randn(n, n, device="cuda", generator=g).to(torch.bfloat16)
            w = torch.randn(n, n, device="cuda", generator=g).to(torch.bfloat16)
            arms["hipblaslt"] = lambda: torch.mm(x, w.t())
        times = {k: [] for k in arms}
        for _ in range(a.rounds):
            for k, fn in arms.items():
                times[k].append(_time(fn, a.iters))
        rec = {"op": name}
        for k, v in times.items():
            us = statistics.median(v)
            rec[f"{k}_us"] = round(us, 1)
            rec[f"{k}_tflops"] = round(flops / us / 1e6, 1)
        rec["err"] = {t: round(e, 5) for t, e in errs.items()}
        G.set_glds(True, -1)
        G.set_tile_group(0)
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
