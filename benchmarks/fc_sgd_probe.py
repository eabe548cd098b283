"""The fc weight-gradient GEMM fused with the SGD step (ops.fc_backward_weight_sgd, table key
"fws") on AlexNet's fc6 / fc7 at batch 256, for each MN-major tile: median time and the
parameter stream rate (18 bytes per parameter: fp32 w and momentum read and written, the bf16
shadow written).  Interleaved rounds in one process.

    python benchmarks/fc_sgd_probe.py [--tiles 1,2,17,23,40,41] [--rounds 7]"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cxxnet_amd import ops  # noqa: E402
from cxxnet_amd.ops import gemm as G  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tiles", default="-1,1,2,17,23,40,41")
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--groups", default="8", help="tile-order groups (ops.gemm.set_tile_group) to A/B")
    ap.add_argument("--flush", type=int, default=0,
                    help="overwrite 1 GB before every timed call (w / m then come from HBM; the fill's dirty lines "
                         "are written back during the call, so times read high)")
    ap.add_argument("--ops", default="fc6,fc7")
    a = ap.parse_args()
    junk = torch.empty(1 << 28, device="cuda") if a.flush else None
    B = a.batch
    for name, nin, nout in (("fc6", 9216, 4096), ("fc7", 4096, 4096), ("fc8", 4096, 1000)):
        if name not in a.ops.split(","):
            continue
        g = torch.Generator(device="cuda").manual_seed(1)
        x = torch.randn(B, nin, device="cuda", generator=g).to(torch.bfloat16)
        dy = torch.randn(B, nout, device="cuda", generator=g).to(torch.bfloat16)
        w = torch.randn(nout, nin, device="cuda", generator=g) * 0.02
        m = torch.zeros(nout, nin, device="cuda")
        wb = w.to(torch.bfloat16)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        arms = [(int(t), int(gi)) for t in a.tiles.split(",") for gi in a.groups.split(",")]
        times = {arm: [] for arm in arms}
        for _ in range(a.rounds):
            for arm in arms:
                t, gi = arm
                G.set_glds(True, t)
                G.set_tile_group(gi)
                assert ops.fc_backward_weight_sgd(x, dy, w, m, wb, 1e-6, 0.0, 0.9, 0.0)
                torch.cuda.synchronize()
                tot = 0.0
                for _ in range(a.iters):
                    if junk is not None:
                        junk.fill_(1.0)
                    s.record()
                    ops.fc_backward_weight_sgd(x, dy, w, m, wb, 1e-6, 0.0, 0.9, 0.0)
                    e.record()
                    e.synchronize()
                    tot += s.elapsed_time(e) * 1e3
                times[arm].append(tot / a.iters)
        G.set_glds(True, -1)
        G.set_tile_group(8)
        rec = {"op": name, "batch": B, "flush": a.flush}
        for (t, gi), v in times.items():
            us = statistics.median(v)
            tag = (f"t{t}" if t >= 0 else "tdef") + f"g{gi}"
            rec[f"{tag}_us"] = round(us, 1)
            rec[f"{tag}_TBps"] = round(18 * nin * nout / us / 1e6, 2)
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
