"""Time the direct small-map conv kernels (csrc/kernels/conv_direct.hip) against the implicit-GEMM
path the tile table picks, per AlexNet op at a given batch (one process, interleaved rounds).

  python benchmarks/conv_direct_probe.py [--batch 256] [--iters 20] [--rounds 3]

Prints one JSON line per (op, path) with the median time in us and TFLOP/s.
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cxxnet_amd.ops import gemm  # noqa: E402
from cxxnet_amd.ops.gemm import ConvGeom  # noqa: E402

# name -> (H, C, Cout, K, pad, groups)
OPS = {
    "conv2": (27, 96, 256, 5, 2, 2),
    "conv3": (13, 256, 384, 3, 1, 1),
    "conv4": (13, 384, 384, 3, 1, 2),
    "conv5": (13, 384, 256, 3, 1, 2),
    # VGG-16 conv5_x (batch 64) and GoogLeNet inception 4c / 4e 3 x 3 (batch 128)
    "vgg_c5": (14, 512, 512, 3, 1, 1),
    "goog_4c": (14, 128, 256, 3, 1, 1),
    "goog_4e": (14, 160, 320, 3, 1, 1),
}


def _time(fn, iters):
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(iters):
        ev[0].record()
        fn()
        ev[1].record()
        ev[1].synchronize()
        ts.append(ev[0].elapsed_time(ev[1]) * 1e3)
    ts.sort()
    return ts[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--ops", default="conv3,conv4,conv5")
    ap.add_argument("--paths", default="table,200,201,202,203",
                    help="tile ids to force (200-202: the direct kernel's schedules) or 'table' (the shipped pick)")
    ap.add_argument("--dirs", default="fwd,dgrad")
    a = ap.parse_args()
    dev = "cuda"
    res = {}
    for name in a.ops.split(","):
        H, C, Cout, K, pad, G = OPS[name]
        N = a.batch
        g = ConvGeom(N, H, H, C, H, H, Cout, K, K, 1, pad, pad, G)
        x = torch.randn(N, H, H, C, device=dev).to(torch.bfloat16)
        w = (torch.randn(Cout, K, K, C // G, device=dev) * 0.05).to(torch.bfloat16)
        b = torch.zeros(Cout, device=dev)
        y = torch.empty(N, H, H, Cout, device=dev, dtype=torch.bfloat16)
        wt = torch.empty_like(w)
        gemm.conv_weight_flip_multi([(w, wt, g)])
        dx = torch.relu(torch.randn(N, H, H, C, device=dev)).to(torch.bfloat16)
        db = torch.zeros(C, device=dev)
        flop = 2.0 * N * H * H * Cout * K * K * (C // G)
        fns = {
            "fwd": lambda: gemm.conv_forward(x, w, b, y, g, relu=True),
            "dgrad": lambda: gemm.conv_backward_data(y, w, dx, g, wt_buf=wt, mask_relu=True, wt_ready=True,
                                                     dbias=db),
        }
        for r in range(a.rounds):
            for op, fn in fns.items():
                if op not in a.dirs.split(","):
                    continue
                for path in a.paths.split(","):
                    gemm._glds_cfg["tile"] = -1 if path == "table" else int(path)
                    t = _time(fn, a.iters)
                    res.setdefault((name, op, path), []).append(t)
    gemm._glds_cfg["tile"] = -1
    for (name, op, path), ts in res.items():
        H, C, Cout, K, pad, G = OPS[name]
        flop = 2.0 * a.batch * H * H * Cout * K * K * (C // G)
        t = sorted(ts)[len(ts) // 2]
        print(json.dumps({"op": f"{name}_{op}", "path": path, "batch": a.batch, "us": round(t, 1),
                          "tflops": round(flop / t / 1e6, 1), "rounds_us": [round(v, 1) for v in ts]}))


if __name__ == "__main__":
    main()
