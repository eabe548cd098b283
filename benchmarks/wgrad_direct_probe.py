"""Time the direct weight-gradient kernel (csrc/kernels/conv_wgrad_direct.hip) per AlexNet /
VGG op over split counts (0: the kernel's own choice), one process, interleaved rounds.

    python benchmarks/wgrad_direct_probe.py [--ops conv3,conv4,conv5] [--splits 0,4,8,12,16]"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cxxnet_amd.ops import gemm  # noqa: E402
from cxxnet_amd.ops.gemm import ConvGeom  # noqa: E402

# name -> (N, H, C, Cout, K, pad, groups)
OPS = {
    "conv2": (256, 27, 96, 256, 5, 2, 2),
    "conv3": (256, 13, 256, 384, 3, 1, 1),
    "conv4": (256, 13, 384, 384, 3, 1, 2),
    "conv5": (256, 13, 384, 256, 3, 1, 2),
    "vgg_c5": (64, 14, 512, 512, 3, 1, 1),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ops", default="conv3,conv4,conv5")
    ap.add_argument("--splits", default="0,4,6,8,12,16")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    res = {}
    for name in a.ops.split(","):
        N, H, C, Cout, K, pad, G = OPS[name]
        g = ConvGeom(N, H, H, C, H, H, Cout, K, K, 1, pad, pad, G)
        x = torch.randn(N, H, H, C, device="cuda").to(torch.bfloat16)
        dy = torch.randn(N, H, H, Cout, device="cuda").to(torch.bfloat16)
        dw = torch.zeros(Cout, K, K, C // G, device="cuda")
        db = torch.zeros(Cout, device="cuda") if K == 3 else None
        flop = 2.0 * N * H * H * Cout * K * K * (C // G)
        for _ in range(a.rounds):
            for sp in a.splits.split(","):
                sp = int(sp)
                assert gemm.conv_wgrad_direct(x, dy, dw, g, splits=sp, db=db)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                torch.cuda.synchronize()
                e0.record()
                for _ in range(a.iters):
                    gemm.conv_wgrad_direct(x, dy, dw, g, splits=sp, db=db)
                e1.record()
                e1.synchronize()
                res.setdefault((name, sp), []).append(e0.elapsed_time(e1) * 1e3 / a.iters)
        for sp in a.splits.split(","):
            ts = sorted(res[(name, int(sp))])
            t = ts[len(ts) // 2]
            print(json.dumps({"op": name, "splits": int(sp), "us": round(t, 1), "tflops": round(flop / t / 1e6, 1)}),
                  flush=True)


if __name__ == "__main__":
    main()
