"""Every AlexNet (batch 256) GEMM-shaped op: our MFMA kernel vs the vendor
libraries on the same shape (MIOpen conv via F.conv2d channels-last bf16 and
hipBLASLt via torch.mm for the GEMM-equivalent problem).  Prints one JSON line
per op with microseconds and TFLOP/s.

  python benchmarks/gemm_ceiling.py [--iters 20]
"""
import argparse
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cxxnet_amd import ops  # noqa: E402
from cxxnet_amd.ops.gemm import ConvGeom, conv_out_size  # noqa: E402

N = 256
# conv1 as the model runs it: 3 channels on rows padded to 228 pixels (NeuralNet._pad_input_channels)
PHYS_W = {"conv1": 228}
CONVS = {"conv1": (3, 227, 96, 11, 4, 0, 1), "conv2": (96, 27, 256, 5, 1, 2, 2), "conv3": (256, 13, 384, 3, 1, 1, 1),
         "conv4": (384, 13, 384, 3, 1, 1, 2), "conv5": (384, 13, 256, 3, 1, 1, 2)}
FCS = {"fc6": (9216, 4096), "fc7": (4096, 4096), "fc8": (4096, 1000)}
# VGG-16 (batch 64): the distinct 3x3 / pad 1 conv shapes (C, H, Cout) and its fc layers
VGG_CONVS = {"c1_1": (4, 224, 64), "c1_2": (64, 224, 64), "c2_1": (64, 112, 128), "c2_2": (128, 112, 128),
             "c3_1": (128, 56, 256), "c3_2": (256, 56, 256), "c4_1": (256, 28, 512), "c4_2": (512, 28, 512),
             "c5": (512, 14, 512)}
VGG_FCS = {"fc6": (25088, 4096), "fc7": (4096, 4096), "fc8": (4096, 1000)}


def timeit(fn, iters):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1000.0 / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--model", default="alexnet", choices=["alexnet", "vgg16"])
    ap.add_argument("--batch", type=int, default=0)
    ap.add_argument("--no-lib", action="store_true")
    ap.add_argument("--fc-only", action="store_true")
    a = ap.parse_args()
    global N, CONVS, FCS
    if a.model == "vgg16":
        N = a.batch or 64
        CONVS = {k: (c, h, co, 3, 1, 1, 1) for k, (c, h, co) in VGG_CONVS.items()}
        FCS = VGG_FCS
    elif a.batch:
        N = a.batch
    bf = torch.bfloat16
    dev = "cuda"
    for name, (C, H, Cout, K, s, p, g) in ({} if a.fc_only else CONVS).items():
        Wp = PHYS_W.get(name, H) if a.model == "alexnet" else H
        Ho, Wo = conv_out_size(H, Wp, K, K, s, p, p)
        geo = ConvGeom(N, H, Wp, C, Ho, Wo, Cout, K, K, s, p, p, g)
        x = torch.randn(N, H, Wp, C, device=dev).to(bf)
        w = (torch.randn(Cout, K, K, C // g, device=dev) * 0.05).to(bf)
        y = torch.randn(N, Ho, Wo, Cout, device=dev).to(bf)
        dw = torch.zeros(Cout, K, K, C // g, device=dev)
        wt = torch.empty_like(w)
        flop = 2.0 * N * Ho * Wo * Cout * K * K * (C // g)
        xn = x.permute(0, 3, 1, 2)  # channels-last NCHW view
        wn = w.permute(0, 3, 1, 2).contiguous(memory_format=torch.channels_last)
        yn = y.permute(0, 3, 1, 2)
        res = {
            "fwd": (lambda: ops.conv_forward(x, w, None, y, geo),
                    lambda: F.conv2d(xn, wn, None, s, p, 1, g)),
            "dgrad": (lambda: ops.conv_backward_data(y, w, x, geo, wt),
                      lambda: torch.nn.grad.conv2d_input(xn.shape, wn, yn, s, p, 1, g)),
            "wgrad": (lambda: ops.conv_backward_weight(x, y, dw, geo),
                      lambda: torch.nn.grad.conv2d_weight(xn, wn.shape, yn, s, p, 1, g)),
        }
        for kind, (ours, lib) in res.items():
            if name in ("conv1", "c1_1") and kind == "dgrad":
                continue
            t0 = timeit(ours, a.iters)
            try:
                t1 = timeit(lib, a.iters) if not a.no_lib else float("nan")
            except Exception as ex:  # noqa: BLE001
                t1 = float("nan")
                print("lib failed", name, kind, ex, file=sys.stderr)
            print(json.dumps({"model": a.model, "batch": N, "op": f"{name}_{kind}", "ours_us": round(t0, 1), "lib_us": round(t1, 1),
                              "ours_tflops": round(flop / t0 / 1e6, 1), "lib_tflops": round(flop / t1 / 1e6, 1)}),
                  flush=True)
    for name, (nin, nout) in FCS.items():
        x = torch.randn(N, nin, device=dev).to(bf)
        w = (torch.randn(nout, nin, device=dev) * 0.02).to(bf)
        y = torch.empty(N, nout, device=dev, dtype=bf)
        dy = torch.randn(N, nout, device=dev).to(bf)
        dx = torch.empty(N, nin, device=dev, dtype=bf)
        dw = torch.zeros(nout, nin, device=dev)
        flop = 2.0 * N * nin * nout
        res = {
            "fwd": (lambda: ops.fc_forward(x, w, None, y), lambda: torch.mm(x, w.t())),
            "dgrad": (lambda: ops.fc_backward_data(dy, w, dx), lambda: torch.mm(dy, w)),
            "wgrad": (lambda: ops.fc_backward_weight(x, dy, dw, overwrite=True), lambda: torch.mm(dy.t(), x)),
        }
        for kind, (ours, lib) in res.items():
            t0 = timeit(ours, a.iters)
            t1 = timeit(lib, a.iters) if not a.no_lib else float("nan")
            print(json.dumps({"model": a.model, "batch": N, "op": f"{name}_{kind}", "ours_us": round(t0, 1), "lib_us": round(t1, 1),
                              "ours_tflops": round(flop / t0 / 1e6, 1), "lib_tflops": round(flop / t1 / 1e6, 1)}),
                  flush=True)
    if a.no_lib:
        return
    # plain large GEMM: the library's best case on this box
    m = k = n = 8192
    A = torch.randn(m, k, device=dev).to(bf)
    B = torch.randn(k, n, device=dev).to(bf)
    t = timeit(lambda: torch.mm(A, B), a.iters)
    print(json.dumps({"op": "hipblaslt_8192^3", "lib_us": round(t, 1), "lib_tflops": round(2.0 * m * n * k / t / 1e6, 1)}))


if __name__ == "__main__":
    main()
