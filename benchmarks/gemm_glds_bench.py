"""A/B the LDS-DMA GEMM (csrc/kernels/gemm_glds.hip) against the register-staged kernel
(csrc/kernels/gemm_mfma.hip) on every AlexNet (batch 256) GEMM it serves, per tile
variant, and check that the outputs agree.

  python benchmarks/gemm_glds_bench.py [--iters 20] [--ops conv2_fwd,fc6_fwd] > out.jsonl
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cxxnet_amd import ops  # noqa: E402
from cxxnet_amd.ops import gemm as G  # noqa: E402

N = 256
BF = torch.bfloat16
CONV = {"conv1": (4, 227, 96, 11, 4, 0, 1), "conv2": (96, 27, 256, 5, 1, 2, 2), "conv3": (256, 13, 384, 3, 1, 1, 1),
        "conv4": (384, 13, 384, 3, 1, 1, 2), "conv5": (384, 13, 256, 3, 1, 1, 2)}
FC = {"fc6": (9216, 4096), "fc7": (4096, 4096), "fc8": (4096, 1000),
      "sq8192": (8192, 8192), "sq4096": (4096, 4096)}  # square GEMMs (batch = nin): main-loop ceiling
# VGG-16 at batch 64 ("vgg.c3_2_fwd"): 3x3 pad 1 convs (C, H, Cout)
VGG = {"c1_2": (64, 224, 64), "c2_1": (64, 112, 128), "c2_2": (128, 112, 128), "c3_1": (128, 56, 256),
       "c3_2": (256, 56, 256), "c4_1": (256, 28, 512), "c4_2": (512, 28, 512), "c5": (512, 14, 512)}


def timeit(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1000.0


def make(name):
    global N
    N = 256
    if name.startswith("conv:"):  # generic: conv:C:H:Cout:K:stride:pad:groups:N_kind
        layer, kind = name.rsplit("_", 1)
        C, H, Cout, K, st, pd, grp, N = (int(v) for v in layer.split(":")[1:])
        CONV[layer] = (C, H, Cout, K, st, pd, grp)
    elif name.startswith("vgg."):
        layer, kind = name[4:].rsplit("_", 1)
        C, H, Cout = VGG[layer]
        CONV[name] = (C, H, Cout, 3, 1, 1, 1)
        layer = name
        N = 64
    else:
        layer, kind = name.split("_")
    g = torch.Generator(device="cuda").manual_seed(0)
    if layer.startswith("sq"):
        N = FC[layer][0]
    if layer in FC:
        nin, nout = FC[layer]
        x = torch.randn(N, nin, device="cuda", generator=g).to(BF)
        w = (torch.randn(nout, nin, device="cuda", generator=g) * 0.02).to(BF)
        b = torch.randn(nout, device="cuda", generator=g) * 0.1
        y = torch.empty(N, nout, device="cuda", dtype=BF)
        if kind == "dgrad":
            dy = torch.randn(N, nout, device="cuda", generator=g).to(BF)
            dx = torch.empty(N, nin, device="cuda", dtype=BF)
            return (lambda: ops.fc_backward_data(dy, w, dx)), dx, 2.0 * N * nin * nout
        if kind == "wgrad":
            dy = torch.randn(N, nout, device="cuda", generator=g).to(BF)
            dw = torch.empty(nout, nin, device="cuda")
            return (lambda: ops.fc_backward_weight(x, dy, dw, overwrite=True)), dw, 2.0 * N * nin * nout
        return (lambda: ops.fc_forward(x, w, b, y, relu=not layer.startswith("sq"))), y, 2.0 * N * nin * nout
    C, H, Cout, K, s, p, grp = CONV[layer]
    Ho, Wo = G.conv_out_size(H, H, K, K, s, p, p)
    geo = G.ConvGeom(N, H, H, C, Ho, Wo, Cout, K, K, s, p, p, grp)
    w = (torch.randn(Cout, K, K, C // grp, device="cuda", generator=g) * 0.05).to(BF)
    flops = 2.0 * N * Ho * Wo * Cout * (C // grp) * K * K
    if kind == "fwd":
        x = torch.randn(N, H, H, C, device="cuda", generator=g).to(BF)
        b = torch.randn(Cout, device="cuda", generator=g) * 0.1
        y = torch.empty(N, Ho, Wo, Cout, device="cuda", dtype=BF)
        return (lambda: ops.conv_forward(x, w, b, y, geo, relu=True)), y, flops
    dy = torch.randn(N, Ho, Wo, Cout, device="cuda", generator=g).to(BF)
    if kind == "wgrad":
        x = torch.randn(N, H, H, C, device="cuda", generator=g).to(BF)
        dw = torch.zeros(Cout, K, K, C // grp, device="cuda")
        return (lambda: (dw.zero_(), ops.conv_backward_weight(x, dy, dw, geo))), dw, flops
    dx = torch.empty(N, H, H, C, device="cuda", dtype=BF)
    wt = torch.empty_like(w)
    return (lambda: ops.conv_backward_data(dy, w, dx, geo, wt)), dx, flops


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--ops", default="conv1_fwd,conv1_wgrad,conv2_fwd,conv2_dgrad,conv2_wgrad,conv3_fwd,conv3_dgrad,conv3_wgrad,conv4_fwd,"
                                     "conv4_dgrad,conv4_wgrad,conv5_fwd,conv5_dgrad,conv5_wgrad,fc6_fwd,fc6_dgrad,"
                                     "fc6_wgrad,fc7_fwd,fc7_dgrad,fc7_wgrad,fc8_fwd,fc8_dgrad,fc8_wgrad")
    ap.add_argument("--tiles", default="0,1,2,7,10,13,15,17")
    a = ap.parse_args()
    for name in a.ops.replace(";", ",").split(","):
        run, out, flops = make(name)
        G.set_glds(False)
        run()
        torch.cuda.synchronize()
        ref = out.float().clone()
        t_old = timeit(run, a.iters)
        rec = {"op": name, "old_us": round(t_old, 1), "old_tflops": round(flops / t_old / 1e6, 1)}
        for t in [int(v) for v in a.tiles.split(",")]:
            G.set_glds(True, t)
            out.zero_()
            run()
            torch.cuda.synchronize()
            err = ((out.float() - ref).abs().max() / ref.abs().max().clamp_min(1e-6)).item()
            us = timeit(run, a.iters)
            rec[f"t{t}_us"] = round(us, 1)
            rec[f"t{t}_err"] = round(err, 4)
        G.set_glds(True, -1)
        rec["auto_us"] = round(timeit(run, a.iters), 1)
        rec["auto_tflops"] = round(flops / rec["auto_us"] / 1e6, 1)
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
