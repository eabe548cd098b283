"""Per-kernel timing of the hand-written HIP kernels on AlexNet shapes (batch 256)
against the vendor path PyTorch-ROCm would use (MIOpen conv / hipBLASLt GEMM), both bf16.

Usage: python benchmarks/bench_kernels.py [--batch 256] [--iters 20]
Prints one JSON line per op: {"op", "ours_ms", "torch_ms", "tflops_ours", "tflops_torch"}.
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
    return s.elapsed_time(e) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    N = a.batch
    dev = "cuda"
    bf = torch.bfloat16
    convs = [("conv1", 4, 227, 96, 11, 4, 0, 1), ("conv2", 96, 27, 256, 5, 1, 2, 2),
             ("conv3", 256, 13, 384, 3, 1, 1, 1), ("conv4", 384, 13, 384, 3, 1, 1, 2),
             ("conv5", 384, 13, 256, 3, 1, 1, 2)]
    for name, C, H, Cout, K, s, p, g in convs:
        Ho, Wo = conv_out_size(H, H, K, K, s, p, p)
        geo = ConvGeom(N, H, H, C, Ho, Wo, Cout, K, K, s, p, p, g)
        x = torch.randn(N, H, H, C, device=dev).to(bf)
        w = (torch.randn(Cout, K, K, C // g, device=dev) * 0.05).to(bf)
        b = torch.zeros(Cout, device=dev)
        y = torch.empty(N, Ho, Wo, Cout, device=dev, dtype=bf)
        dw = torch.zeros(Cout, K, K, C // g, device=dev)
        dx = torch.empty_like(x)
        wt = torch.empty_like(w)
        flops = 2.0 * N * Ho * Wo * Cout * K * K * (C // g)
        t_f = timeit(lambda: ops.conv_forward(x, w, b, y, geo, relu=True), a.iters)
        t_w = timeit(lambda: ops.conv_backward_weight(x, y, dw, geo), a.iters)
        t_d = timeit(lambda: ops.conv_backward_data(y, w, dx, geo, wt), a.iters) if name != "conv1" else float("nan")
        # vendor reference: channels_last bf16 conv via MIOpen
        xt = x.permute(0, 3, 1, 2)
        wt_ = w.permute(0, 3, 1, 2).contiguous(memory_format=torch.channels_last)
        xt.requires_grad_(True)
        wt_.requires_grad_(True)
        out = F.conv2d(xt, wt_, None, s, p, 1, g)
        go = torch.randn_like(out)
        r_f = timeit(lambda: F.conv2d(xt, wt_, None, s, p, 1, g), a.iters)
        r_b = timeit(lambda: torch.autograd.grad(F.conv2d(xt, wt_, None, s, p, 1, g), (xt, wt_), go), a.iters) - r_f
        ours_b = t_w + (0 if name == "conv1" else t_d)
        print(json.dumps({"op": name, "fwd_ms": round(t_f, 4), "wgrad_ms": round(t_w, 4), "dgrad_ms": round(t_d, 4),
                          "torch_fwd_ms": round(r_f, 4), "torch_bwd_ms": round(r_b, 4),
                          "tflops_fwd": round(flops / t_f / 1e9, 1), "tflops_wgrad": round(flops / t_w / 1e9, 1),
                          "tflops_dgrad": round(flops / t_d / 1e9, 1) if t_d == t_d else None,
                          "ours_total_ms": round(t_f + ours_b, 4), "torch_total_ms": round(r_f + r_b, 4)}),
              flush=True)
    for name, nin, nout in [("fc6", 9216, 4096), ("fc7", 4096, 4096), ("fc8", 4096, 1000)]:
        x = torch.randn(N, nin, device=dev).to(bf)
        w = (torch.randn(nout, nin, device=dev) * 0.02).to(bf)
        b = torch.zeros(nout, device=dev)
        y = torch.empty(N, nout, device=dev, dtype=bf)
        dx = torch.empty_like(x)
        dw = torch.zeros(nout, nin, device=dev)
        flops = 2.0 * N * nin * nout
        t_f = timeit(lambda: ops.fc_forward(x, w, b, y), a.iters)
        t_d = timeit(lambda: ops.fc_backward_data(y, w, dx), a.iters)
        t_w = timeit(lambda: ops.fc_backward_weight(x, y, dw), a.iters)
        r_f = timeit(lambda: F.linear(x, w, None), a.iters)
        r_d = timeit(lambda: y @ w, a.iters)
        r_w = timeit(lambda: y.t() @ x, a.iters)
        print(json.dumps({"op": name, "fwd_ms": round(t_f, 4), "dgrad_ms": round(t_d, 4), "wgrad_ms": round(t_w, 4),
                          "torch_fwd_ms": round(r_f, 4), "torch_dgrad_ms": round(r_d, 4),
                          "torch_wgrad_ms": round(r_w, 4),
                          "tflops_fwd": round(flops / t_f / 1e9, 1), "tflops_dgrad": round(flops / t_d / 1e9, 1),
                          "tflops_wgrad": round(flops / t_w / 1e9, 1)}), flush=True)


if __name__ == "__main__":
    main()
