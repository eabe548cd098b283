"""Memory-bound kernels of the AlexNet step at batch 256, timed in isolation
(CUDA events), with the bytes each one must move and the achieved bandwidth.

  python benchmarks/membound.py [--iters 20]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cxxnet_amd import ops  # noqa: E402
from cxxnet_amd.io.data import U8Images  # noqa: E402

N = 256
DEV = "cuda"


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


def report(name, us, nbytes):
    print(json.dumps({"op": name, "us": round(us, 1), "MB": round(nbytes / 1e6, 1),
                      "TB_s": round(nbytes / us / 1e6, 2)}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    bf = torch.bfloat16
    it = a.iters

    # input normalisation
    pix = torch.randint(0, 256, (N, 227, 227, 3), dtype=torch.uint8, device=DEV)
    img = U8Images(pix, torch.zeros((N, 4), dtype=torch.int32, device=DEV), torch.tensor([[1.0, 0.0]] * N, device=DEV),
                   torch.tensor([123.0, 117.0, 104.0], device=DEV), 1, 1.0)
    out = torch.empty((N, 227, 227, 4), dtype=bf, device=DEV)
    report("image_u8_to_nhwc", timeit(lambda: ops.image_to_nhwc(img, out), it), pix.numel() + out.numel() * 2)
    xf = torch.randn(N, 3, 227, 227, device=DEV)
    report("nchw_f32_to_nhwc", timeit(lambda: ops.input_to_nhwc(xf, out), it), xf.numel() * 4 + out.numel() * 2)

    # pooling (pool1 / pool2 / pool5 of AlexNet) fwd / bwd, with and without the folded bias grad
    for name, (H, C) in {"pool1": (55, 96), "pool2": (27, 256), "pool5": (13, 256)}.items():
        Ho = ops.pool_out_size(H, 3, 2, 0)
        x = torch.randn(N, H, H, C, device=DEV).to(bf).clamp_min(0)
        y = torch.empty(N, Ho, Ho, C, dtype=bf, device=DEV)
        st = torch.empty(N, Ho, Ho, C, dtype=torch.uint8, device=DEV)
        dy = torch.randn(N, Ho, Ho, C, device=DEV).to(bf)
        dx = torch.empty_like(x)
        db = torch.zeros(C, device=DEV)
        big = x.numel() * 2
        small = y.numel() * 3
        report(f"{name}_fwd", timeit(lambda: ops.pool_forward(x, y, st, 3, 3, 2, 0, "max", False, mark_mask=True), it),
               big + small)
        report(f"{name}_bwd", timeit(lambda: ops.pool_backward(x, st, dy, dx, 3, 3, 2, 0, "max", 2), it), big + small)
        report(f"{name}_bwd_bias", timeit(lambda: ops.pool_backward(x, st, dy, dx, 3, 3, 2, 0, "max", 2, dbias=db),
                                          it), big + small)
        report(f"{name}_colsum", timeit(lambda: ops.bias_grad(dx.view(-1, C), db), it), big)

    # LRN on pool1 / pool2 outputs
    for name, (H, C) in {"lrn1": (27, 96), "lrn2": (13, 256)}.items():
        x = torch.randn(N, H, H, C, device=DEV).to(bf)
        y = torch.empty_like(x)
        dy = torch.randn_like(x)
        dx = torch.empty_like(x)
        report(f"{name}_fwd", timeit(lambda: ops.lrn_forward(x, y, 5, 0.001, 0.75, 1.0), it), x.numel() * 4)
        report(f"{name}_bwd", timeit(lambda: ops.lrn_backward(x, dy, dx, 5, 0.001, 0.75, 1.0), it), x.numel() * 6)

    # fused optimizer over AlexNet's 61M parameters
    n = 60_965_224
    w = torch.randn(n, device=DEV)
    g = torch.randn(n, device=DEV)
    m = torch.zeros(n, device=DEV)
    wb = torch.empty(n, dtype=bf, device=DEV)
    segs = [(0, n, 0.01, 0.0005, 0.9, 0.0)]
    report("fused_update_sgd", timeit(lambda: ops.fused_update("sgd", w, g, m, None, wb, segs, zero_grad=False), it),
           n * 22)


if __name__ == "__main__":
    main()
