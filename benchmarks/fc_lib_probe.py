"""fc GEMMs: our LDS-DMA / register kernels vs hipBLASLt (torch.mm) with bf16 output and with
fp32 output + our finalize epilogue (bias, relu, relu'-mask -> bf16), the form a library fc
path needs to keep the fused epilogue's arithmetic.  One JSON line per (model, batch, layer, op).

  python benchmarks/fc_lib_probe.py [--iters 30]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cxxnet_amd import native, ops  # noqa: E402

SHAPES = [("alexnet", 256, {"fc6": (9216, 4096), "fc7": (4096, 4096), "fc8": (4096, 1000)}),
          ("alexnet", 32, {"fc6": (9216, 4096), "fc7": (4096, 4096), "fc8": (4096, 1000)}),
          ("vgg16", 64, {"fc6": (25088, 4096), "fc7": (4096, 4096), "fc8": (4096, 1000)})]


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
    ap.add_argument("--iters", type=int, default=30)
    a = ap.parse_args()
    bf = torch.bfloat16
    K = native.kernels()
    st = lambda: torch.cuda.current_stream().cuda_stream  # noqa: E731
    for model, B, fcs in SHAPES:
        for name, (nin, nout) in fcs.items():
            x = torch.randn(B, nin, device="cuda").to(bf)
            w = (torch.randn(nout, nin, device="cuda") * 0.02).to(bf)
            bias = torch.randn(nout, device="cuda")
            y = torch.empty(B, nout, device="cuda", dtype=bf)
            dy = torch.randn(B, nout, device="cuda").to(bf)
            dx = torch.randn(B, nin, device="cuda").to(bf)
            wsf = torch.empty(B, nout, device="cuda")
            wsd = torch.empty(B, nin, device="cuda")
            flop = 2.0 * B * nin * nout

            def lib32_fwd():
                torch.mm(x, w.t(), out_dtype=torch.float32, out=wsf)
                K.cxn_splitk_finalize(wsf.data_ptr(), 1, wsf.numel(), y.data_ptr(), B, nout, bias.data_ptr(), 1, 0,
                                      st())

            def lib32_dgrad():
                torch.mm(dy, w, out_dtype=torch.float32, out=wsd)
                K.cxn_splitk_finalize(wsd.data_ptr(), 1, wsd.numel(), dx.data_ptr(), B, nin, None, 0, 1, st())

            rows = {
                "fwd": (lambda: ops.fc_forward(x, w, bias, y, relu=True), lambda: torch.mm(x, w.t(), out=y), lib32_fwd),
                "dgrad": (lambda: ops.fc_backward_data(dy, w, dx, mask_relu=True), lambda: torch.mm(dy, w, out=dx),
                          lib32_dgrad),
            }
            # correctness of the fp32-out forms against fp32 torch
            ref = torch.relu(x.float() @ w.float().t() + bias)
            lib32_fwd()
            err_f = ((y.float() - ref).norm() / ref.norm()).item()
            for op, (ours, lib16, lib32) in rows.items():
                t0, t1, t2 = timeit(ours, a.iters), timeit(lib16, a.iters), timeit(lib32, a.iters)
                print(json.dumps({"model": model, "batch": B, "op": f"{name}_{op}", "ours_us": round(t0, 1),
                                  "lib_bf16_us": round(t1, 1), "lib_f32_fin_us": round(t2, 1),
                                  "ours_tflops": round(flop / t0 / 1e6, 1), "lib_bf16_tflops": round(flop / t1 / 1e6, 1),
                                  "lib_f32_fin_tflops": round(flop / t2 / 1e6, 1),
                                  "fwd_relerr": round(err_f, 5) if op == "fwd" else None}), flush=True)


if __name__ == "__main__":
    main()
