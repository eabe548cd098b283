"""AlexNet conv1 (11x11 / 4, 96 outputs, batch 256) on 3-channel NHWC input against the 4-channel
(NHWC4) layout: the kernel-row runs are 33 elements (5 16-byte chunks, K = 11 x 40 = 440, 7 K-tiles)
instead of 44 (6 chunks, K = 528, 9 K-tiles).  With C = 3 an image row is 227 * 6 bytes and an
output-pixel step 24 bytes, so the runs' 16-byte LDS-DMA loads start at 2-byte-aligned addresses
(`--align 2`) or, with the width padded to 228, at 8-byte-aligned ones (`--pad-w`).

  CXXNET_ROWRUN_ALIGN=2 python benchmarks/conv1_c3_probe.py [--pad-w]

Checks forward and weight-gradient against fp32 torch and prints one JSON line per variant."""
import argparse
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cxxnet_amd.ops import gemm as G  # noqa: E402
from cxxnet_amd.ops.gemm import ConvGeom  # noqa: E402


TILES = []


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1e3


def rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


def case(N, C, Wp, out):
    dev = "cuda"
    H = W = 227
    torch.manual_seed(0)
    x3 = torch.randn(N, 3, H, W, device=dev)
    w3 = torch.randn(96, 3, 11, 11, device=dev) * 0.05
    dy = torch.randn(N, 96, 55, 55, device=dev)
    xb = x3.to(torch.bfloat16).float()
    wb = w3.to(torch.bfloat16).float()
    dyb = dy.to(torch.bfloat16).float()
    y_ref = F.conv2d(xb, wb, stride=4)
    dw_ref = torch.nn.grad.conv2d_weight(xb, wb.shape, dyb, stride=4)
    x = torch.zeros(N, H, Wp, C, device=dev, dtype=torch.bfloat16)
    x[:, :, :W, :3] = x3.permute(0, 2, 3, 1).to(torch.bfloat16)
    w = torch.zeros(96, 11, 11, C, device=dev, dtype=torch.bfloat16)
    w[..., :3] = w3.permute(0, 2, 3, 1).to(torch.bfloat16)
    g = ConvGeom(N, H, Wp, C, 55, 55, 96, 11, 11, 4, 0, 0, 1)
    y = torch.empty(N, 55, 55, 96, device=dev, dtype=torch.bfloat16)
    G.conv_forward(x, w, None, y, g)
    dyn = dy.permute(0, 2, 3, 1).contiguous().to(torch.bfloat16)
    dw = torch.zeros(96, 11, 11, C, device=dev)
    G.conv_backward_weight(x, dyn, dw, g)
    torch.cuda.synchronize()
    ef = rel(y.permute(0, 3, 1, 2), y_ref)
    ew = rel(dw[..., :3].permute(0, 3, 1, 2), dw_ref)
    tf = timeit(lambda: G.conv_forward(x, w, None, y, g))
    tw = timeit(lambda: G.conv_backward_weight(x, dyn, dw, g))
    for t in TILES:
        G._TUNE["|".join(str(v) for v in ("cr", N, H, Wp, C, 96, 11, 11, 4))] = t
        y.zero_()
        G.conv_forward(x, w, None, y, g)
        torch.cuda.synchronize()
        e = rel(y.permute(0, 3, 1, 2), y_ref)
        us = timeit(lambda: G.conv_forward(x, w, None, y, g))
        r = {"C": C, "W_phys": Wp, "fwd_tile": t, "fwd_us": round(us, 1), "fwd_rel_err": e}
        print(json.dumps(r), flush=True)
        out.write(json.dumps(r) + "\n")
    rec = {"C": C, "W_phys": Wp, "align": G.ROWRUN_ALIGN, "rowrun": G.rowrun_ok(g), "fwd_us": round(tf, 1),
           "wgrad_us": round(tw, 1), "fwd_rel_err": ef, "wgrad_rel_err": ew}
    print(json.dumps(rec), flush=True)
    out.write(json.dumps(rec) + "\n")
    return ef < 2e-2 and ew < 2e-2


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--tiles", default="", help="also time these forward tiles (comma list)")
    ap.add_argument("--out", default="gpurun_out/conv1_c3_probe.jsonl")
    a = ap.parse_args()
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    TILES[:] = [int(t) for t in a.tiles.split(",") if t]
    ok = True
    with open(a.out, "a") as out:
        ok &= case(a.batch, 4, 227, out)
        for wp in (227, 228):
            try:
                ok &= case(a.batch, 3, wp, out)
            except (RuntimeError, ValueError) as e:
                print(json.dumps({"C": 3, "W_phys": wp, "error": str(e)[:200]}), flush=True)
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
