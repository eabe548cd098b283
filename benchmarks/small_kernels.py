"""A/B of the memory-bound helper kernels on AlexNet b256 shapes (GPU):

  pool_bwd   3x3 stride-2 max-unpool: pool_bwd_s2k3 (2x2 input cells, variant 1) against
             pool_bwd_rows (one input pixel per thread, variant 0); outputs must match bitwise
  colsum     the deferred bias gradients of one AlexNet backward pass (colsum_multi): column-chunk
             split (variant 1) against one block per row range (variant 0), checked against
             an fp32 torch sum

  python benchmarks/small_kernels.py [--iters 50] [--out gpurun_out/small_kernels.jsonl]

Prints one JSON line per (case, variant) with the mean time and the effective HBM rate."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cxxnet_amd import native  # noqa: E402
from cxxnet_amd.ops import nn  # noqa: E402


def timeit(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1e3  # us


def set_variant(which, v):
    native.check(native.kernels().cxn_set_kernel_variant(which, v), "set_kernel_variant")


def pool_case(N, H, C, iters, out):
    dev = "cuda"
    K, S, P = 3, 2, 0
    Ho = nn.pool_out_size(H, K, S, P)
    x = torch.randn(N, H, H, C, device=dev).relu_().to(torch.bfloat16) - 0.1
    x = x.to(torch.bfloat16)
    y = torch.empty(N, Ho, Ho, C, device=dev, dtype=torch.bfloat16)
    st = torch.empty(N, Ho, Ho, C, device=dev, dtype=torch.uint8)
    nn.pool_forward(x, y, st, K, K, S, P, "max", relu=True, mark_mask=True)
    dy = torch.randn_like(y)
    res = {}
    for v in (0, 1):
        set_variant(0, v)
        dx = torch.empty_like(x)
        nn.pool_backward(x, st, dy, dx, K, K, S, P, "max", relu=2)
        torch.cuda.synchronize()
        res[v] = dx
        us = timeit(lambda: nn.pool_backward(x, st, dy, dx, K, K, S, P, "max", relu=2), iters)
        byts = x.numel() * 2 + dy.numel() * 3
        rec = {"case": f"pool_bwd N{N} {H}x{H}x{C}", "variant": v, "us": round(us, 2),
               "TBps": round(byts / us / 1e6, 2)}
        print(json.dumps(rec), flush=True)
        out.write(json.dumps(rec) + "\n")
    set_variant(0, 1)
    same = torch.equal(res[0], res[1])
    print(json.dumps({"case": f"pool_bwd N{N} {H}", "bitwise_equal": same}), flush=True)
    return same


def colsum_case(iters, out):
    dev = "cuda"
    # (rows, C, masked): AlexNet b256 -- conv1/conv2/conv5 through their max-pools (pooled
    # rows, offsets carry relu'), conv3/conv4 plain, fc6/fc7/fc8
    segs = [(256 * 27 * 27, 96, True), (256 * 13 * 13, 256, True), (256 * 13 * 13, 384, False),
            (256 * 13 * 13, 384, False), (256 * 6 * 6, 256, True), (256, 4096, False), (256, 4096, False),
            (256, 1000, False)]
    items, refs = [], []
    for rows, C, m in segs:
        d = torch.randn(rows, C, device=dev).to(torch.bfloat16)
        mk = None
        if m:
            mk = torch.randint(0, 9, (rows, C), device=dev, dtype=torch.uint8)
            mk |= (torch.rand(rows, C, device=dev) < 0.5).to(torch.uint8) * 128
        db = torch.zeros(C, device=dev)
        items.append((d, db, mk))
        dm = d.float() if mk is None else d.float() * (mk < 128).float()
        refs.append(dm.sum(0))
    byts = sum(d.numel() * (3 if m is not None else 2) for d, _, m in items if d.shape[1] % 8 == 0)
    ok = True
    for v in (0, 1):
        set_variant(1, v)
        for _, db, _ in items:
            db.zero_()
        nn.bias_grad_multi(items)
        torch.cuda.synchronize()
        err = max(((db - r).abs().max() / (r.abs().max() + 1e-6)).item() for (_, db, _), r in zip(items, refs))
        ok = ok and err < 1e-3
        us = timeit(lambda: nn.bias_grad_multi(items), iters)
        rec = {"case": "colsum_multi alexnet b256", "variant": v, "us": round(us, 2),
               "TBps": round(byts / us / 1e6, 2), "max_rel_err": err}
        print(json.dumps(rec), flush=True)
        out.write(json.dumps(rec) + "\n")
    set_variant(1, 1)
    return ok


def image_case(iters, out):
    """u8 [B][227][227][3] -> bf16 node: NHWC4 (image_u8c3_nhwc4) vs 3 channels on 228-pixel rows
    (image_u8c3_nhwc3p), mean subtraction (mode 1)."""
    from cxxnet_amd.io.data import U8Images
    B, h, w = 256, 227, 227
    pix = torch.randint(0, 256, (B, h, w, 3), dtype=torch.uint8, device="cuda")
    cm = torch.ones(B, 2, device="cuda")
    cm[:, 1] = 0
    img = U8Images(pix, torch.zeros(B, 4, dtype=torch.int32, device="cuda"), cm,
                   torch.tensor([120.0, 110.0, 100.0], device="cuda"), 1, 1.0)
    for cp, wp in ((4, 227), (3, 228)):
        node = torch.zeros(B, h, wp, cp, dtype=torch.bfloat16, device="cuda")
        us = timeit(lambda: nn.image_to_nhwc(img, node), iters)
        byts = pix.numel() + node.numel() * 2
        rec = {"case": f"image_u8 -> nhwc{cp} row {wp}", "us": round(us, 2), "TBps": round(byts / us / 1e6, 2)}
        print(json.dumps(rec), flush=True)
        out.write(json.dumps(rec) + "\n")
    return True


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--out", default="gpurun_out/small_kernels.jsonl")
    ap.add_argument("--only-image", action="store_true")
    a = ap.parse_args()
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    ok = True
    with open(a.out, "w") as out:
        ok &= image_case(a.iters, out)
        if a.only_image:
            return 0 if ok else 1
        ok &= pool_case(256, 55, 96, a.iters, out)
        ok &= pool_case(256, 27, 256, a.iters, out)
        ok &= pool_case(256, 13, 256, a.iters, out)
        ok &= pool_case(64, 112, 64, a.iters, out)
        ok &= colsum_case(a.iters, out)
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
