"""Conv weight-gradient (register-staged split-K kernel) over tile x split, for one geometry:
  python benchmarks/wgrad_split_probe.py C:H:Cout:K:stride:pad:groups:N [...] > out.jsonl
Checks each variant against the default path's output."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cxxnet_amd import ops  # noqa: E402
from cxxnet_amd.ops import gemm as G  # noqa: E402


def timeit(fn, iters=20):
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


def main():
    for spec in sys.argv[1:]:
        C, H, Cout, K, st, pd, grp, N = (int(v) for v in spec.split(":"))
        Ho, Wo = G.conv_out_size(H, H, K, K, st, pd, pd)
        g = G.ConvGeom(N, H, H, C, Ho, Wo, Cout, K, K, st, pd, pd, grp)
        x = torch.randn(N, H, H, C, device="cuda").to(torch.bfloat16)
        dy = torch.randn(N, Ho, Wo, Cout, device="cuda").to(torch.bfloat16)
        dw = torch.zeros(Cout, K, K, C // grp, device="cuda")
        flops = 2.0 * N * Ho * Wo * Cout * (C // grp) * K * K
        ops.conv_backward_weight(x, dy, dw, g)
        torch.cuda.synchronize()
        ref = dw.clone()
        rec = {"op": spec, "default_us": round(timeit(lambda: (dw.zero_(), ops.conv_backward_weight(x, dy, dw, g))), 1)}
        cg, kd, P = g.cg_in, g.kdim, g.N * g.Ho * g.Wo
        A = G._op(x, cg, 0, kd, P, H=g.H, W=g.W, C=g.C, Ho=g.Ho, Wo=g.Wo, KH=g.KH, KW=g.KW, stride=g.stride,
                  pad_h=g.pad_y, pad_w=g.pad_x, dil=1, Cg=cg)
        B = G._op(dy, g.cg_out, g.Cout, g.cg_out, P)
        for tile in (0, 5, 1, 2):
            for split in (32, 64, 128, 256, 512, 1024):
                def run():
                    dw.zero_()
                    G._gemm(A, B, G.GATHER_MN, G.DIRECT_MN, 8, 8, dw, g.cg_out * kd, kd, epi=G.EPI_F32_ATOMIC,
                            groups=g.groups, ksplit=split, tile=tile)
                try:
                    run()
                except RuntimeError:
                    rec[f"t{tile}"] = "unsupported"
                    break
                torch.cuda.synchronize()
                err = ((dw - ref).norm() / ref.norm()).item()
                us = timeit(run)
                rec[f"t{tile}_s{split}"] = [round(us, 1), round(err, 5)]
        best = min((v[0], k) for k, v in rec.items() if k.startswith("t") and isinstance(v, list))
        rec["best"] = best
        rec["default_tflops"] = round(flops / rec["default_us"] / 1e6, 1)
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
