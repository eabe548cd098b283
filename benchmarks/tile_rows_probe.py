"""Which output rows / columns of an LDS-DMA tile come out wrong (fc forward, forced tile).

  python benchmarks/tile_rows_probe.py

Found the 96-row tile bug: the epilogue's intra-wave LDS hand-off needed a wave fence when some
lanes sit out the row loop (gemm_glds.hip wave_lds_handoff)."""
import sys
import torch
sys.path.insert(0, ".")
from cxxnet_amd import ops
from cxxnet_amd.ops import gemm as G

for tile in (7, 71, 72, 73, 74, 75):
    for nout, nin, B in ((96, 64, 128), (96, 128, 128), (192, 256, 128)):
        g = torch.Generator(device="cuda").manual_seed(0)
        x = torch.randn(B, nin, device="cuda", generator=g).to(torch.bfloat16)
        w = torch.randn(nout, nin, device="cuda", generator=g).to(torch.bfloat16)
        y = torch.zeros(B, nout, device="cuda", dtype=torch.bfloat16)
        G.set_glds(True, tile)
        ops.fc_forward(x, w, None, y)
        G.set_glds(True, -1)
        torch.cuda.synchronize()
        ref = x.float() @ w.float().t()
        err = (y.float() - ref).abs() > 0.05 * ref.abs().max()
        bad_i = err.any(0).nonzero().flatten().tolist()   # output channels (A rows)
        bad_j = err.any(1).nonzero().flatten().tolist()   # batch rows (B rows)
        print(f"tile {tile} nout {nout} nin {nin}: bad A rows {len(bad_i)} {bad_i[:24]}; bad B rows {len(bad_j)} "
              f"{bad_j[:20]}", flush=True)
        if bad_i:
            i, j = bad_i[0], bad_j[0]
            print("   y", y[j, i - 2:i + 3].float().tolist(), "ref", ref[j, i - 2:i + 3].tolist(), flush=True)
