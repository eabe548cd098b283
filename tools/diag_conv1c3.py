"""Which entries of the 3-channel row-run conv1 forward / weight gradient are wrong (GPU diagnostic)."""
import torch
import torch.nn.functional as F
from cxxnet_amd import ops
from cxxnet_amd.ops import gemm as G
from cxxnet_amd.ops.gemm import ConvGeom

DEV = "cuda"
for N in (2, 16):
    torch.manual_seed(N)
    H = W = 227
    x3 = torch.randn(N, 3, H, W, device=DEV).to(torch.bfloat16).float()
    w3 = (torch.randn(96, 3, 11, 11, device=DEV) * 0.05).to(torch.bfloat16).float()
    dy = torch.randn(N, 96, 55, 55, device=DEV).to(torch.bfloat16).float()
    y_ref = F.conv2d(x3, w3, stride=4) + 0.5
    dw_ref = torch.nn.grad.conv2d_weight(x3, w3.shape, dy, stride=4)  # co, c, kh, kw
    x = torch.zeros(N, H, 228, 3, device=DEV, dtype=torch.bfloat16)
    x[:, :, :W] = x3.permute(0, 2, 3, 1).to(torch.bfloat16)
    w = w3.permute(0, 2, 3, 1).contiguous().to(torch.bfloat16)
    g = ConvGeom(N, H, 228, 3, 55, 55, 96, 11, 11, 4, 0, 0, 1)
    dyb = dy.permute(0, 2, 3, 1).contiguous().to(torch.bfloat16)
    for tile in (-1, 1, 7, 10, 15):
        G._glds_cfg["tile"] = tile
        try:
            y = torch.empty(N, 55, 55, 96, device=DEV, dtype=torch.bfloat16)
            ops.conv_forward(x, w, torch.full((96,), 0.5, device=DEV), y, g)
            torch.cuda.synchronize()
            yrel = ((y.permute(0, 3, 1, 2).float() - y_ref).norm() / y_ref.norm()).item()
            print(f"N {N} tile {tile}: fwd relerr {yrel:.4f}", flush=True)
        except Exception as e:  # noqa: BLE001
            print(f"N {N} tile {tile}: fwd {type(e).__name__}: {e}", flush=True)
        try:
            dw = torch.zeros(96, 11, 11, 3, device=DEV)
            ops.conv_backward_weight(x, dyb, dw, g)
            torch.cuda.synchronize()
        except Exception as e:  # noqa: BLE001
            print(f"N {N} tile {tile}: wgrad {type(e).__name__}: {e}", flush=True)
            continue
        d = (dw.permute(0, 3, 1, 2) - dw_ref).abs()  # co, c, kh, kw
        rel = (d.max() / dw_ref.abs().max()).item()
        nrel = ((dw.permute(0, 3, 1, 2) - dw_ref).norm() / dw_ref.norm()).item()
        bad = d > 0.05 * dw_ref.abs().max()
        print(f"N {N} tile {tile}: wgrad maxrel {rel:.4f} normrel {nrel:.4f} bad {int(bad.sum())} / {bad.numel()}",
              flush=True)
        if bad.any():
            print("  bad per c", bad.sum((0, 2, 3)).tolist(), "per kh", bad.sum((0, 1, 3)).tolist(),
                  "per kw", bad.sum((0, 1, 2)).tolist(), "per co(first 8)", bad.sum((1, 2, 3))[:8].tolist())
    G._glds_cfg["tile"] = -1
print("tuned:", {k: v for k, v in G._TUNE.items() if k.startswith("cr|") or k.startswith("cwr|")})
print("rejected:", G.TUNE_REJECTED)
