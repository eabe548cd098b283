"""Which entries of the 3-channel row-run conv1 weight gradient are wrong (GPU diagnostic)."""
import torch
from cxxnet_amd import ops
from cxxnet_amd.ops import gemm as G
from cxxnet_amd.ops.gemm import ConvGeom

DEV = "cuda"
for N in (2,):
    torch.manual_seed(N)
    H = W = 227
    x3 = torch.randn(N, 3, H, W, device=DEV).to(torch.bfloat16).float()
    w3 = (torch.randn(96, 3, 11, 11, device=DEV) * 0.05).to(torch.bfloat16).float()
    dy = torch.randn(N, 96, 55, 55, device=DEV).to(torch.bfloat16).float()
    dw_ref = torch.nn.grad.conv2d_weight(x3, w3.shape, dy, stride=4)  # co, c, kh, kw
    x = torch.zeros(N, H, 228, 3, device=DEV, dtype=torch.bfloat16)
    x[:, :, :W] = x3.permute(0, 2, 3, 1).to(torch.bfloat16)
    g = ConvGeom(N, H, 228, 3, 55, 55, 96, 11, 11, 4, 0, 0, 1)
    dyb = dy.permute(0, 2, 3, 1).contiguous().to(torch.bfloat16)
    for tile in (-1, 1, 7, 10, 15):
        G._glds_cfg["tile"] = tile
        dw = torch.zeros(96, 11, 11, 3, device=DEV)
        ops.conv_backward_weight(x, dyb, dw, g)
        torch.cuda.synchronize()
        d = (dw.permute(0, 3, 1, 2) - dw_ref).abs()  # co, c, kh, kw
        rel = (d.max() / dw_ref.abs().max()).item()
        bad = d > 0.05 * dw_ref.abs().max()
        print(f"tile {tile}: relerr {rel:.4f} bad {int(bad.sum())} / {bad.numel()}")
        if bad.any():
            print("  bad per c", bad.sum((0, 2, 3)).tolist(), "per kh", bad.sum((0, 1, 3)).tolist(),
                  "per kw", bad.sum((0, 1, 2)).tolist(), "per co(first 8)", bad.sum((1, 2, 3))[:8].tolist())
    G._glds_cfg["tile"] = -1
