"""Run a few GEMM-shaped ops in isolation (for rocprofv3 PMC collection).
  python benchmarks/kernel_probe.py conv1_wgrad conv3_fwd fc6_fwd vgg_c3_2_fwd ..."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cxxnet_amd import ops  # noqa: E402
from cxxnet_amd.ops.gemm import ConvGeom, conv_out_size  # noqa: E402

N = 256
CASES = {"conv1": (4, 227, 96, 11, 4, 0, 1), "conv2": (96, 27, 256, 5, 1, 2, 2), "conv3": (256, 13, 384, 3, 1, 1, 1),
         "conv4": (384, 13, 384, 3, 1, 1, 2), "conv5": (384, 13, 256, 3, 1, 1, 2)}


FCS = {"fc6": (9216, 4096), "fc7": (4096, 4096), "fc8": (4096, 1000), "sq8192": (8192, 8192), "sq4096": (4096, 4096)}
VGG = {"c1_2": (64, 224, 64), "c2_1": (64, 112, 128), "c2_2": (128, 112, 128), "c3_2": (256, 56, 256), "c4_2": (512, 28, 512),
       "c5": (512, 14, 512)}


def run_fc(layer, kind, iters):
    nin, nout = FCS[layer]
    N = nin if layer.startswith("sq") else globals()["N"]
    bf = torch.bfloat16
    x = torch.randn(N, nin, device="cuda").to(bf)
    w = (torch.randn(nout, nin, device="cuda") * 0.02).to(bf)
    y = torch.empty(N, nout, device="cuda", dtype=bf)
    dy = torch.randn(N, nout, device="cuda").to(bf)
    dw = torch.zeros(nout, nin, device="cuda")
    for _ in range(iters):
        if kind == "fwd":
            ops.fc_forward(x, w, None, y)
        elif kind == "dgrad":
            ops.fc_backward_data(dy, w, x)
        else:
            ops.fc_backward_weight(x, dy, dw, overwrite=True)
    torch.cuda.synchronize()


def run(name, iters=5):
    n = N
    if name.startswith("conv1c3_"):  # AlexNet conv1 on the 3-channel 228-pixel-row input node
        kind = name.split("_")[1]
        geo = ConvGeom(n, 227, 228, 3, 55, 55, 96, 11, 11, 4, 0, 0, 1)
        x = torch.randn(n, 227, 228, 3, device="cuda").to(torch.bfloat16)
        w = (torch.randn(96, 11, 11, 3, device="cuda") * 0.05).to(torch.bfloat16)
        y = torch.randn(n, 55, 55, 96, device="cuda").to(torch.bfloat16)
        dw = torch.zeros(96, 11, 11, 3, device="cuda")
        for _ in range(iters):
            if kind == "fwd":
                ops.conv_forward(x, w, None, y, geo, relu=True)
            else:
                ops.conv_backward_weight(x, y, dw, geo)
        torch.cuda.synchronize()
        return
    if name.startswith("conv:"):  # generic: conv:C:H:Cout:K:stride:pad:groups:N_kind
        layer, kind = name.rsplit("_", 1)
        C, H, Cout, K, s, p, g, n = (int(v) for v in layer.split(":")[1:])
    elif name.startswith("vgg_"):
        layer, kind = name[4:].rsplit("_", 1)
        C, H, Cout = VGG[layer]
        K, s, p, g = 3, 1, 1, 1
        n = 64
    else:
        layer, kind = name.split("_")
        if layer in FCS:
            return run_fc(layer, kind, iters)
        C, H, Cout, K, s, p, g = CASES[layer]
    Ho, Wo = conv_out_size(H, H, K, K, s, p, p)
    geo = ConvGeom(n, H, H, C, Ho, Wo, Cout, K, K, s, p, p, g)
    bf = torch.bfloat16
    x = torch.randn(n, H, H, C, device="cuda").to(bf)
    w = (torch.randn(Cout, K, K, C // g, device="cuda") * 0.05).to(bf)
    y = torch.randn(n, Ho, Wo, Cout, device="cuda").to(bf)
    dw = torch.zeros(Cout, K, K, C // g, device="cuda")
    wt = torch.empty_like(w)
    for _ in range(iters):
        if kind == "fwd":
            ops.conv_forward(x, w, None, y, geo)
        elif kind == "wgrad":
            ops.conv_backward_weight(x, y, dw, geo)
        else:
            ops.conv_backward_data(y, w, x, geo, wt)
    torch.cuda.synchronize()


if __name__ == "__main__":
    for n in sys.argv[1:]:
        run(n)
