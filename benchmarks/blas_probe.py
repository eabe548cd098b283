"""hipBLASLt (torch.mm) on square bf16 GEMMs, for rocprofv3 PMC collection next to our kernels:
    python benchmarks/blas_probe.py 8192 [iters]"""
import sys

import torch

n = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
it = int(sys.argv[2]) if len(sys.argv) > 2 else 5
g = torch.Generator(device="cuda").manual_seed(1)
x = torch.randn(n, n, device="cuda", generator=g).to(torch.bfloat16)
w = torch.randn(n, n, device="cuda", generator=g).to(torch.bfloat16)
for _ in range(it):
    y = torch.mm(x, w.t())
torch.cuda.synchronize()
