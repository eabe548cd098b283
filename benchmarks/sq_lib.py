"""hipBLASLt (torch.matmul, bf16) on square GEMMs: the library ceiling next to gemm_glds_bench's sq ops."""
import json
import torch
for n in (4096, 8192):
    a = torch.randn(n, n, device="cuda").to(torch.bfloat16)
    b = torch.randn(n, n, device="cuda").to(torch.bfloat16)
    for _ in range(3):
        a @ b.t()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(20):
        a @ b.t()
    e.record()
    torch.cuda.synchronize()
    us = s.elapsed_time(e) / 20 * 1000
    print(json.dumps({"op": f"lib_sq{n}", "us": round(us, 1), "tflops": round(2 * n ** 3 / us / 1e6, 1)}))
