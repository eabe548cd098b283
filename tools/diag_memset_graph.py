"""cxn_zero (hipMemsetAsync) inside a captured HIP graph: does every replay zero the range?"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from cxxnet_amd import ops
    t = torch.ones(4096, device="cuda")
    src = torch.arange(500, device="cuda", dtype=torch.float32)
    s = torch.cuda.Stream()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        g.capture_begin()
        ops.zero_(t[100:1100])
        t[2000:2100].add_(1.0)
        ops.copy_(t[3000:3500], src)  # library device-to-device copy (hipMemcpyAsync)
        g.capture_end()
    torch.cuda.synchronize()
    for i in range(3):
        t.fill_(7.0)
        g.replay()
        torch.cuda.synchronize()
        print(f"replay {i}: zeroed range max {t[100:1100].abs().max().item()} outside {t[0:100].max().item()} "
              f"{t[1100:2000].max().item()} add range {t[2000:2100].max().item()} "
              f"copy ok {bool(torch.equal(t[3000:3500], src))}", flush=True)


if __name__ == "__main__":
    main()
