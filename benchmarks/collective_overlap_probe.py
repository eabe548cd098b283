"""Does the compute stream wait for an async all-gather?  One rank (RCCL), kernel trace read
back with torch.profiler: an all-gather of `--mb` MB issued async, then a compute kernel on the
current stream.  Variants: issued from the compute stream (as FullConnectLayer.forward does) and
from a side stream that first waits for the compute stream.  Prints the compute kernel's start
relative to the gather copy's end (negative: it overlapped).

    CXXNET_DIST_FORCE=1 python benchmarks/collective_overlap_probe.py [--mb 256]"""
import argparse
import json
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cxxnet_amd.parallel.dp import init_distributed  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mb", type=int, default=256)
    a = ap.parse_args()
    os.environ.setdefault("CXXNET_DIST_FORCE", "1")
    init_distributed()
    dev = torch.device("cuda", torch.cuda.current_device())
    n = a.mb * (1 << 20) // 2
    src = torch.randn(n, device=dev).to(torch.bfloat16)
    out = torch.empty(n * dist.get_world_size(), device=dev, dtype=torch.bfloat16)
    m = torch.randn(4096, 4096, device=dev, dtype=torch.bfloat16)
    side = torch.cuda.Stream()
    res = {}
    for variant in ("compute_stream", "side_stream"):
        for _ in range(3):
            torch.cuda.synchronize()
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
            ev[0].record()
            if variant == "compute_stream":
                work = dist.all_gather_into_tensor(out, src, async_op=True)
            else:
                side.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(side):
                    work = dist.all_gather_into_tensor(out, src, async_op=True)
            ev[1].record()
            for _ in range(4):
                m2 = m @ m  # compute on the current stream
            ev[2].record()
            work.wait()
            if variant != "compute_stream":
                torch.cuda.current_stream().wait_stream(side)
            ev[3].record()
            torch.cuda.synchronize()
        t_mm = ev[1].elapsed_time(ev[2])
        t_all = ev[0].elapsed_time(ev[3])
        res[variant] = {"matmuls_ms": round(t_mm, 3), "total_ms": round(t_all, 3)}
    solo = []
    for _ in range(3):
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(4):
            m2 = m @ m
        e1.record()
        torch.cuda.synchronize()
        solo.append(e0.elapsed_time(e1))
    res["matmuls_alone_ms"] = round(min(solo), 3)
    print(json.dumps({"mb": a.mb, **res}))
    del m2


if __name__ == "__main__":
    main()
