"""Host-side cost of one training step vs its GPU time.

  python benchmarks/host_overhead.py [--batch 32] [--model alexnet] [--graph 0|1]

* host_ms: wall time to ENQUEUE one step while the GPU is held busy by a long sleep kernel
  queued first (so the host never waits on the device: pure Python + launch cost);
* gpu_ms: (wall time from the start of the sleep to the end of the K queued steps minus the
  sleep's own duration) / K -- the steps run back to back on the device, no host gaps;
* wall_ms: plain back-to-back steps (what training sees).
Host-bound when host_ms approaches gpu_ms.  CXXNET_DIST_FORCE=1 runs the data-parallel
machinery (RCCL collectives at world 1, per-bucket side-stream updates, forward gating).
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _sleep_ms(ms):
    # torch.cuda._sleep spins for a number of GPU cycles; calibrate once
    t0 = torch.cuda.Event(enable_timing=True)
    t1 = torch.cuda.Event(enable_timing=True)
    t0.record()
    torch.cuda._sleep(10_000_000)
    t1.record()
    t1.synchronize()
    per_cycle_ms = t0.elapsed_time(t1) / 10_000_000
    return int(ms / per_cycle_ms)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--model", default="alexnet")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--graph", type=int, default=-1, help="cuda_graph (-1: the trainer's default, launch lists)")
    a = ap.parse_args()
    from cxxnet_amd.io.data import DataBatch
    from cxxnet_amd.models import load_conf
    from cxxnet_amd.nnet import NetTrainer
    from cxxnet_amd.parallel import init_distributed
    init_distributed()
    extra = [("cuda_graph", str(a.graph))] if a.graph >= 0 else []
    pairs = load_conf(a.model, [("batch_size", str(a.batch)), ("eval_train", "0"), ("dev", "gpu"), ("silent", "1")]
                      + extra)
    tr = NetTrainer()
    for k, v in pairs:
        if not k.startswith("metric"):
            tr.set_param(k, v)
    tr.init_model()
    c, h, w = tr.net_cfg.input_shape
    batch = DataBatch(torch.randn(a.batch, c, h, w, device="cuda"), torch.zeros(a.batch, 1, device="cuda"))
    for _ in range(6):
        tr.update(batch, local=True)
    torch.cuda.synchronize()
    # plain back-to-back steps
    t0 = time.perf_counter()
    for _ in range(4 * a.steps):
        tr.update(batch, local=True)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / (4 * a.steps) * 1000
    # host enqueue cost with the GPU held busy
    cyc = _sleep_ms(200.0)
    s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s0.record()
    torch.cuda._sleep(cyc)
    s1.record()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        tr.update(batch, local=True)
    host = (time.perf_counter() - t0) / a.steps * 1000
    e1 = torch.cuda.Event(enable_timing=True)
    e1.record()
    e1.synchronize()
    sleep_ms = s0.elapsed_time(s1)
    gpu = s1.elapsed_time(e1) / a.steps
    rec = {"model": a.model, "batch": a.batch, "graph": a.graph, "dp": tr.reducer.active,
           "host_ms_per_step": round(host, 3), "gpu_ms_per_step": round(gpu, 3), "wall_ms_per_step": round(wall, 3),
           "host_over_gpu": round(host / gpu, 3), "sleep_ms": round(sleep_ms, 1)}
    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
