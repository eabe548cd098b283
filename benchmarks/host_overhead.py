"""Host-side cost of one training step: wall time of enqueueing K steps without a sync
(the step is CPU-bound when it approaches the GPU step time), then the synced step time.

  python benchmarks/host_overhead.py [--batch 256] [--model alexnet]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--model", default="alexnet")
    ap.add_argument("--steps", type=int, default=20)
    a = ap.parse_args()
    from cxxnet_amd.io.data import DataBatch
    from cxxnet_amd.models import load_conf
    from cxxnet_amd.nnet import NetTrainer
    pairs = load_conf(a.model, [("batch_size", str(a.batch)), ("eval_train", "0"), ("dev", "gpu"), ("silent", "1")])
    tr = NetTrainer()
    for k, v in pairs:
        if not k.startswith("metric"):
            tr.set_param(k, v)
    tr.init_model()
    c, h, w = tr.net_cfg.input_shape
    batch = DataBatch(torch.randn(a.batch, c, h, w, device="cuda"), torch.zeros(a.batch, 1, device="cuda"))
    for _ in range(5):
        tr.update(batch, local=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        tr.update(batch, local=True)
    t_host = (time.perf_counter() - t0) / a.steps * 1000
    torch.cuda.synchronize()
    t_all = (time.perf_counter() - t0) / a.steps * 1000
    print(json.dumps({"model": a.model, "batch": a.batch, "host_ms_per_step": round(t_host, 3),
                      "wall_ms_per_step": round(t_all, 3)}))


if __name__ == "__main__":
    main()
