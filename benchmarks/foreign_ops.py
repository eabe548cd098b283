"""List the GPU kernels of one eager training step that do NOT come from libcxxnet_kernels.so
(torch elementwise kernels, allocator fills, copies), with the Python call site that issued
them.  The C++ launch-list replay (NeuralNet record/replay) replays only library launches, so a
step segment must contain none of these.

  python benchmarks/foreign_ops.py [--model alexnet] [--batch 32] [--set k=v ...]
"""
import argparse
import collections
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="alexnet")
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--set", action="append", default=[])
    a = ap.parse_args()
    from cxxnet_amd.io.data import DataBatch
    from cxxnet_amd.models import load_conf
    from cxxnet_amd.nnet import NetTrainer
    from cxxnet_amd.parallel import init_distributed
    init_distributed()
    over = [("batch_size", str(a.batch)), ("eval_train", "0"), ("dev", "gpu"), ("silent", "1"), ("cuda_graph", "0")]
    over += [tuple(kv.split("=", 1)) for kv in a.set]
    tr = NetTrainer()
    for k, v in load_conf(a.model, over):
        if not k.startswith("metric"):
            tr.set_param(k, v)
    tr.init_model()
    c, h, w = tr.net_cfg.input_shape
    batch = DataBatch(torch.randn(a.batch, c, h, w, device="cuda"), torch.zeros(a.batch, 1, device="cuda"))
    for _ in range(4):
        tr.update(batch, local=True)
    torch.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
        tr.update(batch, local=True)
        torch.cuda.synchronize()
    kern = collections.Counter()
    foreign = collections.Counter()
    for ev in prof.events():
        if ev.device_type != torch.autograd.DeviceType.CUDA:
            continue
        kern[ev.name] += 1
    # CPU-side torch ops that launched device work: their stacks name the Python call site
    for ev in prof.events():
        if ev.device_type == torch.autograd.DeviceType.CUDA or not ev.name.startswith("aten::"):
            continue
        if not (ev.kernels or []) and getattr(ev, "device_time_total", 0) == 0:
            continue
        site = next((f for f in (ev.stack or []) if "cxxnet_amd" in f), "?")
        foreign[(ev.name, site)] += 1
    print(json.dumps({"model": a.model, "batch": a.batch, "set": a.set,
                      "kernels": sum(kern.values()),
                      "foreign_ops": [{"op": k[0], "site": k[1], "n": n} for k, n in foreign.most_common()],
                      "kernel_names": dict(kern.most_common())}), flush=True)


if __name__ == "__main__":
    main()
