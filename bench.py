"""Flagship benchmark: AlexNet (reference example/ImageNet/ImageNet.conf) training
throughput in images/sec on N MI355X GPUs of one node.

  python bench.py --gpus N --steps K --warmup W
For N > 1 run under torchrun (one process per GPU, RCCL over xGMI).

Weak scaling: every GPU trains on a fixed per-GPU batch of 256 images (the conf's
batch size), so the global batch is 256*N.  Data is synthetic 3x227x227 batches
resident on the device with random-init weights (no dataset / checkpoint on the box).
By default they are uint8 HWC images -- what the imgbin/img pipeline hands over after
JPEG decode and crop -- normalised (mean subtraction) and converted to NHWC bf16 by the
fused augment kernel inside the step; --input f32 feeds float NCHW batches instead.
A step is the full training step: input normalisation/layout conversion, forward, loss
gradient, backward, gradient all-reduce (N > 1) and the fused SGD-momentum update.
"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

BASELINE_IMG_S = None  # filled from BASELINE.json "measured" when present


def _baseline():
    try:
        with open(os.path.join(ROOT, "BASELINE.json")) as f:
            b = json.load(f)
        m = b.get("measured", {}).get("torch_eager_alexnet_img_s_per_gpu")
        return float(m) if m else None
    except Exception:
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=256, help="per-GPU batch")
    ap.add_argument("--model", default="alexnet")
    ap.add_argument("--input", default="u8", choices=["u8", "f32"],
                    help="u8: decoded-image batches (uint8 HWC) normalised on the GPU by the fused augment kernel, "
                         "as the imgbin pipeline delivers them; f32: float NCHW batches")
    ap.add_argument("--graph", type=int, default=0,
                    help="replay forward/backward as HIP graphs (1 GPU; the optimizer stays eager). Off by default: "
                         "the AlexNet and GoogLeNet steps are GPU-bound, graph replay measured -0.4%%/+0.5%% "
                         "(profiles/r16_graph_ab.jsonl)")
    a = ap.parse_args()

    from cxxnet_amd.models import load_conf
    from cxxnet_amd.nnet import NetTrainer
    from cxxnet_amd.io.data import DataBatch
    from cxxnet_amd.parallel import init_distributed
    import torch.distributed as dist

    rank, world = init_distributed()
    if world != a.gpus and rank == 0:
        print(f"warning: --gpus {a.gpus} but WORLD_SIZE={world}", file=sys.stderr)
    dev = torch.device("cuda", torch.cuda.current_device())
    torch.cuda.set_device(dev)

    global_batch = a.batch * world
    pairs = load_conf(a.model, [("batch_size", str(global_batch)), ("eval_train", "0"), ("dev", "gpu"),
                                ("silent", "1"), ("cuda_graph", str(a.graph))])
    pairs = [(k, v) for k, v in pairs if not k.startswith("metric")]
    tr = NetTrainer()
    for k, v in pairs:
        tr.set_param(k, v)
    tr.init_model()
    c, h, w = tr.net_cfg.input_shape
    g = torch.Generator(device="cpu").manual_seed(1234 + rank)
    if a.input == "u8":
        from cxxnet_amd.io.data import U8Images
        pix = torch.randint(0, 256, (a.batch, h, w, c), generator=g, dtype=torch.uint8).to(dev)
        prm = torch.zeros((a.batch, 4), dtype=torch.int32, device=dev)
        cm = torch.tensor([[1.0, 0.0]] * a.batch, device=dev)
        mean = torch.tensor([123.68, 116.78, 103.94][:c], device=dev)  # mean_value subtraction (ImageNet RGB)
        data = U8Images(pix, prm, cm, mean, 1, 1.0)
        desc = f"synthetic uint8 {c}x{h}x{w} images on device, mean subtraction fused on GPU; random-init weights"
    else:
        data = torch.randn(a.batch, c, h, w, generator=g).to(dev)
        desc = f"synthetic fp32 {c}x{h}x{w} batches on device; random-init weights"
    label = torch.randint(0, 1000, (a.batch, 1), generator=g).float().to(dev)
    batch = DataBatch(data, label)

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    for _ in range(a.warmup):
        tr.update(batch, local=True)
    barrier()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        tr.update(batch, local=True)
    barrier()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = t.item()
    ms = el / a.steps * 1000.0
    value = global_batch * a.steps / el
    base = _baseline()
    if rank == 0:
        out = {
            "metric": "images/sec (whole node) AlexNet ImageNet training at 1/2/4/8 MI355X",
            "value": round(value, 1), "unit": "images/sec", "n_gpus": world, "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": round(ms, 3), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": round(value / (base * world), 3) if base else None,
            "dtype": "bf16", "data": desc,
            "config": {"model": a.model, "global_batch": global_batch, "per_gpu_batch": a.batch,
                       "seq_len": None, "parallelism": f"dp{world}", "input_shape": [c, h, w]},
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
