"""Flagship benchmark: AlexNet (reference example/ImageNet/ImageNet.conf) training
throughput in images/sec on N MI355X GPUs of one node.

  python bench.py --gpus N --steps K --warmup W [--scaling weak|strong] [--model alexnet]

One process per GPU, RCCL over xGMI.  Under torchrun (WORLD_SIZE set) every rank runs
the step; with --gpus N > 1 and no WORLD_SIZE this script launches
`python -m torch.distributed.run --nproc-per-node N` on itself as a CHILD process before
anything touches the GPU, and exits with its code.  A run whose process group does not
hold exactly N ranks exits non-zero.

Scaling modes (the reference's batch_size is the GLOBAL batch, split ceil(B/ndev) per
device: src/nnet/nnet_impl-inl.hpp:147-155, example/ImageNet/ImageNet.conf:108):
  weak   (default) every GPU trains a fixed per-GPU batch of --batch (256) images, the
         global batch is 256*N: the per-GPU work of the conf's 1-GPU run, N times over;
  strong the global batch is --batch (256) and each rank takes ceil(256/N) rows, exactly
         the reference's multi-device semantics for the conf as written.
With the default weak scaling and N > 1 the same run also times the strong configuration
(ImageNet.conf's global batch of 256 over the N ranks) and reports it as the nested "strong"
record of the one JSON line (--strong-record 0 skips it).

Data is synthetic 3x227x227 batches resident on the device with random-init weights (no
dataset / checkpoint on the box).  By default they are uint8 HWC images -- what the
imgbin/img pipeline hands over after JPEG decode and crop -- normalised (mean
subtraction) and converted to NHWC bf16 by the fused augment kernel inside the step;
--input f32 feeds float NCHW batches instead.  A step is the full training step: input
normalisation/layout conversion, forward, loss gradient, backward, gradient reduction
(N > 1: bucketed fp32 all-reduce overlapped with backward, per-bucket optimizer on a side
stream; --dp-mode shard: reduce-scatter, sliced optimizer, bf16 weight all-gather; see
cxxnet_amd/parallel/dp.py) and the fused SGD-momentum update.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

MODEL_NAMES = {"alexnet": "AlexNet ImageNet", "inception_v1": "GoogLeNet/Inception-v1 ImageNet",
               "vgg16": "VGG-16 ImageNet", "mnist_mlp": "MNIST-MLP", "mnist_conv": "MNIST-conv",
               "bowl": "Kaggle-bowl convnet"}


def _args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=15)
    ap.add_argument("--batch", type=int, default=256,
                    help="weak: per-GPU batch; strong: global batch split over the ranks")
    ap.add_argument("--scaling", default="weak", choices=["weak", "strong"])
    ap.add_argument("--strong-record", type=int, default=1,
                    help="with --scaling weak and N > 1, also time the conf's own configuration (global "
                         "batch --batch split over the ranks, strong scaling) and add it as a nested "
                         "\"strong\" record to the one JSON line")
    ap.add_argument("--model", default="alexnet")
    ap.add_argument("--input", default="u8", choices=["u8", "f32"],
                    help="u8: decoded-image batches (uint8 HWC) normalised on the GPU by the fused augment kernel, "
                         "as the imgbin pipeline delivers them; f32: float NCHW batches")
    ap.add_argument("--graph", type=int, default=-1,
                    help="replay forward/backward as HIP graphs (the optimizer and collectives stay eager). "
                         "-1 (default) = the trainer's auto rule: on under data parallelism at per-GPU batch <= 64 "
                         "(strong scaling); the 1-GPU AlexNet / GoogLeNet steps are GPU-bound, graph replay measured "
                         "-0.4%%/+0.5%% (profiles/early-r16_graph_ab.jsonl)")
    ap.add_argument("--dp-mode", default="auto", choices=["auto", "shard", "allreduce"],
                    help="gradient reduction: auto = fp32 all-reduce (shard: reduce-scatter, sliced update, "
                         "bf16 all-gather)")
    ap.add_argument("--bucket-mb", type=float, default=64.0)
    ap.add_argument("--device", default="gpu", choices=["gpu", "cpu"],
                    help="cpu: gloo ranks on the host (test hook for the launcher and the DP path)")
    ap.add_argument("--set", action="append", default=[], metavar="KEY=VAL",
                    help="extra conf overrides, e.g. --set dp_comm_dtype=bf16")
    return ap.parse_args(argv)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _spawn(a) -> int:
    """Re-launch this script as N ranks (child process; nothing here has touched the GPU)."""
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", "4")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd, env=env)


def _baseline(model):
    """Same-model torch-eager img/s per GPU from BASELINE.json "measured" (None if absent)."""
    try:
        with open(os.path.join(ROOT, "BASELINE.json")) as f:
            b = json.load(f)
        m = b.get("measured", {}).get(f"torch_eager_{model}_img_s_per_gpu")
        return float(m) if m else None
    except Exception:
        return None



def _measure(a, world, rank, dev, global_batch, local_batch):
    """Build the trainer at (global_batch, local_batch), run a.warmup untimed steps, then time
    a.steps steps bracketed by a barrier + device synchronisation; returns the MAX over ranks."""
    import torch
    import torch.distributed as dist
    from cxxnet_amd.models import load_conf
    from cxxnet_amd.nnet import NetTrainer
    from cxxnet_amd.io.data import DataBatch
    lo = min(rank * local_batch, global_batch)
    my_rows = min(local_batch, global_batch - lo)  # the reference's ceil split: the last rank may hold fewer

    over = [("batch_size", str(global_batch)), ("eval_train", "0"), ("dev", a.device), ("silent", "1"),
            ("cuda_graph", str(a.graph)), ("dp_mode", a.dp_mode), ("dp_bucket_mb", str(a.bucket_mb))]
    for kv in a.set:
        k, v = kv.split("=", 1)
        over.append((k.strip(), v.strip()))
    pairs = load_conf(a.model, over)
    pairs = [(k, v) for k, v in pairs if not k.startswith("metric")]
    tr = NetTrainer()
    for k, v in pairs:
        tr.set_param(k, v)
    tr.init_model()
    assert tr._local_batch() == local_batch, (tr._local_batch(), local_batch)
    c, h, w = tr.net_cfg.input_shape
    g = torch.Generator(device="cpu").manual_seed(1234 + rank)
    if a.input == "u8":
        from cxxnet_amd.io.data import U8Images
        pix = torch.randint(0, 256, (my_rows, h, w, c), generator=g, dtype=torch.uint8).to(dev)
        prm = torch.zeros((my_rows, 4), dtype=torch.int32, device=dev)
        cm = torch.tensor([[1.0, 0.0]] * my_rows, device=dev)
        mean = torch.tensor([123.68, 116.78, 103.94][:c], device=dev)  # mean_value subtraction (ImageNet RGB)
        data = U8Images(pix, prm, cm, mean, 1, 1.0)
        desc = (f"synthetic uint8 {c}x{h}x{w} images on device, mean subtraction fused on GPU; "
                f"random-init weights")
    else:
        data = torch.randn(my_rows, c, h, w, generator=g).to(dev)
        desc = f"synthetic fp32 {c}x{h}x{w} batches on device; random-init weights"
    ncls = 10 if a.model.startswith("mnist") else 1000
    label = torch.randint(0, ncls, (my_rows, 1), generator=g).float().to(dev)
    batch = DataBatch(data, label)

    def barrier():
        if world > 1:
            dist.barrier()
        if dev.type == "cuda":
            torch.cuda.synchronize()

    for _ in range(a.warmup):
        tr.update(batch, local=True)
    barrier()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        tr.update(batch, local=True)
    tr.reducer.sync()
    barrier()
    el = time.perf_counter() - t0
    per_rank = [el]
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64, device=dev)
        allt = [torch.zeros_like(t) for _ in range(world)]
        dist.all_gather(allt, t)
        per_rank = [float(x.item()) for x in allt]
        el = max(per_rank)
    return el, per_rank, tr, c, h, w, desc


def _dp_info(tr):
    red = tr.reducer
    return {"mode": ("shard" if red.shard else "allreduce") if red.active else "none",
            "buckets": len(red.buckets) if red.active else 0,
            "comm_bytes_per_step_per_rank": tr.comm_bytes_per_step(),
            "fullc_gather": any(getattr(c.layer, "_gathering", None) is not None and c.layer._gathering()
                                for c in tr.net.connections),
            "overlapped_update": red.handles_update}


def main():
    a = _args()
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return _spawn(a)

    import torch
    if a.device == "cpu":
        os.environ.setdefault("CXXNET_DIST_BACKEND", "gloo")
    from cxxnet_amd.parallel import init_distributed
    import torch.distributed as dist

    rank, world = init_distributed()
    if world != a.gpus:
        print(f"bench.py: --gpus {a.gpus} but the process group holds {world} rank(s)", file=sys.stderr)
        return 2
    if a.device == "gpu":
        dev = torch.device("cuda", torch.cuda.current_device())
        torch.cuda.set_device(dev)
    else:
        dev = torch.device("cpu")
        a.input = "f32"

    if a.scaling == "weak":
        local_batch = a.batch
        global_batch = a.batch * world
    else:
        global_batch = a.batch
        local_batch = (a.batch + world - 1) // world

    el, per_rank, tr, c, h, w, desc = _measure(a, world, rank, dev, global_batch, local_batch)
    ms = el / a.steps * 1000.0
    value = global_batch * a.steps / el
    base = _baseline(a.model)
    dp = _dp_info(tr)
    strong = None
    if a.scaling == "weak" and world > 1 and a.strong_record:
        # the conf's own configuration: its global batch split over the ranks
        del tr
        if dev.type == "cuda":
            torch.cuda.empty_cache()
        sg, sl = a.batch, (a.batch + world - 1) // world
        sel, sper, str_, *_ = _measure(a, world, rank, dev, sg, sl)
        strong = {"value": round(sg * a.steps / sel, 1), "unit": "images/sec", "scaling": "strong",
                  "global_batch": sg, "per_gpu_batch": sl, "ms_per_step": round(sel / a.steps * 1000.0, 3),
                  "per_rank_ms_per_step": [round(x / a.steps * 1000.0, 3) for x in sper], "dp": _dp_info(str_)}
    elif a.scaling == "weak" and world == 1:
        strong = "identical to the weak record at one GPU (global batch = per-GPU batch)"
    if rank == 0:
        name = MODEL_NAMES.get(a.model, a.model)
        out = {
            "metric": f"images/sec (whole node) {name} training at 1/2/4/8 MI355X",
            "value": round(value, 1), "unit": "images/sec", "n_gpus": world, "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": round(ms, 3), "higher_is_better": True,
            "scaling": a.scaling,
            "vs_baseline": round(value / (base * world), 3) if base else None,
            "dtype": "bf16" if dev.type == "cuda" else "fp32", "data": desc,
            "config": {"model": a.model, "global_batch": global_batch, "per_gpu_batch": local_batch,
                       "seq_len": None, "parallelism": f"dp{world}", "input_shape": [c, h, w]},
            "world_size": world,
            "per_rank_ms_per_step": [round(x / a.steps * 1000.0, 3) for x in per_rank],
            "dp": dp,
            "strong": strong,
            "baseline": (f"torch eager {a.model} {base:.0f} img/s per GPU x {world} (BASELINE.json measured)"
                         if base else None),
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
