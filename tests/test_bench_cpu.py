"""bench.py launcher contract on the CPU (gloo ranks): `--gpus N` without torchrun spawns N
ranks itself, reports the process group's size, and a rank-count mismatch exits non-zero."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, timeout=600):
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env["OMP_NUM_THREADS"] = "2"
    return subprocess.run([sys.executable] + args, cwd=ROOT, env=env, capture_output=True, text=True,
                          timeout=timeout)


def _json(stdout):
    lines = [l for l in stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, stdout
    return json.loads(lines[0])


def test_bench_self_launches_two_ranks():
    r = _run(["bench.py", "--gpus", "2", "--device", "cpu", "--model", "mnist_mlp", "--batch", "8",
              "--steps", "2", "--warmup", "1"])
    assert r.returncode == 0, r.stderr[-3000:]
    out = _json(r.stdout)
    assert out["n_gpus"] == 2 and out["world_size"] == 2
    assert out["scaling"] == "weak" and out["config"]["global_batch"] == 16
    assert len(out["per_rank_ms_per_step"]) == 2
    assert out["dp"]["comm_bytes_per_step_per_rank"] > 0
    assert "AlexNet" not in out["metric"]


def test_bench_strong_scaling_splits_global_batch():
    r = _run(["bench.py", "--gpus", "2", "--device", "cpu", "--model", "mnist_mlp", "--batch", "10",
              "--steps", "2", "--warmup", "1", "--scaling", "strong", "--dp-mode", "shard"])
    assert r.returncode == 0, r.stderr[-3000:]
    out = _json(r.stdout)
    assert out["scaling"] == "strong"
    assert out["config"]["global_batch"] == 10 and out["config"]["per_gpu_batch"] == 5
    assert out["dp"]["mode"] == "shard"


def test_bench_rank_mismatch_fails():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = str(s.getsockname()[1])
    r = _run(["-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1", "--master-addr", "127.0.0.1",
              "--master-port", port, "bench.py", "--gpus", "2", "--device", "cpu", "--model", "mnist_mlp",
              "--batch", "8", "--steps", "1", "--warmup", "0"])
    assert r.returncode != 0
    assert "process group holds 1" in r.stderr


def test_bench_8_ranks_weak():
    r = _run(["bench.py", "--gpus", "8", "--device", "cpu", "--model", "mnist_mlp", "--batch", "8",
              "--steps", "2", "--warmup", "1"])
    assert r.returncode == 0, r.stderr[-3000:]
    out = _json(r.stdout)
    assert out["n_gpus"] == 8 and out["world_size"] == 8 and len(out["per_rank_ms_per_step"]) == 8
    assert out["config"]["global_batch"] == 64 and out["dp"]["mode"] == "allreduce"
    # the same run times the conf's own (strong-scaling) configuration: 8 images over 8 ranks
    st = out["strong"]
    assert st["scaling"] == "strong" and st["global_batch"] == 8 and st["per_gpu_batch"] == 1
    assert st["value"] > 0 and len(st["per_rank_ms_per_step"]) == 8


def test_bench_8_ranks_strong_alexnet_fullc_gather():
    """AlexNet at the strong-scaling split (256 over 8 ranks = 32 rows each): fullc_gather's
    default (auto) all-gathers the fc layers' [in | out-grad] rows instead of reducing their
    58.6 M gradient values, so a rank hands <= 40 MB per step to collectives (fp32 here; the GPU
    gathers bf16) against 244 MB of fp32 gradients without it."""
    r = _run(["bench.py", "--gpus", "8", "--device", "cpu", "--model", "alexnet", "--batch", "256",
              "--scaling", "strong", "--steps", "1", "--warmup", "0"], timeout=900)
    assert r.returncode == 0, r.stderr[-3000:]
    out = _json(r.stdout)
    assert out["config"]["per_gpu_batch"] == 32 and out["dp"]["fullc_gather"]
    assert out["dp"]["comm_bytes_per_step_per_rank"] <= 40e6, out["dp"]
