"""Data parallelism through the GPU path: 2 ranks (gloo backend, both on the one GPU of the
test box -- RCCL refuses two ranks per device) must match the single-process GPU step on the
whole batch.  Exercises the bucketed all-reduce launched from the backprop hook, the
overlapped per-bucket optimizer on the side stream, the rank-0 broadcast and the replica
consistency check, with the HIP kernels doing the math (the 8-GPU RCCL run is the driver's)."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from test_dp_gloo import CONF

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _make(batch, extra=()):
    from cxxnet_amd import native
    from cxxnet_amd.nnet import NetTrainer
    tr = NetTrainer()
    for k, v in list(native.rt().parse_config(CONF)) + [("batch_size", str(batch)), ("dev", "gpu"),
                                                        ("eval_train", "0"), ("silent", "1"), ("seed", "5"),
                                                        ("cuda_graph", "0")] + \
            list(extra):
        tr.set_param(k, v)
    tr.init_model()
    return tr


def _data(B):
    g = torch.Generator().manual_seed(11)
    return torch.randn(B, 3, 8, 8, generator=g), torch.randint(0, 5, (B, 1), generator=g).float()


def _worker(rank, world, port, steps, out, extra, backend="gloo"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), CXXNET_DIST_BACKEND=backend, CXXNET_DIST_FORCE="1")
    import torch.distributed as dist
    from cxxnet_amd.io.data import DataBatch
    from cxxnet_amd.parallel import init_distributed
    init_distributed()
    tr = _make(8, extra)
    assert tr.reducer.update_fn is not None  # overlapped per-bucket update is on under DP
    x, y = _data(8)
    for _ in range(steps):
        tr.update(DataBatch(x.cuda(), y.cuda()))
    torch.cuda.synchronize()
    assert tr.reducer.check_consistency() == 0.0
    graph = any(k == "cuda_graph" and v == "1" for k, v in extra)
    if graph:
        assert tr._graphs, "the data-parallel step did not run as graph segments"
        fwd, bwd = next(iter(tr._graphs.values()))[:2]
        assert sum(callable(i) and not isinstance(i, torch.cuda.CUDAGraph) for i in fwd + bwd) > 0
    if any(k == "fullc_gather" and v == "1" for k, v in extra) and not graph:
        # the gathered fc layer the kernel covers (f1: 16 x 128; f2's 5 outputs are not a multiple
        # of 8) ran its SGD step inside the weight-gradient GEMM
        fcs = [c.layer for c in tr.net.connections if c.layer.type_name == "fullc"]
        assert tr.net.ctx.dp_active and len(tr.net.updater.fused_offsets) == 1, \
            (tr.net.updater.fused_offsets, [f._gathering() for f in fcs], list(tr._lists), list(tr._graphs))
    tr.reducer.sync_master()  # sharded: each rank updated only its slice of the fp32 masters
    torch.save(tr.net.arena.w.cpu(), out + f".r{rank}")
    # per parameter too: with fullc_gather the arena pads the gathered layers' segments to
    # world * ALIGN boundaries, so the flat layout differs from the single-process arena
    a = tr.net.arena
    torch.save([a.w[sp.offset:sp.offset + sp.numel].cpu() for _, sp in a.specs], out + f".p{rank}")
    dist.destroy_process_group()


@pytest.mark.parametrize("extra", [(), (("dp_comm_dtype", "bf16"),), (("update_period", "2"),),
                                   (("dp_mode", "allreduce"),), (("cuda_graph", "1"),),
                                   # the gloo CPU tests' 1e-4 bound: deterministic GEMMs (no fp32
                                   # atomics), so only the 2-rank sum order differs (measured 1e-9)
                                   (("deterministic", "1"),),
                                   (("deterministic", "1"), ("dp_mode", "allreduce")),
                                   # the gathered fc path with two real ranks: [x | dy] row
                                   # all-gathers and the SGD step fused into the weight-gradient
                                   # GEMM, under launch lists, graph segments, and bit-equal to
                                   # the single-GPU step in deterministic mode
                                   (("fullc_gather", "1"),),
                                   (("fullc_gather", "1"), ("launch_replay", "0")),
                                   (("fullc_gather", "1"), ("cuda_graph", "1")),
                                   (("fullc_gather", "1"), ("dp_mode", "shard")),
                                   (("fullc_gather", "1"), ("deterministic", "1"))])
def test_dp_two_ranks_gpu_equals_single(tmp_path, extra):
    steps = 4
    out = str(tmp_path / "w")
    mp.spawn(_worker, args=(2, _free_port(), steps, out, list(extra)), nprocs=2, join=True)
    r0 = torch.load(out + ".r0", weights_only=True)
    r1 = torch.load(out + ".r1", weights_only=True)
    assert torch.equal(r0, r1), "replicas diverged"
    from cxxnet_amd.io.data import DataBatch
    tr = _make(8, list(extra))
    x, y = _data(8)
    for _ in range(steps):
        tr.update(DataBatch(x.cuda(), y.cuda()))
    torch.cuda.synchronize()
    a = tr.net.arena
    w = torch.cat([a.w[sp.offset:sp.offset + sp.numel].cpu() for _, sp in a.specs])
    a0 = _make(8, list(extra)).net.arena  # same seed: the initial weights
    w0 = torch.cat([a0.w[sp.offset:sp.offset + sp.numel].cpu() for _, sp in a0.specs])
    p0 = torch.cat(torch.load(out + ".p0", weights_only=True))
    err = ((p0 - w).norm() / (w - w0).norm()).item()  # relative to the distance trained
    print(f"dp 2-rank vs single, {extra}: err {err:.3g}")
    # default mode: fp32 atomics in the weight gradients make the summation order run-dependent,
    # and a 1-ulp flip of a bf16 weight shadow moves later activations by bf16 ulps
    tol = 1e-4 if ("deterministic", "1") in extra else 5e-2
    assert err < tol, err


@pytest.mark.parametrize("graph", [0, 1])
@pytest.mark.parametrize("mode", ["shard", "allreduce"])
def test_rccl_single_rank_forced_is_exact(tmp_path, mode, graph):
    """The RCCL ("nccl") backend at world 1 with dp_force: reduce-scatter / all-reduce,
    the side-stream waits on the async work handles, the sliced overlapped update, the
    bf16 all-gather and the per-bucket forward gating all execute on the MI355X.  With
    one rank every collective is an identity and the fused update is elementwise, so the
    weights must equal the plain single-GPU run bit for bit.  graph=1 replays the
    forward / backward as HIP-graph segments cut around the bucket collectives and waits
    (step 1 eager, step 2 captures, steps 3-5 replay)."""
    steps = 5
    out = str(tmp_path / "w")
    extra = [("dp_mode", mode), ("dp_bucket_mb", "0.002"), ("cuda_graph", str(graph))]
    mp.spawn(_worker, args=(1, _free_port(), steps, out, extra, "nccl"), nprocs=1, join=True)
    r0 = torch.load(out + ".r0", weights_only=True)
    from cxxnet_amd.io.data import DataBatch
    tr = _make(8, [])
    x, y = _data(8)
    for _ in range(steps):
        tr.update(DataBatch(x.cuda(), y.cuda()))
    torch.cuda.synchronize()
    assert torch.equal(r0[: tr.net.arena.total], tr.net.arena.w.cpu())


@pytest.mark.parametrize("mode", ["shard", "allreduce"])
def test_rccl_forced_fullc_gather_fused_sgd(tmp_path, mode):
    """fullc_gather under data parallelism (RCCL, world 1 forced): the fc layers all-gather
    [in | out-grad] rows and -- their gradient being global -- take the SGD step inside the
    weight-gradient GEMM (EPI_F32_SGD), as the single-GPU path does; the conv layers' buckets
    are reduced (sharded or all-reduced).  Bit-exact against the single-GPU run."""
    steps = 4
    out = str(tmp_path / "w")
    # eager steps on both sides (a planned step -- launch list or graph -- runs the arena update)
    extra = [("dp_mode", mode), ("dp_bucket_mb", "0.002"), ("fullc_gather", "1"), ("launch_replay", "0")]
    mp.spawn(_worker, args=(1, _free_port(), steps, out, extra, "nccl"), nprocs=1, join=True)
    r0 = torch.load(out + ".r0", weights_only=True)
    from cxxnet_amd.io.data import DataBatch
    tr = _make(8, [("launch_replay", "0")])
    x, y = _data(8)
    for _ in range(steps):
        tr.update(DataBatch(x.cuda(), y.cuda()))
    torch.cuda.synchronize()
    assert len(tr.net.updater.fused_offsets) == 1  # the single-GPU run fuses the same fc step
    assert torch.equal(r0[: tr.net.arena.total], tr.net.arena.w.cpu())


@pytest.mark.parametrize("mode", ["shard", "allreduce"])
def test_rccl_forced_fullc_gather_graph_segments(tmp_path, mode):
    """cuda_graph = 1 with fullc_gather under RCCL: RCCL cannot join a capturing stream, so
    the fc layers cut the graphs around their row all-gathers (ctx.graph_cut) and every replay
    re-issues them on persistent buffers; step 1 eager (fused SGD), step 2 captures, steps 3-5
    replay.  Bit-exact against the single-GPU run."""
    steps = 5
    out = str(tmp_path / "w")
    extra = [("dp_mode", mode), ("dp_bucket_mb", "0.002"), ("fullc_gather", "1"), ("cuda_graph", "1")]
    mp.spawn(_worker, args=(1, _free_port(), steps, out, extra, "nccl"), nprocs=1, join=True)
    r0 = torch.load(out + ".r0", weights_only=True)
    from cxxnet_amd.io.data import DataBatch
    tr = _make(8, [])
    x, y = _data(8)
    for _ in range(steps):
        tr.update(DataBatch(x.cuda(), y.cuda()))
    torch.cuda.synchronize()
    assert torch.equal(r0[: tr.net.arena.total], tr.net.arena.w.cpu())
