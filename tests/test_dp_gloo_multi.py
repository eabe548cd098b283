"""Data parallelism at 4 and 8 ranks on the CPU (gloo): every reduction mode must equal the
single-process step on the whole global batch, replicas must stay bit-identical, and the
sharded mode's save path (a collective on every rank) must write the same model and
optimizer state as the replicated mode.  Also the reference's device pruning
(src/nnet/nnet_impl-inl.hpp:344-354): batch_size=10 over 8 devices uses 5, and a rank beyond
the pruned count (torchrun started with 8) idles with zero gradients."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from test_dp_gloo import CONF, _data, _make


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, steps, out, mode, update_period, B, save_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    if mode == "shard_inplace":
        os.environ["CXXNET_DP_INPLACE"] = "1"
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from cxxnet_amd.io.data import DataBatch
    extra = [("update_period", str(update_period))]
    if mode in ("shard", "shard_inplace"):
        extra += [("dp_mode", "shard")]
    elif mode == "gather":
        extra += [("fullc_gather", "1")]
    elif mode == "shard_gather":  # sharded conv buckets + all-gathered fc layers
        extra += [("fullc_gather", "1"), ("dp_mode", "shard")]
    elif mode == "auto":  # fullc_gather left at its default (auto: gather when fewer bytes move)
        extra += [("dp_mode", "allreduce")]
    else:
        extra += [("dp_mode", "allreduce")]
    if mode in ("allreduce", "shard", "shard_inplace"):
        extra += [("fullc_gather", "0")]  # every gradient through the bucket collectives
    tr = _make(B, extra)
    assert tr.reducer.shard == (mode in ("shard", "shard_inplace", "shard_gather"))
    if "gather" in mode:
        assert len(tr.reducer.extra_ranges) == 2  # both fc weight matrices
    elif mode == "auto":
        # f1 (128 -> 16) gathers: 4 ranks x 3 rows x 144 values x 2 B < 128 x 16 x 4 B of gradient;
        # f2 (16 -> 5) does not: 504 B of rows against 320 B of gradient
        assert len(tr.reducer.extra_ranges) == 1
    else:
        assert not tr.reducer.extra_ranges
    if mode == "shard_inplace":
        assert tr.reducer.inplace
    x, y = _data(B)
    for _ in range(steps):
        tr.update(DataBatch(x, y))
    assert tr.reducer.check_consistency() == 0.0
    line = tr.evaluate(None, "train")
    # the CLI's save protocol: the collective part on every rank, then rank 0 serialises
    tr.prepare_save(opt_state=True)
    blob = tr.save_model(sync=False) if rank == 0 else None
    if rank == 0:
        tr.save_optimizer_state(os.path.join(save_dir, "opt.state"), sync=False)
    a = tr.net.arena
    if rank == 0:
        torch.save([(sp.offset, sp.numel) for _, sp in a.specs], os.path.join(save_dir, "layout.pt"))
    torch.save({"w": a.w.clone(), "m1": a.m1.clone(), "line": line, "params": _params(tr), "blob": blob,
                "idle": tr.idle, "active": tr.active_ranks()}, f"{out}.r{rank}")
    dist.destroy_process_group()


def _params(tr):
    """Per-parameter fp32 master weights (the arena layout differs between world sizes:
    fullc_gather segments sit on world*ALIGN boundaries)."""
    return [tr.net.arena.w[s.offset:s.offset + s.numel].clone() for _, s in tr.net.arena.specs]


def _opt_params(tr, m1):
    return [m1[s.offset:s.offset + s.numel] for _, s in tr.net.arena.specs]


def _make_world_layout(tmp_path, world):
    return torch.load(str(tmp_path / "layout.pt"), weights_only=True)


def _close(a, b):
    return len(a) == len(b) and all(torch.allclose(x, y, rtol=1e-4, atol=1e-6) for x, y in zip(a, b))


def _run(tmp_path, world, mode, update_period, B, steps=3):
    out = str(tmp_path / "dp")
    mp.spawn(_worker, args=(world, _free_port(), steps, out, mode, update_period, B, str(tmp_path)),
             nprocs=world, join=True)
    return [torch.load(f"{out}.r{r}", weights_only=True) for r in range(world)]


def _single(B, update_period, steps=3):
    from cxxnet_amd.io.data import DataBatch
    tr = _make(B, [("update_period", str(update_period))])
    x, y = _data(B)
    for _ in range(steps):
        tr.update(DataBatch(x, y))
    return tr


@pytest.mark.parametrize("world,mode,update_period,B", [
    (4, "allreduce", 1, 10),      # uneven ceil split 3+3+3+1
    (4, "shard", 2, 12),          # sharded, gradient accumulation
    (4, "gather", 1, 10),         # fullc_gather, uneven
    (8, "shard_inplace", 1, 16),  # RCCL's in-place reduce-scatter / all-gather layout, on gloo
    (8, "allreduce", 2, 17),      # ceil split 3*5+2, update_period 2
    (8, "gather", 1, 16),
    (4, "shard_gather", 1, 10),   # fullc_gather composed with the sharded update
    (8, "shard_gather", 2, 16),
    (4, "auto", 1, 10),           # the default: fullc_gather = auto picks the gather for both fc layers
])
def test_dp_multi_rank_equals_single_process(tmp_path, world, mode, update_period, B):
    rs = _run(tmp_path, world, mode, update_period, B)
    for r in rs[1:]:
        assert torch.equal(rs[0]["w"], r["w"]), "replicas diverged"
    tr = _single(B, update_period)
    assert _close(rs[0]["params"], _params(tr))
    assert rs[0]["line"] == tr.evaluate(None, "train")
    assert rs[0]["blob"] is not None
    # optimizer state: sharded mode gathers every rank's momentum slice before the save; the
    # saved state is in the multi-rank arena layout, compared per parameter
    m1 = torch.load(str(tmp_path / "opt.state"), weights_only=True)["m1_params"]
    keys = [f"{li}:{s.tag}" for li, s in tr.net.arena.specs]
    assert _close([m1[k] for k in keys], _opt_params(tr, tr.net.arena.m1))


def test_device_pruning_rule():
    from cxxnet_amd.nnet.trainer import prune_devices
    # reference: step = ceil(B / ndev); drop devices while step * (ndev - 1) >= B
    assert prune_devices(10, 8) == 5
    assert prune_devices(256, 8) == 8
    assert prune_devices(9, 8) == 5
    assert prune_devices(3, 8) == 3
    assert prune_devices(1, 8) == 1
    assert prune_devices(5, 4) == 3
    assert prune_devices(7, 4) == 4


def test_idle_ranks_batch10_world8(tmp_path):
    """torchrun with 8 ranks and batch_size = 10: ranks 0-4 hold 2 rows each, ranks 5-7 idle
    (stand-in rows, zero loss weight) -- the result equals the single-process step."""
    rs = _run(tmp_path, 8, "allreduce", 1, 10)
    assert [r["idle"] for r in rs] == [False] * 5 + [True] * 3
    assert all(r["active"] == 5 for r in rs)
    for r in rs[1:]:
        assert torch.equal(rs[0]["w"], r["w"])
    tr = _single(10, 1)
    assert _close(rs[0]["params"], _params(tr))
    assert rs[0]["line"] == tr.evaluate(None, "train")


def test_cli_launcher_prunes_devices(tmp_path, monkeypatch):
    """cxxnet conf dev=gpu:0-7 batch_size=10 launches 5 ranks (reference warning printed)."""
    from cxxnet_amd import cli
    conf = tmp_path / "a.conf"
    conf.write_text("dev = gpu:0-7\nbatch_size = 10\n")
    seen = {}

    def fake_call(cmd, env=None):
        seen["cmd"], seen["env"] = cmd, env
        return 0
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(cli.subprocess, "call", fake_call)
    assert cli._maybe_spawn_ranks([str(conf)]) == 0
    assert "--nproc-per-node=5" in seen["cmd"]
    assert seen["env"]["HIP_VISIBLE_DEVICES"] == "0,1,2,3,4"
    # batch 1 over 8 devices: one device, no launcher
    assert cli._maybe_spawn_ranks([str(conf), "batch_size=1"]) is None


def test_merge_tune_timings():
    from cxxnet_amd.ops.gemm import merge_tune_timings
    r0 = {"cf|a": {1: 10.0, 7: 9.0}, "cf|b": {1: 5.0}}
    r1 = {"cf|a": {1: 8.0, 7: 12.0}, "cd|c": {10: 3.0, 15: 2.0}}
    m = merge_tune_timings([r0, r1])
    assert m == {"cf|a": 1, "cf|b": 1, "cd|c": 15}  # cf|a: 18 vs 21 summed
    # a tile only one rank could run is not eligible when the ranks share another
    m2 = merge_tune_timings([{"k": {1: 5.0, 2: 1.0}}, {"k": {1: 6.0}}])
    assert m2 == {"k": 1}


def _tune_worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from cxxnet_amd.ops import gemm
    # mocked per-rank timings: each rank alone would pick a different tile
    gemm.TUNED_HERE.clear()
    gemm.TUNED_HERE["cf|x"] = {1: 1.0 + rank, 7: 2.5 - rank}
    gemm._TUNE["cf|x"] = min(gemm.TUNED_HERE["cf|x"], key=gemm.TUNED_HERE["cf|x"].get)
    local = gemm._TUNE["cf|x"]
    gemm.sync_tune_table()
    torch.save({"local": local, "synced": gemm._TUNE["cf|x"]}, f"{out}.r{rank}")
    dist.destroy_process_group()


def test_tile_choice_is_rank_consistent(tmp_path):
    """Ranks whose own timings disagree adopt one tile (sum of times over the ranks)."""
    out = str(tmp_path / "tune")
    mp.spawn(_tune_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    r = [torch.load(f"{out}.r{i}", weights_only=True) for i in range(2)]
    assert r[0]["local"] != r[1]["local"]
    assert r[0]["synced"] == r[1]["synced"] == 1  # 1.0 + 2.0 = 3.0 < 2.5 + 1.5 = 4.0
