"""Data-parallel correctness on the CPU with the gloo backend (2 ranks): a DP step over a
global batch split across ranks must equal the single-process step on the whole batch
(reference semantics: loss scaled by the GLOBAL batch, summed gradients, identical
update on every replica -- src/nnet/nnet_impl-inl.hpp:141-185)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

CONF = """
netconfig=start
layer[0->1] = conv:c1
  kernel_size = 3
  nchannel = 8
  pad = 1
layer[1->2] = relu
layer[2->3] = max_pooling
  kernel_size = 2
  stride = 2
layer[3->4] = flatten
layer[4->5] = fullc:f1
  nhidden = 16
layer[5->6] = relu
layer[6->7] = fullc:f2
  nhidden = 5
layer[7->7] = softmax
netconfig=end
input_shape = 3,8,8
random_type = xavier
momentum = 0.9
eta = 0.05
wd = 0.001
dp_bucket_mb = 0.001
"""


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _data(B):
    g = torch.Generator().manual_seed(11)
    return torch.randn(B, 3, 8, 8, generator=g), torch.randint(0, 5, (B, 1), generator=g).float()


def _make(batch, extra=()):
    from cxxnet_amd import native
    from cxxnet_amd.nnet import NetTrainer
    tr = NetTrainer()
    for k, v in list(native.rt().parse_config(CONF)) + [("batch_size", str(batch)), ("dev", "cpu"),
                                                        ("eval_train", "1"), ("metric", "error"),
                                                        ("silent", "1"), ("seed", "5")] + list(extra):
        tr.set_param(k, v)
    tr.init_model()
    return tr


def _worker(rank, world, port, steps, out, update_period, shard=0, B=8):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from cxxnet_amd.io.data import DataBatch
    extra = [("update_period", str(update_period))]
    if shard == 2:  # fullc_gather on both fc layers instead of sharding
        extra += [("fullc_gather", "1")]
    else:  # every gradient through the bucket collectives (fullc_gather off, not auto)
        extra += [("update_on_server", str(shard)), ("fullc_gather", "0")]
    tr = _make(B, extra)
    assert sum(getattr(s, "no_reduce", False) for _, s in tr.net.arena.specs) == (2 if shard == 2 else 0)
    if rank == 1:
        # different local init: the rank-0 broadcast must overwrite it
        pass
    x, y = _data(B)
    for _ in range(steps):
        tr.update(DataBatch(x, y))
    assert tr.reducer.check_consistency() == 0.0
    line = tr.evaluate(None, "train")
    tr.reducer.sync_master()
    params = [tr.net.arena.w[sp.offset:sp.offset + sp.numel].clone() for _, sp in tr.net.arena.specs]
    rec = {"w": tr.net.arena.w.clone(), "line": line, "params": params}
    torch.save(rec, out if rank == 0 else out + ".r1")
    dist.destroy_process_group()


@pytest.mark.parametrize("update_period,shard,B", [(1, 0, 8), (2, 0, 8), (1, 1, 8), (2, 1, 8), (1, 2, 8), (2, 2, 8),
                                                   (1, 0, 7), (1, 2, 7)])
def test_dp_two_ranks_equals_single_process(tmp_path, update_period, shard, B):
    """shard=1: update_on_server (reduce-scatter, sliced update, all-gather);
    shard=2: fullc_gather (fc weight gradients from all-gathered activations).
    B=7: uneven ceil split (4 + 3 rows), as the reference allows."""
    from cxxnet_amd.io.data import DataBatch
    steps = 4
    out = str(tmp_path / "dp.pt")
    mp.spawn(_worker, args=(2, _free_port(), steps, out, update_period, shard, B), nprocs=2, join=True)
    r0 = torch.load(out, weights_only=True)
    r1 = torch.load(out + ".r1", weights_only=True)
    assert torch.equal(r0["w"], r1["w"]), "replicas diverged"
    # single process, whole batch
    tr = _make(B, [("update_period", str(update_period))])
    x, y = _data(B)
    for _ in range(steps):
        tr.update(DataBatch(x, y))
    # per parameter: the 2-rank arena carries extra padding (fullc_gather segments sit on
    # world*ALIGN boundaries)
    single = [tr.net.arena.w[sp.offset:sp.offset + sp.numel] for _, sp in tr.net.arena.specs]
    assert len(single) == len(r0["params"])
    for a, b in zip(r0["params"], single):
        assert torch.allclose(a, b, rtol=1e-4, atol=1e-6)
    assert r0["line"] == tr.evaluate(None, "train")


def test_bucket_plan_covers_arena():
    from cxxnet_amd.parallel.dp import GradReducer
    tr = _make(4)
    red = GradReducer(tr.net.arena, bucket_mb=0.001)
    covered = torch.zeros(tr.net.arena.total, dtype=torch.bool)
    for b in red.buckets:
        covered[b.start:b.end] = True
    for _, s in tr.net.arena.specs:
        assert covered[s.offset:s.offset + s.numel].all()
    # buckets are in reverse layer order: the first is ready first in backward
    lis = [b.li_min for b in red.buckets]
    assert lis == sorted(lis, reverse=True)


def test_shard_bucket_plan():
    """Sharded buckets tile the arena exactly, split evenly over 4 ranks, and are
    ready in backward order."""
    from unittest import mock

    from cxxnet_amd.parallel import dp
    with mock.patch.object(dp, "world_info", return_value=(1, 4)), \
            mock.patch.object(dp.GradReducer, "broadcast_params", lambda self, src=0: None):
        tr = _make(4, [("fullc_gather", "0")])  # (auto would all-gather the fc layers at world 4)
        red = dp.GradReducer(tr.net.arena, bucket_mb=0.001, shard=True)
    assert red.shard and red.buckets[0].start == 0 and red.buckets[-1].end == tr.net.arena.total
    for a, b in zip(red.buckets, red.buckets[1:]):
        assert a.end == b.start
    for b in red.buckets:
        assert (b.end - b.start) % (64 * 4) == 0
    lis = [b.li_min for b in red.buckets]
    assert lis == sorted(lis, reverse=True)
    own = red.owned_ranges()
    assert all(hi - lo == (b.end - b.start) // 4 for (lo, hi), b in zip(own, red.buckets))
