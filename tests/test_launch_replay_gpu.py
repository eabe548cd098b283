"""The native launch-list executor (csrc/kernels/launch_list.hip, NetTrainer._list_step): a step
recorded once into C++ launch lists and replayed must produce bit-identical weights to the eager
Python executor, on one GPU and on the data-parallel path (RCCL at world 1: bucket collectives,
side-stream updates and fullc_gather all-gathers run eagerly between the replayed segments)."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from test_dp_gloo import CONF

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _unfused_fc_sgd():
    """Both arms take the same fc path: the eager step would otherwise fuse the fc SGD step
    into a one-slice weight-grad GEMM while a planned step runs the arena update after the
    (possibly split-K) GEMM -- equal math, different fp32 summation order."""
    from cxxnet_amd.nnet import trainer as trainer_mod
    saved = trainer_mod._FUSE_FC_SGD
    trainer_mod._FUSE_FC_SGD = False
    yield
    trainer_mod._FUSE_FC_SGD = saved


def _make(batch, extra=(), conf=None, model=None):
    from cxxnet_amd import native
    from cxxnet_amd.models import load_conf
    from cxxnet_amd.nnet import NetTrainer
    tr = NetTrainer()
    base = list(native.rt().parse_config(conf or CONF)) if model is None else \
        [(k, v) for k, v in load_conf(model, []) if not k.startswith("metric")]
    # deterministic: no fp32 atomics in the weight gradients, so the arms can agree bit for bit
    for k, v in base + [("batch_size", str(batch)), ("dev", "gpu"), ("eval_train", "0"), ("silent", "1"),
                        ("seed", "5"), ("cuda_graph", "0"), ("deterministic", "1")] + list(extra):
        tr.set_param(k, v)
    tr.init_model()
    return tr


def _data(B, shape=(3, 8, 8), ncls=5):
    g = torch.Generator().manual_seed(11)
    return torch.randn(B, *shape, generator=g), torch.randint(0, ncls, (B, 1), generator=g).float()


def _train(tr, x, y, steps):
    from cxxnet_amd.io.data import DataBatch
    for _ in range(steps):
        tr.update(DataBatch(x.cuda(), y.cuda()))
    torch.cuda.synchronize()
    return tr.net.arena.w.cpu()


def test_replay_equals_eager_small_net():
    x, y = _data(8)
    w_eager = _train(_make(8, [("launch_replay", "0")]), x, y, 5)
    tr = _make(8, [("launch_replay", "1")])
    w_rep = _train(tr, x, y, 5)
    assert tr._lists, "the step was not recorded"
    fwd, bwd = tr._lists[8][:2]
    assert sum(getattr(i, "n", 0) for i in fwd + bwd) > 5
    assert torch.equal(w_eager, w_rep)


@pytest.mark.parametrize("model,batch", [("alexnet", 16), ("inception_v1", 8)])
def test_replay_equals_eager_models(model, batch):
    """Real graphs: dropout (device step counter), LRN, concat, fused epilogues, fc SGD off."""
    from cxxnet_amd.models import load_conf
    shape = tuple(int(v) for v in dict(load_conf(model, [])).get("input_shape", "3,227,227").split(","))
    x, y = _data(batch, shape, 1000)
    w_eager = _train(_make(batch, [("launch_replay", "0")], model=model), x, y, 4)
    tr = _make(batch, [("launch_replay", "1")], model=model)
    w_rep = _train(tr, x, y, 4)
    assert tr._lists
    assert torch.equal(w_eager, w_rep)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, port, steps, out, extra):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1",
                      LOCAL_RANK="0", CXXNET_DIST_BACKEND="nccl", CXXNET_DIST_FORCE="1")
    import torch.distributed as dist
    from cxxnet_amd.nnet import trainer as trainer_mod
    from cxxnet_amd.parallel import init_distributed
    trainer_mod._FUSE_FC_SGD = False  # as the parent's arm (spawned: the fixture does not reach here)
    init_distributed()
    tr = _make(8, extra)
    x, y = _data(8)
    w = _train(tr, x, y, steps)
    assert tr._lists and not tr._graphs
    tr.reducer.sync_master()
    torch.save(tr.net.arena.w.cpu(), out)
    dist.destroy_process_group()


@pytest.mark.parametrize("extra", [
    [("dp_mode", "allreduce"), ("fullc_gather", "0")],
    [("dp_mode", "shard"), ("fullc_gather", "0")],
    [("dp_mode", "allreduce"), ("fullc_gather", "1")],
], ids=["allreduce", "shard", "gather"])
def test_replay_data_parallel_rccl_world1(tmp_path, extra):
    steps = 5
    out = str(tmp_path / "w.pt")
    ex = extra + [("dp_bucket_mb", "0.002"), ("launch_replay", "1")]
    mp.spawn(_worker, args=(_free_port(), steps, out, ex), nprocs=1, join=True)
    r0 = torch.load(out, weights_only=True)
    x, y = _data(8)
    w = _train(_make(8, [("launch_replay", "0")]), x, y, steps)
    assert torch.equal(r0[: w.numel()], w)
