"""Deterministic mode (deterministic = 1): two identical training runs on the GPU produce
bitwise-identical weights.  Conv weight-grad split-K goes through ordered fp32 slabs instead
of atomics, cross-block channel sums run as one ordered pass, autotuning is off.
(Reference analogue: the pairtest differential check, src/layer/pairtest_layer-inl.hpp.)"""
import pytest
import torch

from cxxnet_amd.io.data import DataBatch
from cxxnet_amd.models import load_conf
from cxxnet_amd.nnet import NetTrainer

pytestmark = pytest.mark.gpu


def _run(model, batch, steps, extra=()):
    pairs = [(k, v) for k, v in load_conf(model) if not k.startswith("metric")]
    pairs += [("batch_size", str(batch)), ("eval_train", "0"), ("silent", "1"), ("dev", "gpu"), ("seed", "3"),
              ("deterministic", "1")] + list(extra)
    tr = NetTrainer()
    for k, v in pairs:
        tr.set_param(k, v)
    tr.init_model()
    c, h, w = tr.net_cfg.input_shape
    g = torch.Generator().manual_seed(5)
    x = torch.randn(batch, c, h, w, generator=g).cuda()
    y = torch.randint(0, 1000, (batch, 1), generator=g).float().cuda()
    for _ in range(steps):
        tr.update(DataBatch(x, y))
    torch.cuda.synchronize()
    return tr.net.arena.w.clone(), tr.net.arena.m1.clone()


@pytest.fixture
def restore_modes():
    from cxxnet_amd.ops import gemm
    tune = gemm._glds_cfg["tune"]
    yield
    gemm.set_deterministic(False)
    gemm._glds_cfg["tune"] = tune


@pytest.mark.parametrize("model,batch", [("alexnet", 64), ("inception_v1", 8)])
def test_two_runs_bitwise_equal(model, batch, restore_modes):
    w1, m1 = _run(model, batch, 3)
    w2, m2 = _run(model, batch, 3)
    assert torch.equal(w1, w2)
    assert torch.equal(m1, m2)
    assert m1.abs().sum().item() > 0


def test_batch_norm_channel_sums_deterministic(restore_modes):
    from cxxnet_amd import ops
    from cxxnet_amd.ops import gemm
    gemm.set_deterministic(True)
    x = torch.randn(4096, 96, device="cuda").to(torch.bfloat16)
    outs = []
    for _ in range(3):
        st = ops.layer_ops.BNState(96, x.device)
        y = torch.empty_like(x)
        ops.layer_ops.bn_forward(x.clone(), y, torch.ones(96, device="cuda"), torch.zeros(96, device="cuda"), 1e-5, st, True)
        outs.append(st.mean.clone())
    assert all(torch.equal(outs[0], o) for o in outs[1:])
