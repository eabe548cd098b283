"""fc weight-gradient GEMM fused with the SGD step (FullConnectLayer._fused_sgd,
gemm_glds EPI_F32_SGD): the fused path must give bitwise the weights, momentum and bf16
shadow of the unfused path (gradient stored, then the fused optimizer launch), with
momentum, weight decay, gradient clipping and a learning-rate schedule, through a relu-fused
fc -> relu -> fc chain (relu' applied by the scratch copy-back) and an fc whose shape the
kernel does not cover (fallback)."""
import pytest
import torch

from cxxnet_amd import native
from cxxnet_amd.io.data import DataBatch
from cxxnet_amd.nnet import NetTrainer
from cxxnet_amd.nnet import trainer as trainer_mod

pytestmark = pytest.mark.gpu

CONF = """
netconfig=start
layer[0->1] = conv:c1
  kernel_size = 3
  nchannel = 16
  pad = 1
layer[1->2] = relu
layer[2->3] = flatten
layer[3->4] = fullc:f1
  nhidden = 96
layer[4->5] = relu
layer[5->6] = fullc:f2
  nhidden = 36
layer[6->7] = relu
layer[7->8] = fullc:f3
  nhidden = 10
layer[8->8] = softmax
netconfig=end
input_shape = 3,8,8
"""


def _train(fuse, steps, extra):
    trainer_mod._FUSE_FC_SGD = fuse
    tr = NetTrainer()
    for k, v in list(native.rt().parse_config(CONF)) + [("batch_size", "32"), ("dev", "gpu"), ("eval_train", "0"),
                                                        ("silent", "1"), ("seed", "3"), ("cuda_graph", "0"),
                                                        ("deterministic", "1")] + extra:
        tr.set_param(k, v)
    tr.init_model()
    g = torch.Generator().manual_seed(1)
    for _ in range(steps):
        x = torch.randn(32, 3, 8, 8, generator=g)
        y = torch.randint(0, 10, (32, 1), generator=g).float()
        tr.update(DataBatch(x.cuda(), y.cuda()))
    torch.cuda.synchronize()
    a = tr.net.arena
    return tr, a.w.clone(), a.m1.clone(), a.wb.clone()


@pytest.mark.parametrize("extra", [
    [("eta", "0.05"), ("momentum", "0.9"), ("wd", "0.0005")],
    [("eta", "0.1"), ("momentum", "0.5"), ("wd", "0.001"), ("clip_gradient", "0.01"), ("lr:schedule", "expdecay"),
     ("lr:gamma", "0.5"), ("lr:step", "2")],
])
def test_fused_fc_sgd_is_bitwise_the_unfused_step(extra):
    saved = trainer_mod._FUSE_FC_SGD
    try:
        tr, w1, m1, b1 = _train(True, 5, extra)
        assert tr._sgd_fuse_target()[0] is not None
        _, w0, m0, b0 = _train(False, 5, extra)
    finally:
        trainer_mod._FUSE_FC_SGD = saved
    assert torch.equal(w1, w0), (w1 - w0).abs().max().item()
    assert torch.equal(m1, m0)
    assert torch.equal(b1, b0)
    assert (m1 != 0).any()


def test_fusion_off_for_other_updaters():
    tr, *_ = _train(True, 1, [("updater", "nag")])
    assert tr._sgd_fuse_target()[0] is None


def test_fused_fc_sgd_on_side_stream_is_bitwise(monkeypatch):
    """CXXNET_FC_SGD_SIDE=1: the fused fc steps run on a side stream overlapping the backward
    below them (x copied aside, data gradient first on the main stream, joined at the end of the
    pass) and give bitwise the main-stream result."""
    extra = [("eta", "0.05"), ("momentum", "0.9"), ("wd", "0.0005")]
    saved = trainer_mod._FUSE_FC_SGD
    try:
        monkeypatch.setenv("CXXNET_FC_SGD_SIDE", "1")
        tr, w1, m1, b1 = _train(True, 5, extra)
        assert getattr(tr.net, "_fc_side", None) is not None, "the side stream was not used"
        monkeypatch.setenv("CXXNET_FC_SGD_SIDE", "0")
        _, w0, m0, b0 = _train(True, 5, extra)
    finally:
        trainer_mod._FUSE_FC_SGD = saved
    assert torch.equal(w1, w0), (w1 - w0).abs().max().item()
    assert torch.equal(m1, m0)
    assert torch.equal(b1, b0)
