"""fc -> relu -> dropout -> fc fused on the GPU (NeuralNet._fuse_dropout: the dropout mask in
the fc forward's split-K finalize or a separate dropout launch, the 1 / pkeep scale in the next
fc's data-gradient epilogue) against the unfused layers: one training step must give bitwise
the same weights (pkeep = 0.5: the scale is a power of two, so rounding cannot differ), at a
batch that takes the split-K path (256) and one that does not (8)."""
import pytest
import torch

from cxxnet_amd import native
from cxxnet_amd.io.data import DataBatch
from cxxnet_amd.nnet import NetTrainer

pytestmark = pytest.mark.gpu

NET = """
netconfig=start
layer[0->1] = flatten
layer[1->2] = fullc:f1
  nhidden = 1024
layer[2->3] = relu
layer[3->3] = dropout
  threshold = 0.5
layer[3->4] = fullc:f2
  nhidden = 512
layer[4->5] = relu
layer[5->5] = dropout
  threshold = 0.5
layer[5->6] = fullc:f3
  nhidden = 16
layer[6->6] = softmax
netconfig=end
input_shape = 4,16,16
"""


def _step(batch, fuse, monkeypatch):
    monkeypatch.setenv("CXXNET_FUSE_DROPOUT", fuse)
    tr = NetTrainer()
    for k, v in list(native.rt().parse_config(NET)) + [("batch_size", str(batch)), ("dev", "gpu"), ("seed", "3"),
                                                       ("eval_train", "0"), ("silent", "1"), ("eta", "0.1"),
                                                       ("deterministic", "1")]:
        tr.set_param(k, v)
    tr.init_model()
    drops = [c.layer for c in tr.net.connections if type(c.layer).__name__ == "DropoutLayer"]
    assert all(d.fused_into_producer == (fuse == "1") for d in drops)
    g = torch.Generator().manual_seed(1)
    x = torch.randn(batch, 4, 16, 16, generator=g).cuda()
    y = torch.randint(0, 16, (batch, 1), generator=g).float().cuda()
    for _ in range(2):
        tr.update(DataBatch(x, y))
    torch.cuda.synchronize()
    return tr.net.arena.w.clone()


@pytest.mark.parametrize("batch", [256, 8])
def test_fused_dropout_bitwise(batch, monkeypatch):
    # the heuristic tile for every shape (no per-process timing): both nets then run the same
    # split-K decomposition, whatever the timing of the first one's shapes said
    from cxxnet_amd.ops import gemm
    monkeypatch.setitem(gemm._glds_cfg, "tune", False)
    a = _step(batch, "0", monkeypatch)
    b = _step(batch, "1", monkeypatch)
    assert torch.equal(a, b), (a - b).abs().max().item()
