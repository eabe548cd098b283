"""Max pooling on integer keys for inputs that can only be >= 0 (NeuralNet._mark_nonneg ->
PoolingLayer.input_nonneg -> ops.pool_forward(nonneg=True)): which pools qualify (CPU) and
bitwise equality with the float-compare kernels on tie-heavy inputs with signed zeros (GPU)."""
import pytest
import torch

from cxxnet_amd import ops
from cxxnet_amd.models import load_conf
from cxxnet_amd.nnet import NetTrainer


def _net(model, batch):
    tr = NetTrainer()
    for k, v in load_conf(model, [("batch_size", str(batch)), ("dev", "cpu")]):
        if not k.startswith("metric"):
            tr.set_param(k, v)
    tr.init_model()
    return tr.net


@pytest.mark.parametrize("model", ["alexnet", "inception_v1", "vgg16"])
def test_every_max_pool_after_relu_is_marked(model):
    net = _net(model, 2)
    pools = [c.layer for c in net.connections if type(c.layer).__name__ == "PoolingLayer" and c.layer.mode == "max"]
    assert pools and all(p.input_nonneg for p in pools)


def test_pool_on_unrectified_input_is_not_marked():
    from cxxnet_amd import native
    conf = """
netconfig=start
layer[0->1] = conv:c1
  kernel_size = 3
  nchannel = 8
layer[1->2] = max_pooling
  kernel_size = 2
  stride = 2
layer[2->3] = relu
layer[3->4] = max_pooling
  kernel_size = 2
  stride = 2
layer[4->5] = flatten
layer[5->6] = fullc:f
  nhidden = 4
layer[6->6] = softmax
netconfig=end
input_shape = 3,12,12
"""
    tr = NetTrainer()
    for k, v in list(native.rt().parse_config(conf)) + [("batch_size", "2"), ("dev", "cpu")]:
        tr.set_param(k, v)
    tr.init_model()
    pools = [c.layer for c in tr.net.connections if type(c.layer).__name__ == "PoolingLayer"]
    assert [p.input_nonneg for p in pools] == [False, True]


def test_in_place_writer_after_relu_clears_the_mark():
    """relu -> in-place batch_norm (a self-loop that can make values negative) -> max_pool: the
    pool must take the float-compare path."""
    from cxxnet_amd import native
    conf = """
netconfig=start
layer[0->1] = conv:c1
  kernel_size = 3
  nchannel = 8
layer[1->2] = relu
layer[2->2] = batch_norm
layer[2->3] = max_pooling
  kernel_size = 2
  stride = 2
layer[3->4] = flatten
layer[4->5] = fullc:f
  nhidden = 4
layer[5->5] = softmax
netconfig=end
input_shape = 3,12,12
"""
    tr = NetTrainer()
    for k, v in list(native.rt().parse_config(conf)) + [("batch_size", "2"), ("dev", "cpu")]:
        tr.set_param(k, v)
    tr.init_model()
    pools = [c.layer for c in tr.net.connections if type(c.layer).__name__ == "PoolingLayer"]
    assert [p.input_nonneg for p in pools] == [False]


@pytest.mark.gpu
@pytest.mark.parametrize("K,S,P,H", [(3, 2, 0, 27), (3, 1, 1, 14), (2, 2, 0, 28), (3, 2, 0, 13)])
def test_integer_key_pool_matches_float_compare(K, S, P, H):
    N, C = 3, 64
    g = torch.Generator(device="cuda").manual_seed(K * 10 + H)
    vals = torch.tensor([0.0, -0.0, 1.0, 2.0, 0.5], device="cuda")
    x = vals[torch.randint(0, 5, (N, H, H, C), generator=g, device="cuda")].to(torch.bfloat16)
    Ho = (H + 2 * P - K) // S + 1
    if S > 1:
        Ho = min(H + 2 * P - K + S - 1, H + 2 * P - 1) // S + 1  # the layer's ceil mode
    out = {}
    for nn in (False, True):
        y = torch.empty(N, Ho, Ho, C, device="cuda", dtype=torch.bfloat16)
        st = torch.empty(N, Ho, Ho, C, device="cuda", dtype=torch.uint8)
        ops.pool_forward(x, y, st, K, K, S, P, "max", mark_mask=True, nonneg=nn)
        out[nn] = (y.float(), st.clone())
    assert torch.equal(out[False][0], out[True][0])
    assert torch.equal(out[False][1], out[True][1])


def test_lrn_bias_fusion_targets(monkeypatch):
    """NeuralNet._fuse_lrn_bias: GoogLeNet's norm2 sums conv2's bias gradient (conv2 -> relu ->
    norm2, the relu fused); AlexNet's LRNs follow max-pools and take no conv."""
    monkeypatch.setenv("CXXNET_FUSE", "2")  # the GPU's graph fusion on a CPU net
    goog = _net("inception_v1", 2)
    lrns = [c.layer for c in goog.connections if type(c.layer).__name__ == "LRNLayer"]
    tied = [l for l in lrns if l.bias_of is not None]
    assert len(tied) == 1 and tied[0].bias_of.b is not None and tied[0].bias_of.geo.KH == 3
    alex = _net("alexnet", 2)
    assert all(c.layer.bias_of is None for c in alex.connections if type(c.layer).__name__ == "LRNLayer")


@pytest.mark.parametrize("model,batch,expect", [("vgg16", 64, 2), ("alexnet", 256, 0), ("inception_v1", 128, 0)])
def test_dgrad_bias_auto_takes_only_large_layers(monkeypatch, model, batch, expect):
    """NeuralNet._fuse_dgrad_bias in its default ("auto") mode: only a conv whose output
    gradient is >= 150 MB has its bias summed by the upper conv's data-gradient epilogue --
    VGG-16's conv1_1 and conv2_1 at batch 64, nothing in AlexNet or GoogLeNet."""
    monkeypatch.setenv("CXXNET_FUSE", "2")
    monkeypatch.delenv("CXXNET_DGRAD_BIAS", raising=False)
    net = _net(model, batch)
    below = [c.layer.bias_below for c in net.connections if getattr(c.layer, "bias_below", None) is not None]
    assert len(below) == expect


def test_bias_fusions_skip_sibling_groups(monkeypatch):
    """A sibling group (GoogLeNet's 1x1 convs on one input) sums its biases over its shared
    buffer, so no other layer may take a member's bias: with every dgrad-bias fusion forced on,
    no pool / LRN / conv names a sibling member or lead as its bias target."""
    monkeypatch.setenv("CXXNET_FUSE", "2")
    monkeypatch.setenv("CXXNET_DGRAD_BIAS", "1")
    net = _net("inception_v1", 2)
    targets = [t for c in net.connections for t in (getattr(c.layer, "bias_below", None),
                                                     getattr(c.layer, "bias_of", None)) if t is not None]
    assert targets
    assert not any(getattr(t, "sib", None) or getattr(t, "sib_member", False) for t in targets)
