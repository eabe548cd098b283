"""Executor + layer semantics on the CPU path against independent torch autograd models.

The torch models restate the reference semantics (ceil-mode pooling, cross-channel
LRN with knorm, in-place activations, loss gradient scaled by 1/batch) directly with
autograd, so a wiring or formula error in any layer shows up as a gradient mismatch.
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from cxxnet_amd import native
from cxxnet_amd.io.data import DataBatch
from cxxnet_amd.nnet import NetTrainer


def make(conf, batch, extra=()):
    tr = NetTrainer()
    for k, v in list(native.rt().parse_config(conf)) + [("batch_size", str(batch)), ("dev", "cpu"),
                                                        ("eval_train", "0"), ("silent", "1")] + list(extra):
        tr.set_param(k, v)
    tr.init_model()
    return tr


def grads_of(tr, x, y):
    tr.net.set_input(x)
    tr.net.set_labels(y)
    tr.net.forward(True)
    tr.net.backprop(False)
    return {(li, s.tag): s.g.clone() for li, s in tr.net.arena.specs}


def weights(tr, li, tag):
    for l, s in tr.net.arena.specs:
        if l == li and s.tag == tag:
            return s.w.clone()
    raise KeyError((li, tag))


def lrn_ref(x, n, alpha, beta, knorm):
    sq = (x * x)
    half = n // 2
    pad = F.pad(sq, (0, 0, 0, 0, half, half))
    s = sum(pad[:, i:i + x.shape[1]] for i in range(n))
    return x * (knorm + alpha / n * s).pow(-beta)


CONV_NET = """
netconfig=start
layer[0->1] = conv:c1
  kernel_size = 3
  stride = 2
  nchannel = 8
  pad = 1
layer[1->2] = relu
layer[2->3] = max_pooling
  kernel_size = 3
  stride = 2
layer[3->4] = lrn
  local_size = 5
  alpha = 0.01
  beta = 0.75
  knorm = 2
layer[4->5] = conv:c2
  kernel_size = 3
  nchannel = 6
  ngroup = 2
  pad = 1
layer[5->6] = tanh
layer[6->7] = avg_pooling
  kernel_size = 2
  stride = 2
layer[7->8] = flatten
layer[8->9] = fullc:f1
  nhidden = 12
layer[9->10] = sigmoid
layer[10->11] = fullc:f2
  nhidden = 5
layer[11->11] = softmax
netconfig=end
input_shape = 4,15,15
random_type = xavier
init_bias = 0.1
"""


def test_conv_net_gradients_match_autograd():
    B = 3
    tr = make(CONV_NET, B)
    g = torch.Generator().manual_seed(0)
    x = torch.randn(B, 4, 15, 15, generator=g)
    y = torch.randint(0, 5, (B, 1), generator=g).float()
    ours = grads_of(tr, x, y)

    # independent autograd model with the same weights (logical layouts)
    def conv_w(li):
        layer = tr.net.connections[li].layer
        w = layer.to_logical(weights(tr, li, "wmat"))  # (G, Cout/G, Cg*k*k)
        lp = layer.lp
        return w.reshape(lp.num_channel, lp.num_input_channel // lp.num_group, lp.kernel_height,
                         lp.kernel_width).requires_grad_(True)
    w1, w2 = conv_w(0), conv_w(4)
    b1 = weights(tr, 0, "bias").requires_grad_(True)
    b2 = weights(tr, 4, "bias").requires_grad_(True)
    wf1 = weights(tr, 8, "wmat").requires_grad_(True)
    bf1 = weights(tr, 8, "bias").requires_grad_(True)
    wf2 = weights(tr, 10, "wmat").requires_grad_(True)
    bf2 = weights(tr, 10, "bias").requires_grad_(True)
    h = F.relu(F.conv2d(x, w1, b1, stride=2, padding=1))
    h = F.max_pool2d(h, 3, 2, ceil_mode=True)
    h = lrn_ref(h, 5, 0.01, 0.75, 2.0)
    h = torch.tanh(F.conv2d(h, w2, b2, padding=1, groups=2))
    h = F.avg_pool2d(h, 2, 2, ceil_mode=True)
    h = h.reshape(B, -1)
    h = torch.sigmoid(h @ wf1.t() + bf1)
    logits = h @ wf2.t() + bf2
    loss = F.cross_entropy(logits, y.long().view(-1), reduction="sum") / B
    loss.backward()

    def cmp(key, ref):
        got = ours[key]
        assert torch.allclose(got.reshape(ref.shape), ref, rtol=1e-3, atol=1e-5), \
            (key, (got.reshape(ref.shape) - ref).abs().max().item())

    layer0 = tr.net.connections[0].layer
    layer4 = tr.net.connections[4].layer
    cmp((0, "wmat"), layer0.from_logical(w1.grad.reshape(1, 8, -1)))
    cmp((0, "bias"), b1.grad)
    cmp((4, "wmat"), layer4.from_logical(w2.grad.reshape(2, 3, -1)))
    cmp((4, "bias"), b2.grad)
    cmp((8, "wmat"), wf1.grad)
    cmp((8, "bias"), bf1.grad)
    cmp((10, "wmat"), wf2.grad)
    cmp((10, "bias"), bf2.grad)


def test_prop_to_input_and_dropout_identity_at_test():
    conf = """
netconfig=start
layer[+1] = fullc:f1
  nhidden = 7
layer[+0] = dropout
  threshold = 0.5
layer[+1] = fullc:f2
  nhidden = 3
layer[+0] = softmax
netconfig=end
input_shape = 1,1,5
"""
    tr = make(conf, 4)
    x = torch.randn(4, 1, 1, 5)
    y = torch.zeros(4, 1)
    tr.net.set_input(x)
    tr.net.set_labels(y)
    tr.net.forward(False)
    p1 = tr.net.nodes[-1].fp32_view.clone()
    tr.net.forward(False)
    assert torch.equal(p1, tr.net.nodes[-1].fp32_view)  # dropout is identity at test time
    assert torch.allclose(p1.sum(1), torch.ones(4))


def test_relu_max_pooling_and_sum_pooling():
    conf = """
netconfig=start
layer[0->1] = relu_max_pooling
  kernel_size = 3
  stride = 2
layer[1->2] = sum_pooling
  kernel_size = 2
  stride = 1
layer[2->3] = flatten
layer[3->4] = fullc:f
  nhidden = 4
layer[4->4] = softmax
netconfig=end
input_shape = 2,9,9
"""
    B = 2
    tr = make(conf, B)
    x = torch.randn(B, 2, 9, 9)
    y = torch.tensor([[1.0], [3.0]])
    ours = grads_of(tr, x, y)
    wf = weights(tr, 3, "wmat").requires_grad_(True)
    bf = weights(tr, 3, "bias").requires_grad_(True)
    h = F.max_pool2d(F.relu(x), 3, 2, ceil_mode=True)
    h = F.avg_pool2d(h, 2, 1, ceil_mode=True) * 4
    logits = h.reshape(B, -1) @ wf.t() + bf
    loss = F.cross_entropy(logits, y.long().view(-1), reduction="sum") / B
    loss.backward()
    assert torch.allclose(ours[(3, "wmat")], wf.grad, rtol=1e-4, atol=1e-6)
    assert torch.allclose(ours[(3, "bias")], bf.grad, rtol=1e-4, atol=1e-6)


def test_batch_norm_and_prelu_gradients():
    conf = """
netconfig=start
layer[0->1] = conv:c
  kernel_size = 3
  nchannel = 4
layer[1->2] = batch_norm:bn
layer[2->3] = prelu:pr
layer[3->4] = flatten
layer[4->5] = fullc:f
  nhidden = 3
layer[5->5] = softmax
netconfig=end
input_shape = 2,6,6
"""
    B = 4
    tr = make(conf, B)
    x = torch.randn(B, 2, 6, 6)
    y = torch.randint(0, 3, (B, 1)).float()
    ours = grads_of(tr, x, y)
    layer0 = tr.net.connections[0].layer
    w = layer0.to_logical(weights(tr, 0, "wmat")).reshape(4, 2, 3, 3).requires_grad_(True)
    b = weights(tr, 0, "bias").requires_grad_(True)
    slope = weights(tr, 1, "wmat").requires_grad_(True)
    bias = weights(tr, 1, "bias").requires_grad_(True)
    pr = weights(tr, 2, "bias").requires_grad_(True)
    wf = weights(tr, 4, "wmat").requires_grad_(True)
    bf = weights(tr, 4, "bias").requires_grad_(True)
    h = F.conv2d(x, w, b)
    mean = h.mean((0, 2, 3), keepdim=True)
    var = ((h - mean) ** 2).mean((0, 2, 3), keepdim=True)
    h = (h - mean) / torch.sqrt(var + 1e-10) * slope.view(1, -1, 1, 1) + bias.view(1, -1, 1, 1)
    h = torch.where(h > 0, h, h * pr.clamp(0, 1).view(1, -1, 1, 1))
    # the net flattens in NCHW order
    logits = h.reshape(B, -1) @ wf.t() + bf
    loss = F.cross_entropy(logits, y.long().view(-1), reduction="sum") / B
    loss.backward()
    assert torch.allclose(ours[(1, "wmat")], slope.grad, rtol=1e-3, atol=1e-5)
    assert torch.allclose(ours[(1, "bias")], bias.grad, rtol=1e-3, atol=1e-5)
    assert torch.allclose(ours[(2, "bias")], pr.grad, rtol=1e-3, atol=1e-5)
    assert torch.allclose(ours[(0, "wmat")].reshape(-1).abs().sum(),
                          layer0.from_logical(w.grad.reshape(1, 4, -1)).abs().sum(), rtol=1e-3)


def test_concat_split_bias_graph():
    conf = """
netconfig=start
layer[0->1,2] = split
layer[1->3] = fullc:a
  nhidden = 3
layer[2->4] = fullc:b
  nhidden = 5
layer[3,4->5] = concat
layer[5->5] = bias:bb
layer[5->6] = fullc:c
  nhidden = 2
layer[6->6] = softmax
netconfig=end
input_shape = 1,1,6
"""
    B = 3
    tr = make(conf, B)
    x = torch.randn(B, 1, 1, 6)
    y = torch.tensor([[0.0], [1.0], [1.0]])
    ours = grads_of(tr, x.clone(), y)
    wa, ba = weights(tr, 1, "wmat").requires_grad_(True), weights(tr, 1, "bias").requires_grad_(True)
    wb, bb = weights(tr, 2, "wmat").requires_grad_(True), weights(tr, 2, "bias").requires_grad_(True)
    bias = weights(tr, 4, "bias").requires_grad_(True)
    wc, bc = weights(tr, 5, "wmat").requires_grad_(True), weights(tr, 5, "bias").requires_grad_(True)
    xi = x.view(B, 6)
    h = torch.cat([xi @ wa.t() + ba, xi @ wb.t() + bb], 1) + bias
    logits = h @ wc.t() + bc
    loss = F.cross_entropy(logits, y.long().view(-1), reduction="sum") / B
    loss.backward()
    for key, ref in [((1, "wmat"), wa.grad), ((2, "wmat"), wb.grad), ((4, "bias"), bias.grad),
                     ((5, "wmat"), wc.grad)]:
        assert torch.allclose(ours[key], ref, rtol=1e-4, atol=1e-6), key


def test_multi_step_sgd_matches_autograd_sgd():
    """5 full training steps (SGD momentum, tag-scoped lr/wd) against torch autograd +
    a hand-written reference update (src/updater/sgd_updater-inl.hpp:73-84)."""
    conf = CONV_NET + """
momentum = 0.9
wmat:lr = 0.05
wmat:wd = 0.001
bias:lr = 0.1
bias:wd = 0.0
"""
    B = 4
    tr = make(conf, B)
    g = torch.Generator().manual_seed(3)
    x = torch.randn(B, 4, 15, 15, generator=g)
    y = torch.randint(0, 5, (B, 1), generator=g).float()

    l0, l4 = tr.net.connections[0].layer, tr.net.connections[4].layer
    params = {
        "w1": l0.to_logical(weights(tr, 0, "wmat")).reshape(8, 4, 3, 3),
        "b1": weights(tr, 0, "bias"),
        "w2": l4.to_logical(weights(tr, 4, "wmat")).reshape(6, 4, 3, 3),
        "b2": weights(tr, 4, "bias"),
        "wf1": weights(tr, 8, "wmat"), "bf1": weights(tr, 8, "bias"),
        "wf2": weights(tr, 10, "wmat"), "bf2": weights(tr, 10, "bias"),
    }
    mom = {k: torch.zeros_like(v) for k, v in params.items()}

    def loss_fn(p):
        h = F.relu(F.conv2d(x, p["w1"], p["b1"], stride=2, padding=1))
        h = F.max_pool2d(h, 3, 2, ceil_mode=True)
        h = lrn_ref(h, 5, 0.01, 0.75, 2.0)
        h = torch.tanh(F.conv2d(h, p["w2"], p["b2"], padding=1, groups=2))
        h = F.avg_pool2d(h, 2, 2, ceil_mode=True).reshape(B, -1)
        h = torch.sigmoid(h @ p["wf1"].t() + p["bf1"])
        logits = h @ p["wf2"].t() + p["bf2"]
        return F.cross_entropy(logits, y.long().view(-1), reduction="sum") / B

    for step in range(5):
        tr.update(DataBatch(x, y))
        ps = {k: v.clone().requires_grad_(True) for k, v in params.items()}
        loss_fn(ps).backward()
        for k in params:
            lr, wd = (0.05, 0.001) if k.startswith("w") else (0.1, 0.0)
            mom[k] = 0.9 * mom[k] - lr * (ps[k].grad + wd * params[k])
            params[k] = params[k] + mom[k]
    got = l0.to_logical(weights(tr, 0, "wmat")).reshape(8, 4, 3, 3)
    assert torch.allclose(got, params["w1"], rtol=1e-3, atol=1e-5)
    assert torch.allclose(weights(tr, 10, "wmat"), params["wf2"], rtol=1e-3, atol=1e-5)
    assert torch.allclose(weights(tr, 8, "bias"), params["bf1"], rtol=1e-3, atol=1e-5)


def test_exotic_layers_train_cpu():
    """batch_norm / prelu (noisy) / split / ch_concat / bias / insanity in one net: two CPU
    training steps stay finite and move every parameter."""
    import torch
    from cxxnet_amd import native
    from cxxnet_amd.io.data import DataBatch
    from cxxnet_amd.nnet import NetTrainer
    from test_layer_kernels_gpu import EXOTIC
    tr = NetTrainer()
    for k, v in list(native.rt().parse_config(EXOTIC)) + [("batch_size", "4"), ("dev", "cpu"), ("seed", "2"),
                                                          ("silent", "1"), ("eval_train", "0")]:
        tr.set_param(k, v)
    tr.init_model()
    before = tr.net.arena.w.clone()
    g = torch.Generator().manual_seed(0)
    x, y = torch.randn(4, 8, 8, 8, generator=g), torch.randint(0, 10, (4, 1), generator=g).float()
    for _ in range(2):
        tr.update(DataBatch(x, y))
    assert torch.isfinite(tr.net.nodes[-1].fp32_view).all()
    for _, s in tr.net.arena.specs:
        assert not torch.equal(before[s.offset:s.offset + s.numel], tr.net.arena.w[s.offset:s.offset + s.numel]), s.tag


def test_pool_tie_all_matches_reference_unpool():
    """pool_tie = all: the reference's value-compare unpool (pooling_layer-inl.hpp:55-86):
    every input equal to its window's max receives that window's gradient."""
    import torch
    from cxxnet_amd import ops
    N, H, W, C, K, S = 1, 5, 5, 2, 3, 2
    x = torch.zeros(N, H, W, C)
    x[0, 0, 0, 0] = 1.0
    x[0, 0, 2, 0] = 1.0          # tie with (0,0) inside window (0,0), and the max of window (0,1)
    Ho = ops.pool_out_size(H, K, S)
    y = torch.empty(N, Ho, Ho, C)
    ops.pool_forward(x, y, None, K, K, S, 0, "max")
    dy = torch.arange(1, N * Ho * Ho * C + 1, dtype=torch.float32).view(N, Ho, Ho, C)
    dx = torch.empty_like(x)
    ops.pool_backward_tie_all(x, y, dy, dx, K, K, S, 0)
    # brute force
    ref = torch.zeros_like(x)
    for ho in range(Ho):
        for wo in range(Ho):
            for c in range(C):
                win = x[0, ho * S:ho * S + K, wo * S:wo * S + K, c]
                m = win.max()
                for kh in range(win.shape[0]):
                    for kw in range(win.shape[1]):
                        if win[kh, kw] == m:
                            ref[0, ho * S + kh, wo * S + kw, c] += dy[0, ho, wo, c]
    assert torch.equal(dx, ref)
    assert dx[0, 0, 0, 0] == dy[0, 0, 0, 0] and dx[0, 0, 2, 0] == dy[0, 0, 0, 0] + dy[0, 0, 1, 0]


@pytest.mark.parametrize("algo", ["sgd", "nag", "adam"])
def test_clip_gradient_is_sgd_only(algo):
    """Only the reference SGD updater clips (sgd_updater-inl.hpp:77-81); NAG and Adam ignore
    clip_gradient (nag_updater-inl.hpp:66-72, adam_updater-inl.hpp:74-82)."""
    from cxxnet_amd import ops
    n = 64
    g0 = torch.linspace(-3, 3, n)
    runs = []
    for clip in (0.0, 0.5):
        w, g, m, m2 = torch.ones(n), g0.clone(), torch.zeros(n), torch.zeros(n)
        ops.fused_update(algo, w, g, m, m2, None, [(0, n, 0.1, 0.0, 0.9, clip)])
        runs.append(w)
    if algo == "sgd":
        assert not torch.equal(runs[0], runs[1])
        assert torch.allclose(runs[1], 1 - 0.1 * g0.clamp(-0.5, 0.5))
    else:
        assert torch.equal(runs[0], runs[1])


def test_rand_fill_host_statistics_and_determinism():
    from cxxnet_amd.ops.layer_ops import rand_fill
    a = rand_fill(torch.empty(200003), 7, "normal", 0.0, 0.02)
    b = rand_fill(torch.empty(200003), 7, "normal", 0.0, 0.02)
    c = rand_fill(torch.empty(200003), 8, "normal", 0.0, 0.02)
    assert torch.equal(a, b) and not torch.equal(a, c)
    assert abs(a.mean().item()) < 3e-4 and abs(a.std().item() / 0.02 - 1) < 1e-2
    u = rand_fill(torch.empty(100000), 7, "uniform", -1.0, 1.0)
    assert u.min().item() >= -1.0 and u.max().item() < 1.0 and abs(u.mean().item()) < 1e-2


DROP_NET = """
netconfig=start
layer[0->1] = flatten
layer[1->2] = fullc:f1
  nhidden = 24
layer[2->3] = relu
layer[3->3] = dropout
  threshold = 0.5
layer[3->4] = fullc:f2
  nhidden = 16
layer[4->5] = relu
layer[5->5] = dropout
  threshold = 0.25
layer[5->6] = fullc:f3
  nhidden = 5
layer[6->6] = softmax
netconfig=end
input_shape = 2,3,4
"""


def test_fused_fc_relu_dropout_matches_unfused(monkeypatch):
    """NeuralNet._fuse_dropout: the fc forward applies the dropout mask and the next fc's
    data-gradient scales by 1 / pkeep under the relu'-mask -- the same gradients as the
    separate relu and dropout layers (CPU executor with fusion forced on, CXXNET_FUSE=2)."""
    B = 6
    x = torch.randn(B, 2, 3, 4)
    y = torch.randint(0, 5, (B, 1)).float()
    out = {}
    for mode in ("0", "2"):
        monkeypatch.setenv("CXXNET_FUSE", mode)
        torch.manual_seed(0)
        tr = make(DROP_NET, B, [("seed", "7")])
        if mode == "2":
            fused = [c.layer for c in tr.net.connections if type(c.layer).__name__ == "DropoutLayer"]
            assert all(d.fused_into_producer for d in fused)
        out[mode] = grads_of(tr, x, y)
        out[mode + "p"] = tr.net.nodes[-1].data.clone()
    for k in out["0"]:
        assert torch.allclose(out["0"][k], out["2"][k], rtol=1e-5, atol=1e-6), k
    assert torch.allclose(out["0p"], out["2p"], rtol=1e-5, atol=1e-6)
