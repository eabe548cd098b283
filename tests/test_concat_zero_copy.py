"""Zero-copy ch_concat (NeuralNet._fuse_concat): the branch convs write relu(z) into channel
slices of the concat output and read their output gradient from those slices; relu' is applied
by the concat output's consumer (split sum / pooling backward).  On the CPU executor with
fusion forced (CXXNET_FUSE=2) the fused graph must train exactly what the unfused graph trains
(reference semantics: src/layer/concat_layer-inl.hpp:38-76, split_layer-inl.hpp:24-40)."""
import os

import pytest
import torch

from cxxnet_amd.io.data import DataBatch
from cxxnet_amd.nnet import NetTrainer

CONF = """
netconfig=start
layer[0->c0] = conv:c0
  kernel_size = 3
  nchannel = 16
  pad = 1
layer[c0->c0r] = relu
layer[c0r->s1,s2,s3] = split
layer[s1->a] = conv:a
  kernel_size = 1
  nchannel = 8
layer[a->ar] = relu
layer[s2->b0] = conv:b0
  kernel_size = 1
  nchannel = 8
layer[b0->b0r] = relu
layer[b0r->b] = conv:b
  kernel_size = 3
  nchannel = 16
  pad = 1
layer[b->br] = relu
layer[s3->pp] = max_pooling
  kernel_size = 3
  stride = 1
  pad = 1
layer[pp->c] = conv:c
  kernel_size = 1
  nchannel = 8
layer[c->cr] = relu
layer[ar,br,cr->cat] = ch_concat
layer[cat->t1,t2] = split
layer[t1->d] = conv:d
  kernel_size = 1
  nchannel = 8
layer[d->dr] = relu
layer[t2->e] = conv:e
  kernel_size = 3
  nchannel = 16
  pad = 1
layer[e->er] = relu
layer[dr,er->cat2] = ch_concat
layer[cat2->p] = {pool}
  kernel_size = 3
  stride = 2
layer[p->fl] = flatten
layer[fl->fc] = fullc:fc
  nhidden = 10
layer[fc->fc] = softmax
netconfig=end
input_shape = 8,9,9
batch_size = 4
eta = 0.05
momentum = 0.9
wd = 0.0001
seed = 3
silent = 1
"""


def _trainer(pool, fuse, monkeypatch):
    from cxxnet_amd import native
    monkeypatch.setenv("CXXNET_FUSE", fuse)
    tr = NetTrainer()
    path = os.path.join(os.environ.get("TMPDIR", "/tmp"), f"zc_{os.getpid()}.conf")
    with open(path, "w") as f:
        f.write(CONF.replace("{pool}", pool))
    for k, v in native.rt().parse_config_file(path):
        tr.set_param(k, v)
    tr.set_param("dev", "cpu")
    tr.init_model()
    return tr


@pytest.mark.parametrize("pool", ["max_pooling", "avg_pooling"])
def test_zero_copy_concat_matches_unfused_cpu(pool, monkeypatch):
    fused = _trainer(pool, "2", monkeypatch)
    plain = _trainer(pool, "0", monkeypatch)
    net = fused.net
    zc = [c for c in net.connections if getattr(c.layer, "zero_copy", False)]
    assert len(zc) == 2, "both concats should be zero-copy"
    # the branch conv outputs are channel slices of the concat buffers
    cat = net.nodes[net.cfg.node_names.index("cat")]
    for name, off in (("a", 0), ("b", 8), ("c", 24)):
        n = net.nodes[net.cfg.node_names.index(name)]
        assert not n.data.is_contiguous()
        assert n.data.data_ptr() == cat.data.data_ptr() + off * cat.data.element_size()
    plain.net.arena.w.copy_(fused.net.arena.w)
    plain.net.arena.sync_shadow()
    g = torch.Generator().manual_seed(0)
    for _ in range(3):
        x = torch.randn(4, 8, 9, 9, generator=g)
        y = torch.randint(0, 10, (4, 1), generator=g).float()
        fused.update(DataBatch(x, y))
        plain.update(DataBatch(x, y))
    assert torch.allclose(fused.net.arena.m1, plain.net.arena.m1, rtol=1e-4, atol=1e-6)
    assert torch.allclose(fused.net.arena.w, plain.net.arena.w, rtol=1e-5, atol=1e-7)


def test_zero_copy_concat_can_be_turned_off(monkeypatch):
    monkeypatch.setenv("CXXNET_CONCAT_ZC", "0")
    tr = _trainer("max_pooling", "2", monkeypatch)
    assert not any(getattr(c.layer, "zero_copy", False) for c in tr.net.connections)
