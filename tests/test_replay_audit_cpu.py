"""Launch-list replay safety is opt-in (Layer.replay_audited): every registered layer type is
either audited -- and then covered by tests/test_launch_hygiene_gpu.py's all-layer net, which
fails on any torch kernel in its forward / backward -- or replays never take a step it is in."""
from cxxnet_amd.layers import _FACTORY, LayerContext, create_layer
from cxxnet_amd.layers.base import Layer

# the layer classes test_every_audited_layer_launches_only_library_kernels builds
AUDITED = {"FullConnectLayer", "ConvolutionLayer", "ActivationLayer", "PoolingLayer", "LRNLayer", "DropoutLayer",
           "FlattenLayer", "SoftmaxLayer", "BiasLayer", "SplitLayer", "ConcatLayer", "BatchNormLayer"}


def test_base_layer_is_not_replay_safe():
    assert Layer.replay_audited is False


def test_every_registered_layer_is_audited_or_eager():
    import torch
    ctx = LayerContext(torch.device("cpu"))
    seen = set()
    for tid in sorted(_FACTORY):
        lay = create_layer(tid, ctx)
        name = type(lay).__name__
        if lay.replay_safe():
            assert name in AUDITED, f"layer type {tid} ({name}) replays without being in the audited GPU net"
            seen.add(name)
    assert seen == AUDITED
