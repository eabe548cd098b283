"""Layer registry: reference type id (src/layer/layer.h:284-315) -> implementation."""
from __future__ import annotations

from .base import BinReader, BinWriter, Layer, LayerContext, Node, ParamSpec  # noqa: F401
from .std import (ActivationLayer, ConvolutionLayer, DropoutLayer, FlattenLayer, FullConnectLayer, L2LossLayer,
                  LRNLayer, MultiLogisticLayer, PoolingLayer, SoftmaxLayer)

K_SHARED = 0
K_PAIRTEST_GAP = 1024

_FACTORY = {
    1: FullConnectLayer,
    2: SoftmaxLayer,
    3: lambda ctx: ActivationLayer(ctx, "relu"),
    4: lambda ctx: ActivationLayer(ctx, "sigmoid"),
    5: lambda ctx: ActivationLayer(ctx, "tanh"),
    7: FlattenLayer,
    8: DropoutLayer,
    10: ConvolutionLayer,
    11: lambda ctx: PoolingLayer(ctx, "max"),
    12: lambda ctx: PoolingLayer(ctx, "sum"),
    13: lambda ctx: PoolingLayer(ctx, "avg"),
    15: LRNLayer,
    19: lambda ctx: ActivationLayer(ctx, "xelu"),
    21: lambda ctx: PoolingLayer(ctx, "max", relu=True),
    26: L2LossLayer,
    27: MultiLogisticLayer,
}


def register(type_id: int, ctor):
    _FACTORY[type_id] = ctor


def create_layer(type_id: int, ctx: LayerContext) -> Layer:
    if type_id >= K_PAIRTEST_GAP:
        from .extra import PairTestLayer
        return PairTestLayer(ctx, create_layer(type_id // K_PAIRTEST_GAP, ctx),
                             create_layer(type_id % K_PAIRTEST_GAP, ctx))
    ctor = _FACTORY.get(type_id)
    if ctor is None:
        raise ValueError(f"unknown layer type id {type_id}")
    layer = ctor(ctx)
    layer.type_id = type_id
    return layer


# extra layers register themselves
from . import extra  # noqa: E402,F401
