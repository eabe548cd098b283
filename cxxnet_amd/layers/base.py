"""Core layer types: Node, ParamSpec, Layer base, and tensor (de)serialization.

Reference: src/layer/layer.h (Node 30-71, ILayer 161-279), src/layer/param.h.

Node storage is NHWC.  A node's logical shape is the reference's (batch, c, h, w);
its device buffer is ``data[batch][h][w][cp]`` with cp >= c physical channels
(only the network input may be padded, so the first conv can use 8-byte
vector gathers).  On the GPU activations are bf16, on the CPU fp32.
"""
from __future__ import annotations

import math
import struct
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from .. import native


class Node:
    def __init__(self, name: str):
        self.name = name
        self.shape: Tuple[int, int, int, int] = (0, 0, 0, 0)  # (b, c, h, w)
        self.cp = 0
        self.wp = 0  # physical row width when > w (row-padded first-conv input, NeuralNet._pad_input_channels)
        self.data: Optional[torch.Tensor] = None
        self.fp32_view: Optional[torch.Tensor] = None  # loss layers expose fp32 predictions here
        # zero-copy split outputs: `data` aliases the split input (read-only in forward) and the
        # consumer writes its input gradient into this private buffer instead
        self.grad_buf: Optional[torch.Tensor] = None

    @property
    def gdst(self) -> torch.Tensor:
        """Where a layer writes the gradient w.r.t. this node (normally the node itself)."""
        return self.grad_buf if self.grad_buf is not None else self.data

    def gmat(self) -> torch.Tensor:
        g = self.gdst
        return g.view(g.shape[0], -1)

    def set_shape(self, b, c, h, w, cp=None):
        self.shape = (int(b), int(c), int(h), int(w))
        self.cp = int(cp if cp is not None else c)
        self.wp = int(w)

    @property
    def batch(self):
        return self.shape[0]

    def is_mat(self) -> bool:
        """Reference convention: a matrix node is (batch, 1, 1, n)."""
        return self.shape[1] == 1 and self.shape[2] == 1

    def alloc(self, device, dtype):
        b, c, h, w = self.shape
        self.data = torch.zeros((b, h, max(w, self.wp), self.cp), device=device, dtype=dtype)

    def mat(self) -> torch.Tensor:
        """(batch, c*h*w) view (reference Node::mat); physical order is NHWC."""
        return self.data.view(self.data.shape[0], -1)

    def to_nchw(self) -> torch.Tensor:
        from ..ops import nhwc_to_nchw
        return nhwc_to_nchw(self.data, self.shape[1], self.shape[3])


@dataclass
class ParamSpec:
    """A trainable tensor of a layer: lives in the flat fp32 arena."""
    tag: str                       # "wmat" or "bias" (updater tag scoping)
    shape: Tuple[int, ...]         # internal (device) layout
    init: Callable[[torch.Tensor], None]
    # views into the arena, set by ParamArena.bind
    w: Optional[torch.Tensor] = None   # fp32 master
    g: Optional[torch.Tensor] = None   # fp32 gradient (accumulated, zeroed by the updater)
    wb: Optional[torch.Tensor] = None  # compute copy (bf16 on GPU, == w on CPU)
    offset: int = 0
    # True when the layer can WRITE (not accumulate) this gradient on the first
    # micro-batch of an update cycle, so the arena need not zero it beforehand
    overwrite: bool = False

    @property
    def numel(self):
        n = 1
        for s in self.shape:
            n *= s
        return n


class LayerContext:
    """Per-net state shared by layers (reference LabelInfo + RNG + device)."""

    def __init__(self, device: torch.device, seed: int = 0):
        self.device = torch.device(device)
        # is_gpu: the HIP-kernel (bf16) path; a GPU context in reference precision (fp32) runs the
        # CPU path's torch formulas on device tensors (ops.mode)
        from ..ops.mode import reference_precision
        self.on_device = self.device.type == "cuda"
        self.is_gpu = self.on_device and not reference_precision()
        self.act_dtype = torch.bfloat16 if self.is_gpu else torch.float32
        self.seed = seed
        # set by the trainer around an update step's backprop: the arena updater when the fc
        # weight steps are fused into their weight-gradient GEMMs, and the step's epoch
        self.sgd_fuse = None
        self.epoch = 0
        # bias gradients queued during a backward pass (NeuralNet.backprop flushes them in one
        # launch); None = compute each one immediately
        self.deferred_bias = None
        # conv layers whose flipped data-gradient weights were prepared for this backward pass
        # (one multi-tensor launch in NeuralNet.backprop); None = each layer flips its own
        self.flipped = None
        self.gen = torch.Generator(device="cpu")
        self.gen.manual_seed(seed)
        self.label_fields: Dict[str, torch.Tensor] = {}
        self.label_name_map: Dict[str, int] = {"label": 0}
        self.step = 0  # forward counter, feeds counter-based RNG (dropout)

    def bias_grad(self, dy2d, db, mask=None):
        """db += column sums of dy2d (mask: see ops.bias_grad), now or (deferred) at the end
        of the backward pass."""
        if self.deferred_bias is not None and self.is_gpu:
            self.deferred_bias.append((dy2d, db, mask))
            return
        from .. import ops
        ops.bias_grad(dy2d, db, mask)


class Layer:
    """Base layer.  Subclasses implement init_connection/forward/backprop."""
    type_name = "layer"
    allow_sharing = True


    # Opt-in: a layer class sets replay_audited = True once its GPU forward / backward has been
    # checked to launch only library kernels with step-invariant arguments.  Anything else (a
    # new layer, a torch op in forward / backward) keeps the eager executor, where every op
    # runs every step; a replayed plan would silently skip torch ops.
    replay_audited = False

    def replay_safe(self) -> bool:
        """Whether this layer's GPU forward / backward launch only library kernels whose
        arguments are step-invariant (per-step values read from device memory), so that the
        C++ launch-list executor can record the step once and replay it (NetTrainer._list_step).
        False unless the class is audited (replay_audited); audited classes with
        configuration-dependent torch ops override this."""
        return bool(type(self).replay_audited)

    def __init__(self, ctx: LayerContext):
        self.ctx = ctx
        self.lp = native.rt().LayerParam()
        self.params: List[ParamSpec] = []
        self.layer_index = -1
        # set by the executor's relu fusion: the input node holds relu(z) of a fused
        # producer, so the gradient this layer writes into it must be masked by relu'(z)
        self.grad_mask_relu = False

    # ---- configuration
    def set_param(self, name: str, val: str):
        self.lp.set_param(name, val)

    def init_connection(self, nodes_in: Sequence[Node], nodes_out: Sequence[Node]):
        raise NotImplementedError

    def declare_params(self) -> List[ParamSpec]:
        """Called after init_connection; returns the trainable tensors."""
        return self.params

    def on_batch_size_changed(self, nodes_in, nodes_out):
        pass

    # ---- compute
    def forward(self, is_train: bool, nodes_in: Sequence[Node], nodes_out: Sequence[Node]):
        raise NotImplementedError

    def backprop(self, prop_grad: bool, nodes_in: Sequence[Node], nodes_out: Sequence[Node]):
        raise NotImplementedError

    # ---- model io (reference SaveModel/LoadModel byte layout)
    def save_model(self, fo: "BinWriter"):
        pass

    def load_model(self, fi: "BinReader"):
        pass

    # ---- helpers
    def _init_weight(self, t: torch.Tensor, in_num: int, out_num: int):
        """LayerParam::RandInitWeight (reference src/layer/param.h:114-138), on a logical-layout tensor."""
        lp = self.lp
        # one seed per tensor from the context generator; the draws themselves run where t
        # lives (ops.rand_fill: a HIP kernel on the GPU, the same hash on the host)
        from ..ops.layer_ops import rand_fill
        seed = int(torch.randint(0, 2**31 - 1, (1,), generator=self.ctx.gen).item())
        if lp.random_type == 0:
            rand_fill(t, seed, "normal", 0.0, lp.init_sigma)
        elif lp.random_type == 1:
            a = math.sqrt(3.0 / (in_num + out_num))
            if lp.init_uniform > 0:
                a = lp.init_uniform
            rand_fill(t, seed, "uniform", -a, a)
        elif lp.random_type == 2:
            if lp.num_hidden > 0:
                sigma = math.sqrt(2.0 / lp.num_hidden)
            else:
                sigma = math.sqrt(2.0 / (lp.num_channel * lp.kernel_width * lp.kernel_height))
            rand_fill(t, seed, "normal", 0.0, sigma)


# ----------------------------------------------------------------------------- binary io
class BinWriter:
    def __init__(self):
        self.parts: List[bytes] = []

    def write(self, b: bytes):
        self.parts.append(bytes(b))

    def write_tensor(self, t: torch.Tensor):
        """mshadow SaveBinary: uint32 shape[dim] + contiguous fp32 rows."""
        t = t.detach().to("cpu", torch.float32).contiguous()
        self.write(struct.pack("<%dI" % t.dim(), *t.shape))
        self.write(t.numpy().tobytes())

    def getvalue(self) -> bytes:
        return b"".join(self.parts)


class BinReader:
    def __init__(self, data: bytes, pos: int = 0):
        self.data = data
        self.pos = pos

    def read(self, n: int) -> bytes:
        if self.pos + n > len(self.data):
            raise ValueError("invalid model file: unexpected end of stream")
        b = self.data[self.pos:self.pos + n]
        self.pos += n
        return b

    def read_tensor(self, dim: int) -> torch.Tensor:
        shape = struct.unpack("<%dI" % dim, self.read(4 * dim))
        n = 1
        for s in shape:
            n *= s
        arr = np.frombuffer(self.read(4 * n), dtype="<f4").copy()
        return torch.from_numpy(arr).view(*shape)

    def read_layer_param(self):
        return native.rt().LayerParam.from_bytes(self.read(328))
