"""Remaining reference layers: bias, split, concat, ch_concat, batch_norm, prelu,
insanity, insanity_max_pooling, fixconn, pairtest.

On the GPU every one of them runs hand-written HIP kernels: batch_norm / prelu / insanity /
insanity_max_pooling in csrc/kernels/layer_kernels.hip (ops/layer_ops.py), concat / split /
bias on the channel-copy / add / column-sum kernels, fixconn on the MFMA GEMM.  The CPU
executor runs the same formulas in fp32 torch with the same counter-hash random draws.
"""
from __future__ import annotations

import torch

from .. import ops
from ..ops import layer_ops as L
from .base import BinReader, BinWriter, Layer, ParamSpec
from .std import PoolingLayer, _bias_init, _check


def _feat_axis(node):
    """Per-channel axis of an NHWC node buffer (reference: dim 1 for conv nodes,
    dim 3 for matrix nodes).  Physical layout is [b][h][w][c]."""
    return 3 if node.shape[1] != 1 else 2


def _num_feat(node):
    return node.shape[1] if node.shape[1] != 1 else node.shape[3]


class BiasLayer(Layer):
    """`bias` -- reference src/layer/bias_layer-inl.hpp:14-83 (self-loop on a matrix node)."""
    replay_audited = True  # library kernels only (tests/test_launch_hygiene_gpu.py)
    type_name = "bias"

    def init_connection(self, nodes_in, nodes_out):
        _check(len(nodes_in) == 1 and len(nodes_out) == 1, "BiasLayer: only support 1-1 connection")
        _check(nodes_in[0] is nodes_out[0], "BiasLayer is a self-loop Layer")
        _check(nodes_in[0].is_mat(), "BiasLayer: input need to be a matrix")
        n = nodes_in[0].shape[3]
        self.params = [ParamSpec("bias", (n,), _bias_init(self.lp.init_bias))]

    def forward(self, is_train, nodes_in, nodes_out):
        m = nodes_in[0].mat()
        if self.ctx.is_gpu:  # y = 1*x + b on the BN affine kernel: mean 0, inv 1, slope 1
            st = self._affine(m.shape[1], m.device)
            L.affine_forward(m, m, st.mean, st.inv, self._ones, self.params[0].w)
        else:
            m.copy_((m.float() + self.params[0].w).to(m.dtype))

    def _affine(self, C, device):
        if getattr(self, "_st", None) is None:
            self._st = L.BNState(C, device)
            self._st.inv.fill_(1.0)
            self._ones = torch.ones(C, dtype=torch.float32, device=device)
        return self._st

    def backprop(self, prop_grad, nodes_in, nodes_out):
        ops.bias_grad(nodes_in[0].mat(), self.params[0].g)

    def save_model(self, fo: BinWriter):
        fo.write(self.lp.to_bytes())
        fo.write_tensor(self.params[0].w)

    def load_model(self, fi: BinReader):
        self.lp = fi.read_layer_param()
        self.loaded = [fi.read_tensor(1)]

    def loaded_values(self):
        return self.loaded


class SplitLayer(Layer):
    """`split` -- reference src/layer/split_layer-inl.hpp:12-45: 1 -> n copies, grads summed.

    Zero-copy on the GPU (the executor sets `alias` when every consumer of every output only
    reads its input in forward: conv / fullc / pooling / lrn): the outputs ARE the input buffer,
    each consumer writes its data-gradient into its output node's private grad buffer, and
    backward sums those into the input node -- no forward copies."""
    replay_audited = True  # library kernels only (tests/test_launch_hygiene_gpu.py)
    type_name = "split"
    alias = False
    skip_grads = frozenset()
    folded = False  # set per step by a sibling group's lead (ConvolutionLayer.backprop)

    def init_connection(self, nodes_in, nodes_out):
        _check(len(nodes_in) == 1 and len(nodes_out) >= 1, "SplitLayer: only support 1-n connection")
        for o in nodes_out:
            o.set_shape(*nodes_in[0].shape, cp=nodes_in[0].cp)

    def forward(self, is_train, nodes_in, nodes_out):
        if self.alias:
            return
        # one read of the input per 4 outputs (ops.fanout_copy), not one per output
        ops.fanout_copy(nodes_in[0].data, [o.data for o in nodes_out])

    def backprop(self, prop_grad, nodes_in, nodes_out):
        if not prop_grad:
            return
        # the output gradients summed in one pass (fp32 accumulation, one rounding); masked by
        # relu' when the input is a zero-copy concat of relu outputs (NeuralNet._fuse_concat).
        # skip_grads: outputs whose consumer's data-gradient a fused sibling wrote into another
        # output's slot (NeuralNet._fuse_siblings)
        if self.folded:  # the group's data-gradient GEMM summed and masked already
            return
        skip = self.skip_grads
        ops.sum_into(nodes_in[0].gdst, [o.gdst for o in nodes_out if id(o) not in skip], mask_relu=self.grad_mask_relu)


class ConcatLayer(Layer):
    """`concat` (dim 3) / `ch_concat` (dim 1) -- reference src/layer/concat_layer-inl.hpp:11-79,
    2-4 inputs.  On NHWC buffers ch_concat is a strided channel copy per input."""
    replay_audited = True  # library kernels only (tests/test_launch_hygiene_gpu.py)

    def __init__(self, ctx, dim):
        super().__init__(ctx)
        self.dim = dim
        self.type_name = "ch_concat" if dim == 1 else "concat"
        # inputs that hold relu(z) of a fused conv/fullc -> relu producer: the gradient slice
        # copied back into them is masked by relu'(z) (the activation they still hold)
        self.grad_mask_inputs = set()
        # the inputs are channel slices of the output buffer (NeuralNet._fuse_concat): no copies
        self.zero_copy = False
        # zero-copy inputs that moved into a sibling group's buffer H (NeuralNet._fuse_siblings):
        # (group, H channel offset, output channel offset, channels); h_copies: with H bound
        self.copy_from_h = []
        self.h_copies = []

    def init_connection(self, nodes_in, nodes_out):
        _check(len(nodes_in) > 1 and len(nodes_out) == 1, "Concat layer only support n-1 connection")
        _check(len(nodes_in) <= 4, "More than 4 input node is unspported")
        s0 = list(nodes_in[0].shape)
        tot = 0
        for n in nodes_in:
            _check(n.cp == n.shape[1], "Concat: padded-channel inputs are not supported")
            tot += n.shape[self.dim]
            for j in range(4):
                if j != self.dim:
                    _check(n.shape[j] == s0[j], "Concat shape doesn't match")
        s0[self.dim] = tot
        nodes_out[0].set_shape(*s0)

    def _pieces(self, nodes_in, nodes_out):
        out = nodes_out[0]
        if self.dim == 1:
            off = 0
            for n in nodes_in:
                yield n.data, out.data, off, n.shape[1]
                off += n.shape[1]
        else:
            # width concat: in NHWC this is concat along axis 2 (w); matrix nodes are the common case
            off = 0
            for n in nodes_in:
                yield n, out, off, n.shape[3]
                off += n.shape[3]

    def forward(self, is_train, nodes_in, nodes_out):
        if self.zero_copy:
            out = nodes_out[0].data
            for H, hoff, coff, c in self.h_copies:  # sibling outputs computed into H
                ops.channel_copy(H[: out.shape[0]], hoff, out, coff, c)
            return
        if self.dim == 1:
            if ops.concat_channels([n.data for n in nodes_in], nodes_out[0].data):
                return
            for src, dst, off, c in self._pieces(nodes_in, nodes_out):
                ops.channel_copy(src, 0, dst, off, c)
        else:
            # width concat: rows of [B*H][W_i*C] into [B*H][W*C] at a column offset
            out = nodes_out[0].data
            B, H, W, C = out.shape
            off = 0
            for n in nodes_in:
                wi = n.data.shape[2]
                ops.channel_copy(n.data.reshape(B * H, wi * C), 0, out.view(B * H, W * C), off * C, wi * C)
                off += wi

    def backprop(self, prop_grad, nodes_in, nodes_out):
        if not prop_grad:
            return
        if self.zero_copy:
            out = nodes_out[0].data
            for H, hoff, coff, c in self.h_copies:  # the slice's gradient back into H, times relu'
                ops.channel_copy(out, coff, H[: out.shape[0]], hoff, c, mask_relu=True)
            return
        if self.dim == 1:
            if ops.concat_channels([n.gdst for n in nodes_in], nodes_out[0].data, backward=True,
                                   mask=self.grad_mask_inputs):
                return
            for k, (src, dst, off, c) in enumerate(self._pieces(nodes_in, nodes_out)):
                ops.channel_copy(dst, off, nodes_in[k].gdst, 0, c, mask_relu=k in self.grad_mask_inputs)
        else:
            out = nodes_out[0].data
            B, H, W, C = out.shape
            off = 0
            for k, n in enumerate(nodes_in):
                wi = n.data.shape[2]
                ops.channel_copy(out.view(B * H, W * C), off * C, n.gdst.view(B * H, wi * C), 0, wi * C,
                                 mask_relu=k in self.grad_mask_inputs)
                off += wi


class BatchNormLayer(Layer):
    """`batch_norm` -- reference src/layer/batch_norm_layer-inl.hpp:14-197.  Batch
    statistics in both train and test (no running mean), eps default 1e-10; slope is
    visited as "wmat", bias as "bias"; the checkpoint holds slope + bias only."""
    replay_audited = True  # library kernels only (tests/test_launch_hygiene_gpu.py)
    type_name = "batch_norm"

    def __init__(self, ctx):
        super().__init__(ctx)
        self.init_slope = 1.0
        self.init_bias = 0.0
        self.eps = 1e-10

    def set_param(self, name, val):
        super().set_param(name, val)
        if name == "init_slope":
            self.init_slope = float(val)
        elif name == "init_bias":
            self.init_bias = float(val)
        elif name == "eps":
            self.eps = float(val)

    def init_connection(self, nodes_in, nodes_out):
        _check(len(nodes_in) == 1 and len(nodes_out) == 1, "BNLayer: only support 1-1 connection")
        nodes_out[0].set_shape(*nodes_in[0].shape, cp=nodes_in[0].cp)
        self.channel = _num_feat(nodes_in[0])
        self.params = [ParamSpec("wmat", (self.channel,), _bias_init(self.init_slope)),
                       ParamSpec("bias", (self.channel,), _bias_init(self.init_bias))]

    def _view(self, node):
        # -> [rows][channels] view of the NHWC / matrix buffer
        return node.data.view(-1, self.channel)

    def _state(self, device):
        if getattr(self, "_st", None) is None:
            self._st = L.BNState(self.channel, device)
        return self._st

    def forward(self, is_train, nodes_in, nodes_out):
        x = self._view(nodes_in[0])
        L.bn_forward(x, self._view(nodes_out[0]), self.params[0].w, self.params[1].w, self.eps,
                     self._state(x.device), is_train)

    def backprop(self, prop_grad, nodes_in, nodes_out):
        g = self._view(nodes_out[0])
        L.bn_backward(g, self._view(nodes_in[0]), self.params[0].w, self.params[0].g, self.params[1].g,
                      self._state(g.device), prop_grad)

    def save_model(self, fo: BinWriter):
        fo.write_tensor(self.params[0].w)
        fo.write_tensor(self.params[1].w)

    def load_model(self, fi: BinReader):
        self.loaded = [fi.read_tensor(1), fi.read_tensor(1)]

    def loaded_values(self):
        return self.loaded


class PReluLayer(Layer):
    """`prelu` -- reference src/layer/prelu_layer-inl.hpp:48-173 (per-channel slope
    clamped to [0,1], optional multiplicative train-time noise `random`; the slope is
    visited with tag "bias")."""
    type_name = "prelu"


    def replay_safe(self) -> bool:
        return False  # host-side per-step values / torch ops: the eager executor runs it

    def __init__(self, ctx):
        super().__init__(ctx)
        self.init_slope = 0.25
        self.init_random = 0
        self.random = 0.0
        self.seed = int(torch.randint(0, 2**31 - 1, (1,), generator=ctx.gen).item())

    def set_param(self, name, val):
        super().set_param(name, val)
        if name == "init_slope":
            self.init_slope = float(val)
        elif name == "random_slope":
            self.init_random = int(val)
        elif name == "random":
            self.random = float(val)

    def init_connection(self, nodes_in, nodes_out):
        _check(len(nodes_in) == 1 and len(nodes_out) == 1, "PReluLayer: only support 1-1 connection")
        nodes_out[0].set_shape(*nodes_in[0].shape, cp=nodes_in[0].cp)
        self.channel = _num_feat(nodes_in[0])

        def init(t):
            if self.init_random == 0:
                t.fill_(self.init_slope)
            else:
                from ..ops.layer_ops import rand_fill
                rand_fill(t, int(torch.randint(0, 2**31 - 1, (1,), generator=self.ctx.gen).item()), "uniform",
                          0.0, self.init_slope)
        self.params = [ParamSpec("bias", (self.channel,), init)]

    def _noise(self, is_train):
        return self.random if is_train else 0.0

    def forward(self, is_train, nodes_in, nodes_out):
        self._train = is_train
        L.prelu_forward(nodes_in[0].data.view(-1, self.channel), nodes_out[0].data.view(-1, self.channel),
                        self.params[0].w, self.seed, self.ctx.step_counter, self._noise(is_train))

    def backprop(self, prop_grad, nodes_in, nodes_out):
        x = nodes_in[0].data.view(-1, self.channel)
        L.prelu_backward(x, nodes_out[0].data.view(-1, self.channel), x, self.params[0].w, self.params[0].g,
                         self.seed, self.ctx.step_counter, self._noise(getattr(self, "_train", True)), prop_grad)

    def save_model(self, fo: BinWriter):
        fo.write_tensor(self.params[0].w)

    def load_model(self, fi: BinReader):
        self.loaded = [fi.read_tensor(1)]

    def loaded_values(self):
        return self.loaded


class InsanityLayer(Layer):
    """`insanity` (randomized leaky relu) -- reference src/layer/insanity_layer-inl.hpp:14-102:
    x / U[lb,ub] for x<=0 in training, x / ((lb+ub)/2) at test; calm_start/calm_end anneal."""
    type_name = "insanity"


    def replay_safe(self) -> bool:
        return False  # host-side per-step values / torch ops: the eager executor runs it

    def __init__(self, ctx):
        super().__init__(ctx)
        self.lb, self.ub = 5.0, 10.0
        self.step = 0
        self.sat_start = self.sat_end = 0
        self.delta = 0.0
        self.inited = False
        self.seed = int(torch.randint(0, 2**31 - 1, (1,), generator=ctx.gen).item())

    def set_param(self, name, val):
        super().set_param(name, val)
        if name == "lb":
            self.lb = float(val)
        elif name == "ub":
            self.ub = float(val)
        elif name == "calm_start":
            self.sat_start = int(val)
        elif name == "calm_end":
            self.sat_end = int(val)

    def init_connection(self, nodes_in, nodes_out):
        _check(len(nodes_in) == 1 and len(nodes_out) == 1, "InsanityLayer: only support 1-1 connection")
        nodes_out[0].set_shape(*nodes_in[0].shape, cp=nodes_in[0].cp)

    def forward(self, is_train, nodes_in, nodes_out):
        if not self.inited:
            self.inited = True
            d = (self.ub + self.lb) / 2.0
            span = (self.sat_end - self.sat_start)
            self.delta = (self.ub - d) / span if span != 0 else 0.0
        if self.sat_start < self.step < self.sat_end:
            self.ub -= self.delta * self.step
            self.lb += self.delta * self.step
            self.step += 1
        x = nodes_in[0].data
        self._train = is_train
        y2 = nodes_out[0].data if nodes_out[0] is not nodes_in[0] else None
        L.insanity_forward(x, x, y2, self.lb, self.ub, is_train, self.seed, self.ctx.step_counter)

    def backprop(self, prop_grad, nodes_in, nodes_out):
        if prop_grad:
            y = nodes_in[0].data
            L.insanity_backward(y, nodes_out[0].data, y, self.lb, self.ub, getattr(self, "_train", True), self.seed,
                                self.ctx.step_counter)


class InsanityPoolingLayer(PoolingLayer):
    """`insanity_max_pooling` -- reference src/layer/insanity_pooling_layer-inl.hpp:222-286:
    in training each source pixel is shifted by +-1 in y or x with probability (1-keep)/4."""


    def replay_safe(self) -> bool:
        return False  # host-side per-step values / torch ops: the eager executor runs it

    def __init__(self, ctx):
        super().__init__(ctx, "max")
        self.type_name = "insanity_max_pooling"
        self.keep = 1.0
        self.seed = int(torch.randint(0, 2**31 - 1, (1,), generator=ctx.gen).item())

    def set_param(self, name, val):
        super().set_param(name, val)
        if name == "keep":
            self.keep = float(val)

    def forward(self, is_train, nodes_in, nodes_out):
        self._shifted = is_train and self.keep < 1.0
        if not self._shifted:
            return super().forward(is_train, nodes_in, nodes_out)
        y = nodes_out[0].data
        if getattr(self, "ysave", None) is None or self.ysave.shape != y.shape:
            self.ysave = torch.empty_like(y)
        L.ins_pool_forward(nodes_in[0].data, y, self.ysave, self.lp.kernel_height, self.lp.stride, self.keep,
                           self.seed, self.ctx.step_counter)

    def backprop(self, prop_grad, nodes_in, nodes_out):
        if not prop_grad:
            return
        if not getattr(self, "_shifted", False):
            return super().backprop(prop_grad, nodes_in, nodes_out)
        x = nodes_in[0].data
        if getattr(self, "gscratch", None) is None or self.gscratch.shape != x.shape:
            self.gscratch = torch.empty_like(x)
        # gather-form unpool reads shifted neighbours of x: write to scratch, then copy back
        L.ins_pool_backward(x, self.ysave, nodes_out[0].data, self.gscratch, self.lp.kernel_height, self.lp.stride,
                            self.keep, self.seed, self.ctx.step_counter)
        ops.channel_copy(self.gscratch, 0, x, 0, x.shape[-1])


class FixConnectLayer(Layer):
    """`fixconn` -- reference src/layer/fixconn_layer-inl.hpp:14-92: fixed sparse weight
    from a text file (`nrow ncol nnz` then `row col value` triples); no weight gradient."""
    type_name = "fixconn"


    def replay_safe(self) -> bool:
        return False  # host-side per-step values / torch ops: the eager executor runs it

    def __init__(self, ctx):
        super().__init__(ctx)
        self.fname = "NULL"

    def set_param(self, name, val):
        super().set_param(name, val)
        if name == "fixconn_weight":
            self.fname = val

    def init_connection(self, nodes_in, nodes_out):
        _check(len(nodes_in) == 1 and len(nodes_out) == 1, "FixConnLayer: Layer only support 1-1 connection")
        _check(nodes_in[0].is_mat(), "FixConnLayer: input need to be a matrix")
        _check(self.lp.num_hidden > 0, "FixConncLayer: must set nhidden correctly")
        _check(self.fname != "NULL", "FixConnLayer: must specify fixconn_weight")
        nin = nodes_in[0].shape[3]
        nodes_out[0].set_shape(nodes_in[0].batch, 1, 1, self.lp.num_hidden)
        w = torch.zeros(self.lp.num_hidden, nin)
        with open(self.fname) as f:
            toks = f.read().split()
        nrow, ncol, nnz = int(toks[0]), int(toks[1]), int(toks[2])
        _check(nrow == w.shape[0] and ncol == w.shape[1], "FixConnLayer: fixconn_weight shape do not match architecture")
        for i in range(nnz):
            r, c, v = int(toks[3 + 3 * i]), int(toks[4 + 3 * i]), float(toks[5 + 3 * i])
            _check(r < nrow and c < ncol, "FixConnLayer: fixconn_weight index exceed matrix shape")
            w[r, c] = v
        self.w_host = w
        self.wdev = None

    def forward(self, is_train, nodes_in, nodes_out):
        x = nodes_in[0].mat()
        if self.wdev is None:
            self.wdev = self.w_host.to(x.device, x.dtype)
        ops.fc_forward(x, self.wdev, None, nodes_out[0].mat())

    def backprop(self, prop_grad, nodes_in, nodes_out):
        if prop_grad:
            ops.fc_backward_data(nodes_out[0].mat(), self.wdev, nodes_in[0].mat())


class PairTestLayer(Layer):
    """`pairtest-A-B` -- reference src/layer/pairtest_layer-inl.hpp:14-200: runs master and
    slave on identical inputs and reports forward/backward discrepancies (relative L1 error
    > 1e-5, or a bf16-aware bound on the GPU).  `master:`/`slave:` key prefixes configure
    each side.  The master's results are propagated."""
    type_name = "pairtest"
    allow_sharing = False


    def replay_safe(self) -> bool:
        return False  # host-side per-step values / torch ops: the eager executor runs it

    def __init__(self, ctx, master, slave):
        super().__init__(ctx)
        self.master, self.slave = master, slave
        self.tol = 1e-5 if not ctx.is_gpu else 2e-2
        self.reports = []

    def set_param(self, name, val):
        if name.startswith("master:"):
            self.master.set_param(name[7:], val)
        elif name.startswith("slave:"):
            self.slave.set_param(name[6:], val)
        else:
            self.master.set_param(name, val)
            self.slave.set_param(name, val)

    def init_connection(self, nodes_in, nodes_out):
        from .base import Node
        self.master.init_connection(nodes_in, nodes_out)
        self.s_in = [Node(n.name + "@slave") for n in nodes_in]
        self.s_out = [Node(n.name + "@slave") for n in nodes_out]
        for a, b in zip(self.s_in, nodes_in):
            a.set_shape(*b.shape, cp=b.cp)
        self.slave.init_connection(self.s_in, self.s_out)
        self.params = list(self.master.declare_params()) + list(self.slave.declare_params())
        self.n_master = len(self.master.params)

    def _alloc(self):
        for n in self.s_in + self.s_out:
            if n.data is None:
                n.alloc(self.ctx.device, self.ctx.act_dtype)

    @staticmethod
    def _relerr(a, b):
        a, b = a.float(), b.float()
        return ((a - b).abs().sum() / (b.abs().sum() + 1e-12)).item()

    def _cmp(self, what, a, b):
        e = self._relerr(a, b)
        if e > self.tol:
            msg = f"[pairtest] {self.master.type_name}-{self.slave.type_name} {what}: rel err {e:.3e}"
            self.reports.append(msg)
            print(msg)

    def forward(self, is_train, nodes_in, nodes_out):
        self._alloc()
        for a, b in zip(self.s_in, nodes_in):
            a.data.copy_(b.data)
        for pm, ps in zip(self.master.params, self.slave.params):
            self._cmp("weight", ps.w, pm.w)
        self.master.forward(is_train, nodes_in, nodes_out)
        self.slave.forward(is_train, self.s_in, self.s_out)
        for i, (a, b) in enumerate(zip(self.s_out, nodes_out)):
            self._cmp(f"forward out[{i}]", a.data, b.data)

    def backprop(self, prop_grad, nodes_in, nodes_out):
        for a, b in zip(self.s_out, nodes_out):
            a.data.copy_(b.data)
        self.master.backprop(prop_grad, nodes_in, nodes_out)
        self.slave.backprop(prop_grad, self.s_in, self.s_out)
        for pm, ps in zip(self.master.params, self.slave.params):
            self._cmp("grad", ps.g, pm.g)
        if prop_grad:
            for i, (a, b) in enumerate(zip(self.s_in, nodes_in)):
                self._cmp(f"backprop in[{i}]", a.data, b.data)

    def save_model(self, fo):
        self.master.save_model(fo)
        self.slave.save_model(fo)

    def load_model(self, fi):
        self.master.load_model(fi)
        self.slave.load_model(fi)

    def loaded_values(self):
        out = []
        for l in (self.master, self.slave):
            if hasattr(l, "loaded_values"):
                out += l.loaded_values()
        return out


def _register():
    from . import register
    register(17, BiasLayer)
    register(23, SplitLayer)
    register(18, lambda ctx: ConcatLayer(ctx, 3))
    register(28, lambda ctx: ConcatLayer(ctx, 1))
    register(30, BatchNormLayer)
    register(29, PReluLayer)
    register(24, InsanityLayer)
    register(25, InsanityPoolingLayer)
    register(31, FixConnectLayer)


_register()
