"""Standard layers: fullc, conv, activations, pooling, lrn, dropout, flatten, losses.

Every layer reproduces the forward/backward semantics of the reference layer cited
in its docstring; the device work is done by cxxnet_amd.ops (HIP kernels on the GPU).
Gradients of inputs overwrite the input node (the reference's buffer-sharing scheme:
the same node holds the activation in forward and its gradient in backward).
"""
from __future__ import annotations

import os

import torch

from .. import ops
from ..ops.gemm import ConvGeom, conv_out_size, deterministic
from .base import BinReader, BinWriter, Layer, Node, ParamSpec

# CXXNET_CONV_PREPAD=0 disables the zero-bordered-copy path of few-channel padded convs
_PREPAD = os.environ.get("CXXNET_CONV_PREPAD", "1") != "0"


def _check(cond, msg):
    if not cond:
        raise ValueError(msg)




def _bias_init(val):
    return lambda t: t.fill_(val)


# ============================================================================ fullc
class FullConnectLayer(Layer):
    """`fullc` -- reference src/layer/fullc_layer-inl.hpp:13-146.
    out = in . W^T + b;  gW += out_g^T . in;  gb += sum_rows(out_g);  in_g = out_g . W
    """
    replay_audited = True  # library kernels only (tests/test_launch_hygiene_gpu.py)
    type_name = "fullc"

    def __init__(self, ctx):
        super().__init__(ctx)
        self.fullc_gather = -1  # 1 on, 0 off, -1 auto (_gathering)
        self.fuse_relu = False
        self.fuse_dropout = None  # the DropoutLayer behind a fused relu (NeuralNet._fuse_dropout)
        self.grad_alpha = 1.0     # data-gradient scale: 1 / pkeep of a fused dropout in front
        self._dx = None
        self._rows = 0
        self._gbuf = {}      # persistent gather sources / outputs (graph-capturable)
        self._xwork = None   # the forward's all-gather of x, waited in backprop
        self._dywork = None  # world > 1: backprop's dy all-gather in flight

    def set_param(self, name, val):
        super().set_param(name, val)
        if name == "fullc_gather":
            self.fullc_gather = -1 if str(val).strip().lower() == "auto" else int(val)

    def init_connection(self, nodes_in, nodes_out):
        _check(len(nodes_in) == 1 and len(nodes_out) == 1, "FullcLayer: only support 1-1 connection")
        x = nodes_in[0]
        _check(x.is_mat(), "FullcLayer: input need to be a matrix")
        _check(self.lp.num_hidden > 0, "FullcLayer: must set nhidden correctly")
        nin = x.shape[1] * x.shape[2] * x.shape[3]
        if self.lp.num_input_node == 0:
            self.lp.num_input_node = nin
        else:
            _check(self.lp.num_input_node == nin, "FullcLayer: input hidden nodes is not consistent")
        nodes_out[0].set_shape(x.batch, 1, 1, self.lp.num_hidden)
        self._rows = x.batch
        nh, ni = self.lp.num_hidden, self.lp.num_input_node

        def init_w(t):
            self._init_weight(t, ni, nh)
        self.params = [ParamSpec("wmat", (nh, ni), init_w, overwrite=True)]
        self.params[0].no_reduce = self._gathering()
        if self.lp.no_bias == 0:
            self.params.append(ParamSpec("bias", (nh,), _bias_init(self.lp.init_bias)))

    @property
    def w(self):
        return self.params[0]

    @property
    def b(self):
        return self.params[1] if len(self.params) > 1 else None

    def _gathering(self) -> bool:
        """fullc_gather (reference fullc_layer-inl.hpp:120-122 + async_updater-inl.hpp:
        67-93): instead of all-reducing the nout x nin weight gradient, all-gather the
        B x (nin + nout) activations/gradients of every rank and form the global
        gradient locally.  Under data parallelism only (dp_force: a one-rank process group
        runs the gather too -- the RCCL path on one GPU).

        fullc_gather = -1 (auto, the default) gathers when the gathered rows are fewer bytes
        than the fp32 gradient they replace: world * B_local * (nin + nout) * 2 (bf16) <
        nin * nout * 4.  AlexNet fc6 at 8 x 32 rows: 6.8 MB against 151 MB; the layer then
        also takes its SGD step inside the weight-gradient GEMM (_fused_sgd).  The result is
        the same global gradient either way; only the traffic differs."""
        from ..parallel.dp import world_info
        world = world_info()[1]
        if not (world > 1 or bool(getattr(self.ctx, "dp_force", False))):
            return False
        if self.fullc_gather >= 0:
            return bool(self.fullc_gather)
        if self.ctx.is_gpu:
            import torch.distributed as dist
            if dist.get_backend() != "nccl":  # gloo rehearsal ranks on a GPU: device tensors stay on all-reduce
                return False
        nin, nout = self.lp.num_input_node, self.lp.num_hidden
        return world * max(self._rows, 1) * (nin + nout) * 2 < nin * nout * 4

    def _collective(self, fn):
        """Run the collective call fn now -- or, while the step is being captured as HIP
        graphs or recorded as C++ launch lists (NetTrainer._capture_plans / _record_plans set
        ctx.graph_cut), end the current segment and keep fn as an eager call between segments:
        RCCL cannot join a capturing stream, a launch list holds library kernels only, and
        every replay re-issues the gather on the same persistent buffers."""
        cut = getattr(self.ctx, "graph_cut", None)
        if cut is not None:
            cut(fn)
        else:
            fn()

    def _gather_io(self, key, t, rows):
        """(source, output) of the all-gather of matrix t: persistent buffers, the source
        zero-padded to `rows` (the node's capacity = the trainer's ceil(B/world) split, equal
        on every rank), so an uneven split still gathers equal pieces and zero rows add
        nothing to dW = dy^T x."""
        import torch.distributed as dist
        world = dist.get_world_size()
        cols = t.shape[1]
        buf = self._gbuf.get(key)
        if buf is None or buf[1].shape != (world * rows, cols) or buf[1].dtype != t.dtype:
            src = torch.zeros((rows, cols), dtype=t.dtype, device=t.device)
            buf = (src, torch.empty((world * rows, cols), dtype=t.dtype, device=t.device))
            self._gbuf[key] = buf
        src, out = buf
        if t.shape[0] == rows and t.is_contiguous():
            return t, out
        ops.copy_(src[: t.shape[0]], t.contiguous())
        return src, out

    def forward(self, is_train, nodes_in, nodes_out):
        bias = self.b.w if self.b is not None else None
        x = nodes_in[0].mat()
        if is_train and self._gathering():
            # backprop overwrites the input node with its gradient: gather it now (async:
            # the gather overlaps the rest of the forward and the backward above this layer)
            import torch.distributed as dist
            src, out = self._gather_io("x", x, nodes_in[0].shape[0])

            def gather_x():
                self._xwork = dist.all_gather_into_tensor(out, src, async_op=True)
            self._collective(gather_x)
        d = self.fuse_dropout
        drop = (d.seed, self.ctx.step_counter, 1.0 - d.threshold) if (d is not None and is_train) else None
        ops.fc_forward(x, self.w.wb, bias, nodes_out[0].mat(), relu=self.fuse_relu, drop=drop)

    def _dx_scratch(self, x):
        if self._dx is None or self._dx.shape[0] < x.shape[0] or self._dx.shape[1] != x.shape[1]:
            self._dx = torch.empty_like(x)
        return self._dx[:x.shape[0]]

    def _fused_sgd(self, x, dy, prop_grad, nodes_in, xw=None, dyw=None, gx=None) -> bool:
        """SGD step of the weights fused into the weight-gradient GEMM (ctx.sgd_fuse = the
        arena updater, set by the trainer when eligible): one GPU, or -- under data
        parallelism -- a fullc_gather layer, whose gradient is formed from the all-gathered
        rows (xw, dyw) and is the same global gradient on every rank.  The data gradient reads
        the OLD shadow weights, so it runs first, into a scratch buffer (x, which the
        weight-gradient still needs, lives where it goes); the scratch is copied back (with
        relu' when fused) after the update.  gx: that data gradient, already computed (the
        gathered path runs it while the dy all-gather is in flight)."""
        upd = getattr(self.ctx, "sgd_fuse", None)
        if upd is None or not (getattr(self.ctx, "grad_overwrite", False) and self.w.overwrite) or not self.ctx.is_gpu:
            return False
        if getattr(self.ctx, "sgd_fuse_gather_only", False) and xw is None:
            return False  # a gradient still to be reduced: the step must follow the reduction
        # under data parallelism the trainer hands out the updater for gathered layers only
        assert not getattr(self.ctx, "dp_active", False) or getattr(self.ctx, "sgd_fuse_gather_only", False)
        spec = self.w
        lr, wd, mom, clip = upd.hyper(spec, self.ctx.epoch)
        # a planned step (launch list / HIP graph) reads the schedule values from the updater's
        # device table, refreshed before every replay (NetTrainer._stage_fused_sgd)
        hyp = upd.hyper_dev(spec) if getattr(self.ctx, "sgd_hyp_dev", False) else None
        a = upd.arena
        m = a.m1[spec.offset:spec.offset + spec.numel].view(spec.shape)
        side = getattr(self.ctx, "fc_side", None)
        if side is not None and xw is not None:
            # data parallel, gathered rows: the data gradient (local rows, old shadow weights) on
            # the main stream, then the fused step on `side` -- it reads only the gathered copies,
            # so the conv backward below runs beside it (joined at the end of NeuralNet.backprop)
            if prop_grad and gx is None:
                gx = self._dx_scratch(x)
                ops.fc_backward_data(dy, spec.wb, gx, alpha=self.grad_alpha)
            ready = torch.cuda.Event()
            ready.record()
            side.wait_event(ready)
            with torch.cuda.stream(side):
                ok = ops.fc_backward_weight_sgd(xw, dyw, spec.w, m, spec.wb, lr, wd, mom, clip, hyp)
            self.ctx.fc_side_used = True
            if ok:
                upd.fused_offsets.add(spec.offset)
            else:
                torch.cuda.current_stream().wait_stream(side)
                ops.fc_backward_weight(xw, dyw, spec.g, overwrite=True)
            if gx is not None:
                dst = nodes_in[0].gmat()
                ops.channel_copy(gx, 0, dst, 0, dst.shape[1], mask_relu=self.grad_mask_relu)
            return True
        if side is not None and xw is None:
            # side stream: x is copied aside (its buffer receives the data gradient), the data
            # gradient reads the old shadow weights on the main stream, then the fused step runs
            # on `side` (joined at the end of the backward pass, NeuralNet.backprop)
            if getattr(self, "_xs", None) is None or self._xs.shape != x.shape:
                self._xs = torch.empty_like(x)
            ops.copy_(self._xs, x)  # a library copy: recorded launch lists repeat it
            if prop_grad:
                ops.fc_backward_data(dy, spec.wb, nodes_in[0].gmat(), mask_relu=self.grad_mask_relu,
                                     alpha=self.grad_alpha)
            ready = torch.cuda.Event()
            ready.record()
            side.wait_event(ready)
            # the side stream reads tensors the main stream allocated: keep the allocator from
            # recycling them until its work is done (dy is a persistent node today; this keeps it
            # safe if it ever becomes a temporary)
            dy.record_stream(side)
            self._xs.record_stream(side)
            with torch.cuda.stream(side):
                ok = ops.fc_backward_weight_sgd(self._xs, dy, spec.w, m, spec.wb, lr, wd, mom, clip, hyp)
            self.ctx.fc_side_used = True
            if ok:
                upd.fused_offsets.add(spec.offset)
            else:
                torch.cuda.current_stream().wait_stream(side)
                ops.fc_backward_weight(self._xs, dy, spec.g, overwrite=True)
            return True
        if prop_grad and gx is None:
            gx = self._dx_scratch(x)
            ops.fc_backward_data(dy, spec.wb, gx, alpha=self.grad_alpha)
        xg, dyg = (x, dy) if xw is None else (xw, dyw)
        if ops.fc_backward_weight_sgd(xg, dyg, spec.w, m, spec.wb, lr, wd, mom, clip, hyp):
            upd.fused_offsets.add(spec.offset)
        else:  # the kernel does not cover this shape: plain gradient, updated by the updater
            ops.fc_backward_weight(xg, dyg, spec.g, overwrite=True)
        if gx is not None:
            dst = nodes_in[0].gmat()
            ops.channel_copy(gx, 0, dst, 0, dst.shape[1], mask_relu=self.grad_mask_relu)
        return True

    def backprop(self, prop_grad, nodes_in, nodes_out):
        x, dy = nodes_in[0].mat(), nodes_out[0].mat()
        overwrite = getattr(self.ctx, "grad_overwrite", False) and self.w.overwrite
        if not self._gathering() and self._fused_sgd(x, dy, prop_grad, nodes_in):
            if self.b is not None:
                self.ctx.bias_grad(dy, self.b.g)
            return
        if self._gathering():
            import torch.distributed as dist
            dsrc, dyw = self._gather_io("dy", dy, nodes_out[0].shape[0])
            x_all = self._gbuf["x"][1]
            # world > 1: the dy all-gather runs while the data gradient (local rows, old weights)
            # is formed into a scratch buffer -- x's buffer, where it goes, may still be the x
            # gather's source; at world 1 there is nothing to overlap and the extra segment cut
            # of a recorded step costs more (profiles/r5_dp_world1.md), so the gather comes first
            early = dist.get_world_size() > 1
            gx = None
            if early:
                def gather_dy_async():
                    self._dywork = dist.all_gather_into_tensor(dyw, dsrc, async_op=True)
                self._collective(gather_dy_async)
                if prop_grad:
                    gx = self._dx_scratch(x)
                    ops.fc_backward_data(dy, self.w.wb, gx, alpha=self.grad_alpha)

            def gather_dy():
                # the compute stream waits for both gathers (no host block)
                if early:
                    self._dywork.wait()
                    self._dywork = None
                else:
                    dist.all_gather_into_tensor(dyw, dsrc)
                if self._xwork is not None:
                    self._xwork.wait()
                    self._xwork = None
            self._collective(gather_dy)
            if self._fused_sgd(x, dy, prop_grad, nodes_in, xw=x_all, dyw=dyw, gx=gx):
                if self.b is not None:
                    self.ctx.bias_grad(dy, self.b.g)
                return
            ops.fc_backward_weight(x_all, dyw, self.w.g, overwrite=overwrite)
            if gx is not None:
                if self.b is not None:
                    self.ctx.bias_grad(dy, self.b.g)
                dst = nodes_in[0].gmat()
                ops.channel_copy(gx, 0, dst, 0, dst.shape[1], mask_relu=self.grad_mask_relu)
                return
        else:
            ops.fc_backward_weight(x, dy, self.w.g, overwrite=overwrite)
        if self.b is not None:
            self.ctx.bias_grad(dy, self.b.g)
        if prop_grad:
            ops.fc_backward_data(dy, self.w.wb, nodes_in[0].gmat(), mask_relu=self.grad_mask_relu,
                                 alpha=self.grad_alpha)

    def save_model(self, fo: BinWriter):
        fo.write(self.lp.to_bytes())
        fo.write_tensor(self.w.w.view(self.w.shape))
        fo.write_tensor(self.b.w if self.b is not None else torch.zeros(self.lp.num_hidden))

    def load_model(self, fi: BinReader):
        self.lp = fi.read_layer_param()
        self.loaded = [fi.read_tensor(2), fi.read_tensor(1)]

    def loaded_values(self):
        w, b = self.loaded
        out = [w]
        if self.lp.no_bias == 0:
            out.append(b)
        return out


# ============================================================================ conv
def _pixel_rows(t: torch.Tensor) -> torch.Tensor:
    """[pixels][C] view of an NHWC activation; a channel slice of a zero-copy ch_concat buffer
    (NeuralNet._fuse_concat) keeps the full buffer's pixel stride as its row stride."""
    if t.is_contiguous():
        return t.view(-1, t.shape[-1])
    n, h, w, c = t.shape
    return t.as_strided((n * h * w, c), (t.stride(2), 1))


class ConvolutionLayer(Layer):
    """`conv` -- reference src/layer/convolution_layer-inl.hpp:12-228.

    Weights are stored internally as [Cout][KH][KW][Cin/g] (NHWC-friendly); the
    checkpoint keeps the reference (g, Cout/g, Cin/g*KH*KW) layout in (ci, kh, kw) order.
    The im2col buffer never exists: the MFMA kernel gathers patches on the fly.
    """
    replay_audited = True  # library kernels only (tests/test_launch_hygiene_gpu.py)
    type_name = "conv"

    def __init__(self, ctx):
        super().__init__(ctx)
        self.fuse_relu = False
        self.geo = None
        self._wt = None
        self._xpad = None
        self._prepad_on = False
        self.bias_done = False  # set by a fused max-pool backward that already summed the bias gradient
        # the conv below whose bias gradient this conv's data-gradient epilogue sums
        # (NeuralNet._fuse_dgrad_bias); None = not fused
        self.bias_below = None
        # sibling group (NeuralNet._fuse_siblings): the lead holds the group (dict), the other
        # members compute nothing themselves
        self.sib = None
        self.sib_member = False

    def init_connection(self, nodes_in, nodes_out):
        _check(len(nodes_in) == 1 and len(nodes_out) == 1, "ConvolutionLayer: only support 1-1 connection")
        lp = self.lp
        x = nodes_in[0]
        b, c, h, w = x.shape
        _check(lp.num_channel > 0, "must set nchannel correctly")
        _check(lp.kernel_height > 0 and lp.kernel_width > 0, "must set kernel_size correctly")
        _check(lp.kernel_width <= w + 2 * lp.pad_x and lp.kernel_height <= h + 2 * lp.pad_y,
               "kernel size exceed input")
        if lp.num_input_channel == 0:
            lp.num_input_channel = c
        else:
            _check(lp.num_input_channel == c, "ConvolutionLayer: number of input channels is not consistent")
        G = lp.num_group
        _check(c % G == 0 and lp.num_channel % G == 0, "ConvolutionLayer: channels must divide ngroup")
        Ho, Wo = conv_out_size(h, w, lp.kernel_height, lp.kernel_width, lp.stride, lp.pad_y, lp.pad_x)
        nodes_out[0].set_shape(b, lp.num_channel, Ho, Wo)
        self.cin_phys = x.cp
        # physical row width: the row-padded 3-channel input (NeuralNet._pad_input_channels)
        self.geo = ConvGeom(b, h, max(w, x.wp), x.cp, Ho, Wo, lp.num_channel, lp.kernel_height, lp.kernel_width,
                            lp.stride, lp.pad_y, lp.pad_x, G)
        cg_l, cg_p = c // G, x.cp // G
        kh, kw, co = lp.kernel_height, lp.kernel_width, lp.num_channel
        # few input channels with padding (VGG's 3x3 pad-1 first conv on 4 channels): forward and
        # weight-grad run on a zero-bordered copy of x, so the row-gather GEMM (whole kernel-row
        # runs, pad 0 only) serves them instead of the per-tap gather with 4-channel chunks
        self._prepad_on = (cg_p % 8 != 0 and G == 1 and (lp.pad_y or lp.pad_x) and x.cp % 4 == 0
                           and _PREPAD)

        def init_w(t):
            logical = torch.empty(G, co // G, cg_l * kh * kw, device=t.device)
            self._init_weight(logical, cg_l * kh * kw, co // G)
            t.copy_(self.from_logical(logical))
        self.params = [ParamSpec("wmat", (co, kh, kw, cg_p), init_w)]
        if lp.no_bias == 0:
            self.params.append(ParamSpec("bias", (co,), _bias_init(lp.init_bias)))

    # logical (G, Cout/G, Cg*KH*KW) in (ci, kh, kw) order  <->  internal [Cout][KH][KW][Cg_phys]
    def from_logical(self, logical: torch.Tensor) -> torch.Tensor:
        lp = self.lp
        G, co, kh, kw = lp.num_group, lp.num_channel, lp.kernel_height, lp.kernel_width
        cg_l = lp.num_input_channel // G
        cg_p = self.cin_phys // G
        t = logical.reshape(co, cg_l, kh, kw).permute(0, 2, 3, 1)
        out = torch.zeros(co, kh, kw, cg_p, dtype=logical.dtype, device=logical.device)
        out[..., :cg_l] = t
        return out

    def to_logical(self, internal: torch.Tensor) -> torch.Tensor:
        lp = self.lp
        G, co, kh, kw = lp.num_group, lp.num_channel, lp.kernel_height, lp.kernel_width
        cg_l = lp.num_input_channel // G
        t = internal.detach().float().cpu()[..., :cg_l].permute(0, 3, 1, 2)  # co, cg, kh, kw
        return t.reshape(G, co // G, cg_l * kh * kw).contiguous()

    def on_batch_size_changed(self, nodes_in, nodes_out):
        self.geo.N = nodes_in[0].data.shape[0]

    @property
    def w(self):
        return self.params[0]

    @property
    def b(self):
        return self.params[1] if len(self.params) > 1 else None

    def _padded(self, x, refresh):
        """(input, geometry) for forward / weight-grad: x itself, or (pre-pad path) the
        zero-bordered copy of x with a pad-0 geometry.  refresh=False reuses the forward's copy
        (x is unchanged until this layer's own backprop writes its gradient)."""
        g = self.geo
        if not (self._prepad_on and self.ctx.is_gpu):
            return x, g
        N = x.shape[0]
        H2, W2 = g.H + 2 * g.pad_y, g.W + 2 * g.pad_x
        if self._xpad is None or self._xpad.shape[0] < N:
            self._xpad = torch.zeros(N, H2, W2, g.C, dtype=x.dtype, device=x.device)
            refresh = True
        xp = self._xpad[:N]
        if refresh:
            ops.pad_interior(x, xp, g.pad_y, g.pad_x)
        return xp, ConvGeom(N, H2, W2, g.C, g.Ho, g.Wo, g.Cout, g.KH, g.KW, g.stride, 0, 0, g.groups)

    def _sib_geo(self, cout):
        g = self.geo
        return ConvGeom(g.N, g.H, g.W, g.C, g.Ho, g.Wo, cout, 1, 1, 1, 0, 0, 1)

    def forward(self, is_train, nodes_in, nodes_out):
        self.geo.N = nodes_in[0].data.shape[0]
        if self.sib_member:  # computed by the group's lead
            return
        bias = self.b.w if self.b is not None else None
        S = self.sib
        if S is not None:  # all siblings as one GEMM into their group buffer H
            ops.conv_forward(nodes_in[0].data, S["w_all"], S["b_all"], S["H"][:self.geo.N], self._sib_geo(S["ctot"]),
                             relu=self.fuse_relu)
            return
        # few-channel first layers on direct kernels that pad on the fly (GoogLeNet conv1: the
        # row-run forward; VGG conv1_1: conv_fewc); a zero-bordered copy is then built only by a
        # weight-gradient pass that needs it
        if self.geo.C <= 4 and ops.gemm.conv_rowrun_fwd2(nodes_in[0].data, self.w.wb, bias, nodes_out[0].data,
                                                         self.geo, relu=self.fuse_relu):
            self._xpad_stale = True
            return
        if ops.gemm.fewc_preferred(self.geo) and ops.gemm.conv_forward_fewc(
                nodes_in[0].data, self.w.wb, bias, nodes_out[0].data, self.geo, relu=self.fuse_relu):
            self._xpad_stale = True
            return
        x, geo = self._padded(nodes_in[0].data, True)
        self._xpad_stale = False
        ops.conv_forward(x, self.w.wb, bias, nodes_out[0].data, geo, relu=self.fuse_relu)

    def backprop(self, prop_grad, nodes_in, nodes_out):
        if self.sib_member:  # the group's lead runs this layer's backward with its own
            return
        x, dy = nodes_in[0].data, nodes_out[0].data
        self.geo.N = x.shape[0]
        S = self.sib
        if S is not None:
            # every sibling at once: their dy is H itself (the consumers of the slices wrote it)
            H = S["H"][:x.shape[0]]
            gall = self._sib_geo(S["ctot"])
            ops.conv_backward_weight(x, H, S["w_g"], gall)
            if S["b_g"] is not None:
                self.ctx.bias_grad(_pixel_rows(H), S["b_g"])
            if prop_grad:
                ready = self.ctx.flipped is not None and id(self) in self.ctx.flipped
                fold = S.get("fold")  # the split's sum folded into this GEMM (NeuralNet._fuse_siblings)
                if fold is not None:
                    sp = fold["split"]
                    dst, add = fold["dst"].gdst[:x.shape[0]], fold["add"].gdst[:x.shape[0]]
                    sp.folded = ops.gemm.conv_backward_data_add(H, S["w_all"], dst, add, gall, S["wt"],
                                                                mask_relu=sp.grad_mask_relu, wt_ready=ready)
                    if sp.folded:
                        return
                ops.conv_backward_data(H, S["w_all"], S["dx_node"].gdst, gall, S["wt"], wt_ready=ready)
            return
        want_db = self.b is not None and not self.bias_done and self.ctx.is_gpu
        if self.geo.C <= 4 and self.ctx.is_gpu and ops.gemm.conv_wgrad_rowrun(x, dy, self.w.g, self.geo):
            db_done = False  # (few-channel first layer, padding staged on the fly: no bordered copy)
        else:
            xw, geo = self._padded(x, getattr(self, "_xpad_stale", False))
            self._xpad_stale = False
            db_done = ops.conv_backward_weight(xw, dy, self.w.g, geo, db=self.b.g if want_db else None)
        if self.bias_done:  # summed by the max-pool behind this conv (NeuralNet._fuse_pool_bias)
            self.bias_done = False
        elif self.b is not None and not db_done:  # (db_done: summed by the weight-gradient kernel)
            self.ctx.bias_grad(_pixel_rows(dy), self.b.g)
        if prop_grad:
            ready = self.ctx.flipped is not None and id(self) in self.ctx.flipped
            below = self.bias_below
            db = None
            if below is not None and below.b is not None and self.ctx.is_gpu and not deterministic():
                db = below.b.g
            if ops.conv_backward_data(dy, self.w.wb, nodes_in[0].gdst, self.geo, self.flip_target()[1],
                                      mask_relu=self.grad_mask_relu, wt_ready=ready, dbias=db):
                below.bias_done = True

    def extra_flip_targets(self):
        """Flip items besides flip_target(): a sibling group's stacked weights."""
        S = self.sib
        if S is None:
            return []
        return [(S["w_all"], S["wt"], self._sib_geo(S["ctot"]))]

    def flip_target(self):
        """(weights, flipped-weights buffer, geometry) of the data-gradient GEMM."""
        if self._wt is None or self._wt.shape != self.w.wb.shape:
            self._wt = torch.empty_like(self.w.wb)
        return self.w.wb, self._wt, self.geo

    def save_model(self, fo: BinWriter):
        fo.write(self.lp.to_bytes())
        fo.write_tensor(self.to_logical(self.w.w.view(self.w.shape)))
        fo.write_tensor(self.b.w if self.b is not None else torch.zeros(self.lp.num_channel))

    def load_model(self, fi: BinReader):
        self.lp = fi.read_layer_param()
        self.loaded = [fi.read_tensor(3), fi.read_tensor(1)]

    def loaded_values(self):
        w, b = self.loaded
        out = [self.from_logical(w)]
        if self.lp.no_bias == 0:
            out.append(b)
        return out


# ============================================================================ activations
class ActivationLayer(Layer):
    """`relu`/`sigmoid`/`tanh` -- reference src/layer/activation_layer-inl.hpp:11-40;
    `xelu` -- src/layer/xelu_layer-inl.hpp:15-50.  Applied in place on the input node
    and copied to the output node; the gradient is expressed through the output."""
    replay_audited = True  # library kernels only (tests/test_launch_hygiene_gpu.py)

    def __init__(self, ctx, kind):
        super().__init__(ctx)
        self.kind = kind
        self.type_name = kind
        self.b = 5.0
        self.fused_into_producer = False

    def set_param(self, name, val):
        super().set_param(name, val)
        if name == "b":
            self.b = float(val)

    def init_connection(self, nodes_in, nodes_out):
        _check(len(nodes_in) == 1 and len(nodes_out) == 1, "ActivationLayer: only support 1-1 connection")
        nodes_out[0].set_shape(*nodes_in[0].shape, cp=nodes_in[0].cp)

    def forward(self, is_train, nodes_in, nodes_out):
        x, y = nodes_in[0], nodes_out[0]
        if self.fused_into_producer:
            # the producer's epilogue applied the activation and y aliases x: nothing to do
            return
        if x is y:
            ops.act_forward(self.kind, x.data, x.data, None, self.b)
        else:
            ops.act_forward(self.kind, x.data, y.data, x.data, self.b)

    def backprop(self, prop_grad, nodes_in, nodes_out):
        if self.fused_into_producer:
            return  # relu' was applied by the layer that wrote this node's gradient
        x, y = nodes_in[0], nodes_out[0]
        # x holds f(input) (in-place forward), y holds the incoming gradient
        ops.act_backward(self.kind, x.data, y.data, x.data, self.b)


# ============================================================================ pooling
class PoolingLayer(Layer):
    """`max_pooling`/`sum_pooling`/`avg_pooling`/`relu_max_pooling` --
    reference src/layer/pooling_layer-inl.hpp:11-114 (ceil-mode windows).  Extension: `pad`
    is honoured (the reference parses but ignores it).

    Max-unpool ties: the reference compares values, so EVERY input equal to a window's max
    gets the gradient (`unpool<red::maximum>`, :55-86).  The default here (`pool_tie = first`)
    routes it to the first maximum only, recorded as a uint8 offset in forward (no saved
    output, no re-read of it in backward).  `pool_tie = all` reproduces the reference: the
    pooled output is saved and the backward compares values (ops.pool_backward_tie_all).
    Ties only occur between bit-identical activations (e.g. windows of relu zeros, which get
    no gradient through a fused relu either way)."""
    replay_audited = True  # library kernels only (tests/test_launch_hygiene_gpu.py)

    def __init__(self, ctx, mode, relu=False):
        super().__init__(ctx)
        self.mode = mode
        self.relu = relu
        self.type_name = ("relu_" if relu else "") + {"max": "max", "sum": "sum", "avg": "avg"}[mode] + "_pooling"
        self.state = None
        self.tie_all = False
        self.ysave = None
        # the conv in front whose bias gradient this pool's backward provides (executor fusion,
        # NeuralNet._fuse_pool_bias); None = not fused
        self.bias_of = None
        # (LRN layer, its output node) run inside this pool's kernels (NeuralNet._fuse_pool_lrn)
        self.fused_lrn = None
        # the input can only hold values >= 0 (NeuralNet._mark_nonneg): max on integer keys
        self.input_nonneg = False
        self._dbpart = None

    def set_param(self, name, val):
        super().set_param(name, val)
        if name == "pool_tie":
            if val not in ("first", "all"):
                raise ValueError("pool_tie must be first or all")
            self.tie_all = val == "all"

    def init_connection(self, nodes_in, nodes_out):
        _check(len(nodes_in) == 1 and len(nodes_out) == 1, "PoolingLayer: only support 1-1 connection")
        lp = self.lp
        b, c, h, w = nodes_in[0].shape
        _check(lp.kernel_height > 0 and lp.kernel_width > 0, "must set kernel_size correctly")
        _check(lp.kernel_width <= w + 2 * lp.pad_x and lp.kernel_height <= h + 2 * lp.pad_y,
               "kernel size exceed input")
        ho = ops.pool_out_size(h, lp.kernel_height, lp.stride, lp.pad_y)
        wo = ops.pool_out_size(w, lp.kernel_width, lp.stride, lp.pad_x)
        nodes_out[0].set_shape(b, c, ho, wo, cp=nodes_in[0].cp)

    def _state(self, y: Node):
        # max mode: first-max window offsets (uint8); sum/avg need no state
        if self.mode != "max":
            return None
        if self.state is None or self.state.shape != y.data.shape:
            self.state = torch.empty(y.data.shape, dtype=torch.uint8, device=y.data.device)
        return self.state

    def _tie_all(self) -> bool:
        return self.tie_all and self.mode == "max"

    def replay_safe(self) -> bool:
        return not self._tie_all()  # keeps its output with a torch copy

    def forward(self, is_train, nodes_in, nodes_out):
        lp = self.lp
        if self.fused_lrn is not None:
            lrn, yout = self.fused_lrn
            st = self._state(nodes_out[0])  # (also in eval: the fused kernel always writes offsets)
            # bit 2: the input can only be >= 0 (NeuralNet._mark_nonneg): max on integer keys
            flags = int(bool(self.relu)) | (2 if self._mask_in_state() else 0) | (4 if self.input_nonneg else 0)
            if ops.pool_lrn_forward(nodes_in[0].data, nodes_out[0].data, st, yout.data, flags, lrn.nsize, lrn.alpha,
                                    lrn.beta, lrn.knorm):
                return
            ops.pool_forward(nodes_in[0].data, nodes_out[0].data, st, lp.kernel_height, lp.kernel_width, lp.stride,
                             lp.pad_y, self.mode, self.relu, mark_mask=self._mask_in_state(), nonneg=self.input_nonneg)
            ops.lrn_forward(nodes_out[0].data, yout.data, lrn.nsize, lrn.alpha, lrn.beta, lrn.knorm)
            return
        st = self._state(nodes_out[0]) if is_train else None
        ops.pool_forward(nodes_in[0].data, nodes_out[0].data, st, lp.kernel_height, lp.kernel_width, lp.stride,
                         lp.pad_y, self.mode, self.relu, mark_mask=self._mask_in_state(), nonneg=self.input_nonneg)
        if is_train and self._tie_all():
            y = nodes_out[0].data
            if self.ysave is None or self.ysave.shape != y.shape:
                self.ysave = torch.empty_like(y)
            self.ysave.copy_(y)  # the output node is overwritten by its gradient before backprop

    def _mask_in_state(self) -> bool:
        lp = self.lp
        return (self.ctx.is_gpu and (self.relu or self.grad_mask_relu) and not self._tie_all()
                and ops.pool_mask_in_state(self.mode, lp.kernel_height, lp.kernel_width))

    def backprop(self, prop_grad, nodes_in, nodes_out):
        if not prop_grad:
            return
        lp = self.lp
        x = nodes_in[0].data
        relu = self.relu or self.grad_mask_relu
        if self._tie_all():
            ops.pool_backward_tie_all(x, self.ysave, nodes_out[0].data, nodes_in[0].gdst, lp.kernel_height,
                                      lp.kernel_width, lp.stride, lp.pad_y, relu=relu)
            return
        if relu and self._mask_in_state():
            relu = 2  # relu' of the argmax was recorded by the forward: no read of x
        if self.fused_lrn is not None and self._fused_backprop(nodes_in, nodes_out, relu):
            return
        conv = self.bias_of
        if conv is not None and conv.b is not None and relu in (0, 2) and self.ctx.is_gpu and not deterministic():
            # the conv's bias gradient from this pool's output gradient (before it is consumed)
            dy = nodes_out[0].data
            self.ctx.bias_grad(dy.view(-1, dy.shape[-1]), conv.b.g,
                               self.state.view(-1, dy.shape[-1]) if relu == 2 else None)
            conv.bias_done = True
        ops.pool_backward(x, self.state, nodes_out[0].data, nodes_in[0].gdst, lp.kernel_height, lp.kernel_width, lp.stride,
                          lp.pad_y, self.mode, relu)

    def _fused_backprop(self, nodes_in, nodes_out, relu) -> bool:
        """Backward of the fused pool -> LRN pair: the LRN's output gradient (held by its output
        node) straight to this pool's input gradient.  When the fused kernel declines, the LRN
        backward runs here into the pooled gradient and False sends the caller down the plain
        pool backward."""
        lrn, yout = self.fused_lrn
        pooled = nodes_out[0].data  # still the pooled output: the LRN layer's backprop did nothing
        if relu in (0, 2):
            conv = self.bias_of
            db = None
            part = None
            if conv is not None and conv.b is not None and self.ctx.is_gpu and not deterministic():
                rows = ops.lrn_pool_backward_rows(nodes_in[0].data.shape, pooled.shape, lrn.nsize)
                C = pooled.shape[-1]
                if rows > 0:
                    if self._dbpart is None or self._dbpart.shape[0] < rows or self._dbpart.shape[1] != C:
                        self._dbpart = torch.empty((rows, C), dtype=torch.float32, device=pooled.device)
                    db, part = conv.b.g, self._dbpart
            if ops.lrn_pool_backward(pooled, yout.data, self.state, nodes_in[0].gdst, int(relu == 2), lrn.nsize,
                                     lrn.alpha, lrn.beta, lrn.knorm, dbias=db, part=part):
                if db is not None:
                    conv.bias_done = True
                return True
        ops.lrn_backward(pooled, yout.data, nodes_out[0].gdst, lrn.nsize, lrn.alpha, lrn.beta, lrn.knorm)
        return False


# ============================================================================ LRN
class LRNLayer(Layer):
    """`lrn` -- reference src/layer/lrn_layer-inl.hpp:12-89 (cross-channel, knorm/alpha/beta)."""
    replay_audited = True  # library kernels only (tests/test_launch_hygiene_gpu.py)
    type_name = "lrn"

    def __init__(self, ctx):
        super().__init__(ctx)
        self.nsize = 3
        self.alpha = 0.0
        self.beta = 0.0
        self.knorm = 1.0
        self.tmp = None
        # the conv in front whose bias gradient this layer's backward sums (NeuralNet._fuse_lrn_bias)
        self.bias_of = None

    def set_param(self, name, val):
        super().set_param(name, val)
        if name == "local_size":
            self.nsize = int(val)
        elif name == "alpha":
            self.alpha = float(val)
        elif name == "beta":
            self.beta = float(val)
        elif name == "knorm":
            self.knorm = float(val)

    def init_connection(self, nodes_in, nodes_out):
        _check(len(nodes_in) == 1 and len(nodes_out) == 1, "LRNLayer: only support 1-1 connection")
        _check(nodes_in[0] is not nodes_out[0], "LRNLayer: input and output must be different nodes")
        nodes_out[0].set_shape(*nodes_in[0].shape, cp=nodes_in[0].cp)

    fused_with_pool = False  # NeuralNet._fuse_pool_lrn: the max-pool in front runs this layer

    def forward(self, is_train, nodes_in, nodes_out):
        if self.fused_with_pool:
            return
        ops.lrn_forward(nodes_in[0].data, nodes_out[0].data, self.nsize, self.alpha, self.beta, self.knorm)

    def backprop(self, prop_grad, nodes_in, nodes_out):
        if not prop_grad or self.fused_with_pool:
            return
        x = nodes_in[0].data
        conv = self.bias_of
        if conv is not None and conv.b is not None and self.ctx.is_gpu and not deterministic():
            if ops.lrn_backward_bias(x, nodes_out[0].data, nodes_in[0].gdst, self.nsize, self.alpha, self.beta,
                                     self.knorm, conv.b.g, mask_relu=self.grad_mask_relu):
                conv.bias_done = True
                return
        # in place: the LDS-staged kernel reads a pixel's whole channel row before writing it
        ops.lrn_backward(x, nodes_out[0].data, nodes_in[0].gdst, self.nsize, self.alpha, self.beta, self.knorm,
                         mask_relu=self.grad_mask_relu)


# ============================================================================ dropout
class DropoutLayer(Layer):
    """`dropout` -- reference src/layer/dropout_layer-inl.hpp:12-66 (self-loop;
    mask = (u < pkeep)/pkeep).  The mask is a counter-based hash, regenerated in
    backward instead of stored."""
    replay_audited = True  # library kernels only (tests/test_launch_hygiene_gpu.py)
    type_name = "dropout"

    def __init__(self, ctx):
        super().__init__(ctx)
        self.threshold = 0.0
        self.seed = int(torch.randint(0, 2**31 - 1, (1,), generator=ctx.gen).item())

    def set_param(self, name, val):
        super().set_param(name, val)
        if name == "threshold":
            self.threshold = float(val)

    def init_connection(self, nodes_in, nodes_out):
        _check(len(nodes_in) == 1 and len(nodes_out) == 1, "DropoutLayer: only support 1-1 connection")
        _check(nodes_in[0] is nodes_out[0], "DropoutLayer is an self-loop Layer")
        _check(0.0 <= self.threshold < 1.0, "DropoutLayer: invalid dropout threshold")

    fused_into_producer = False  # NeuralNet._fuse_dropout: the fc around it applies the mask

    def forward(self, is_train, nodes_in, nodes_out):
        if is_train and self.threshold > 0 and not self.fused_into_producer:
            x = nodes_in[0].data
            ops.dropout_apply(x, x, self.seed, 1.0 - self.threshold, self.ctx.step_counter)

    def backprop(self, prop_grad, nodes_in, nodes_out):
        if self.threshold > 0 and not self.fused_into_producer:
            x = nodes_in[0].data
            ops.dropout_apply(x, x, self.seed, 1.0 - self.threshold, self.ctx.step_counter)


# ============================================================================ flatten
class FlattenLayer(Layer):
    """`flatten` -- reference src/layer/flatten_layer-inl.hpp:11-40: (B,C,H,W) -> (B,1,1,CHW)
    in NCHW feature order (so fullc weights keep the reference meaning)."""
    replay_audited = True  # library kernels only (tests/test_launch_hygiene_gpu.py)
    type_name = "flatten"

    def init_connection(self, nodes_in, nodes_out):
        _check(len(nodes_in) == 1 and len(nodes_out) == 1, "FlattenLayer: only support 1-1 connection")
        b, c, h, w = nodes_in[0].shape
        _check(nodes_in[0].cp == c, "FlattenLayer: padded-channel input is not supported")
        nodes_out[0].set_shape(b, 1, 1, c * h * w)
        self.dims = (c, h * w)

    def forward(self, is_train, nodes_in, nodes_out):
        x, y = nodes_in[0].data, nodes_out[0].data
        c, hw = self.dims
        if hw == 1 or c == 1:
            ops.copy_(y.view(-1), x.view(-1))
        else:
            ops.transpose(x, y, x.shape[0], hw, c)

    def backprop(self, prop_grad, nodes_in, nodes_out):
        if not prop_grad:
            return
        x, y = nodes_in[0].data, nodes_out[0].data
        c, hw = self.dims
        if hw == 1 or c == 1:
            ops.copy_(x.view(-1), y.view(-1))
        else:
            ops.transpose(y, x, x.shape[0], c, hw)


# ============================================================================ losses
class LossLayerBase(Layer):
    """reference src/layer/loss/loss_layer_base-inl.hpp:11-133.  Self-loop on a matrix
    node; gradient (pred - target) scaled by grad_scale / (batch_size * update_period)
    with the GLOBAL batch size.  Computed on device (no host round trip)."""
    replay_audited = True  # library kernels only (tests/test_launch_hygiene_gpu.py)
    kind = "softmax"

    def __init__(self, ctx):
        super().__init__(ctx)
        self.target = "label"
        self.grad_scale = 1.0
        self.batch_size = 0
        self.update_period = 1
        self.p32 = None

    def set_param(self, name, val):
        super().set_param(name, val)
        if name == "target":
            self.target = val
        elif name == "grad_scale":
            self.grad_scale = float(val)
        elif name == "batch_size":
            self.batch_size = int(val)
        elif name == "update_period":
            self.update_period = int(val)

    def init_connection(self, nodes_in, nodes_out):
        _check(len(nodes_in) == 1 and len(nodes_out) == 1, "LossLayer: only support 1-1 connection")
        _check(nodes_in[0] is nodes_out[0], "LossLayer is an self-loop Layer")
        _check(nodes_in[0].is_mat(), "LossLayer: input need to be a matrix")
        _check(self.target in self.ctx.label_name_map, f"LossLayer: unknown target={self.target}")

    def _p32(self, node):
        m = node.mat()
        if self.p32 is None or self.p32.shape != m.shape:
            self.p32 = torch.empty(m.shape, dtype=torch.float32, device=m.device)
        node.fp32_view = self.p32
        return self.p32

    def backprop(self, prop_grad, nodes_in, nodes_out):
        label = self.ctx.label_fields[self.target]
        bs = self.batch_size if self.batch_size > 0 else nodes_in[0].batch
        # loss_weight 0: an idle data-parallel rank (trainer.active_ranks) adds zero gradients
        scale = self.grad_scale / (bs * self.update_period) * getattr(self.ctx, "loss_weight", 1.0)
        node = nodes_in[0].mat()
        ops.loss_grad(self.kind, node, label[: node.shape[0]], scale, self.p32)


class SoftmaxLayer(LossLayerBase):
    """`softmax` -- reference src/layer/loss/softmax_layer-inl.hpp:12-33."""
    type_name = "softmax"
    kind = "softmax"

    def forward(self, is_train, nodes_in, nodes_out):
        m = nodes_in[0].mat()
        ops.softmax_forward(m, m, self._p32(nodes_in[0]))


class L2LossLayer(LossLayerBase):
    """`l2_loss` -- reference src/layer/loss/l2_loss_layer-inl.hpp (fwd identity, grad x - y)."""
    type_name = "l2_loss"
    kind = "l2"

    def replay_safe(self) -> bool:
        return False  # fp32 copy of the scores through torch

    def forward(self, is_train, nodes_in, nodes_out):
        m = nodes_in[0].mat()
        self._p32(nodes_in[0]).copy_(m)


class MultiLogisticLayer(LossLayerBase):
    """`multi_logistic` -- reference src/layer/loss/multi_logistic_layer-inl.hpp (fwd sigmoid, grad s - y)."""
    type_name = "multi_logistic"
    kind = "multi_logistic"

    def replay_safe(self) -> bool:
        return False  # fp32 copy of the scores through torch

    def forward(self, is_train, nodes_in, nodes_out):
        m = nodes_in[0].mat()
        ops.act_forward("sigmoid", m, m)
        self._p32(nodes_in[0]).copy_(m)
