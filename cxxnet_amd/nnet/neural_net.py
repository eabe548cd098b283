"""Per-device executor: nodes, connections, parameter arena, forward/backprop.

Behavioural parity with reference src/nnet/neural_net-inl.hpp:22-297 (NeuralNet):
  * layers are created from NetConfig in conf order; `share[tag]` reuses the primary
    layer object (weight tying);
  * every layer receives the global config (defcfg) then its own layercfg;
  * Forward copies the batch into node 0, runs layers in order; Backprop runs them in
    reverse, with prop_grad=False for layer 0 unless prop_to_input.
MI355X-first differences:
  * one stream, no per-layer host sync (the reference waits after every parameterised
    layer's backprop, :148): gradients stay on device, comm is event/stream ordered;
  * parameters live in a flat arena updated by one fused kernel (nnet/arena.py);
  * graph-level fusion on the GPU: conv/fullc -> relu pairs become a relu epilogue with
    the relu output node aliasing its input (the reference's in-place activation), and
    relu' is applied by the layer that writes that node's gradient (GEMM data-grad
    epilogue or pooling backward) -- no separate activation kernels.
"""
from __future__ import annotations

import os
from typing import Dict, List, Optional, Sequence

import torch

from .. import native, ops
from ..layers import K_SHARED, LayerContext, Node, create_layer
from ..layers.base import BinReader, BinWriter
from ..updater import ArenaUpdater
from .arena import ParamArena
from ..ops.mode import frozen
from ..io.data import U8Images
from ..io.jpeg_stage import JpegCoefImages

K_CONV, K_FULLC, K_RELU, K_MAXPOOL, K_DROPOUT = 10, 1, 3, 11, 8
K_SPLIT, K_CONCAT, K_CHCONCAT, K_SUMPOOL, K_AVGPOOL, K_LRN = 23, 18, 28, 12, 13, 15
K_RELU_MAXPOOL = 21
# queued bias-gradient bytes (dy read by the column sums) that trigger a side-stream launch
_BIAS_FLUSH_BYTES = int(float(os.environ.get("CXXNET_BIAS_FLUSH_MB", "16")) * (1 << 20))
# layers that only READ their input node in forward and write the input gradient through
# Node.gdst: they may consume a zero-copy split output
_SPLIT_SAFE = (K_CONV, K_FULLC, K_MAXPOOL, K_SUMPOOL, K_AVGPOOL, K_LRN)


class Connection:
    def __init__(self, layer, type_id, nodes_in, nodes_out, shared=False):
        self.layer = layer
        self.type = type_id
        self.nodes_in = nodes_in
        self.nodes_out = nodes_out
        self.shared = shared
        self.owner = None  # index of the connection that owns the parameters


class NeuralNet:
    def __init__(self, cfg, batch_size: int, device="cpu", seed: int = 0, fuse: Optional[bool] = None):
        self.cfg = cfg
        self.max_batch = int(batch_size)
        self.device = torch.device(device)
        self.trace_layers = 0
        self.ctx = LayerContext(self.device, seed)
        self.ctx.label_name_map = dict(cfg.label_name_map)
        self.ctx.step_counter = torch.zeros(1, dtype=torch.int32, device=self.device)
        if fuse is None:
            # CXXNET_FUSE=0: no graph fusion; 2: fusion on the CPU executor too (the fp32 torch
            # path implements every fused epilogue, so CPU tests can check the fused graph)
            mode = os.environ.get("CXXNET_FUSE", "1")
            fuse = mode == "2" or (self.ctx.is_gpu and mode != "0")
        self.fuse = fuse
        self.nodes: List[Node] = []
        self.connections: List[Connection] = []
        self.arena: Optional[ParamArena] = None
        self.updater: Optional[ArenaUpdater] = None
        self.cur_batch = self.max_batch
        self.epoch_counter = 0

    # ------------------------------------------------------------------ construction
    def _configure_layer(self, i, layer):
        for k, v in self.cfg.defcfg:
            layer.set_param(k, v)
        for k, v in self.cfg.layercfg[i]:
            layer.set_param(k, v)

    def init_net(self):
        cfg = self.cfg
        self.nodes = [Node(n) for n in cfg.node_names]
        c, h, w = cfg.input_shape
        self.nodes[0].set_shape(self.max_batch, c, h, w)
        for i in range(cfg.extra_data_num):
            es = cfg.extra_shape[3 * i:3 * i + 3]
            self.nodes[i + 1].set_shape(self.max_batch, *es)
        self.connections = []
        for i, info in enumerate(cfg.layers):
            nin = [self.nodes[j] for j in info.nindex_in]
            nout = [self.nodes[j] for j in info.nindex_out]
            if info.type == K_SHARED:
                prim = self.connections[info.primary_layer_index]
                if not prim.layer.allow_sharing:
                    raise ValueError("some layer you set shared do not allow sharing")
                self.connections.append(Connection(prim.layer, prim.type, nin, nout, shared=True))
                self.connections[-1].owner = prim.owner
            else:
                layer = create_layer(info.type, self.ctx)
                layer.layer_index = i
                self.connections.append(Connection(layer, info.type, nin, nout))
                self.connections[-1].owner = i
        for i, c_ in enumerate(self.connections):
            if not c_.shared:
                self._configure_layer(i, c_.layer)
        self._pad_input_channels()

    def _pad_input_channels(self):
        """First-layer conv on the GPU: pad input channels to a multiple of 4 so the
        implicit-GEMM gather can use 8-byte vector loads (weights get zero columns).

        Exception, the 3-channel strided pad-0 conv that is the input's only reader (AlexNet
        conv1, 11x11 / 4): its GEMMs read whole kernel-row runs (ops.gemm.rowrun_ok), and with
        3 channels a run is 33 elements -- 5 16-byte chunks, K = 11 x 40 = 440 -- against 44
        (6 chunks, K = 528) with a zero 4th channel.  The node then keeps 3 channels and pads
        each image row to a multiple of 4 pixels instead, so that every row and every 4-pixel
        output step starts 8-byte aligned (forward 165 -> 120 us at batch 256,
        profiles/r3_conv1_c3_probe.jsonl).  CXXNET_CONV1_C3=0 keeps the 4-channel layout."""
        if not self.ctx.is_gpu:
            return
        n0 = self.nodes[0]
        b, c, h, w = n0.shape
        readers = [conn for conn in self.connections if any(n is n0 for n in conn.nodes_in)]
        for conn in readers:
            if conn.type == K_CONV and conn.nodes_in[0] is n0 and c % 8 != 0:
                lp = conn.layer.lp
                wp = (w + 3) // 4 * 4
                if (c == 3 and len(readers) == 1 and lp.num_group == 1 and lp.pad_y == 0 and lp.pad_x == 0
                        and (lp.stride * c * 2) % 8 == 0 and lp.kernel_width <= w
                        and (wp - lp.kernel_width) // lp.stride == (w - lp.kernel_width) // lp.stride
                        and os.environ.get("CXXNET_CONV1_C3", "1") != "0" and not ops.gemm.deterministic()):
                    n0.cp, n0.wp = 3, wp
                    return
                n0.cp = (c + 3) // 4 * 4
                return

    def _connect(self):
        """Shape inference (InitConnection) in conf order."""
        for conn in self.connections:
            conn.layer.init_connection(conn.nodes_in, conn.nodes_out)

    def _fuse(self):
        if not self.fuse:
            self._mark_nonneg()
            return
        producers: Dict[int, list] = {}
        consumers: Dict[int, list] = {}
        for i, conn in enumerate(self.connections):
            self_loop = len(conn.nodes_in) == 1 and conn.nodes_out == conn.nodes_in
            for n in conn.nodes_out:
                if not self_loop:
                    producers.setdefault(id(n), []).append(i)
            for n in conn.nodes_in:
                consumers.setdefault(id(n), []).append((i, self_loop))
        self.aliases = {}
        for i, conn in enumerate(self.connections):
            if conn.type != K_RELU or conn.shared or conn.nodes_in[0] is conn.nodes_out[0]:
                continue
            a, b = conn.nodes_in[0], conn.nodes_out[0]
            prod = producers.get(id(a), [])
            if len(prod) != 1:
                continue
            p = self.connections[prod[0]]
            if p.type not in (K_CONV, K_FULLC) or p.shared:
                continue
            if len(consumers.get(id(a), [])) != 1:  # only the relu reads a
                continue
            cons = consumers.get(id(b), [])
            real = [(j, sl) for j, sl in cons if not sl]
            loops = [j for j, sl in cons if sl]
            if len(real) != 1 or any(self.connections[j].type != K_DROPOUT for j in loops):
                continue
            j = real[0][0]
            cj = self.connections[j]
            if j == 0 or cj.shared:
                continue
            if cj.type in (K_CONCAT, K_CHCONCAT):
                # concat backward copies the gradient slice back into b masked by relu'(z)
                p.layer.fuse_relu = True
                conn.layer.fused_into_producer = True
                cj.layer.grad_mask_inputs.add(cj.nodes_in.index(b))
                self.aliases[id(b)] = a
                continue
            if cj.type not in (K_CONV, K_FULLC, K_MAXPOOL, K_LRN) or len(cj.nodes_in) != 1:
                continue
            # commit: producer epilogue applies relu, b aliases a, consumer masks the gradient
            p.layer.fuse_relu = True
            conn.layer.fused_into_producer = True
            cj.layer.grad_mask_relu = True
            self.aliases[id(b)] = a
            self._fuse_dropout(p, [self.connections[k] for k in loops], cj)

        self._fuse_concat(producers, consumers)
        self._fuse_split(producers, consumers)
        self._fuse_siblings(producers, consumers)
        self._fuse_pool_bias(producers, consumers)
        self._fuse_dgrad_bias(producers, consumers)
        self._fuse_pool_lrn(producers, consumers)
        self._fuse_lrn_bias(producers, consumers)
        self._mark_nonneg()

    def _mark_nonneg(self):
        """Nodes that can only hold values >= 0 (relu outputs -- fused into their producer or
        not -- and what max-pool / LRN / dropout / split / concat make of them); a max-pool
        reading one gets input_nonneg, and its kernels then take the window maximum on integer
        keys of the bf16 bits (ops.pool_forward(nonneg=True))."""
        nn = set()
        for conn in self.connections:
            lay, t = conn.layer, conn.type
            ins = conn.nodes_in
            if t == K_RELU or (t in (K_CONV, K_FULLC) and getattr(lay, "fuse_relu", False)):
                ok = True
            elif t in (K_MAXPOOL, K_RELU_MAXPOOL):
                ok = t == K_RELU_MAXPOOL or bool(getattr(lay, "relu", False)) or all(id(n) in nn for n in ins)
                lay.input_nonneg = all(id(n) in nn for n in ins)
            elif t in (K_LRN, K_DROPOUT, K_SPLIT, K_CHCONCAT, K_CONCAT):
                ok = all(id(n) in nn for n in ins)
            else:
                ok = False
            for n in conn.nodes_out:
                if ok:
                    nn.add(id(n))
                else:  # a later writer (an in-place batch_norm / prelu / bias on a relu output) can make it negative
                    nn.discard(id(n))
        for b, a in getattr(self, "aliases", {}).items():  # b = fused relu(a): a holds relu(z) too
            if b in nn:
                nn.add(id(a))

    def _fuse_pool_lrn(self, producers, consumers):
        """Max-pool (3x3 / 2, pad 0) -> LRN (AlexNet pool1 -> lrn1, pool2 -> lrn2): one kernel per
        direction (ops.pool_lrn_forward / ops.lrn_pool_backward).  The pool's forward also writes
        the LRN output, and its backward takes the LRN's output gradient straight to the pool's
        input gradient (the LRN layer launches nothing): the pooled output is not re-read in
        forward and the pooled gradient never goes to memory.  The pool's output must be read by
        the LRN alone.  CXXNET_FUSE_POOL_LRN=0 keeps the two layers apart."""
        if os.environ.get("CXXNET_FUSE_POOL_LRN", "1") == "0" or not self.ctx.is_gpu:
            return
        for conn in self.connections:
            lay = conn.layer
            if conn.type not in (K_MAXPOOL, K_RELU_MAXPOOL) or conn.shared or len(conn.nodes_in) != 1:
                continue
            lp = lay.lp
            if (getattr(lay, "mode", None) != "max" or lay.tie_all or lp.kernel_height != 3 or lp.kernel_width != 3
                    or lp.stride != 2 or lp.pad_y != 0 or lp.pad_x != 0):
                continue
            out = conn.nodes_out[0]
            cons = consumers.get(id(out), [])
            if len(cons) != 1 or cons[0][1]:
                continue
            cj = self.connections[cons[0][0]]
            if cj.type != K_LRN or cj.shared or cj.nodes_in[0] is not out or cj.layer.grad_mask_relu:
                continue
            if out.cp % 8 or cj.layer.nsize // 2 > 4:
                continue
            lay.fused_lrn = (cj.layer, cj.nodes_out[0])
            cj.layer.fused_with_pool = True

    def _fuse_dropout(self, p, loops, cj):
        """fc -> relu -> dropout -> fc (AlexNet fc6 / fc7): the producer's forward applies the
        dropout mask on the way out (the split-K finalize, ops.fc_forward(drop=...)) and the
        consumer's data-gradient scales by 1 / pkeep: the stored activation is relu(z) * mask /
        pkeep, so the relu'-mask the consumer already applies (old value > 0) is exactly the
        dropout mask as well -- the dropout layer launches nothing in either direction.
        CXXNET_FUSE_DROPOUT=0 keeps the separate dropout kernels."""
        if os.environ.get("CXXNET_FUSE_DROPOUT", "1") == "0" or len(loops) != 1:
            return
        d = loops[0]
        if p.type != K_FULLC or cj.type != K_FULLC or d.shared or not 0.0 < d.layer.threshold < 1.0:
            return
        p.layer.fuse_dropout = d.layer
        cj.layer.grad_alpha = 1.0 / (1.0 - d.layer.threshold)
        d.layer.fused_into_producer = True

    def _fuse_dgrad_bias(self, producers, consumers):
        """Bias gradient of a conv whose output (through a fused relu) is read by one other conv
        alone: that conv's data-gradient GEMM writes exactly this gradient, and its epilogue sums
        it per channel on the way out (ops.conv_backward_data(dbias=...)), so the gradient is not
        re-read by the column-sum pass.  The epilogue sums, the per-wave partial rows and one
        reduce launch per fused conv cost about what the saved read does on small layers (every
        layer fused: AlexNet +2 %, VGG-16 +1.4 %, GoogLeNet +17 %,
        profiles/r6_ab_dgrad_bias_negative.jsonl), so by default ("auto") only layers whose
        gradient is at least CXXNET_DGRAD_BIAS_MIN_MB (150) MB are fused: VGG-16's conv1_1 and
        conv2_1 at batch 64, -0.5 % (profiles/r6_ab_dgrad_bias_min_mb.jsonl).  CXXNET_DGRAD_BIAS=1
        fuses every eligible layer, 0 none."""
        mode = os.environ.get("CXXNET_DGRAD_BIAS", "auto")
        if mode == "0":
            return
        min_mb = float(os.environ.get("CXXNET_DGRAD_BIAS_MIN_MB", "150" if mode == "auto" else "0"))
        for conn in self.connections:
            if conn.type != K_CONV or conn.shared or len(conn.nodes_in) != 1:
                continue
            node = conn.nodes_in[0]
            b, c, h, w = node.shape
            if b * c * h * w * 2 < min_mb * 1e6:
                continue
            src = self.aliases.get(id(node), node)
            prod = producers.get(id(src), [])
            if len(prod) != 1:
                continue
            p = self.connections[prod[0]]
            if p.type != K_CONV or p.shared or p is conn or len(consumers.get(id(src), [])) != 1:
                continue
            if getattr(p.layer, "sib", None) or getattr(p.layer, "sib_member", False):
                continue  # a sibling group sums its biases together (it would count twice)
            if src is not node and len(consumers.get(id(node), [])) != 1:
                continue
            conn.layer.bias_below = p.layer

    def _fuse_lrn_bias(self, producers, consumers):
        """Bias gradient of a conv whose output (through a fused relu) is read by an LRN alone
        (GoogLeNet conv2 -> relu -> norm2): the LRN's input gradient is that conv's output
        gradient, so the LRN backward sums it per channel as it stores it
        (ops.lrn_backward_bias) instead of the column-sum pass re-reading it.  GPU only, not in
        deterministic mode (the layer checks both).  CXXNET_LRN_BIAS=0 turns it off."""
        if os.environ.get("CXXNET_LRN_BIAS", "1") == "0":
            return
        for conn in self.connections:
            lay = conn.layer
            if conn.type != K_LRN or conn.shared or len(conn.nodes_in) != 1 or getattr(lay, "fused_with_pool", False):
                continue
            node = conn.nodes_in[0]
            src = self.aliases.get(id(node), node)
            prod = producers.get(id(src), [])
            if len(prod) != 1:
                continue
            p = self.connections[prod[0]]
            if p.type != K_CONV or p.shared or len(consumers.get(id(src), [])) != 1:
                continue
            if getattr(p.layer, "sib", None) or getattr(p.layer, "sib_member", False):
                continue  # a sibling group sums its biases together
            if src is not node and len(consumers.get(id(node), [])) != 1:
                continue
            lay.bias_of = p.layer

    def _fuse_pool_bias(self, producers, consumers):
        """Bias gradient of a conv that feeds a max-pool, taken from the pool's OUTPUT gradient:
        each window routes its gradient to one input pixel, relu' of that pixel is recorded in
        the window's offset byte, so the pool sums dy_pool (masked) instead of the conv summing
        its own stride^2-times larger dy (ops.bias_grad mask).  The conv's output (or the fused
        relu's alias of it) must be read by the pool alone.  CXXNET_POOL_BIAS=0 turns it off."""
        if os.environ.get("CXXNET_POOL_BIAS", "1") == "0":
            return
        for conn in self.connections:
            lay = conn.layer
            if conn.type not in (K_MAXPOOL, K_RELU_MAXPOOL) or conn.shared or len(conn.nodes_in) != 1:
                continue
            if getattr(lay, "mode", None) != "max":
                continue
            node = conn.nodes_in[0]
            src = self.aliases.get(id(node), node)  # a fused relu's output aliases the conv output
            prod = producers.get(id(src), [])
            if len(prod) != 1:
                continue
            p = self.connections[prod[0]]
            if p.type != K_CONV or p.shared or len(consumers.get(id(src), [])) != 1:
                continue
            if getattr(p.layer, "sib", None) or getattr(p.layer, "sib_member", False):
                continue  # a sibling group sums its biases together
            if src is not node and len(consumers.get(id(node), [])) != 1:
                continue
            lay.bias_of = p.layer

    def _fuse_concat(self, producers, consumers):
        """Zero-copy ch_concat (reference src/layer/concat_layer-inl.hpp:38-76 copies): when
        every input is the fused relu output of its own conv, read by the concat alone, each
        conv writes relu(z) straight into its channel slice of the concat output (the GEMM
        epilogue's row stride is the full channel count) and reads its output gradient from
        that slice in backward -- the concat moves no bytes either way.
        relu' of the slices is applied by the layer that writes the concat output's gradient
        (its single consumer: split, or a pooling layer, gets grad_mask_relu), since every
        channel of the output is a relu output and still holds it at that point.
        CXXNET_CONCAT_ZC=0 keeps the copying concat."""
        self.concat_views = {}
        if os.environ.get("CXXNET_CONCAT_ZC", "1") == "0":
            return
        for i, conn in enumerate(self.connections):
            if conn.type != K_CHCONCAT or conn.shared or conn.layer.dim != 1:
                continue
            out = conn.nodes_out[0]
            cons = consumers.get(id(out), [])
            if len(cons) != 1 or cons[0][1]:
                continue
            cj = self.connections[cons[0][0]]
            if cj.shared or len(cj.nodes_in) != 1 or cj.type not in (K_SPLIT, K_MAXPOOL, K_AVGPOOL, K_SUMPOOL):
                continue
            if cj.type != K_SPLIT and getattr(cj.layer, "tie_all", False):
                continue
            views, off, ok = {}, 0, True
            for b in conn.nodes_in:
                a = self.aliases.get(id(b))  # b = fused relu(a)
                prod = producers.get(id(a), []) if a is not None else []
                c = b.shape[1]
                if (a is None or len(prod) != 1 or len(consumers.get(id(b), [])) != 1 or id(a) in views
                        or c % 8 or off % 8 or a.cp != c):
                    ok = False
                    break
                p = self.connections[prod[0]]
                if p.type != K_CONV or p.shared or not p.layer.fuse_relu:
                    ok = False
                    break
                views[id(a)] = (a, out, off, c)
                off += c
            if not ok or off != out.shape[1] or out.cp != off:
                continue
            conn.layer.zero_copy = True
            conn.layer.grad_mask_inputs.clear()
            cj.layer.grad_mask_relu = True
            self.concat_views.update(views)

    def _fuse_split(self, producers, consumers):
        """Zero-copy split: when the split is its input's only reader and every output feeds
        exactly one read-only-in-forward layer, the outputs alias the input buffer and each
        consumer's data-gradient goes to the output node's private grad buffer (summed by the
        split's backward).  Saves one full activation copy per branch per step."""
        self.split_alias = {}
        for i, conn in enumerate(self.connections):
            if conn.type != K_SPLIT or conn.shared or len(conn.nodes_in) != 1:
                continue
            a = conn.nodes_in[0]
            if len(consumers.get(id(a), [])) != 1:
                continue
            ok = True
            for o in conn.nodes_out:
                cons = consumers.get(id(o), [])
                if o is a or len(producers.get(id(o), [])) != 1 or len(cons) != 1 or cons[0][1]:
                    ok = False
                    break
                j = cons[0][0]
                cj = self.connections[j]
                if j == 0 or cj.type not in _SPLIT_SAFE or len(cj.nodes_in) != 1 or cj.layer.grad_mask_relu:
                    ok = False
                    break
            if not ok:
                continue
            conn.layer.alias = True
            for o in conn.nodes_out:
                self.split_alias[id(o)] = a

    def _fuse_siblings(self, producers, consumers):
        """Sibling 1x1 convs (an inception module's 1x1, 3x3_reduce and 5x5_reduce: same input
        through a zero-copy split, 1x1 / stride 1 / pad 0, relu fused) as ONE GEMM per
        direction.  Their outputs become channel slices of one buffer H [pixels][C1 + C2 + ...]:
        the first sibling (the lead) computes all of them in one forward GEMM, the consumers of
        the slices read them in place (strided NHWC) and write their input gradients back into
        them, so H's gradient is contiguous and one weight-gradient and one data-gradient GEMM
        over all of H replace one per sibling.  A sibling whose output was a zero-copy concat
        slice (the 1x1) moves into H; the concat copies that slice in (forward) and its gradient
        back (backward, relu'-masked) -- two small copies instead of two GEMMs.  The arena lays
        each group's weights out as one matrix and its biases as one vector (ParamArena.build
        groups); checkpoints stay per layer.  The split sums one gradient per group instead of
        one per sibling.  Reference: src/layer/split_layer-inl.hpp:29-41,
        src/layer/convolution_layer-inl.hpp:70-106.  CXXNET_FUSE_SIBLINGS=0 turns it off."""
        self.sib_groups = []
        self.sib_views = {}
        if (os.environ.get("CXXNET_FUSE_SIBLINGS", "1") == "0" or not self.ctx.is_gpu
                or os.environ.get("CXXNET_DGRAD_BIAS", "0") == "1"):
            return
        views = getattr(self, "concat_views", {})
        for conn in self.connections:
            if conn.type != K_SPLIT or conn.shared or not getattr(conn.layer, "alias", False):
                continue
            x = conn.nodes_in[0]
            if x.cp % 8:
                continue
            mem = []
            for o in conn.nodes_out:
                cons = consumers.get(id(o), [])
                if len(cons) != 1 or cons[0][1]:
                    continue
                j = cons[0][0]
                cj = self.connections[j]
                lay = cj.layer
                if cj.type != K_CONV or cj.shared or not getattr(lay, "fuse_relu", False):
                    continue
                lp = lay.lp
                if (lp.kernel_height != 1 or lp.kernel_width != 1 or lp.stride != 1 or lp.pad_y or lp.pad_x
                        or lp.num_group != 1 or lp.num_channel % 8 or getattr(lay, "_prepad_on", False)):
                    continue
                a = cj.nodes_out[0]
                if id(a) in views:  # a zero-copy concat slice: movable if it is a ch_concat input
                    cc = self._concat_of(a, consumers)
                    if cc is None:
                        continue
                else:  # read in place as a strided NHWC slice of H: only convolutions can
                    rd = consumers.get(id(self._alias_of(a)), [])
                    if not rd or any(sl or self.connections[k].type != K_CONV for k, sl in rd):
                        continue
                mem.append((j, o))
            mem.sort(key=lambda t: t[0])
            if len(mem) < 2 or len({self.connections[j].layer.lp.no_bias for j, _ in mem}) != 1:
                continue
            gi = len(self.sib_groups)
            group = [j for j, _ in mem]
            self.sib_groups.append(group)
            off = 0
            for j, _ in mem:
                a = self.connections[j].nodes_out[0]
                if id(a) in views:  # the concat copies this slice from H instead
                    _, out, coff, c = views.pop(id(a))
                    cc = self._concat_of(a, consumers)
                    cc.layer.copy_from_h.append((gi, off, coff, a.cp))
                self.sib_views[id(a)] = (a, gi, off, a.cp)
                off += a.cp
            for j, _ in mem[1:]:
                self.connections[j].layer.sib_member = True
            lead = self.connections[group[0]].layer
            lead.sib = {"gi": gi, "layers": [self.connections[j].layer for j in group], "ctot": off,
                        "dx_node": mem[0][1]}
            # the data-gradient of every sibling lands in the lead's slot of the split
            conn.layer.skip_grads = {id(o) for _, o in mem[1:]}
            # one other split output (the pool branch) whose backward runs before the lead's: the
            # lead's data-gradient GEMM adds its gradient and writes the split's input gradient
            # (relu'-masked as the split would), and the split's sum is skipped
            others = [o for o in conn.nodes_out if id(o) not in {id(m) for _, m in mem}]
            if (len(others) == 1 and os.environ.get("CXXNET_FOLD_SPLIT_SUM", "1") != "0"
                    and all(j > group[0] for j, _ in consumers.get(id(others[0]), []))):
                lead.sib["fold"] = {"split": conn.layer, "dst": conn.nodes_in[0], "add": others[0]}

    def _alias_of(self, a):
        """The node that reads a fused-relu conv output a: relu(a)'s alias node, or a itself."""
        b = next((bb for bb, src in self.aliases.items() if src is a), None)  # b = relu(a) alias key
        return a if b is None else next((n for n in self.nodes if id(n) == b), a)

    def _concat_of(self, a, consumers):
        """The zero-copy ch_concat connection that a fused-relu conv output a feeds, or None."""
        node = self._alias_of(a)
        for j, _ in consumers.get(id(node), []):
            cj = self.connections[j]
            if cj.type == K_CHCONCAT and getattr(cj.layer, "zero_copy", False):
                return cj
        return None

    def _sibling_views(self):
        """Arena views of each sibling group (after _build_arena): the stacked weights (compute
        copy and gradient) and biases."""
        a = self.arena
        wb = a.wb if a.wb is not None else a.w
        for conn in self.connections:
            S = getattr(conn.layer, "sib", None)
            if not S:
                continue
            lays = S["layers"]
            cin = lays[0].geo.C
            ctot = S["ctot"]
            w0 = lays[0].w.offset
            S["w_all"] = wb[w0:w0 + ctot * cin].view(ctot, 1, 1, cin)
            S["w_g"] = a.g[w0:w0 + ctot * cin].view(ctot, 1, 1, cin)
            S["wt"] = torch.empty_like(S["w_all"])
            if lays[0].b is not None:
                b0 = lays[0].b.offset
                S["b_all"] = a.w[b0:b0 + ctot]
                S["b_g"] = a.g[b0:b0 + ctot]
            else:
                S["b_all"] = S["b_g"] = None

    def _alloc_nodes(self):
        dt = self.ctx.act_dtype
        aliases = dict(getattr(self, "aliases", {}))
        splits = getattr(self, "split_alias", {})
        aliases.update(splits)
        views = getattr(self, "concat_views", {})
        sibs = getattr(self, "sib_views", {})
        for n in self.nodes:
            if id(n) not in aliases and id(n) not in views and id(n) not in sibs:
                n.alloc(self.device, dt)
        for a, out, off, c in views.values():  # conv outputs that are channel slices of a concat
            a.data = out.data[..., off:off + c]
        # sibling conv outputs: channel slices of their group's buffer H (NeuralNet._fuse_siblings)
        hbuf = {}
        for a, gi, off, c in sibs.values():
            if gi not in hbuf:
                cbc = sum(cc for _, g2, _, cc in sibs.values() if g2 == gi)
                b, _, h, w = a.shape
                hbuf[gi] = torch.zeros((b, h, w, cbc), device=self.device, dtype=dt)
            a.data = hbuf[gi][..., off:off + c]
        for conn in self.connections:
            S = getattr(conn.layer, "sib", None)
            if S:
                S["H"] = hbuf[S["gi"]]
            if getattr(conn.layer, "copy_from_h", None):
                conn.layer.h_copies = [(hbuf[gi], hoff, coff, c) for gi, hoff, coff, c in conn.layer.copy_from_h]
        pending = [n for n in self.nodes if id(n) in aliases]
        for _ in range(len(pending) + 1):  # resolve chains (split of a relu alias, ...)
            left = []
            for n in pending:
                src = aliases[id(n)]
                if src.data is None:
                    left.append(n)
                else:
                    n.data = src.data
            pending = left
            if not pending:
                break
        assert not pending, "unresolved node aliases"
        for n in self.nodes:
            if id(n) in splits:
                n.grad_buf = torch.zeros_like(n.data)

    def _build_arena(self):
        # a shared layer's backprop runs once per use: its gradients must accumulate, so
        # they are zeroed at the start of an update cycle instead of overwritten
        for conn in self.connections:
            if conn.shared:
                for spec in conn.layer.params:
                    spec.overwrite = False
        specs = []
        for i, conn in enumerate(self.connections):
            if not conn.shared:
                specs.append((i, conn.layer.declare_params()))
        self.arena = ParamArena(self.device, torch.bfloat16 if self.ctx.is_gpu else None)
        self.arena.build(specs, groups=getattr(self, "sib_groups", ()))
        self._sibling_views()

    def _init_updater(self):
        self.updater = ArenaUpdater(self.cfg.updater_type, self.arena, self.arena.segments(), self.cfg.defcfg,
                                    self.cfg.layercfg)

    def init_model(self):
        """Fresh model: build, connect, random-init every parameter (reference InitModel)."""
        self.init_net()
        self._connect()
        self._fuse()
        self._alloc_nodes()
        self._build_arena()
        # drawn in reverse layer order, each layer's tensors in declaration order -- not in arena
        # order, which sibling groups (ParamArena.build groups) rearrange: a seed gives the same
        # initial weights with and without the groups
        for i in range(len(self.connections) - 1, -1, -1):
            conn = self.connections[i]
            if conn.shared:
                continue
            for spec in conn.layer.params:
                # drawn where the arena lives (device RNG kernel on the GPU), in logical layout
                t = torch.zeros(spec.shape, dtype=torch.float32, device=self.device)
                spec.init(t)
                spec.w.copy_(t)
        self.arena.sync_shadow()
        self._init_updater()

    def load_model(self, fi: BinReader):
        """Reference LoadModel: per-layer blob in layer order, shared layers skipped."""
        self.init_net()
        for conn in self.connections:
            if not conn.shared:
                conn.layer.load_model(fi)
        self._connect()
        self._fuse()
        self._alloc_nodes()
        self._build_arena()
        for conn in self.connections:
            if conn.shared or not hasattr(conn.layer, "loaded_values"):
                continue
            vals = conn.layer.loaded_values()
            for spec, v in zip(conn.layer.params, vals):
                spec.w.copy_(v.reshape(spec.shape))
        self.arena.sync_shadow()
        self._init_updater()

    def save_model(self, fo: BinWriter):
        for conn in self.connections:
            if not conn.shared:
                conn.layer.save_model(fo)

    # ------------------------------------------------------------------ execution
    def adjust_batch_size(self, b: int):
        if b > self.max_batch:
            raise ValueError("cannot set batch size larger than max batch")
        if b == self.cur_batch:
            return
        self.cur_batch = b
        # layers may now reallocate shape-dependent buffers: recorded launch lists and captured
        # graphs of every batch size are stale (NetTrainer._drop_stale_plans)
        self.batch_gen = getattr(self, "batch_gen", 0) + 1
        for conn in self.connections:
            conn.layer.on_batch_size_changed(conn.nodes_in, conn.nodes_out)

    def node_view(self, n: Node) -> torch.Tensor:
        return n.data[: self.cur_batch]

    def set_input(self, data: torch.Tensor, extra: Sequence[torch.Tensor] = ()):
        """data: (b, c, h, w) float tensor (any device)."""
        b = data.shape[0]
        self.adjust_batch_size(b)
        n0 = self.nodes[0]
        if isinstance(data, (U8Images, JpegCoefImages)):
            ops.image_to_nhwc(data, n0.data[:b])
        else:
            src = data.to(self.device, non_blocking=True)
            ops.input_to_nhwc(src, n0.data[:b])
        for i, e in enumerate(extra):
            ops.input_to_nhwc(e.to(self.device, non_blocking=True), self.nodes[i + 1].data[:b])

    def set_labels(self, labels: torch.Tensor):
        """labels: (b, label_width) float; split into named fields by label_vec ranges."""
        lab = labels.to(self.device, torch.float32, non_blocking=True)
        if lab.dim() == 1:
            lab = lab.view(-1, 1)
        # staged in one persistent buffer: loss layers (and captured HIP graphs) read the
        # labels from a fixed address
        buf = getattr(self, "_label_buf", None)
        if buf is None or buf.shape[0] < lab.shape[0] or buf.shape[1] != lab.shape[1]:
            buf = self._label_buf = torch.empty((max(self.max_batch, lab.shape[0]), lab.shape[1]),
                                                dtype=torch.float32, device=self.device)
        buf[: lab.shape[0]].copy_(lab, non_blocking=True)
        lab = buf[: lab.shape[0]]
        fields = {}
        for name, idx in self.cfg.label_name_map.items():
            a, b = self.cfg.label_range[idx]
            fields[name] = lab[:, a:b]
        self.ctx.label_fields = fields

    def _range(self, i: int, phase: str):
        """roctx range per layer (trace_layers = 1): rocprofv3 --marker-trace shows which
        layer each kernel belongs to."""
        if not self.trace_layers or self.device.type != "cuda":
            return _NoRange
        conn = self.connections[i]
        return _LayerRange(f"{phase}:{i}:{conn.layer.type_name}")

    def forward(self, is_train: bool, pre_hook=None):
        """pre_hook(layer_index) runs before each layer: the data-parallel reducer uses it
        to make the compute stream wait for the bucket holding that layer's weights (the
        reference's per-layer UpdateWait, neural_net-inl.hpp:125-131) and nothing more."""
        if self.ctx.is_gpu:  # a library launch: HIP graphs and recorded launch lists replay it
            native.check(native.kernels().cxn_add_i32(self.ctx.step_counter.data_ptr(), 1, ops.gemm._stream()),
                         "add_i32")
        else:
            self.ctx.step_counter.add_(1)
        with _BatchView(self):
            for i, conn in enumerate(self.connections):
                if pre_hook is not None:
                    pre_hook(conn.owner)
                with self._range(i, "fwd"):
                    conn.layer.forward(is_train, conn.nodes_in, conn.nodes_out)

    def backprop(self, prop_to_input: bool = False, hook=None, first: bool = False, hook_due=None):
        """Reverse pass.  hook(layer_index) runs after each layer's backprop (used by the
        data-parallel bucketer to launch reductions as soon as gradients are final).

        first=True marks the first micro-batch of an update cycle: accumulated gradients
        are zeroed here and overwrite-capable ones (fullc weights) are stored instead of
        accumulated -- replacing the reference's `dw = 0` after every update with less
        memory traffic."""
        self.ctx.grad_overwrite = bool(first)
        if first:
            self.arena.zero_accumulated_grads()
        # the bias gradients are queued and summed in one multi-tensor launch: at the end of the
        # pass, or -- with a data-parallel bucket hook -- right before the hook that launches a
        # bucket (hook_due(i): the hook would launch one after layer i), since a bucket needs every
        # gradient of its layers.  The dy buffers they read are not rewritten later in the pass.
        from ..ops.gemm import deterministic
        from ..ops.mode import reference_precision
        # (the fp32 reference mode sums each bias gradient at once, as the CPU path does)
        defer = self.ctx.is_gpu and not deterministic() and not reference_precision()
        self.ctx.deferred_bias = [] if defer else None
        if self.ctx.is_gpu:
            # every conv data-gradient's flipped weights in one launch (weights do not change
            # during the pass: data-parallel bucket updates only start after a layer's backward)
            flips, seen = [], set()
            for i, conn in enumerate(self.connections):
                lay = conn.layer
                if getattr(lay, "sib_member", False):
                    continue
                if hasattr(lay, "flip_target") and (i != 0 or prop_to_input) and id(lay) not in seen:
                    seen.add(id(lay))
                    if getattr(lay, "sib", None) is None:  # (a group lead flips the stacked weights)
                        flips.append(lay.flip_target())
                    flips.extend(lay.extra_flip_targets())
            from ..ops.gemm import conv_weight_flip_multi
            conv_weight_flip_multi(flips)
            self.ctx.flipped = seen
        side = self._bias_stream() if defer and hook is None else None
        # fused fc SGD steps (memory-bound: w / m / shadow streams) on a side stream, overlapping
        # the compute-bound conv backward below them; joined at the end of the pass.  Under data
        # parallelism (a bucket hook) only the fullc_gather layers fuse, from their gathered rows
        # (FullConnectLayer._fused_sgd)
        self.ctx.fc_side = self._fc_side_stream(dp=hook is not None) if self.ctx.is_gpu else None
        self.ctx.fc_side_used = False
        with _BatchView(self):
            for i in range(len(self.connections) - 1, -1, -1):
                conn = self.connections[i]
                with self._range(i, "bwd"):
                    conn.layer.backprop(i != 0 or prop_to_input, conn.nodes_in, conn.nodes_out)
                if hook is not None:
                    if self.ctx.deferred_bias and (hook_due is None or hook_due(i)):
                        self._flush_bias(None)
                    hook(i)
                if side is not None and self._pending_bias_bytes() >= _BIAS_FLUSH_BYTES:
                    self._flush_bias(side)
            if defer:
                if side is not None:
                    self._flush_bias(side)
                    torch.cuda.current_stream().wait_stream(side)
                else:
                    self._flush_bias(None)
            if self.ctx.fc_side_used:
                torch.cuda.current_stream().wait_stream(self.ctx.fc_side)
            self.ctx.fc_side = None
        self.ctx.deferred_bias = None
        self.ctx.flipped = None

    def _bias_stream(self):
        """Side stream for the queued bias-gradient column sums (memory-bound) so that they
        overlap the compute-bound weight / data-gradient GEMMs of the layers below
        (CXXNET_BIAS_SIDE=1); None = all of them in one launch at the end on the main stream,
        the default: interleaved A/B on one MI355X measured AlexNet b256 -0.6 %, GoogLeNet b128
        +2.0 %, VGG-16 b64 +0.5 % ms/step with the side stream (profiles/r2_ab_bias_side.jsonl)
        -- the column sums steal HBM and CU slots from the GEMMs they overlap."""
        if os.environ.get("CXXNET_BIAS_SIDE", "0") != "1" or frozen():
            return None
        if getattr(self, "_side", None) is None:
            self._side = torch.cuda.Stream(device=self.device)
        return self._side

    def _fc_side_stream(self, dp=False):
        """Side stream of the fc weight-gradient GEMMs with the fused SGD step: they stream
        each fc layer's fp32 master, momentum and bf16 shadow (18 B / parameter, AlexNet fc6:
        680 MB) and so are HBM-bound, while the conv backward that follows is MFMA-bound.
        One GPU: off unless CXXNET_FC_SGD_SIDE=1 -- AlexNet b256 2.320 -> 2.375 ms and VGG-16 b64
        9.40 -> 9.41 ms with it in round 3 (profiles/r3_ab_fc_sgd_side.jsonl), 1.801 / 1.806 vs
        1.813 / 1.796 ms in round 6: the concurrent HBM stream slows the GEMMs it overlaps by as
        much as it hides.  Data parallel (the fullc_gather layers' step from the gathered rows,
        8x the GEMM work at world 8): on unless CXXNET_FC_SGD_SIDE=0 -- RCCL forced at world 1,
        AlexNet b256 2.072 -> 2.014-2.024 ms (profiles/r6_dp_world1.md).  Not under HIP-graph
        capture."""
        env = os.environ.get("CXXNET_FC_SGD_SIDE", "")
        if frozen() or env == "0" or (env != "1" and not dp):
            return None
        if getattr(self, "_fc_side", None) is None:
            self._fc_side = torch.cuda.Stream(device=self.device)
        return self._fc_side

    def _pending_bias_bytes(self) -> int:
        q = self.ctx.deferred_bias
        return sum(d.numel() * d.element_size() for d, _, _ in q) if q else 0

    def _flush_bias(self, side):
        """Launch the queued bias gradients (one colsum_multi) -- on `side` after the work
        enqueued so far on the main stream, or on the main stream when side is None.  The dy
        buffers they read are not rewritten later in the pass, and the gradients are read only
        after the main stream waited for `side` at the end of the pass."""
        pending = self.ctx.deferred_bias
        if not pending:
            return
        self.ctx.deferred_bias = []
        from ..ops.nn import bias_fast_ok
        if side is not None:
            # only the workspace-free one-launch kernel leaves the main stream (the fallback
            # kernels share the op workspace with main-stream GEMMs)
            fast = [it for it in pending if bias_fast_ok(it[0], it[2])]
            pending = [it for it in pending if not bias_fast_ok(it[0], it[2])]
            if fast:
                side.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(side):
                    ops.bias_grad_multi(fast)
        if pending:
            ops.bias_grad_multi(pending)

    def update(self, epoch: int, ranges=None):
        self.updater.update(epoch, ranges)

    def start_round(self, r: int):
        if self.updater is not None:
            self.updater.start_round(r)


class _NoRangeT:
    def __enter__(self):
        return self

    def __exit__(self, *exc):
        return False


_NoRange = _NoRangeT()


class _LayerRange:
    def __init__(self, name):
        self.name = name

    def __enter__(self):
        torch.cuda.nvtx.range_push(self.name)  # roctx on ROCm builds
        return self

    def __exit__(self, *exc):
        torch.cuda.nvtx.range_pop()
        return False


class _BatchView:
    """Narrows every node buffer to the current batch for the duration of a pass."""

    def __init__(self, net: NeuralNet):
        self.net = net

    def __enter__(self):
        net = self.net
        if net.cur_batch == net.max_batch:
            self.saved = None
            return
        self.saved = [(n, n.data, n.grad_buf) for n in net.nodes]
        seen = {}
        for n, d, g in self.saved:
            key = (d.data_ptr(), tuple(d.shape), tuple(d.stride()))  # a concat slice may share a base pointer
            if key not in seen:
                seen[key] = d[: net.cur_batch]
            n.data = seen[key]
            if g is not None:
                n.grad_buf = g[: net.cur_batch]

    def __exit__(self, *exc):
        if self.saved is not None:
            for n, d, g in self.saved:
                n.data = d
                n.grad_buf = g
        return False
