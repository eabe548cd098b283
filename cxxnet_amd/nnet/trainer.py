"""Trainer: the INetTrainer API (reference src/nnet/nnet.h:18-100) over one device
per process, data-parallel across processes.

Reference: CXXNetThreadTrainer, src/nnet/nnet_impl-inl.hpp:16-455 -- device list,
batch split step = ceil(batch/ndev), metric[label,node] parsing, Update with
update_period, Predict (argmax or raw), ExtractFeature (name or top[-k]), Evaluate,
Set/GetWeight, CopyModelFrom (finetune copy-by-name), and the model file:
  int32 net_type | NetConfig | int64 epoch_counter | uint64 len + per-layer blob.
"""
from __future__ import annotations

import functools
import os
import struct
from typing import List, Optional, Tuple

import numpy as np
import torch

from .. import native
from ..io.data import DEVICE_IO_LOCK
from ..layers.base import BinReader, BinWriter
from ..parallel.dp import GradReducer, world_info

# CXXNET_FUSE_FC_SGD=0 keeps the fc weight steps in the fused optimizer launch
_FUSE_FC_SGD = os.environ.get("CXXNET_FUSE_FC_SGD", "1") != "0"
from ..utils.metric import DeviceMetricSet, MetricSet
from .neural_net import NeuralNet


class LaunchList:
    """One recorded run of library launches (csrc/kernels/launch_list.hip), replayed from C++."""
    __slots__ = ("h", "n")

    def __init__(self, h):
        self.h = h
        self.n = native.kernels().cxn_rec_size(h) if h else 0

    def replay(self):
        if self.n:
            from ..ops.gemm import _stream
            native.check(native.kernels().cxn_rec_replay(self.h, _stream()), "rec_replay")

    def __del__(self):
        if self.h:
            try:
                native.kernels().cxn_rec_free(self.h)
            except Exception:
                pass
            self.h = None


def _dist_ready() -> bool:
    import torch.distributed as dist
    return dist.is_available() and dist.is_initialized()


def prune_devices(batch_size: int, ndev: int) -> int:
    """Number of devices that cover a batch (reference nnet_impl-inl.hpp:344-354)."""
    ndev = max(int(ndev), 1)
    step = max((batch_size + ndev - 1) // ndev, 1)
    while ndev > 1 and step * (ndev - 1) >= batch_size:
        ndev -= 1
    return ndev


def parse_devices(val: str):
    """'gpu', 'gpu:0-3', 'gpu:0,1', 'cpu' -> (kind, [ids])."""
    kind = val.split(":")[0]
    ids = []
    if ":" in val:
        spec = val.split(":", 1)[1]
        if "-" in spec:
            a, b = spec.split("-")
            ids = list(range(int(a), int(b) + 1))
        else:
            ids = [int(x) for x in spec.split(",") if x != ""]
    return kind, ids


class NetTrainer:
    def __init__(self, net_type: int = 0):
        self.net_type = net_type
        self.batch_size = 100
        self.update_period = 1
        self.sample_counter = 0
        self.eval_train = 1
        self.epoch_counter = 0
        self.seed = 0
        self.silent = 0
        self.dev = "cpu"
        self.device_ids: List[int] = []
        self.type_pserver = "UNSPECIFIED"
        self.bucket_mb = 64.0
        self.comm_dtype = "fp32"
        self.shard_update = 0
        # data-parallel reduction: auto = replicated all-reduce (the path every backend runs
        # the same way); shard = reduce-scatter / sliced update / all-gather (opt-in, also
        # update_on_server = 1)
        self.dp_mode = "auto"
        self.dp_force = int(os.environ.get("CXXNET_DIST_FORCE", "0"))
        self.test_on_server = 0
        # overlapped per-bucket optimizer: on by default only under data parallelism
        # (1 GPU: the memory-bound update just competes with the memory-bound
        # pool/LRN backward, measured -1.7%)
        self.overlap_update = int(os.environ.get("CXXNET_OVERLAP_UPDATE", "-1"))
        # HIP-graph replay of the forward and backward passes (update_period 1): every
        # layer kernel of a step is launched by graph replays instead of one host call
        # each; the optimizer and (data parallel) the collectives stay eager launches, so
        # lr schedules still apply.  1 = on, 0 = off.
        # -1 (auto): on under data parallelism at per-GPU batch <= 64, where the Python
        # launch cost of ~150 kernels would otherwise approach the GPU step time
        self.cuda_graph = int(os.environ.get("CXXNET_CUDA_GRAPH", "-1"))
        self._graphs = {}
        self._graph_warm = {}
        # native launch-list executor (csrc/kernels/launch_list.hip): when graphs are not used,
        # the step's library launches are recorded once into C++ lists and replayed from C++
        # (one call per segment instead of ~10 us of Python per kernel); -1 auto, 0 off, 1 on
        self.launch_replay = int(os.environ.get("CXXNET_LAUNCH_REPLAY", "-1"))
        self._lists = {}
        self._list_warm = {}
        self._plan_gen = None  # NeuralNet.batch_gen the recorded / captured plans were made at
        # failure detection: every N updates, fail fast if any gradient was non-finite
        # (the reference only zeroes NaN inside clip, sgd_updater-inl.hpp:17)
        self.check_nonfinite = 0
        self._nf_flag = None
        self.deterministic = int(os.environ.get("CXXNET_DETERMINISTIC", "0"))
        # "bf16": HIP kernels; "fp32": the reference formulas in fp32 on the GPU (ops.mode)
        self.precision = os.environ.get("CXXNET_PRECISION", "bf16")
        # observability: HIP-event timers around forward / backward+reduce / optimizer
        self.profile_step = 0
        self.trace_layers = int(os.environ.get("CXXNET_TRACE_LAYERS", "0"))  # roctx range per layer
        self._timers = []
        self.step_times = {"fwd": 0.0, "bwd": 0.0, "opt": 0.0, "steps": 0}
        self.cfg: List[Tuple[str, str]] = []
        self.metric = MetricSet()
        self.train_metric = MetricSet()
        self.metric_specs: List[Tuple[str, str]] = []  # (metric, label field)
        self.eval_nodes: List[Tuple[str, int]] = []
        self.net_cfg = native.rt().NetConfig()
        self.net: Optional[NeuralNet] = None
        self.reducer: Optional[GradReducer] = None
        self.rank, self.world = world_info()
        self._rows = 0  # rows of the current batch that belong to this rank (0: idle rank)

    # ------------------------------------------------------------------ configuration
    def set_param(self, name: str, val: str):
        if name == "dev":
            kind, ids = parse_devices(val)
            self.dev = kind
            self.device_ids = ids
        elif name == "batch_size":
            self.batch_size = int(val)
        elif name == "update_period":
            self.update_period = int(val)
        elif name == "eval_train":
            self.eval_train = int(val)
        elif name == "seed":
            self.seed = int(val)
        elif name == "silent":
            self.silent = int(val)
        elif name == "param_server":
            self.type_pserver = val
        elif name == "dp_bucket_mb":
            self.bucket_mb = float(val)
        elif name == "dp_comm_dtype":
            self.comm_dtype = val
        elif name in ("update_on_server", "dp_shard_update"):
            self.shard_update = int(val)
        elif name == "dp_mode":
            if val not in ("auto", "shard", "allreduce"):
                raise ValueError(f"dp_mode must be auto, shard or allreduce, not {val}")
            self.dp_mode = val
        elif name == "dp_force":
            self.dp_force = int(val)
        elif name == "test_on_server":
            self.test_on_server = int(val)
        elif name == "overlap_update":
            self.overlap_update = int(val)
        elif name == "cuda_graph":
            self.cuda_graph = int(val)
        elif name == "launch_replay":
            self.launch_replay = int(val)
        elif name == "precision":
            if val not in ("bf16", "fp32"):
                raise ValueError(f"precision must be bf16 or fp32, not {val}")
            self.precision = val
        elif name == "check_nonfinite":
            self.check_nonfinite = int(val)
        elif name == "deterministic":
            # bitwise-reproducible steps on the GPU (ops.gemm.set_deterministic)
            self.deterministic = int(val)
        elif name == "profile_step":
            self.profile_step = int(val)
        elif name == "trace_layers":
            self.trace_layers = int(val)
        if name.startswith("metric"):
            import re
            m = re.match(r"metric\[([^,\]]+),([^\]]+)\]", name)
            if m:
                self.metric.add_metric(val, m.group(1))
                self.train_metric.add_metric(val, m.group(1))
                self.metric_specs.append((val, m.group(1)))
                self.eval_nodes.append((m.group(2), 0))
            else:
                m1 = re.match(r"metric\[([^\]]+)\]", name)
                field = m1.group(1) if m1 else "label"
                self.metric.add_metric(val, field)
                self.train_metric.add_metric(val, field)
                self.metric_specs.append((val, field))
                self.eval_nodes.append(("", -1))
        self.cfg.append((name, val))

    def _device(self) -> torch.device:
        if self.dev == "gpu" and torch.cuda.is_available():
            if self.world > 1:
                return torch.device("cuda", torch.cuda.current_device())
            idx = self.device_ids[0] if self.device_ids else 0
            return torch.device("cuda", idx)
        return torch.device("cpu")

    def _local_batch(self) -> int:
        step = max((self.batch_size + self.world - 1) // self.world, 1)
        return step

    def active_ranks(self) -> int:
        """Ranks that hold rows of the global batch: the reference drops devices while
        step * (ndev - 1) >= batch_size, keeping step = ceil(batch / ndev_requested)
        (src/nnet/nnet_impl-inl.hpp:344-354).  The launchers start only that many ranks;
        a rank beyond it (torchrun started with more) is IDLE: it runs the same schedule on
        stand-in rows with a zero loss weight, so it joins every collective and adds zero."""
        return prune_devices(self.batch_size, self.world)

    @property
    def idle(self) -> bool:
        return self.rank >= self.active_ranks()

    def _use_shard(self) -> bool:
        if self.shard_update or self.dp_mode == "shard":
            return True
        return False

    def _apply_modes(self):
        from ..ops.mode import set_reference_precision
        set_reference_precision(self._device().type == "cuda" and self.precision == "fp32")
        if self._device().type == "cuda":
            from ..ops import gemm
            if self.deterministic or gemm.deterministic():
                gemm.set_deterministic(bool(self.deterministic))

    def _make_net(self) -> NeuralNet:
        self._apply_modes()
        net = NeuralNet(self.net_cfg, self._local_batch(), self._device(), seed=self.seed)
        net.ctx.dp_shard = self._use_shard()
        net.ctx.dp_force = bool(self.dp_force) and self.world == 1 and _dist_ready()
        return net

    def _forward_global_params(self, net: NeuralNet):
        # the loss layers need the GLOBAL batch size and the update period
        for conn in net.connections:
            if hasattr(conn.layer, "batch_size") and conn.layer.batch_size == 0:
                conn.layer.batch_size = self.batch_size
            if hasattr(conn.layer, "update_period"):
                conn.layer.update_period = self.update_period

    def _init_eval_nodes(self):
        self.eval_ids = []
        for name, flag in self.eval_nodes:
            if flag == -1 or name == "":
                self.eval_ids.append(len(self.net.nodes) - 1)
            else:
                self.eval_ids.append(self.net_cfg.node_name_map[name])
        if not self.eval_ids:
            self.eval_ids = []

    @property
    def device_metrics(self) -> bool:
        return isinstance(self.train_metric, DeviceMetricSet)

    def _use_device_metrics(self):
        """On the GPU, metrics are accumulated on the device and read back only when
        printed (DeviceMetricSet); the CPU path keeps the native host MetricSet."""
        if self._device().type != "cuda" or self.device_metrics:
            return
        self.metric, self.train_metric = DeviceMetricSet(), DeviceMetricSet()
        for name, field in self.metric_specs:
            self.metric.add_metric(name, field)
            self.train_metric.add_metric(name, field)

    def _post_init(self):
        self._use_device_metrics()
        self._forward_global_params(self.net)
        self.net.trace_layers = self.trace_layers
        self._init_eval_nodes()
        self.reducer = GradReducer(self.net.arena, self.bucket_mb, True, self.comm_dtype,
                                   shard=self._use_shard(), force=bool(self.dp_force))
        if self.overlap_update == 1 or (self.overlap_update == -1 and self.reducer.active):
            net = self.net
            self.reducer.enable_overlapped_update(lambda ranges: net.update(self.epoch_counter, ranges))
        self.reducer.broadcast_params()

    def init_model(self):
        self.net_cfg.configure(self.cfg)
        self.net = self._make_net()
        self.net.init_model()
        self._post_init()

    # ------------------------------------------------------------------ model io
    def prepare_save(self, opt_state: bool = False):
        """Collective part of a save: every rank calls it (sharded mode gathers the fp32
        masters and, with opt_state, the optimizer state), then rank 0 serialises with
        save_model(sync=False) / save_optimizer_state(sync=False)."""
        if self.reducer is not None:
            self.reducer.sync_master(opt_state=opt_state)

    def save_model(self, sync: bool = True) -> bytes:
        if sync:
            self.prepare_save()
        fo = BinWriter()
        self.net.save_model(fo)
        blob = fo.getvalue()
        return self.net_cfg.save_net() + struct.pack("<qQ", self.epoch_counter, len(blob)) + blob

    def load_model(self, data: bytes, pos: int = 0):
        used = self.net_cfg.load_net(data[pos:])
        pos += used
        self.epoch_counter, blen = struct.unpack_from("<qQ", data, pos)
        pos += 16
        blob = data[pos:pos + blen]
        self.net_cfg.configure(self.cfg)
        self.net = self._make_net()
        self.net.load_model(BinReader(blob))
        self._post_init()

    def copy_model_from_bytes(self, data: bytes, pos: int = 0):
        """Finetune from a model file: parse the old structure and per-layer blobs
        (no device net is built for it) and copy every layer whose name matches."""
        from ..layers import LayerContext, create_layer
        old = native.rt().NetConfig()
        pos += old.load_net(data[pos:])
        _, blen = struct.unpack_from("<qQ", data, pos)
        fi = BinReader(data[pos + 16:pos + 16 + blen])
        ctx = LayerContext("cpu")
        loaded = {}
        for i, info in enumerate(old.layers):
            if info.type == 0:
                continue
            layer = create_layer(info.type, ctx)
            layer.load_model(fi)
            if info.name:
                loaded[info.name] = layer
        for name, li in self.net_cfg.layer_name_map.items():
            src = loaded.get(name)
            if src is None or not hasattr(src, "loaded"):
                continue
            dst = self.net.connections[li].layer
            vals = list(src.loaded)
            if hasattr(dst, "from_logical") and len(vals) and vals[0].dim() == 3:
                vals[0] = dst.from_logical(vals[0])
            if len(dst.params) < 1:
                continue
            for spec, v in zip(dst.params, vals):
                if v.numel() != spec.numel:
                    raise ValueError(f"CopyModelFrom: layer {name} shape mismatch")
                spec.w.copy_(v.reshape(spec.shape))
            print(f"Copying layer {name}")
        self.net.arena.sync_shadow()
        if self.reducer is not None:
            self.reducer.broadcast_params()

    def copy_model_from(self, other: "NetTrainer"):
        """Finetune: copy every layer whose name matches (reference nnet_impl-inl.hpp:101-134)."""
        src_map = dict(other.net_cfg.layer_name_map)
        for name, li in self.net_cfg.layer_name_map.items():
            if name not in src_map:
                continue
            sl = other.net.connections[src_map[name]].layer
            dl = self.net.connections[li].layer
            if len(sl.params) != len(dl.params):
                continue
            ok = all(tuple(a.shape) == tuple(b.shape) for a, b in zip(sl.params, dl.params))
            if not ok:
                raise ValueError(f"CopyModelFrom: layer {name} shape mismatch")
            print(f"Copying layer {name}")
            for a, b in zip(sl.params, dl.params):
                b.w.copy_(a.w.to(b.w.device))
        self.net.arena.sync_shadow()

    # ------------------------------------------------------------------ training
    def start_round(self, r: int):
        self.net.start_round(r)
        # every rank calls start_round at the same point: adopt one tile choice for whatever any
        # rank timed since the last sync (a short last batch, eval forwards)
        self._sync_tiles(force=True)
        if self.test_on_server and self.reducer is not None:
            self.reducer.check_consistency()

    def _slice(self, t: torch.Tensor, b: int):
        step = self._local_batch()
        lo = min(self.rank * step, b)
        hi = min((self.rank + 1) * step, b)
        return t[lo:hi]

    def _set_batch(self, batch, local=False):
        b = batch.batch_size
        self.net.ctx.loss_weight = 1.0
        if local:  # batch already holds this rank's rows
            data, extra, label = batch.data, batch.extra_data, batch.label
        elif self.world > 1 and self.idle:
            # idle rank (more ranks than the batch needs): the first rows of the batch stand in,
            # with a zero loss weight -- every gradient is zero, every collective is joined
            n = min(self._local_batch(), b)
            data, extra, label = batch.data[:n], [e[:n] for e in batch.extra_data], batch.label[:n]
            self.net.ctx.loss_weight = 0.0
            self._rows = 0
            self.net.set_input(data, extra)
            self.net.set_labels(label)
            return n
        else:
            data = self._slice(batch.data, b)
            extra = [self._slice(e, b) for e in batch.extra_data]
            label = self._slice(batch.label, b)
        self.net.set_input(data, extra)
        self.net.set_labels(label)
        self._rows = data.shape[0]
        return data.shape[0]

    def update(self, batch, local=False):
        """One training step on a global batch (each rank takes its slice), or on this
        rank's rows directly when local=True."""
        need_update = (self.sample_counter + 1) % self.update_period == 0
        first = self.sample_counter % self.update_period == 0
        if self.net.updater is not None:  # offsets of fc steps fused into this step's GEMMs
            self.net.updater.fused_offsets.clear()
        self._set_batch(batch, local)
        net = self.net
        self._cur_batch = batch
        ev = self._events()
        if self.net.ctx.is_gpu:
            self._drop_stale_plans()
        if self._graph_step(ev) or self._list_step(ev):
            self._after_step(ev)
            self._sync_tiles()
            return
        net.forward(True, pre_hook=self.reducer.before_forward)
        self._mark(ev, 1)
        evals = self._train_eval(batch)
        if need_update:
            self.reducer.start_step()
            net.ctx.sgd_fuse, net.ctx.sgd_fuse_gather_only = self._sgd_fuse_target()
            net.ctx.dp_active = self.reducer.active
            net.ctx.epoch = self.epoch_counter
            red = self.reducer
            hook = red.hook if (red.active or red.update_fn is not None) else None
            try:
                net.backprop(False, hook=hook, first=first, hook_due=red.due if hook is not None else None)
            finally:
                net.ctx.sgd_fuse, net.ctx.sgd_fuse_gather_only = None, False
            self.reducer.finish()
            self._check_grads()
            self._mark(ev, 2)
            if self.reducer.handles_update:
                pass  # per bucket on the side stream; the next forward gates on it
            elif self.reducer.shard:
                net.update(self.epoch_counter, self.reducer.owned_ranges())
                self.reducer.gather_params()
            else:
                net.update(self.epoch_counter)
        else:
            net.backprop(False, first=first)
            self._mark(ev, 2)
        self._after_step(ev)
        if evals is not None:
            self.train_metric.add_eval(evals, self._label_fields(batch))
        self._sync_tiles()
        self.sample_counter += 1
        if self.sample_counter >= self.update_period:
            self.sample_counter = 0
            self.epoch_counter += 1

    def _sync_tiles(self, force: bool = False):
        """Data parallelism: after each of the first two updates (the eager step that times
        the GEMM tile-table misses, and the step after it -- eager or graph-replayed) and at
        every round start (force), every rank adopts the same tile choice for every signature
        any rank timed (ops.gemm.sync_tune_table) -- fixed points in the schedule, so every
        rank enters the collective."""
        if self.world <= 1 or self.net is None or not self.net.ctx.is_gpu:
            return
        self._tile_syncs = getattr(self, "_tile_syncs", 0)
        if self._tile_syncs < 2 or force:
            self._tile_syncs += 1
            from ..ops import gemm
            gemm.sync_tune_table()

    def comm_bytes_per_step(self) -> int:
        """Bytes handed to collectives per update step on this rank: the gradient buckets
        (GradReducer.comm_bytes_per_step) plus, for every fullc_gather layer, the all-gathered
        [in | out-grad] rows (bf16, world x local rows each)."""
        red = self.reducer
        tot = red.comm_bytes_per_step() if red is not None else 0
        if self.world > 1 or (red is not None and red.active):
            for conn in self.net.connections:
                lay = conn.layer
                if getattr(lay, "_gathering", None) is not None and lay._gathering():
                    rows = conn.nodes_in[0].shape[0]
                    nin = lay.lp.num_input_node
                    nout = lay.lp.num_hidden
                    esz = 2 if self.net.ctx.is_gpu else 4
                    tot += rows * (nin + nout) * esz * max(self.world, 1)
        return tot

    # ------------------------------------------------------------------ step instrumentation
    def _events(self):
        if not self.profile_step or self.net.device.type != "cuda":
            return None
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
        ev[0].record()
        return ev

    @staticmethod
    def _mark(ev, i):
        if ev is not None:
            ev[i].record()

    def _after_step(self, ev):
        if ev is not None:
            ev[3].record()
            self._timers.append(ev)
            if len(self._timers) >= 8:  # resolve in batches: no per-step host sync
                self.flush_timers()

    def flush_timers(self):
        """Fold the recorded step events into step_times (ms totals)."""
        if not self._timers:
            return
        self._timers[-1][3].synchronize()
        st = self.step_times
        for e in self._timers:
            st["fwd"] += e[0].elapsed_time(e[1])
            st["bwd"] += e[1].elapsed_time(e[2])
            st["opt"] += e[2].elapsed_time(e[3])
            st["steps"] += 1
        self._timers = []

    def timing_report(self, reset: bool = True) -> str:
        """`fwd x ms, bwd+comm y ms, opt z ms per step, N img/s` since the last report."""
        self.flush_timers()
        st = self.step_times
        n = st["steps"]
        if n == 0:
            return ""
        tot = (st["fwd"] + st["bwd"] + st["opt"]) / n
        ips = self._local_batch() * self.world / (tot / 1000.0) if tot > 0 else 0.0
        out = (f"fwd {st['fwd'] / n:.2f} ms, bwd+comm {st['bwd'] / n:.2f} ms, opt {st['opt'] / n:.2f} ms "
               f"per step, {ips:.0f} img/s")
        if reset:
            self.step_times = {"fwd": 0.0, "bwd": 0.0, "opt": 0.0, "steps": 0}
        return out

    def _check_grads(self):
        """Fail fast on non-finite gradients (check_nonfinite = N: flag accumulated on the
        device every update, read back every N updates)."""
        if not self.check_nonfinite:
            return
        from .. import ops
        g = self.net.arena.g
        if self._nf_flag is None:
            self._nf_flag = torch.zeros(1, dtype=torch.int32, device=g.device)
        ops.nonfinite(g, self._nf_flag)
        if (self.epoch_counter + 1) % self.check_nonfinite == 0 and int(self._nf_flag.item()):
            raise FloatingPointError(f"non-finite gradient detected by update {self.epoch_counter + 1} "
                                     f"(check_nonfinite = {self.check_nonfinite})")

    # ------------------------------------------------------------------ optimizer state sidecar
    def save_optimizer_state(self, path: str, sync: bool = True):
        """Momentum / second moment and counters next to a model file (the model file itself
        stays byte-compatible with the reference layout, which has no optimizer state)."""
        if sync:
            self.prepare_save(opt_state=True)
        a = self.net.arena
        # per parameter, keyed "layer:tag": the arena layout depends on the world size
        # (fullc_gather segments sit on world * ALIGN boundaries), so a raw arena dump would map
        # momentum onto the wrong parameters when resumed at another world size
        state = {"m1_params": self._per_param(a.m1), "epoch_counter": torch.tensor([self.epoch_counter]),
                 "step_counter": self.net.ctx.step_counter.detach().cpu()}
        if a.m2 is not None:
            state["m2_params"] = self._per_param(a.m2)
        torch.save(state, path)

    def _per_param(self, buf):
        return {f"{li}:{s.tag}": buf[s.offset:s.offset + s.numel].detach().cpu().clone()
                for li, s in self.net.arena.specs}

    def _load_per_param(self, buf, params, path):
        for li, s in self.net.arena.specs:
            key = f"{li}:{s.tag}"
            t = params.get(key)
            if t is None or t.numel() != s.numel:
                raise ValueError(f"optimizer state {path}: parameter {key} missing or of another size")
            buf[s.offset:s.offset + s.numel].copy_(t.reshape(-1))

    def load_optimizer_state(self, path: str):
        state = torch.load(path, map_location="cpu", weights_only=True)
        a = self.net.arena
        if "m1_params" in state:
            self._load_per_param(a.m1, state["m1_params"], path)
            if "m2_params" in state:
                a.ensure_second_moment()
                self._load_per_param(a.m2, state["m2_params"], path)
        else:  # round-3 sidecars: the raw arena of a run at the same world size
            if state["m1"].numel() != a.m1.numel():
                raise ValueError(f"optimizer state {path}: {state['m1'].numel()} values, net has {a.m1.numel()}")
            a.m1.copy_(state["m1"])
            if "m2" in state:
                a.ensure_second_moment()
                a.m2.copy_(state["m2"])
        self.net.ctx.step_counter.copy_(state["step_counter"])

    def _sgd_fuse_target(self):
        """(updater, gather_only): the arena updater when the fc weight steps may run inside
        the weight-gradient GEMM (FullConnectLayer._fused_sgd) -- SGD, one micro-batch per
        update, no non-finite check (the gradient never reaches memory) -- else None.
        gather_only is True under data parallelism: then only fullc_gather layers may fuse,
        whose all-gathered gradient is already global; any other gradient must be reduced
        before its step (_fused_sgd asserts the pairing)."""
        net, red = self.net, self.reducer
        if not _FUSE_FC_SGD or net.device.type != "cuda" or self.update_period != 1 or self.check_nonfinite:
            return None, False
        upd = net.updater
        if upd is None or upd.algo != "sgd" or red is None:
            return None, False
        if red.active:
            return upd, True
        if red.handles_update:
            # one process with the per-bucket side-stream update (overlap_update = 1): the
            # buckets step the weights, so nothing fuses
            return None, False
        return upd, False

    def _graph_eligible(self) -> bool:
        net, red = self.net, self.reducer
        if not (self.cuda_graph != 0 and net.ctx.is_gpu and self.update_period == 1 and red is not None):
            return False
        if red.active and not red.handles_update:
            # data parallel without the overlapped update: the collectives (and, sharded, the
            # owned-range update + parameter gather) live in the eager step only
            return False
        # (fullc_gather layers issue their all-gathers through ctx.graph_cut: eager calls between
        # graph segments, like the bucket collectives)
        if self.cuda_graph < 0:
            # auto: data parallel at per-GPU batch <= 64, and only when the C++ launch lists
            # cannot take the step -- they replay the same plan faster (AlexNet b32, RCCL forced
            # at world 1: 1.233 vs 1.307 ms with fullc_gather, 1.139 vs 1.198 ms without,
            # profiles/r4_dp_graph_vs_lists_b32.jsonl: fewer, cheaper segment launches)
            if not (red.handles_update and self._local_batch() <= 64):
                return False
            return self.launch_replay == 0 or not all(c.layer.replay_safe() for c in net.connections)
        if red.handles_update:  # data parallel: segmented graphs around the collectives
            return True
        return self.world == 1 and not red.shard

    def _capture_plans(self):
        """Record the forward and backward passes as lists of HIP graphs with eager calls
        between them.  Without a reducer hook this is one graph per pass.  Under data
        parallelism (overlapped per-bucket update) the forward is cut before each layer
        that must wait for a bucket (the wait is an eager stream-event wait) and the
        backward is cut after each layer that completes a bucket (the eager call launches
        its RCCL collective and side-stream update), so collectives and waits stay
        outside the graphs and replays keep the eager schedule.  fullc_gather layers cut the
        graphs themselves around their row all-gathers (ctx.graph_cut)."""
        net, red = self.net, self.reducer
        dp = red.handles_update
        red.sync()
        torch.cuda.synchronize()
        pool = torch.cuda.graph_pool_handle()
        cur = {}

        def begin(plan):
            g = torch.cuda.CUDAGraph()
            g.capture_begin(pool=pool)
            cur["g"], cur["plan"] = g, plan

        def end():
            cur["g"].capture_end()
            cur["plan"].append(cur["g"])

        def cut(fn):
            plan = cur["plan"]
            end()
            plan.append(fn)
            begin(plan)

        waited, ready = set(), set()

        def fwd_hook(li):
            new = [bi for bi in red.layer_buckets.get(li, ()) if bi not in waited]
            if new:
                waited.update(new)
                cut(functools.partial(red.before_forward, li))

        def bwd_due(li):
            return any(bi not in ready and li <= b.li_min for bi, b in enumerate(red.buckets))

        def bwd_hook(li):
            bs = [bi for bi, b in enumerate(red.buckets) if bi not in ready and li <= b.li_min]
            if bs:
                ready.update(bs)
                cut(functools.partial(red.ready_buckets, bs))

        fwd, bwd = [], []
        net.ctx.graph_cut = cut
        try:
            with torch.cuda.stream(torch.cuda.Stream()):
                begin(fwd)
                net.forward(True, pre_hook=fwd_hook if dp else None)
                end()
                self._plan_fuse(True)  # (stages the device schedule row before capturing)
                begin(bwd)
                net.backprop(False, hook=bwd_hook if dp else None, first=True, hook_due=bwd_due if dp else None)
                end()
        finally:
            net.ctx.graph_cut = None
            self._plan_fuse(False)
        torch.cuda.synchronize()
        fused = frozenset(net.updater.fused_offsets) if net.updater is not None else frozenset()
        if net.updater is not None:
            net.updater.fused_offsets.clear()  # the capture ran nothing; the replays add them back
        return fwd, bwd, fused

    @staticmethod
    def _replay(plan):
        for item in plan:
            if isinstance(item, (torch.cuda.CUDAGraph, LaunchList)):
                item.replay()
            else:
                item()

    # ------------------------------------------------------------------ native launch lists
    def _list_eligible(self) -> bool:
        """The C++ launch-list executor runs a step when HIP graphs do not (under data
        parallelism it is the auto choice, _graph_eligible).  Auto (-1): in the host-bound regime
        only -- per-GPU batch <= 32 on one GPU (<= 64 data parallel), where Python enqueues a
        step about as slowly as the GPU runs it; larger steps are GPU-bound and stay eager.  A
        planned step keeps the fused fc SGD steps (schedule values from the updater's device
        table, _plan_fuse)."""
        net, red = self.net, self.reducer
        if self.launch_replay == 0 or not net.ctx.is_gpu or self.update_period != 1 or red is None:
            return False
        if red.active and not red.handles_update:
            return False  # as _graph_eligible: the reduction runs in the eager step only
        if self._graph_eligible():
            return False
        if not all(c.layer.replay_safe() for c in net.connections):
            return False
        if self.launch_replay < 0:
            # host-bound regime: per-GPU batch <= 32 on one GPU, <= 64 under data parallelism
            # (where the collectives add host work between the segments)
            return self._local_batch() <= (64 if red.handles_update else 32)
        return True

    def _drop_stale_plans(self):
        """Launch lists and HIP graphs hold raw addresses of layer buffers; a batch-size change
        lets layers reallocate shape-dependent ones (pool state, softmax scores, pad copies), so
        plans made before it may point at freed memory.  Drop them all; the next steps warm up
        and record again (plans are per batch size, and batch sizes rarely alternate)."""
        gen = getattr(self.net, "batch_gen", 0)
        if self._plan_gen == gen:
            return
        if self._lists or self._graphs:
            torch.cuda.synchronize()  # no replay of the old plans is still running
        self._lists.clear()
        self._list_warm.clear()
        self._graphs.clear()
        self._graph_warm.clear()
        self._plan_gen = gen

    def _list_step(self, ev=None) -> bool:
        """One training step replayed from recorded C++ launch lists: the forward and backward
        passes as runs of library launches, with the same eager calls between them as the
        graph plan (bucket collectives and waits, fullc_gather all-gathers).  The first step
        of each batch size runs eagerly (GEMM tile tuning, lazy buffers); the second runs AND
        records (_record_step); later steps replay.  Returns False to take the eager path."""
        if not self._list_eligible():
            return False
        net, red = self.net, self.reducer
        key = net.cur_batch
        plans = self._lists.get(key)
        if plans is None:
            if self._list_warm.get(key, 0) < 1:
                self._list_warm[key] = 1
                return False
            self._lists[key] = self._record_step(ev)
            return True
        fwd, bwd, fused = plans[0], plans[1], plans[3]
        self._replay(fwd)
        self._mark(ev, 1)
        self._finish_planned_step(ev, lambda: self._replay(bwd), fused)
        return True

    def _plan_fuse(self, on: bool):
        """Fused fc SGD steps inside a planned step being recorded / captured: the same
        eligibility as the eager step (_sgd_fuse_target), with the schedule values read from
        the updater's device table (ArenaUpdater.stage_hyper) so every replay follows the lr /
        momentum schedule.  Returns whether the plan fuses."""
        net = self.net
        if not on:
            net.ctx.sgd_fuse, net.ctx.sgd_fuse_gather_only, net.ctx.sgd_hyp_dev = None, False, False
            return False
        upd, gather_only = self._sgd_fuse_target()
        net.ctx.sgd_fuse, net.ctx.sgd_fuse_gather_only = upd, gather_only
        net.ctx.sgd_hyp_dev = upd is not None
        net.ctx.dp_active = self.reducer.active
        net.ctx.epoch = self.epoch_counter
        if upd is not None:
            upd.stage_hyper(self.epoch_counter)
        return upd is not None

    def _finish_planned_step(self, ev, run_bwd, fused=None):
        """The part of a planned (graph / launch-list) step after the forward: training
        metrics, the backward (run_bwd) framed by the reducer, the optimizer.  fused: the arena
        offsets whose SGD step the plan's backward runs inside fc weight-gradient GEMMs (the
        optimizer and the per-bucket updates skip them); their device schedule row is
        refreshed first."""
        net, red = self.net, self.reducer
        # a planned step reduces gradients only through the overlapped per-bucket update; the
        # eligibility rules (_graph_eligible / _list_eligible) keep every other DP mode eager
        assert red.handles_update or not red.active, "planned step under DP without the overlapped update"
        if fused:
            net.updater.stage_hyper(self.epoch_counter)
            net.updater.fused_offsets.update(fused)
        evals = self._train_eval(self._cur_batch)
        if red.handles_update:
            red.start_step()
            run_bwd()
            red.finish()
            self._check_grads()
            self._mark(ev, 2)
        else:
            run_bwd()
            self._check_grads()
            self._mark(ev, 2)
            net.update(self.epoch_counter)
        if evals is not None:
            self.train_metric.add_eval(evals, self._label_fields(self._cur_batch))
        self.epoch_counter += 1

    def _record_step(self, ev):
        """Run one step while recording its library launches into C++ lists, cut at the same
        points as _capture_plans (here the eager calls also run, since the recording run is
        a real step).  Allocations of the recording run come from a private memory pool kept
        with the plan, so every address a list holds stays valid for its replays."""
        from ..ops.mode import set_recording
        net, red = self.net, self.reducer
        dp = red.handles_update
        k = native.kernels()
        pool = torch.cuda.MemPool()
        cur = {}

        def begin(plan):
            native.check(k.cxn_rec_begin(), "rec_begin")
            cur["plan"] = plan

        def end():
            cur["plan"].append(LaunchList(k.cxn_rec_end()))

        def cut(fn):
            plan = cur["plan"]
            end()
            fn()
            plan.append(fn)
            begin(plan)

        waited, ready = set(), set()

        def fwd_hook(li):
            new = [bi for bi in red.layer_buckets.get(li, ()) if bi not in waited]
            if new:
                waited.update(new)
                cut(functools.partial(red.before_forward, li))

        def bwd_due(li):
            return any(bi not in ready and li <= b.li_min for bi, b in enumerate(red.buckets))

        def bwd_hook(li):
            bs = [bi for bi, b in enumerate(red.buckets) if bi not in ready and li <= b.li_min]
            if bs:
                ready.update(bs)
                cut(functools.partial(red.ready_buckets, bs))

        fwd, bwd = [], []

        def record_bwd():
            self._plan_fuse(True)
            begin(bwd)
            try:
                net.backprop(False, hook=bwd_hook if dp else None, first=True, hook_due=bwd_due if dp else None)
            finally:
                end()
                self._plan_fuse(False)

        net.ctx.graph_cut = cut
        set_recording(True)
        try:
            with torch.cuda.use_mem_pool(pool):
                begin(fwd)
                try:
                    net.forward(True, pre_hook=fwd_hook if dp else None)
                finally:
                    end()
                self._mark(ev, 1)
                self._finish_planned_step(ev, record_bwd)
        finally:
            set_recording(False)
            net.ctx.graph_cut = None
            h = k.cxn_rec_end()  # an exception left a list open: drop it
            if h:
                k.cxn_rec_free(h)
        fused = frozenset(net.updater.fused_offsets) if net.updater is not None else frozenset()
        return fwd, bwd, pool, fused

    def _graph_step(self, ev=None) -> bool:
        """One training step as HIP-graph replays of the forward and backward passes plus
        the eager optimizer (1 GPU) or, under data parallelism, graph segments around the
        eager bucket collectives and the side-stream per-bucket update.  The first step of
        each batch size runs eagerly (it autotunes the GEMM tiles and allocates the layers'
        persistent buffers); the second captures.  Inputs and labels live in static node /
        label buffers, so a replay reads the batch that _set_batch just staged.  Returns
        False to take the eager path."""
        if not self._graph_eligible():
            return False
        net, red = self.net, self.reducer
        key = net.cur_batch
        gr = self._graphs.get(key)
        if gr is None:
            if self._graph_warm.get(key, 0) < 1:
                self._graph_warm[key] = 1
                return False
            try:
                with DEVICE_IO_LOCK:  # no input-thread allocations during a global-mode capture
                    gr = self._capture_plans()
            except Exception as e:  # a layer that syncs with the host (e.g. pairtest): stay eager
                if not self.silent:
                    print(f"cuda_graph: capture failed ({type(e).__name__}: {e}); running eagerly")
                self.cuda_graph = 0
                torch.cuda.synchronize()
                return False
            self._graphs[key] = gr
        fwd, bwd, fused = gr
        self._replay(fwd)
        self._mark(ev, 1)
        self._finish_planned_step(ev, lambda: self._replay(bwd), fused)
        return True

    # ------------------------------------------------------------------ inference
    def _node_output(self, nid: int) -> torch.Tensor:
        node = self.net.nodes[nid]
        if node.fp32_view is not None:
            out = node.fp32_view[: self.net.cur_batch]
            return out.view(out.shape[0], *node.shape[1:])
        with_data = node.data[: self.net.cur_batch]
        from ..ops import nhwc_to_nchw
        return nhwc_to_nchw(with_data, node.shape[1], node.shape[3])

    def _gather(self, t: torch.Tensor) -> torch.Tensor:
        if self.world == 1:
            return t
        import torch.distributed as dist
        n = torch.tensor([t.shape[0]], device=t.device)
        sizes = [torch.zeros_like(n) for _ in range(self.world)]
        dist.all_gather(sizes, n)
        mx = int(max(s.item() for s in sizes))
        pad = torch.zeros((mx,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
        pad[: t.shape[0]] = t
        outs = [torch.empty_like(pad) for _ in range(self.world)]
        dist.all_gather(outs, pad)
        return torch.cat([o[: int(s.item())] for o, s in zip(outs, sizes)], 0)

    def _train_eval(self, batch):
        """Training metrics of this step (eval_train): on the device they are accumulated
        right here, enqueued behind the forward pass (the loss layer keeps its fp32 scores,
        backprop only rewrites the bf16 node) -- no host copy; the host path returns the
        scores for MetricSet.add_eval after the step."""
        if not self.eval_train or not self.eval_ids:
            return None
        if self.device_metrics:
            self.train_metric.add_eval(self._eval_scores(), self.net.ctx.label_fields, rows=self._rows)
            return None
        return self._collect_eval()

    def _eval_scores(self) -> List[torch.Tensor]:
        """Device (B, K) fp32 score views of the eval nodes, each node computed once."""
        seen = {}
        out = []
        for nid in self.eval_ids:
            if nid not in seen:
                seen[nid] = self._node_output(nid).reshape(self.net.cur_batch, -1).float()
            out.append(seen[nid])
        return out

    def _metric_reduce(self):
        if self.world == 1:
            return None
        import torch.distributed as dist

        def red(t):
            dist.all_reduce(t, op=dist.ReduceOp.SUM)
            return t
        return red

    def _collect_eval(self) -> List[np.ndarray]:
        out = []
        for nid in self.eval_ids:
            t = self._gather(self._node_output(nid).reshape(self.net.cur_batch, -1)[: self._rows].float())
            out.append(t.cpu().numpy())
        return out

    def _label_fields(self, batch):
        lab = batch.label.float().cpu().numpy()
        if lab.ndim == 1:
            lab = lab.reshape(-1, 1)
        out = {}
        for name, idx in self.net_cfg.label_name_map.items():
            a, b = self.net_cfg.label_range[idx]
            out[name] = lab[:, a:b]
        return out

    def forward_to(self, node_ids: List[int], batch) -> List[np.ndarray]:
        self.reducer.sync()
        self._set_batch(batch)
        self.net.forward(False)
        return [self._gather(self._node_output(n)[: self._rows].contiguous().float()).cpu().numpy()
                for n in node_ids]

    def predict(self, batch) -> np.ndarray:
        out = self.forward_to([len(self.net.nodes) - 1], batch)[0]
        out = out.reshape(out.shape[0], -1)
        if out.shape[1] != 1:
            return out.argmax(1).astype(np.float32)
        return out[:, 0].astype(np.float32)

    def extract_feature(self, batch, node_name: str) -> np.ndarray:
        import re
        m = re.match(r"top\[-(\d+)\]", node_name)
        nnode = len(self.net.nodes)
        if m:
            off = int(m.group(1))
            if not (1 <= off <= nnode):
                raise ValueError("ExtractFeature: offset must be within num_node range")
            nid = nnode - off
        else:
            if node_name not in self.net_cfg.node_name_map:
                raise ValueError(f"ExtractFeature: Cannot find node name: {node_name}")
            nid = self.net_cfg.node_name_map[node_name]
        return self.forward_to([nid], batch)[0]

    def evaluate(self, it, data_name: str) -> str:
        ret = ""
        if self.eval_train != 0:
            if self.device_metrics:
                ret += self.train_metric.print("train", self._metric_reduce())
            else:
                ret += self.train_metric.print("train")
            self.train_metric.clear()
        if it is None:
            return ret
        self.metric.clear()
        it.before_first()
        if self.device_metrics:
            while it.next():
                batch = it.value()
                self.reducer.sync()
                b = self._set_batch(batch)
                self.net.forward(False)
                n = batch.batch_size - batch.num_batch_padd  # valid rows of the global batch
                lo = min(self.rank * self._local_batch(), batch.batch_size)
                self.metric.add_eval(self._eval_scores(), self.net.ctx.label_fields, rows=max(0, min(b, n - lo)))
            return ret + self.metric.print(data_name, self._metric_reduce())
        while it.next():
            batch = it.value()
            scores = self.forward_to(self.eval_ids, batch)
            n = batch.batch_size - batch.num_batch_padd
            scores = [s[:n].reshape(n, -1) for s in scores]
            fields = {k: v[:n] for k, v in self._label_fields(batch).items()}
            self.metric.add_eval(scores, fields)
        ret += self.metric.print(data_name)
        return ret

    # ------------------------------------------------------------------ weights
    def _param(self, layer_name: str, tag: str):
        if tag not in ("bias", "wmat"):
            raise ValueError("NNet.SetWeight: weight tag can only be bias or wmat")
        li = self.net_cfg.get_layer_index(layer_name)
        layer = self.net.connections[li].layer
        for p in layer.params:
            if p.tag == tag:
                return layer, p
        raise ValueError(f"layer {layer_name} has no {tag}")

    def get_weight(self, layer_name: str, tag: str) -> np.ndarray:
        if self.reducer is not None:
            self.reducer.sync_master()
        layer, p = self._param(layer_name, tag)
        w = p.w.detach().float().cpu()
        if hasattr(layer, "to_logical") and tag == "wmat":
            w = layer.to_logical(w)
        return w.reshape(w.shape[0], -1).numpy() if w.dim() > 1 else w.reshape(1, -1).numpy()

    def set_weight(self, weight: np.ndarray, layer_name: str, tag: str):
        if self.reducer is not None:
            self.reducer.sync_master()
        layer, p = self._param(layer_name, tag)
        w = torch.as_tensor(np.asarray(weight, dtype=np.float32))
        if hasattr(layer, "from_logical") and tag == "wmat":
            lp = layer.lp
            G = lp.num_group
            w = layer.from_logical(w.reshape(G, lp.num_channel // G, -1))
        p.w.copy_(w.reshape(p.shape))
        self.net.arena.sync_shadow()
