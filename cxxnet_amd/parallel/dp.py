"""Data parallelism: one process per GPU, RCCL collectives over xGMI.

Replaces the reference's mshadow-ps "local"/"dist" parameter server
(src/updater/async_updater-inl.hpp:94-127, src/nnet/nnet_impl-inl.hpp:376-390):
  * init: rank 0's weights are broadcast (reference serialises a model blob on
    device 0 and loads it on the others, nnet_impl-inl.hpp:70-81);
  * every step the fp32 gradient arena is reduced (SUM -- the loss is already
    scaled by the global batch, loss_layer_base-inl.hpp:62) in BUCKETS.  The arena is
    laid out in reverse layer order, so bucket k only needs the layers above some
    index: its collective is launched from the backprop hook the moment that layer
    finishes and runs on RCCL's stream while backward continues on the compute
    stream (the reference's priority push/pull, priority = -layer);
  * the optimizer for a bucket runs on a side stream as soon as that bucket is
    reduced (the reference's pull callback, async_updater-inl.hpp:200-221), and the
    NEXT forward gates each layer on the event of the bucket holding its weights
    (the reference's per-layer UpdateWait -> PullWait, neural_net-inl.hpp:125-131).

Two reduction modes:
  * replicated (``dp_mode = allreduce``): fp32 all-reduce of each bucket, every rank
    runs the optimizer on the whole bucket.  8 B/param on the wire.
  * sharded (``dp_mode = shard``, opt-in; also ``update_on_server = 1``; ``dp_mode = auto``
    stays on the replicated all-reduce).  This maps the reference's parameter server
    (nnet_ps_server.cpp:54-89: each server owns some keys, workers push gradients and
    pull updated weights) onto collectives: each bucket is REDUCE-SCATTERED (fp32), rank
    r updates the fp32 master / optimizer state of its 1/N slice only, and the bf16
    compute weights of the slice are ALL-GATHERED.  6 B/param on the wire and 1/N of
    the optimizer's HBM traffic per GPU, with the same numerics as the replicated mode
    (the compute weights are the bf16 rounding of an fp32 master updated with an fp32
    summed gradient in both).  The fp32 masters of other ranks' slices are fetched only
    when needed (save / get_weight).

Bucket size defaults to 64 MB: AlexNet's 244 MB of gradients become 3-4 messages, large
enough to run at link rate over the 7 xGMI links of a ring, small enough that the
fc8/fc7 buckets overlap the conv backward.  With 288 GB of HBM per GPU, buckets are
sized for overlap, never for memory.

``dp_force = 1`` runs the collectives even with a single rank (world 1): the RCCL path
(async work handles, side-stream waits, per-bucket gating) then executes on a one-GPU box.
"""
from __future__ import annotations

import os
from typing import List, Optional

import torch
import torch.distributed as dist


def world_info():
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


class Bucket:
    def __init__(self, start, end, li_min):
        self.start, self.end, self.li_min = start, end, li_min
        self.work = None      # reduction in flight
        self.ag_work = None   # sharded: all-gather of the compute weights in flight
        self.buf = None
        self.out = None       # sharded: this rank's reduced chunk
        self.agin = None      # sharded: all-gather source
        self.ready = False
        self.done = None      # event on the side stream: bucket reduced, updated (and gathered)
        self.final = None     # event on the compute stream: the bucket's gradients are final
        self.pending = False  # done recorded but not yet waited for by the compute stream

    def own(self, rank, world):
        c = (self.end - self.start) // world
        return self.start + rank * c, self.start + (rank + 1) * c

    @property
    def numel(self):
        return self.end - self.start


class GradReducer:
    def __init__(self, arena, bucket_mb: float = 64.0, overlap: bool = True, comm_dtype: str = "fp32",
                 group=None, shard: bool = False, force: bool = False):
        self.arena = arena
        self.group = group
        self.rank, self.world = world_info()
        self.force = bool(force) and dist.is_available() and dist.is_initialized()
        self.overlap = overlap
        self.shard = bool(shard) and (self.world > 1 or self.force)
        self.comm_dtype = torch.bfloat16 if comm_dtype == "bf16" else torch.float32
        limit = max(1, int(bucket_mb * (1 << 20) / 4))
        # at least ~4 buckets: a model whose gradients fit one bucket (GoogLeNet: 7M parameters,
        # 28 MB) would otherwise reduce nothing until the whole backward is done, leaving the
        # collective, the update and the all-gather exposed in front of the next forward
        limit = min(limit, max(1 << 18, arena.total // 4))
        self.buckets: List[Bucket] = []
        self.update_fn = None      # overlapped per-bucket optimizer (enable_overlapped_update)
        self.side = None
        self.extra_ranges = []     # fullc_gather segments: updated after backward
        # RCCL runs reduce-scatter / all-gather IN PLACE (output = this rank's chunk of the
        # input): no staging buffers and no copies; gloo gets separate buffers
        # (CXXNET_DP_INPLACE=1 takes the in-place path on gloo too: the CPU tests exercise RCCL's
        # aliasing layout -- gloo honours the same in-place semantics)
        self.inplace = (self.comm_dtype == torch.float32 and dist.is_available() and dist.is_initialized()
                        and (dist.get_backend(group) == "nccl" or os.environ.get("CXXNET_DP_INPLACE") == "1"))
        if self.shard:
            self._shard_buckets(limit)
        else:
            self._plain_buckets(limit)
        self._map_layers()

    # ------------------------------------------------------------------ bucket plans
    def _plain_buckets(self, limit):
        cur_start, cur_end, cur_li = None, 0, None
        for li, spec in self.arena.specs:  # arena order = reverse layer order
            li = getattr(spec, "grad_li", li)  # the layer after whose backprop the gradient is final
            s, e = spec.offset, spec.offset + spec.numel
            if getattr(spec, "no_reduce", False):  # fullc_gather: gradient is already global
                self.extra_ranges.append((s, e))
                if cur_start is not None and cur_end > cur_start:
                    self.buckets.append(Bucket(cur_start, cur_end, cur_li))
                cur_start, cur_end, cur_li = None, 0, None
                continue
            if cur_start is None:
                cur_start, cur_li = s, li
            if e - cur_start > limit and cur_end > cur_start:
                self.buckets.append(Bucket(cur_start, cur_end, cur_li))
                cur_start, cur_li = s, li
            cur_end = e
            cur_li = min(cur_li, li)
        if cur_start is not None and cur_end > cur_start:
            self.buckets.append(Bucket(cur_start, cur_end, cur_li))

    def _shard_buckets(self, limit):
        """Buckets cut at multiples of world*ALIGN (the arena total is one too), so
        every bucket splits into equal aligned per-rank chunks.  A cut may fall inside
        a segment; a bucket is launched once every layer it touches is done."""
        from ..nnet.arena import ALIGN
        q = ALIGN * max(self.world, 1)
        total = self.arena.total
        assert total % q == 0, "arena must be padded to world*ALIGN"
        segs = [(spec.offset, spec.offset + spec.numel, getattr(spec, "grad_li", li)) for li, spec in self.arena.specs
                if not getattr(spec, "no_reduce", False)]
        # fullc_gather segments (q-aligned by the arena) hold a global gradient: every rank
        # updates them whole, they are cut out of the reduced runs
        runs, pos = [], 0
        for li, spec in self.arena.specs:
            if getattr(spec, "no_reduce", False):
                lo, hi = spec.offset, (spec.offset + spec.numel + q - 1) // q * q
                assert lo % q == 0, "fullc_gather segment not aligned to world*ALIGN"
                self.extra_ranges.append((spec.offset, spec.offset + spec.numel))
                if lo > pos:
                    runs.append((pos, lo))
                pos = hi
        if total > pos:
            runs.append((pos, total))
        for r0, r1 in runs:
            start = r0
            while start < r1:
                end = min(r1, start + max(q, (limit + q - 1) // q * q))
                # extend to the end of the segment that the cut falls into, rounded up to q
                for a, b, _ in segs:
                    if a < end < b:
                        end = min(r1, (b + q - 1) // q * q)
                        break
                lis = [li for a, b, li in segs if a < end and b > start]
                if lis:
                    self.buckets.append(Bucket(start, end, min(lis)))
                start = end
        if self.inplace:
            return
        for b in self.buckets:
            c = (b.end - b.start) // self.world
            b.out = torch.empty(c, dtype=self.comm_dtype, device=self.arena.g.device)
            sh = self.arena.wb if self.arena.wb is not None else self.arena.w
            b.agin = torch.empty(c, dtype=sh.dtype, device=sh.device)

    def _map_layers(self):
        """layer index -> buckets holding (part of) that layer's parameters."""
        self.layer_buckets = {}
        for li, spec in self.arena.specs:
            li = getattr(spec, "fwd_li", li)  # the layer whose forward reads it
            s, e = spec.offset, spec.offset + spec.numel
            for bi, b in enumerate(self.buckets):
                if b.start < e and s < b.end:
                    self.layer_buckets.setdefault(li, []).append(bi)

    def owned_ranges(self):
        """[start, end) arena ranges this rank updates (sharded mode): its slice of every
        bucket, plus the fullc_gather segments, which every rank updates whole."""
        return [b.own(self.rank, self.world) for b in self.buckets] + list(self.extra_ranges)

    @property
    def active(self):
        return self.world > 1 or self.force

    @property
    def handles_update(self) -> bool:
        """The optimizer runs inside the reducer (per bucket, on the side stream)."""
        return self.update_fn is not None

    def comm_bytes_per_step(self) -> int:
        """Bytes handed to the collectives per update step on each rank (algorithm bytes:
        the bucket payloads, not the ring's 2(N-1)/N wire factor)."""
        if not self.active:
            return 0
        tot = 0
        esz = 2 if self.comm_dtype == torch.bfloat16 else 4
        for b in self.buckets:
            tot += b.numel * esz
            if self.shard:
                sh = self.arena.wb if self.arena.wb is not None else self.arena.w
                tot += b.numel * sh.element_size()
        return tot

    def broadcast_params(self, src: int = 0):
        if not self.active:
            return
        dist.broadcast(self.arena.w, src=src, group=self.group)
        self.arena.sync_shadow()

    def enable_overlapped_update(self, update_fn):
        """Run the optimizer per bucket on a side stream as soon as the bucket's
        gradients are final (and, under data parallelism, reduced), so the update of
        the large fc layers overlaps the conv backward.  In sharded mode the
        update covers this rank's slice and is followed by the all-gather of the bucket's
        compute weights.  GPU only."""
        if not self.arena.g.is_cuda:
            return False
        self.update_fn = update_fn
        self.side = torch.cuda.Stream(device=self.arena.g.device)
        for b in self.buckets:
            b.done = torch.cuda.Event()
            b.final = torch.cuda.Event()  # gradients final on the compute stream (reused every step)
        return True

    # ------------------------------------------------------------------ per step
    def start_step(self):
        # a bucket still pending from the previous step must be consumed before its
        # gradient range is rewritten: wait for all of them (normally the forward did)
        self.sync()
        for b in self.buckets:
            b.work = None
            b.ag_work = None
            b.ready = False

    def _launch(self, b: Bucket):
        g = self.arena.g[b.start:b.end]
        if self.shard:
            if self.inplace:
                lo, hi = b.own(self.rank, self.world)
                b.buf = None
                b.work = dist.reduce_scatter_tensor(self.arena.g[lo:hi], g, op=dist.ReduceOp.SUM,
                                                    group=self.group, async_op=True)
                return
            src = g if self.comm_dtype == torch.float32 else g.to(self.comm_dtype)
            b.buf = src  # keep the (possibly converted) source alive until the op is done
            b.work = dist.reduce_scatter_tensor(b.out, src, op=dist.ReduceOp.SUM, group=self.group,
                                                async_op=True)
            return
        if self.comm_dtype == torch.float32:
            b.buf = None
            b.work = dist.all_reduce(g, op=dist.ReduceOp.SUM, group=self.group, async_op=True)
        else:
            b.buf = g.to(self.comm_dtype)
            b.work = dist.all_reduce(b.buf, op=dist.ReduceOp.SUM, group=self.group, async_op=True)

    def _ready(self, b: Bucket):
        """Bucket b's gradients are final on the compute stream."""
        b.ready = True
        if self.active:
            self._launch(b)
        if self.update_fn is None:
            return
        b.final.record()
        with torch.cuda.stream(self.side):
            self.side.wait_event(b.final)
            if self.active:
                b.work.wait()  # the side stream waits for the collective (no host block)
                if self.shard and not self.inplace:
                    lo, hi = b.own(self.rank, self.world)
                    self.arena.g[lo:hi].copy_(b.out)
                elif b.buf is not None:
                    self.arena.g[b.start:b.end].copy_(b.buf)
                if b.buf is not None:
                    b.buf.record_stream(self.side)
                b.buf = None
                b.work = None
            if self.shard:
                self.update_fn([b.own(self.rank, self.world)])
                a = self.arena
                sh = a.wb if a.wb is not None else a.w
                lo, hi = b.own(self.rank, self.world)
                src = sh[lo:hi]
                if not self.inplace:
                    b.agin.copy_(src)
                    src = b.agin
                # issued with the side stream current: RCCL's stream waits for the update
                b.ag_work = dist.all_gather_into_tensor(sh[b.start:b.end], src, group=self.group,
                                                        async_op=True)
                b.ag_work.wait()  # the side stream waits for the gather
                b.ag_work = None
            else:
                self.update_fn([(b.start, b.end)])
            b.done.record(self.side)
            b.pending = True

    def ready_buckets(self, indices):
        """Launch buckets `indices` (their gradients are final on the compute stream)."""
        for bi in indices:
            b = self.buckets[bi]
            if not b.ready:
                self._ready(b)

    def due(self, layer_index: int) -> bool:
        """Whether hook(layer_index) launches a bucket (the executor flushes queued gradient
        work of the pass before it)."""
        if not self.overlap or not (self.active or self.update_fn is not None):
            return False
        return any(not b.ready and layer_index <= b.li_min for b in self.buckets)

    def hook(self, layer_index: int):
        """Called after each layer's backprop (reverse order)."""
        if not self.overlap or not (self.active or self.update_fn is not None):
            return
        for b in self.buckets:
            if not b.ready and layer_index <= b.li_min:
                self._ready(b)

    def finish(self):
        """Launch what is left.  With the overlapped update nothing waits here: the next
        forward gates each layer on its bucket (before_forward); otherwise the compute
        stream waits for every reduction."""
        if self.update_fn is not None:
            for b in self.buckets:
                if not b.ready:
                    self._ready(b)
            if self.extra_ranges:  # fullc_gather segments: their gradient is complete now
                self.update_fn(self.extra_ranges)
            return
        if not self.active:
            return
        for b in self.buckets:
            if b.work is None:
                self._launch(b)
                b.ready = True
        for b in self.buckets:
            b.work.wait()
            if self.shard:
                if not self.inplace:
                    lo, hi = b.own(self.rank, self.world)
                    self.arena.g[lo:hi].copy_(b.out)
                b.buf = None
            elif b.buf is not None:
                self.arena.g[b.start:b.end].copy_(b.buf)
                b.buf = None
            b.work = None

    def before_forward(self, layer_index: int):
        """Per-bucket gating: the compute stream waits for the buckets holding this
        layer's weights (reduced, updated and, sharded, gathered) and nothing else."""
        if self.update_fn is None:
            return
        for bi in self.layer_buckets.get(layer_index, ()):
            b = self.buckets[bi]
            if b.pending:
                torch.cuda.current_stream().wait_event(b.done)
                b.pending = False

    def sync(self):
        """Make the current stream wait for every outstanding bucket (before anything
        other than a gated training forward reads the weights: eval, save, get/set)."""
        if self.update_fn is None:
            return
        cur = torch.cuda.current_stream()
        for b in self.buckets:
            if b.pending:
                cur.wait_event(b.done)
                b.pending = False

    def gather_params(self):
        """Sharded mode without the overlapped update (CPU / gloo), after the local
        update: every rank's fresh slice of the compute weights to every rank."""
        if not self.shard or self.update_fn is not None:
            return
        a = self.arena
        sh = a.wb if a.wb is not None else a.w
        works = []
        for b in self.buckets:
            lo, hi = b.own(self.rank, self.world)
            src = sh[lo:hi]
            if not self.inplace:
                b.agin.copy_(src)
                src = b.agin
            works.append(dist.all_gather_into_tensor(sh[b.start:b.end], src, group=self.group, async_op=True))
        for w in works:
            w.wait()

    def sync_master(self, opt_state: bool = False):
        """Sharded mode: gather the fp32 master weights (for save / get_weight) and, with
        opt_state, the optimizer state (momentum, Adam's second moment) -- each rank updates
        only its owned slices of them.  A COLLECTIVE: every rank must call it (the CLI does
        so before rank 0 serialises the model)."""
        self.sync()
        if not self.shard:
            return
        a = self.arena
        tensors = []
        if a.wb is not None:  # without a shadow the compute weights ARE the masters: gathered every step
            tensors.append(a.w)
        if opt_state:
            tensors.append(a.m1)
            if a.m2 is not None:
                tensors.append(a.m2)
        for t in tensors:
            for b in self.buckets:
                lo, hi = b.own(self.rank, self.world)
                src = t[lo:hi].clone()
                dist.all_gather_into_tensor(t[b.start:b.end], src, group=self.group)

    def check_consistency(self) -> float:
        """Max |w - w_rank0| over the compute weights of every replica (the
        reference's test_on_server check, async_updater-inl.hpp:50-52,148-153).
        Raises if the replicas diverged."""
        self.sync()
        if not self.active:
            return 0.0
        a = self.arena
        sh = a.wb if a.wb is not None else a.w
        ref = sh.clone()
        dist.broadcast(ref, src=0, group=self.group)
        diff = (sh.float() - ref.float()).abs().max().reshape(1)
        dist.all_reduce(diff, op=dist.ReduceOp.MAX, group=self.group)
        d = float(diff.item())
        if d != 0.0:
            raise RuntimeError(f"data-parallel replicas diverged: max |w - w_rank0| = {d:g}")
        return d

    def allreduce_tensor(self, t: torch.Tensor):
        if self.active:
            dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group)
        return t


def init_distributed(backend: Optional[str] = None):
    """Initialise torch.distributed from the torchrun environment (RANK/WORLD_SIZE/...).
    CXXNET_DIST_FORCE=1 initialises a process group even for a single rank (so the RCCL
    code path can run on one GPU)."""
    if not dist.is_available() or dist.is_initialized():
        return world_info()
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    force = os.environ.get("CXXNET_DIST_FORCE", "0") == "1"
    if ws <= 1 and not force:
        return 0, 1
    if backend is None:
        backend = os.environ.get("CXXNET_DIST_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    if ws <= 1:
        if "MASTER_PORT" not in os.environ:  # a free local port: a fixed one collides across jobs
            import socket
            with socket.socket() as s:
                s.bind(("127.0.0.1", 0))
                os.environ["MASTER_PORT"] = str(s.getsockname()[1])
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("WORLD_SIZE", "1")
    kw = {}
    if backend == "nccl" and torch.cuda.is_available():
        # one process per GPU; bind the communicator to it eagerly
        dev = torch.device("cuda", int(os.environ.get("LOCAL_RANK", "0")) % torch.cuda.device_count())
        torch.cuda.set_device(dev)
        kw["device_id"] = dev
    elif torch.cuda.is_available():
        # rehearsing N ranks on one card with the gloo backend: ranks share devices round-robin
        torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")) % torch.cuda.device_count())
    dist.init_process_group(backend=backend, **kw)
    return world_info()
