"""Data parallelism: one process per GPU, RCCL all-reduce over xGMI.

Replaces the reference's mshadow-ps "local"/"dist" parameter server
(src/updater/async_updater-inl.hpp:94-127, src/nnet/nnet_impl-inl.hpp:376-390):
  * init: rank 0's weights are broadcast (reference serialises a model blob on
    device 0 and loads it on the others, nnet_impl-inl.hpp:70-81);
  * every step: the fp32 gradient arena is reduced (SUM -- the loss is already
    scaled by the global batch, loss_layer_base-inl.hpp:62) in BUCKETS.  The arena is
    laid out in reverse layer order, so bucket k only needs the layers above some
    index: its all-reduce is launched from the backprop hook the moment that layer
    finishes, and runs on RCCL's stream while backward continues on the compute
    stream (the reference's priority push/pull, priority = -layer);
  * the same fused optimizer then runs on every replica.
Bucket size defaults to 64 MB: AlexNet's 244 MB of gradients become 4-5 messages,
large enough to run at link rate on 7 xGMI links, small enough that the fc8/fc7
buckets overlap conv backward.
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
        self.work = None
        self.buf = None


class GradReducer:
    def __init__(self, arena, bucket_mb: float = 64.0, overlap: bool = True, comm_dtype: str = "fp32",
                 group=None):
        self.arena = arena
        self.group = group
        self.rank, self.world = world_info()
        self.overlap = overlap
        self.comm_dtype = torch.bfloat16 if comm_dtype == "bf16" else torch.float32
        limit = max(1, int(bucket_mb * (1 << 20) / 4))
        self.buckets: List[Bucket] = []
        cur_start, cur_end, cur_li = None, 0, None
        for li, spec in arena.specs:  # arena order = reverse layer order
            s, e = spec.offset, spec.offset + spec.numel
            if cur_start is None:
                cur_start, cur_li = s, li
            if e - cur_start > limit and cur_end > cur_start:
                self.buckets.append(Bucket(cur_start, cur_end, cur_li))
                cur_start = s
            cur_end = e
            cur_li = li
        if cur_start is not None and cur_end > cur_start:
            self.buckets.append(Bucket(cur_start, cur_end, cur_li))

    @property
    def active(self):
        return self.world > 1

    def broadcast_params(self, src: int = 0):
        if not self.active:
            return
        dist.broadcast(self.arena.w, src=src, group=self.group)
        self.arena.sync_shadow()

    def start_step(self):
        for b in self.buckets:
            b.work = None

    def _launch(self, b: Bucket):
        g = self.arena.g[b.start:b.end]
        if self.comm_dtype == torch.float32:
            b.buf = None
            b.work = dist.all_reduce(g, op=dist.ReduceOp.SUM, group=self.group, async_op=True)
        else:
            b.buf = g.to(self.comm_dtype)
            b.work = dist.all_reduce(b.buf, op=dist.ReduceOp.SUM, group=self.group, async_op=True)

    def hook(self, layer_index: int):
        """Called after each layer's backprop (reverse order)."""
        if not self.active or not self.overlap:
            return
        for b in self.buckets:
            if b.work is None and layer_index <= b.li_min:
                self._launch(b)

    def finish(self):
        """Launch what is left and make the compute stream wait for every reduction."""
        if not self.active:
            return
        for b in self.buckets:
            if b.work is None:
                self._launch(b)
        for b in self.buckets:
            b.work.wait()
            if b.buf is not None:
                self.arena.g[b.start:b.end].copy_(b.buf)
                b.buf = None
            b.work = None

    def allreduce_tensor(self, t: torch.Tensor):
        if self.active:
            dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group)
        return t


def init_distributed(backend: Optional[str] = None):
    """Initialise torch.distributed from the torchrun environment (RANK/WORLD_SIZE/...)."""
    if not dist.is_available() or dist.is_initialized():
        return world_info()
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    if ws <= 1:
        return 0, 1
    if backend is None:
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    if backend == "nccl":
        torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")))
    dist.init_process_group(backend=backend)
    return world_info()
