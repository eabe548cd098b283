"""Flat parameter arena.

Every trainable tensor of the net lives in ONE contiguous fp32 buffer (master
weights), with same-layout buffers for the gradient and optimizer state, plus a
bf16 compute shadow on the GPU.  One fused kernel then updates the whole model,
and data-parallel gradient reduction works on large contiguous ranges (buckets)
instead of per-tensor messages (contrast the reference's per-key push/pull,
src/updater/async_updater-inl.hpp:94-127).

Segments are laid out in REVERSE layer order, so the gradients that backward
produces first (last layers) are at the front of the buffer: a bucket is ready as
soon as backward has passed its lowest layer.
"""
from __future__ import annotations

from typing import List, Sequence

import os

import torch

ALIGN = 64  # elements; keeps every view 256-B aligned in fp32 and 128-B in bf16


class ParamArena:
    def __init__(self, device: torch.device, shadow_dtype=None):
        self.device = torch.device(device)
        self.shadow_dtype = shadow_dtype
        self.specs = []          # (layer_index, ParamSpec)
        self.total = 0
        self.w = self.g = self.m1 = self.m2 = self.wb = None

    def build(self, layer_specs: Sequence[tuple], groups: Sequence[Sequence[int]] = ()):
        """layer_specs: [(layer_index, [ParamSpec, ...]), ...] in forward order.

        groups: layer-index lists (forward order) whose weights must be ONE matrix and whose
        biases one vector (sibling convs computed as one GEMM, NeuralNet._fuse_siblings): the
        group is laid out at its first layer's place, weights back to back in the listed order,
        then the biases, 8-element aligned inside (ALIGN after).  Every member spec gets
        grad_li / fwd_li = the first layer: its gradient is final after that layer's backprop and
        that layer's forward reads it (data-parallel buckets and forward gating)."""
        from ..parallel.dp import world_info
        # a multiple of world*ALIGN, so that sharded buckets split into equal,
        # aligned per-rank chunks (parallel/dp.py, update_on_server); a segment whose gradient
        # is not reduced (fullc_gather) starts and ends on such a boundary, so the reduced runs
        # between them split evenly too
        q = ALIGN * world_info()[1]
        off = 0
        self.specs = []
        by_li = dict(layer_specs)
        lead_of = {li: g[0] for g in groups for li in g}
        group_of = {g[0]: list(g) for g in groups}
        for li, specs in sorted(layer_specs, key=lambda t: -t[0]):
            if li in lead_of and lead_of[li] != li:
                continue  # laid out with its group's first layer
            if li in group_of:
                members = group_of[li]
                for kind in (0, 1):  # weights, then biases
                    for m in members:
                        ps = by_li[m]
                        if kind < len(ps):
                            s = ps[kind]
                            s.offset = off
                            s.grad_li = s.fwd_li = li
                            self.specs.append((m, s))
                            off += (s.numel + 7) // 8 * 8
                off = (off + ALIGN - 1) // ALIGN * ALIGN
                continue
            for s in specs:
                nr = getattr(s, "no_reduce", False)
                if nr:
                    off = (off + q - 1) // q * q
                s.offset = off
                self.specs.append((li, s))
                off += (s.numel + ALIGN - 1) // ALIGN * ALIGN
                if nr:
                    off = (off + q - 1) // q * q
        self.total = max((off + q - 1) // q * q, q)
        dev = self.device
        self.w = torch.zeros(self.total, dtype=torch.float32, device=dev)
        self.g = torch.zeros(self.total, dtype=torch.float32, device=dev)
        self.m1 = torch.zeros(self.total, dtype=torch.float32, device=dev)
        self.m2 = None
        self.wb = torch.zeros(self.total, dtype=self.shadow_dtype, device=dev) if self.shadow_dtype else None
        for _, s in self.specs:
            n = s.numel
            s.w = self.w[s.offset:s.offset + n].view(s.shape)
            s.g = self.g[s.offset:s.offset + n].view(s.shape)
            s.wb = self.wb[s.offset:s.offset + n].view(s.shape) if self.wb is not None else s.w

    def accumulate_ranges(self):
        """Merged [start, end) arena ranges whose gradients are ACCUMULATED (atomics /
        +=) and so must be zero at the start of an update cycle."""
        if getattr(self, "_acc_ranges", None) is None:
            rs = sorted((s.offset, s.offset + s.numel) for _, s in self.specs if not s.overwrite)
            merged = []
            for a, b in rs:
                # segments are ALIGN-padded: bridge gaps between neighbours
                if merged and a - merged[-1][1] < ALIGN:
                    merged[-1][1] = max(merged[-1][1], b)
                else:
                    merged.append([a, b])
            self._acc_ranges = [tuple(r) for r in merged]
        return self._acc_ranges

    def zero_accumulated_grads(self):
        from .. import ops  # a library memset: launch lists record it (a torch zero_ they would not)
        torch_zero = os.environ.get("CXXNET_ZERO_TORCH", "0") == "1"  # diagnostics
        rs = self.accumulate_ranges()
        if not torch_zero and ops.zero_ranges(self.g, rs):  # every range in one launch
            return
        for a, b in rs:
            if torch_zero:
                self.g[a:b].zero_()
            else:
                ops.zero_(self.g[a:b])

    def ensure_second_moment(self):
        if self.m2 is None:
            self.m2 = torch.zeros_like(self.w)

    def sync_shadow(self):
        """Refresh the bf16 compute copy from the fp32 masters."""
        if self.wb is not None:
            self.wb.copy_(self.w)

    def zero_grad(self):
        self.g.zero_()

    def reset_state(self):
        self.m1.zero_()
        if self.m2 is not None:
            self.m2.zero_()

    def segments(self):
        return [(li, s) for li, s in self.specs]

    def used_range(self, li_min: int) -> int:
        """Arena prefix length covering every segment with layer index >= li_min."""
        end = 0
        for li, s in self.specs:
            if li >= li_min:
                end = max(end, s.offset + s.numel)
        return end
