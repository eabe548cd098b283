"""Updaters: SGD (momentum), NAG, Adam with the reference's learning-rate and
momentum schedules and tag-scoped hyper-parameters.

Reference: src/updater/param.h (UpdaterParam, ScheduleEpoch 76-95, SetParam 101-133),
src/updater/sgd_updater-inl.hpp, nag_updater-inl.hpp, adam_updater-inl.hpp,
src/updater/updater_impl-inl.hpp (one updater per (layer, tag)).

The math runs in ONE fused kernel over the whole parameter arena
(csrc/kernels/optim_kernels.hip); this module computes the per-segment scalars.
"""
from __future__ import annotations

import math
from typing import List, Sequence, Tuple

from .. import ops


class UpdaterParam:
    """Mirror of reference UpdaterParam with identical defaults and key handling."""

    def __init__(self, tag: str):
        self.tag = tag
        self.round = 0
        self.silent = 0
        self.base_lr = 0.01
        self.learning_rate = 0.01
        self.wd = 0.0
        self.momentum = 0.9
        self.lr_schedule = 0
        self.momentum_schedule = 0
        self.lr_step = 1
        self.lr_gamma = 0.5
        self.lr_alpha = 0.5
        self.lr_factor = 0.1
        self.lr_minimum = 0.00001
        self.start_epoch = 0
        self.base_momentum = 0.5
        self.final_momentum = 0.90
        self.saturation_epoch = 0
        self.clip_gradient = 0.0

    def set_param(self, name: str, val: str):
        t = self.tag
        if name.startswith(t) and len(name) > len(t) and name[len(t)] == ":":
            name = name[len(t) + 1:]
        if name in ("lr", "eta"):
            self.base_lr = float(val)
        elif name == "wd":
            self.wd = float(val)
        elif name == "momentum":
            self.momentum = float(val)
        elif name == "silent":
            self.silent = int(val)
        elif name == "momentum_schedule":
            self.momentum_schedule = int(val)
        elif name == "clip_gradient":
            self.clip_gradient = float(val)
        elif name == "final_momentum":
            self.final_momentum = float(val)
        elif name == "base_momentum":
            self.base_momentum = float(val)
        elif name == "saturation_epoch":
            self.saturation_epoch = int(val)
        if name.startswith("lr:") or name.startswith("eta:"):
            sub = name[3:] if name.startswith("lr:") else name[4:]
            if sub == "schedule":
                self.lr_schedule = {"constant": 0, "expdecay": 1, "polydecay": 2, "factor": 3}.get(val, self.lr_schedule)
            elif sub == "gamma":
                self.lr_gamma = float(val)
            elif sub == "alpha":
                self.lr_alpha = float(val)
            elif sub == "step":
                self.lr_step = int(val)
            elif sub == "factor":
                self.lr_factor = float(val)
            elif sub == "minimum_lr":
                self.lr_minimum = float(val)
            elif sub == "start_epoch":
                self.start_epoch = int(val)

    def schedule_epoch(self, epoch: int):
        """Reference ScheduleEpoch (src/updater/param.h:76-95), including its quirks."""
        s = self.lr_schedule
        if s == 0:
            lr = self.base_lr
        elif s == 1:
            lr = self.base_lr * math.pow(self.lr_gamma, float(epoch) / self.lr_step)
        elif s == 2:
            lr = self.base_lr * math.pow(1.0 + (epoch // self.lr_step) * self.lr_gamma, -self.lr_alpha)
        elif s == 3:
            lr = self.base_lr * math.pow(self.lr_factor, epoch // self.lr_step)
        else:
            raise ValueError("unknown schedule type")
        if self.momentum_schedule and self.saturation_epoch:
            self.momentum += (self.final_momentum - self.base_momentum) / self.saturation_epoch * epoch + \
                self.base_momentum
        self.momentum = min(self.momentum, self.final_momentum)
        lr = max(lr, self.lr_minimum)
        if epoch < self.start_epoch:
            lr = self.base_lr
        self.learning_rate = lr


class ArenaUpdater:
    """All updaters of a net, applied by one fused kernel launch per step."""

    def __init__(self, algo: str, arena, segments: Sequence[Tuple[int, object]], defcfg, layercfg):
        if algo not in ("sgd", "nag", "adam"):
            raise ValueError(f"unknown updater type {algo}")
        self.algo = algo
        self.arena = arena
        self.entries = []  # (ParamSpec, UpdaterParam)
        # arena offsets whose SGD step already ran this step inside the fc weight-gradient
        # GEMM (ops.fc_backward_weight_sgd); update() skips them (every call of the step: the
        # overlapped update calls it once per bucket); the trainer clears the set per step
        self.fused_offsets = set()
        self.beta1 = 0.1
        self.beta2 = 0.001
        for li, spec in segments:
            p = UpdaterParam(spec.tag)
            for k, v in defcfg:
                p.set_param(k, v)
                self._adam_key(k, v)
            for k, v in layercfg[li]:
                p.set_param(k, v)
            self.entries.append((spec, p))
        if algo == "adam":
            arena.ensure_second_moment()

    def _adam_key(self, k, v):
        if k == "beta1":
            self.beta1 = float(v)
        elif k == "beta2":
            self.beta2 = float(v)

    def start_round(self, r: int):
        for _, p in self.entries:
            p.round = r

    def segments(self, epoch: int) -> List[tuple]:
        segs = []
        for spec, p in self.entries:
            if self.algo == "adam":
                fix1 = 1.0 - math.pow(1.0 - self.beta1, epoch + 1)
                fix2 = 1.0 - math.pow(1.0 - self.beta2, epoch + 1)
                lr = p.base_lr * math.sqrt(fix2) / fix1
                segs.append((spec.offset, spec.numel, lr, p.wd, 0.0, p.clip_gradient))
            else:
                p.schedule_epoch(epoch)
                segs.append((spec.offset, spec.numel, p.learning_rate, p.wd, p.momentum, p.clip_gradient))
        return segs

    def hyper(self, spec, epoch: int):
        """(lr, wd, momentum, clip) of `spec` for this epoch's update (the same cached
        schedule values update() uses)."""
        if getattr(self, "_seg_epoch", None) != epoch:
            self._segs = self.segments(epoch)
            self._seg_epoch = epoch
        for off, _, lr, wd, mom, clip in self._segs:
            if off == spec.offset:
                return lr, wd, mom, clip
        raise KeyError(f"no updater segment at arena offset {spec.offset}")

    def stage_hyper(self, epoch: int):
        """Refresh the device table of every entry's (lr, wd, momentum, clip) for this epoch's
        update: the fused fc steps of a recorded launch list / captured graph read their
        schedule values from it (ops.fc_backward_weight_sgd hyp), one host-to-device copy per
        step."""
        import torch
        if getattr(self, "_hyp_dev", None) is None:
            dev = self.arena.w.device
            pin = dev.type == "cuda"
            # a ring of pinned sources: slot k is rewritten only after the copy that read it
            # (event), so staging never waits on the GPU unless the host runs 16 steps ahead
            self._hyp_host = [torch.zeros((len(self.entries), 4), dtype=torch.float32, pin_memory=pin)
                              for _ in range(16)]
            self._hyp_ev = [None] * 16
            self._hyp_slot = 0
            self._hyp_dev = torch.zeros((len(self.entries), 4), dtype=torch.float32, device=dev)
            self._hyp_row = {spec.offset: i for i, (spec, _) in enumerate(self.entries)}
        if getattr(self, "_seg_epoch", None) != epoch:
            self._segs = self.segments(epoch)
            self._seg_epoch = epoch
        if getattr(self, "_hyp_epoch", None) == epoch:
            return
        k = self._hyp_slot = (self._hyp_slot + 1) % len(self._hyp_host)
        if self._hyp_ev[k] is not None:
            self._hyp_ev[k].synchronize()
        host = self._hyp_host[k]
        host.copy_(torch.tensor([seg[2:6] for seg in self._segs], dtype=torch.float32))
        self._hyp_dev.copy_(host, non_blocking=True)
        if self._hyp_dev.is_cuda:
            self._hyp_ev[k] = torch.cuda.Event()
            self._hyp_ev[k].record()
        self._hyp_epoch = epoch

    def hyper_dev(self, spec):
        """Device row (lr, wd, momentum, clip) of `spec` (stage_hyper fills it)."""
        return self._hyp_dev[self._hyp_row[spec.offset]]

    def update(self, epoch: int, ranges=None):
        """ranges: optional [start, end) arena ranges to update (sharded data
        parallelism updates only this rank's slice; the overlapped update calls this once
        per gradient bucket).  The schedules are evaluated ONCE per epoch, however many
        calls an update is split into: the momentum schedule accumulates on every
        ScheduleEpoch call (reference param.h:84-87), once per update."""
        a = self.arena
        if getattr(self, "_seg_epoch", None) != epoch:
            self._segs = self.segments(epoch)
            self._seg_epoch = epoch
        segs = self._segs
        if self.fused_offsets:  # cleared by the trainer at the start of each step
            segs = [sg for sg in segs if sg[0] not in self.fused_offsets]
        if ranges is not None:
            segs = _clip_segments(segs, ranges)
        # gradients are reset by the next cycle's first backprop (NeuralNet.backprop(first=True))
        ops.fused_update(self.algo, a.w, a.g, a.m1, a.m2, a.wb, segs, self.beta1, self.beta2, zero_grad=False)


def _clip_segments(segs, ranges):
    out = []
    for off, n, *hyper in segs:
        for lo, hi in ranges:
            a, b = max(off, lo), min(off + n, hi)
            if a < b:
                out.append((a, b - a, *hyper))
    return out
