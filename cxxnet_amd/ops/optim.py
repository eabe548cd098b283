"""Fused optimizer step over the flat parameter arena (csrc/kernels/optim_kernels.hip).

CPU path reproduces the same formulas in fp32 torch.
"""
from __future__ import annotations

import ctypes
from typing import List, Sequence

import torch

from .. import native
from .gemm import _stream

ALGO = {"sgd": 0, "nag": 1, "adam": 2}


def fused_update(algo: str, w: torch.Tensor, g: torch.Tensor, st1: torch.Tensor, st2, wb,
                 segs: Sequence[tuple], d1: float = 0.1, d2: float = 0.001, zero_grad: bool = True):
    """Apply one optimizer step to every segment.

    segs: [(offset, n, lr, wd, mom, clip), ...] element ranges of the flat buffers.
    The gradient range is zeroed afterwards; wb (bf16 shadow) is refreshed when given.
    """
    a = ALGO[algo]
    if not w.is_cuda:
        for off, n, lr, wd, mom, clip in segs:
            ws, gs, ms = w[off:off + n], g[off:off + n], st1[off:off + n]
            gv = gs.clone()
            if clip != 0.0 and a == 0:  # SGD only (reference sgd_updater-inl.hpp:77-81)
                gv = torch.nan_to_num(gv, nan=0.0).clamp(-clip, clip)
            if a == 0:
                ms.mul_(mom).add_(-lr * (gv + wd * ws))
                ws.add_(ms)
            elif a == 1:
                old = ms.clone()
                ms.mul_(mom).add_(-lr * (gv + wd * ws))
                ws.add_((1 + mom) * ms - mom * old)
            else:
                if wd > 0:
                    gv = gv - wd * ws
                m2 = st2[off:off + n]
                ms.add_(d1 * (gv - ms))
                m2.add_(d2 * (gv * gv - m2))
                ws.sub_(lr * (ms / (m2.sqrt() + 1e-8)))
            if zero_grad:
                gs.zero_()
            if wb is not None:
                wb[off:off + n].copy_(ws)
        return
    nseg = len(segs)
    offs = (ctypes.c_long * nseg)(*[int(s[0]) for s in segs])
    ns = (ctypes.c_long * nseg)(*[int(s[1]) for s in segs])
    hyper = (ctypes.c_float * (4 * nseg))(*[float(v) for s in segs for v in s[2:6]])
    rc = native.kernels().cxn_fused_update(
        ctypes.cast(offs, ctypes.c_void_p), ctypes.cast(ns, ctypes.c_void_p), ctypes.cast(hyper, ctypes.c_void_p),
        nseg, w.data_ptr(), g.data_ptr(), st1.data_ptr(), st2.data_ptr() if st2 is not None else None,
        wb.data_ptr() if wb is not None else None, a | (16 if zero_grad else 0), float(d1), float(d2), _stream())
    native.check(rc, "fused_update")


def nonfinite(g: torch.Tensor, flag: torch.Tensor):
    """flag (int32[1]) |= any(!isfinite(g))."""
    if not g.is_cuda:
        if not torch.isfinite(g).all():
            flag.fill_(1)
        return
    native.check(native.kernels().cxn_nonfinite_check(g.data_ptr(), g.numel(), flag.data_ptr(), _stream()),
                 "nonfinite")


def scale_(x: torch.Tensor, s: float):
    if not x.is_cuda:
        x.mul_(s)
        return
    native.check(native.kernels().cxn_scale_f32(x.data_ptr(), x.numel(), float(s), _stream()), "scale")
