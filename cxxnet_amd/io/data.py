"""DataBatch and the iterator interface (reference src/io/data.h:18-186)."""
from __future__ import annotations

import os
import threading
from dataclasses import dataclass, field
from typing import List, Optional

import numpy as np
import torch

# Held by HIP graph capture (nnet/trainer.py) and by every input prefetch: a global-mode capture
# forbids allocations on other threads (pinned host buffers, the prefetch's device copies), so the
# image iterator builds a whole batch under it.
DEVICE_IO_LOCK = threading.RLock()
_copy_streams = {}


def input_device() -> torch.device:
    """The GPU this process trains on (one process per GPU: LOCAL_RANK, parallel/dp.py)."""
    return torch.device("cuda", int(os.environ.get("LOCAL_RANK", "0")) % max(torch.cuda.device_count(), 1))


class DevicePrefetch:
    """A batch's host-to-device copies issued early, from the iterator's thread, on a side
    stream: with a thread buffer they overlap the previous training step instead of opening
    the next one (40+ MB per AlexNet batch, about 1 ms of PCIe).  Sources should be pinned
    (asynchronous DMA).  ``take`` orders the current stream after the copies."""

    def __init__(self, tensors, dev: torch.device, lo: int = 0):
        self.dev = dev
        self.lo = lo  # first batch row the copied tensors hold
        with DEVICE_IO_LOCK:
            s = _copy_streams.get(dev.index)
            if s is None:
                s = _copy_streams[dev.index] = torch.cuda.Stream(dev)
            with torch.cuda.device(dev), torch.cuda.stream(s):
                self.tensors = [t.to(dev, non_blocking=True) for t in tensors]
                self.event = torch.cuda.Event()
                self.event.record(s)

    def take(self, dev) -> Optional[list]:
        if torch.device(dev) != self.dev:
            return None
        cur = torch.cuda.current_stream(self.dev)
        cur.wait_event(self.event)
        for t in self.tensors:
            t.record_stream(cur)  # made on the copy stream, consumed on this one
        return self.tensors


class U8Images:
    """A batch of decoded images still in uint8, with the augmenter's arithmetic
    pending.  The image iterators emit this instead of a float tensor so that only
    uint8 pixels cross PCIe; ``ops.image_to_nhwc`` applies mean/contrast/
    illumination/scale and the NHWC-bf16 conversion in one GPU kernel, and
    ``to_float`` is the fp32 reference of the same arithmetic (the CPU path).

    pix  uint8 (B, h, w, C): pixels after crop and mirror (RGB order)
    prm  int32 (B, 4): crop_y, crop_x, mirrored, 0 (for full-size mean images)
    cm   float32 (B, 2): contrast, illumination
    mean None | float32 (C,) | (C, Hm, Wm) full-size | (C, h, w) crop-size
    mode 0 none, 1 per-channel value, 2 full-size mean image, 3 crop-size mean image
    Reference: src/io/iter_augment_proc-inl.hpp:98-162.
    """

    def __init__(self, pix, prm, cm, mean=None, mode=0, scale=1.0, pf=None, rows=None):
        self.pix, self.prm, self.cm, self.mean, self.mode, self.scale = pix, prm, cm, mean, mode, float(scale)
        self.pf, self.rows = pf, rows  # DevicePrefetch of (pix, prm, cm) and the rows of it this view is

    def prefetch(self, dev: torch.device, lo: int = 0, hi: Optional[int] = None):
        """Copy rows [lo, hi) to `dev` ahead of the step (a data-parallel rank decodes and trains
        only its own rows; the rest of the batch is never read on this rank)."""
        hi = self.pix.shape[0] if hi is None else hi
        self.pf = DevicePrefetch([self.pix[lo:hi], self.prm[lo:hi], self.cm[lo:hi]], dev, lo)
        self.rows = (0, self.pix.shape[0])

    def on_device(self, dev):
        """(pix, prm, cm) on `dev` from the prefetch, or None (also when this view reaches
        rows the prefetch did not copy)."""
        if self.pf is None:
            return None
        r0, r1 = self.rows[0] - self.pf.lo, self.rows[1] - self.pf.lo
        if r0 < 0 or r1 > self.pf.tensors[0].shape[0]:
            return None
        got = self.pf.take(dev)
        return None if got is None else [t[r0:r1] for t in got]

    @property
    def shape(self):
        B, h, w, C = self.pix.shape
        return (B, C, h, w)

    def __getitem__(self, sl):
        if not isinstance(sl, slice):
            raise TypeError("U8Images supports row slices only")
        rows = None
        if self.pf is not None:
            lo, hi, step = sl.indices(self.rows[1] - self.rows[0])
            rows = (self.rows[0] + lo, self.rows[0] + max(hi, lo)) if step == 1 else None
        return U8Images(self.pix[sl], self.prm[sl], self.cm[sl], self.mean, self.mode, self.scale,
                        self.pf if rows is not None else None, rows)

    def clone(self):
        return U8Images(self.pix.clone(), self.prm.clone(), self.cm.clone(), self.mean, self.mode, self.scale,
                        self.pf, self.rows)

    def to_float(self) -> torch.Tensor:
        """fp32 NCHW batch (reference arithmetic, CPU)."""
        d = self.pix.permute(0, 3, 1, 2).float()
        if self.mode == 0:
            return d * self.scale
        B, C, h, w = d.shape
        ct = self.cm[:, 0].view(B, 1, 1, 1).float()
        il = self.cm[:, 1].view(B, 1, 1, 1).float()
        mean = self.mean.float()
        if self.mode == 1:
            m = mean.view(1, C, 1, 1)
        elif self.mode == 3:
            m = mean.view(1, C, h, w)
        else:
            rows = []
            for b in range(B):
                y0, x0, mir = (int(v) for v in self.prm[b, :3])
                mb = mean[:, y0:y0 + h, x0:x0 + w]
                rows.append(mb.flip(2) if mir else mb)
            m = torch.stack(rows)
        return ((d - m) * ct + il) * self.scale


def dense(data) -> torch.Tensor:
    """Float NCHW view of a batch's data whatever its storage."""
    return data.to_float() if hasattr(data, "to_float") else data  # U8Images, io.jpeg_stage.JpegCoefImages


@dataclass
class DataBatch:
    """One mini-batch: data (b,c,h,w) float32, label (b, label_width) float32,
    inst_index (b,) uint32, num_batch_padd = padded tail rows, extra_data list."""
    data: torch.Tensor
    label: torch.Tensor
    inst_index: Optional[np.ndarray] = None
    num_batch_padd: int = 0
    extra_data: List[torch.Tensor] = field(default_factory=list)

    @property
    def batch_size(self):
        return int(self.data.shape[0])


class DataIterator:
    """IIterator<DataBatch>: set_param -> init -> (before_first, next/value)*."""

    def set_param(self, name: str, val: str):
        pass

    def init(self):
        pass

    def before_first(self):
        raise NotImplementedError

    def next(self) -> bool:
        raise NotImplementedError

    def value(self) -> DataBatch:
        raise NotImplementedError

    def __iter__(self):
        self.before_first()
        while self.next():
            yield self.value()

    def close(self):
        pass
