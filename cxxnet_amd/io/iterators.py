"""Data iterators and the `iter = ...` chain factory.

Reference: src/io/data.cpp:23-75 (CreateIterator), iter_mnist-inl.hpp,
iter_batch_proc-inl.hpp (BatchAdaptIterator, ThreadBufferIterator),
iter_mem_buffer-inl.hpp, iter_attach_txt-inl.hpp.
New: `iter = synthetic` -- random batches generated ON the device (zero host->device
traffic) for throughput benchmarks.
"""
from __future__ import annotations

import queue
import threading
import weakref
from typing import List, Optional, Tuple

import numpy as np
import torch

from .. import native
from .augment import on_exit
from .data import DataBatch, DataIterator


def _parse_shape(val: str) -> Tuple[int, int, int]:
    a = [int(x) for x in val.split(",")]
    if len(a) != 3:
        raise ValueError("input_shape must be three consecutive integers without space example: 1,1,200")
    return a[0], a[1], a[2]


class MNISTIterator(DataIterator):
    """`iter = mnist` -- gz idx files, /256 scaling, optional shuffle, flat (B,1,1,784)
    or (B,1,28,28) with input_flat=0; drops the last partial batch."""

    def __init__(self):
        self.silent = 0
        self.batch_size = 100
        self.mode = 1
        self.shuffle = 0
        self.inst_offset = 0
        self.path_img = self.path_label = ""
        self.seed = 0

    def set_param(self, name, val):
        if name == "silent":
            self.silent = int(val)
        elif name == "batch_size":
            self.batch_size = int(val)
        elif name == "input_flat":
            self.mode = int(val)
        elif name == "shuffle":
            self.shuffle = int(val)
        elif name == "index_offset":
            self.inst_offset = int(val)
        elif name == "path_img":
            self.path_img = val
        elif name == "path_label":
            self.path_label = val
        elif name == "seed_data":
            self.seed = int(val)

    def init(self):
        imgs, labels = native.rt().load_mnist(self.path_img, self.path_label)
        n, r, c = imgs.shape
        inst = np.arange(n, dtype=np.uint32) + self.inst_offset
        if self.shuffle:
            rng = native.rt().Metric  # noqa: F841 (kept for symmetry; shuffle below uses rand_r stream)
            perm = _rand_r_shuffle(np.arange(n), self.seed)
            imgs, labels, inst = imgs[perm], labels[perm], inst[perm]
        self.imgs = imgs
        self.labels = labels
        self.inst = inst
        self.shape = (1, 1, r * c) if self.mode == 1 else (1, r, c)
        if not self.silent:
            print(f"MNISTIterator: load {n} images, shuffle={self.shuffle}, "
                  f"shape={self.batch_size},{','.join(map(str, self.shape))}")
        self.loc = 0

    def before_first(self):
        self.loc = 0

    def next(self):
        if self.loc + self.batch_size <= self.imgs.shape[0]:
            s = slice(self.loc, self.loc + self.batch_size)
            data = torch.from_numpy(self.imgs[s]).view(self.batch_size, *self.shape)
            label = torch.from_numpy(self.labels[s]).view(-1, 1)
            self.out = DataBatch(data, label, self.inst[s])
            self.loc += self.batch_size
            return True
        return False

    def value(self):
        return self.out


def _rand_r_shuffle(arr: np.ndarray, seed: int) -> np.ndarray:
    """Fisher-Yates with the reference's rand_r stream (src/utils/random.h)."""
    import ctypes
    libc = ctypes.CDLL(None)
    state = ctypes.c_uint(seed)
    out = arr.copy()
    for i in range(len(out) - 1, 0, -1):
        r = libc.rand_r(ctypes.byref(state))
        j = int(np.floor(r / (2147483647 + 1.0) * (i + 1)))
        out[i], out[j] = out[j], out[i]
    return out


class SyntheticIterator(DataIterator):
    """`iter = synthetic` -- fixed random batches resident on the target device.

    Keys: input_shape=c,h,w, batch_size, num_class (labels uniform in [0,num_class)),
    num_batch (batches per round, default 100), synthetic_device=gpu|cpu, label_width,
    synthetic_dtype=float32|uint8 (uint8: decoded-image batches normalised on the device).
    """

    def __init__(self):
        self.shape = (3, 227, 227)
        self.batch_size = 256
        self.num_class = 1000
        self.num_batch = 100
        self.device = "gpu"
        self.label_width = 1
        self.seed = 0

    def set_param(self, name, val):
        if name == "input_shape":
            self.shape = _parse_shape(val)
        elif name == "batch_size":
            self.batch_size = int(val)
        elif name == "num_class":
            self.num_class = int(val)
        elif name == "num_batch":
            self.num_batch = int(val)
        elif name == "synthetic_device":
            self.device = val
        elif name == "label_width":
            self.label_width = int(val)
        elif name == "seed_data":
            self.seed = int(val)
        elif name == "synthetic_dtype":
            self.dtype = val

    def init(self):
        dev = torch.device("cuda") if (self.device == "gpu" and torch.cuda.is_available()) else torch.device("cpu")
        g = torch.Generator(device="cpu").manual_seed(self.seed)
        if getattr(self, "dtype", "float32") in ("uint8", "u8"):
            # decoded-image form: uint8 HWC, normalised on the device by the augment kernel
            from .data import U8Images
            c, h, w = self.shape
            B = self.batch_size
            pix = torch.randint(0, 256, (B, h, w, c), generator=g, dtype=torch.uint8)
            data = U8Images(pix.to(dev), torch.zeros((B, 4), dtype=torch.int32, device=dev),
                            torch.tensor([[1.0, 0.0]] * B, device=dev), torch.full((c,), 127.5, device=dev), 1,
                            1.0 / 64)
            label = torch.randint(0, self.num_class, (B, self.label_width), generator=g).float()
            self.batch = DataBatch(data, label.to(dev), np.arange(B, dtype=np.uint32))
            self.i = 0
            return
        data = torch.randn((self.batch_size,) + tuple(self.shape), generator=g)
        label = torch.randint(0, self.num_class, (self.batch_size, self.label_width), generator=g).float()
        self.batch = DataBatch(data.to(dev), label.to(dev), np.arange(self.batch_size, dtype=np.uint32))
        self.i = 0

    def before_first(self):
        self.i = 0

    def next(self):
        if self.i < self.num_batch:
            self.i += 1
            return True
        return False

    def value(self):
        return self.batch


_LIVE_BUFFERS: "weakref.WeakSet" = weakref.WeakSet()


@on_exit
def _stop_live_buffers():
    """Join prefetch threads before the interpreter finalizes: a daemon thread that is
    inside a native call (the page reader) when Python tears down is killed while
    unwinding through C++ frames, which aborts the process."""
    for it in list(_LIVE_BUFFERS):
        it._stop()


class ThreadBufferIterator(DataIterator):
    """`iter = threadbuffer` -- background prefetch of whole batches (reference
    ThreadBufferIterator, iter_batch_proc-inl.hpp:136-224; buffer_size default 2)."""

    def __init__(self, base: DataIterator):
        self.base = base
        self.buffer_size = 2
        self.thread = None

    def set_param(self, name, val):
        self.base.set_param(name, val)
        if name == "buffer_size":
            self.buffer_size = int(val)

    def init(self):
        self.base.init()

    def _run(self, q: "queue.Queue", stop: threading.Event):
        self.base.before_first()
        # a base that allocates every batch afresh (the image iterators, whose pixels
        # sit in page-locked memory) is handed over as is; others reuse their buffers
        fresh = getattr(self.base, "fresh_batches", False)
        while not stop.is_set():
            b = self.base.value() if self.base.next() else None
            if b is not None and not fresh:
                b = DataBatch(b.data.clone(), b.label.clone(), None if b.inst_index is None else b.inst_index.copy(),
                              b.num_batch_padd, [e.clone() for e in b.extra_data])
            while not stop.is_set():
                try:
                    q.put(b, timeout=0.1)
                    break
                except queue.Full:
                    continue
            if b is None:
                return

    def _stop(self):
        if self.thread is not None:
            self.stop.set()
            try:
                while True:
                    self.q.get_nowait()
            except queue.Empty:
                pass
            self.thread.join()
            self.thread = None

    def before_first(self):
        self._stop()
        _LIVE_BUFFERS.add(self)
        self.q = queue.Queue(maxsize=self.buffer_size)
        self.stop = threading.Event()
        self.thread = threading.Thread(target=self._run, args=(self.q, self.stop), daemon=True)
        self.thread.start()

    def next(self):
        if self.thread is None:
            self.before_first()
        b = self.q.get()
        if b is None:
            self.thread.join()
            self.thread = None
            return False
        self.out = b
        return True

    def value(self):
        return self.out

    def close(self):
        self._stop()
        self.base.close()


class DenseBufferIterator(DataIterator):
    """`iter = membuffer` -- caches the first max_nbatch (100) batches in RAM."""

    def __init__(self, base):
        self.base = base
        self.max_nbatch = 100
        self.silent = 0

    def set_param(self, name, val):
        self.base.set_param(name, val)
        if name == "max_nbatch":
            self.max_nbatch = int(val)
        elif name == "silent":
            self.silent = int(val)

    def init(self):
        self.base.init()
        self.buf = []
        self.base.before_first()
        while len(self.buf) < self.max_nbatch and self.base.next():
            b = self.base.value()
            self.buf.append(DataBatch(b.data.clone(), b.label.clone(),
                                      None if b.inst_index is None else b.inst_index.copy(), b.num_batch_padd,
                                      [e.clone() for e in b.extra_data]))
        if not self.silent:
            print(f"DenseBufferIterator: load {len(self.buf)} batches")
        self.i = 0

    def before_first(self):
        self.i = 0

    def next(self):
        if self.i < len(self.buf):
            self.out = self.buf[self.i]
            self.i += 1
            return True
        return False

    def value(self):
        return self.out


class AttachTxtIterator(DataIterator):
    """`iter = attachtxt` -- adds an extra dense input read from a text file keyed by
    instance index (reference iter_attach_txt-inl.hpp:15-99).  File: `nrow ncol` header
    then rows `index v1 ... vncol`."""

    def __init__(self, base):
        self.base = base
        self.filename = ""
        self.shape = None

    def set_param(self, name, val):
        self.base.set_param(name, val)
        if name == "filename":
            self.filename = val
        elif name == "extra_data_shape[0]":
            self.shape = _parse_shape(val)

    def init(self):
        self.base.init()
        with open(self.filename) as f:
            toks = f.read().split()
        nrow, ncol = int(toks[0]), int(toks[1])
        self.table = {}
        p = 2
        for _ in range(nrow):
            idx = int(toks[p])
            self.table[idx] = np.array([float(x) for x in toks[p + 1:p + 1 + ncol]], dtype=np.float32)
            p += 1 + ncol
        self.ncol = ncol

    def before_first(self):
        self.base.before_first()

    def next(self):
        if not self.base.next():
            return False
        b = self.base.value()
        rows = np.stack([self.table.get(int(i), np.zeros(self.ncol, np.float32)) for i in b.inst_index])
        shape = self.shape or (1, 1, self.ncol)
        extra = torch.from_numpy(rows).view(len(rows), *shape)
        self.out = DataBatch(b.data, b.label, b.inst_index, b.num_batch_padd, list(b.extra_data) + [extra])
        return True

    def value(self):
        return self.out


def create_iterator(cfg: List[Tuple[str, str]]) -> DataIterator:
    """Build an iterator chain from the pairs between `iter = <type>` and `iter = end`."""
    it: Optional[DataIterator] = None
    for name, val in cfg:
        if name == "iter":
            if val == "end":
                break
            if val == "mnist":
                if it is not None:
                    raise ValueError("mnist can not chain over other iterator")
                it = MNISTIterator()
                continue
            if val == "synthetic":
                if it is not None:
                    raise ValueError("synthetic can not chain over other iterator")
                it = SyntheticIterator()
                continue
            if val in ("imgbin", "imgbinx", "img"):
                if it is not None:
                    raise ValueError("image iterator can not chain over other iterator")
                from .image import create_image_iterator
                it = create_image_iterator(val)
                continue
            if val == "threadbuffer":
                if it is None:
                    raise ValueError("must specify input of threadbuffer")
                it = ThreadBufferIterator(it)
                continue
            if val == "membuffer":
                if it is None:
                    raise ValueError("must specify input of memory buffer")
                it = DenseBufferIterator(it)
                continue
            if val == "attachtxt":
                if it is None:
                    raise ValueError("must specify input of attach txt buffer")
                it = AttachTxtIterator(it)
                continue
            raise ValueError(f"unknown iterator type {val}")
        if it is not None:
            it.set_param(name, val)
    if it is None:
        raise ValueError("must specify iterator by iter=itername")
    return it
