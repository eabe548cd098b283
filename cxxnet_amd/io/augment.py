"""Decode + augmentation of one image, and the decode worker processes.

This module imports only the standard library, numpy and Pillow: it is also the
program the decode workers run (``python -I augment.py``), so a worker starts in
~0.1 s with ~40 MB of memory instead of importing torch and the framework.

Reference: src/io/iter_augment_proc-inl.hpp:98-198 (crop / mirror / mean / contrast /
illumination) and src/io/image_augmenter-inl.hpp:74-161 (affine warp).

Why processes: Pillow's JPEG decoder releases the GIL, but everything around it
(Image.open, the array export, cropping, the RNG) does not.  On 8 host cores a thread
pool tops out at ~3.4k decodes/s while processes scale with cores (~7.6k/s at 8;
profiles/r2_io_throughput.md).  Workers are started with subprocess (never forked
from the trainer, which holds a GPU context, and never re-importing the user's main
script the way multiprocessing does); each writes its crops straight into a /dev/shm
batch buffer, so only encoded bytes go down the pipe and only crop parameters come
back.
"""
from __future__ import annotations

import atexit
import io as _io
import itertools
import math
import mmap
import os
import pickle
import subprocess
import sys
import threading
import traceback
import weakref
from typing import List, Optional, Tuple

import numpy as np


# ----------------------------------------------------------------------------- augmenter
class AugmentParam:
    """Every key of AugmentIterator::SetParam and ImageAugmenter::SetParam."""

    def __init__(self):
        self.shape = (3, 224, 224)
        self.rand_crop = 0
        self.rand_mirror = 0
        self.mirror = 0
        self.crop_y_start = -1
        self.crop_x_start = -1
        self.scale = 1.0
        self.image_mean = ""
        self.mean_value: Optional[Tuple[float, float, float]] = None
        self.max_random_contrast = 0.0
        self.max_random_illumination = 0.0
        self.max_rotate_angle = 0
        self.max_shear_ratio = 0.0
        self.max_aspect_ratio = 0.0
        self.min_crop_size = -1
        self.max_crop_size = -1
        self.min_random_scale = 1.0
        self.max_random_scale = 1.0
        self.min_img_size = 0.0
        self.max_img_size = 1e10
        self.fill_value = 255
        self.rotate = -1
        self.rotate_list: List[int] = []
        self.seed = 0
        self.silent = 0

    def set_param(self, name, val):
        if name == "input_shape":
            a = [int(x) for x in val.split(",")]
            if len(a) != 3:
                raise ValueError("input_shape must be three consecutive integers without space example: 1,1,200")
            self.shape = tuple(a)
        elif name == "seed_data":
            self.seed = int(val)
        elif name == "divideby":
            self.scale = 1.0 / float(val)
        elif name == "scale":
            self.scale = float(val)
        elif name == "mean_value":
            a = [float(x) for x in val.split(",")]
            if len(a) != 3:
                raise ValueError("mean value must be three consecutive float without space example: 128,127.5,128.2")
            self.mean_value = tuple(a)
        elif name == "image_mean":
            self.image_mean = val
        elif name == "rotate_list":
            self.rotate_list = [int(x) for x in val.split(",") if x]
        elif name in ("rand_crop", "rand_mirror", "mirror", "crop_y_start", "crop_x_start", "max_rotate_angle",
                      "min_crop_size", "max_crop_size", "fill_value", "rotate", "silent"):
            setattr(self, name, int(float(val)))
        elif name in ("max_random_contrast", "max_random_illumination", "max_shear_ratio", "max_aspect_ratio",
                      "min_random_scale", "max_random_scale", "min_img_size", "max_img_size"):
            setattr(self, name, float(val))

    def need_affine(self) -> bool:
        """ImageAugmenter::NeedProcess (image_augmenter-inl.hpp:156-161)."""
        if self.max_rotate_angle > 0 or self.max_shear_ratio > 0 or self.rotate > 0 or self.rotate_list:
            return True
        return self.min_crop_size > 0 and self.max_crop_size > 0


def _open(payload):
    """Decoded RGB Pillow image (JPEG/PNG/...; other modes converted to RGB)."""
    from PIL import Image
    im = Image.open(_io.BytesIO(payload) if isinstance(payload, (bytes, bytearray, memoryview)) else payload)
    if im.mode != "RGB":
        im = im.convert("RGB")
    return im


def _decode(payload) -> np.ndarray:
    return np.asarray(_open(payload))


def _affine(img: np.ndarray, p: AugmentParam, rng: np.random.Generator) -> np.ndarray:
    """Random rotate/shear/scale/aspect warp, then crop to the input shape
    (ImageAugmenter::Process, image_augmenter-inl.hpp:74-121)."""
    from PIL import Image
    H, W = img.shape[:2]
    s = rng.random() * p.max_shear_ratio * 2 - p.max_shear_ratio
    angle = int(rng.integers(p.max_rotate_angle * 2)) - p.max_rotate_angle if p.max_rotate_angle > 0 else 0
    if p.rotate > 0:
        angle = p.rotate
    if p.rotate_list:
        # the reference samples NextUInt32(size-1): the last entry is never drawn
        angle = p.rotate_list[int(rng.integers(len(p.rotate_list) - 1)) if len(p.rotate_list) > 1 else 0]
    a = math.cos(angle / 180.0 * math.pi)
    b = math.sin(angle / 180.0 * math.pi)
    scale = rng.random() * (p.max_random_scale - p.min_random_scale) + p.min_random_scale
    ratio = rng.random() * p.max_aspect_ratio * 2 - p.max_aspect_ratio + 1
    hs = 2 * scale / (1 + ratio)
    ws = ratio * hs
    new_w = int(max(p.min_img_size, min(p.max_img_size, scale * W)))
    new_h = int(max(p.min_img_size, min(p.max_img_size, scale * H)))
    m00, m01 = hs * a - s * b * ws, hs * b + s * a * ws
    m10, m11 = -b * ws, a * ws
    m02 = (new_w - (m00 * W + m01 * H)) / 2
    m12 = (new_h - (m10 * W + m11 * H)) / 2
    det = m00 * m11 - m01 * m10
    i00, i01, i10, i11 = m11 / det, -m01 / det, -m10 / det, m00 / det
    inv = (i00, i01, -(i00 * m02 + i01 * m12), i10, i11, -(i10 * m02 + i11 * m12))
    fill = (p.fill_value,) * 3
    out = Image.fromarray(img).transform((new_w, new_h), Image.AFFINE, inv, resample=Image.BICUBIC, fillcolor=fill)
    res = np.asarray(out)
    ch, cw = p.shape[1], p.shape[2]
    y, x = res.shape[0] - ch, res.shape[1] - cw
    if y < 0 or x < 0:
        raise ValueError("augmented image is smaller than input_shape")
    if p.rand_crop:
        y, x = int(rng.integers(y + 1)), int(rng.integers(x + 1))
    else:
        y, x = y // 2, x // 2
    return res[y:y + ch, x:x + cw]


def _augment_one(payload, p: AugmentParam, seed: int, mean_mode: int):
    """Decode + geometric augmentation of one instance.  Returns (pixels (h,w,C) uint8,
    (crop_y, crop_x, mirrored), (contrast, illumination))."""
    rng = np.random.Generator(np.random.PCG64(seed))
    img = _open(payload)
    if p.need_affine():
        img = _affine(np.asarray(img), p, rng)
    ch, cw = p.shape[1], p.shape[2]
    if ch == 1:  # flat input: no crop (reference: img_ = data * scale_)
        return np.asarray(img), (0, 0, 0), (1.0, 0.0)
    H, W = img.shape[:2] if isinstance(img, np.ndarray) else img.size[::-1]
    if H < ch or W < cw:
        raise ValueError("Data size must be bigger than the input size to net.")
    yy, xx = H - ch, W - cw
    if p.rand_crop and (yy or xx):
        yy, xx = int(rng.integers(yy + 1)), int(rng.integers(xx + 1))
    else:
        yy, xx = yy // 2, xx // 2
    if H != ch and p.crop_y_start != -1:
        yy = p.crop_y_start
    if W != cw and p.crop_x_start != -1:
        xx = p.crop_x_start
    contrast = rng.random() * p.max_random_contrast * 2 - p.max_random_contrast + 1
    illum = rng.random() * p.max_random_illumination * 2 - p.max_random_illumination
    if mean_mode == 0:
        mirror = bool(p.rand_mirror and rng.random() < 0.5)   # `mirror=1` is ignored here (reference)
        contrast, illum = 1.0, 0.0
    else:
        mirror = bool((p.rand_mirror and rng.random() < 0.5) or p.mirror == 1)
    if isinstance(img, np.ndarray):
        crop = img[yy:yy + ch, xx:xx + cw]
        if mirror:
            crop = crop[:, ::-1]
    else:
        # crop and mirror inside Pillow: only the crop is exported, already contiguous
        # (a negative-stride numpy view costs ~0.6 ms per 227x227 copy)
        from PIL import Image
        im = img.crop((xx, yy, xx + cw, yy + ch))
        if mirror:
            im = im.transpose(Image.Transpose.FLIP_LEFT_RIGHT)
        crop = np.asarray(im)
    return crop, (yy, xx, int(mirror)), (contrast, illum)


# ----------------------------------------------------------------------------- shared batch buffer
_SHM_SEQ = itertools.count()


class ShmBuffer:
    """A named /dev/shm file mapped into this process (the decode workers map it too)."""

    def __init__(self, nbytes: int):
        # never reused within a process: workers cache their mappings by name
        self.name = f"cxxnet_io_{os.getpid()}_{next(_SHM_SEQ)}_{os.urandom(4).hex()}"
        self.path = "/dev/shm/" + self.name
        fd = os.open(self.path, os.O_CREAT | os.O_EXCL | os.O_RDWR, 0o600)
        try:
            os.ftruncate(fd, nbytes)
            self.map = mmap.mmap(fd, nbytes)
        finally:
            os.close(fd)
        self.size = nbytes
        _LIVE_SHM.add(self)

    def array(self, shape) -> np.ndarray:
        return np.ndarray(shape, np.uint8, buffer=self.map)

    def close(self):
        if self.map is not None:
            try:
                self.map.close()
            except BufferError:  # a numpy view is still alive; the mapping goes with it
                pass
            self.map = None
            try:
                os.unlink(self.path)
            except FileNotFoundError:
                pass


def shm_available() -> bool:
    return os.path.isdir("/dev/shm") and os.access("/dev/shm", os.W_OK)


# ----------------------------------------------------------------------------- worker side
def _worker_main():
    import signal
    signal.signal(signal.SIGINT, signal.SIG_IGN)  # the parent handles Ctrl-C; we exit on EOF
    proto_in = sys.stdin.buffer
    proto_out = os.fdopen(os.dup(1), "wb")
    os.dup2(2, 1)  # stray prints go to stderr, never into the result stream
    maps = {}
    while True:
        try:
            task = pickle.load(proto_in)
        except EOFError:
            return
        name, shape, aug, mean_mode, items = task
        try:
            m = maps.get(name)
            if m is None:
                for k in list(maps)[:-3]:  # buffers of closed iterators
                    maps.pop(k).close()
                fd = os.open("/dev/shm/" + name, os.O_RDWR)
                try:
                    m = maps[name] = mmap.mmap(fd, 0)
                finally:
                    os.close(fd)
            p = AugmentParam.__new__(AugmentParam)
            p.__dict__.update(aug)
            B, h, w, C = shape
            out = np.ndarray((B, h, w, C), np.uint8, buffer=m)
            res = []
            for row, payload, seed in items:
                img, prm, cm = _augment_one(payload, p, seed, mean_mode)
                out[row] = img[..., :C]
                res.append((row, prm, cm))
            msg = ("ok", res)
        except Exception:  # noqa: BLE001 -- reported to the parent, which raises
            msg = ("err", traceback.format_exc())
        pickle.dump(msg, proto_out, protocol=pickle.HIGHEST_PROTOCOL)
        proto_out.flush()


# ----------------------------------------------------------------------------- parent side
class DecodePool:
    """`n` decode worker processes; one batch at a time (a lock serialises users)."""

    def __init__(self, n: int):
        self.n = n
        self.lock = threading.Lock()
        env = dict(os.environ, OMP_NUM_THREADS="1")
        self.procs = [subprocess.Popen([sys.executable, "-I", os.path.abspath(__file__)],
                                       stdin=subprocess.PIPE, stdout=subprocess.PIPE, env=env)
                      for _ in range(n)]
        _LIVE_POOLS.add(self)

    def imap(self, shm: ShmBuffer, shape, aug: AugmentParam, mean_mode: int, items: list):
        """Decode `items` = [(row, payload, seed)] into rows of `shm`.  Yields, chunk by
        chunk in order, (first index, end index into `items`, [(row, crop params,
        (contrast, illum))]) as soon as that chunk is in the buffer, so the caller can
        copy it out while later chunks are still being decoded."""
        if not items:
            return
        nchunk = min(len(items), 2 * self.n)
        step = (len(items) + nchunk - 1) // nchunk
        bounds = [(k, min(k + step, len(items))) for k in range(0, len(items), step)]
        augd = dict(vars(aug))
        with self.lock:
            sent = []
            try:
                for j, (lo, hi) in enumerate(bounds):
                    w = self.procs[j % self.n]
                    pickle.dump((shm.name, shape, augd, mean_mode, items[lo:hi]), w.stdin,
                                protocol=pickle.HIGHEST_PROTOCOL)
                    w.stdin.flush()
                    sent.append(w)
                err = None
                for j, w in enumerate(sent):  # each worker answers in FIFO order
                    try:
                        kind, val = pickle.load(w.stdout)
                    except EOFError:
                        raise RuntimeError(f"decode worker {w.pid} exited (code {w.poll()})") from None
                    sent[j] = None
                    if kind != "ok":
                        err = err or val
                    elif err is None:
                        yield bounds[j][0], bounds[j][1], val
                if err is not None:
                    raise RuntimeError("image decode failed in a worker process:\n" + err)
            finally:
                for w in sent:  # keep the protocol in step if the caller stopped early
                    if w is not None:
                        try:
                            pickle.load(w.stdout)
                        except Exception:  # noqa: BLE001
                            pass

    def close(self):
        for w in self.procs:
            try:
                w.stdin.close()
            except OSError:
                pass
        for w in self.procs:
            try:
                w.wait(timeout=5)
            except subprocess.TimeoutExpired:
                w.kill()
                w.wait()
        self.procs = []


_LIVE_POOLS: "weakref.WeakSet[DecodePool]" = weakref.WeakSet()
_LIVE_SHM: "weakref.WeakSet[ShmBuffer]" = weakref.WeakSet()
_EXIT_HOOKS: list = []


def on_exit(fn):
    """Run `fn` at interpreter exit before the decode workers are stopped (prefetch
    threads must be joined first: they may be waiting on a worker)."""
    _EXIT_HOOKS.append(fn)
    return fn


@atexit.register
def _shutdown():
    for fn in _EXIT_HOOKS:
        fn()
    for p in list(_LIVE_POOLS):
        p.close()
    for b in list(_LIVE_SHM):
        b.close()


def default_decode_process() -> int:
    """min(16, host cores) when there are at least 4 (16 = one MI355X's share of a
    node's cores), else 0 (decode in threads)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return min(16, n) if n >= 4 else 0


def default_native_threads() -> int:
    """Threads of the native decode pool: this process's share of the host cores (the cores
    it may run on / the ranks of this node -- LOCAL_WORLD_SIZE, one process per GPU), at most
    32 (AlexNet at ~120k img/s needs about 32 decode threads per GPU with the GPU decode stage,
    profiles/r5_io_gpu_decode_stage.jsonl)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    ranks = max(1, int(os.environ.get("LOCAL_WORLD_SIZE", "1") or 1))
    return max(1, min(32, n // ranks))


if __name__ == "__main__":
    _worker_main()
