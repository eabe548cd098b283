"""Image iterators: `iter = img | imgbin | imgbinx`, the augmenter and the batch adapter.

Reference behaviour:
  * img      -- src/io/iter_img-inl.hpp:20-137 (list + image_root, imread, shuffle)
  * imgbin   -- src/io/iter_thread_imbin-inl.hpp:20-285 (list + 64 MB BinaryPage files,
                multi-part lists, image_conf_prefix/ids ranges, dist sharding, PS_RANK)
  * imgbinx  -- src/io/iter_thread_imbin_x-inl.hpp:150-345 (part-order shuffle, in-page
                shuffle, labels read page by page)
  * augment  -- src/io/iter_augment_proc-inl.hpp:98-198 (crop / mirror / mean image or
                mean_value / contrast / illumination / scale, mean image auto-generation)
  * affine   -- src/io/image_augmenter-inl.hpp:74-161 (rotate / shear / aspect / scale
                warp, rotate_list, fill_value)
  * batching -- src/io/iter_batch_proc-inl.hpp:16-120 (round_batch, num_batch_padd,
                test_skipread)

MI355X-first design:
  * The page reader is native (``_cxxnet_rt.ImageBinReader``: a C++ thread streams
    64 MB pages ahead of the consumer).
  * Records are pulled serially (deterministic order and RNG), then decoded and
    geometrically augmented by the native decode pool (``_cxxnet_rt.JpegDecodePool``,
    csrc/runtime/jpeg_decode.h: C++ threads over libjpeg-turbo, crop-window-only decode,
    no interpreter per image) straight into the page-locked batch buffer -- the
    reference's decode thread (iter_thread_imbin_x-inl.hpp:150-388, utils/decoder.h).
    Affine augmentation and non-JPEG records take the Pillow path: worker processes
    writing into a shared batch buffer (io/augment.py; a thread pool when
    decode_process = 0).
  * A batch leaves the host as uint8 (``U8Images``).  Mean subtraction, contrast,
    illumination, scale and the NHWC-bf16 conversion happen on the GPU in one fused
    kernel (``ops.image_to_nhwc``).  That is 4x less PCIe traffic than fp32 and
    keeps no float image on the host.
  * Under data parallelism each rank decodes only the rows of the global batch
    that the trainer will hand to it.

Decoding uses Pillow (OpenCV is not available here).  Pixels are RGB like the
reference's BGR->RGB conversion.  The affine warp uses Pillow's bicubic resampler,
so warped pixels are not bit-identical to OpenCV's INTER_CUBIC (parity unpinned).
"""
from __future__ import annotations

import os
from concurrent.futures import ThreadPoolExecutor
from dataclasses import dataclass
from typing import Iterator, List, Optional, Tuple

import numpy as np
import torch

from .. import native
from .augment import AugmentParam, DecodePool, ShmBuffer, _augment_one, default_decode_process, default_native_threads, shm_available
from . import jpeg_stage
from .data import DEVICE_IO_LOCK, DataBatch, DataIterator, U8Images, input_device
from .jpeg_stage import JpegCoefImages


# ----------------------------------------------------------------------------- records
@dataclass
class Record:
    index: int
    label: np.ndarray          # float32 (label_width,)
    payload: object            # bytes (encoded image) or str (path)


def _read_list(path: str, label_width: int) -> List[Tuple[int, np.ndarray, str]]:
    out = []
    for e in native.rt().parse_image_list(path, label_width):
        out.append((int(e.index), np.asarray(e.labels, dtype=np.float32), e.path))
    return out


class _Source:
    """Instance source: yields Records in reference order."""

    def set_param(self, name: str, val: str):
        pass

    def init(self):
        pass

    def records(self) -> Iterator[Record]:
        raise NotImplementedError


class ImageListSource(_Source):
    """`iter = img`: image_list + image_root, optional per-epoch shuffle."""

    def __init__(self):
        self.path_list = "img.lst"
        self.root = ""
        self.shuffle = 0
        self.label_width = 1
        self.silent = 0
        self.seed = 0
        self.entries: List[Tuple[int, np.ndarray, str]] = []
        self._epoch = 0

    def set_param(self, name, val):
        if name == "image_list":
            self.path_list = val
        elif name == "image_root":
            self.root = val
        elif name == "shuffle":
            self.shuffle = int(val)
        elif name == "label_width":
            self.label_width = int(val)
        elif name == "silent":
            self.silent = int(val)
        elif name == "seed_data":
            self.seed = int(val)

    def init(self):
        self.entries = _read_list(self.path_list, self.label_width)
        if not self.silent:
            print(f"ImageIterator:image_list={self.path_list}")

    def records(self):
        order = np.arange(len(self.entries))
        if self.shuffle:
            order = np.random.default_rng(self.seed + 7919 * self._epoch).permutation(len(self.entries))
        self._epoch += 1
        for i in order:
            idx, lab, path = self.entries[i]
            yield Record(idx, lab, self.root + path)


class ImageBinSource(_Source):
    """`iter = imgbin`: list lines consumed in lock-step with objects of the paged
    .bin files (one or more list/bin pairs, or image_conf_prefix + image_conf_ids)."""

    def __init__(self):
        self.lists: List[str] = []
        self.bins: List[str] = []
        self.conf_prefix = ""
        self.conf_ids = ""
        self.dist_num_worker = 0
        self.dist_worker_rank = 0
        self.label_width = 1
        self.silent = 0

    def set_param(self, name, val):
        if name == "image_list":
            self.lists.append(val)
        elif name == "image_bin":
            self.bins.append(val)
        elif name == "image_conf_prefix":
            self.conf_prefix = val
        elif name == "image_conf_ids":
            self.conf_ids = val
        elif name == "dist_num_worker":
            self.dist_num_worker = int(val)
        elif name == "dist_worker_rank":
            self.dist_worker_rank = int(val)
        elif name == "label_width":
            self.label_width = int(val)
        elif name == "silent":
            self.silent = int(val)

    def _parse_conf(self):
        """Reference ParseImageConf (iter_thread_imbin-inl.hpp:187-217)."""
        if os.environ.get("PS_RANK") is not None:
            self.dist_worker_rank = int(os.environ["PS_RANK"])
        if not self.conf_prefix:
            return
        if self.lists or self.bins:
            raise ValueError("you can either set image_conf_prefix or image_bin/image_list")
        try:
            lb, ub = (int(v) for v in self.conf_ids.split("-"))
        except ValueError:
            raise ValueError("image_conf_ids only support range, like 1-100") from None
        n = ub + 1 - lb
        if self.dist_num_worker > 1:
            step = (n + self.dist_num_worker - 1) // self.dist_num_worker
            begin = min(self.dist_worker_rank * step, n) + lb
            end = min((self.dist_worker_rank + 1) * step, n) + lb
            lb, ub = begin, end - 1
            if lb > ub:
                raise ValueError("ThreadImagePageIterator: too many workers such that idlist cannot be divided")
        for i in range(lb, ub + 1):
            stem = self.conf_prefix % i
            self.lists.append(stem + ".lst")
            self.bins.append(stem + ".bin")

    def init(self):
        self._parse_conf()
        if not self.lists or len(self.lists) != len(self.bins):
            raise ValueError("List/Bin number not consist")
        if not self.silent:
            print(f"ThreadImagePageIterator:image_list={','.join(self.lists)}, bin={','.join(self.bins)}")

    def records(self):
        reader = native.rt().ImageBinReader(self.bins, 4)
        for lst in self.lists:
            entries = _read_list(lst, self.label_width)
            pos = 0
            while pos < len(entries):  # runs of up to 64 objects, one copy per run (zero-copy views)
                got = reader.next_run(min(64, len(entries) - pos))
                if got is None:
                    raise ValueError(f"image bin has fewer objects than list {lst}")
                blob, spans = got
                mv = memoryview(blob)
                for (idx, lab, _), (o, n) in zip(entries[pos:pos + len(spans)], spans):
                    yield Record(idx, lab, mv[o:o + n])
                pos += len(spans)


class ImageBinXSource(ImageBinSource):
    """`iter = imgbinx`: like imgbin, plus part-order and in-page shuffling
    (labels are read page by page so they stay aligned with shuffled objects)."""

    def __init__(self):
        super().__init__()
        self.shuffle = 0
        self.seed = 0
        self._epoch = 0

    def set_param(self, name, val):
        super().set_param(name, val)
        if name == "shuffle":
            self.shuffle = int(val)
        elif name == "seed_data":
            self.seed = int(val)

    def records(self):
        rng = np.random.default_rng(121 + self.seed + 104729 * self._epoch)
        self._epoch += 1
        order = np.arange(len(self.bins))
        if self.shuffle:
            order = rng.permutation(len(self.bins))
        for part in order:
            reader = native.rt().ImageBinReader([self.bins[part]], 2)
            entries = _read_list(self.lists[part], self.label_width)
            pos = 0
            while True:
                objs = reader.next_page()
                if objs is None:
                    break
                page = entries[pos:pos + len(objs)]
                if len(page) != len(objs):
                    raise ValueError(f"invalid list format: {self.lists[part]} shorter than {self.bins[part]}")
                pos += len(objs)
                inner = rng.permutation(len(objs)) if self.shuffle else range(len(objs))
                for j in inner:
                    yield Record(page[j][0], page[j][1], objs[j])


# ----------------------------------------------------------------------------- batch iterator
def consumer_device(dev: Optional[str]) -> Optional[torch.device]:
    """The CUDA device the trainer configured by `dev` trains on, or None when the batches are
    consumed on the host (NetTrainer._device's rule): 'cpu' -> None; under torch.distributed the
    rank's device (LOCAL_RANK); 'gpu:N' -> cuda:N; no `dev` key seen -> the rank's GPU when one is
    present."""
    if not torch.cuda.is_available():
        return None
    if dev is None:
        return input_device()
    from ..nnet.trainer import parse_devices
    kind, ids = parse_devices(dev)
    if kind != "gpu":
        return None
    try:
        import torch.distributed as dist
        if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
            return input_device()
    except Exception:  # noqa: BLE001
        pass
    return torch.device("cuda", ids[0] if ids else 0)


def _dist_rows(batch_size: int) -> Tuple[int, int]:
    """Rows of the global batch this rank trains on (same rule as NetTrainer._slice)."""
    world, rank = 1, 0
    try:
        import torch.distributed as dist
        if dist.is_available() and dist.is_initialized():
            world, rank = dist.get_world_size(), dist.get_rank()
    except Exception:  # noqa: BLE001
        pass
    step = max((batch_size + world - 1) // world, 1)
    return min(rank * step, batch_size), min((rank + 1) * step, batch_size)


class ImageBatchIterator(DataIterator):
    """BatchAdaptIterator(AugmentIterator(<source>)) with a parallel decode stage.

    Extra keys (new): decode_native (default 1: JPEG records without affine augmentation
    are decoded by the native C++ pool of decode_native_threads threads, default this
    rank's share of the host cores, at most 32: io/augment.py default_native_threads), decode_gpu (default: on when a GPU is present; with the native
    pool, the host only entropy-decodes and the GPU runs IDCT / upsampling / colour / crop,
    io/jpeg_stage.py), prefetch_device (default: on with a GPU; the batch's host-to-device
    copies are issued from the iterator's thread on a side stream, io/data.py DevicePrefetch),
    decode_process (default min(16, host cores) when there are at
    least 4, else 0: the Pillow path decodes in that many worker processes, io/augment.py,
    writing into a shared-memory batch; 0 = use threads), decode_thread (threads when
    decode_process is 0; default min(8, cpus)), shard_decode (default 1: under
    torch.distributed each rank decodes only its own rows of the batch).  Results do not
    depend on the worker counts: every record's augmentation draws are seeded from the
    iterator's stream (the native and Pillow paths draw crops from different generators, so
    switching decode_native changes which crops a seed picks, not their distribution)."""

    fresh_batches = True  # every next() returns newly allocated tensors

    def __init__(self, source: _Source):
        self.source = source
        self.aug = AugmentParam()
        self.batch_size = 1
        self.label_width = 1
        self.round_batch = 0
        self.test_skipread = 0
        self.silent = 0
        self.decode_thread = min(8, os.cpu_count() or 1)
        self.decode_process = -1
        self._shm = None
        self._shm_fin = None
        self._procs = None
        self.shard_decode = 1
        self.decode_native = 1
        self.decode_native_threads = 0
        self.decode_gpu = -1
        self.prefetch_device = -1
        self.dev = None  # the trainer's `dev` (global conf key): the device the batches feed
        self._dev: Optional[torch.device] = None
        self._jpeg = None
        self._pool: Optional[ThreadPoolExecutor] = None
        self.mean: Optional[torch.Tensor] = None
        self.mean_mode = 0
        self.out: Optional[DataBatch] = None
        self._it: Optional[Iterator[Record]] = None
        self._overflow = 0
        self._head = True
        self._seed_rng = np.random.default_rng(0)

    def set_param(self, name, val):
        self.source.set_param(name, val)
        self.aug.set_param(name, val)
        if name == "batch_size":
            self.batch_size = int(val)
        elif name == "label_width":
            self.label_width = int(val)
        elif name == "round_batch":
            self.round_batch = int(val)
        elif name == "test_skipread":
            self.test_skipread = int(val)
        elif name == "silent":
            self.silent = int(val)
        elif name == "decode_thread":
            self.decode_thread = max(1, int(val))
        elif name == "decode_process":
            self.decode_process = int(val)
        elif name == "shard_decode":
            self.shard_decode = int(val)
        elif name == "decode_native":
            self.decode_native = int(val)
        elif name == "decode_native_threads":
            self.decode_native_threads = int(val)
        elif name == "decode_gpu":
            self.decode_gpu = int(val)
        elif name == "prefetch_device":
            self.prefetch_device = int(val)
        elif name == "dev":
            self.dev = val

    # ------------------------------------------------------------------ setup
    def init(self):
        self.source.init()
        self._seed_rng = np.random.default_rng(self.aug.seed)
        self._pool = ThreadPoolExecutor(self.decode_thread, thread_name_prefix="cxxnet-decode")
        if self.decode_process < 0:
            self.decode_process = default_decode_process()
        if not shm_available():
            self.decode_process = 0
        self._dev = consumer_device(self.dev)
        if self.prefetch_device < 0:
            self.prefetch_device = int(self._dev is not None)
        elif self._dev is None:
            self.prefetch_device = 0  # nothing on a GPU consumes the batches
        C, h, w = self.aug.shape
        if self.decode_native and h > 1 and C <= 3 and not self.aug.need_affine():
            rt = native.rt()
            if rt.JpegDecodePool.available():
                n = self.decode_native_threads or default_native_threads()
                self._jpeg = rt.JpegDecodePool(n)
                if self.decode_gpu < 0:  # default: on only when a GPU consumes the batches
                    self.decode_gpu = int(self._dev is not None)
            elif not self.silent:
                print(f"native JPEG decoder unavailable ({rt.JpegDecodePool.error()}): decoding with Pillow")
        if self.aug.mean_value is not None and any(v > 0 for v in self.aug.mean_value):
            # the reference subtracts mean_value[i] from channel i (iter_augment_proc-inl.hpp:64-67,128)
            self.mean = torch.tensor(self.aug.mean_value, dtype=torch.float32)
            self.mean_mode = 1
        elif self.aug.image_mean:
            if os.path.exists(self.aug.image_mean):
                if not self.silent:
                    print(f"loading mean image from {self.aug.image_mean}")
                self.mean = load_mean_image(self.aug.image_mean)
            else:
                self.mean = self._create_mean_image()
            self.mean_mode = 3 if tuple(self.mean.shape) == (C, h, w) else 2
        self.before_first()

    def _create_mean_image(self) -> torch.Tensor:
        """One full pass over un-normalised crops (x scale), averaged and saved in
        mshadow binary format (iter_augment_proc-inl.hpp:171-198)."""
        if not self.silent:
            print(f"cannot find {self.aug.image_mean}: create mean image, this will take some time...")
        acc = None
        n = 0
        for recs in self._chunks(self.source.records(), 256):
            outs = self._decode_rows(recs, 0)
            for pix, _, _ in outs:
                a = pix.astype(np.float64)
                acc = a if acc is None else acc + a
                n += 1
        if n == 0:
            raise ValueError("input iterator failed.")
        mean = torch.from_numpy((acc / n * self.aug.scale).astype(np.float32)).permute(2, 0, 1).contiguous()
        save_mean_image(self.aug.image_mean, mean)
        if not self.silent:
            print(f"save mean image to {self.aug.image_mean}..")
        return mean

    @staticmethod
    def _chunks(it, n):
        buf = []
        for r in it:
            buf.append(r)
            if len(buf) == n:
                yield buf
                buf = []
        if buf:
            yield buf

    def _decode_rows(self, recs: List[Record], mean_mode: int):
        seeds = [int(s) for s in self._seed_rng.integers(0, 2 ** 63 - 1, size=len(recs))]
        return list(self._pool.map(lambda a: _augment_one(a[0].payload, self.aug, a[1], mean_mode),
                                   zip(recs, seeds)))

    # ------------------------------------------------------------------ iteration
    def before_first(self):
        if self.round_batch == 0 or self._overflow == 0:
            self._it = self.source.records()
        else:
            self._overflow = 0
        self._head = True

    def _take(self) -> Optional[Record]:
        try:
            return next(self._it)
        except StopIteration:
            return None

    def next(self) -> bool:
        if self.test_skipread and not self._head and self.out is not None:
            return True
        self._head = False
        if self._overflow:
            return False
        B = self.batch_size
        recs: List[Record] = []
        while len(recs) < B:
            r = self._take()
            if r is None:
                break
            recs.append(r)
        if not recs:
            return False
        padd = 0
        if len(recs) < B:
            if self.round_batch:
                self._it = self.source.records()
                while len(recs) < B:
                    r = self._take()
                    if r is None:
                        raise ValueError("number of input must be bigger than batch size")
                    recs.append(r)
                    self._overflow += 1
                padd = self._overflow
            else:
                padd = B - len(recs)
        if torch.cuda.is_available():  # pinned allocations: not while a HIP graph is being captured
            with DEVICE_IO_LOCK:
                self.out = self._make_batch(recs, padd)
        else:
            self.out = self._make_batch(recs, padd)
        return True

    def _make_batch(self, recs: List[Record], padd: int) -> DataBatch:
        B = self.batch_size
        C, h, w = self.aug.shape
        lw = self.label_width
        lab = np.zeros((B, lw), dtype=np.float32)
        index = np.zeros(B, dtype=np.uint32)
        if recs and all(len(r.label) >= lw for r in recs):  # one stack, not a numpy store per record
            lab[: len(recs)] = np.stack([r.label[:lw] for r in recs])
        else:
            for i, r in enumerate(recs):
                lab[i, : min(lw, len(r.label))] = r.label[:lw]
        index[: len(recs)] = np.fromiter((r.index for r in recs), dtype=np.uint32, count=len(recs))
        label = torch.from_numpy(lab)
        lo, hi = (_dist_rows(B) if self.shard_decode else (0, B))
        rows = [(i, r) for i, r in enumerate(recs) if lo <= i < hi]
        # seeds are drawn for every record so results do not depend on the sharding
        seeds = self._seed_rng.integers(0, 2 ** 63 - 1, size=len(recs)).tolist()
        pinned = torch.cuda.is_available()  # async host-to-device copies of the crop parameters too
        prm_t = torch.empty((B, 4), dtype=torch.int32, pin_memory=pinned)
        cm_t = torch.empty((B, 2), dtype=torch.float32, pin_memory=pinned)
        prm, cm = prm_t.numpy(), cm_t.numpy()
        prm.fill(0)
        cm[:, 0], cm[:, 1] = 1.0, 0.0
        if self._jpeg is not None and self.decode_gpu > 0:
            data = self._stage_jpeg(rows, seeds, (B, h, w, C))
            if self.prefetch_device:
                data.prefetch(self._dev)
            return DataBatch(data, label, index, padd)
        if self._jpeg is not None:
            pix = self._decode_native(rows, seeds, (B, h, w, C), prm, cm)
        elif self.decode_process > 0 and h > 1:
            pix = self._decode_procs(rows, seeds, (B, h, w, C), prm, cm)
        else:
            pix = self._decode_threads(rows, seeds, (B, h, w, C), prm, cm)
        data = U8Images(pix, prm_t, cm_t, self.mean, self.mean_mode, self.aug.scale)
        if self.prefetch_device and h > 1:
            data.prefetch(self._dev, lo, hi)  # only this rank's decoded rows cross PCIe
        return DataBatch(data, label, index, padd)

    @staticmethod
    def _host_buffer(shape) -> torch.Tensor:
        """Destination of one batch: page-locked when a GPU will consume it, so the
        host-to-device copy is a straight DMA."""
        return torch.empty(shape, dtype=torch.uint8, pin_memory=torch.cuda.is_available())

    def _decode_threads(self, rows, seeds, shape, prm, cm) -> torch.Tensor:
        B, h, w, C = shape
        outs = list(self._pool.map(lambda a: _augment_one(a[1].payload, self.aug, seeds[a[0]], self.mean_mode),
                                   rows))
        if h == 1:  # flat input: keep the decoded size
            h, w = outs[0][0].shape[:2] if outs else (1, 1)
        dst = self._host_buffer((B, h, w, C))
        pix = dst.numpy()
        done = np.zeros(B, dtype=bool)
        for (i, _), (img, p, c) in zip(rows, outs):
            pix[i] = img[..., :C]
            prm[i, :3] = p
            cm[i] = c
            done[i] = True
        pix[~done] = 0  # padding rows / other ranks' rows
        return dst

    def _decode_native(self, rows, seeds, shape, prm, cm) -> torch.Tensor:
        """Every row through the native pool (GIL released, crops written in place); the rows it
        reports back (non-JPEG / CMYK / corrupt) through Pillow with the same seed."""
        B, h, w, C = shape
        dst = self._host_buffer(shape)
        pix = dst.numpy()
        a = self.aug
        cfg = (h, w, C, a.rand_crop, a.rand_mirror, a.mirror, a.crop_y_start, a.crop_x_start,
               a.max_random_contrast, a.max_random_illumination, self.mean_mode)
        items = [(i, r.payload, seeds[i]) for i, r in rows]
        failed = set(self._jpeg.decode(items, cfg, pix, prm, cm)) if items else set()
        for i, r in rows:
            if i in failed:
                img, p, c = _augment_one(r.payload, a, seeds[i], self.mean_mode)
                pix[i] = img[..., :C]
                prm[i, :3] = p
                cm[i] = c
        done = np.zeros(B, dtype=bool)
        done[[i for i, _ in rows]] = True
        pix[~done] = 0  # padding rows / other ranks' rows
        return dst

    def _crop_cfg(self, h, w, C):
        a = self.aug
        return (h, w, C, a.rand_crop, a.rand_mirror, a.mirror, a.crop_y_start, a.crop_x_start,
                a.max_random_contrast, a.max_random_illumination, self.mean_mode)

    def _stage_jpeg(self, rows, seeds, shape) -> JpegCoefImages:
        """decode_gpu: the native pool entropy-decodes the rows into a pinned coefficient stage
        and the GPU finishes the decode inside the step's input stage (io/jpeg_stage.py); rows
        the stage does not take are decoded to pixels here (native, then Pillow)."""
        B, h, w, C = shape
        cfg = self._crop_cfg(h, w, C)
        items = [(i, r.payload, seeds[i]) for i, r in rows]
        pinned = torch.cuda.is_available()
        coef, bwin, meta, nblk, prm, cm, failed = jpeg_stage.stage_batch(self._jpeg, items, cfg, B, h, w, C, pinned)
        fb = jpeg_stage.fallback_rows(self._jpeg, items, failed, cfg, shape, prm, cm, pinned,
                                      lambda payload, seed: _augment_one(payload, self.aug, seed, self.mean_mode))
        return JpegCoefImages(coef, bwin, meta, nblk, prm, cm, (h, w, C), fb, failed, self.mean, self.mean_mode,
                              self.aug.scale)

    def _decode_procs(self, rows, seeds, shape, prm, cm) -> torch.Tensor:
        nbytes = int(np.prod(shape))
        if self._shm is None or self._shm.size < nbytes:
            self._free_shm()
            import weakref
            self._shm = ShmBuffer(nbytes)
            self._shm_fin = weakref.finalize(self, self._shm.close)
            self._shm_fin.atexit = False  # io.augment's exit hook runs it after the prefetch threads stop
        if self._procs is None:
            import weakref
            self._procs = DecodePool(self.decode_process)
            weakref.finalize(self, self._procs.close).atexit = False
        items = [(i, r.payload if isinstance(r.payload, (str, bytes)) else bytes(r.payload), seeds[i])
                 for i, r in rows]
        dst = self._host_buffer(shape)
        pix = dst.numpy()
        src = self._shm.array(shape)
        done = np.zeros(shape[0], dtype=bool)
        for lo, hi, res in self._procs.imap(self._shm, shape, self.aug, self.mean_mode, items):
            for i, p, c in res:
                prm[i, :3] = p
                cm[i] = c
            r0, r1 = items[lo][0], items[hi - 1][0] + 1  # rows of a chunk are consecutive
            np.copyto(pix[r0:r1], src[r0:r1])
            done[r0:r1] = True
        pix[~done] = 0  # padding rows / other ranks' rows
        return dst

    def _free_shm(self):
        if self._shm_fin is not None:
            self._shm_fin()
        self._shm = self._shm_fin = None

    def value(self):
        if self._head:
            raise RuntimeError("must call Next to get value")
        return self.out

    def close(self):
        if self._pool is not None:
            self._pool.shutdown(wait=False)
            self._pool = None
        if self._procs is not None:
            self._procs.close()
            self._procs = None
        self._free_shm()



def save_mean_image(path: str, mean: torch.Tensor):
    from ..layers.base import BinWriter
    w = BinWriter()
    w.write_tensor(mean)
    with open(path, "wb") as f:
        f.write(w.getvalue())


def load_mean_image(path: str) -> torch.Tensor:
    from ..layers.base import BinReader
    with open(path, "rb") as f:
        return BinReader(f.read()).read_tensor(3)


def create_image_iterator(kind: str) -> DataIterator:
    src = {"img": ImageListSource, "imgbin": ImageBinSource, "imgbinx": ImageBinXSource}[kind]()
    return ImageBatchIterator(src)

