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
    geometrically augmented by a thread pool.  Pillow releases the GIL in its
    decoders, so this scales over host cores.
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

import io as _io
import math
import os
from concurrent.futures import ThreadPoolExecutor
from dataclasses import dataclass
from typing import Iterator, List, Optional, Tuple

import numpy as np
import torch

from .. import native
from .data import DataBatch, DataIterator, U8Images


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
            for idx, lab, _ in _read_list(lst, self.label_width):
                buf = reader.next()
                if buf is None:
                    raise ValueError(f"image bin has fewer objects than list {lst}")
                yield Record(idx, lab, buf)


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


def _decode(payload) -> np.ndarray:
    from PIL import Image
    im = Image.open(_io.BytesIO(payload) if isinstance(payload, (bytes, bytearray)) else payload)
    im = im.convert("RGB")
    return np.asarray(im)


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
    rng = np.random.default_rng(seed)
    img = _decode(payload)
    if p.need_affine():
        img = _affine(img, p, rng)
    ch, cw = p.shape[1], p.shape[2]
    if ch == 1:  # flat input: no crop (reference: img_ = data * scale_)
        return img, (0, 0, 0), (1.0, 0.0)
    H, W = img.shape[:2]
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
    crop = img[yy:yy + ch, xx:xx + cw]
    if mirror:
        crop = crop[:, ::-1]
    return crop, (yy, xx, int(mirror)), (contrast, illum)


# ----------------------------------------------------------------------------- batch iterator
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

    Extra keys (new): decode_thread (default min(8, cpus)), shard_decode (default 1:
    under torch.distributed each rank decodes only its own rows of the batch)."""

    def __init__(self, source: _Source):
        self.source = source
        self.aug = AugmentParam()
        self.batch_size = 1
        self.label_width = 1
        self.round_batch = 0
        self.test_skipread = 0
        self.silent = 0
        self.decode_thread = min(8, os.cpu_count() or 1)
        self.shard_decode = 1
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
        elif name == "shard_decode":
            self.shard_decode = int(val)

    # ------------------------------------------------------------------ setup
    def init(self):
        self.source.init()
        self._seed_rng = np.random.default_rng(self.aug.seed)
        self._pool = ThreadPoolExecutor(self.decode_thread, thread_name_prefix="cxxnet-decode")
        C, h, w = self.aug.shape
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
        self.out = self._make_batch(recs, padd)
        return True

    def _make_batch(self, recs: List[Record], padd: int) -> DataBatch:
        B = self.batch_size
        C, h, w = self.aug.shape
        lw = self.label_width
        label = torch.zeros((B, lw), dtype=torch.float32)
        index = np.zeros(B, dtype=np.uint32)
        for i, r in enumerate(recs):
            label[i, : min(lw, len(r.label))] = torch.from_numpy(r.label[:lw])
            index[i] = r.index
        lo, hi = (_dist_rows(B) if self.shard_decode else (0, B))
        rows = [(i, r) for i, r in enumerate(recs) if lo <= i < hi]
        # seeds are drawn for every record so results do not depend on the sharding
        seeds = [int(s) for s in self._seed_rng.integers(0, 2 ** 63 - 1, size=len(recs))]
        outs = list(self._pool.map(lambda a: _augment_one(a[1].payload, self.aug, seeds[a[0]], self.mean_mode),
                                   rows))
        if h == 1:  # flat input: keep the decoded size
            hh, ww = outs[0][0].shape[:2] if outs else (1, 1)
        else:
            hh, ww = h, w
        pix = torch.zeros((B, hh, ww, C), dtype=torch.uint8)
        prm = torch.zeros((B, 4), dtype=torch.int32)
        cm = torch.zeros((B, 2), dtype=torch.float32)
        cm[:, 0] = 1.0
        for (i, _), (img, p, c) in zip(rows, outs):
            if img.shape[2] != C:
                img = img[..., :C]
            pix[i] = torch.from_numpy(np.ascontiguousarray(img))
            prm[i, :3] = torch.tensor(p, dtype=torch.int32)
            cm[i] = torch.tensor(c, dtype=torch.float32)
        if torch.cuda.is_available():
            pix = pix.pin_memory()
        data = U8Images(pix, prm, cm, self.mean, self.mean_mode, self.aug.scale)
        return DataBatch(data, label, index, padd)

    def value(self):
        if self._head:
            raise RuntimeError("must call Next to get value")
        return self.out

    def close(self):
        if self._pool is not None:
            self._pool.shutdown(wait=False)
            self._pool = None


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

