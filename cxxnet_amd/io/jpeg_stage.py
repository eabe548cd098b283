"""GPU JPEG decode stage: the host entropy-decodes, the GPU does everything after.

Reference: src/io/iter_thread_imbin_x-inl.hpp:270-388 (decode threads feeding the batch) and
src/utils/decoder.h:21-104 (libjpeg decode of one record).  The reference decodes every image
to pixels on host threads; on a host feeding an MI355X that is the bottleneck (about 2.3k
images/s per busy core, profiles/r4_io_native_decode_train.jsonl, against ~118k images/s of
AlexNet training per GPU).  Here the split is:

  host (runtime/jpeg_decode.h ReadCoefCrop, the native thread pool, GIL released):
      jpeg_read_coefficients (Huffman / arithmetic decoding, the serial part), the record's
      crop / mirror / contrast draws, and a copy of the crop window's coefficient blocks
      (plus one chroma sample of upsampling context per side) into a pinned staging batch;
  GPU (csrc/kernels/jpeg_kernels.hip, inside the training step's input stage):
      dequantise + islow IDCT of every staged block (8 threads per block, LDS transpose),
      then fancy chroma upsampling + YCbCr->RGB + crop + mirror into the uint8 batch that
      the image kernel turns into the network input.

The integer arithmetic is libjpeg's (jidctint.c, jdsample.c, jdcolor.c), so a decoded batch is
bit-identical to libjpeg-turbo's decode of the same crops (the CPU native path);
``decode_reference`` below is the same arithmetic in numpy, checked against libjpeg on the
CPU (tests/test_jpeg_stage_cpu.py) and against the kernels on the GPU
(tests/test_jpeg_stage_gpu.py).  Records the stage does not take (non-JPEG, CMYK, 12-bit,
4:4:0 or exotic sampling) are decoded to pixels on the host as before and copied over their rows.
"""
from typing import List, Optional

import numpy as np
import torch

from .data import DevicePrefetch, U8Images

META = 80  # int32 per window (runtime/jpeg_decode.h CoefMetaField)
BLK0, BW, BH, BY0, BX0, DW, DH, RH, RV, NCOMP, VALID, QUANT = 0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 16


def stage_capacity(batch: int, h: int, w: int) -> int:
    """Blocks a batch can need: three full-rate windows of an unaligned h x w crop (4:4:4,
    the worst case; 4:2:0 uses about half)."""
    return batch * 3 * (-(-h // 8) + 1) * (-(-w // 8) + 1)


class JpegCoefImages:
    """A batch still in entropy-decoded form (rows r0..r1 of the staged batch).  Duck-types
    the parts of U8Images the trainer touches (shape, row slices, clone, to_float);
    ``to_u8(device)`` finishes the decode (GPU kernels, or the numpy reference on the CPU)."""

    def __init__(self, coef, bwin, meta, nblk, prm, cm, hwc, fb_pix=None, fb_rows=(), mean=None, mode=0,
                 scale=1.0, r0=0, r1=None, pf=None):
        self.coef, self.bwin, self.meta, self.nblk = coef, bwin, meta, int(nblk)
        self.prm_all, self.cm_all, self.hwc = prm, cm, tuple(hwc)
        self.fb_pix, self.fb_rows = fb_pix, sorted(fb_rows)
        self.mean, self.mode, self.scale = mean, mode, float(scale)
        self.r0, self.r1 = r0, meta.shape[0] if r1 is None else r1
        self.pf = pf  # DevicePrefetch of (coef[:nblk], bwin[:nblk], meta, prm[, fallback pixels])

    def prefetch(self, dev: torch.device):
        """Issue the batch's host-to-device copies now, on a side stream (the iterator's thread)."""
        ts = [self.coef[:self.nblk], self.bwin[:self.nblk], self.meta, self.prm_all]
        self.pf = DevicePrefetch(ts + ([self.fb_pix] if self.fb_pix is not None else []), dev)

    @property
    def shape(self):
        h, w, C = self.hwc
        return (self.r1 - self.r0, C, h, w)

    @property
    def prm(self):
        return self.prm_all[self.r0:self.r1]

    @property
    def cm(self):
        return self.cm_all[self.r0:self.r1]

    def _view(self, r0, r1):
        return JpegCoefImages(self.coef, self.bwin, self.meta, self.nblk, self.prm_all, self.cm_all, self.hwc,
                              self.fb_pix, self.fb_rows, self.mean, self.mode, self.scale, r0, r1, self.pf)

    def __getitem__(self, sl):
        if not isinstance(sl, slice) or sl.step not in (None, 1):
            raise TypeError("JpegCoefImages supports contiguous row slices only")
        lo, hi, _ = sl.indices(self.r1 - self.r0)
        return self._view(self.r0 + lo, self.r0 + max(hi, lo))

    def clone(self):  # the staged buffers are never written after the batch is made
        return self._view(self.r0, self.r1)

    def to_u8(self, device=None) -> U8Images:
        dev = torch.device(device) if device is not None else torch.device("cpu")
        h, w, C = self.hwc
        staged = None
        if dev.type == "cuda":
            from .. import ops
            staged = self.pf.take(dev) if self.pf is not None else None
            pix = ops.jpeg_decode(self.coef, self.bwin, self.meta, self.nblk, self.prm_all, self.r0, self.r1, h, w, C,
                                  dev, staged[:4] if staged is not None else None)
        else:
            pix = torch.from_numpy(decode_reference(self.coef[:self.nblk].numpy(), self.bwin[:self.nblk].numpy(),
                                                    self.meta.numpy(), self.prm_all.numpy(), self.r0, self.r1,
                                                    h, w, C))
        rows = [i for i in self.fb_rows if self.r0 <= i < self.r1]
        if rows:
            idx = torch.tensor([i - self.r0 for i in rows], dtype=torch.long)
            src = staged[4][rows] if staged is not None else self.fb_pix[rows]
            pix.index_copy_(0, idx.to(pix.device), src.to(pix.device, non_blocking=True))
        prm, cm = self.prm, self.cm
        if staged is not None:  # the crop rows on the device too (the image kernel's prm)
            prm = staged[3][self.r0:self.r1]
            cm = cm.to(dev, non_blocking=True)
        return U8Images(pix, prm, cm, self.mean, self.mode, self.scale)

    def to_float(self) -> torch.Tensor:
        return self.to_u8().to_float()


# ---------------------------------------------------------------------- numpy reference
_F = dict(F0298=2446, F0390=3196, F0541=4433, F0765=6270, F0899=7373, F1175=9633, F1501=12299, F1847=15137,
          F1961=16069, F2053=16819, F2562=20995, F3072=25172)


def _idct8(v: List[np.ndarray], shift: int) -> List[np.ndarray]:
    """jidctint.c jpeg_idct_islow, one pass over 8 int64 arrays."""
    f = _F
    z2, z3 = v[2], v[6]
    z1 = (z2 + z3) * f["F0541"]
    tmp2, tmp3 = z1 - z3 * f["F1847"], z1 + z2 * f["F0765"]
    tmp0, tmp1 = (v[0] + v[4]) << 13, (v[0] - v[4]) << 13
    t10, t13, t11, t12 = tmp0 + tmp3, tmp0 - tmp3, tmp1 + tmp2, tmp1 - tmp2
    tmp0, tmp1, tmp2, tmp3 = v[7], v[5], v[3], v[1]
    z1, z2, z3, z4 = tmp0 + tmp3, tmp1 + tmp2, tmp0 + tmp2, tmp1 + tmp3
    z5 = (z3 + z4) * f["F1175"]
    tmp0, tmp1, tmp2, tmp3 = tmp0 * f["F0298"], tmp1 * f["F2053"], tmp2 * f["F3072"], tmp3 * f["F1501"]
    z1, z2, z3, z4 = z1 * -f["F0899"], z2 * -f["F2562"], z3 * -f["F1961"] + z5, z4 * -f["F0390"] + z5
    tmp0, tmp1, tmp2, tmp3 = tmp0 + z1 + z3, tmp1 + z2 + z4, tmp2 + z2 + z3, tmp3 + z1 + z4
    r = 1 << (shift - 1)
    o = [None] * 8
    o[0], o[7] = (t10 + tmp3 + r) >> shift, (t10 - tmp3 + r) >> shift
    o[1], o[6] = (t11 + tmp2 + r) >> shift, (t11 - tmp2 + r) >> shift
    o[2], o[5] = (t12 + tmp1 + r) >> shift, (t12 - tmp1 + r) >> shift
    o[3], o[4] = (t13 + tmp0 + r) >> shift, (t13 - tmp0 + r) >> shift
    return o


def idct_reference(coef: np.ndarray, quant: np.ndarray) -> np.ndarray:
    """(n, 64) int16 natural-order coefficients x (n, 64) steps -> (n, 64) uint8 samples."""
    d = coef.astype(np.int64).reshape(-1, 8, 8) * quant.astype(np.int64).reshape(-1, 8, 8)
    ws = _idct8([d[:, k, :] for k in range(8)], 11)  # pass 1: columns; ws[k] = row k, (n, col)
    ws = np.stack(ws, 1).astype(np.int32).astype(np.int64)  # (n, row, col), int workspace
    o = _idct8([ws[:, :, k] for k in range(8)], 18)  # pass 2: rows; o[k] = column k, (n, row)
    j = np.stack(o, 2).astype(np.int32) & 1023
    out = np.where(j < 128, j + 128, np.where(j < 512, 255, np.where(j < 896, 0, j - 896)))
    return out.astype(np.uint8).reshape(-1, 64)


def decode_reference(coef, bwin, meta, prm, r0, r1, h, w, C) -> np.ndarray:
    """The GPU stage in numpy: (r1 - r0, h, w, C) uint8 (zeros for rows the stage does not hold)."""
    meta = meta.reshape(-1, 3, META)
    planes = idct_reference(coef, meta.reshape(-1, META)[bwin, QUANT:QUANT + 64]) if len(coef) else coef
    out = np.zeros((r1 - r0, h, w, C), np.uint8)
    yy, xx = np.mgrid[0:h, 0:w]
    for b in range(r0, r1):
        m = meta[b]
        if m[0, VALID] == 0:
            continue
        Y = prm[b, 0] + yy
        X = prm[b, 1] + (w - 1 - xx if prm[b, 2] else xx)

        def plane(k):
            wk = m[k]
            n = wk[BW] * wk[BH]
            p = planes[wk[BLK0]:wk[BLK0] + n].reshape(wk[BH], wk[BW], 8, 8).transpose(0, 2, 1, 3)
            p = p.reshape(wk[BH] * 8, wk[BW] * 8).astype(np.int64)
            return lambda sy, sx: p[sy - wk[BY0] * 8, sx - wk[BX0] * 8]

        lum = plane(0)(Y, X)
        if m[0, NCOMP] == 1:
            rgb = [lum, lum, lum]
        else:
            ch = []
            for k in (1, 2):
                wk, S = m[k], plane(k)
                if wk[RH] == 1:
                    ch.append(S(Y, X))
                    continue
                cx, odd = X >> 1, (X & 1) == 1
                if wk[RV] == 1:
                    s = S(Y, cx)
                    ev = np.where(cx == 0, s, (3 * s + S(Y, np.maximum(cx - 1, 0)) + 1) >> 2)
                    od = np.where(cx == wk[DW] - 1, s, (3 * s + S(Y, np.minimum(cx + 1, wk[DW] - 1)) + 2) >> 2)
                else:
                    cy = Y >> 1
                    ny = np.where((Y & 1) == 1, np.minimum(cy + 1, wk[DH] - 1), np.maximum(cy - 1, 0))

                    def cs(c):
                        return 3 * S(cy, c) + S(ny, c)
                    t = cs(cx)
                    ev = np.where(cx == 0, (t * 4 + 8) >> 4, (3 * t + cs(np.maximum(cx - 1, 0)) + 8) >> 4)
                    od = np.where(cx == wk[DW] - 1, (t * 4 + 7) >> 4,
                                  (3 * t + cs(np.minimum(cx + 1, wk[DW] - 1)) + 7) >> 4)
                ch.append(np.where(odd, od, ev))
            cb, cr = ch[0] - 128, ch[1] - 128
            rgb = [lum + ((91881 * cr + 32768) >> 16), lum + ((-46802 * cr - 22554 * cb + 32768) >> 16),
                   lum + ((116130 * cb + 32768) >> 16)]
        for k in range(C):
            out[b - r0, :, :, k] = np.clip(rgb[k], 0, 255)
    return out


def stage_batch(pool, items, cfg, B: int, h: int, w: int, C: int, pinned: bool):
    """Run the host half over `items` [(row, payload, seed)]: returns (coef, bwin, meta, nblk,
    prm, cm, failed rows)."""
    cap = stage_capacity(B, h, w)
    coef = torch.empty((cap, 64), dtype=torch.int16, pin_memory=pinned)
    bwin = torch.empty((cap,), dtype=torch.int32, pin_memory=pinned)
    meta = torch.empty((B, 3, META), dtype=torch.int32, pin_memory=pinned)
    meta.numpy().fill(0)  # numpy fills: torch's parallel fill wakes its OpenMP pool, which then
    prm = torch.empty((B, 4), dtype=torch.int32, pin_memory=pinned)  # spins against the decode threads
    prm.numpy().fill(0)
    cm = torch.empty((B, 2), dtype=torch.float32, pin_memory=pinned)
    cm.numpy()[:, 0], cm.numpy()[:, 1] = 1.0, 0.0
    failed, nblk = pool.decode_coef(items, cfg, coef.numpy(), bwin.numpy(), meta.numpy(), prm.numpy(), cm.numpy())
    return coef, bwin, meta, nblk, prm, cm, list(failed)


def fallback_rows(pool, items, failed, cfg, shape, prm, cm, pinned: bool, pillow_one) -> Optional[torch.Tensor]:
    """Host pixel decode of the rows the stage reported back (CPU native decoder, then Pillow)."""
    if not failed:
        return None
    fb = torch.empty(shape, dtype=torch.uint8, pin_memory=pinned)
    pix = fb.numpy()
    pix.fill(0)
    sel = [it for it in items if it[0] in set(failed)]
    again = set(pool.decode(sel, cfg, pix, prm.numpy(), cm.numpy()))
    for i, payload, seed in sel:
        if i in again:
            img, p, c = pillow_one(payload, seed)
            pix[i] = img[..., :shape[3]]
            prm[i, :3] = torch.as_tensor(p)
            cm[i] = torch.as_tensor(c)
    return fb
