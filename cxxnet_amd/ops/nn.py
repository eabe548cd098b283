"""Memory-bound layer ops (pooling, LRN, activations, dropout, softmax/loss,
layout conversion, bias gradient).  GPU: csrc/kernels/nn_kernels.hip; CPU: fp32 torch.

All activations are NHWC (see ops/gemm.py for the layout contract).
"""
from __future__ import annotations

import ctypes
import math

import torch
import torch.nn.functional as F

from .. import native
from .mode import native as _native_t
from .gemm import _stream

ACT_KIND = {"relu": 0, "sigmoid": 1, "tanh": 2, "xelu": 3}


def _k():
    return native.kernels()


# ----------------------------------------------------------------------------- layout
def input_to_nhwc(x_nchw: torch.Tensor, out: torch.Tensor, scale: float = 1.0):
    """NCHW fp32 batch -> NHWC node (bf16 on GPU), zero-padding extra channels (and, for a
    row-padded node of physical width out.shape[2] > W, leaving the pad columns zero)."""
    N, C, H, W = x_nchw.shape
    Cp, Wp = out.shape[-1], out.shape[2]
    if Wp < W:
        raise ValueError(f"input batch {tuple(x_nchw.shape)} does not fit node {tuple(out.shape)}")
    if not _native_t(out):
        out.zero_()
        out[:, :, :W, :C].copy_(x_nchw.permute(0, 2, 3, 1) * scale)
        return
    x = x_nchw.contiguous().float()
    native.check(_k().cxn_nchw_f32_to_nhwc_bf16(x.data_ptr(), out.data_ptr(), N, C, H, W, Cp, Wp, float(scale),
                                                _stream()), "nchw_to_nhwc")


def jpeg_decode(coef, bwin, meta, nblk: int, prm, r0: int, r1: int, h: int, w: int, C: int, dev,
                staged=None) -> torch.Tensor:
    """GPU half of the JPEG stage (io/jpeg_stage.py): staged coefficient blocks -> uint8
    (r1 - r0, h, w, C) crops of rows r0..r1 on `dev` (dequantise + islow IDCT, then fancy
    upsampling + YCbCr->RGB + crop + mirror; csrc/kernels/jpeg_kernels.hip).  staged: device
    copies of (coef[:nblk], bwin[:nblk], meta, prm) already made (io/data.py DevicePrefetch)."""
    B = int(meta.shape[0])
    if not (0 <= r0 <= r1 <= B) or nblk > coef.shape[0] or tuple(meta.shape[1:]) != (3, 80):
        raise ValueError("jpeg_decode: inconsistent stage")
    out = torch.empty((r1 - r0, h, w, C), dtype=torch.uint8, device=dev)
    if r1 == r0:
        return out
    if staged is not None:
        coef_d, bwin_d, meta_d, prm_d = staged
    else:
        meta_d = meta.to(dev, non_blocking=True)
        prm_d = prm.to(dev, torch.int32, non_blocking=True).contiguous()
        coef_d = coef[:nblk].to(dev, non_blocking=True)
        bwin_d = bwin[:nblk].to(dev, non_blocking=True)
    plane = torch.empty((max(nblk, 1), 64), dtype=torch.uint8, device=dev)
    # host-side bounds of what the kernels will index (numpy: a torch CPU reduction would wake
    # its OpenMP pool, whose spinning threads then slow the decode threads down)
    if nblk > 0:
        bw = bwin[:nblk].numpy()
        if int(bw.max()) >= B * 3 or int(bw.min()) < 0:
            raise ValueError("jpeg_decode: block window id out of range")
    m = meta.numpy().reshape(B * 3, 80)
    v = m[:, 10] != 0
    if v.any() and int((m[v, 0] + m[v, 1] * m[v, 2]).max()) > nblk:  # blk0 + bw * bh
        raise ValueError("jpeg_decode: window outside the staged blocks")
    if nblk > 0:
        native.check(_k().cxn_jpeg_idct(coef_d.data_ptr(), bwin_d.data_ptr(), meta_d.data_ptr(), nblk,
                                        plane.data_ptr(), _stream()), "jpeg_idct")
    native.check(_k().cxn_jpeg_color(plane.data_ptr(), meta_d[r0:].data_ptr(), prm_d[r0:].data_ptr(), r1 - r0, h, w, C,
                                     out.data_ptr(), _stream()), "jpeg_color")
    return out


_CONST = {}


def _device_const(t: torch.Tensor, dev) -> torch.Tensor:
    """fp32 device copy of a host tensor that does not change between batches (the iterator's
    mean), made once: a pageable copy per step would stall the host on the stream."""
    key = (id(t), str(dev))
    hit = _CONST.get(key)
    if hit is None or hit[0] is not t:
        hit = _CONST[key] = (t, t.to(dev, torch.float32).contiguous())
    return hit[1]


def image_to_nhwc(img, out: torch.Tensor):
    """U8Images batch -> NHWC input node with the augmenter arithmetic fused
    (GPU: one kernel over uint8 pixels; CPU: the fp32 reference)."""
    from ..io.jpeg_stage import JpegCoefImages
    if isinstance(img, JpegCoefImages):  # finish the JPEG decode where the batch is going
        img = img.to_u8(out.device if _native_t(out) else None)
    if not _native_t(out):
        input_to_nhwc(img.to_float(), out)
        return
    B, C, h, w = img.shape
    Cp, Wp = out.shape[-1], out.shape[2]
    if tuple(out.shape[:2]) != (B, h) or Wp < w or Cp < C:
        raise ValueError(f"image batch {tuple(img.shape)} does not fit input node {tuple(out.shape)}")
    dev = out.device
    got = img.on_device(dev) if hasattr(img, "on_device") else None
    if got is not None:  # copied by the iterator's prefetch (io/data.py DevicePrefetch)
        pix, prm, cm = (t.contiguous() for t in got)
    else:
        pix = img.pix.to(dev, non_blocking=True).contiguous()
        prm = img.prm.to(dev, torch.int32, non_blocking=True).contiguous()
        cm = img.cm.to(dev, torch.float32, non_blocking=True).contiguous()
    mean = _device_const(img.mean, dev) if img.mean is not None else None
    Hm = Wm = 0
    if img.mode == 2:
        Hm, Wm = int(img.mean.shape[1]), int(img.mean.shape[2])
        if int(img.prm[:, 0].max()) + h > Hm or int(img.prm[:, 1].max()) + w > Wm:
            raise ValueError("crop offsets fall outside the mean image")
    elif img.mode == 3 and tuple(img.mean.shape) != (C, h, w):
        raise ValueError("crop-size mean image has the wrong shape")
    elif img.mode == 1 and img.mean.numel() < C:
        raise ValueError("mean_value needs one value per channel")
    native.check(_k().cxn_image_u8_to_nhwc_bf16(
        pix.data_ptr(), prm.data_ptr(), cm.data_ptr(), mean.data_ptr() if mean is not None else None,
        B, h, w, C, Cp, Wp, Hm, Wm, int(img.mode), float(img.scale), out.data_ptr(), _stream()), "image_to_nhwc")


def nhwc_to_nchw(x: torch.Tensor, C: int, W: int = 0) -> torch.Tensor:
    """NHWC node (any dtype) -> NCHW fp32 tensor with C logical channels (and W logical
    columns of a row-padded node; 0 = all)."""
    N, H, Wp, Cp = x.shape
    W = W or Wp
    if not _native_t(x):
        return x[:, :, :W, :C].permute(0, 3, 1, 2).float().contiguous()
    if not x.is_contiguous():  # a channel slice of a zero-copy ch_concat buffer
        x = x.contiguous()
    out = torch.empty((N, C, H, W), dtype=torch.float32, device=x.device)
    native.check(_k().cxn_nhwc_bf16_to_nchw_f32(x.data_ptr(), out.data_ptr(), N, C, H, W, Cp, Wp, _stream()),
                 "nhwc_to_nchw")
    return out


def copy_(dst: torch.Tensor, src: torch.Tensor):
    """dst <- src for contiguous tensors of equal size: a library copy on the GPU (recorded into
    launch lists, so a replayed step repeats it), torch on the CPU."""
    if not (_native_t(src) and dst.is_contiguous() and src.is_contiguous()):
        dst.copy_(src)
        return
    assert dst.numel() == src.numel() and dst.dtype == src.dtype
    native.check(_k().cxn_copy_d2d(dst.data_ptr(), src.data_ptr(), src.numel() * src.element_size(), _stream()),
                 "copy_d2d")


def zero_ranges(buf: torch.Tensor, ranges) -> bool:
    """Zero the float ranges [(a, b), ...] of the contiguous fp32 buffer buf in one launch (GPU,
    at most 16 ranges; recorded into launch lists like every library launch).  False: not
    served (CPU tensor, other dtype, too many ranges) -- the caller zeroes them one by one."""
    if not ranges:
        return True
    if not _native_t(buf) or buf.dtype != torch.float32 or not buf.is_contiguous() or len(ranges) > 16:
        return False
    if any(a < 0 or b > buf.numel() or b < a for a, b in ranges):
        raise ValueError("zero_ranges: range outside the buffer")
    import ctypes
    offs = (ctypes.c_long * len(ranges))(*[a for a, _ in ranges])
    lens = (ctypes.c_long * len(ranges))(*[b - a for a, b in ranges])
    native.check(_k().cxn_zero_ranges(buf.data_ptr(), offs, lens, len(ranges), _stream()), "zero_ranges")
    return True


def zero_(t: torch.Tensor):
    """t <- 0 for a contiguous tensor: a library memset on the GPU (recorded into launch lists,
    so a replayed step repeats it -- a torch zero_() would run only in the recording step),
    torch on the CPU."""
    if not (t.is_cuda and t.is_contiguous()):
        t.zero_()
        return
    native.check(_k().cxn_zero(t.data_ptr(), t.numel() * t.element_size(), _stream()), "zero")


def pad_interior(x: torch.Tensor, xp: torch.Tensor, py: int, px: int):
    """xp[:, py:py+H, px:px+W] <- x (NHWC; xp's border is left as is): a library kernel on the
    GPU, so launch lists record it; torch on the CPU."""
    N, H, W, C = x.shape
    if not (_native_t(x) and x.is_contiguous() and xp.is_contiguous()):
        xp[:, py:py + H, px:px + W].copy_(x)
        return
    assert xp.shape[0] == N and xp.shape[3] == C and xp.dtype == x.dtype
    native.check(_k().cxn_pad_interior(x.data_ptr(), xp.data_ptr(), N, H, W, C, xp.shape[1], xp.shape[2], py, px,
                                       _stream()), "pad_interior")


def transpose(x: torch.Tensor, y: torch.Tensor, B: int, R: int, Cc: int):
    """y[b][Cc][R] = x[b][R][Cc]."""
    if not _native_t(x):
        y.view(B, Cc, R).copy_(x.view(B, R, Cc).transpose(1, 2))
        return
    native.check(_k().cxn_transpose(x.data_ptr(), y.data_ptr(), B, R, Cc, _stream()), "transpose")


# ----------------------------------------------------------------------------- pooling
POOL_MODE = {"max": 0, "sum": 1, "avg": 2}


def pool_out_size(H, k, s, p=0):
    """Reference ceil rule (src/layer/pooling_layer-inl.hpp:103-106), with optional pad."""
    Hp = H + 2 * p
    return min(Hp - k + s - 1, Hp - 1) // s + 1


def _pool_ref(x, KH, KW, S, P, mode, relu, Ho, Wo):
    """x NHWC fp32 -> (out NHWC, arg) with reference window semantics (ceil windows,
    avg = sum/(k*k)); arg = first-max window offset kh*KW+kw (max mode)."""
    xn = x.permute(0, 3, 1, 2)
    if relu:
        xn = xn.clamp_min(0)
    N, C, H, W = xn.shape
    padv = -math.inf if mode == 0 else 0.0
    need_h = (Ho - 1) * S + KH - H - P
    need_w = (Wo - 1) * S + KW - W - P
    xp = F.pad(xn, (P, max(need_w, 0), P, max(need_h, 0)), value=padv)
    arg = None
    if mode == 0:
        out, ind = F.max_pool2d(xp, (KH, KW), S, return_indices=True)
        out, ind = out[:, :, :Ho, :Wo], ind[:, :, :Ho, :Wo]
        Wp = xp.shape[3]
        ih, iw = ind // Wp, ind % Wp
        ho = torch.arange(Ho, device=x.device).view(1, 1, Ho, 1) * S
        wo = torch.arange(Wo, device=x.device).view(1, 1, 1, Wo) * S
        arg = ((ih - ho) * KW + (iw - wo)).to(torch.uint8).permute(0, 2, 3, 1)
    else:
        out = F.avg_pool2d(xp, (KH, KW), S) * (KH * KW)
        if mode == 2:
            out = out / (KH * KW)
        out = out[:, :, :Ho, :Wo]
    return out.permute(0, 2, 3, 1), arg


def pool_forward(x, y, state, KH, KW, S, P, mode: str, relu=False, mark_mask=False, nonneg=False):
    """y = pool(x).  state: uint8 [N][Ho][Wo][C] first-max window offsets (max mode, may be None).
    mark_mask (GPU, max mode, window < 128): also record relu'(max) in bit 7 of the
    offsets so that pool_backward(relu=2) needs no input read.  nonneg: x can only hold values
    >= 0 (a relu output); the max is then taken on integer keys of the bf16 bits."""
    N, H, W, C = x.shape
    Ho, Wo = y.shape[1], y.shape[2]
    m = POOL_MODE[mode]
    if m == 0 and KH * KW > 255:
        raise ValueError("max pooling window larger than 255 elements is not supported")
    if not _native_t(x):
        out, arg = _pool_ref(x, KH, KW, S, P, m, relu, Ho, Wo)
        y.copy_(out)
        if state is not None and arg is not None:
            state.copy_(arg)
        return
    flags = int(bool(relu)) | (2 if (mark_mask and m == 0 and KH * KW < 128 and state is not None) else 0)
    flags |= 4 if nonneg else 0
    native.check(_k().cxn_pool_fwd(x.data_ptr(), y.data_ptr(),
                                   state.data_ptr() if (state is not None and m == 0) else None,
                                   N, H, W, C, Ho, Wo, KH, KW, S, P, m, flags, _stream()), "pool_fwd")


def pool_mask_in_state(mode: str, KH: int, KW: int) -> bool:
    """Whether pool_forward(mark_mask=True) encodes relu' in the max offsets."""
    return POOL_MODE[mode] == 0 and KH * KW < 128


def pool_backward(x, state, dy, dx, KH, KW, S, P, mode: str, relu=False, dbias=None):
    """dx = unpool(dy) (max: to the recorded first maximum); relu: times relu'(x)
    (relu=2 on the GPU: relu' from the offsets written by pool_forward(mark_mask=True)).
    dx may alias x (element-local read-before-write).
    dbias (fp32 [C], optional): += per-channel sum of dx (the producing conv's bias
    gradient, computed here instead of in a separate pass over dx)."""
    N, H, W, C = x.shape
    Ho, Wo = dy.shape[1], dy.shape[2]
    m = POOL_MODE[mode]
    if not _native_t(x):
        g = torch.zeros_like(dy.new_empty(N, H + 2 * P + KH + S, W + 2 * P + KW + S, C))
        for ho in range(Ho):
            hs = ho * S
            for wo in range(Wo):
                ws = wo * S
                gv = dy[:, ho, wo, :]
                if m == 0:
                    a = state[:, ho, wo, :].long()
                    for kh in range(KH):
                        for kw in range(KW):
                            g[:, hs + kh, ws + kw, :] += (a == kh * KW + kw).to(g.dtype) * gv
                else:
                    sc = 1.0 / (KH * KW) if m == 2 else 1.0
                    g[:, hs:hs + KH, ws:ws + KW, :] += gv[:, None, None, :] * sc
        g = g[:, P:P + H, P:P + W, :]
        if relu:
            g = g * (x > 0).to(g.dtype)
        dx.copy_(g)
        if dbias is not None:
            dbias.add_(g.reshape(-1, C).sum(0))
        return
    if dbias is not None and C % 8:
        native.check(_k().cxn_pool_bwd(x.data_ptr(), state.data_ptr() if m == 0 else None, dy.data_ptr(),
                                       dx.data_ptr(), N, H, W, C, Ho, Wo, KH, KW, S, P, m, int(relu), None, None, 0,
                                       _stream()), "pool_bwd")
        bias_grad(dx.reshape(-1, C), dbias)
        return
    ws = _workspace(4096 * C, x.device) if dbias is not None else None
    native.check(_k().cxn_pool_bwd(x.data_ptr(), state.data_ptr() if m == 0 else None, dy.data_ptr(),
                                   dx.data_ptr(), N, H, W, C, Ho, Wo, KH, KW, S, P, m, int(relu),
                                   dbias.data_ptr() if dbias is not None else None,
                                   ws.data_ptr() if ws is not None else None, ws.numel() if ws is not None else 0,
                                   _stream()), "pool_bwd")


def pool_lrn_forward(x, pooled, state, y, relu_flags, nsize, alpha, beta, knorm) -> bool:
    """Fused max-pool (3x3 / 2, pad 0, ceil mode) -> LRN: pooled = pool(x) with the first-max
    offsets in state (bit 7 = relu' of the max when relu_flags & 2), y = lrn(pooled).  Same
    values as pool_forward + lrn_forward.  relu_flags & 1: max over relu(x); & 4: x is known to
    be >= 0 (a fused conv -> relu output; the kernel then takes the max on integer keys).  False when the fused kernel does not serve the
    shape (nothing was done)."""
    N, H, W, C = x.shape
    Ho, Wo = pooled.shape[1], pooled.shape[2]
    if not _native_t(x):
        return False
    rc = _k().cxn_pool_lrn_fwd(x.data_ptr(), pooled.data_ptr(), state.data_ptr(), y.data_ptr(), N, H, W, C, Ho, Wo,
                               int(relu_flags), int(nsize), float(alpha), float(beta), float(knorm), _stream())
    if rc == -1:
        return False
    native.check(rc, "pool_lrn_fwd")
    return True


def lrn_pool_backward(pooled, dy, state, dx, relu_bit, nsize, alpha, beta, knorm, dbias=None, part=None) -> bool:
    """Backward of the fused max-pool -> LRN: dx = unpool(lrn'(pooled, dy)) routed by state
    (relu_bit: a window whose bit 7 is set routes nothing), without storing the pooled
    gradient.  dbias (+= the masked pooled gradient's column sums, the bias gradient of the
    conv in front) needs part, an fp32 scratch of at least lrn_pool_backward_rows(...) x C.
    False when the fused kernel does not serve the shape (nothing was done)."""
    N, H, W, C = dx.shape
    Ho, Wo = pooled.shape[1], pooled.shape[2]
    if not _native_t(dy):
        return False
    rc = _k().cxn_lrn_pool_bwd(pooled.data_ptr(), dy.data_ptr(), state.data_ptr(), dx.data_ptr(), N, H, W, C, Ho, Wo,
                               int(relu_bit), int(nsize), float(alpha), float(beta), float(knorm),
                               dbias.data_ptr() if dbias is not None else None,
                               part.data_ptr() if part is not None else None,
                               part.shape[0] if part is not None else 0, int(_det()), _stream())
    if rc == -1:
        return False
    if rc < 0:
        native.check(rc, "lrn_pool_bwd")
    return True


def lrn_pool_backward_rows(x_shape, pooled_shape, nsize) -> int:
    """Partial rows lrn_pool_backward needs for its bias sum (0: not served)."""
    N, H, W, C = x_shape
    rc = _k().cxn_lrn_pool_bwd(None, None, None, None, N, H, W, C, pooled_shape[1], pooled_shape[2], 1, int(nsize),
                               0.0, 0.0, 1.0, None, None, -1, 0, None)
    return max(int(rc), 0)


def pool_backward_tie_all(x, y, dy, dx, KH, KW, S, P, relu=False):
    """Max-unpool with the reference tie rule (pooling_layer-inl.hpp:55-86): every input
    equal to its window's max y gets that window's gradient; relu: max over relu(x), the
    gradient masked by relu'(x).  y: the saved pooled output."""
    N, H, W, C = x.shape
    Ho, Wo = dy.shape[1], dy.shape[2]
    if not _native_t(x):
        xv = x.clamp_min(0) if relu else x
        g = torch.zeros((N, H + 2 * P + KH + S, W + 2 * P + KW + S, C), dtype=dy.dtype, device=dy.device)
        xp = torch.full_like(g, float("nan"))  # padding never equals a max
        xp[:, P:P + H, P:P + W, :] = xv
        for ho in range(Ho):
            hs = ho * S
            for wo in range(Wo):
                ws = wo * S
                win = xp[:, hs:hs + KH, ws:ws + KW, :]
                eq = (win == y[:, ho:ho + 1, wo:wo + 1, :]).to(g.dtype)
                g[:, hs:hs + KH, ws:ws + KW, :] += eq * dy[:, ho:ho + 1, wo:wo + 1, :]
        g = g[:, P:P + H, P:P + W, :]
        if relu:
            g = g * (x > 0).to(g.dtype)
        dx.copy_(g)
        return
    native.check(_k().cxn_pool_bwd_tie_all(x.data_ptr(), y.data_ptr(), dy.data_ptr(), dx.data_ptr(), N, H, W, C,
                                           Ho, Wo, KH, KW, S, P, int(bool(relu)), _stream()), "pool_bwd_tie_all")


# ----------------------------------------------------------------------------- LRN
def _lrn_norm(x, nsize, alpha, knorm):
    C = x.shape[-1]
    half = nsize // 2
    sq = x * x
    pad = F.pad(sq, (half, half))
    s = sum(pad[..., i:i + C] for i in range(nsize))
    return knorm + alpha / nsize * s


def lrn_forward(x, y, nsize, alpha, beta, knorm):
    if not _native_t(x):
        y.copy_(x * _lrn_norm(x, nsize, alpha, knorm).pow(-beta))
        return
    N, H, W, C = x.shape
    native.check(_k().cxn_lrn_fwd(x.data_ptr(), y.data_ptr(), N * H * W, C, nsize, float(alpha), float(beta),
                                  float(knorm), _stream()), "lrn_fwd")


def lrn_backward_bias(x, dy, dx, nsize, alpha, beta, knorm, dbias, mask_relu=False) -> bool:
    """lrn_backward plus dbias (fp32 [C]) += the column sums of the stored dx: the bias gradient
    of the conv in front, summed on the way out instead of by a later column-sum pass (per-block
    sums in a scratch, added into dbias with atomics: not for deterministic mode).  False when the kernel does not
    serve the shape (nothing was done)."""
    if not _native_t(x):
        return False
    N, H, W, C = x.shape
    part = _workspace(4096 * C, x.device)  # per-block sums, added up by a second launch
    rc = _k().cxn_lrn_bwd_db(x.data_ptr(), dy.data_ptr(), dx.data_ptr(), N * H * W, C, nsize, float(alpha),
                             float(beta), float(knorm), int(bool(mask_relu)), dbias.data_ptr(), part.data_ptr(),
                             part.numel(), _stream())
    if rc == -1:
        return False
    native.check(rc, "lrn_bwd_db")
    return True


def lrn_backward(x, dy, dx, nsize, alpha, beta, knorm, mask_relu=False):
    """dx = d LRN / dx (dx may alias x; it must not alias dy).  mask_relu: x is relu(z) of a
    fused producer, so dx is also multiplied by relu'(z) = (x > 0)."""
    if not _native_t(x):
        norm = _lrn_norm(x, nsize, alpha, knorm)
        t = dy * x * norm.pow(-beta - 1)
        C = x.shape[-1]
        half = nsize // 2
        tp = F.pad(t, (half, half))
        s = sum(tp[..., i:i + C] for i in range(nsize))
        g = dy * norm.pow(-beta) - 2 * beta * alpha / nsize * x * s
        if mask_relu:
            g = torch.where(x > 0, g, torch.zeros_like(g))
        dx.copy_(g)
        return
    N, H, W, C = x.shape
    native.check(_k().cxn_lrn_bwd(x.data_ptr(), dy.data_ptr(), dx.data_ptr(), N * H * W, C, nsize, float(alpha),
                                  float(beta), float(knorm), int(bool(mask_relu)), _stream()), "lrn_bwd")


# ----------------------------------------------------------------------------- activations
def _act_ref(kind, x, b):
    if kind == "relu":
        return x.clamp_min(0)
    if kind == "sigmoid":
        return torch.sigmoid(x)
    if kind == "tanh":
        return torch.tanh(x)
    return torch.where(x > 0, x, x / b)


def _act_grad_ref(kind, y, b):
    if kind == "relu":
        return (y > 0).to(y.dtype)
    if kind == "sigmoid":
        return y * (1 - y)
    if kind == "tanh":
        return 1 - y * y
    return torch.where(y > 0, torch.ones_like(y), torch.full_like(y, 1.0 / b))


def act_forward(kind, x, y, y2=None, b=5.0):
    """y = f(x); when y2 is given it also receives f(x) (in-place write of the input node)."""
    if not _native_t(x):
        out = _act_ref(kind, x, b)
        y.copy_(out)
        if y2 is not None:
            y2.copy_(out)
        return
    native.check(_k().cxn_act_fwd(x.data_ptr(), y.data_ptr(), y2.data_ptr() if y2 is not None else None, x.numel(),
                                  ACT_KIND[kind], float(b), _stream()), "act_fwd")


def act_backward(kind, y, dy, dx, b=5.0):
    """dx = dy * f'(y) (gradient in terms of the forward output)."""
    if not _native_t(y):
        dx.copy_(dy * _act_grad_ref(kind, y, b))
        return
    native.check(_k().cxn_act_bwd(y.data_ptr(), dy.data_ptr(), dx.data_ptr(), y.numel(), ACT_KIND[kind], float(b),
                                  _stream()), "act_bwd")


# ----------------------------------------------------------------------------- dropout
def _hash_u32(idx: torch.Tensor, seed: int) -> torch.Tensor:
    # identical to hash_u32 in nn_kernels.hip, in int64 arithmetic masked to 32 bits
    M = 0xFFFFFFFF
    x = idx ^ ((seed * 0x9E3779B9) & M)
    x = x ^ (x >> 16); x = (x * 0x7FEB352D) & M
    x = x ^ (x >> 15); x = (x * 0x846CA68B) & M
    x = x ^ (x >> 16)
    return x


def effective_seed(seed: int, counter=None) -> int:
    if counter is None:
        return seed & 0xFFFFFFFF
    c = int(counter.item()) & 0xFFFFFFFF
    return int(_hash_u32(torch.tensor([c], dtype=torch.int64), seed & 0xFFFFFFFF).item())


def dropout_mask_ref(n: int, seed: int, pkeep: float, device="cpu") -> torch.Tensor:
    idx = torch.arange(n, dtype=torch.int64, device=device)
    t = min(int(pkeep * 4294967296.0), 0xFFFFFFFF)
    return (_hash_u32(idx, seed & 0xFFFFFFFF) < t).float() / pkeep


def dropout_apply(x, y, seed: int, pkeep: float, counter=None):
    """y = x * mask(seed[, counter]) / pkeep; forward and backward use the same call (x may alias y).

    counter: optional int32 device tensor; the mask seed is hash(counter, seed), read on
    device, so a captured HIP graph draws a new mask on every replay.
    """
    if not _native_t(x):
        m = dropout_mask_ref(x.numel(), effective_seed(seed, counter), pkeep, x.device).view_as(x).to(x.dtype)
        y.copy_(x * m)
        return
    native.check(_k().cxn_dropout(x.data_ptr(), y.data_ptr(), x.numel(), seed & 0xFFFFFFFF,
                                  counter.data_ptr() if counter is not None else None, float(pkeep),
                                  _stream()), "dropout")


# ----------------------------------------------------------------------------- softmax / losses
def softmax_forward(x, y, p32=None):
    """Row softmax of x[rows][K] into y (and the fp32 copy p32)."""
    if not _native_t(x):
        p = torch.softmax(x.float(), dim=1)
        y.copy_(p)
        if p32 is not None:
            p32.copy_(p)
        return
    rows, K = x.shape
    native.check(_k().cxn_softmax(x.data_ptr(), y.data_ptr(), p32.data_ptr() if p32 is not None else None, rows, K,
                                  _stream()), "softmax")


LOSS_KIND = {"softmax": 0, "l2": 1, "multi_logistic": 2}


def loss_grad(kind: str, node, label, scale: float, p32=None):
    """node <- (pred - target) * scale, pred = p32 if given else node.  label fp32 [rows][lw]."""
    rows, K = node.shape
    lw = label.shape[1]
    if not _native_t(node):
        p = p32 if p32 is not None else node
        if kind == "softmax":
            oh = torch.zeros_like(p)
            oh.scatter_(1, label[:, :1].long(), 1.0)
            node.copy_((p - oh) * scale)
        else:
            node.copy_((p - label) * scale)
        return
    native.check(_k().cxn_loss_grad(p32.data_ptr() if p32 is not None else None, node.data_ptr(), label.data_ptr(),
                                    rows, K, lw, float(scale), LOSS_KIND[kind], _stream()), "loss_grad")


# ----------------------------------------------------------------------------- reductions / misc
_WS = {}


def _workspace(n: int, device) -> torch.Tensor:
    """Reusable fp32 scratch (per device) for per-block partial sums; used in stream
    order on the compute stream only."""
    key = str(device)
    t = _WS.get(key)
    if t is None or t.numel() < n:
        from .mode import retire
        retire(t)  # a recorded / captured step may still point at it
        t = torch.empty(max(n, 1 << 16), dtype=torch.float32, device=device)
        _WS[key] = t
    return t


def bias_grad(dy2d, db, mask=None):
    """db[C] += sum over rows of dy2d[rows][C].  mask (uint8 [rows][C], optional): max-pool
    offsets recorded with relu' in bit 7 (pool_forward(mark_mask=True)); an entry whose bit 7
    is set counts as zero -- dy2d is then a max-pool's output gradient and the sum is the
    bias gradient of the conv in front of the pool (see colsum_multi)."""
    if not _native_t(dy2d):
        if mask is not None:
            dy2d = dy2d * (mask < 128).to(dy2d.dtype)
        db.add_(dy2d.float().sum(0))
        return
    if mask is not None or (bias_fast_ok(dy2d) and not _det()):
        # one launch (per-block partials, one atomic per channel per block); the two-pass
        # colsum below keeps a fixed summation order for deterministic mode
        bias_grad_multi([(dy2d, db, mask)])
        return
    if not dy2d.is_contiguous():  # a channel slice of a zero-copy ch_concat output
        dy2d = _rows_contiguous(dy2d)
    rows, C = dy2d.shape
    n = max(4096, -(-rows // 512)) * C
    ws = _workspace(n, dy2d.device)
    native.check(_k().cxn_colsum(dy2d.data_ptr(), db.data_ptr(), rows, C, ws.data_ptr(), ws.numel(), _stream()),
                 "colsum")


def _rows_contiguous(d):
    """Contiguous copy of a [rows][C] GPU view with unit column stride (a channel slice of a
    wider NHWC buffer) through the library's channel copy: a torch .contiguous() would not be
    part of a recorded launch list, and its replay would read a stale temporary."""
    rows, C = d.shape
    if d.stride(1) != 1:
        raise ValueError("bias gradient: unit column stride expected")
    out = torch.empty((rows, C), dtype=d.dtype, device=d.device)
    native.check(_k().cxn_channel_copy(d.data_ptr(), d.stride(0), 0, out.data_ptr(), C, 0, C, rows, 0, _stream()),
                 "channel_copy")
    return out


def _det() -> bool:
    from .gemm import deterministic
    return deterministic()


def _rows_ok(d) -> bool:
    """[rows][C] with unit column stride and a row stride that is a multiple of 8 elements
    (contiguous, or a channel slice of a wider NHWC buffer), 16-byte aligned."""
    return d.dim() == 2 and d.stride(1) == 1 and (d.stride(0) % 8 == 0 or d.shape[0] == 1) and \
        d.stride(0) >= d.shape[1] and d.data_ptr() % 16 == 0


def bias_fast_ok(d, m=None) -> bool:
    """Served by the one-launch colsum_multi kernel (no workspace, no temporaries)."""
    return _native_t(d) and d.shape[1] % 8 == 0 and _rows_ok(d) and \
        (m is None or (m.is_contiguous() and d.is_contiguous()))


def bias_grad_multi(items):
    """Every (dy2d, db[, mask]) of `items`: db[C] += sum over rows of dy2d (masked as in
    bias_grad), in one launch for the GPU tensors with C % 8 == 0 (the rest one by one)."""
    items = [tuple(it) + (None,) * (3 - len(it)) for it in items]
    fast = [it for it in items if bias_fast_ok(it[0], it[2])]
    for d, b, m in items:
        if not bias_fast_ok(d, m):
            if m is not None and _native_t(d):
                # (no torch math here: a launch list would not record it) a contiguous copy of
                # d makes the one-launch masked kernel applicable
                dc = _rows_contiguous(d) if not d.is_contiguous() else d
                if not (bias_fast_ok(dc, m) and m.is_contiguous()):
                    raise RuntimeError(f"masked bias gradient: no GPU kernel for {tuple(d.shape)}")
                fast.append((dc, b, m))
            else:
                bias_grad(d, b, m)
    if not fast:
        return
    n = len(fast)
    dys = (ctypes.c_void_p * n)(*[d.data_ptr() for d, _, _ in fast])
    dbs = (ctypes.c_void_p * n)(*[b.data_ptr() for _, b, _ in fast])
    rows = (ctypes.c_long * n)(*[d.shape[0] for d, _, _ in fast])
    cs = (ctypes.c_int * n)(*[d.shape[1] for d, _, _ in fast])
    lds = (ctypes.c_long * n)(*[d.stride(0) if d.shape[0] > 1 else d.shape[1] for d, _, _ in fast])
    masks = None
    if any(m is not None for _, _, m in fast):
        masks = (ctypes.c_void_p * n)(*[m.data_ptr() if m is not None else None for _, _, m in fast])
    native.check(_k().cxn_colsum_multi(ctypes.cast(dys, ctypes.c_void_p), ctypes.cast(dbs, ctypes.c_void_p),
                                       ctypes.cast(rows, ctypes.c_void_p), ctypes.cast(cs, ctypes.c_void_p),
                                       ctypes.cast(masks, ctypes.c_void_p) if masks is not None else None, n,
                                       _stream(), ctypes.cast(lds, ctypes.c_void_p)), "colsum_multi")


def cast_to_bf16(src_f32, dst_bf16):
    if not _native_t(src_f32):
        dst_bf16.copy_(src_f32)
        return
    native.check(_k().cxn_cast_f32_bf16(src_f32.data_ptr(), dst_bf16.data_ptr(), src_f32.numel(), _stream()), "cast")


def add(a, b, y):
    if not _native_t(a):
        torch.add(a, b, out=y)
        return
    native.check(_k().cxn_add_bf16(a.data_ptr(), b.data_ptr(), y.data_ptr(), a.numel(), _stream()), "add")


def _vec8(*ts):
    return all(t.is_contiguous() and t.dtype == torch.bfloat16 and t.data_ptr() % 16 == 0 and t.numel() % 8 == 0
               for t in ts)


def fanout_copy(src, dsts):
    """dst[k] = src for every dst (split forward): the source is read once per 4 copies."""
    if not _native_t(src) or not _vec8(src, *dsts):
        for d in dsts:
            d.copy_(src)
        return
    for k in range(0, len(dsts), 4):
        ds = list(dsts[k:k + 4])
        ptr = [d.data_ptr() for d in ds] + [None] * (4 - len(ds))
        native.check(_k().cxn_fanout_bf16(src.data_ptr(), *ptr, len(ds), src.numel(), _stream()), "fanout")


def sum_into(y, srcs, mask_relu=False):
    """y = sum(srcs) (split backward), accumulated in fp32 and rounded once per 4 terms;
    y may alias srcs[0].  mask_relu: y holds relu(z) on entry (a zero-copy ch_concat of fused
    conv+relu branches, NeuralNet._fuse_concat) and the sum is kept only where y > 0."""
    if len(srcs) == 1:
        if mask_relu:
            C = y.shape[-1]
            channel_copy(srcs[0], 0, y, 0, C, mask_relu=True)
        elif y.data_ptr() != srcs[0].data_ptr():
            y.copy_(srcs[0])
        return
    if not _native_t(y) or not _vec8(y, *srcs) or (mask_relu and len(srcs) > 4):
        acc = srcs[0].float()
        for t in srcs[1:]:
            acc = acc + t.float()
        if mask_relu:
            acc = torch.where(y > 0, acc, torch.zeros_like(acc))
        y.copy_(acc)
        return
    first, rest = srcs[0], list(srcs[1:])
    while rest:
        part = [first] + rest[:3]
        rest = rest[3:]
        ptr = [t.data_ptr() for t in part] + [None] * (4 - len(part))
        native.check(_k().cxn_sum_bf16(*ptr, len(part), y.data_ptr(), y.numel(), _stream(), int(mask_relu)), "sum")
        first = y


def concat_channels(ins, out, backward=False, mask=()):
    """NHWC channel concat of `ins` into `out` (forward) or the gradient slices of `out` back
    into `ins` (backward; relu' for the input indices in `mask`), one launch on the GPU.
    Returns False when the kernel does not cover the shapes (the caller copies per input)."""
    if not _native_t(out) or len(ins) > 4:
        return False
    n = len(ins)
    Ct = out.shape[-1]
    npix = out.numel() // Ct
    if any(t.numel() // t.shape[-1] != npix or not t.is_contiguous() or t.data_ptr() % 16 for t in ins) or \
            not out.is_contiguous() or out.data_ptr() % 16:
        return False
    ptrs = (ctypes.c_void_p * n)(*[t.data_ptr() for t in ins])
    cs = (ctypes.c_int * n)(*[t.shape[-1] for t in ins])
    m = sum(1 << k for k in mask)
    rc = _k().cxn_concat(ctypes.cast(ptrs, ctypes.c_void_p), ctypes.cast(cs, ctypes.c_void_p), n, out.data_ptr(), Ct,
                         npix, int(bool(backward)), m, _stream())
    if rc == -1:
        return False
    native.check(rc, "concat")
    return True


def channel_copy(src, soff, dst, doff, cc, accumulate=False, mask_relu=False):
    """dst[..., doff:doff+cc] (+)= src[..., soff:soff+cc] for NHWC tensors with equal pixel counts.
    mask_relu: dst holds relu(z) on entry; the copy keeps src only where dst > 0 (relu')."""
    Cs, Cd = src.shape[-1], dst.shape[-1]
    npix = src.numel() // Cs
    if not _native_t(src):
        d = dst.view(npix, Cd)[:, doff:doff + cc]
        s = src.view(npix, Cs)[:, soff:soff + cc]
        if accumulate:
            d.add_(s)
        elif mask_relu:
            d.copy_(torch.where(d > 0, s, torch.zeros_like(s)))
        else:
            d.copy_(s)
        return
    mode = 2 if mask_relu else int(bool(accumulate))
    native.check(_k().cxn_channel_copy(src.data_ptr(), Cs, soff, dst.data_ptr(), Cd, doff, cc, npix,
                                       mode, _stream()), "channel_copy")
