"""Ops of the less common layers: batch_norm, prelu, insanity, insanity_max_pooling.

GPU: csrc/kernels/layer_kernels.hip.  CPU: the same formulas in fp32 torch, with the SAME
counter-hash random draws as the kernels (element index of the NHWC buffer, seed
hash(step counter, layer seed)), so the CPU executor is an exact oracle for the GPU one.
"""
from __future__ import annotations

import torch

from .. import native
from .mode import native as _native_t
from .gemm import _stream
from .nn import _hash_u32, effective_seed


def _k():
    return native.kernels()


def _ctr(counter):
    return counter.data_ptr() if counter is not None else None


def uniform_ref(n: int, seed: int, device="cpu") -> torch.Tensor:
    """u01 of layer_kernels.hip: hash(i, seed) * 2^-32 in fp32."""
    idx = torch.arange(n, dtype=torch.int64, device=device)
    return _hash_u32(idx, seed & 0xFFFFFFFF).to(torch.float32) * 2.3283064365386963e-10


def rand_fill(t: torch.Tensor, seed: int, dist: str, a: float, b: float):
    """Fill fp32 tensor t in place: dist "uniform" a + (b - a) u, "normal" a + b z.  On the
    GPU one rand_fill launch (layer_kernels.hip); on the host the same counter hash in int64
    arithmetic and the same float32 Box-Muller, chunked to bound the index arrays."""
    assert t.dtype == torch.float32 and t.is_contiguous()
    n = t.numel()
    d = 0 if dist == "uniform" else 1
    seed &= 0xFFFFFFFF
    if t.is_cuda:  # fp32 kernel: also in reference-precision mode
        native.check(_k().cxn_rand_fill(t.data_ptr(), n, seed, d, float(a), float(b), _stream()), "rand_fill")
        return t
    flat = t.view(-1)
    step = 1 << 24
    scale = torch.tensor(5.9604644775390625e-08, dtype=torch.float32)
    for lo in range(0, n, step):
        idx = torch.arange(lo, min(n, lo + step), dtype=torch.int64)
        u1 = (_hash_u32(2 * idx, seed) >> 8).to(torch.float32) * scale
        if d == 0:
            v = torch.tensor(a, dtype=torch.float32) + torch.tensor(b - a, dtype=torch.float32) * u1
        else:
            u2 = (_hash_u32(2 * idx + 1, seed) >> 8).to(torch.float32) * scale
            z = torch.sqrt(-2.0 * torch.log(1.0 - u1)) * torch.cos(6.283185307179586 * u2)
            v = torch.tensor(a, dtype=torch.float32) + torch.tensor(b, dtype=torch.float32) * z
        flat[lo:lo + idx.numel()] = v
    return t


# ----------------------------------------------------------------------------- batch norm
class BNState:
    """Per-layer device buffers: mean, inv (fp32 [C]), workspaces, the saved input copy."""

    def __init__(self, C, device):
        self.mean = torch.zeros(C, dtype=torch.float32, device=device)
        self.inv = torch.zeros(C, dtype=torch.float32, device=device)
        self.ws = torch.zeros(3 * C, dtype=torch.float32, device=device)
        self.coef = torch.zeros(3 * C, dtype=torch.float32, device=device)
        self.xsave = None


def bn_forward(x2d, y2d, slope, bias, eps, st: BNState, is_train: bool):
    """Reference BatchNormLayer::Forward (batch_norm_layer-inl.hpp:98-137): batch statistics in
    train AND test; in training the input node is overwritten with x-hat and a copy of x is
    kept for backward."""
    rows, C = x2d.shape
    if not _native_t(x2d):
        x = x2d.float()
        mean = x.mean(0)
        var = ((x - mean) ** 2).mean(0)
        inv = 1.0 / torch.sqrt(var + eps)
        xh = (x - mean) * inv
        st.mean.copy_(mean)
        st.inv.copy_(inv)
        if is_train:
            st.xsave = x2d.clone()
            x2d.copy_(xh)
        y2d.copy_(xh * slope + bias)
        return
    k = _k()
    native.check(k.cxn_bn_stats(x2d.data_ptr(), st.ws.data_ptr(), st.mean.data_ptr(), st.inv.data_ptr(), rows, C,
                                float(eps), _stream()), "bn_stats")
    xsave = None
    if is_train:
        if st.xsave is None or st.xsave.shape != x2d.shape:
            st.xsave = torch.empty_like(x2d)
        xsave = st.xsave
    # xhat overwrites x in place (element-wise: safe with y distinct)
    native.check(k.cxn_bn_fwd(x2d.data_ptr(), y2d.data_ptr(), x2d.data_ptr() if is_train else None,
                              xsave.data_ptr() if xsave is not None else None, st.mean.data_ptr(), st.inv.data_ptr(),
                              slope.data_ptr(), bias.data_ptr(), rows, C, _stream()), "bn_fwd")


def affine_forward(x2d, y2d, mean, inv, slope, bias):
    """y = (x - mean) * inv * slope + bias per channel (GPU; the bias layer uses it with 0/1/1)."""
    rows, C = x2d.shape
    native.check(_k().cxn_bn_fwd(x2d.data_ptr(), y2d.data_ptr(), None, None, mean.data_ptr(), inv.data_ptr(),
                                 slope.data_ptr(), bias.data_ptr(), rows, C, _stream()), "affine")


def bn_backward(g2d, dx2d, slope, gslope, gbias, st: BNState, prop_grad: bool):
    """Reference BatchNormLayer::Backprop (batch_norm_layer-inl.hpp:138-179)."""
    rows, C = g2d.shape
    if not _native_t(g2d):
        x = st.xsave.float()
        g = g2d.float()
        mean, inv = st.mean, st.inv
        scale = 1.0 / rows
        d = x - mean
        ve = 1.0 / (inv * inv)
        gvar = (g * slope * d).sum(0) * -0.5 * inv / ve
        gexp = (g * slope).sum(0) * -inv + gvar * scale * (-2.0 * d).sum(0)
        gslope.add_((g * d).sum(0) * inv)
        gbias.add_(g.sum(0))
        if prop_grad:
            dx2d.copy_(g * slope * inv + gvar * scale * 2.0 * d + gexp * scale)
        return
    if not prop_grad:
        # weight gradients only: the coefficient kernel also accumulates gslope/gbias
        dx2d = torch.empty_like(g2d)
    native.check(_k().cxn_bn_bwd(g2d.data_ptr(), st.xsave.data_ptr(), dx2d.data_ptr(), st.mean.data_ptr(),
                                 st.inv.data_ptr(), slope.data_ptr(), gslope.data_ptr(), gbias.data_ptr(),
                                 st.ws.data_ptr(), st.coef.data_ptr(), rows, C, _stream()), "bn_bwd")


# ----------------------------------------------------------------------------- prelu
def _prelu_mask_ref(x2d, slope, seed, counter, rnd):
    rows, C = x2d.shape
    m = slope.float().expand(rows, C)
    if rnd > 0:
        u = uniform_ref(rows * C, effective_seed(seed, counter), x2d.device).view(rows, C)
        m = m * (1 + u * rnd * 2.0 - rnd)
    return m.clamp(0, 1)


def prelu_forward(x2d, y2d, slope, seed, counter, rnd):
    """y = x > 0 ? x : x * clamp(slope * noise, 0, 1)   (reference prelu_layer-inl.hpp:111-135)."""
    rows, C = x2d.shape
    if not _native_t(x2d):
        x = x2d.float()
        y2d.copy_(torch.where(x > 0, x, x * _prelu_mask_ref(x2d, slope, seed, counter, rnd)))
        return
    native.check(_k().cxn_prelu(x2d.data_ptr(), None, y2d.data_ptr(), slope.data_ptr(), rows, C, seed & 0xFFFFFFFF,
                                _ctr(counter), float(rnd), 0, _stream()), "prelu_fwd")


def prelu_backward(x2d, g2d, dx2d, slope, gslope, seed, counter, rnd, prop_grad, ws=None):
    """gslope += sum min(x, 0) * g; dx = x > 0 ? g : g * mask  (reference :137-152).  dx may alias x."""
    rows, C = x2d.shape
    if not _native_t(x2d):
        x, g = x2d.float(), g2d.float()
        gslope.add_((torch.clamp(x, max=0) * g).sum(0))
        if prop_grad:
            dx2d.copy_(torch.where(x > 0, g, g * _prelu_mask_ref(x2d, slope, seed, counter, rnd)))
        return
    k = _k()
    if ws is None:
        ws = torch.empty(3 * C, dtype=torch.float32, device=x2d.device)
    native.check(k.cxn_chan_reduce(x2d.data_ptr(), g2d.data_ptr(), None, ws.data_ptr(), rows, C, 3, _stream()),
                 "prelu_slope_grad")
    gslope.add_(ws[:C])
    if prop_grad:
        native.check(k.cxn_prelu(x2d.data_ptr(), g2d.data_ptr(), dx2d.data_ptr(), slope.data_ptr(), rows, C,
                                 seed & 0xFFFFFFFF, _ctr(counter), float(rnd), 1, _stream()), "prelu_bwd")


# ----------------------------------------------------------------------------- insanity
def _insanity_div_ref(n, lb, ub, train, seed, counter, device):
    if not train:
        return torch.full((n,), 0.5 * (lb + ub), dtype=torch.float32, device=device)
    u = uniform_ref(n, effective_seed(seed, counter), device)
    return lb + u * (ub - lb)


def insanity_forward(x, y, y2, lb, ub, train, seed, counter):
    """y (and y2) = x > 0 ? x : x / U[lb, ub)  (test: / ((lb + ub) / 2))."""
    if not _native_t(x):
        d = _insanity_div_ref(x.numel(), lb, ub, train, seed, counter, x.device).view_as(x)
        xf = x.float()
        out = torch.where(xf > 0, xf, xf / d)
        y.copy_(out)
        if y2 is not None:
            y2.copy_(out)
        return
    native.check(_k().cxn_insanity(x.data_ptr(), None, y.data_ptr(), y2.data_ptr() if y2 is not None else None,
                                   x.numel(), float(lb), float(ub), int(train), seed & 0xFFFFFFFF, _ctr(counter), 0,
                                   _stream()), "insanity_fwd")


def insanity_backward(y, g, dx, lb, ub, train, seed, counter):
    """dx = y > 0 ? g : g / d with forward's draws (dx may alias y)."""
    if not _native_t(y):
        d = _insanity_div_ref(y.numel(), lb, ub, train, seed, counter, y.device).view_as(y)
        yf, gf = y.float(), g.float()
        dx.copy_(torch.where(yf > 0, gf, gf / d))
        return
    native.check(_k().cxn_insanity(y.data_ptr(), g.data_ptr(), dx.data_ptr(), None, y.numel(), float(lb), float(ub),
                                   int(train), seed & 0xFFFFFFFF, _ctr(counter), 1, _stream()), "insanity_bwd")


# ----------------------------------------------------------------------------- insanity pooling
def _shift_ref(N, H, W, C, keep, seed, counter, device):
    """Flat NHWC source index each input element is read from."""
    u = uniform_ref(N * H * W * C, effective_seed(seed, counter), device).view(N, H, W, C)
    d = (1.0 - keep) / 4.0
    yy = torch.arange(H, device=device).view(1, H, 1, 1).expand(N, H, W, C)
    xx = torch.arange(W, device=device).view(1, 1, W, 1).expand(N, H, W, C)
    ly = torch.where((u >= keep) & (u < keep + d), (yy - 1).clamp_min(0), yy)
    ly = torch.where((u >= keep + d) & (u < keep + 2 * d), (yy + 1).clamp_max(H - 1), ly)
    lx = torch.where((u >= keep + 2 * d) & (u < keep + 3 * d), (xx - 1).clamp_min(0), xx)
    lx = torch.where(u >= keep + 3 * d, (xx + 1).clamp_max(W - 1), lx)
    n = torch.arange(N, device=device).view(N, 1, 1, 1)
    c = torch.arange(C, device=device).view(1, 1, 1, C)
    return ((n * H + ly) * W + lx) * C + c


def ins_pool_forward(x, y, ysave, K, S, keep, seed, counter):
    N, H, W, C = x.shape
    Ho, Wo = y.shape[1], y.shape[2]
    if not _native_t(x):
        src = x.reshape(-1)[_shift_ref(N, H, W, C, keep, seed, counter, x.device)].float()  # shifted image
        out = torch.full((N, Ho, Wo, C), float("-inf"), device=x.device)
        for py in range(Ho):
            for px in range(Wo):
                win = src[:, py * S:min(py * S + K, H), px * S:min(px * S + K, W), :]
                out[:, py, px, :] = win.amax(dim=(1, 2))
        y.copy_(out)
        if ysave is not None:
            ysave.copy_(out)
        return
    native.check(_k().cxn_ins_pool_fwd(x.data_ptr(), y.data_ptr(), ysave.data_ptr() if ysave is not None else None,
                                       N, H, W, C, Ho, Wo, K, S, float(keep), seed & 0xFFFFFFFF, _ctr(counter),
                                       _stream()), "ins_pool_fwd")


def ins_pool_backward(x, ypool, gy, dx, K, S, keep, seed, counter):
    """dx must not alias x."""
    N, H, W, C = x.shape
    Ho, Wo = gy.shape[1], gy.shape[2]
    if not _native_t(x):
        vsrc = x.reshape(-1)[_shift_ref(N, H, W, C, keep, seed, counter, x.device)].float()
        out = torch.zeros(N, H, W, C, device=x.device)
        yp, g = ypool.float(), gy.float()
        for py in range(Ho):
            for px in range(Wo):
                y0, y1, x0, x1 = py * S, min(py * S + K, H), px * S, min(px * S + K, W)
                hit = (vsrc[:, y0:y1, x0:x1, :] == yp[:, py:py + 1, px:px + 1, :]).float()
                out[:, y0:y1, x0:x1, :] += hit * g[:, py:py + 1, px:px + 1, :]
        dx.copy_(out)
        return
    native.check(_k().cxn_ins_pool_bwd(x.data_ptr(), ypool.data_ptr(), gy.data_ptr(), dx.data_ptr(), N, H, W, C, Ho,
                                       Wo, K, S, float(keep), seed & 0xFFFFFFFF, _ctr(counter), _stream()),
                 "ins_pool_bwd")
