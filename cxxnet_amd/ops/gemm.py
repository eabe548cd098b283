"""GEMM-shaped ops: convolution (fwd / data-grad / weight-grad) and fully-connected.

Layout contract (both devices):
  * activations are NHWC: x[N][H][W][C];  a "matrix" node (B,1,1,N) is x[B][N].
  * conv weights are [Cout][KH][KW][Cin/groups] (channels fastest).
  * fc weights are [nout][nin] (reference layout, src/layer/fullc_layer-inl.hpp:29).
On the GPU, activations/weights are bf16 and every op runs the hand-written MFMA
kernel in csrc/kernels/gemm_mfma.hip.  On the CPU, the same semantics run in fp32
through torch (the reference's CPU path; also the numerics oracle for tests).

Reference: src/layer/convolution_layer-inl.hpp:70-155 (im2col + GEMM per group),
src/layer/fullc_layer-inl.hpp:101-130.
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass

import torch
import torch.nn.functional as F

from .. import native
from .mode import frozen, native as _native_t

DIRECT_K, DIRECT_MN, GATHER_K, GATHER_MN = 0, 1, 2, 3
EPI_BF16, EPI_F32, EPI_F32_ACC, EPI_F32_ATOMIC = 0, 1, 2, 3
NUM_CU = 256


_RAW_STREAM = getattr(torch._C, "_cuda_getCurrentRawStream", None)
_CUR_DEV = getattr(torch._C, "_cuda_getDevice", None)


def _stream():
    """The current HIP stream handle.  Every library launch asks for it: the raw C accessors
    cost ~0.3 us where torch.cuda.current_stream() (lazy-init and availability checks, a Stream
    object) cost several, 60+ times per step."""
    if _RAW_STREAM is not None:
        return _RAW_STREAM(_CUR_DEV())
    return ctypes_stream(torch.cuda.current_stream())


def ctypes_stream(s) -> int:
    return s.cuda_stream


@dataclass
class ConvGeom:
    N: int
    H: int
    W: int
    C: int          # physical input channels (>= logical, first layer may be padded)
    Ho: int
    Wo: int
    Cout: int
    KH: int
    KW: int
    stride: int
    pad_y: int
    pad_x: int
    groups: int

    @property
    def cg_in(self):
        return self.C // self.groups

    @property
    def cg_out(self):
        return self.Cout // self.groups

    @property
    def kdim(self):
        return self.KH * self.KW * self.cg_in


def _span_bytes(t) -> int:
    """Bytes from t's first element to one past its last: numel * size for a contiguous tensor;
    for a strided view (a channel slice of a zero-copy ch_concat buffer) the span its elements
    cover, so the kernel's buffer descriptor still ends at the view's last element."""
    if t.is_contiguous() or t.numel() == 0:
        return t.numel() * t.element_size()
    return (sum((n - 1) * st for n, st in zip(t.shape, t.stride())) + 1) * t.element_size()


def _pix(t) -> int:
    """Pixel stride (elements) of an NHWC activation: its channel count when contiguous, the
    full buffer's channel count for a channel slice."""
    return t.shape[-1] if t.is_contiguous() else t.stride(-2)


def _like(t) -> torch.Tensor:
    """Uninitialised tensor with t's shape AND strides (tuning scratch for a strided output:
    the kernel is launched with the output's row stride)."""
    if t.is_contiguous():
        return torch.empty_like(t)
    base = torch.empty(_span_bytes(t) // t.element_size(), dtype=t.dtype, device=t.device)
    return base.as_strided(t.shape, t.stride())


def _op(t, gstride=0, ld=0, rows=0, kdim=0, **geo):
    o = native.CxnOperand()
    o.ptr = t.data_ptr()
    o.nbytes = _span_bytes(t)  # bound of the kernel's buffer descriptor
    o.gstride = gstride
    o.ld = ld
    o.rows = rows
    o.kdim = kdim
    o.H = geo.get("H", 0); o.W = geo.get("W", 0); o.C = geo.get("C", 0)
    o.Ho = geo.get("Ho", 0); o.Wo = geo.get("Wo", 0)
    o.KH = geo.get("KH", 1); o.KW = geo.get("KW", 1)
    o.stride = geo.get("stride", 1); o.pad_h = geo.get("pad_h", 0); o.pad_w = geo.get("pad_w", 0)
    o.dil = geo.get("dil", 1); o.Cg = geo.get("Cg", 1)
    return o


# tile id -> (BM, BN); must match TILES in gemm_mfma.hip
TILES = {0: (128, 128), 1: (64, 64), 2: (64, 128), 3: (32, 128), 4: (96, 128), 5: (128, 64), 6: (128, 96),
         7: (128, 32)}
CONV_FWD_TILES = (0, 4, 2, 3, 1)
CONV_FWD_TILES_V4 = (0, 4, 2, 3)
WGRAD_TILES = (0, 5, 6, 7)
FC_TILES = (0, 5, 1)


def _cdiv(a, b):
    return -(-a // b)


def _pick(candidates, rows_i, rows_j, groups, min_blocks=2 * NUM_CU):
    """Least padded work first; among equals the larger tile; then enough blocks to
    fill the chip (256 CUs x 2 blocks)."""
    def cost(t):
        bm, bn = TILES[t]
        nb = _cdiv(rows_i, bm) * _cdiv(rows_j, bn) * groups
        padded = _cdiv(rows_i, bm) * bm * _cdiv(rows_j, bn) * bn
        starve = max(0.0, 1.0 - nb / min_blocks)  # fraction of the chip left idle
        return (padded * (1.0 + starve), -bm * bn)
    return min(candidates, key=cost)


# ----------------------------------------------------------------------------- LDS-DMA kernel
# gemm_glds.hip: both operands K-major (conv fwd / dgrad, fc fwd), 4 waves, one block per CU.
# Only the tiles the shipped table (glds_tune_gfx950.json) or a default pick uses are compiled;
# tests/test_tile_table_cpu.py checks this dict against the kernels' dispatch switches.  Tiles
# measured and retired in rounds 2-5 are listed in gemm_glds.hip's dispatch comment.
GLDS_TILES = {1: (128, 128), 2: (128, 128), 7: (64, 128), 10: (128, 64), 15: (64, 64), 17: (128, 128),
              # 8 waves, two per SIMD
              21: (256, 256), 23: (128, 128), 25: (64, 512),
              # pipelined variants (gemm_glds.hip PIPE: setprio around the MFMA clusters, both
              # k-steps' fragments read ahead of the MFMAs) and 8-wave 128x256 / 64x256 tiles
              30: (128, 256), 31: (128, 256), 34: (256, 256), 37: (64, 128), 38: (128, 256), 39: (64, 256),
              40: (128, 128), 41: (128, 128),
              # 96-row / 96-column tiles: 96-channel convs (AlexNet conv1) without idle rows
              72: (96, 128), 75: (64, 96),
              # 32-row tiles (K-major A): convs with 16..48 output channels (GoogLeNet's 5x5-reduce and
              # pool-projection layers) and their data-gradients onto 16..48 input channels
              76: (32, 128), 77: (32, 64), 78: (32, 256),
              # 48 computed rows on 64 staged (AlexNet conv2's data-gradient: 48 channels per group)
              79: (48, 128),
              # 8-wave 3/4-width tile against wave quantisation: AlexNet conv3's data-gradient has
              # 169 256x256 tiles for 256 CUs, 226 of 256x192
              82: (256, 192),
              # one wave per SIMD, address-free DMA issue (gemm_4w.hip)
              114: (128, 128),
              # direct 3x3 halo convolution (conv_halo.hip): output channels x 256-pixel patch, and
              # the persistent patch walk for one 128-channel output block (133)
              130: (64, 256), 131: (128, 256), 133: (128, 256),
              # direct 3x3 weight-gradient on resident halo / dy tiles (conv_wgrad_halo.hip): 64 x 64
              # channel pairs, persistent over 128-pixel patches (140 auto width, 141 16, 142 32)
              140: (64, 64), 141: (64, 64), 142: (64, 64)}
# operand loaders of gemm_glds.hip
GL_K, GL_KG, GL_MN, GL_MNG, GL_KR = 0, 1, 2, 3, 4  # K_DIRECT, K_GATHER, MN_DIRECT, MN_GATHER, K_ROWGATHER
EPI_F32_ACC_G, EPI_F32_ATOMIC_G, EPI_BF16_DB_G = 2, 3, 5
_glds_cfg = {"on": os.environ.get("CXXNET_GEMM_GLDS", "1") != "0",
             "tile": int(os.environ.get("CXXNET_GLDS_TILE", "-1")),
             "tune": os.environ.get("CXXNET_GEMM_TUNE", "1") != "0",
             # op classes routed to it: conv fwd, conv1-style row-gather fwd, conv dgrad, conv wgrad, fc fwd, fc wgrad
             "ops": set(os.environ.get("CXXNET_GLDS_OPS", "cf,cr,cd,cw,fc,fw").split(","))}
# conv weight-grad ("cw"): on every AlexNet layer together the LDS-DMA form is 0.6% slower than the
# register-staged split-K kernel (profiles/early-r14_ab_glds_ops.jsonl), but per layer it wins conv4
# (0.3% of the step, profiles/early-r15_ab_cw_layers.jsonl, early-r15_ab_cw_tiles.jsonl), so the register
# kernel is a tuning candidate (REG) and the shipped table keeps it for conv2/3/5.  The
# row-run weight-grad for few-channel convs ("cwr", conv1) is 3% faster as a kernel but its
# padded-buffer zero + fold-back pass makes the whole step 1.1% slower (profiles/early-r15_ab_cwr.jsonl)
# Autotuning candidates: the 2-stage tiles that run 2-5 blocks per CU measured best on every
# AlexNet shape (profiles/early-r14_glds_tiles.jsonl); 2 covers the fc weight-gradients; the 8-wave
# 128x256 / 64x256 tiles and the pipelined variants (30-41) win conv2/conv3 forward, fc6 forward
# and several VGG shapes (profiles/r2_sweep_tiles.jsonl).
GLDS_CANDS = (1, 7, 10, 15, 2, 17, 21, 25, 30, 31, 34, 37, 38, 39, 40, 41, 72, 75, 76, 77, 78, 79,
              82, 114, 130, 131, 133)
# the halo data-gradient tiles (130 / 131) hand over the lower conv's bias gradient from their
# epilogue (EPI_BF16_DB) instead of a separate column-sum pass; CXXNET_HALO_DB=0 turns that off
_HALO_DB = os.environ.get("CXXNET_HALO_DB", "1") != "0"
# conv weight-grad shapes missing from the shipped table are timed on first use too (else the
# register kernel runs them)
_CW_TUNE = os.environ.get("CXXNET_CW_TUNE", "0") == "1"
# Pseudo-tile: the register-staged kernel (gemm_mfma.hip) with its heuristic tile.  A candidate
# for conv forward / data-grad / weight-grad, where it still wins some shapes (conv2 forward on
# AlexNet timed alone: 172 vs 186 us, profiles/early-r15_glds_8wave.jsonl "old_us").
REG = 99
# Tuning database: {signature: tile}.  A shipped table for gfx950 (written by
# benchmarks/tune_db.py on an MI355X) makes tile choice deterministic across runs and
# data-parallel ranks; shapes it does not hold are timed on first use.
TUNE_DB = os.environ.get("CXXNET_GEMM_TUNE_DB", os.path.join(os.path.dirname(os.path.abspath(__file__)),
                                                               "glds_tune_gfx950.json"))


def _load_tune_db(path):
    import json
    try:
        with open(path) as f:
            return {str(k): int(v) for k, v in json.load(f).items()}
    except (OSError, ValueError):
        return {}


_TUNE = _load_tune_db(TUNE_DB)


def save_tune_db(path=None):
    """Write every tile choice made so far (shipped + newly timed) as JSON."""
    import json
    with open(path or TUNE_DB, "w") as f:
        json.dump(dict(sorted(_TUNE.items())), f, indent=0)


_DET = {"on": False}


def set_deterministic(on: bool = True):
    """Deterministic mode: bitwise-reproducible training steps.  The conv weight-grad
    split-K writes one fp32 slab per K slice and sums the slabs in slice order (no fp32
    atomics), cross-block channel / bias-grad sums run as one ordered pass (the kernels'
    cxn_set_deterministic flag), and GEMM tile autotuning is off (timing-dependent picks
    could differ between runs): the shipped table or the heuristic tile is used."""
    _DET["on"] = bool(on)
    if on:
        _glds_cfg["tune"] = False
    if torch.cuda.is_available():
        native.kernels().cxn_set_deterministic(1 if on else 0)


def deterministic() -> bool:
    return _DET["on"]


def set_tile_group(group_i: int) -> int:
    """Tile order of the LDS-DMA kernels (csrc/kernels/common.h tile_ij): 0 = i fastest over all
    i-tiles, n = i fastest in groups of n i-tiles.  Returns the previous setting."""
    return int(native.kernels().cxn_gemm_set_group(int(group_i)))


def set_glds(on: bool = True, tile: int = -1, tune: bool = True, ops=None):
    """Enable/disable the LDS-DMA GEMM path, force its tile, turn autotuning off, or pick
    the op classes it serves (subset of cf, cd, cw, fc, fw)."""
    _glds_cfg.update(on=bool(on), tile=int(tile), tune=bool(tune))
    if ops is not None:
        _glds_cfg["ops"] = set(ops)


def _use(op: str) -> bool:
    return _glds_cfg["on"] and op in _glds_cfg["ops"]


# CXXNET_TUNE_LOG=1: report every signature timed on first use (a table miss) on stderr
_TUNE_LOG = os.environ.get("CXXNET_TUNE_LOG", "0") == "1"
TUNE_REJECTED = []  # (signature, tile, relative error) of candidates that failed the output check


def _agrees(a: torch.Tensor, ref: torch.Tensor, tol: float = 2e-2) -> float:
    """Norm-relative difference of a candidate's output from the reference tile's output
    (inf when the candidate produced non-finite values the reference did not)."""
    a, ref = a.float(), ref.float()
    if not bool(torch.isfinite(a).all()) and bool(torch.isfinite(ref).all()):
        return float("inf")
    den = ref.norm().item()
    return (a - ref).norm().item() / max(den, 1e-30)


def _tuned_tile(key, run, out, default, extra=(), tune=True, cands=None):
    """Tile for a GEMM signature: the fastest candidate, timed once per process on a
    scratch output (the first call of each shape pays a few extra launches and one host
    sync); the heuristic pick when tuning is off or a graph is being captured.

    A candidate is eligible only if its output agrees with the heuristic tile's output on
    the same operands (norm-relative difference < 2e-2; bf16 rounding and split-K order
    differ by ~1e-3): a tile that computes the wrong thing fast can never win on time
    (commit cecf60b withdrew 96-row tiles that were timing-eligible at 0.8 relative error; the cause,
    an unfenced intra-wave LDS hand-off in the epilogue, is fixed in gemm_glds.hip wave_lds_handoff).
    Scratch outputs start from the live output's contents, so masked (mask_relu) and
    accumulating epilogues see the same inputs for every candidate."""
    if _glds_cfg["tile"] >= 0:
        return _glds_cfg["tile"]
    key = "|".join(str(k) for k in key)
    t = _TUNE.get(key)
    if t is not None:
        return t
    if not (tune and _glds_cfg["tune"]) or frozen():
        return default()
    if _TUNE_LOG:
        import sys
        print(f"gemm tune: timing {key} (not in the tile table)", file=sys.stderr, flush=True)
    init = _like(out)
    init.copy_(out)
    ref = _like(out)
    ref.copy_(init)
    dflt = default()
    ref_tile = dflt
    have_ref = bool(run(dflt, ref))
    if not have_ref and REG in extra:
        ref.copy_(init)
        ref_tile = REG
        have_ref = bool(run(REG, ref))
    scratch = _like(out)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best, best_ms = None, float("inf")
    timed = {}
    for tile in (GLDS_CANDS if cands is None else tuple(cands)) + tuple(extra):
        scratch.copy_(init)
        if not run(tile, scratch):
            continue
        if have_ref and tile != ref_tile:
            err = _agrees(scratch, ref)
            if not err < 2e-2:
                TUNE_REJECTED.append((key, tile, err))
                continue
        ts = []
        for _ in range(3):
            s.record()
            run(tile, scratch)
            e.record()
            e.synchronize()
            ts.append(s.elapsed_time(e))
        ms = sorted(ts)[1]
        timed[tile] = ms
        if ms < best_ms:
            best, best_ms = tile, ms
    _TUNE[key] = best if best is not None else dflt
    if timed:
        TUNED_HERE[key] = timed
    return _TUNE[key]


# Signatures timed by THIS process (table misses): {signature: {tile: ms}}.  Under data
# parallelism each rank times its misses on its own, so two ranks could settle on different
# tiles and the slower pick would hold every step of the job; sync_tune_table() makes the
# choice rank-consistent.
TUNED_HERE = {}


def merge_tune_timings(per_rank):
    """Rank-consistent tile choice from every rank's timings ([{signature: {tile: ms}}] in rank
    order): per signature, the tile with the smallest summed time over the ranks that timed it
    (a tile some rank rejected or could not run is not eligible); ties go to the lower tile id."""
    out = {}
    keys = set()
    for d in per_rank:
        keys.update(d)
    for k in sorted(keys):
        have = [d[k] for d in per_rank if k in d]
        common = set(have[0])
        for h in have[1:]:
            common &= set(h)
        if not common:  # no tile every timing rank could run: the lowest rank's pick
            h = have[0]
            out[k] = min(h, key=lambda t: (h[t], t))
            continue
        out[k] = min(common, key=lambda t: (sum(h[t] for h in have), t))
    return out


def sync_tune_table(group=None):
    """Collective (every data-parallel rank calls it at the same point): exchange the tile
    timings of this process's table misses and adopt the merged choice on every rank."""
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(group) == 1:
        return {}
    objs = [None] * dist.get_world_size(group)
    dist.all_gather_object(objs, {k: dict(v) for k, v in TUNED_HERE.items()}, group=group)
    merged = merge_tune_timings(objs)
    for k, t in merged.items():
        _TUNE[k] = int(t)
    TUNED_HERE.clear()
    return merged


def _pick_glds(rows_i, rows_j, groups, nblocks_target=NUM_CU):
    """Padded MFMA work divided by the fraction of the last dispatch wave that is busy
    (one 4-wave block per CU), then the larger tile."""
    def cost(t):
        bm, bn = GLDS_TILES[t]
        nb = _cdiv(rows_i, bm) * _cdiv(rows_j, bn) * groups
        padded = _cdiv(rows_i, bm) * bm * _cdiv(rows_j, bn) * bn * groups
        waves = _cdiv(nb, nblocks_target)
        return (padded * waves * nblocks_target / nb, -bm * bn, t)
    return min((1, 7, 10, 15), key=cost)


def _glds(a, b, amode, bmode, out, out_gstride, ldc, *, alpha=1.0, bias=None, bias_gstride=0, relu=False,
          mask_relu=False, epi=EPI_BF16, groups=1, ksplit=1, kstride=0, tile=None, dbias=None, dws=None,
          dws_ld=0) -> bool:
    """Run the LDS-DMA kernel; False when it does not support the operands (caller falls back)."""
    if not _glds_cfg["on"]:
        return False
    if tile is None:
        tile = _glds_cfg["tile"] if _glds_cfg["tile"] >= 0 else _pick_glds(a.rows, b.rows, groups)
    rc = native.kernels().cxn_gemm_glds(
        a, b, amode, bmode, out.data_ptr(), out_gstride, ldc, float(alpha),
        bias.data_ptr() if bias is not None else None, bias_gstride, int(relu), int(mask_relu), epi, tile, groups,
        ksplit, kstride, dbias.data_ptr() if dbias is not None else None,
        dws.data_ptr() if dws is not None else None, dws.numel() if dws is not None else 0, int(dws_ld), _stream())
    if rc == -1:
        return False
    native.check(rc, "gemm_glds")
    LAST_GLDS[0] = tile
    return True


LAST_GLDS = [None]  # tile of the last LDS-DMA launch (tests check that a forced tile really ran)


def _pick_tile(rows_i, rows_j, groups):
    return _pick(FC_TILES, rows_i, rows_j, groups)


def _gemm(a, b, amode, bmode, va, vb, out, out_gstride, ldc, *, alpha=1.0, bias=None, bias_gstride=0,
          relu=False, mask_relu=False, epi=EPI_BF16, groups=1, ksplit=1, tile=None, kstride=0):
    if tile is None:
        tile = _pick_tile(a.rows, b.rows, groups)
    rc = native.kernels().cxn_gemm(
        a, b, amode, bmode, va, vb, out.data_ptr(), out_gstride, ldc, float(alpha),
        bias.data_ptr() if bias is not None else None, bias_gstride, int(relu), int(mask_relu), epi, tile, groups,
        ksplit, kstride, _stream())
    native.check(rc, "gemm")


def _effective_split(kdim, split):
    """The kernel's own clamp (launch_t): slices of ceil(ktiles/split) k-tiles."""
    kt = -(-kdim // 64)
    split = max(1, min(split, kt))
    per = -(-kt // split)
    return -(-kt // per)


def _finalize(ws, split, slab, out, rows, ldc, bias, relu, mask_relu, drop):
    """out = epilogue(sum of the split-K fp32 slabs); drop = (seed, counter, pkeep): the dropout
    of a fused fc -> relu -> dropout applied on the way out (same mask as ops.dropout_apply)."""
    k = native.kernels()
    bp = bias.data_ptr() if bias is not None else None
    if drop is not None:
        seed, counter, pkeep = drop
        native.check(k.cxn_splitk_finalize_dropout(ws.data_ptr(), split, slab, out.data_ptr(), rows, ldc, bp, int(relu),
                                                   seed & 0xFFFFFFFF,
                                                   counter.data_ptr() if counter is not None else None,
                                                   float(pkeep), _stream()), "splitk_finalize_dropout")
        return
    native.check(k.cxn_splitk_finalize(ws.data_ptr(), split, slab, out.data_ptr(), rows, ldc, bp, int(relu),
                                       int(mask_relu), _stream()), "splitk_finalize")


def _gemm_bf16_out(a, b, amode, bmode, out, ldc, *, bias=None, relu=False, mask_relu=False, alpha=1.0,
                   drop=None) -> bool:
    """out (bf16, [rows_j][ldc]) = epilogue(alpha * A . B) for a single-group GEMM, with split-K
    through fp32 slabs + one finalize pass when the output tile grid is too small to
    fill the chip (the FC layers at batch 256: 64 tiles of 128x128 for fc6).  drop: see
    _finalize; returns True when the dropout was applied (only the split-K path fuses it)."""
    # fc data-grad (A MN-major) stays on the register-staged kernel: its LDS-DMA form measured
    # slower on AlexNet's fc6-8 (profiles/early-r14_glds_tiles.jsonl)
    if bmode == DIRECT_K and amode == DIRECT_K and alpha == 1.0 and _use("fc"):
        r = _fc_glds(a, b, GL_K, out, ldc, bias, relu, mask_relu, drop)
        if r is not None:
            return r
    tile = _pick(FC_TILES, a.rows, b.rows, 1, min_blocks=1)
    split = _auto_split(a.rows, b.rows, 1, a.kdim, tile, min_ktiles=8)
    if split > 1 and a.kdim >= 2048 and ldc % 8 == 0 and ldc == a.rows:
        split = _effective_split(a.kdim, split)
        slab = b.rows * ldc
        ws = torch.empty((split, slab), dtype=torch.float32, device=out.device)
        _gemm(a, b, amode, bmode, 8, 8, ws, 0, ldc, alpha=alpha, epi=EPI_F32, ksplit=split, tile=tile, kstride=slab)
        _finalize(ws, split, slab, out, b.rows, ldc, bias, relu, mask_relu, drop)
        return drop is not None
    _gemm(a, b, amode, bmode, 8, 8, out, 0, ldc, alpha=alpha, bias=bias, relu=relu, mask_relu=mask_relu, epi=EPI_BF16,
          tile=tile)
    return False


def _fc_glds(a, b, amode, out, ldc, bias, relu, mask_relu, drop=None):
    """fc forward (A = W, K-major) / data-grad (A = W, MN-major) on the LDS-DMA kernel.  None
    when the kernel does not serve the shape; else whether the dropout (drop) was applied."""
    key = ("fc", amode, a.rows, b.rows, a.kdim, ldc)
    got = {}

    def run(t, o):
        r = _fc_glds_tile(a, b, amode, o, ldc, bias, relu, mask_relu, t, drop)
        got["drop"] = r == 2
        return bool(r)
    tile = _tuned_tile(key, run, out, lambda: 1 if amode == GL_MN else _pick_glds(a.rows, b.rows, 1))
    if not run(tile, out):
        return None
    return got["drop"]


def _fc_glds_tile(a, b, amode, out, ldc, bias, relu, mask_relu, tile, drop=None) -> int:
    """split-K through fp32 slabs when the output tile grid cannot fill the chip (fc6 at
    batch 256: 32 tiles of 128x256).  0: not served, 1: done, 2: done with the dropout."""
    bm, bn = GLDS_TILES[tile]
    tiles = _cdiv(a.rows, bm) * _cdiv(b.rows, bn)
    ktiles = _cdiv(a.kdim, 64)
    split = max(1, min(NUM_CU // max(tiles, 1), ktiles // 8))
    if split > 1 and ldc % 8 == 0 and ldc == a.rows:
        split = _effective_split(a.kdim, split)
        slab = b.rows * ldc
        ws = torch.empty((split, slab), dtype=torch.float32, device=out.device)
        if not _glds(a, b, amode, GL_K, ws, 0, ldc, epi=EPI_F32, ksplit=split, kstride=slab, tile=tile):
            return 0
        _finalize(ws, split, slab, out, b.rows, ldc, bias, relu, mask_relu, drop)
        return 2 if drop is not None else 1
    return int(_glds(a, b, amode, GL_K, out, 0, ldc, bias=bias, relu=relu, mask_relu=mask_relu, tile=tile))


def _auto_split(rows_i, rows_j, groups, kdim, tile=0, target=2 * NUM_CU, min_ktiles=4):
    bm, bn = TILES[tile]
    tiles = -(-rows_i // bm) * -(-rows_j // bn) * groups
    ktiles = -(-kdim // 64)
    split = max(1, min(target // max(tiles, 1), ktiles // min_ktiles))
    return split


def _wgrad_cands(rows_i, rows_j, groups, kdim):
    """(tile, K-slice count) candidates of the register-staged split-K weight-gradient GEMM,
    encoded tile * 100000 + slices.  Its slices meet in fp32 atomics, whose cost grows with
    the slice count (on GoogLeNet's 160->320 3x3 weight-grad 72 us at 14 slices, 553 us at
    512) while too few slices leave CUs idle (its 64->64 1x1: 205 us at 32, 38 us at 512;
    profiles/r2_wgrad_split_sweep.jsonl), so the count is timed per shape: the chip-filling
    count (4 blocks per CU) and its halvings, for each weight-grad tile."""
    ktiles = -(-kdim // 64)
    out = []
    for tile in WGRAD_TILES:
        bm, bn = TILES[tile]
        tiles = -(-rows_i // bm) * -(-rows_j // bn) * groups
        occ = max(1, min(4 * NUM_CU // tiles, ktiles // 4))
        out += [tile * 100000 + sp for sp in sorted({max(1, occ >> k) for k in range(5)})]
    return tuple(out)


# ----------------------------------------------------------------------------- convolution
def conv_out_size(H, W, KH, KW, stride, pad_y, pad_x):
    """Reference rule (src/layer/convolution_layer-inl.hpp:174-177)."""
    return (H + 2 * pad_y - KH) // stride + 1, (W + 2 * pad_x - KW) // stride + 1


ROWRUN_ALIGN = int(os.environ.get("CXXNET_ROWRUN_ALIGN", "8") or 8)  # as gemm_glds.hip g_rowrun_align


def rowrun_ok(g: ConvGeom) -> bool:
    """Few-channel conv served by the kernel-row-run GEMMs (K_ROWGATHER forward, row-run MN
    gather weight-grad): pad 0, one group, and every image row and output-pixel step of x at
    ROWRUN_ALIGN bytes (the runs' 16-byte DMAs start at a pixel)."""
    return (g.groups == 1 and g.pad_y == 0 and g.pad_x == 0 and g.C % 8 != 0 and
            (g.W * g.C * 2) % ROWRUN_ALIGN == 0 and (g.stride * g.C * 2) % ROWRUN_ALIGN == 0)


def _w_nchw(w: torch.Tensor) -> torch.Tensor:
    # [Cout][KH][KW][Cg] -> [Cout][Cg][KH][KW]
    return w.permute(0, 3, 1, 2).contiguous()


_wpad = {}


def _row_padded_weights(w, g: ConvGeom):
    """[Cout][KH][KW][C] -> [Cout][KH][roundup(KW*C, 8)] with zero tails (refreshed every call:
    the optimizer rewrites w each step).  The buffer is cached per weight tensor."""
    L = g.KW * g.C
    lp = (L + 7) // 8 * 8
    key = (w.data_ptr(), tuple(w.shape))
    buf = _wpad.get(key)
    if buf is None:
        buf = _wpad[key] = torch.empty((g.Cout, g.KH, lp), dtype=w.dtype, device=w.device)
    native.check(native.kernels().cxn_pad_rows(w.data_ptr(), buf.data_ptr(), g.Cout * g.KH, L, lp, _stream()),
                 "pad_rows")
    return buf, lp


_wgpad = {}
_detws = {}


def _det_ws(n, device):
    buf = _detws.get(str(device))
    if buf is None or buf.numel() < n:
        from .mode import retire
        retire(buf)  # a recorded / captured step may still point at it
        buf = _detws[str(device)] = torch.empty(n, dtype=torch.float32, device=device)
    return buf[:n]


def _add_rows(src, dst, rows, L, Ls):
    """dst[r][0:L] += src[r][0:L] for fp32 [rows][Ls] -> [rows][L] (the row-padded weight-grad
    buffer into the layer's gradient), as a library kernel."""
    native.check(native.kernels().cxn_add_rows_f32(src.data_ptr(), dst.data_ptr(), rows, L, Ls, _stream()),
                 "add_rows_f32")


def _wgrad_pad_buf(cout, kr, device):
    """fp32 [Cout][KH * roundup(KW*C, 8)] accumulation buffer of the row-run weight-grad."""
    key = (cout, kr, str(device))
    buf = _wgpad.get(key)
    if buf is None:
        buf = _wgpad[key] = torch.empty((cout, kr), dtype=torch.float32, device=device)
    return buf


_FEWC = os.environ.get("CXXNET_FEWC", "1") != "0"
# direct row-run forward (conv_rowrun.hip: input rows staged once per 4 output rows) for the
# few-channel pad-0 first layer (AlexNet conv1) instead of the K_ROWGATHER GEMM
_ROWRUN_DIRECT = os.environ.get("CXXNET_ROWRUN_DIRECT", "1") != "0"
# the AlexNet conv1 class on conv_rowrun_direct.hip's forward (flattened pixels x (kernel row,
# 4-element chunk) GEMM out of staged input rows, no row-padded weight copy) ahead of both
_ROWRUN_FWD2 = os.environ.get("CXXNET_ROWRUN_FWD2", "1") != "0"


def conv_rowrun_fwd2(x, w, bias, y, g: ConvGeom, relu=False) -> bool:
    """y = conv(x, w) + bias (relu) for a few-channel first layer on conv_rowrun_direct.hip's
    forward (flattened pixels x (kernel row, 4-element chunk) GEMM out of staged input rows, no
    row-padded weight copy): the AlexNet / GoogLeNet conv1 classes.  False when not served."""
    if not (_ROWRUN_FWD2 and _native_t(x) and g.groups == 1 and g.pad_y == g.pad_x and x.is_contiguous()
            and w.is_contiguous() and _pix(y) % 4 == 0 and y.stride(-1) == 1 and _pix(x) == g.C):
        return False
    rc = native.kernels().cxn_conv_rowrun_fwd2(
        x.data_ptr(), w.data_ptr(), bias.data_ptr() if bias is not None else None, y.data_ptr(), g.N, g.H, g.W,
        g.C, g.Ho, g.Wo, g.Cout, _pix(y), g.KH, g.KW, g.stride, g.pad_y, int(relu), _stream())
    if rc == -1:
        return False
    native.check(rc, "conv_rowrun_fwd2")
    return True


def fewc_ok(x, g: ConvGeom) -> bool:
    """Few-channel first-layer forward kernel (conv_fewc.hip): 4-channel NHWC input, one group,
    16..128 output channels (multiple of 16), at most 64 taps, any stride / padding."""
    return (_FEWC and _native_t(x) and g.C == 4 and g.groups == 1 and g.Cout % 16 == 0 and g.Cout <= 128
            and g.KH * g.KW <= 64 and g.pad_y == g.pad_x and x.is_contiguous() and g.W == x.shape[2])


def fewc_preferred(g: ConvGeom) -> bool:
    """Where the few-channel kernel beats the GEMM inside the training step: stride 1 (VGG-16
    conv1_1: 9.47 -> 9.44 ms/step); on GoogLeNet's 7x7 / 2 conv1 it lost, 5.78 -> 5.90 ms
    (profiles/r3_ab_fewc.jsonl)."""
    return g.stride == 1


def conv_forward_fewc(x, w, bias, y, g: ConvGeom, relu=False) -> bool:
    """y = relu?(conv(x, w) + bias) on the few-channel kernel; False when it does not serve the shape."""
    if not fewc_ok(x, g):
        return False
    rc = native.kernels().cxn_conv_fewc_fwd(x.data_ptr(), w.data_ptr(), bias.data_ptr() if bias is not None else None,
                                           y.data_ptr(), g.N, g.H, g.W, g.Ho, g.Wo, g.Cout, g.KH, g.KW, g.stride,
                                           g.pad_y, _pix(y), int(relu), _stream())
    if rc == -1:
        return False
    native.check(rc, "conv_fewc_fwd")
    return True


def conv_forward(x, w, bias, y, g: ConvGeom, relu=False):
    """y = conv(x, w) + bias (optionally relu).  x/y NHWC."""
    if not _native_t(x):
        xn = x.permute(0, 3, 1, 2)
        out = F.conv2d(xn, _w_nchw(w), bias, stride=g.stride, padding=(g.pad_y, g.pad_x), groups=g.groups)
        if relu:
            out = out.clamp_min(0)
        y.copy_(out.permute(0, 2, 3, 1))
        return
    cg = g.cg_in
    va = 8 if cg % 8 == 0 else 4
    if g.C == 4 and conv_rowrun_fwd2(x, w, bias, y, g, relu):  # padded 4-channel first layers (GoogLeNet conv1)
        return
    if cg % va and not rowrun_ok(g):
        raise ValueError(f"conv: channels per group ({cg}) must be a multiple of 4 on the GPU path")
    kd = g.kdim
    A = _op(w, g.cg_out * kd, kd, g.cg_out, kd)
    # C = the input's pixel stride: a channel slice of a wider buffer (sibling outputs,
    # NeuralNet._fuse_siblings) is read in place
    B = _op(x, cg, 0, g.N * g.Ho * g.Wo, kd, H=g.H, W=g.W, C=_pix(x), Ho=g.Ho, Wo=g.Wo, KH=g.KH, KW=g.KW,
            stride=g.stride, pad_h=g.pad_y, pad_w=g.pad_x, dil=1, Cg=cg)
    def reg(o):
        tile = _pick(CONV_FWD_TILES if va == 8 else CONV_FWD_TILES_V4, g.cg_out, g.N * g.Ho * g.Wo, g.groups)
        _gemm(A, B, DIRECT_K, GATHER_K, va, va, o, g.cg_out, _pix(o), bias=bias, bias_gstride=g.cg_out, relu=relu,
              tile=tile, epi=EPI_BF16, groups=g.groups)
        return True
    if va == 8 and _use("cf"):
        def run(t, o):
            if t == REG:
                return reg(o)
            if t in DIRECT_TILES:
                return _CD != "0" and conv_direct_forward(x, w, bias, o, g, relu=relu, variant=DIRECT_TILES[t])
            return _glds(A, B, GL_K, GL_KG, o, g.cg_out, _pix(o), bias=bias, bias_gstride=g.cg_out, relu=relu,
                         groups=g.groups, tile=t)
        key = ("cf", g.N, g.H, g.W, g.C, g.Cout, g.KH, g.KW, g.stride, g.pad_y, g.pad_x, g.groups)
        extra = (REG,) + (tuple(DIRECT_TILES) if _cd_serves(g, x, y) else ())
        t = _tuned_tile(key, run, y, lambda: _pick_glds(A.rows, B.rows, g.groups), extra=extra)
        if run(t, y):
            return
        if t in DIRECT_TILES and run(_pick_glds(A.rows, B.rows, g.groups), y):  # (direct kernel switched off)
            return
    if va != 8 and rowrun_ok(g) and (_use("cr") or g.C % 4):
        # few input channels (conv1: 11x11 taps of 4 channels): each kernel row's KW*C
        # elements are contiguous in NHWC; the GEMM reads them as zero-padded runs
        if conv_rowrun_fwd2(x, w, bias, y, g, relu):
            return
        wp, lp = _row_padded_weights(w, g)
        if _ROWRUN_DIRECT and x.is_contiguous() and y.shape[-1] == _pix(y):
            rc = native.kernels().cxn_conv_rowrun_fwd(
                x.data_ptr(), x.numel() * x.element_size(), wp.data_ptr(), bias.data_ptr() if bias is not None else None,
                y.data_ptr(), g.N, g.H, g.W, g.C, g.Ho, g.Wo, g.Cout, g.KH, lp, g.stride, _pix(y), int(relu), _stream())
            if rc == 0:
                return
            if rc != -1:
                native.check(rc, "conv_rowrun_fwd")
        kr = g.KH * lp
        Ar = _op(wp, 0, kr, g.Cout, kr)
        Br = _op(x, 0, 0, g.N * g.Ho * g.Wo, kr, H=g.H, W=g.W, C=g.C, Ho=g.Ho, Wo=g.Wo, KH=g.KH, KW=g.KW,
                 stride=g.stride, pad_h=0, pad_w=0, dil=1, Cg=g.C)
        run = lambda t, o: _glds(Ar, Br, GL_K, GL_KR, o, 0, _pix(o), bias=bias, relu=relu, tile=t)  # noqa: E731
        key = ("cr", g.N, g.H, g.W, g.C, g.Cout, g.KH, g.KW, g.stride)
        if run(_tuned_tile(key, run, y, lambda: 1), y):
            return
    if cg % va:
        raise RuntimeError(f"conv: no GPU kernel for {cg} channels per group ({g})")
    reg(y)


# gemm_glds tiles whose epilogue takes a second destination (cxn_gemm_glds_split)
SPLIT_CANDS = tuple(t for t in GLDS_CANDS if t not in (114, 130, 131, 133))


def conv_forward_split(x, w, bias, y, y2, split, g: ConvGeom, relu=False):
    """One GEMM for convs that read the same input (the sibling 1x1 convs of an inception
    module, NeuralNet._fuse_siblings): w [Cout][KH][KW][Cin] stacks their weights, output
    channels [0, split) go to y and [split, Cout) to y2 (each NHWC, any pixel stride)."""
    if not _native_t(x):
        t = torch.empty(y.shape[:-1] + (g.Cout,), dtype=y.dtype, device=y.device)
        conv_forward(x, w, bias, t, g, relu=relu)
        y.copy_(t[..., :split])
        y2.copy_(t[..., split:])
        return
    cg = g.cg_in
    kd = g.kdim
    A = _op(w, g.cg_out * kd, kd, g.cg_out, kd)
    B = _op(x, cg, 0, g.N * g.Ho * g.Wo, kd, H=g.H, W=g.W, C=_pix(x), Ho=g.Ho, Wo=g.Wo, KH=g.KH, KW=g.KW,
            stride=g.stride, pad_h=g.pad_y, pad_w=g.pad_x, dil=1, Cg=cg)

    def run(t, o):
        if t == REG or not _glds_cfg["on"]:
            return False
        rc = native.kernels().cxn_gemm_glds_split(
            A, B, GL_K, GL_KG, o.data_ptr(), _pix(o), y2.data_ptr(), _pix(y2), int(split),
            bias.data_ptr() if bias is not None else None, int(relu), t, _stream())
        if rc == -1:
            return False
        native.check(rc, "gemm_glds_split")
        LAST_GLDS[0] = t
        return True
    key = ("cfs", g.N, g.H, g.W, g.C, g.Cout, split)
    if cg % 8 == 0 and g.groups == 1 and _use("cf"):
        t = _tuned_tile(key, run, y, lambda: _pick_glds(A.rows, B.rows, 1), cands=SPLIT_CANDS)
        if run(t, y):
            return
    # no two-destination tile for this shape: the two channel ranges as two GEMMs
    for lo, hi, o in ((0, split, y), (split, g.Cout, y2)):
        gi = ConvGeom(g.N, g.H, g.W, g.C, g.Ho, g.Wo, hi - lo, g.KH, g.KW, g.stride, g.pad_y, g.pad_x, 1)
        conv_forward(x, w[lo:hi], bias[lo:hi] if bias is not None else None, o, gi, relu=relu)


def conv_weight_flip_multi(items):
    """wt = w with (Cout, Cin) swapped and the taps reversed (the data-gradient GEMM's weight
    operand), for every (w, wt, geometry) of `items` in one launch."""
    items = [it for it in items if _native_t(it[0])]
    if not items:
        return
    n = len(items)
    ws = (ctypes.c_void_p * n)(*[w.data_ptr() for w, _, _ in items])
    wts = (ctypes.c_void_p * n)(*[wt.data_ptr() for _, wt, _ in items])
    dims = (ctypes.c_int * (5 * n))(*[v for _, _, g in items for v in (g.groups, g.cg_out, g.KH, g.KW, g.cg_in)])
    native.check(native.kernels().cxn_conv_weight_flip_multi(ctypes.cast(ws, ctypes.c_void_p),
                                                             ctypes.cast(wts, ctypes.c_void_p),
                                                             ctypes.cast(dims, ctypes.c_void_p), n, _stream()),
                 "conv_weight_flip_multi")


def conv_backward_data(dy, w, dx, g: ConvGeom, wt_buf=None, mask_relu=False, wt_ready=False, dbias=None) -> bool:
    """dx = conv_transpose(dy, w); dx overwritten.  mask_relu: dx holds relu(z) on entry
    (fused producer->relu) and the result is multiplied by relu'(z).  wt_ready: wt_buf already
    holds the flipped weights (conv_weight_flip_multi at the start of the backward pass).
    dbias (fp32 [C], optional): += column sums of the stored dx -- the bias gradient of the conv
    that produced x -- inside the GEMM epilogue (EPI_BF16_DB).  Returns True when dbias was
    accumulated; False when the chosen kernel has no such epilogue (the caller sums dx itself)."""
    if not _native_t(dy):
        dyn = dy.permute(0, 3, 1, 2)
        out = torch.nn.grad.conv2d_input((g.N, g.C, g.H, g.W), _w_nchw(w), dyn, stride=g.stride,
                                         padding=(g.pad_y, g.pad_x), groups=g.groups).permute(0, 2, 3, 1)
        if mask_relu:
            out = out * (dx > 0).to(out.dtype)
        dx.copy_(out)
        return False
    cg_in, cg_out = g.cg_in, g.cg_out
    if cg_out % 8:
        raise ValueError("conv dgrad: output channels per group must be a multiple of 8 on the GPU path")
    if wt_buf is None:
        wt_buf = torch.empty_like(w)
    if not wt_ready:
        native.check(native.kernels().cxn_conv_weight_flip(w.data_ptr(), wt_buf.data_ptr(), g.groups, cg_out, g.KH,
                                                           g.KW, cg_in, _stream()), "conv_weight_flip")
    kd = g.KH * g.KW * cg_out
    A = _op(wt_buf, cg_in * kd, kd, cg_in, kd)
    B = _op(dy, cg_out, 0, g.N * g.H * g.W, kd, H=g.Ho, W=g.Wo, C=_pix(dy), Ho=g.H, Wo=g.W, KH=g.KH,
            KW=g.KW, stride=1, pad_h=g.KH - 1 - g.pad_y, pad_w=g.KW - 1 - g.pad_x, dil=g.stride, Cg=cg_out)
    def reg(o):
        tile = _pick(CONV_FWD_TILES, cg_in, g.N * g.H * g.W, g.groups)
        _gemm(A, B, DIRECT_K, GATHER_K, 8, 8, o, cg_in, _pix(o), epi=EPI_BF16, groups=g.groups, mask_relu=mask_relu,
              tile=tile)
        return True
    if g.stride == 1 and _use("cd"):
        dg = ConvGeom(g.N, g.H, g.W, g.Cout, g.H, g.W, g.C, g.KH, g.KW, 1, g.pad_y, g.pad_x, g.groups)

        def run(t, o):
            if t == REG:
                return reg(o)
            if t in DIRECT_TILES:
                return _CD != "0" and conv_direct_data(dy, wt_buf, o, g, mask_relu=mask_relu,
                                                       variant=DIRECT_TILES[t])
            return _glds(A, B, GL_K, GL_KG, o, cg_in, _pix(o), groups=g.groups, mask_relu=mask_relu, tile=t)
        key = ("cd", g.N, g.H, g.W, g.C, g.Cout, g.KH, g.KW, g.stride, g.pad_y, g.pad_x, g.groups)
        extra = (REG,) + (tuple(DIRECT_TILES) if _cd_serves(dg, dy, dx) else ())
        t = _tuned_tile(key, run, dx, lambda: _pick_glds(A.rows, B.rows, g.groups), extra=extra)
        if t in DIRECT_TILES and _CD != "0":
            db = dbias if dbias is not None and not deterministic() else None
            if conv_direct_data(dy, wt_buf, dx, g, mask_relu=mask_relu, dbias=db, variant=DIRECT_TILES[t]):
                return db is not None
            t = _pick_glds(A.rows, B.rows, g.groups)
        if dbias is not None and t != REG and (t not in (130, 131) or _HALO_DB):
            from .nn import _workspace
            ws = _workspace((-(-B.rows // 16) + 8) * g.C, dx.device)  # >= tiles_j * waves_j rows
            if _glds(A, B, GL_K, GL_KG, dx, cg_in, _pix(dx), groups=g.groups, mask_relu=mask_relu, tile=t,
                     epi=EPI_BF16_DB_G, bias_gstride=cg_in, dbias=dbias, dws=ws, dws_ld=g.C):
                return True
        if run(t, dx):
            return False
    reg(dx)
    return False


def conv_backward_data_add(dy, w, dx, add, g: ConvGeom, wt_buf, mask_relu=False, wt_ready=False) -> bool:
    """dx = mask(conv_transpose(dy, w) + add): the data gradient with a second gradient `add`
    (laid out like dx) summed in the GEMM epilogue -- the split after a sibling group folds its
    gradient sum into the group's data-gradient GEMM (NeuralNet._fuse_siblings).  Only on a tuned
    LDS-DMA tile of this signature ("cd" table entry); False (nothing done) otherwise, and the
    caller takes the separate data-gradient + sum path."""
    if not _native_t(dy) or g.stride != 1 or not _use("cd") or g.cg_out % 8 or _pix(add) != _pix(dx):
        return False
    if tuple(add.shape) != tuple(dx.shape) or not _glds_cfg["on"]:
        return False
    key = "|".join(str(k) for k in ("cd", g.N, g.H, g.W, g.C, g.Cout, g.KH, g.KW, g.stride, g.pad_y, g.pad_x,
                                    g.groups))
    cg_in, cg_out = g.cg_in, g.cg_out
    kd = g.KH * g.KW * cg_out
    A = _op(wt_buf, cg_in * kd, kd, cg_in, kd)
    B = _op(dy, cg_out, 0, g.N * g.H * g.W, kd, H=g.Ho, W=g.Wo, C=_pix(dy), Ho=g.H, Wo=g.W, KH=g.KH,
            KW=g.KW, stride=1, pad_h=g.KH - 1 - g.pad_y, pad_w=g.KW - 1 - g.pad_x, dil=g.stride, Cg=cg_out)
    t = _glds_cfg["tile"] if _glds_cfg["tile"] >= 0 else _TUNE.get(key)
    if t is None:  # not tuned yet: the plain path tunes it; with tuning off, its default pick
        if _glds_cfg["tune"] and not frozen():
            return False
        t = _pick_glds(A.rows, B.rows, g.groups)
    if t == REG or t == 114 or 130 <= t <= 142:
        return False
    if not wt_ready:
        native.check(native.kernels().cxn_conv_weight_flip(w.data_ptr(), wt_buf.data_ptr(), g.groups, cg_out, g.KH,
                                                           g.KW, cg_in, _stream()), "conv_weight_flip")
    rc = native.kernels().cxn_gemm_glds_add(A, B, GL_K, GL_KG, dx.data_ptr(), cg_in, _pix(dx), add.data_ptr(),
                                            int(mask_relu), t, g.groups, _stream())
    if rc == -1:  # (a flip done here is repeated by the caller's path: the same values)
        return False
    native.check(rc, "gemm_glds_add")
    LAST_GLDS[0] = t
    return True


# Direct small-map forward / data gradient (conv_direct.hip: gap-slot layout, taps as constant
# LDS offsets, persistent blocks).  "auto" / "1": wherever it serves the shape; "0": off (the
# implicit GEMMs run).
_CD = os.environ.get("CXXNET_CONV_DIRECT", "auto")
_cd_ws = {}
# Pseudo-tiles of the tile table for the direct kernel's schedules (cxn_conv_direct variant):
# 200 persistent blocks with two stage buffers, 201 one block per item (two per CU), 202 as 200
# with four LDS-DMA loader waves per block, 203 version 2 (eight waves, two per SIMD, paired taps,
# persistent double-buffered stages).  Tuning candidates of the "cf" / "cd" signatures it
# serves (in-step picks at the strong-scaling batches: profiles/r6_step_tune_direct_b{32,64,128}.jsonl).
DIRECT_TILES = {200: 0, 201: 1, 202: 2, 203: 3}


def _cd_workspace(n, device):
    buf = _cd_ws.get(str(device))
    if buf is None or buf.numel() < n:
        from .mode import retire
        retire(buf)
        buf = _cd_ws[str(device)] = torch.empty(max(n, 1 << 16), dtype=torch.float32, device=device)
    return buf


def _cd_ok(g: ConvGeom, *ts) -> bool:
    if _CD == "0" or (_glds_cfg["tile"] >= 0 and _glds_cfg["tile"] not in DIRECT_TILES):
        return False  # (a forced LDS-DMA tile id means a test / probe wants that kernel)
    if g.stride != 1 or g.Ho != g.H or g.Wo != g.W or g.KH != g.KW or g.pad_y != (g.KH - 1) // 2 or g.pad_x != g.pad_y:
        return False
    return all(t.stride(-1) == 1 and (t.is_contiguous() or t.stride(-2) * t.shape[-2] == t.stride(-3))
               for t in ts)


def _cd_serves(g: ConvGeom, *ts) -> bool:
    """The direct kernel's shape rule (cxn_conv_direct), without launching anything."""
    if not _cd_ok(g, *ts):
        return False
    if g.KH == 5 and g.H == 27 and g.W == 27:  # paired-tap form (AlexNet conv2)
        return g.cg_in % 16 == 0 and (g.cg_out % 64 == 0 or g.cg_out % 48 == 0)
    return g.KH == 3 and g.H == g.W and g.H in (13, 14) and g.cg_in % 32 == 0 and g.cg_out % 64 == 0


def conv_direct_forward(x, w, bias, y, g: ConvGeom, relu=False, variant=0) -> bool:
    """y = conv(x, w) + bias (relu optional) on the direct small-map kernel; False when it does
    not serve the shape."""
    if not _cd_ok(g, x, y):
        return False
    rc = int(native.kernels().cxn_conv_direct(
        x.data_ptr(), _pix(x), w.data_ptr(), bias.data_ptr() if bias is not None else None, y.data_ptr(), _pix(y),
        None, 0, None, g.N, g.H, g.W, g.cg_in, g.cg_out, g.groups, g.KH, int(relu), 0, int(variant), _stream()))
    if rc == -1:
        return False
    native.check(rc, "conv_direct")
    return True


def conv_direct_data(dy, wt, dx, g: ConvGeom, mask_relu=False, dbias=None, variant=0) -> bool:
    """dx = conv_transpose(dy, w) (wt: the flipped weights), relu'-masked when mask_relu, and
    dbias += the column sums of the stored dx; False when the kernel does not serve the shape."""
    if not _cd_ok(g, dy, dx):
        return False
    k = native.kernels()
    args = (g.N, g.H, g.W, g.cg_out, g.cg_in, g.groups, g.KH, int(mask_relu))
    ws, n = None, 0
    if dbias is not None:
        need = int(k.cxn_conv_direct(None, _pix(dy), None, None, None, _pix(dx), None, 0, None, *args, 2, 0, None))
        if need <= 0:
            return False
        ws = _cd_workspace(need, dx.device)
        n = ws.numel()
    rc = int(k.cxn_conv_direct(dy.data_ptr(), _pix(dy), wt.data_ptr(), None, dx.data_ptr(), _pix(dx),
                               ws.data_ptr() if ws is not None else None, n,
                               dbias.data_ptr() if dbias is not None else None, *args,
                               2 if dbias is not None else 1, int(variant), _stream()))
    if rc == -1:
        return False
    native.check(rc, "conv_direct")
    return True


# Direct small-map weight gradient (conv_wgrad_direct.hip: gap-slot K walk, resident x / dy
# stages, partial tiles reduced in a fixed order -- no atomics, deterministic).  "1" / "auto":
# use it wherever it serves the shape; "0": off (the split-K GEMMs run).
_WGD = os.environ.get("CXXNET_WGRAD_DIRECT", "auto")
_wgd_ws = {}


def _wgd_workspace(n, device):
    buf = _wgd_ws.get(str(device))
    if buf is None or buf.numel() < n:
        from .mode import retire
        retire(buf)  # a recorded / captured step may still point at it
        buf = _wgd_ws[str(device)] = torch.empty(max(n, 1 << 20), dtype=torch.float32, device=device)
    return buf


def conv_wgrad_direct(x, dy, dw, g: ConvGeom, splits: int = 0, db=None) -> bool:
    """dw += the weight gradient on the direct small-map kernel (and db += the bias gradient,
    the sum of dy over pixels, when db is given); False when it does not serve the shape (or is
    switched off)."""
    if _WGD == "0" or _glds_cfg["tile"] >= 0 or not _native_t(x) or g.Ho != g.H or g.Wo != g.W:
        return False  # (a forced LDS-DMA tile id means a test / probe wants that kernel)
    if not (x.is_contiguous() or x.stride(-1) == 1) or dy.stride(-1) != 1:
        return False
    k = native.kernels()
    args = (g.N, g.H, g.W, _pix(x), _pix(dy), g.cg_in, g.cg_out, g.groups, g.KH, g.KW, g.pad_y, g.pad_x, g.stride,
            int(splits))
    need = int(k.cxn_conv_wgrad_direct(None, None, None, None, None, 0, *args, 1.0, None))
    if need <= 0:
        return False
    ws = _wgd_workspace(need, dw.device)
    rc = int(k.cxn_conv_wgrad_direct(x.data_ptr(), dy.data_ptr(), dw.data_ptr(), db.data_ptr() if db is not None else None,
                                     ws.data_ptr(), ws.numel(), *args, 1.0, _stream()))
    if rc == -1:
        return False
    native.check(rc, "conv_wgrad_direct")
    return True


def conv_wgrad_rowrun(x, dy, dw, g: ConvGeom) -> bool:
    """dw += the weight gradient of a few-channel first layer (AlexNet / GoogLeNet conv1 class) on
    the direct kernel-row-run kernel (conv_rowrun_direct.hip conv_wgrad_rowrun: transposed LDS
    reads straight out of staged input rows, fixed-order partial sums); False when not served."""
    if _WGD == "0" or _glds_cfg["tile"] >= 0 or not _native_t(x) or g.groups != 1 or g.pad_y != g.pad_x:
        return False
    if not x.is_contiguous() or _pix(x) != g.C or dy.stride(-1) != 1 or not dw.is_contiguous():
        return False
    k = native.kernels()
    args = (g.N, g.H, g.W, g.C, g.Ho, g.Wo, g.Cout, _pix(dy), g.KH, g.KW, g.stride, g.pad_y)
    need = int(k.cxn_conv_wgrad_rowrun(None, None, None, None, 0, *args, 1.0, None))
    if need <= 0:
        return False
    ws = _wgd_workspace(need, dw.device)
    rc = int(k.cxn_conv_wgrad_rowrun(x.data_ptr(), dy.data_ptr(), dw.data_ptr(), ws.data_ptr(), ws.numel(), *args, 1.0,
                                     _stream()))
    if rc == -1:
        return False
    native.check(rc, "conv_wgrad_rowrun")
    return True


def conv_backward_weight(x, dy, dw, g: ConvGeom, db=None) -> bool:
    """dw += sum over pixels of dy (x) im2col(x).  dw fp32 [Cout][KH][KW][Cg].  db (fp32 [Cout],
    optional): the kernel may also add the bias gradient (sum of dy over pixels); returns True
    when it did (else the caller sums dy itself).
    (Folding the bias gradient into this GEMM was measured a wash on GoogLeNet and its
    extra registers slowed every weight-grad kernel by 5-25%: profiles/r2_inception_bias_fold.md,
    profiles/r2_ab_bias_fold_regression.md.)"""
    if not _native_t(x):
        xn = x.permute(0, 3, 1, 2)
        dyn = dy.permute(0, 3, 1, 2)
        gw = torch.nn.grad.conv2d_weight(xn, (g.Cout, g.cg_in, g.KH, g.KW), dyn, stride=g.stride,
                                         padding=(g.pad_y, g.pad_x), groups=g.groups)
        dw.add_(gw.permute(0, 2, 3, 1))
        return
    cg = g.cg_in
    va = 8 if cg % 8 == 0 else 4
    kd = g.kdim
    P = g.N * g.Ho * g.Wo
    A = _op(x, cg, 0, kd, P, H=g.H, W=g.W, C=_pix(x), Ho=g.Ho, Wo=g.Wo, KH=g.KH, KW=g.KW, stride=g.stride,
            pad_h=g.pad_y, pad_w=g.pad_x, dil=1, Cg=cg)
    B = _op(dy, g.cg_out, _pix(dy), g.cg_out, P)

    def reg_run(code, o):
        _gemm(A, B, GATHER_MN, DIRECT_MN, va, 8, o, g.cg_out * kd, kd, epi=EPI_F32_ATOMIC, groups=g.groups,
              ksplit=code % 100000, tile=code // 100000)
        return True

    def reg_default():
        tile = _pick(WGRAD_TILES, kd, g.cg_out, g.groups, min_blocks=1)
        return tile * 100000 + _auto_split(kd, g.cg_out, g.groups, P, tile)

    def reg(o):
        if _glds_cfg["tile"] >= 0:  # a forced LDS-DMA tile id means nothing here
            return reg_run(reg_default(), o)
        key = ("cws", g.N, g.H, g.W, g.C, g.Cout, g.KH, g.KW, g.stride, g.pad_y, g.pad_x, g.groups)
        return reg_run(_tuned_tile(key, reg_run, o, reg_default, cands=_wgrad_cands(kd, g.cg_out, g.groups, P)), o)
    rowrun = va != 8 and rowrun_ok(g)
    if conv_wgrad_direct(x, dy, dw, g, db=db):  # deterministic as well: no atomics, fixed split order
        return db is not None
    if g.C <= 4 and conv_wgrad_rowrun(x, dy, dw, g):  # few-channel first layers (likewise deterministic)
        return False
    if _DET["on"] and not (rowrun and cg % va):
        # one fp32 slab per K slice, summed in slice order into dw: bitwise reproducible
        tile = _pick(WGRAD_TILES, kd, g.cg_out, g.groups, min_blocks=1)
        split = _effective_split(P, _auto_split(kd, g.cg_out, g.groups, P, tile))
        slab = g.Cout * kd
        ws = _det_ws(split * slab, dw.device)
        _gemm(A, B, GATHER_MN, DIRECT_MN, va, 8, ws, g.cg_out * kd, kd, epi=EPI_F32, groups=g.groups,
              ksplit=split, tile=tile, kstride=slab)
        native.check(native.kernels().cxn_splitk_accumulate(ws.data_ptr(), split, slab, dw.data_ptr(), _stream()),
                     "splitk_accumulate")
        return
    if _use("cw") and va == 8:
        def run(t, o):
            if t == REG:
                return reg(o)
            bm, bn = GLDS_TILES[t]
            tiles = _cdiv(kd, bm) * _cdiv(g.cg_out, bn) * g.groups
            split = max(1, min(2 * NUM_CU // max(tiles, 1), _cdiv(P, 64) // 16))
            return _glds(A, B, GL_MNG, GL_MN, o, g.cg_out * kd, kd, epi=EPI_F32_ATOMIC_G, groups=g.groups,
                         ksplit=split, tile=t)
        key = ("cw", g.N, g.H, g.W, g.C, g.Cout, g.KH, g.KW, g.stride, g.pad_y, g.pad_x, g.groups)
        # shapes missing from the table keep the register kernel: timed alone, the LDS-DMA form
        # wins shapes where it loses inside the step (conv2/conv3 above)
        if run(_tuned_tile(key, run, dw, lambda: REG, extra=(REG,), tune=_CW_TUNE), dw):
            return
    if rowrun and (_use("cwr") or g.C % 4 or _DET["on"]):
        # few input channels (conv1): the KW*C im2col rows of one kernel row are one contiguous run
        # of x, so the transposed gather reads each run as Cg = roundup(KW*C, 8) "channels" of a
        # 1-wide kernel; the result lands in a row-padded fp32 buffer whose pad columns are dropped
        lp = (g.KW * g.C + 7) // 8 * 8
        kr = g.KH * lp
        Ar = _op(x, lp, 0, kr, P, H=g.H, W=g.W, C=g.C, Ho=g.Ho, Wo=g.Wo, KH=g.KH, KW=1, stride=g.stride,
                 pad_h=0, pad_w=0, dil=1, Cg=lp)
        ws = _wgrad_pad_buf(g.Cout, kr, dw.device)

        def run(t, o):
            bm, bn = GLDS_TILES[t]
            split = max(1, min(2 * NUM_CU // max(_cdiv(kr, bm) * _cdiv(g.Cout, bn), 1), _cdiv(P, 64) // 16))
            if _DET["on"]:  # one K slice: each output is one atomic add onto zero, bitwise reproducible
                split = 1
            return _glds(Ar, B, GL_MNG, GL_MN, o, 0, kr, epi=EPI_F32_ATOMIC_G, ksplit=split, tile=t)
        key = ("cwr", g.N, g.H, g.W, g.C, g.Cout, g.KH, g.KW, g.stride)
        from .nn import zero_
        zero_(ws)  # library memset / add below: a replayed launch list repeats them (torch ops it would not)
        if run(_tuned_tile(key, run, ws, lambda: 1), ws):
            _add_rows(ws, dw, g.Cout * g.KH, g.KW * g.C, lp)
            return
    if cg % va:
        raise RuntimeError(f"conv weight-grad: no GPU kernel for {cg} channels per group ({g})")
    reg(dw)


# ----------------------------------------------------------------------------- fully connected
def fc_forward(x, w, bias, y, relu=False, out_fp32=False, drop=None):
    """y[B][nout] = x[B][nin] . w[nout][nin]^T + bias.  drop = (seed, counter, pkeep): then
    y = dropout(y) as ops.dropout_apply(y, y, seed, pkeep, counter) (fused into the split-K
    finalize where the GEMM takes that path)."""
    if not _native_t(x):
        out = x @ w.t()
        if bias is not None:
            out = out + bias
        if relu:
            out = out.clamp_min(0)
        y.copy_(out)
        if drop is not None:
            from .nn import dropout_apply
            dropout_apply(y, y, drop[0], drop[2], drop[1])
        return
    Bn, nin = x.shape
    nout = w.shape[0]
    A = _op(w, 0, nin, nout, nin)
    Bo = _op(x, 0, nin, Bn, nin)
    if out_fp32:
        _gemm(A, Bo, DIRECT_K, DIRECT_K, 8, 8, y, 0, nout, bias=bias, relu=relu, epi=EPI_F32)
        done = False
    else:
        done = _gemm_bf16_out(A, Bo, DIRECT_K, DIRECT_K, y, nout, bias=bias, relu=relu, drop=drop)
    if drop is not None and not done:
        from .nn import dropout_apply
        dropout_apply(y, y, drop[0], drop[2], drop[1])


def fc_backward_data(dy, w, dx, mask_relu=False, alpha=1.0):
    """dx[B][nin] = alpha * dy[B][nout] . w[nout][nin]  (mask_relu: see conv_backward_data;
    with the dropout of a fused fc -> relu -> dropout in front, alpha = 1 / pkeep: dx already
    holds the dropped-out activation, so relu'-masking by it applies the dropout mask too)."""
    if not _native_t(dy):
        out = dy @ w
        if alpha != 1.0:
            out = out * alpha
        if mask_relu:
            out = out * (dx > 0).to(out.dtype)
        dx.copy_(out)
        return
    Bn, nout = dy.shape
    nin = w.shape[1]
    A = _op(w, 0, nin, nin, nout)
    Bo = _op(dy, 0, nout, Bn, nout)
    _gemm_bf16_out(A, Bo, DIRECT_MN, DIRECT_K, dx, nin, mask_relu=mask_relu, alpha=alpha)


def fc_backward_weight_sgd(x, dy, w, m, wb, lr, wd, mom, clip, hyp=None) -> bool:
    """The fc weight-gradient dy^T . x fused with the SGD step of those weights: the
    epilogue applies m = mom*m - lr*(clip(g) + wd*w); w += m; wb = bf16(w) to the fp32
    master w, momentum m and bf16 shadow wb ([nout][nin] slices of the arena) and the
    gradient never goes to memory.  Same arithmetic as the fused optimizer, so the
    result is bitwise the unfused one.  False when the LDS-DMA kernel does not cover the
    shape (the caller then takes the unfused path).  hyp (fp32 device [4], optional): the
    kernel reads (lr, wd, mom, clip) from it instead -- a recorded / captured step then follows
    the schedule through a per-step host-to-device refresh of hyp."""
    if not (_native_t(x) and _glds_cfg["on"] and _use("fw")):
        return False
    Bn, nin = x.shape
    nout = dy.shape[1]
    A = _op(x, 0, nin, nin, Bn)
    Bo = _op(dy, 0, nout, nout, Bn)
    # the SGD epilogue streams w / m / wb: its own tile entry ("fws"), else the plain weight-grad one
    tile = _glds_cfg["tile"]
    if tile < 0:
        tile = _TUNE.get(f"fws|{nin}|{nout}|{Bn}")
        if tile is None:
            tile = _TUNE.get(f"fw|{nin}|{nout}|{Bn}", 1)
    rc = native.kernels().cxn_gemm_glds_sgd(A, Bo, nin, 1.0, w.data_ptr(), m.data_ptr(), wb.data_ptr(), float(lr),
                                            float(wd), float(mom), float(clip),
                                            hyp.data_ptr() if hyp is not None else None, tile, _stream())
    if rc == -1:
        return False
    native.check(rc, "gemm_glds_sgd")
    return True


def fc_backward_weight(x, dy, dw, overwrite=False):
    """dw[nout][nin] += dy^T . x  (fp32 accumulate; overwrite=True stores instead)."""
    if not _native_t(x):
        if overwrite:
            dw.copy_(dy.t() @ x)
        else:
            dw.add_(dy.t() @ x)
        return
    Bn, nin = x.shape
    nout = dy.shape[1]
    A = _op(x, 0, nin, nin, Bn)
    Bo = _op(dy, 0, nout, nout, Bn)
    if _use("fw"):
        epi = EPI_F32 if overwrite else EPI_F32_ACC_G
        run = lambda t, o: _glds(A, Bo, GL_MN, GL_MN, o, 0, nin, epi=epi, tile=t)  # noqa: E731
        if overwrite:
            tile = _tuned_tile(("fw", nin, nout, Bn), run, dw, lambda: 1)
        else:  # += epilogue: never time it on the live buffer
            tile = _TUNE.get(f"fw|{nin}|{nout}|{Bn}", 1) if _glds_cfg["tile"] < 0 else _glds_cfg["tile"]
        if run(tile, dw):
            return
    _gemm(A, Bo, DIRECT_MN, DIRECT_MN, 8, 8, dw, 0, nin, epi=EPI_F32 if overwrite else EPI_F32_ACC)
