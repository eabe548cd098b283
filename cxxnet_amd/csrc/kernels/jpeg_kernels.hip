// GPU half of the JPEG decode stage: dequantise + islow IDCT of every staged coefficient block,
// then fancy chroma upsampling + YCbCr->RGB + crop + mirror into the uint8 batch the image
// kernel (nn_kernels.hip image_u8_*) turns into the network input.
//
// Reference behaviour: src/utils/decoder.h:21-104 (libjpeg decode of one record to RGB) and the
// crop / mirror of src/io/iter_augment_proc-inl.hpp:98-162.  The host (runtime/jpeg_decode.h
// ReadCoefCrop) keeps only the entropy decoding; the arithmetic here is libjpeg's integer
// arithmetic (jidctint.c islow IDCT with 64-bit intermediates, jdsample.c h2v1 / h2v2 fancy
// upsampling with edge replication, jdcolor.c fixed-point YCbCr->RGB), so the batch is
// bit-identical to libjpeg-turbo's decode of the same crop (tests/test_jpeg_stage_*).
//
// Layout (see runtime/jpeg_decode.h CoefStage): coef int16 [nblk][64] natural-order blocks,
// bwin int32 [nblk] window id (row * 3 + component), meta int32 [B][3][80] window tables.
// Samples are written block-linear (plane[blk][64]), in the coefficient block order, so the
// IDCT needs no geometry at all and the colour kernel finds a sample through its window.
#include <cstdlib>

#include "common.h"

namespace {

constexpr int kMeta = 80, kBlk0 = 0, kBw = 1, kBh = 2, kBy0 = 3, kBx0 = 4, kDw = 5, kDh = 6, kRh = 7, kRv = 8,
              kNcomp = 9, kValid = 10, kQuant = 16;

// jidctint.c constants (CONST_BITS 13, PASS1_BITS 2)
constexpr long long F0298 = 2446, F0390 = 3196, F0541 = 4433, F0765 = 6270, F0899 = 7373, F1175 = 9633,
                    F1501 = 12299, F1847 = 15137, F1961 = 16069, F2053 = 16819, F2562 = 20995, F3072 = 25172;

__device__ __forceinline__ long long descale(long long x, int n) { return (x + (1LL << (n - 1))) >> n; }

// One 8-point islow IDCT (jidctint.c jpeg_idct_islow, either pass): in[0..7] -> o[0..7] before
// the pass's descale; `shift` = that pass's descale.
__device__ __forceinline__ void idct8(const long long *in, long long *o, int shift) {
  long long z2 = in[2], z3 = in[6];
  long long z1 = (z2 + z3) * F0541;
  long long tmp2 = z1 - z3 * F1847, tmp3 = z1 + z2 * F0765;
  long long tmp0 = (in[0] + in[4]) * (1LL << 13), tmp1 = (in[0] - in[4]) * (1LL << 13);
  const long long t10 = tmp0 + tmp3, t13 = tmp0 - tmp3, t11 = tmp1 + tmp2, t12 = tmp1 - tmp2;
  tmp0 = in[7], tmp1 = in[5], tmp2 = in[3], tmp3 = in[1];
  z1 = tmp0 + tmp3, z2 = tmp1 + tmp2, z3 = tmp0 + tmp2;
  long long z4 = tmp1 + tmp3;
  const long long z5 = (z3 + z4) * F1175;
  tmp0 *= F0298, tmp1 *= F2053, tmp2 *= F3072, tmp3 *= F1501;
  z1 *= -F0899, z2 *= -F2562, z3 *= -F1961, z4 *= -F0390;
  z3 += z5, z4 += z5;
  tmp0 += z1 + z3, tmp1 += z2 + z4, tmp2 += z2 + z3, tmp3 += z1 + z4;
  o[0] = descale(t10 + tmp3, shift), o[7] = descale(t10 - tmp3, shift);
  o[1] = descale(t11 + tmp2, shift), o[6] = descale(t11 - tmp2, shift);
  o[2] = descale(t12 + tmp1, shift), o[5] = descale(t12 - tmp1, shift);
  o[3] = descale(t13 + tmp0, shift), o[4] = descale(t13 - tmp0, shift);
}

// libjpeg's post-IDCT range-limit table (jdmaster.c prepare_range_limit_table) as arithmetic:
// index (value & 1023): [0,128) -> +128, [128,512) -> 255, [512,896) -> 0, [896,1024) -> -896
__device__ __forceinline__ uint32_t idct_limit(long long v) {
  const int j = static_cast<int>(v) & 1023;
  return j < 128 ? j + 128 : j < 512 ? 255u : j < 896 ? 0u : j - 896;
}

// 8 threads per block, 32 blocks per workgroup: thread (blk, r) loads row r of the block (16 B,
// the wave reads 1 KB contiguous), dequantises into LDS; pass 1 = column r, pass 2 = row r.
__global__ void __launch_bounds__(256) jpeg_idct(const int16_t *__restrict__ coef, const int *__restrict__ bwin,
                                                 const int *__restrict__ meta, long nblk, uint8_t *__restrict__ plane) {
  __shared__ int deq[32][8][9];
  __shared__ int ws[32][8][9];
  const int lb = threadIdx.x >> 3, r = threadIdx.x & 7;
  const long blk = static_cast<long>(blockIdx.x) * 32 + lb;
  const bool live = blk < nblk;
  if (live) {
    const int4 raw = *reinterpret_cast<const int4 *>(coef + blk * 64 + r * 8);
    const int *q = meta + static_cast<long>(bwin[blk]) * kMeta + kQuant + r * 8;
    const int4 q0 = *reinterpret_cast<const int4 *>(q), q1 = *reinterpret_cast<const int4 *>(q + 4);
    const int16_t *c = reinterpret_cast<const int16_t *>(&raw);
    const int qq[8] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w};
#pragma unroll
    for (int k = 0; k < 8; ++k) deq[lb][r][k] = static_cast<int>(c[k]) * qq[k];
  }
  __syncthreads();
  if (live) {  // pass 1: column r
    long long in[8], o[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) in[k] = deq[lb][k][r];
    idct8(in, o, 13 - 2);
#pragma unroll
    for (int k = 0; k < 8; ++k) ws[lb][k][r] = static_cast<int>(o[k]);
  }
  __syncthreads();
  if (live) {  // pass 2: row r
    long long in[8], o[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) in[k] = ws[lb][r][k];
    idct8(in, o, 13 + 2 + 3);
    uint2 out;
    out.x = idct_limit(o[0]) | idct_limit(o[1]) << 8 | idct_limit(o[2]) << 16 | idct_limit(o[3]) << 24;
    out.y = idct_limit(o[4]) | idct_limit(o[5]) << 8 | idct_limit(o[6]) << 16 | idct_limit(o[7]) << 24;
    *reinterpret_cast<uint2 *>(plane + blk * 64 + r * 8) = out;
  }
}

struct Win {
  int blk0, bw, by0, bx0, dw, dh, rh, rv;
};

__device__ __forceinline__ Win load_win(const int *m) {
  return Win{m[kBlk0], m[kBw], m[kBy0], m[kBx0], m[kDw], m[kDh], m[kRh], m[kRv]};
}

// component sample (sy, sx) (component grid; inside the staged window by construction)
__device__ __forceinline__ int sample(const uint8_t *__restrict__ plane, const Win &w, int sy, int sx) {
  const long b = w.blk0 + static_cast<long>((sy >> 3) - w.by0) * w.bw + ((sx >> 3) - w.bx0);
  return plane[b * 64 + (sy & 7) * 8 + (sx & 7)];
}

// chroma at luma position (Y, X): jdsample.c fancy upsampling (h2v2: triangle filter over the
// 3*nearer + farther row sums; h2v1: 3*nearer + farther; rows / columns past the edge repeat it)
__device__ __forceinline__ int chroma(const uint8_t *__restrict__ plane, const Win &w, int Y, int X) {
  if (w.rh == 1) return sample(plane, w, Y, X);
  const int cx = X >> 1;
  const bool odd = X & 1;
  if (w.rv == 1) {
    const int s = sample(plane, w, Y, cx);
    if (!odd) return cx == 0 ? s : (3 * s + sample(plane, w, Y, cx - 1) + 1) >> 2;
    return cx == w.dw - 1 ? s : (3 * s + sample(plane, w, Y, cx + 1) + 2) >> 2;
  }
  const int cy = Y >> 1;
  const int ny = (Y & 1) ? min(cy + 1, w.dh - 1) : max(cy - 1, 0);
  auto colsum = [&](int c) { return 3 * sample(plane, w, cy, c) + sample(plane, w, ny, c); };
  const int t = colsum(cx);
  if (!odd) return cx == 0 ? (t * 4 + 8) >> 4 : (3 * t + colsum(cx - 1) + 8) >> 4;
  return cx == w.dw - 1 ? (t * 4 + 7) >> 4 : (3 * t + colsum(cx + 1) + 7) >> 4;
}

__device__ __forceinline__ uint32_t clamp255(int v) { return static_cast<uint32_t>(min(max(v, 0), 255)); }

// one thread per output pixel of the crop; grid (cdiv(w, 256), B * h)
__global__ void __launch_bounds__(256) jpeg_color(const uint8_t *__restrict__ plane, const int *__restrict__ meta,
                                                  const int *__restrict__ prm, int h, int w, int C,
                                                  uint8_t *__restrict__ out) {
  const int x = blockIdx.x * blockDim.x + threadIdx.x;
  const int b = blockIdx.y / h, y = blockIdx.y - b * h;
  if (x >= w) return;
  const int *m = meta + static_cast<long>(b) * 3 * kMeta;
  uint8_t *o = out + (static_cast<long>(blockIdx.y) * w + x) * C;
  if (m[kValid] == 0) {  // padding row, another rank's row, or one the CPU decodes
    for (int k = 0; k < C; ++k) o[k] = 0;
    return;
  }
  const int Y = prm[b * 4] + y, X = prm[b * 4 + 1] + (prm[b * 4 + 2] ? w - 1 - x : x);
  const int yv = sample(plane, load_win(m), Y, X);
  uint32_t rgb[3];
  if (m[kNcomp] == 1) {
    rgb[0] = rgb[1] = rgb[2] = static_cast<uint32_t>(yv);
  } else {
    // jdcolor.c build_ycc_rgb_table (SCALEBITS 16) evaluated in place
    const int cb = chroma(plane, load_win(m + kMeta), Y, X) - 128;
    const int cr = chroma(plane, load_win(m + 2 * kMeta), Y, X) - 128;
    rgb[0] = clamp255(yv + ((91881 * cr + 32768) >> 16));
    rgb[1] = clamp255(yv + ((-46802 * cr + -22554 * cb + 32768) >> 16));
    rgb[2] = clamp255(yv + ((116130 * cb + 32768) >> 16));
  }
  for (int k = 0; k < C; ++k) o[k] = static_cast<uint8_t>(rgb[k]);
}

// The same output, one thread per pair of source columns (2c, 2c + 1): the two pixels share their
// chroma column c, so the triangle filter's row sums of c and its neighbours are loaded once for
// both (h2v2: 6 chroma gathers per component for two pixels instead of 8), and the window / crop
// fields are read once per two pixels.  grid (cdiv(pairs, 64), B * h), 64 threads.
__global__ void __launch_bounds__(64) jpeg_color2(const uint8_t *__restrict__ plane, const int *__restrict__ meta,
                                                  const int *__restrict__ prm, int h, int w, int C,
                                                  uint8_t *__restrict__ out) {
  const int b = blockIdx.y / h, y = blockIdx.y - b * h;
  const int *m = meta + static_cast<long>(b) * 3 * kMeta;
  const int xx = prm[b * 4], mir = prm[b * 4 + 2];
  const int c = (prm[b * 4 + 1] >> 1) + static_cast<int>(blockIdx.x * blockDim.x + threadIdx.x);
  const int X0 = 2 * c, x0 = X0 - prm[b * 4 + 1];  // crop column of source column X0 (x0 + 1 for X0 + 1)
  const bool v0 = x0 >= 0 && x0 < w, v1 = x0 + 1 >= 0 && x0 + 1 < w;
  if (!v0 && !v1) return;
  uint8_t *orow = out + static_cast<long>(blockIdx.y) * w * C;
  const int o0 = mir ? w - 1 - x0 : x0, o1 = mir ? w - 2 - x0 : x0 + 1;
  if (m[kValid] == 0) {
    for (int k = 0; k < C; ++k) {
      if (v0) orow[o0 * C + k] = 0;
      if (v1) orow[o1 * C + k] = 0;
    }
    return;
  }
  (void)xx;
  const int Y = prm[b * 4] + y;
  const Win wl = load_win(m);
  const int y0 = v0 ? sample(plane, wl, Y, X0) : 0, y1 = v1 ? sample(plane, wl, Y, X0 + 1) : 0;
  uint32_t rgb0[3], rgb1[3];
  if (m[kNcomp] == 1) {
    rgb0[0] = rgb0[1] = rgb0[2] = static_cast<uint32_t>(y0);
    rgb1[0] = rgb1[1] = rgb1[2] = static_cast<uint32_t>(y1);
  } else {
    int ch0[2], ch1[2];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const Win wc = load_win(m + (k + 1) * kMeta);
      if (wc.rh == 1) {
        ch0[k] = v0 ? sample(plane, wc, Y, X0) : 0;
        ch1[k] = v1 ? sample(plane, wc, Y, X0 + 1) : 0;
      } else if (wc.rv == 1) {  // h2v1: 3 * nearer + farther, edges repeat
        const int s = sample(plane, wc, Y, c);
        ch0[k] = c == 0 ? s : (3 * s + sample(plane, wc, Y, c - 1) + 1) >> 2;
        ch1[k] = c == wc.dw - 1 ? s : (3 * s + sample(plane, wc, Y, c + 1) + 2) >> 2;
      } else {  // h2v2: the column sums 3 * nearer row + farther row of c - 1, c, c + 1
        const int cy = Y >> 1;
        const int ny = (Y & 1) ? min(cy + 1, wc.dh - 1) : max(cy - 1, 0);
        const int t = 3 * sample(plane, wc, cy, c) + sample(plane, wc, ny, c);
        ch0[k] = c == 0 ? (t * 4 + 8) >> 4
                        : (3 * t + 3 * sample(plane, wc, cy, c - 1) + sample(plane, wc, ny, c - 1) + 8) >> 4;
        ch1[k] = c == wc.dw - 1 ? (t * 4 + 7) >> 4
                                : (3 * t + 3 * sample(plane, wc, cy, c + 1) + sample(plane, wc, ny, c + 1) + 7) >> 4;
      }
    }
    const int cb0 = ch0[0] - 128, cr0 = ch0[1] - 128, cb1 = ch1[0] - 128, cr1 = ch1[1] - 128;
    rgb0[0] = clamp255(y0 + ((91881 * cr0 + 32768) >> 16));
    rgb0[1] = clamp255(y0 + ((-46802 * cr0 + -22554 * cb0 + 32768) >> 16));
    rgb0[2] = clamp255(y0 + ((116130 * cb0 + 32768) >> 16));
    rgb1[0] = clamp255(y1 + ((91881 * cr1 + 32768) >> 16));
    rgb1[1] = clamp255(y1 + ((-46802 * cr1 + -22554 * cb1 + 32768) >> 16));
    rgb1[2] = clamp255(y1 + ((116130 * cb1 + 32768) >> 16));
  }
  for (int k = 0; k < C; ++k) {
    if (v0) orow[o0 * C + k] = static_cast<uint8_t>(rgb0[k]);
    if (v1) orow[o1 * C + k] = static_cast<uint8_t>(rgb1[k]);
  }
}

}  // namespace

#define S_ static_cast<hipStream_t>(stream)
#define RET return hipGetLastError() == hipSuccess ? 0 : -3

// coef int16 [nblk][64] (16-byte aligned), bwin int32 [nblk], meta int32 [B][3][80], plane uint8 [nblk][64]
CXN_API int cxn_jpeg_idct(const void *coef, const int *bwin, const int *meta, long nblk, void *plane, void *stream) {
  if (nblk <= 0) return 0;
  if (reinterpret_cast<uintptr_t>(coef) % 16 != 0 || reinterpret_cast<uintptr_t>(meta) % 16 != 0 ||
      reinterpret_cast<uintptr_t>(plane) % 8 != 0)
    return -2;
  CXN_LAUNCH((jpeg_idct), cdiv(nblk, 32), 256, 0, S_, (const int16_t *)coef, bwin, meta, nblk, (uint8_t *)plane);
  RET;
}

// plane from cxn_jpeg_idct, prm int32 [B][4] (crop y, x, mirrored) -> out uint8 [B][h][w][C]
CXN_API int cxn_jpeg_color(const void *plane, const int *meta, const int *prm, int B, int h, int w, int C, void *out,
                           void *stream) {
  if (C < 1 || C > 3 || B <= 0 || h <= 0 || w <= 0) return -2;
  static const int pairs_env = [] {  // CXN_JPEG_COLOR_PAIRS=0: the one-pixel-per-thread kernel (A/B)
    const char *e = getenv("CXN_JPEG_COLOR_PAIRS");
    return e != nullptr ? atoi(e) : 1;
  }();
  if (pairs_env) {  // w / 2 + 1 column pairs cover any crop start parity
    CXN_LAUNCH((jpeg_color2), dim3(cdiv(w / 2 + 1, 64), B * h), 64, 0, S_, (const uint8_t *)plane, meta, prm, h, w,
               C, (uint8_t *)out);
    RET;
  }
  CXN_LAUNCH((jpeg_color), dim3(cdiv(w, 256), B * h), 256, 0, S_, (const uint8_t *)plane, meta, prm, h, w, C,
             (uint8_t *)out);
  RET;
}
