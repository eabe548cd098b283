// Memory-bound layer kernels for gfx950, all on NHWC bf16 activations with
// 16-byte (8 x bf16) vector accesses per lane.
//
//   layout      : NCHW fp32 -> NHWC bf16 (input, channel pad), NHWC -> NCHW, conv weight flip
//   pooling     : max/sum/avg fwd + gather-form bwd (reference src/layer/pooling_layer-inl.hpp:42-111)
//   lrn         : cross-channel LRN fwd/bwd      (reference src/layer/lrn_layer-inl.hpp:53-74)
//   activation  : relu/sigmoid/tanh/xelu fwd/bwd (reference src/layer/op.h, activation_layer-inl.hpp)
//   dropout     : counter-hash mask, no mask storage (reference src/layer/dropout_layer-inl.hpp:44-57)
//   softmax     : row softmax + (p - onehot) * scale grad on device (reference loss/softmax_layer-inl.hpp)
//   bias grad   : column sums of an [rows][C] bf16 matrix into fp32 (reference K5/K11)
#include "common.h"

namespace {

constexpr int NT = 256;

__device__ __forceinline__ int grid_stride_start() { return blockIdx.x * blockDim.x + threadIdx.x; }
__device__ __forceinline__ int grid_stride() { return gridDim.x * blockDim.x; }

static inline int nblocks(long n, int per_block = NT, int cap = 256 * 16) {
  long b = (n + per_block - 1) / per_block;
  if (b < 1) b = 1;
  return static_cast<int>(b > cap ? cap : b);
}

// ------------------------------------------------------------------ layout
// x: NCHW fp32 [N][C][H][W] -> y: NHWC bf16 [N][H][Wp][Cp] (channels >= C zero-filled; columns
// >= W of a row-padded node are left as they are)
__global__ void nchw_f32_to_nhwc_bf16(const float *__restrict__ x, bf16_t *__restrict__ y, int N, int C, int H,
                                      int W, int Cp, int Wp, float scale) {
  const long total = static_cast<long>(N) * H * W;
  for (long pix = grid_stride_start(); pix < total; pix += grid_stride()) {
    const long n = pix / (static_cast<long>(H) * W);
    const long hw = pix - n * H * W;
    const float *src = x + n * C * H * W + hw;
    const long row = pix / W;
    bf16_t *dst = y + (row * Wp + (pix - row * W)) * Cp;
    if (Cp == 4) {
      float v[4];
#pragma unroll
      for (int c = 0; c < 4; ++c) v[c] = c < C ? src[static_cast<long>(c) * H * W] * scale : 0.f;
      *reinterpret_cast<uint2 *>(dst) = make_uint2(pack2(v[0], v[1]),
                                                   pack2(v[2], v[3]));
      continue;
    }
    for (int c = 0; c < Cp; ++c) dst[c] = c < C ? f2bf(src[static_cast<long>(c) * H * W] * scale) : 0;
  }
}

// Decoded image batch -> NHWC bf16 input node, with the reference augmenter's
// arithmetic fused in (src/io/iter_augment_proc-inl.hpp:98-162).  The host has
// already cropped and mirrored the uint8 pixels (cheap row copies); mean
// subtraction, contrast, illumination, scale and the bf16/NHWC/channel-pad
// conversion run here so only uint8 crosses PCIe.
//   pix  u8 [B][h][w][C]          prm int [B][4] = {crop_y, crop_x, mirrored, 0}
//   cm   f32 [B][2] = {contrast, illumination}
//   mode 0: y = d*scale                      (no mean)
//        1: y = ((d - mean[c])*ct + il)*scale (mean_value)
//        2: mean image [C][Hm][Wm] of the uncropped size, read at the crop offset
//        3: mean image [C][h][w] of the crop size
__global__ void image_u8_to_nhwc_bf16(const uint8_t *__restrict__ pix, const int *__restrict__ prm,
                                      const float *__restrict__ cm, const float *__restrict__ mean, int B, int h,
                                      int w, int C, int Cp, int Wp, int Hm, int Wm, int mode, float scale,
                                      bf16_t *__restrict__ y) {
  // grid: x over blockIdx.x*NT + tid, one image row (b, r) per blockIdx.y: no per-pixel division
  const int row = blockIdx.y;
  const int b = row / h, r = row - b * h;
  const int x = blockIdx.x * blockDim.x + threadIdx.x;
  if (x >= w) return;
  const long p = static_cast<long>(row) * w + x;
  const uint8_t *src = pix + p * C;
  float ct = 1.f, il = 0.f;
  if (mode != 0) {
    ct = cm[2 * b];
    il = cm[2 * b + 1];
  }
  const int xs = (mode == 2 && prm[4 * b + 2]) ? (w - 1 - x) : x;
  float v[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    v[c] = 0.f;
    if (c < C && c < Cp) {
      const float d = static_cast<float>(src[c]);
      if (mode == 0) {
        v[c] = d * scale;
      } else {
        float m;
        if (mode == 1) m = mean[c];
        else if (mode == 2) m = mean[(static_cast<long>(c) * Hm + prm[4 * b] + r) * Wm + prm[4 * b + 1] + xs];
        else m = mean[(static_cast<long>(c) * h + r) * w + x];
        v[c] = ((d - m) * ct + il) * scale;
      }
    }
  }
  bf16_t *dst = y + (static_cast<long>(row) * Wp + x) * Cp;
  if (Cp == 4) {  // one 8-byte store per pixel
    *reinterpret_cast<uint2 *>(dst) = make_uint2(pack2(v[0], v[1]),
                                                 pack2(v[2], v[3]));
  } else {
    for (int c = 0; c < Cp; ++c) dst[c] = c < 8 ? f2bf(v[c]) : static_cast<bf16_t>(0);
  }
}

// Fast path of the above for the common case: C = 3, Cp = 4, mode 0/1, pixel count a
// multiple of 4.  Four pixels per thread: three aligned 4-byte loads, two 16-byte stores.
__global__ void image_u8c3_nhwc4(const uint32_t *__restrict__ pix, const float *__restrict__ cm,
                                 const float *__restrict__ mean, long quads, FastDiv fd_hw, int mode, float scale,
                                 uint4 *__restrict__ y) {
  for (long q = grid_stride_start(); q < quads; q += grid_stride()) {
    const uint32_t w0 = pix[3 * q], w1 = pix[3 * q + 1], w2 = pix[3 * q + 2];
    const uint32_t bytes[3] = {w0, w1, w2};
    float out[16];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t p = static_cast<uint32_t>(4 * q + k);
      float ct = 1.f, il = 0.f;
      if (mode == 1) {
        const uint32_t b = fdiv(p, fd_hw);
        ct = cm[2 * b];
        il = cm[2 * b + 1];
      }
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const int byte = 3 * k + c;
        const float d = static_cast<float>((bytes[byte >> 2] >> (8 * (byte & 3))) & 0xffu);
        out[4 * k + c] = mode == 1 ? ((d - mean[c]) * ct + il) * scale : d * scale;
      }
      out[4 * k + 3] = 0.f;
    }
    y[2 * q] = pack8(out);
    y[2 * q + 1] = pack8(out + 8);
  }
}

// Fast path for the row-padded 3-channel node of a first conv on kernel-row runs
// (NeuralNet._pad_input_channels: AlexNet conv1 reads [B][h][Wp][3] with Wp % 4 == 0, so every
// image row and every 4-pixel group starts 8-byte aligned): one thread per 4 output pixels of a
// padded row, three 8-byte stores; the pad columns (x >= w) get zeros.  mode 0/1.  The 12 source
// bytes of a group start at any byte (rows of w*3 bytes): 4 aligned dword loads + alignbyte.
// Consecutive groups are consecutive 24-byte pieces of y (Wp % 4 == 0), so a full wave's output is
// one 1536-byte run: it goes through LDS and out as 16-byte stores (two per lane, the second on
// half the lanes) instead of three 8-byte stores at a 24-byte lane stride.
__global__ void __launch_bounds__(NT)
image_u8c3_nhwc3p(const uint32_t *__restrict__ pix, long ndw, const float *__restrict__ cm,
                  const float *__restrict__ mean, FastDiv fd_qpr, FastDiv fd_h, int w, int Wp,
                  int mode, float scale, uint32_t total, uint2 *__restrict__ y) {
  __shared__ uint2 stage[NT * 3];
  const uint32_t q0 = blockIdx.x * blockDim.x + (threadIdx.x & ~63u);  // first group of this wave
  const uint32_t q = q0 + (threadIdx.x & 63u);
  if (q0 >= total) return;  // whole wave past the end
  const bool full = q0 + 64 <= total;
  if (!full && q >= total) return;  // (a partial wave stores directly below)
  const uint32_t row = fdiv(q, fd_qpr);
  const int x0 = static_cast<int>(q - row * fd_qpr.d) * 4;
  float ct = 1.f, il = 0.f;
  if (mode == 1) {
    const uint32_t b = fdiv(row, fd_h);
    ct = cm[2 * b];
    il = cm[2 * b + 1];
  }
  const long start = (static_cast<long>(row) * w + x0) * 3;
  const long d0 = start >> 2;
  const uint32_t sh = static_cast<uint32_t>(start & 3) * 8;
  uint32_t d[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) d[t] = pix[min(d0 + t, ndw - 1)];
  // bytes start .. start + 11 of the image batch as three dwords
  const uint32_t e[3] = {__builtin_amdgcn_alignbyte(d[1], d[0], sh >> 3), __builtin_amdgcn_alignbyte(d[2], d[1], sh >> 3),
                         __builtin_amdgcn_alignbyte(d[3], d[2], sh >> 3)};
  float out[12];
#pragma unroll
  for (int k = 0; k < 4; ++k)
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const int byte = 3 * k + c;
      float v = 0.f;
      if (x0 + k < w) {
        const float dv = static_cast<float>((e[byte >> 2] >> (8 * (byte & 3))) & 0xffu);
        v = mode == 1 ? ((dv - mean[c]) * ct + il) * scale : dv * scale;
      }
      out[3 * k + c] = v;
    }
  if (!full) {
    uint2 *dst = y + (static_cast<long>(row) * Wp + x0) * 3 / 4;  // 4 pixels = 24 bytes = three uint2
#pragma unroll
    for (int t = 0; t < 3; ++t)
      dst[t] = make_uint2(pack2(out[4 * t], out[4 * t + 1]),
                          pack2(out[4 * t + 2], out[4 * t + 3]));
    return;
  }
  const int lane = threadIdx.x & 63;
  uint2 *const ws = stage + (threadIdx.x >> 6) * 192;  // this wave's 1536 bytes
#pragma unroll
  for (int t = 0; t < 3; ++t)
    ws[3 * lane + t] = make_uint2(pack2(out[4 * t], out[4 * t + 1]), pack2(out[4 * t + 2], out[4 * t + 3]));
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  // the wave's run starts at y + q0 * 3 uint2 (q0 % 64 == 0: 16-byte aligned when y is)
  uint4 *const dst = reinterpret_cast<uint4 *>(y + static_cast<long>(q0) * 3);
  const uint4 *const src = reinterpret_cast<const uint4 *>(ws);
  dst[lane] = src[lane];
  if (lane < 32) dst[64 + lane] = src[64 + lane];
}

// x: NHWC bf16 [N][H][Wp][Cp] -> y: NCHW fp32 [N][C][H][W]
__global__ void nhwc_bf16_to_nchw_f32(const bf16_t *__restrict__ x, float *__restrict__ y, int N, int C, int H,
                                      int W, int Cp, int Wp) {
  const long total = static_cast<long>(N) * C * H * W;
  for (long i = grid_stride_start(); i < total; i += grid_stride()) {
    const long w = i % W;
    long t = i / W;
    const long h = t % H;
    t /= H;
    const long c = t % C;
    const long n = t / C;
    y[i] = bf2f(x[((n * H + h) * Wp + w) * Cp + c]);
  }
}

// Batched 2-D transpose x[b][R][Cc] -> y[b][Cc][R] (bf16), tiled through LDS.
// Flatten of an NHWC activation into the reference's NCHW feature order is
// transpose(R=HW, Cc=C); its gradient is transpose(R=C, Cc=HW).
__global__ void batched_transpose(const bf16_t *__restrict__ x, bf16_t *__restrict__ y, int R, int Cc) {
  __shared__ bf16_t tile[32][34];
  const long base = static_cast<long>(blockIdx.z) * R * Cc;
  const int r0 = blockIdx.x * 32, c0 = blockIdx.y * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 256 threads: 32 x 8
  for (int r = ty; r < 32; r += 8)
    if (r0 + r < R && c0 + tx < Cc) tile[r][tx] = x[base + static_cast<long>(r0 + r) * Cc + c0 + tx];
  __syncthreads();
  for (int c = ty; c < 32; c += 8)
    if (c0 + c < Cc && r0 + tx < R) y[base + static_cast<long>(c0 + c) * R + r0 + tx] = tile[tx][c];
}

// Small per-item matrices (AlexNet's flatten: 36 x 256 and back): one block per item stages the
// whole matrix in LDS with 8-byte loads (rows padded by 2 elements: the transposed reads of 32
// consecutive rows fall on 32 different banks) and writes the transpose as 4-byte pairs of
// consecutive output elements.  The 32 x 32 tiled form moved 2-byte elements in 4096 blocks
// (7.8 us for 4.7 MB at batch 256).
__global__ void __launch_bounds__(256) batched_transpose_item(const bf16_t *__restrict__ x, bf16_t *__restrict__ y,
                                                                int R, int Cc) {
  extern __shared__ __attribute__((aligned(16))) uint16_t tl[];
  const int ld = Cc + 2;
  const long base = static_cast<long>(blockIdx.x) * R * Cc;
  const uint2 *xs = reinterpret_cast<const uint2 *>(x + base);
  const int nq = R * Cc / 4;
  for (int i = threadIdx.x; i < nq; i += blockDim.x) {
    const uint2 v = xs[i];
    const int e = 4 * i, r = e / Cc, c = e - r * Cc;
    uint32_t *d = reinterpret_cast<uint32_t *>(tl + r * ld + c);  // 4-byte aligned: ld and c are even
    d[0] = v.x;
    d[1] = v.y;
  }
  __syncthreads();
  uint32_t *ys = reinterpret_cast<uint32_t *>(y + base);
  const int np = R * Cc / 2;
  for (int i = threadIdx.x; i < np; i += blockDim.x) {
    const int o = 2 * i, c = o / R, r = o - c * R;  // output (c, r) and (c', r') of o + 1
    const int o1 = o + 1, c1 = o1 / R, r1 = o1 - c1 * R;
    ys[i] = static_cast<uint32_t>(tl[r * ld + c]) | (static_cast<uint32_t>(tl[r1 * ld + c1]) << 16);
  }
}

// Conv weight transform for data-grad: W[g][co][kh][kw][ci] -> Wt[g][ci][KH-1-kh][KW-1-kw][co]
__global__ void conv_weight_flip(const bf16_t *__restrict__ w, bf16_t *__restrict__ wt, int G, int Co, int KH,
                                 int KW, int Ci) {
  const long total = static_cast<long>(G) * Co * KH * KW * Ci;
  for (long i = grid_stride_start(); i < total; i += grid_stride()) {
    long t = i;
    const int ci = t % Ci; t /= Ci;
    const int kw = t % KW; t /= KW;
    const int kh = t % KH; t /= KH;
    const int co = t % Co;
    const int g = t / Co;
    const long o = ((((static_cast<long>(g) * Ci + ci) * KH + (KH - 1 - kh)) * KW + (KW - 1 - kw)) * Co) + co;
    wt[o] = w[i];
  }
}

// Every conv layer's flipped weights of a backward pass in one launch (flat grid, blocks split over
// segments by size; 32-bit index math).  GoogLeNet flipped 56 weight tensors one launch each
// (≈5.7 us apiece, 64-bit divisions per element): 0.3 ms of a 6.8 ms step.
constexpr int FLIP_MAXSEG = 64;
struct FlipSeg {
  const bf16_t *w;
  bf16_t *wt;
  int Co, KH, KW, Ci, total;
};
struct FlipTable {
  FlipSeg s[FLIP_MAXSEG];
  int b0[FLIP_MAXSEG];
  int n;
};
// One block = one 64 x 64 (co, ci) tile of one (group, tap): read as 64 rows of contiguous ci,
// written as 64 rows of contiguous co through an LDS transpose.  (One element per thread with the
// output strided by Co ran at 0.6 TB/s -- 96 us per VGG-16 step.)
__global__ void conv_weight_flip_multi(FlipTable tab) {
  const int bx = blockIdx.x;
  int si = 0;
  for (int i = 1; i < tab.n; ++i)
    if (tab.b0[i] <= bx) si = i;
  const FlipSeg sg = tab.s[si];
  const int tco = (sg.Co + 63) / 64, tci = (sg.Ci + 63) / 64;
  int t = bx - tab.b0[si];
  const int ci0 = (t % tci) * 64; t /= tci;
  const int co0 = (t % tco) * 64; t /= tco;
  const int kw = t % sg.KW; t /= sg.KW;
  const int kh = t % sg.KH;
  const int g = t / sg.KH;
  __shared__ uint32_t tile[64][65];
  const int col = threadIdx.x & 63;
  const unsigned short *w = reinterpret_cast<const unsigned short *>(sg.w);
  unsigned short *wt = reinterpret_cast<unsigned short *>(sg.wt);
  if ((sg.Co & 7) == 0 && (sg.Ci & 7) == 0) {
    // 16-byte accesses: lane (r8, c8) moves 8 consecutive channels of one row (the 2-byte form
    // below issued 8x the memory instructions: AlexNet's 7.5 MB of conv weights took 12 us)
    unsigned short *tl = reinterpret_cast<unsigned short *>(tile);  // [64][130] bf16 (pitch 65 words)
    const int c8 = (threadIdx.x & 7) * 8, r8 = threadIdx.x >> 3;
    for (int r = r8; r < 64; r += NT / 8) {
      const int co = co0 + r, ci = ci0 + c8;
      if (co < sg.Co && ci < sg.Ci) {
        const uint4 v = *reinterpret_cast<const uint4 *>(w + (((g * sg.Co + co) * sg.KH + kh) * sg.KW + kw) * sg.Ci + ci);
        const unsigned short *e = reinterpret_cast<const unsigned short *>(&v);
#pragma unroll
        for (int k = 0; k < 8; ++k) tl[r * 130 + c8 + k] = e[k];
      }
    }
    __syncthreads();
    for (int r = r8; r < 64; r += NT / 8) {  // r = ci within the tile, c8 = first co
      const int ci = ci0 + r, co = co0 + c8;
      if (co < sg.Co && ci < sg.Ci) {
        uint4 v;
        unsigned short *e = reinterpret_cast<unsigned short *>(&v);
#pragma unroll
        for (int k = 0; k < 8; ++k) e[k] = tl[(c8 + k) * 130 + r];
        *reinterpret_cast<uint4 *>(wt + (((g * sg.Ci + ci) * sg.KH + (sg.KH - 1 - kh)) * sg.KW + (sg.KW - 1 - kw)) * sg.Co +
                                   co) = v;
      }
    }
    return;
  }
  for (int r = threadIdx.x >> 6; r < 64; r += NT / 64) {
    const int co = co0 + r, ci = ci0 + col;
    if (co < sg.Co && ci < sg.Ci) tile[r][col] = w[(((g * sg.Co + co) * sg.KH + kh) * sg.KW + kw) * sg.Ci + ci];
  }
  __syncthreads();
  for (int r = threadIdx.x >> 6; r < 64; r += NT / 64) {
    const int ci = ci0 + r, co = co0 + col;
    if (co < sg.Co && ci < sg.Ci)
      wt[(((g * sg.Ci + ci) * sg.KH + (sg.KH - 1 - kh)) * sg.KW + (sg.KW - 1 - kw)) * sg.Co + co] =
          static_cast<unsigned short>(tile[col][r]);
  }
}

// ------------------------------------------------------------------ pooling
// mode: 0 max, 1 sum, 2 avg.  relu bit 0: apply relu before max (relu_max_pooling);
// relu bit 1 (max mode, KH*KW < 128): set bit 7 of the recorded offset when the window
// maximum is <= 0, so the backward can apply relu' of the argmax element without
// re-reading the (large) input: relu'(x[argmax]) = (max > 0).
// Output size follows the reference ceil rule: min(Hp - k + s - 1, Hp - 1) / s + 1, Hp = H + 2 pad.
// Max mode records, per output, the window offset (kh*KW + kw, uint8) of the FIRST maximum.
template <int VEC>
__global__ void pool_fwd(const bf16_t *__restrict__ x, bf16_t *__restrict__ y, uint8_t *__restrict__ arg, int N,
                         int H, int W, int C, int Ho, int Wo, int KH, int KW, int S, int P, int mode, int relu) {
  const int CV = C / VEC;
  const long total = static_cast<long>(N) * Ho * Wo * CV;
  const float inv = 1.0f / (KH * KW);
  for (long idx = grid_stride_start(); idx < total; idx += grid_stride()) {
    const int cv = idx % CV;
    long t = idx / CV;
    const int wo = t % Wo; t /= Wo;
    const int ho = t % Ho;
    const int n = t / Ho;
    const int hs = ho * S - P, ws = wo * S - P;
    const int he = min(hs + KH, H), we = min(ws + KW, W);
    float acc[VEC];
    uint32_t am[VEC];
#pragma unroll
    for (int e = 0; e < VEC; ++e) {
      acc[e] = mode == 0 ? -INFINITY : 0.f;
      am[e] = 0;
    }
    for (int h = max(hs, 0); h < he; ++h)
      for (int w = max(ws, 0); w < we; ++w) {
        const bf16_t *p = x + ((static_cast<long>(n) * H + h) * W + w) * C + cv * VEC;
        const uint32_t off = static_cast<uint32_t>((h - hs) * KW + (w - ws));
        float v[VEC];
        if constexpr (VEC == 8) unpack8(*reinterpret_cast<const uint4 *>(p), v);
        else v[0] = bf2f(*p);
#pragma unroll
        for (int e = 0; e < VEC; ++e) {
          const float a = (relu & 1) ? fmaxf(v[e], 0.f) : v[e];
          if (mode == 0) {
            if (a > acc[e]) {
              acc[e] = a;
              am[e] = off;
            }
          } else {
            acc[e] += a;
          }
        }
      }
    if (mode == 2)
#pragma unroll
      for (int e = 0; e < VEC; ++e) acc[e] *= inv;
    if (mode == 0 && (relu & 2))
#pragma unroll
      for (int e = 0; e < VEC; ++e) am[e] |= acc[e] > 0.f ? 0u : 0x80u;
    if constexpr (VEC == 8) {
      *reinterpret_cast<uint4 *>(y + idx * VEC) = pack8(acc);
      if (arg)
        *reinterpret_cast<uint2 *>(arg + idx * VEC) =
            make_uint2(am[0] | am[1] << 8 | am[2] << 16 | am[3] << 24, am[4] | am[5] << 8 | am[6] << 16 | am[7] << 24);
    } else {
      y[idx] = f2bf(acc[0]);
      if (arg) arg[idx] = static_cast<uint8_t>(am[0]);
    }
  }
}

// Gather-form backward: each input element sums the gradients of the windows that contain
// it.  Max: the window's recorded first-maximum position receives the gradient (the
// reference compares values, src/layer/pooling_layer-inl.hpp:55-86, which with bf16
// activations would hand duplicates to rounding ties).  relu 1: multiply by relu'(x);
// relu 2 (max mode): relu' is encoded in the offsets (bit 7, see pool_fwd), x is not read.
// db (VEC 8 only, nullable): also db[c] += sum over pixels of dx[.][c] -- the bias
// gradient of the conv that produced x, folded in so that dx is never re-read.  The
// launch makes gridDim.x*NT a multiple of C/8, so each thread keeps one channel group.
template <int VEC>
__global__ void pool_bwd(const bf16_t *__restrict__ x, const uint8_t *__restrict__ arg, const bf16_t *__restrict__ dy,
                         bf16_t *__restrict__ dx, int N, int H, int W, int C, int Ho, int Wo, int KH, int KW, int S,
                         int P, int mode, int relu, float *__restrict__ db) {
  const int CV = C / VEC;
  const long total = static_cast<long>(N) * H * W * CV;
  const float inv = 1.0f / (KH * KW);
  float bsum[VEC];
#pragma unroll
  for (int e = 0; e < VEC; ++e) bsum[e] = 0.f;
  for (long idx = grid_stride_start(); idx < total; idx += grid_stride()) {
    const int cv = idx % CV;
    long t = idx / CV;
    const int w = t % W; t /= W;
    const int h = t % H;
    const int n = t / H;
    float xv[VEC], g[VEC];
    if (relu == 1) {
      if constexpr (VEC == 8) unpack8(*reinterpret_cast<const uint4 *>(x + idx * VEC), xv);
      else xv[0] = bf2f(x[idx]);
    }
#pragma unroll
    for (int e = 0; e < VEC; ++e) g[e] = 0.f;
    // windows ho with ho*S - P <= h < ho*S - P + KH
    const int hlo = max(0, (h + P - KH + S) / S), hhi = min(Ho - 1, (h + P) / S);
    const int wlo = max(0, (w + P - KW + S) / S), whi = min(Wo - 1, (w + P) / S);
    for (int ho = hlo; ho <= hhi; ++ho)
      for (int wo = wlo; wo <= whi; ++wo) {
        const long o = ((static_cast<long>(n) * Ho + ho) * Wo + wo) * C + cv * VEC;
        const uint32_t off = static_cast<uint32_t>((h - (ho * S - P)) * KW + (w - (wo * S - P)));
        float gv[VEC];
        uint32_t am[VEC];
        if constexpr (VEC == 8) {
          unpack8(*reinterpret_cast<const uint4 *>(dy + o), gv);
          if (mode == 0) {
            const uint2 a2 = *reinterpret_cast<const uint2 *>(arg + o);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              am[e] = (a2.x >> (8 * e)) & 0xff;
              am[e + 4] = (a2.y >> (8 * e)) & 0xff;
            }
          }
        } else {
          gv[0] = bf2f(dy[o]);
          if (mode == 0) am[0] = arg[o];
        }
#pragma unroll
        for (int e = 0; e < VEC; ++e) {
          if (mode == 0) g[e] += (am[e] == off) ? gv[e] : 0.f;
          else g[e] += mode == 2 ? gv[e] * inv : gv[e];
        }
      }
    if (relu == 1)
#pragma unroll
      for (int e = 0; e < VEC; ++e) g[e] = xv[e] > 0.f ? g[e] : 0.f;
    if constexpr (VEC == 8) {
      const uint4 packed = pack8(g);
      *reinterpret_cast<uint4 *>(dx + idx * VEC) = packed;
      if (db) {  // sum what was stored (bf16-rounded), like a separate pass would
        float r[8];
        unpack8(packed, r);
#pragma unroll
        for (int e = 0; e < 8; ++e) bsum[e] += r[e];
      }
    } else {
      dx[idx] = f2bf(g[0]);
    }
  }
  if constexpr (VEC == 8) {
    if (db) {
      extern __shared__ float red[];  // [C]
      for (int c = threadIdx.x; c < C; c += blockDim.x) red[c] = 0.f;
      __syncthreads();
      const int cv = static_cast<int>((static_cast<long>(blockIdx.x) * blockDim.x + threadIdx.x) % CV);
#pragma unroll
      for (int e = 0; e < 8; ++e) atomicAdd(&red[cv * 8 + e], bsum[e]);
      __syncthreads();
      // per-block partials (a second kernel sums them): thousands of blocks doing
      // atomics on the same C addresses serialise in L2
      for (int c = threadIdx.x; c < C; c += blockDim.x) db[static_cast<long>(blockIdx.x) * C + c] = red[c];
    }
  }
}

// db[c] += sum_b part[b][c].  Block = 32 columns x 8 row groups over one chunk of rows
// (blockIdx.y); one atomic per column per chunk (a few dozen per address).
__global__ void partials_reduce(const float *__restrict__ part, int nb, int C, float *__restrict__ db) {
  const int c = blockIdx.x * 32 + (threadIdx.x & 31);
  const int rg = threadIdx.x >> 5;
  const int per = (nb + gridDim.y - 1) / gridDim.y;
  const int b0 = blockIdx.y * per, b1 = min(nb, b0 + per);
  float s = 0.f;
  if (c < C) {
#pragma unroll 4
    for (int b = b0 + rg; b < b1; b += 8) s += part[static_cast<long>(b) * C + c];
  }
  __shared__ float red[8][33];
  red[rg][threadIdx.x & 31] = s;
  __syncthreads();
  if (rg == 0 && c < C) {
    float t = 0.f;
#pragma unroll
    for (int g = 0; g < 8; ++g) t += red[g][threadIdx.x & 31];
    atomicAdd(db + c, t);
  }
}
static inline dim3 partials_grid(int nb, int C) {
  // one row chunk (a single fixed-order pass, one add per column) in deterministic mode
  return dim3((C + 31) / 32, cxn_deterministic ? 1 : (nb + 63) / 64);
}

// One-element-per-thread forms of pool_fwd / pool_bwd for C % 8 == 0 and < 2^32
// elements: the index split is three 32-bit fast divisions (the grid-stride forms above
// spend most of their issue slots on 64-bit divisions).  Same semantics, including the
// relu' bit.
// SS / KS > 0: stride / square kernel fixed at compile time (3x3/2, 3x3/1, 2x2/2 -- every
// pooling of the model zoo): constant divisions and fully unrolled windows.
// NN (max mode, fixed window, relu & 4 and not relu & 1): the input is a relu output (>= 0), so
// bf16 bits order as unsigned integers and the first max is one v_max_u32 per element over keys
// (bits << 16 | 15 - tap; see pool_lrn_fwd) instead of unpack + compare + two selects.
__device__ __forceinline__ uint32_t nn_key_lo(uint32_t w, uint32_t t) { return ((w << 16) & 0x7fff0000u) | t; }
__device__ __forceinline__ uint32_t nn_key_hi(uint32_t w, uint32_t t) { return (w & 0x7fff0000u) | t; }
template <int SS, int KS, bool NN = false>
__global__ void pool_fwd_rows(const bf16_t *__restrict__ x, bf16_t *__restrict__ y, uint8_t *__restrict__ arg, int H,
                              int W, int C, int Ho, int Wo, int KHr, int KWr, int Sr, int P, int mode, int relu,
                              FastDiv fd_cv, FastDiv fd_row, FastDiv fd_h, uint32_t total) {
  const int S = SS > 0 ? SS : Sr, KH = KS > 0 ? KS : KHr, KW = KS > 0 ? KS : KWr;
  const int CV = C / 8;
  // XCD-aware: consecutive logical blocks (overlapping windows read the same input rows)
  // run on one XCD and share its L2 instead of re-fetching the overlap per XCD
  const uint32_t idx = xcd_remap(blockIdx.x, gridDim.x) * blockDim.x + threadIdx.x;
  if (idx >= total) return;
  const int row = static_cast<int>(fdiv(idx, fd_row));           // n * Ho + ho
  const int e = static_cast<int>(idx) - row * (Wo * CV);
  const int n = static_cast<int>(fdiv(static_cast<uint32_t>(row), fd_h)), ho = row - n * Ho;
  const int wo = static_cast<int>(fdiv(static_cast<uint32_t>(e), fd_cv));
  const int cv = e - wo * CV;
  const int hs = ho * S - P, ws = wo * S - P;
  const int he = min(hs + KH, H), we = min(ws + KW, W);
  float acc[8];
  uint32_t am[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    acc[q] = mode == 0 ? -INFINITY : 0.f;
    am[q] = 0;
  }
  const bf16_t *xb = x + static_cast<long>(n) * H * W * C + cv * 8;
  auto take = [&](const uint4 raw, uint32_t off) {
    float v[8];
    unpack8(raw, v);
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const float a = (relu & 1) ? fmaxf(v[q], 0.f) : v[q];
      if (mode == 0) {
        if (a > acc[q]) {
          acc[q] = a;
          am[q] = off;
        }
      } else {
        acc[q] += a;
      }
    }
  };
  if constexpr (KS > 0) {
    // fixed window: all KS*KS loads issued back to back (clamped addresses, edge taps
    // masked), then reduced in the same h-major order as the generic loop (first max wins)
    uint4 raw[KS * KS];
#pragma unroll
    for (int kh = 0; kh < KS; ++kh)
#pragma unroll
      for (int kw = 0; kw < KS; ++kw) {
        const int h = min(max(hs + kh, 0), H - 1), w = min(max(ws + kw, 0), W - 1);
        raw[kh * KS + kw] = *reinterpret_cast<const uint4 *>(xb + (static_cast<long>(h) * W + w) * C);
      }
    if constexpr (NN) {
      uint32_t best[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) best[q] = 0u;
#pragma unroll
      for (int kh = 0; kh < KS; ++kh)
#pragma unroll
        for (int kw = 0; kw < KS; ++kw)
          if (hs + kh >= 0 && hs + kh < he && ws + kw >= 0 && ws + kw < we) {
            const uint32_t t = 15u - static_cast<uint32_t>(kh * KS + kw);
            const uint4 r = raw[kh * KS + kw];
            const uint32_t wd[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              best[2 * q] = max(best[2 * q], nn_key_lo(wd[q], t));
              best[2 * q + 1] = max(best[2 * q + 1], nn_key_hi(wd[q], t));
            }
          }
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        acc[q] = __uint_as_float(best[q] & 0x7fff0000u);
        am[q] = 15u - (best[q] & 15u);
      }
    } else {
#pragma unroll
      for (int kh = 0; kh < KS; ++kh)
#pragma unroll
        for (int kw = 0; kw < KS; ++kw)
          if (hs + kh >= 0 && hs + kh < he && ws + kw >= 0 && ws + kw < we)
            take(raw[kh * KS + kw], static_cast<uint32_t>(kh * KW + kw));
    }
  } else {
    for (int h = max(hs, 0); h < he; ++h)
      for (int w = max(ws, 0); w < we; ++w)
        take(*reinterpret_cast<const uint4 *>(xb + (static_cast<long>(h) * W + w) * C),
             static_cast<uint32_t>((h - hs) * KW + (w - ws)));
  }
  if (mode == 2) {
    const float inv = 1.0f / (KH * KW);
#pragma unroll
    for (int q = 0; q < 8; ++q) acc[q] *= inv;
  }
  if (mode == 0 && (relu & 2))
#pragma unroll
    for (int q = 0; q < 8; ++q) am[q] |= acc[q] > 0.f ? 0u : 0x80u;
  const long o = (static_cast<long>(row) * Wo + wo) * C + cv * 8;
  *reinterpret_cast<uint4 *>(y + o) = pack8(acc);
  if (arg)
    *reinterpret_cast<uint2 *>(arg + o) =
        make_uint2(am[0] | am[1] << 8 | am[2] << 16 | am[3] << 24, am[4] | am[5] << 8 | am[6] << 16 | am[7] << 24);
}

template <int SS, int KS>
__global__ void pool_bwd_rows(const bf16_t *__restrict__ x, const uint8_t *__restrict__ arg,
                              const bf16_t *__restrict__ dy, bf16_t *__restrict__ dx, int H, int W, int C, int Ho,
                              int Wo, int KHr, int KWr, int Sr, int P, int mode, int relu, FastDiv fd_cv,
                              FastDiv fd_row, FastDiv fd_h, uint32_t total) {
  const int S = SS > 0 ? SS : Sr, KH = KS > 0 ? KS : KHr, KW = KS > 0 ? KS : KWr;
  const int CV = C / 8;
  const uint32_t gidx = xcd_remap(blockIdx.x, gridDim.x) * blockDim.x + threadIdx.x;  // as pool_fwd_rows
  if (gidx >= total) return;
  const int row = static_cast<int>(fdiv(gidx, fd_row));          // n * H + h
  const int e = static_cast<int>(gidx) - row * (W * CV);
  const int n = static_cast<int>(fdiv(static_cast<uint32_t>(row), fd_h)), h = row - n * H;
  const int w = static_cast<int>(fdiv(static_cast<uint32_t>(e), fd_cv));
  const int cv = e - w * CV;
  const long idx = (static_cast<long>(row) * W + w) * C + cv * 8;
  float xv[8], g[8];
  if (relu == 1) unpack8(*reinterpret_cast<const uint4 *>(x + idx), xv);
#pragma unroll
  for (int q = 0; q < 8; ++q) g[q] = 0.f;
  const int hlo = max(0, (h + P - KH + S) / S), hhi = min(Ho - 1, (h + P) / S);
  const int wlo = max(0, (w + P - KW + S) / S), whi = min(Wo - 1, (w + P) / S);
  const float inv = 1.0f / (KH * KW);
  const long nb = static_cast<long>(n) * Ho;
  auto take = [&](const uint4 d, const uint2 a2, int ho, int wo) {
    const uint32_t off = static_cast<uint32_t>((h - (ho * S - P)) * KW + (w - (wo * S - P)));
    float gv[8];
    unpack8(d, gv);
    if (mode == 0) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        g[q] += (((a2.x >> (8 * q)) & 0xff) == off) ? gv[q] : 0.f;
        g[q + 4] += (((a2.y >> (8 * q)) & 0xff) == off) ? gv[q + 4] : 0.f;
      }
    } else {
#pragma unroll
      for (int q = 0; q < 8; ++q) g[q] += mode == 2 ? gv[q] * inv : gv[q];
    }
  };
  if constexpr (KS > 0 && SS > 0) {
    // at most T x T windows cover one input pixel: issue every dy / argmax load first
    // (clamped, masked), then accumulate in the generic loop's order
    constexpr int T = (KS + SS - 1) / SS;
    uint4 d[T * T];
    uint2 a[T * T];
#pragma unroll
    for (int i = 0; i < T; ++i)
#pragma unroll
      for (int j = 0; j < T; ++j) {
        const long o = ((nb + min(hlo + i, Ho - 1)) * Wo + min(wlo + j, Wo - 1)) * C + cv * 8;
        d[i * T + j] = *reinterpret_cast<const uint4 *>(dy + o);
        if (mode == 0) a[i * T + j] = *reinterpret_cast<const uint2 *>(arg + o);
      }
#pragma unroll
    for (int i = 0; i < T; ++i)
#pragma unroll
      for (int j = 0; j < T; ++j)
        if (hlo + i <= hhi && wlo + j <= whi) take(d[i * T + j], a[i * T + j], hlo + i, wlo + j);
  } else {
    for (int ho = hlo; ho <= hhi; ++ho)
      for (int wo = wlo; wo <= whi; ++wo) {
        const long o = ((nb + ho) * Wo + wo) * C + cv * 8;
        take(*reinterpret_cast<const uint4 *>(dy + o),
             mode == 0 ? *reinterpret_cast<const uint2 *>(arg + o) : make_uint2(0u, 0u), ho, wo);
      }
  }
  if (relu == 1)
#pragma unroll
    for (int q = 0; q < 8; ++q) g[q] = xv[q] > 0.f ? g[q] : 0.f;
  *reinterpret_cast<uint4 *>(dx + idx) = pack8(g);
}

// Stride-1 3x3 max pooling (GoogLeNet's inception pool branches) on strips of R output rows per
// thread: each input row of the strip is read once as a 3-tap row maximum (value + kw), and every
// output row takes the row maxima of its three input rows -- (R + 2) * 3 loads per R outputs
// instead of 9 per output.  Same first-max order (kh, then kw) and relu flags as pool_fwd_rows.
// NN: integer keys as pool_fwd_rows (row key bits << 16 | 3 - kw; the output key adds 12 - 3 kh,
// giving bits << 16 | 15 - (3 kh + kw)).
template <int R, bool NN = false>
__global__ void pool_fwd_s1k3(const bf16_t *__restrict__ x, bf16_t *__restrict__ y, uint8_t *__restrict__ arg,
                              int H, int W, int C, int Ho, int Wo, int P, int relu, FastDiv fd_cv, FastDiv fd_row,
                              FastDiv fd_hs, uint32_t total) {
  const int CV = C / 8, HS = (Ho + R - 1) / R;
  const uint32_t idx = xcd_remap(blockIdx.x, gridDim.x) * blockDim.x + threadIdx.x;
  if (idx >= total) return;
  const int row = static_cast<int>(fdiv(idx, fd_row));  // n * HS + strip
  const int e = static_cast<int>(idx) - row * (Wo * CV);
  const int n = static_cast<int>(fdiv(static_cast<uint32_t>(row), fd_hs)), st = row - n * HS;
  const int wo = static_cast<int>(fdiv(static_cast<uint32_t>(e), fd_cv));
  const int cv = e - wo * CV;
  const int ho0 = st * R, h0 = ho0 - P, ws = wo - P;
  const bf16_t *xb = x + static_cast<long>(n) * H * W * C + cv * 8;
  float acc[R][8];
  uint32_t am[R][8];
#pragma unroll
  for (int o = 0; o < R; ++o)
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      acc[o][q] = -INFINITY;
      am[o][q] = 0;
    }
  if constexpr (NN) {
    uint32_t best[R][8];
#pragma unroll
    for (int o = 0; o < R; ++o)
#pragma unroll
      for (int q = 0; q < 8; ++q) best[o][q] = 0u;
#pragma unroll
    for (int r = 0; r < R + 2; ++r) {
      const int h = h0 + r;
      if (h < 0 || h >= H) continue;
      uint4 raw[3];
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
        const int w = min(max(ws + kw, 0), W - 1);
        raw[kw] = *reinterpret_cast<const uint4 *>(xb + (static_cast<long>(h) * W + w) * C);
      }
      uint32_t rk[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) rk[q] = 0u;
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
        if (ws + kw < 0 || ws + kw >= W) continue;
        const uint32_t t = 3u - static_cast<uint32_t>(kw);
        const uint32_t wd[4] = {raw[kw].x, raw[kw].y, raw[kw].z, raw[kw].w};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          rk[2 * q] = max(rk[2 * q], nn_key_lo(wd[q], t));
          rk[2 * q + 1] = max(rk[2 * q + 1], nn_key_hi(wd[q], t));
        }
      }
#pragma unroll
      for (int o = 0; o < R; ++o) {
        const int kh = r - o;
        if (kh < 0 || kh > 2) continue;
#pragma unroll
        for (int q = 0; q < 8; ++q)  // (every row has a valid tap: rk >= 1)
          best[o][q] = max(best[o][q], rk[q] + static_cast<uint32_t>(12 - 3 * kh));
      }
    }
#pragma unroll
    for (int o = 0; o < R; ++o)
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        acc[o][q] = __uint_as_float(best[o][q] & 0x7fff0000u);
        am[o][q] = 15u - (best[o][q] & 15u);
      }
  } else {
#pragma unroll
  for (int r = 0; r < R + 2; ++r) {
    const int h = h0 + r;
    if (h < 0 || h >= H) continue;
    uint4 raw[3];
#pragma unroll
    for (int kw = 0; kw < 3; ++kw) {
      const int w = min(max(ws + kw, 0), W - 1);
      raw[kw] = *reinterpret_cast<const uint4 *>(xb + (static_cast<long>(h) * W + w) * C);
    }
    float hm[8];
    uint32_t hk[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      hm[q] = -INFINITY;
      hk[q] = 0;
    }
#pragma unroll
    for (int kw = 0; kw < 3; ++kw) {
      if (ws + kw < 0 || ws + kw >= W) continue;
      float v[8];
      unpack8(raw[kw], v);
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const float a = (relu & 1) ? fmaxf(v[q], 0.f) : v[q];
        if (a > hm[q]) {
          hm[q] = a;
          hk[q] = kw;
        }
      }
    }
    // output rows o of the strip whose window holds input row r at kh = r - o
#pragma unroll
    for (int o = 0; o < R; ++o) {
      const int kh = r - o;
      if (kh < 0 || kh > 2) continue;
#pragma unroll
      for (int q = 0; q < 8; ++q)
        if (hm[q] > acc[o][q]) {
          acc[o][q] = hm[q];
          am[o][q] = static_cast<uint32_t>(kh * 3) + hk[q];
        }
    }
  }
  }
#pragma unroll
  for (int o = 0; o < R; ++o) {
    const int ho = ho0 + o;
    if (ho >= Ho) break;
    if (relu & 2)
#pragma unroll
      for (int q = 0; q < 8; ++q) am[o][q] |= acc[o][q] > 0.f ? 0u : 0x80u;
    const long off = ((static_cast<long>(n) * Ho + ho) * Wo + wo) * C + cv * 8;
    *reinterpret_cast<uint4 *>(y + off) = pack8(acc[o]);
    if (arg)
      *reinterpret_cast<uint2 *>(arg + off) =
          make_uint2(am[o][0] | am[o][1] << 8 | am[o][2] << 16 | am[o][3] << 24,
                     am[o][4] | am[o][5] << 8 | am[o][6] << 16 | am[o][7] << 24);
  }
}

// Backward of pool_fwd_s1k3 (max mode) on strips of R input rows: the (R + 2) x 3 windows that
// cover the strip are read once each (dy + recorded offset) and routed to the strip's rows;
// contributions arrive in (ho, wo) order as in pool_bwd_rows.  relu 1: times relu'(x); relu 2:
// relu' is in the offsets' bit 7 (a marked window matches no tap).
template <int R>
__global__ void pool_bwd_s1k3(const bf16_t *__restrict__ x, const uint8_t *__restrict__ arg,
                              const bf16_t *__restrict__ dy, bf16_t *__restrict__ dx, int H, int W, int C, int Ho,
                              int Wo, int P, int relu, FastDiv fd_cv, FastDiv fd_row, FastDiv fd_hs, uint32_t total) {
  const int CV = C / 8, HS = (H + R - 1) / R;
  const uint32_t idx = xcd_remap(blockIdx.x, gridDim.x) * blockDim.x + threadIdx.x;
  if (idx >= total) return;
  const int row = static_cast<int>(fdiv(idx, fd_row));  // n * HS + strip
  const int e = static_cast<int>(idx) - row * (W * CV);
  const int n = static_cast<int>(fdiv(static_cast<uint32_t>(row), fd_hs)), st = row - n * HS;
  const int w = static_cast<int>(fdiv(static_cast<uint32_t>(e), fd_cv));
  const int cv = e - w * CV;
  const int h0 = st * R;
  float g[R][8];
#pragma unroll
  for (int o = 0; o < R; ++o)
#pragma unroll
    for (int q = 0; q < 8; ++q) g[o][q] = 0.f;
  // window rows ho = h + P - kh for the strip's rows h0..h0+R-1: ho0 = h0 + P - 2 .. h0 + R - 1 + P
  const int hob = h0 + P - 2;
#pragma unroll
  for (int t = 0; t < R + 2; ++t) {
    const int ho = hob + t;
    if (ho < 0 || ho >= Ho) continue;
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const int wo = w + P - 2 + j;  // kw = w - (wo - P) = 2 - j
      if (wo < 0 || wo >= Wo) continue;
      const long o = ((static_cast<long>(n) * Ho + ho) * Wo + wo) * C + cv * 8;
      float gv[8];
      unpack8(*reinterpret_cast<const uint4 *>(dy + o), gv);
      const uint2 a2 = *reinterpret_cast<const uint2 *>(arg + o);
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const int kh = (h0 + r) - (ho - P);  // the input row's tap in window row ho
        if (kh < 0 || kh > 2) continue;
        const uint32_t off = static_cast<uint32_t>(kh * 3 + (2 - j));
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          g[r][q] += (((a2.x >> (8 * q)) & 0xff) == off) ? gv[q] : 0.f;
          g[r][q + 4] += (((a2.y >> (8 * q)) & 0xff) == off) ? gv[q + 4] : 0.f;
        }
      }
    }
  }
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int h = h0 + r;
    if (h >= H) break;
    const long idx8 = ((static_cast<long>(n) * H + h) * W + w) * C + cv * 8;
    if (relu == 1) {
      float xv[8];
      unpack8(*reinterpret_cast<const uint4 *>(x + idx8), xv);
#pragma unroll
      for (int q = 0; q < 8; ++q) g[r][q] = xv[q] > 0.f ? g[r][q] : 0.f;
    }
    *reinterpret_cast<uint4 *>(dx + idx8) = pack8(g[r]);
  }
}

// Backward of the 3x3 stride-2 max pool (AlexNet's pools) on 2x2 input cells.  In padded
// coordinates hp = h + P, window ho covers hp in [2ho, 2ho + 2], so input rows 2i and 2i + 1 are
// covered by window rows {i - 1, i} and {i}: the 4 windows (i-1..i) x (j-1..j) hold every
// contribution to the cell's 4 pixels.  pool_bwd_rows loads up to 4 windows per PIXEL (16 per
// cell, 9 distinct), all from L2; here each window is loaded once (4 per cell) and the cell's
// 4 outputs are written -- the kernel becomes write-bound.  Contributions are summed in
// (ho, wo) order as in pool_bwd_rows, so both give the same bits.  relu as pool_bwd_s1k3.
__global__ void pool_bwd_s2k3(const bf16_t *__restrict__ x, const uint8_t *__restrict__ arg,
                              const bf16_t *__restrict__ dy, bf16_t *__restrict__ dx, int H, int W, int C, int Ho,
                              int Wo, int P, int relu, int i0, int j0, int WC, FastDiv fd_cv, FastDiv fd_row,
                              FastDiv fd_hc, uint32_t total) {
  const int CV = C / 8;
  const uint32_t idx = xcd_remap(blockIdx.x, gridDim.x) * blockDim.x + threadIdx.x;
  if (idx >= total) return;
  const int row = static_cast<int>(fdiv(idx, fd_row));  // n * HC + cell row
  const int e = static_cast<int>(idx) - row * (WC * CV);
  const int n = static_cast<int>(fdiv(static_cast<uint32_t>(row), fd_hc));
  const int i = row - n * static_cast<int>(fd_hc.d) + i0;
  const int cj = static_cast<int>(fdiv(static_cast<uint32_t>(e), fd_cv));
  const int cv = e - cj * CV, j = cj + j0;
  uint4 d[2][2];
  uint2 a[2][2];
  bool ok[2][2];
#pragma unroll
  for (int p = 0; p < 2; ++p)
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int ho = i - 1 + p, wo = j - 1 + q;
      ok[p][q] = ho >= 0 && ho < Ho && wo >= 0 && wo < Wo;
      const long o = ((static_cast<long>(n) * Ho + min(max(ho, 0), Ho - 1)) * Wo + min(max(wo, 0), Wo - 1)) * C +
                     cv * 8;
      d[p][q] = *reinterpret_cast<const uint4 *>(dy + o);
      a[p][q] = *reinterpret_cast<const uint2 *>(arg + o);
    }
#pragma unroll
  for (int r = 0; r < 2; ++r)
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int h = 2 * i + r - P, w = 2 * j + s - P;
      if (h < 0 || h >= H || w < 0 || w >= W) continue;
      float g[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) g[k] = 0.f;
#pragma unroll
      for (int p = 0; p < 2; ++p)
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const int kh = 2 + r - 2 * p, kw = 2 + s - 2 * q;  // tap of (h, w) in window (i-1+p, j-1+q)
          if (kh > 2 || kw > 2 || !ok[p][q]) continue;
          const uint32_t off = static_cast<uint32_t>(kh * 3 + kw);
          float gv[8];
          unpack8(d[p][q], gv);
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            g[k] += (((a[p][q].x >> (8 * k)) & 0xff) == off) ? gv[k] : 0.f;
            g[k + 4] += (((a[p][q].y >> (8 * k)) & 0xff) == off) ? gv[k + 4] : 0.f;
          }
        }
      const long o = ((static_cast<long>(n) * H + h) * W + w) * C + cv * 8;
      if (relu == 1) {
        float xv[8];
        unpack8(*reinterpret_cast<const uint4 *>(x + o), xv);
#pragma unroll
        for (int k = 0; k < 8; ++k) g[k] = xv[k] > 0.f ? g[k] : 0.f;
      }
      *reinterpret_cast<uint4 *>(dx + o) = pack8(g);
    }
}

// ------------------------------------------------------------------ LRN
// The norm's powers: norm = k + alpha / n * sum(x^2) >= k > 0 (k = 1 in every shipped net), so the
// raw v_log_f32 / v_exp_f32 give exp2f / __log2f's values without their denormal-range fix-ups
// (a compare, a select and a scale per call: a third of the fused pool -> LRN backward's VALU).
__device__ __forceinline__ float lrn_log2(float x) { return __builtin_amdgcn_logf(x); }
__device__ __forceinline__ float lrn_exp2(float x) { return __builtin_amdgcn_exp2f(x); }
// norm[c] = knorm + alpha/n * sum_{c' in [c-h, c+h] clipped} x[c']^2 ; y = x * norm^-beta
// One thread per (pixel, 8 channels); halo of up to 8 channels each side via three 16-B loads.
__device__ __forceinline__ void load_window(const bf16_t *row, int C, int c0, float *buf /*[24]*/) {
  // buf[j] = x[c0 - 8 + j], zero outside [0, C)
#pragma unroll
  for (int b = 0; b < 3; ++b) {
    const int cs = c0 - 8 + 8 * b;
    float v[8];
    if (cs >= 0 && cs + 8 <= C) {
      unpack8(*reinterpret_cast<const uint4 *>(row + cs), v);
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = (cs + e >= 0 && cs + e < C) ? bf2f(row[cs + e]) : 0.f;
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) buf[8 * b + e] = v[e];
  }
}

__global__ void lrn_fwd(const bf16_t *__restrict__ x, bf16_t *__restrict__ y, long npix, int C, int half,
                        float salpha, float beta, float knorm) {
  const int CV = C / 8;
  const long total = npix * CV;
  for (long idx = grid_stride_start(); idx < total; idx += grid_stride()) {
    const long pix = idx / CV;
    const int c0 = (idx % CV) * 8;
    const bf16_t *row = x + pix * C;
    float xb[24];
    load_window(row, C, c0, xb);
    float out[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float s = 0.f;
      for (int d = -half; d <= half; ++d) {
        const float v = xb[8 + e + d];
        s += v * v;
      }
      const float norm = knorm + salpha * s;
      out[e] = xb[8 + e] * lrn_exp2(-beta * lrn_log2(norm));
    }
    *reinterpret_cast<uint4 *>(y + pix * C + c0) = pack8(out);
  }
}

// g_in[c] = g[c] norm[c]^-b - 2 b salpha x[c] sum_{c' in win(c)} g[c'] x[c'] norm[c']^(-b-1)
// (norm recomputed from x: no state tensor is stored)
// LDS-staged LRN backward: block = NT/(C/8) pixels, one thread per 8 channels.
// LDS per pixel: x, g and t = g*x*norm^(-b-1), each with `half` zero pads at both ends.
// mask_relu: the input is relu(z) of a fused producer -> also apply relu'(z) = (x > 0).
__global__ void lrn_bwd_lds(const bf16_t *x, const bf16_t *dy, bf16_t *dx, long npix, int C, int half, float salpha,
                            float beta, float knorm, int mask_relu) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int tpp = C / 8;
  const int ppb = blockDim.x / tpp;
  const int L = C + 2 * half;
  const int pl = threadIdx.x / tpp, cv = threadIdx.x % tpp;
  const long pix = static_cast<long>(blockIdx.x) * ppb + pl;
  const bool active = pl < ppb && pix < npix;
  float *xs = sm + pl * 3 * L;
  float *gs = xs + L;
  float *ts = gs + L;
  const int c0 = cv * 8;
  float xv[8], gv[8];
  if (active) {
    unpack8(*reinterpret_cast<const uint4 *>(x + pix * C + c0), xv);
    unpack8(*reinterpret_cast<const uint4 *>(dy + pix * C + c0), gv);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      xs[half + c0 + e] = xv[e];
      gs[half + c0 + e] = gv[e];
    }
    if (cv == 0)
      for (int h = 0; h < half; ++h) {
        xs[h] = 0.f; xs[half + C + h] = 0.f;
        ts[h] = 0.f; ts[half + C + h] = 0.f;
      }
  }
  __syncthreads();
  float ng[8];
  if (active) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int c = half + c0 + e;
      float s = 0.f;
      for (int d = -half; d <= half; ++d) {
        const float v = xs[c + d];
        s += v * v;
      }
      const float lg = lrn_log2(knorm + salpha * s);
      const float p = lrn_exp2(-beta * lg);         // norm^-b
      ng[e] = gv[e] * p;
      ts[c] = gv[e] * xv[e] * p * lrn_exp2(-lg);    // g x norm^(-b-1)
    }
  }
  __syncthreads();
  if (active) {
    float out[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int c = half + c0 + e;
      float s = 0.f;
      for (int d = -half; d <= half; ++d) s += ts[c + d];
      out[e] = ng[e] - 2.f * beta * salpha * xv[e] * s;
      if (mask_relu && !(xv[e] > 0.f)) out[e] = 0.f;
    }
    *reinterpret_cast<uint4 *>(dx + pix * C + c0) = pack8(out);
  }
}

// Register/shuffle forms: a wave holds floor(64/tpp) whole pixels, tpp = C/8 lanes
// each with 8 channels; the cross-channel window's halo (<= 4 channels per side)
// comes from the neighbouring lanes by ds_bpermute (__shfl), so there is no LDS
// staging and no bank conflicts.  Every lane of the wave executes the shuffles.
struct LrnLane {
  long pix;
  int cv, tpp;
  bool active;
};
__device__ __forceinline__ LrnLane lrn_lane(long npix, int C) {
  LrnLane r;
  r.tpp = C / 8;
  const int ppw = 64 / r.tpp;  // whole pixels per wave
  const int lane = threadIdx.x & 63;
  const long wave = (static_cast<long>(blockIdx.x) * blockDim.x + threadIdx.x) >> 6;
  const int pl = lane / r.tpp;
  r.cv = lane - pl * r.tpp;
  r.pix = wave * ppw + pl;
  r.active = pl < ppw && r.pix < npix;
  return r;
}
// window sum over channels c-h..c+h of v (8 per lane), halo from neighbours
template <int H>
__device__ __forceinline__ void lrn_window_sum(const float *v, const LrnLane &L, float *out) {
  const int lane = threadIdx.x & 63;
  float lo[4], hi[4];  // lo[j] = channel c0-1-j (left lane), hi[j] = channel c0+8+j (right lane)
#pragma unroll
  for (int j = 0; j < H; ++j) {
    const float l = __shfl(v[7 - j], lane - 1);
    const float r = __shfl(v[j], lane + 1);
    lo[j] = L.cv > 0 ? l : 0.f;
    hi[j] = L.cv < L.tpp - 1 ? r : 0.f;
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    float s = 0.f;
#pragma unroll
    for (int d = -H; d <= H; ++d) {
      const int q = e + d;
      s += q < 0 ? lo[-q - 1] : (q > 7 ? hi[q - 8] : v[q]);
    }
    out[e] = s;
  }
}

// grid-stride over (4 waves x whole pixels) groups, at most 4096 blocks: on GoogLeNet's norm2
// (12.8M lanes) 60.5 -> 56.5 us against one-shot blocks.  (The gather-heavy fused pool -> LRN
// forward measured the other way, 78.7 -> 81.8 us on AlexNet, and keeps one-shot blocks.)
template <int H>
__global__ void __launch_bounds__(NT)
lrn_fwd_shfl(const bf16_t *__restrict__ x, bf16_t *__restrict__ y, long npix, int C, float salpha, float beta,
             float knorm, long ngroups) {
  LrnLane L;
  L.tpp = C / 8;
  const int ppw = 64 / L.tpp;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int pl = lane / L.tpp;
  L.cv = lane - pl * L.tpp;
  for (long gi = blockIdx.x; gi < ngroups; gi += gridDim.x) {  // block-uniform: every lane shuffles
    L.pix = (gi * (NT / 64) + wave) * ppw + pl;
    L.active = pl < ppw && L.pix < npix;
    const long off = L.pix * C + L.cv * 8;
    float xv[8], sq[8], s[8];
    if (L.active) unpack8(*reinterpret_cast<const uint4 *>(x + off), xv);
    else
#pragma unroll
      for (int e = 0; e < 8; ++e) xv[e] = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) sq[e] = xv[e] * xv[e];
    lrn_window_sum<H>(sq, L, s);
    if (!L.active) continue;
    float out[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) out[e] = xv[e] * lrn_exp2(-beta * lrn_log2(knorm + salpha * s[e]));
    *reinterpret_cast<uint4 *>(y + off) = pack8(out);
  }
}

// dx may alias x (each lane reads its x/g before any write; the halo comes by shuffle).
template <int H>
__global__ void lrn_bwd_shfl(const bf16_t *x, const bf16_t *__restrict__ dy, bf16_t *dx, long npix, int C,
                             float salpha, float beta, float knorm, int mask_relu) {
  const LrnLane L = lrn_lane(npix, C);
  const long off = L.pix * C + L.cv * 8;
  float xv[8], gv[8], sq[8], s[8];
  if (L.active) {
    unpack8(*reinterpret_cast<const uint4 *>(x + off), xv);
    unpack8(*reinterpret_cast<const uint4 *>(dy + off), gv);
  } else {
#pragma unroll
    for (int e = 0; e < 8; ++e) xv[e] = gv[e] = 0.f;
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) sq[e] = xv[e] * xv[e];
  lrn_window_sum<H>(sq, L, s);
  float ng[8], t[8], ts[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const float lg = lrn_log2(knorm + salpha * s[e]);
    const float p = lrn_exp2(-beta * lg);  // norm^-b
    ng[e] = gv[e] * p;
    t[e] = gv[e] * xv[e] * p * lrn_exp2(-lg);  // g x norm^(-b-1)
  }
  lrn_window_sum<H>(t, L, ts);
  if (!L.active) return;
  float out[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    out[e] = ng[e] - 2.f * beta * salpha * xv[e] * ts[e];
    if (mask_relu && !(xv[e] > 0.f)) out[e] = 0.f;
  }
  *reinterpret_cast<uint4 *>(dx + off) = pack8(out);
}

// lrn_bwd_shfl plus the bias gradient of the conv in front (GoogLeNet conv2 -> relu -> norm2: the
// LRN's input gradient is that conv's output gradient): a grid-stride walk over the same
// (4 waves x whole pixels) groups, each lane summing the bf16 values it stores; the block's lanes
// meet in LDS in a fixed order and add one value per channel to db (not used in deterministic mode).
template <int H>
__global__ void __launch_bounds__(NT)
lrn_bwd_db(const bf16_t *x, const bf16_t *__restrict__ dy, bf16_t *dx, long npix, int C, float salpha, float beta,
           float knorm, int mask_relu, long ngroups, float *__restrict__ db, float *__restrict__ part) {
  __shared__ float red[NT * 8];
  LrnLane L;
  L.tpp = C / 8;
  const int ppw = 64 / L.tpp;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int pl = lane / L.tpp;
  L.cv = lane - pl * L.tpp;
  float bs[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) bs[e] = 0.f;
  for (long gi = blockIdx.x; gi < ngroups; gi += gridDim.x) {  // block-uniform: every lane shuffles
    L.pix = (gi * (NT / 64) + wave) * ppw + pl;
    L.active = pl < ppw && L.pix < npix;
    const long off = L.pix * C + L.cv * 8;
    float xv[8], gv[8], sq[8], sw[8];
    if (L.active) {
      unpack8(*reinterpret_cast<const uint4 *>(x + off), xv);
      unpack8(*reinterpret_cast<const uint4 *>(dy + off), gv);
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) xv[e] = gv[e] = 0.f;
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) sq[e] = xv[e] * xv[e];
    lrn_window_sum<H>(sq, L, sw);
    float ng[8], t[8], ts[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float lg = lrn_log2(knorm + salpha * sw[e]);
      const float pw = lrn_exp2(-beta * lg);
      ng[e] = gv[e] * pw;
      t[e] = gv[e] * xv[e] * pw * lrn_exp2(-lg);
    }
    lrn_window_sum<H>(t, L, ts);
    if (!L.active) continue;
    float out[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      out[e] = ng[e] - 2.f * beta * salpha * xv[e] * ts[e];
      if (mask_relu && !(xv[e] > 0.f)) out[e] = 0.f;
    }
    const uint4 pk = pack8(out);
    *reinterpret_cast<uint4 *>(dx + off) = pk;
    unpack8(pk, out);
#pragma unroll
    for (int e = 0; e < 8; ++e) bs[e] += out[e];
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) red[threadIdx.x * 8 + e] = bs[e];
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += NT) {
    const int cv = c >> 3, e = c & 7;
    float s = 0.f;
    for (int w = 0; w < NT / 64; ++w)
      for (int p = 0; p < ppw; ++p) s += red[(w * 64 + p * L.tpp + cv) * 8 + e];
    if (part != nullptr) part[static_cast<long>(blockIdx.x) * C + c] = s;  // summed by part_rows_colsum
    else atomicAdd(db + c, s);
  }
}

// ------------------------------------------------------------------ fused max-pool -> LRN
// AlexNet's pool1 -> lrn1 and pool2 -> lrn2 (reference pooling_layer-inl.hpp:45-86 and
// lrn_layer-inl.hpp:53-74) as one kernel per direction.  Lanes are laid out as the shuffle LRN
// (whole pooled pixels per wave, C / 8 lanes each), so the cross-channel window sums stay in
// registers.
//   forward : the 3x3 / 2 max window (first max, offset byte, relu' bit as pool_fwd_rows) ->
//             pooled P and the LRN output Y in one pass: P is written (the LRN backward reads it)
//             but not read back;
//   backward: a block owns a band of R cell rows (2x2 input cells, pool_bwd_s2k3's
//             formulation) of one image.  Phase 1 computes the LRN data-gradient of the band's
//             windows (plus the row above, recomputed) from (P, dY) into LDS, masked by relu'
//             (bit 7 of the offset) and rounded to bf16 as the separate layers store it; phase 2
//             routes it from LDS to each cell's four pixels: the pooled gradient never reaches
//             HBM.  With dbias the conv-bias gradient behind a relu'd pool (the _fuse_pool_bias
//             sum of the pooled gradient) is summed over the band's own windows; per-block
//             partial rows in a fixed order.
// NN: the input is known to be >= 0 (a relu output: relu fused into the producing conv).  Then
// bf16 bits order as unsigned integers, and the first max of a window is one v_max_u32 per
// element over keys (bits << 16 | 15 - tap) -- the larger key is the larger value, then the
// earlier tap -- instead of unpack + compare + two selects.  The sign bit is cleared first: a
// relu of -0 may have stored -0 (0x8000), which must rank as 0.
template <int H, bool NN>
__global__ void pool_lrn_fwd(const bf16_t *__restrict__ x, bf16_t *__restrict__ P, uint8_t *__restrict__ arg,
                             bf16_t *__restrict__ Y, int N, int Hin, int Win, int C, int Ho, int Wo, int relu,
                             float salpha, float beta, float knorm) {
  const long npix = static_cast<long>(N) * Ho * Wo;
  const LrnLane L = lrn_lane(npix, C);
  float pv[8];
  uint32_t am[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    pv[q] = 0.f;
    am[q] = 0;
  }
  long o = 0;
  if (L.active) {
    const int n = static_cast<int>(L.pix / (static_cast<long>(Ho) * Wo));
    const int rem = static_cast<int>(L.pix - static_cast<long>(n) * Ho * Wo);
    const int ho = rem / Wo, wo = rem - (rem / Wo) * Wo;
    const int hs = 2 * ho, ws = 2 * wo;
    const bf16_t *xb = x + static_cast<long>(n) * Hin * Win * C + L.cv * 8;
    uint4 raw[9];
#pragma unroll
    for (int kh = 0; kh < 3; ++kh)
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
        const int h = min(hs + kh, Hin - 1), w = min(ws + kw, Win - 1);
        raw[kh * 3 + kw] = *reinterpret_cast<const uint4 *>(xb + (static_cast<long>(h) * Win + w) * C);
      }
    if constexpr (NN) {
      uint32_t best[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) best[q] = 0u;  // below every real key (>= 7)
#pragma unroll
      for (int kh = 0; kh < 3; ++kh)
#pragma unroll
        for (int kw = 0; kw < 3; ++kw) {
          if (hs + kh >= Hin || ws + kw >= Win) continue;
          const uint32_t t = 15u - static_cast<uint32_t>(kh * 3 + kw);
          const uint4 r = raw[kh * 3 + kw];
          const uint32_t wd[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            best[2 * q] = max(best[2 * q], ((wd[q] << 16) & 0x7fff0000u) | t);
            best[2 * q + 1] = max(best[2 * q + 1], (wd[q] & 0x7fff0000u) | t);
          }
        }
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        pv[q] = __uint_as_float(best[q] & 0x7fff0000u);
        am[q] = 15u - (best[q] & 15u);
      }
    } else {
#pragma unroll
      for (int q = 0; q < 8; ++q) pv[q] = -INFINITY;
#pragma unroll
      for (int kh = 0; kh < 3; ++kh)
#pragma unroll
        for (int kw = 0; kw < 3; ++kw) {
          if (hs + kh >= Hin || ws + kw >= Win) continue;
          float v[8];
          unpack8(raw[kh * 3 + kw], v);
#pragma unroll
          for (int q = 0; q < 8; ++q) {
            const float a = (relu & 1) ? fmaxf(v[q], 0.f) : v[q];
            if (a > pv[q]) {
              pv[q] = a;
              am[q] = static_cast<uint32_t>(kh * 3 + kw);
            }
          }
        }
    }
    if (relu & 2)
#pragma unroll
      for (int q = 0; q < 8; ++q) am[q] |= pv[q] > 0.f ? 0u : 0x80u;
    o = L.pix * C + L.cv * 8;
    const uint4 pk = pack8(pv);
    *reinterpret_cast<uint4 *>(P + o) = pk;
    *reinterpret_cast<uint2 *>(arg + o) =
        make_uint2(am[0] | am[1] << 8 | am[2] << 16 | am[3] << 24, am[4] | am[5] << 8 | am[6] << 16 | am[7] << 24);
    unpack8(pk, pv);  // the LRN reads the stored (bf16) P, as the separate kernel would
  }
  float sq[8], sw[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) sq[e] = pv[e] * pv[e];
  lrn_window_sum<H>(sq, L, sw);
  if (!L.active) return;
  float out[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) out[e] = pv[e] * lrn_exp2(-beta * lrn_log2(knorm + salpha * sw[e]));
  *reinterpret_cast<uint4 *>(Y + o) = pack8(out);
}

template <int H>
__global__ void __launch_bounds__(NT)
lrn_pool_bwd(const bf16_t *__restrict__ P, const bf16_t *__restrict__ dY, const uint8_t *__restrict__ arg,
             bf16_t *__restrict__ dx, int Hin, int Win, int C, int Ho, int Wo, int HC, int WC, int R, int nband,
             int relu_bit, float salpha, float beta, float knorm, float *__restrict__ dbias_part) {
  extern __shared__ __attribute__((aligned(16))) char plds[];
  const int tpp = C / 8, ppw = 64 / tpp;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int pl = lane / tpp, cv = lane - pl * tpp;
  const bool lane_ok = pl < ppw;
  LrnLane L;  // lrn_window_sum's view: channel block cv of a pixel of tpp lanes
  L.tpp = tpp;
  L.cv = cv;
  L.pix = 0;
  L.active = lane_ok;
  const int n = blockIdx.x / nband, band = blockIdx.x - n * nband;
  const int c0 = band * R;                                            // first cell row
  const int h_lo = max(c0 - 1, 0), h_hi = min(c0 + R - 1, Ho - 1);    // window rows it reads
  const int nwin = (h_hi - h_lo + 1) * Wo;
  bf16_t *const gl = reinterpret_cast<bf16_t *>(plds);                          // [window][C] gradient
  uint8_t *const al = reinterpret_cast<uint8_t *>(plds + static_cast<size_t>(R + 1) * Wo * C * 2);  // offsets
  const int step = (NT / 64) * ppw;
  // per-image bases (64-bit once); offsets inside one image fit 32 bits (checked by the launcher)
  const long pimg = static_cast<long>(n) * Ho * Wo * C;
  const bf16_t *const Pn = P + pimg;
  const bf16_t *const dYn = dY + pimg;
  const uint8_t *const an = arg + pimg;
  bf16_t *const dxn = dx + static_cast<long>(n) * Hin * Win * C;
  float bsum[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) bsum[k] = 0.f;
  // phase 1: the LRN data-gradient of every window of the band (and of the row above it), masked
  // by relu', rounded to bf16 as the separate layers store it, into LDS with the offsets
  // (window row, column) of this lane's window, advanced by `step` windows per pass (no divides)
  int wr = (wave * ppw + pl) / Wo, wc = (wave * ppw + pl) - wr * Wo;
  for (int base = 0; base < nwin; base += step) {
    const int wi = base + wave * ppw + pl;
    const bool ok = lane_ok && wi < nwin;
    const int ho = h_lo + wr, wo = wc;
    wc += step;
    while (wc >= Wo) {
      wc -= Wo;
      ++wr;
    }
    float xv[8], gv[8];
    uint2 a = make_uint2(0u, 0u);
    if (ok) {
      const int o = (ho * Wo + wo) * C + cv * 8;
      unpack8(*reinterpret_cast<const uint4 *>(Pn + o), xv);
      unpack8(*reinterpret_cast<const uint4 *>(dYn + o), gv);
      a = *reinterpret_cast<const uint2 *>(an + o);
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) xv[e] = gv[e] = 0.f;
    }
    float sq[8], sw[8], t[8], ts[8], ng[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) sq[e] = xv[e] * xv[e];
    lrn_window_sum<H>(sq, L, sw);
#pragma unroll
    for (int e = 0; e < 8; ++e) {  // as lrn_bwd_shfl
      const float lg = lrn_log2(knorm + salpha * sw[e]);
      const float pw = lrn_exp2(-beta * lg);
      ng[e] = gv[e] * pw;
      t[e] = gv[e] * xv[e] * pw * lrn_exp2(-lg);
    }
    lrn_window_sum<H>(t, L, ts);
    if (!ok) continue;
    float gp[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) gp[e] = ng[e] - 2.f * beta * salpha * xv[e] * ts[e];
    unpack8(pack8(gp), gp);
    const uint32_t ab[8] = {a.x & 0xff, (a.x >> 8) & 0xff, (a.x >> 16) & 0xff, a.x >> 24,
                            a.y & 0xff, (a.y >> 8) & 0xff, (a.y >> 16) & 0xff, a.y >> 24};
#pragma unroll
    for (int e = 0; e < 8; ++e) gp[e] = (relu_bit && (ab[e] & 0x80u)) ? 0.f : gp[e];
    if (ho >= c0)  // rows c0.. are this band's own windows (row c0 - 1 belongs to the band above)
#pragma unroll
      for (int e = 0; e < 8; ++e) bsum[e] += gp[e];
    *reinterpret_cast<uint4 *>(gl + static_cast<long>(wi) * C + cv * 8) = pack8(gp);
    *reinterpret_cast<uint2 *>(al + static_cast<long>(wi) * C + cv * 8) =
        make_uint2(a.x & 0x7f7f7f7fu, a.y & 0x7f7f7f7fu);
  }
  __syncthreads();
  // phase 2: per 2x2 input cell the four windows that cover it (pool_bwd_s2k3's formulation)
  const int ncell = (min(c0 + R, HC) - c0) * WC;
  int cr = (wave * ppw + pl) / WC, cc = (wave * ppw + pl) - cr * WC;
  for (int base = 0; base < ncell; base += step) {
    const int ce = base + wave * ppw + pl;
    const int ci = c0 + cr, cj = cc;
    cc += step;
    while (cc >= WC) {
      cc -= WC;
      ++cr;
    }
    if (!lane_ok || ce >= ncell) continue;
    uint4 g[4];
    uint2 a[4];
    bool okw[4];
#pragma unroll
    for (int pq = 0; pq < 4; ++pq) {
      const int ho = ci - 1 + (pq >> 1), wo = cj - 1 + (pq & 1);
      okw[pq] = ho >= 0 && ho < Ho && wo >= 0 && wo < Wo;
      const int wi = okw[pq] ? (ho - h_lo) * Wo + wo : 0;
      g[pq] = *reinterpret_cast<const uint4 *>(gl + static_cast<long>(wi) * C + cv * 8);
      a[pq] = *reinterpret_cast<const uint2 *>(al + static_cast<long>(wi) * C + cv * 8);
    }
#pragma unroll
    for (int rr = 0; rr < 2; ++rr)
#pragma unroll
      for (int sx = 0; sx < 2; ++sx) {
        const int h = 2 * ci + rr, w = 2 * cj + sx;
        if (h >= Hin || w >= Win) continue;
        float out[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) out[k] = 0.f;
#pragma unroll
        for (int pq = 0; pq < 4; ++pq) {
          const int kh = 2 + rr - 2 * (pq >> 1), kw = 2 + sx - 2 * (pq & 1);  // tap of (h, w) in the window
          if (kh > 2 || kw > 2 || !okw[pq]) continue;
          const uint32_t off = static_cast<uint32_t>(kh * 3 + kw);
          float gv[8];
          unpack8(g[pq], gv);
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            out[k] += ((a[pq].x >> (8 * k)) & 0xff) == off ? gv[k] : 0.f;
            out[k + 4] += ((a[pq].y >> (8 * k)) & 0xff) == off ? gv[k + 4] : 0.f;
          }
        }
        *reinterpret_cast<uint4 *>(dxn + (h * Win + w) * C + cv * 8) = pack8(out);
      }
  }
  if (dbias_part != nullptr) {  // the block's column sums in a fixed order (wave, pixel): no atomics
    // (in the window buffer, done with after phase 2: no extra LDS, so no lower occupancy)
    __syncthreads();
    float(*red)[64][9] = reinterpret_cast<float(*)[64][9]>(plds);
#pragma unroll
    for (int k = 0; k < 8; ++k) red[wave][lane][k] = lane_ok ? bsum[k] : 0.f;
    __syncthreads();
    for (int c = threadIdx.x; c < C; c += blockDim.x) {
      const int cc = c >> 3, k = c & 7;
      float acc = 0.f;
      for (int w = 0; w < NT / 64; ++w)
        for (int j = 0; j < ppw; ++j) acc += red[w][j * tpp + cc][k];
      dbias_part[static_cast<long>(blockIdx.x) * C + c] = acc;
    }
  }
}

// db[c] += sum_r part[r][c] over nrows fp32 partial rows of C columns: 32 columns x 8 row groups
// per block over a chunk of `chunk` rows (32: four dependent loads per thread, a few-us kernel
// instead of 11 us at 256), one atomic per column per chunk (one chunk: a fixed
// summation order, the deterministic mode)
__global__ void part_rows_colsum(const float *__restrict__ part, int nrows, int C, float *__restrict__ db, int chunk) {
  const int c = blockIdx.x * 32 + (threadIdx.x & 31);
  const int rg = threadIdx.x >> 5;
  const int r0 = blockIdx.y * chunk, r1 = min(nrows, r0 + chunk);
  float acc = 0.f;
  if (c < C)
    for (int r = r0 + rg; r < r1; r += 8) acc += part[static_cast<long>(r) * C + c];
  __shared__ float red[8][33];
  red[rg][threadIdx.x & 31] = acc;
  __syncthreads();
  if (rg == 0 && c < C) {
    float t = 0.f;
#pragma unroll
    for (int q = 0; q < 8; ++q) t += red[q][threadIdx.x & 31];
    atomicAdd(db + c, t);
  }
}

__global__ void lrn_bwd(const bf16_t *__restrict__ x, const bf16_t *__restrict__ dy, bf16_t *__restrict__ dx,
                        long npix, int C, int half, float salpha, float beta, float knorm, int mask_relu) {
  const int CV = C / 8;
  const long total = npix * CV;
  for (long idx = grid_stride_start(); idx < total; idx += grid_stride()) {
    const long pix = idx / CV;
    const int c0 = (idx % CV) * 8;
    float xb[24], gb[24];
    load_window(x + pix * C, C, c0, xb);
    load_window(dy + pix * C, C, c0, gb);
    // t[j] = g x norm^(-b-1) for channels c0-8+j, j in [8-half, 16+half)
    float normv[24], tv[24];
#pragma unroll
    for (int j = 0; j < 24; ++j) {
      normv[j] = 1.f;
      tv[j] = 0.f;
    }
    for (int j = 8 - half; j < 16 + half; ++j) {
      float s = 0.f;
      for (int d = -half; d <= half; ++d) {
        const int q = j + d;
        const float v = (q >= 0 && q < 24) ? xb[q] : 0.f;
        s += v * v;
      }
      const float norm = knorm + salpha * s;
      normv[j] = norm;
      tv[j] = gb[j] * xb[j] * lrn_exp2((-beta - 1.f) * lrn_log2(norm));
    }
    float out[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int j = 8 + e;
      float s = 0.f;
      for (int d = -half; d <= half; ++d) s += tv[j + d];
      out[e] = gb[j] * lrn_exp2(-beta * lrn_log2(normv[j])) - 2.f * beta * salpha * xb[j] * s;
      if (mask_relu && !(xb[j] > 0.f)) out[e] = 0.f;
    }
    *reinterpret_cast<uint4 *>(dx + pix * C + c0) = pack8(out);
  }
}

// ------------------------------------------------------------------ activations
// kind: 0 relu, 1 sigmoid, 2 tanh, 3 xelu(b).  Backward is written in terms of the
// forward OUTPUT y (the reference stores activations in place, src/layer/op.h:32-73).
__device__ __forceinline__ float act_f(int kind, float x, float b) {
  switch (kind) {
    case 0: return fmaxf(x, 0.f);
    case 1: return 1.f / (1.f + __expf(-x));
    case 2: return tanhf(x);
    default: return x > 0.f ? x : x / b;
  }
}
__device__ __forceinline__ float act_g(int kind, float y, float b) {
  switch (kind) {
    case 0: return y > 0.f ? 1.f : 0.f;
    case 1: return y * (1.f - y);
    case 2: return 1.f - y * y;
    default: return y > 0.f ? 1.f : 1.f / b;
  }
}

// y (and y2 when non-null, the reference's in-place write of the input node) = f(x)
__global__ void act_fwd(const bf16_t *__restrict__ x, bf16_t *y, bf16_t *y2, long n, int kind, float b) {
  const long n8 = n / 8;
  for (long i = grid_stride_start(); i < n8; i += grid_stride()) {
    float v[8];
    unpack8(reinterpret_cast<const uint4 *>(x)[i], v);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = act_f(kind, v[e], b);
    const uint4 o = pack8(v);
    reinterpret_cast<uint4 *>(y)[i] = o;
    if (y2) reinterpret_cast<uint4 *>(y2)[i] = o;
  }
  if (blockIdx.x == 0 && threadIdx.x < n - n8 * 8) {
    const long i = n8 * 8 + threadIdx.x;
    const bf16_t o = f2bf(act_f(kind, bf2f(x[i]), b));
    y[i] = o;
    if (y2) y2[i] = o;
  }
}
__global__ void act_bwd(const bf16_t *y, const bf16_t *dy, bf16_t *dx, long n, int kind, float b) {
  const long n8 = n / 8;
  for (long i = grid_stride_start(); i < n8; i += grid_stride()) {
    float yv[8], g[8];
    unpack8(reinterpret_cast<const uint4 *>(y)[i], yv);
    unpack8(reinterpret_cast<const uint4 *>(dy)[i], g);
#pragma unroll
    for (int e = 0; e < 8; ++e) g[e] *= act_g(kind, yv[e], b);
    reinterpret_cast<uint4 *>(dx)[i] = pack8(g);
  }
  if (blockIdx.x == 0 && threadIdx.x < n - n8 * 8) {
    const long i = n8 * 8 + threadIdx.x;
    dx[i] = f2bf(bf2f(dy[i]) * act_g(kind, bf2f(y[i]), b));
  }
}

// ------------------------------------------------------------------ dropout
// keep iff hash(seed, i) < pkeep * 2^32; x *= keep / pkeep.  The same call with the same
// seed in backward regenerates the mask, so no mask tensor is stored.
__device__ __forceinline__ uint32_t hash_u32(uint32_t x, uint32_t seed) {
  x ^= seed * 0x9E3779B9u;
  x ^= x >> 16; x *= 0x7FEB352Du;
  x ^= x >> 15; x *= 0x846CA68Bu;
  x ^= x >> 16;
  return x;
}
__global__ void dropout_apply(const bf16_t *x, bf16_t *y, long n, uint32_t seed0, const int *counter,
                              uint32_t thresh, float scale) {
  // counter (device, nullable) lets a captured HIP graph draw a fresh mask every replay
  const uint32_t seed = counter ? hash_u32(static_cast<uint32_t>(*counter), seed0) : seed0;
  const long n8 = n / 8;
  if (blockIdx.x == 0 && threadIdx.x < n - n8 * 8) {
    const long i = n8 * 8 + threadIdx.x;
    y[i] = f2bf(hash_u32(static_cast<uint32_t>(i), seed) < thresh ? bf2f(x[i]) * scale : 0.f);
  }
  for (long i = grid_stride_start(); i < n8; i += grid_stride()) {
    float v[8];
    unpack8(reinterpret_cast<const uint4 *>(x)[i], v);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const uint32_t h = hash_u32(static_cast<uint32_t>(i * 8 + e), seed);
      v[e] = h < thresh ? v[e] * scale : 0.f;
    }
    reinterpret_cast<uint4 *>(y)[i] = pack8(v);
  }
}

// ------------------------------------------------------------------ softmax / loss
// One wave per row.  p = softmax(x) written to y (bf16) and optionally pf (fp32).
__global__ void softmax_rows(const bf16_t *__restrict__ x, bf16_t *__restrict__ y, float *__restrict__ pf,
                             int rows, int K) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
  if (row >= rows) return;
  const bf16_t *xr = x + static_cast<long>(row) * K;
  float m = -INFINITY;
  for (int k = lane; k < K; k += 64) m = fmaxf(m, bf2f(xr[k]));
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
  float s = 0.f;
  for (int k = lane; k < K; k += 64) s += __expf(bf2f(xr[k]) - m);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  const float inv = 1.f / s;
  for (int k = lane; k < K; k += 64) {
    const float p = __expf(bf2f(xr[k]) - m) * inv;
    y[static_cast<long>(row) * K + k] = f2bf(p);
    if (pf) pf[static_cast<long>(row) * K + k] = p;
  }
}

// Rows of K <= 64 * NPL: one wave per row, one block per row (every CU gets rows), the row held in
// registers -- all of its loads issued before the first reduction instead of three dependent
// passes over memory (AlexNet fc8 output, 256 x 1000: 9.1 -> a few us).  Same arithmetic as
// softmax_rows: max, sum of exp(x - max), one reciprocal.
template <int NPL>
__global__ void __launch_bounds__(64) softmax_rows_reg(const bf16_t *__restrict__ x, bf16_t *__restrict__ y,
                                                       float *__restrict__ pf, int K) {
  const int lane = threadIdx.x;
  const long base = static_cast<long>(blockIdx.x) * K;
  float v[NPL];
#pragma unroll
  for (int j = 0; j < NPL; ++j) {
    const int k = lane + 64 * j;
    v[j] = k < K ? bf2f(x[base + k]) : -INFINITY;
  }
  float m = v[0];
#pragma unroll
  for (int j = 1; j < NPL; ++j) m = fmaxf(m, v[j]);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < NPL; ++j) {
    v[j] = lane + 64 * j < K ? __expf(v[j] - m) : 0.f;
    s += v[j];
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  const float inv = 1.f / s;
#pragma unroll
  for (int j = 0; j < NPL; ++j) {
    const int k = lane + 64 * j;
    if (k < K) {
      const float p = v[j] * inv;
      y[base + k] = f2bf(p);
      if (pf) pf[base + k] = p;
    }
  }
}

// grad = (p - onehot(label)) * scale, written in place over the bf16 node.  kind 0 softmax,
// 1 l2 (x - y), 2 multi-logistic (sigma - y, node already holds sigma).  label: fp32 [rows][lw]
__global__ void loss_grad(const float *__restrict__ p32, bf16_t *__restrict__ node, const float *__restrict__ label,
                          int rows, int K, int lw, float scale, int kind) {
  const long total = static_cast<long>(rows) * K;
  for (long i = grid_stride_start(); i < total; i += grid_stride()) {
    const int r = i / K, k = i % K;
    const float p = p32 ? p32[i] : bf2f(node[i]);
    float g;
    if (kind == 0) g = p - (static_cast<int>(label[static_cast<long>(r) * lw]) == k ? 1.f : 0.f);
    else g = p - label[static_cast<long>(r) * lw + k];
    node[i] = f2bf(g * scale);
  }
}

// ------------------------------------------------------------------ bias gradient
// db[c] += sum_r dy[r][c]  (dy bf16 [rows][C], C % 8 == 0).  Block = CB column-vectors x RG row
// groups; per-thread fp32 partials, LDS tree over RG, then one fp32 atomic per channel per block
// into db (one launch), or, in deterministic mode (db == nullptr), one partial row per block
// for the fixed-order partials_reduce.
__global__ void colsum_bf16(const bf16_t *__restrict__ dy, float *__restrict__ part, long rows, int C,
                            int rows_per_block, float *__restrict__ db) {
  const int CV = C / 8;
  const int CB = min(CV - static_cast<int>(blockIdx.y) * 64, 64);
  const int RG = NT / CB;
  const int t = threadIdx.x;
  const int cvl = t % CB, rg = t / CB;
  const int cv = blockIdx.y * 64 + cvl;
  const long r0 = static_cast<long>(blockIdx.x) * rows_per_block;
  const long r1 = min(rows, r0 + rows_per_block);
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (rg < RG) {
    constexpr int U = 4;  // independent 16-B loads in flight per thread
    for (long r = r0 + rg; r < r1; r += RG * U) {
      uint4 q[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const long rr = r + static_cast<long>(u) * RG;
        q[u] = rr < r1 ? *reinterpret_cast<const uint4 *>(dy + rr * C + cv * 8) : make_uint4(0, 0, 0, 0);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        float v[8];
        unpack8(q[u], v);
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[e] += v[e];
      }
    }
  }
  __shared__ float red[NT][9];
#pragma unroll
  for (int e = 0; e < 8; ++e) red[t][e] = (rg < RG) ? acc[e] : 0.f;
  __syncthreads();
  for (int q = t; q < CB * 8; q += NT) {
    const int c = q / 8, e = q % 8;
    float s = 0.f;
    for (int g = 0; g < RG; ++g) s += red[g * CB + c][e];
    if (db != nullptr)
      atomicAdd(db + (blockIdx.y * 64 + c) * 8 + e, s);
    else
      part[static_cast<long>(blockIdx.x) * C + (blockIdx.y * 64 + c) * 8 + e] = s;  // reduced by partials_reduce
  }
}

// Every deferred bias gradient of a backward pass in one launch (blockIdx.y = segment):
// db_s[c] += sum_r dy_s[r][c], C_s % 8 == 0, per-block partials -> one atomic per channel.
// A layer's backward only queues its (dy, db); NeuralNet.backprop flushes the queue once at
// the end (dy buffers are not rewritten later in the pass), which replaces one or two small
// launches per conv / fc layer -- GoogLeNet has 57 -- by one.
// A masked segment sums a max-pool's OUTPUT gradient instead of the conv's: every pool window
// routes its gradient to exactly one input pixel, and relu' of that pixel is bit 7 of the
// window's recorded offset (pool_fwd_rows, relu & 2), so sum_pixels dx = sum_windows dy * relu'
// -- the bias gradient of the conv in front of a max-pool at 1/stride^2 of the bytes read.
constexpr int COLSUM_MAXSEG = 64;
struct ColsumSeg {
  const bf16_t *dy;
  const uint8_t *mask;  // nullable: max-pool offsets [rows][C]; entries with bit 7 set count as 0
  float *db;
  long rows;
  long ld;  // dy row stride in elements (>= C: a channel slice of a wider NHWC buffer); mask rows are C
  int C, rpb, nblk, nchunk;
};
struct ColsumTable {
  ColsumSeg s[COLSUM_MAXSEG];
  int b0[COLSUM_MAXSEG];  // first block of each segment on the flat grid
  int n;
};
__global__ void colsum_multi(ColsumTable tab) {
  // flat grid, blocks split over segments by size (a 2-D grid of max-blocks x segments would
  // launch tens of thousands of idle blocks for GoogLeNet's 57 segments)
  const int bx = blockIdx.x;
  int si = 0;
  for (int i = 1; i < tab.n; ++i)
    if (tab.b0[i] <= bx) si = i;
  const ColsumSeg sg = tab.s[si];
  const int blk = bx - tab.b0[si];
  const int CV = sg.C / 8;
  const int t = threadIdx.x;
  // nchunk > 1: each block owns one chunk of 64 column vectors (wide fc segments would
  // otherwise leave one block walking all 4096 columns); 1: the block walks every chunk
  const int rb = blk / sg.nchunk, chunk = blk - rb * sg.nchunk;
  const int cbeg = sg.nchunk > 1 ? chunk * 64 : 0, cend = sg.nchunk > 1 ? min(CV, cbeg + 64) : CV;
  const long r0 = static_cast<long>(rb) * sg.rpb;
  const long r1 = min(sg.rows, r0 + sg.rpb);
  __shared__ float red[NT][9];
  for (int cb = cbeg; cb < cend; cb += 64) {
    const int CB = min(cend - cb, 64);
    const int RG = NT / CB;
    const int cvl = t % CB, rg = t / CB;
    const int cv = cb + cvl;
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (rg < RG) {
      // 8 rows in flight per thread; whole groups of 8 without bounds checks
      constexpr int U = 8;
      const long e0 = (r0 + rg) * sg.C + cv * 8;
      const bf16_t *p = sg.dy + (r0 + rg) * sg.ld + cv * 8;
      const long step = static_cast<long>(RG) * sg.ld;  // masked segments have ld == C
      long r = r0 + rg;
      if (sg.mask == nullptr) {
        for (; r + (U - 1) * RG < r1; r += RG * U, p += U * step) {
          uint4 q[U];
#pragma unroll
          for (int u = 0; u < U; ++u) q[u] = *reinterpret_cast<const uint4 *>(p + u * step);
#pragma unroll
          for (int u = 0; u < U; ++u) {
            float v[8];
            unpack8(q[u], v);
#pragma unroll
            for (int e = 0; e < 8; ++e) acc[e] += v[e];
          }
        }
        for (; r < r1; r += RG, p += step) {
          float v[8];
          unpack8(*reinterpret_cast<const uint4 *>(p), v);
#pragma unroll
          for (int e = 0; e < 8; ++e) acc[e] += v[e];
        }
      } else {
        const uint8_t *mp = sg.mask + e0;
        auto add = [&](const uint4 q, const uint2 m) {
          float v[8];
          unpack8(q, v);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            acc[e] += ((m.x >> (8 * e + 7)) & 1u) ? 0.f : v[e];
            acc[e + 4] += ((m.y >> (8 * e + 7)) & 1u) ? 0.f : v[e + 4];
          }
        };
        for (; r + (U - 1) * RG < r1; r += RG * U, p += U * step, mp += U * step) {
          uint4 q[U];
          uint2 m[U];
#pragma unroll
          for (int u = 0; u < U; ++u) {
            q[u] = *reinterpret_cast<const uint4 *>(p + u * step);
            m[u] = *reinterpret_cast<const uint2 *>(mp + u * step);
          }
#pragma unroll
          for (int u = 0; u < U; ++u) add(q[u], m[u]);
        }
        for (; r < r1; r += RG, p += step, mp += step)
          add(*reinterpret_cast<const uint4 *>(p), *reinterpret_cast<const uint2 *>(mp));
      }
    }
    __syncthreads();  // red is reused by the next column chunk
#pragma unroll
    for (int e = 0; e < 8; ++e) red[t][e] = (rg < RG) ? acc[e] : 0.f;
    __syncthreads();
    for (int q = t; q < CB * 8; q += NT) {
      const int c = q / 8, e = q % 8;
      float sum = 0.f;
      for (int gq = 0; gq < RG; ++gq) sum += red[gq * CB + c][e];
      atomicAdd(sg.db + (cb + c) * 8 + e, sum);
    }
  }
}

// Split-K finalisation: out[r][c] = epilogue(sum_s ws[s][r][c]) with optional bias[c],
// relu, and mask_relu (keep where the OLD out value is > 0).  8 columns per thread.
// out[i] += sum_s ws[s][i], slabs summed in slice order: the deterministic replacement for
// split-K fp32 atomics (conv weight-grad in deterministic mode).
__global__ void splitk_accumulate(const float *__restrict__ ws, int nsplit, long slab, float *__restrict__ out) {
  for (long i = (static_cast<long>(blockIdx.x) * blockDim.x + threadIdx.x) * 4; i < slab;
       i += static_cast<long>(gridDim.x) * blockDim.x * 4) {
    if (i + 4 <= slab) {
      f32x4 acc = *reinterpret_cast<const f32x4 *>(out + i);
      for (int s = 0; s < nsplit; ++s) acc += *reinterpret_cast<const f32x4 *>(ws + s * slab + i);
      *reinterpret_cast<f32x4 *>(out + i) = acc;
    } else {
      for (long e = i; e < slab; ++e) {
        float a = out[e];
        for (int s = 0; s < nsplit; ++s) a += ws[s * slab + e];
        out[e] = a;
      }
    }
  }
}

__device__ __forceinline__ uint32_t hash_u32(uint32_t x, uint32_t seed);
// DROP: the dropout layer behind a fused fc -> relu is applied here as well (keep iff
// hash(seed, flat index) < thresh, kept values * scale), with dropout_apply's mask
template <bool DROP>
__global__ void splitk_finalize(const float *__restrict__ ws, int nsplit, long slab, bf16_t *out, long rows,
                                int cols, const float *__restrict__ bias, int relu, int mask_relu, uint32_t seed0,
                                const int *counter, uint32_t thresh, float scale) {
  // grid: blockIdx.y = row, x over 8-column groups (no 64-bit division per element)
  {
    const long r = blockIdx.y;
    const int c0 = (blockIdx.x * blockDim.x + threadIdx.x) * 8;
    if (c0 >= cols) return;
    const float *p = ws + r * cols + c0;
    float f[8];
    {
      const float4 a = *reinterpret_cast<const float4 *>(p), b = *reinterpret_cast<const float4 *>(p + 4);
      f[0] = a.x; f[1] = a.y; f[2] = a.z; f[3] = a.w; f[4] = b.x; f[5] = b.y; f[6] = b.z; f[7] = b.w;
    }
    for (int sidx = 1; sidx < nsplit; ++sidx) {
      const float4 a = *reinterpret_cast<const float4 *>(p + sidx * slab);
      const float4 b = *reinterpret_cast<const float4 *>(p + sidx * slab + 4);
      f[0] += a.x; f[1] += a.y; f[2] += a.z; f[3] += a.w; f[4] += b.x; f[5] += b.y; f[6] += b.z; f[7] += b.w;
    }
    bf16_t *dst = out + r * cols + c0;
    float old[8];
    if (mask_relu) unpack8(*reinterpret_cast<const uint4 *>(dst), old);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      if (bias) f[e] += bias[c0 + e];
      if (relu) f[e] = fmaxf(f[e], 0.f);
      if (mask_relu && !(old[e] > 0.f)) f[e] = 0.f;
    }
    if constexpr (DROP) {
      const uint32_t seed = counter ? hash_u32(static_cast<uint32_t>(*counter), seed0) : seed0;
      const uint32_t i0 = static_cast<uint32_t>(r * cols + c0);
#pragma unroll
      for (int e = 0; e < 8; ++e) f[e] = hash_u32(i0 + e, seed) < thresh ? f[e] * scale : 0.f;
    }
    *reinterpret_cast<uint4 *>(dst) = pack8(f);
  }
}

// Small / ragged C: one thread per column.
__global__ void colsum_scalar(const bf16_t *__restrict__ dy, float *__restrict__ db, long rows, int C) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  float s = 0.f;
  for (long r = 0; r < rows; ++r) s += bf2f(dy[r * C + c]);
  db[c] += s;
}

// ------------------------------------------------------------------ elementwise helpers
__global__ void cast_f32_bf16(const float *__restrict__ x, bf16_t *__restrict__ y, long n) {
  for (long i = grid_stride_start(); i < n; i += grid_stride()) y[i] = f2bf(x[i]);
}
__global__ void add_bf16(const bf16_t *a, const bf16_t *b, bf16_t *y, long n) {
  const long n8 = n / 8;
  if (blockIdx.x == 0 && threadIdx.x < n - n8 * 8) {
    const long i = n8 * 8 + threadIdx.x;
    y[i] = f2bf(bf2f(a[i]) + bf2f(b[i]));
  }
  for (long i = grid_stride_start(); i < n8; i += grid_stride()) {
    float x[8], z[8];
    unpack8(reinterpret_cast<const uint4 *>(a)[i], x);
    unpack8(reinterpret_cast<const uint4 *>(b)[i], z);
#pragma unroll
    for (int e = 0; e < 8; ++e) x[e] += z[e];
    reinterpret_cast<uint4 *>(y)[i] = pack8(x);
  }
}
// split forward: one read of the source, up to 4 copies written (n8 16-byte vectors)
__global__ void fanout_bf16(const uint4 *__restrict__ src, uint4 *d0, uint4 *d1, uint4 *d2, uint4 *d3, int nd,
                            long n8) {
  for (long i = grid_stride_start(); i < n8; i += grid_stride()) {
    const uint4 v = src[i];
    d0[i] = v;
    if (nd > 1) d1[i] = v;
    if (nd > 2) d2[i] = v;
    if (nd > 3) d3[i] = v;
  }
}
// split backward: y = s0 + s1 (+ s2 + s3) in fp32, rounded once (y may alias s0)
// mask: y holds relu(z) on entry and the sum is kept only where y > 0 (relu') -- the backward
// of a split whose input is a zero-copy ch_concat of fused conv+relu branches
__global__ void sum_bf16(const uint4 *s0, const uint4 *s1, const uint4 *s2, const uint4 *s3, int ns, uint4 *y,
                         long n8, int mask) {
  for (long i = grid_stride_start(); i < n8; i += grid_stride()) {
    float a[8], b[8], z[8];
    if (mask) unpack8(y[i], z);
    unpack8(s0[i], a);
    unpack8(s1[i], b);
#pragma unroll
    for (int e = 0; e < 8; ++e) a[e] += b[e];
    if (ns > 2) {
      unpack8(s2[i], b);
#pragma unroll
      for (int e = 0; e < 8; ++e) a[e] += b[e];
    }
    if (ns > 3) {
      unpack8(s3[i], b);
#pragma unroll
      for (int e = 0; e < 8; ++e) a[e] += b[e];
    }
    if (mask) {
#pragma unroll
      for (int e = 0; e < 8; ++e) a[e] = z[e] > 0.f ? a[e] : 0.f;
    }
    y[i] = pack8(a);
  }
}

// strided channel copy for ch_concat / slicing: dst[p][doff + c] = src[p][soff + c], c < Cc
// mode 0: copy; 1: accumulate (dst += src); 2: relu'-masked copy (dst holds relu(z): keep
// src where dst > 0) -- the backward of a ch_concat whose input came from a fused conv+relu
__global__ void channel_copy(const bf16_t *__restrict__ src, int Cs, int soff, bf16_t *__restrict__ dst, int Cd,
                             int doff, int Cc, long npix, int mode) {
  const long total = npix * Cc;
  for (long i = grid_stride_start(); i < total; i += grid_stride()) {
    const long p = i / Cc;
    const int c = i % Cc;
    const float v = bf2f(src[p * Cs + soff + c]);
    bf16_t *d = dst + p * Cd + doff + c;
    const float o = bf2f(*d);
    *d = f2bf(mode == 1 ? o + v : (mode == 2 && !(o > 0.f)) ? 0.f : v);
  }
}

// 8-channel (16-byte) form of channel_copy when every stride/offset/count is a multiple of 8
// (all GoogLeNet concat branches): one uint4 per lane, 32-bit index math (total8 < 2^31).
__global__ void channel_copy8(const uint4 *__restrict__ src, int Cs8, int soff8, uint4 *__restrict__ dst, int Cd8,
                              int doff8, int Cc8, uint32_t total8, int mode) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < total8; i += gridDim.x * blockDim.x) {
    const uint32_t p = i / static_cast<uint32_t>(Cc8);
    const uint32_t c = i - p * static_cast<uint32_t>(Cc8);
    uint4 v = src[static_cast<size_t>(p) * Cs8 + soff8 + c];
    uint4 *d = dst + static_cast<size_t>(p) * Cd8 + doff8 + c;
    if (mode != 0) {
      float a[8], b[8];
      unpack8(v, a);
      unpack8(*d, b);
#pragma unroll
      for (int e = 0; e < 8; ++e) a[e] = mode == 1 ? a[e] + b[e] : (b[e] > 0.f ? a[e] : 0.f);
      v = pack8(a);
    }
    *d = v;
  }
}

// Channel concat of up to 4 NHWC inputs in ONE launch (every channel count a multiple of 8).
// Forward: out[p][off_k + c] = in_k[p][c].  Backward (bwd = 1): in_k[p][c] = out[p][off_k + c],
// masked by relu'(old in_k) for inputs produced by a fused conv+relu (mask bit k).
struct ConcatArgs {
  uint4 *in[4];
  int c8[4];    // channels / 8 per input
  int off8[4];  // channel offset / 8 in the output
};
__global__ void concat8(ConcatArgs a, int n, uint4 *__restrict__ out, int Ct8, uint32_t total8, int bwd, int mask) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < total8; i += gridDim.x * blockDim.x) {
    const uint32_t p = i / static_cast<uint32_t>(Ct8);
    const int c = static_cast<int>(i - p * static_cast<uint32_t>(Ct8));
    int k = 0;
#pragma unroll
    for (int q = 1; q < 4; ++q)
      if (q < n && c >= a.off8[q]) k = q;
    uint4 *src_in = a.in[k] + static_cast<size_t>(p) * a.c8[k] + (c - a.off8[k]);
    if (!bwd) {
      out[i] = *src_in;
    } else {
      uint4 v = out[i];
      if ((mask >> k) & 1) {
        float g[8], x[8];
        unpack8(v, g);
        unpack8(*src_in, x);
#pragma unroll
        for (int e = 0; e < 8; ++e) g[e] = x[e] > 0.f ? g[e] : 0.f;
        v = pack8(g);
      }
      *src_in = v;
    }
  }
}

// dst[r][0:L] = src[r][0:L], dst[r][L:Lp] = 0 (row-padded copy, e.g. conv1 weights for the
// row-gather GEMM: [Cout][KH][KW*C] -> [Cout][KH][roundup(KW*C, 8)])
__global__ void pad_rows(const bf16_t *__restrict__ src, bf16_t *__restrict__ dst, long rows, int L, int Lp) {
  const long total = rows * Lp;
  for (long i = grid_stride_start(); i < total; i += grid_stride()) {
    const long r = i / Lp;
    const int c = static_cast<int>(i - r * Lp);
    dst[i] = c < L ? src[r * L + c] : static_cast<bf16_t>(0);
  }
}


// Interior of a zero-bordered NHWC copy: dst[n][h + py][w + px][:] = src[n][h][w][:] in units of
// U bytes per pixel-chunk (the pre-pad conv path's input copy; the border stays as written once)
template <typename U>
__global__ void pad_interior(const U *__restrict__ src, U *__restrict__ dst, long npix, int H, int W, int H2, int W2,
                             int py, int px, int cu) {
  const long total = npix * cu;
  for (long i = grid_stride_start(); i < total; i += grid_stride()) {
    const long p = i / cu;
    const int c = static_cast<int>(i - p * cu);
    const long n = p / (static_cast<long>(H) * W);
    const int r = static_cast<int>(p - n * H * W);
    const int h = r / W, w = r - h * W;
    dst[((n * H2 + h + py) * W2 + w + px) * cu + c] = src[i];
  }
}


// dst[r][0:L] += src[r][0:L] (fp32; src rows of Ls >= L elements): the row-padded weight-grad
// buffer of the conv1 row-run path added into the layer's gradient
__global__ void add_rows_f32(const float *__restrict__ src, float *__restrict__ dst, long rows, int L, int Ls) {
  const long total = rows * L;
  for (long i = grid_stride_start(); i < total; i += grid_stride()) {
    const long r = i / L;
    dst[i] += src[r * Ls + (i - r * L)];
  }
}

// Max-unpool with the reference's tie semantics (src/layer/pooling_layer-inl.hpp:55-86,
// `unpool<red::maximum>`): EVERY input of a window that equals the window's max receives
// that window's gradient (pool_tie = all).  Gather form: one thread per input element sums
// over the windows covering it; y is the saved pooled output.  relu: the pooled values were
// max(relu(x)) and the gradient is masked by relu'(x).
__global__ void pool_bwd_tie_all(const bf16_t *__restrict__ x, const bf16_t *__restrict__ y,
                                 const bf16_t *__restrict__ dy, bf16_t *__restrict__ dx, int N, int H, int W, int C,
                                 int Ho, int Wo, int KH, int KW, int S, int P, int relu) {
  const long total = static_cast<long>(N) * H * W * C;
  for (long i = grid_stride_start(); i < total; i += grid_stride()) {
    const int c = static_cast<int>(i % C);
    const long pix = i / C;
    const int w = static_cast<int>(pix % W);
    const long nh = pix / W;
    const int h = static_cast<int>(nh % H);
    const int n = static_cast<int>(nh / H);
    float xv = bf2f(x[i]);
    if (relu) xv = fmaxf(xv, 0.f);
    // windows ho with ho*S - P <= h <= ho*S - P + KH - 1
    const int hp = h + P, wp = w + P;
    const int ho0 = hp - KH + 1 > 0 ? (hp - KH + 1 + S - 1) / S : 0, ho1 = min(Ho - 1, hp / S);
    const int wo0 = wp - KW + 1 > 0 ? (wp - KW + 1 + S - 1) / S : 0, wo1 = min(Wo - 1, wp / S);
    float g = 0.f;
    for (int ho = ho0; ho <= ho1; ++ho)
      for (int wo = wo0; wo <= wo1; ++wo) {
        const long o = ((static_cast<long>(n) * Ho + ho) * Wo + wo) * C + c;
        if (bf2f(y[o]) == xv) g += bf2f(dy[o]);
      }
    if (relu && !(bf2f(x[i]) > 0.f)) g = 0.f;
    dx[i] = f2bf(g);
  }
}

// ------------------------------------------------------------------ evaluation metrics
// Training / eval metrics on the device (reference src/utils/metric.h:20-236), one wave per
// instance row of fp32 scores p[B][K] against labels lab[B][lw]:
//   kind 0 error   : first-max argmax != label[0]   (K == 1: score > 0 is class 1)
//   kind 1 logloss : -log(clamp(p[label[0]], 1e-15, 1 - 1e-15))   (K == 1: binary form)
//   kind 2 rec@n   : (#distinct labels ranked within the top n) / lw, where a label's rank
//                    counts the scores that are larger, or equal at a lower index (the
//                    reference breaks exact ties at random; here the lowest index ranks first,
//                    so at most n labels can hit).
// Each block writes the sums over its rows to part[block][metric]; metric_accum adds the
// block partials, in block order, into a float64 accumulator (deterministic, no atomics).
struct MetricSpec {
  int nm;
  int kind[8];
  int arg[8];
};

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__global__ void __launch_bounds__(256) metric_rows(const float *__restrict__ p, int ldp, const float *__restrict__ lab,
                                                  int ldl, int lw, int B, int K, MetricSpec ms, float *__restrict__ part) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float acc[8];
#pragma unroll
  for (int m = 0; m < 8; ++m) acc[m] = 0.f;
  for (int r = blockIdx.x * 4 + wave; r < B; r += gridDim.x * 4) {
    const float *pr = p + static_cast<long>(r) * ldp;
    const float *lr = lab + static_cast<long>(r) * ldl;
    const int l0 = static_cast<int>(lr[0]);
    // first-max argmax
    float mv = -INFINITY;
    int mi = 0x7fffffff;
    for (int j = lane; j < K; j += 64) {
      const float v = pr[j];
      if (v > mv) { mv = v; mi = j; }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float ov = __shfl_xor(mv, o, 64);
      const int oi = __shfl_xor(mi, o, 64);
      if (ov > mv || (ov == mv && oi < mi)) { mv = ov; mi = oi; }
    }
    for (int m = 0; m < ms.nm; ++m) {
      float v = 0.f;
      if (ms.kind[m] == 0) {
        const int pred = K == 1 ? (pr[0] > 0.f ? 1 : 0) : mi;
        v = pred != l0 ? 1.f : 0.f;
      } else if (ms.kind[m] == 1) {
        if (K != 1) {
          const float q = fminf(fmaxf(pr[l0], 1e-15f), 1.f - 1e-15f);
          v = -logf(q);
        } else {
          const float py = fminf(fmaxf(pr[0], 1e-15f), 1.f - 1e-15f), y = lr[0];
          v = -(y * logf(py) + (1.f - y) * logf(1.f - py));
        }
      } else {
        const int n = ms.arg[m];
        int hits = 0;
        for (int c = 0; c < lw; ++c) {
          const int lc = static_cast<int>(lr[c]);
          bool dup = false;
          for (int d = 0; d < c; ++d) dup |= static_cast<int>(lr[d]) == lc;
          if (dup || lc < 0 || lc >= K) continue;
          const float sl = pr[lc];
          float cnt = 0.f;
          for (int j = lane; j < K; j += 64) cnt += (pr[j] > sl || (pr[j] == sl && j < lc)) ? 1.f : 0.f;
          cnt = wave_sum(cnt);
          hits += cnt < static_cast<float>(n) ? 1 : 0;
        }
        v = static_cast<float>(hits) / static_cast<float>(lw);
      }
      acc[m] += v;  // identical in every lane of the wave
    }
  }
  __shared__ float red[4][8];
  if (lane == 0)
#pragma unroll
    for (int m = 0; m < 8; ++m) red[wave][m] = acc[m];
  __syncthreads();
  if (threadIdx.x < ms.nm)
    part[blockIdx.x * ms.nm + threadIdx.x] =
        red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] + red[3][threadIdx.x];
}

__global__ void metric_accum(const float *__restrict__ part, int nb, int nm, double *__restrict__ acc) {
  const int m = threadIdx.x;
  if (m < nm) {
    double s = 0.0;
    for (int b = 0; b < nb; ++b) s += part[b * nm + m];
    acc[m] += s;
  }
}
}  // namespace

// ================================================================== C ABI
#define S_ static_cast<hipStream_t>(stream)
#define RET return hipGetLastError() == hipSuccess ? 0 : -3

// Wp: the node's physical row width (>= W; row-padded first-conv input, see image_u8c3_nhwc3p)
CXN_API int cxn_nchw_f32_to_nhwc_bf16(const float *x, void *y, int N, int C, int H, int W, int Cp, int Wp,
                                      float scale, void *stream) {
  if (Wp < W) return -2;
  CXN_LAUNCH((nchw_f32_to_nhwc_bf16), nblocks(static_cast<long>(N) * H * W), NT, 0, S_, x, (bf16_t *)y, N, C, H, W, Cp, Wp,
                                                                              scale);
  RET;
}
CXN_API int cxn_image_u8_to_nhwc_bf16(const void *pix, const int *prm, const float *cm, const float *mean, int B,
                                      int h, int w, int C, int Cp, int Wp, int Hm, int Wm, int mode, float scale,
                                      void *y, void *stream) {
  if (Cp < C || Wp < w || (mode != 0 && cm == nullptr) || (mode >= 1 && mean == nullptr) ||
      (mode == 2 && prm == nullptr))
    return -2;
  if (C > 8) return -2;
  const long npix = static_cast<long>(B) * h * w;
  const long nq = static_cast<long>(B) * h * (Wp / 4);
  if (C == 3 && Cp == 3 && mode <= 1 && Wp % 4 == 0 && reinterpret_cast<uintptr_t>(y) % 16 == 0 &&
      reinterpret_cast<uintptr_t>(pix) % 4 == 0 && npix * 3 >= 16 && nq < (1L << 31)) {
    CXN_LAUNCH((image_u8c3_nhwc3p), cdiv(nq, NT), NT, 0, S_, (const uint32_t *)pix, (npix * 3 + 3) / 4, cm, mean,
                                                    make_fastdiv(static_cast<uint32_t>(Wp / 4)),
                                                    make_fastdiv(static_cast<uint32_t>(h)), w, Wp, mode, scale,
                                                    static_cast<uint32_t>(nq), (uint2 *)y);
    RET;
  }
  if (C == 3 && Cp == 4 && Wp == w && mode <= 1 && npix % 4 == 0 && npix < (1L << 32) &&
      reinterpret_cast<uintptr_t>(pix) % 4 == 0) {
    CXN_LAUNCH((image_u8c3_nhwc4), nblocks(npix / 4), NT, 0, S_, (const uint32_t *)pix, cm, mean, npix / 4,
                                                        make_fastdiv(static_cast<uint32_t>(h * w)), mode, scale,
                                                        (uint4 *)y);
    RET;
  }
  dim3 grid(cdiv(w, NT), B * h);
  CXN_LAUNCH((image_u8_to_nhwc_bf16), grid, NT, 0, S_, (const uint8_t *)pix, prm, cm, mean, B, h, w, C, Cp, Wp, Hm, Wm, mode,
                                             scale, (bf16_t *)y);
  RET;
}
CXN_API int cxn_nhwc_bf16_to_nchw_f32(const void *x, float *y, int N, int C, int H, int W, int Cp, int Wp,
                                      void *stream) {
  CXN_LAUNCH((nhwc_bf16_to_nchw_f32), nblocks(static_cast<long>(N) * C * H * W), NT, 0, S_, (const bf16_t *)x, y, N, C, H, W, Cp,
                                                                                  Wp);
  RET;
}
CXN_API int cxn_transpose(const void *x, void *y, int B, int R, int Cc, void *stream) {
  const size_t lds = static_cast<size_t>(R) * (Cc + 2) * 2;
  if (Cc % 4 == 0 && R % 2 == 0 && lds <= 48 * 1024 && B >= 64 && reinterpret_cast<uintptr_t>(x) % 8 == 0 &&
      reinterpret_cast<uintptr_t>(y) % 4 == 0) {
    CXN_LAUNCH((batched_transpose_item), B, 256, lds, S_, (const bf16_t *)x, (bf16_t *)y, R, Cc);
    RET;
  }
  dim3 grid(cdiv(R, 32), cdiv(Cc, 32), B);
  CXN_LAUNCH((batched_transpose), grid, NT, 0, S_, (const bf16_t *)x, (bf16_t *)y, R, Cc);
  RET;
}
CXN_API int cxn_conv_weight_flip(const void *w, void *wt, int G, int Co, int KH, int KW, int Ci, void *stream) {
  CXN_LAUNCH((conv_weight_flip), nblocks(static_cast<long>(G) * Co * KH * KW * Ci), NT, 0, S_, (const bf16_t *)w, (bf16_t *)wt,
                                                                                     G, Co, KH, KW, Ci);
  RET;
}
// ws / wts: n weight tensors [G][Co][KH][KW][Ci] -> [G][Ci][KH'][KW'][Co] (taps reversed);
// dims: 5 ints per tensor (G, Co, KH, KW, Ci)
CXN_API int cxn_conv_weight_flip_multi(const void *const *ws, void *const *wts, const int *dims, int n, void *stream) {
  for (int base = 0; base < n; base += FLIP_MAXSEG) {
    FlipTable tab;
    const int cnt = n - base < FLIP_MAXSEG ? n - base : FLIP_MAXSEG;
    int nblk = 0;
    tab.n = cnt;
    for (int i = 0; i < cnt; ++i) {
      const int *d = dims + 5 * (base + i);
      const long total = static_cast<long>(d[0]) * d[1] * d[2] * d[3] * d[4];
      if (total >= (1L << 31)) return -2;
      tab.s[i] = FlipSeg{static_cast<const bf16_t *>(ws[base + i]), static_cast<bf16_t *>(wts[base + i]), d[1], d[2],
                         d[3], d[4], static_cast<int>(total)};
      tab.b0[i] = nblk;
      nblk += d[0] * d[2] * d[3] * cdiv(d[1], 64) * cdiv(d[4], 64);  // 64 x 64 (co, ci) tiles per (g, tap)
    }
    if (nblk) CXN_LAUNCH((conv_weight_flip_multi), nblk, NT, 0, S_, tab);
  }
  RET;
}
// stride-1 3x3 max pooling on row strips (pool_fwd_s1k3 / pool_bwd_s1k3); CXXNET_POOL_STRIPS=0 keeps
// the one-output-per-thread kernels (A/B)
static const int pool_strips = [] {
  const char *e = getenv("CXXNET_POOL_STRIPS");
  return (e && e[0] == '0') ? 0 : 1;
}();
// kernel variants kept for A/B (benchmarks/small_kernels.py): 0 pool_bwd_s2k3 cells,
// 1 colsum_multi column-chunk split
static int pool_cells = 1;
static int colsum_split = 1;
CXN_API int cxn_set_kernel_variant(int which, int v) {
  if (which == 0) pool_cells = v;
  else if (which == 1) colsum_split = v;
  else return -1;
  return 0;
}

CXN_API int cxn_pool_fwd(const void *x, void *y, void *arg, int N, int H, int W, int C, int Ho, int Wo, int KH, int KW, int S,
                         int P, int mode, int relu, void *stream) {
  if (C % 8 == 0) {
    const long total = static_cast<long>(N) * Ho * Wo * (C / 8);
    if (total >= (1L << 31)) return -2;  // fdiv (mulhi + n) stays exact below 2^31
    // relu & 4: the input is a relu output (>= 0): integer-key max (NN forms)
    const bool nn = mode == 0 && (relu & 4) != 0 && (relu & 1) == 0;
#define CXN_POOL_FWD_T(SSV, KSV, NNV)                                                                        \
  CXN_LAUNCH((pool_fwd_rows<SSV, KSV, NNV>), cdiv(total, NT), NT, 0, S_,                                     \
      (const bf16_t *)x, (bf16_t *)y, (uint8_t *)arg, H, W, C, Ho, Wo, KH, KW, S, P, mode, relu,             \
      make_fastdiv(static_cast<uint32_t>(C / 8)), make_fastdiv(static_cast<uint32_t>(Wo * (C / 8))),        \
      make_fastdiv(static_cast<uint32_t>(Ho)), static_cast<uint32_t>(total))
#define CXN_POOL_FWD(SSV, KSV)                   \
  do {                                           \
    if (nn) CXN_POOL_FWD_T(SSV, KSV, true);      \
    else CXN_POOL_FWD_T(SSV, KSV, false);        \
  } while (0)
    const int sq = KH == KW ? KH : 0;
    if (S == 1 && sq == 3 && mode == 0 && P <= 2 && pool_strips) {
      constexpr int R = 4;
      const int HS = (Ho + R - 1) / R;
      const long tot = static_cast<long>(N) * HS * Wo * (C / 8);
      if (nn)
        CXN_LAUNCH((pool_fwd_s1k3<R, true>), cdiv(tot, NT), NT, 0, S_, (const bf16_t *)x, (bf16_t *)y, (uint8_t *)arg,
                   H, W, C, Ho, Wo, P, relu, make_fastdiv(static_cast<uint32_t>(C / 8)),
                   make_fastdiv(static_cast<uint32_t>(Wo * (C / 8))), make_fastdiv(static_cast<uint32_t>(HS)),
                   static_cast<uint32_t>(tot));
      else
        CXN_LAUNCH((pool_fwd_s1k3<R, false>), cdiv(tot, NT), NT, 0, S_, (const bf16_t *)x, (bf16_t *)y, (uint8_t *)arg,
                   H, W, C, Ho, Wo, P, relu, make_fastdiv(static_cast<uint32_t>(C / 8)),
                   make_fastdiv(static_cast<uint32_t>(Wo * (C / 8))), make_fastdiv(static_cast<uint32_t>(HS)),
                   static_cast<uint32_t>(tot));
    } else if (S == 2 && sq == 3) CXN_POOL_FWD(2, 3);
    else if (S == 1 && sq == 3) CXN_POOL_FWD(1, 3);
    else if (S == 2 && sq == 2) CXN_POOL_FWD(2, 2);
    else CXN_POOL_FWD_T(0, 0, false);
#undef CXN_POOL_FWD
#undef CXN_POOL_FWD_T
  } else {
    CXN_LAUNCH((pool_fwd<1>), nblocks(static_cast<long>(N) * Ho * Wo * C), NT, 0, S_, 
        (const bf16_t *)x, (bf16_t *)y, (uint8_t *)arg, N, H, W, C, Ho, Wo, KH, KW, S, P, mode, relu);
  }
  RET;
}

CXN_API int cxn_pool_bwd_tie_all(const void *x, const void *y, const void *dy, void *dx, int N, int H, int W, int C,
                                 int Ho, int Wo, int KH, int KW, int S, int P, int relu, void *stream) {
  CXN_LAUNCH((pool_bwd_tie_all), nblocks(static_cast<long>(N) * H * W * C), NT, 0, S_, 
      (const bf16_t *)x, (const bf16_t *)y, (const bf16_t *)dy, (bf16_t *)dx, N, H, W, C, Ho, Wo, KH, KW, S, P, relu);
  RET;
}
CXN_API int cxn_pool_bwd(const void *x, const void *arg, const void *dy, void *dx, int N, int H, int W, int C, int Ho,
                         int Wo, int KH, int KW, int S, int P, int mode, int relu, float *db, float *ws,
                         long ws_elems, void *stream) {
  if (C % 8 == 0 && db == nullptr) {
    const long total = static_cast<long>(N) * H * W * (C / 8);
    if (total >= (1L << 31)) return -2;  // fdiv (mulhi + n) stays exact below 2^31
#define CXN_POOL_BWD(SSV, KSV)                                                                                  \
  CXN_LAUNCH((pool_bwd_rows<SSV, KSV>), cdiv(total, NT), NT, 0, S_,                                                       \
      (const bf16_t *)x, (const uint8_t *)arg, (const bf16_t *)dy, (bf16_t *)dx, H, W, C, Ho, Wo, KH, KW, S, P, mode, \
      relu, make_fastdiv(static_cast<uint32_t>(C / 8)), make_fastdiv(static_cast<uint32_t>(W * (C / 8))),          \
      make_fastdiv(static_cast<uint32_t>(H)), static_cast<uint32_t>(total))
    const int sq = KH == KW ? KH : 0;
    if (S == 1 && sq == 3 && mode == 0 && P <= 2 && pool_strips) {
      static const int r_env = [] {  // CXN_POOL_S1K3_R: probe override of the strip height (2 / 4 / 8)
        const char *e = getenv("CXN_POOL_S1K3_R");
        return e != nullptr ? atoi(e) : 4;
      }();
#define CXN_S1K3(RV)                                                                                           \
  {                                                                                                            \
    constexpr int R = RV;                                                                                      \
    const int HS = (H + R - 1) / R;                                                                            \
    const long tot = static_cast<long>(N) * HS * W * (C / 8);                                                  \
    CXN_LAUNCH((pool_bwd_s1k3<R>), cdiv(tot, NT), NT, 0, S_, (const bf16_t *)x, (const uint8_t *)arg,          \
               (const bf16_t *)dy, (bf16_t *)dx, H, W, C, Ho, Wo, P, relu,                                     \
               make_fastdiv(static_cast<uint32_t>(C / 8)), make_fastdiv(static_cast<uint32_t>(W * (C / 8))),   \
               make_fastdiv(static_cast<uint32_t>(HS)), static_cast<uint32_t>(tot));                          \
  }
      if (r_env == 2) CXN_S1K3(2)
      else if (r_env == 8) CXN_S1K3(8)
      else CXN_S1K3(4)
#undef CXN_S1K3
    } else if (S == 2 && sq == 3 && mode == 0 && pool_cells) {
      const int i0 = P / 2, j0 = P / 2;
      const int HC = (P + H - 1) / 2 - i0 + 1, WC = (P + W - 1) / 2 - j0 + 1;
      const long tot = static_cast<long>(N) * HC * WC * (C / 8);
      CXN_LAUNCH((pool_bwd_s2k3), cdiv(tot, NT), NT, 0, S_, 
          (const bf16_t *)x, (const uint8_t *)arg, (const bf16_t *)dy, (bf16_t *)dx, H, W, C, Ho, Wo, P, relu, i0,
          j0, WC, make_fastdiv(static_cast<uint32_t>(C / 8)), make_fastdiv(static_cast<uint32_t>(WC * (C / 8))),
          make_fastdiv(static_cast<uint32_t>(HC)), static_cast<uint32_t>(tot));
    } else if (S == 2 && sq == 3) CXN_POOL_BWD(2, 3);
    else if (S == 1 && sq == 3) CXN_POOL_BWD(1, 3);
    else if (S == 2 && sq == 2) CXN_POOL_BWD(2, 2);
    else CXN_POOL_BWD(0, 0);
#undef CXN_POOL_BWD
    RET;
  }
  if (C % 8 == 0) {
    const long total = static_cast<long>(N) * H * W * C / 8;
    int nb = nblocks(total);
    size_t shm = 0;
    if (db) {  // gridDim*NT must be a multiple of C/8 (fixed channel group per thread)
      const int cv = C / 8;
      int gcd = cv, b = NT;
      while (b) { const int t = gcd % b; gcd = b; b = t; }
      const int m = cv / gcd;
      nb = nb / m * m;
      if (nb < m) nb = m;
      shm = static_cast<size_t>(C) * sizeof(float);
    }
    if (db && (ws == nullptr || ws_elems < static_cast<long>(nb) * C)) return -2;
    CXN_LAUNCH((pool_bwd<8>), nb, NT, shm, S_, (const bf16_t *)x, (const uint8_t *)arg, (const bf16_t *)dy, (bf16_t *)dx, N, H,
                                     W, C, Ho, Wo, KH, KW, S, P, mode, relu, db ? ws : nullptr);
    if (db) CXN_LAUNCH((partials_reduce), partials_grid(nb, C), NT, 0, S_, ws, nb, C, db);
  } else {
    if (db) return -2;
    CXN_LAUNCH((pool_bwd<1>), nblocks(static_cast<long>(N) * H * W * C), NT, 0, S_, 
        (const bf16_t *)x, (const uint8_t *)arg, (const bf16_t *)dy, (bf16_t *)dx, N, H, W, C, Ho, Wo, KH, KW, S, P,
        mode, relu, nullptr);
  }
  RET;
}
CXN_API int cxn_lrn_fwd(const void *x, void *y, long npix, int C, int nsize, float alpha, float beta, float knorm,
                        void *stream) {
  if (C % 8 != 0 || nsize / 2 > 4) return -1;
  const int tpp = C / 8;
  if (tpp <= 64) {  // shuffle form
    const long waves = (npix + 64 / tpp - 1) / (64 / tpp);
    const long ngroups = (waves + NT / 64 - 1) / (NT / 64);
    const int blocks = static_cast<int>(std::min<long>(ngroups, 4096));
    const float sa = alpha / nsize;
#define CXN_LF(HV) CXN_LAUNCH((lrn_fwd_shfl<HV>), blocks, NT, 0, S_, (const bf16_t *)x, (bf16_t *)y, npix, C, sa, beta, \
                              knorm, ngroups)
    switch (nsize / 2) {
      case 0: CXN_LF(0); break;
      case 1: CXN_LF(1); break;
      case 2: CXN_LF(2); break;
      case 3: CXN_LF(3); break;
      default: CXN_LF(4); break;
    }
#undef CXN_LF
    RET;
  }
  CXN_LAUNCH((lrn_fwd), nblocks(npix * C / 8), NT, 0, S_, (const bf16_t *)x, (bf16_t *)y, npix, C, nsize / 2, alpha / nsize,
                                                 beta, knorm);
  RET;
}
// fused max-pool (3x3 / 2, pad 0) -> LRN; see pool_lrn_fwd / lrn_pool_bwd.  -1: not served.
CXN_API int cxn_pool_lrn_fwd(const void *x, void *P, void *arg, void *Y, int N, int Hin, int Win, int C, int Ho, int Wo,
                             int relu, int nsize, float alpha, float beta, float knorm, void *stream) {
  const int tpp = C / 8, half = nsize / 2;
  if (C % 8 || tpp > 64 || half > 4 || Hin < 3 || Win < 3) return -1;
  if (Ho != min(Hin - 2, Hin - 1) / 2 + 1 || Wo != min(Win - 2, Win - 1) / 2 + 1) return -1;  // ceil-mode 3x3 / 2
  const long npix = static_cast<long>(N) * Ho * Wo;
  const long waves = (npix + 64 / tpp - 1) / (64 / tpp);
  const int blocks = static_cast<int>((waves + NT / 64 - 1) / (NT / 64));
  const float sa = alpha / nsize;
  // relu bit 2 (4): the input is a relu output (>= 0): the integer-key max (pool_lrn_fwd NN)
  const bool nn = (relu & 4) != 0 && (relu & 1) == 0;
#define CXN_PLF(HV)                                                                                            \
  if (nn) CXN_LAUNCH((pool_lrn_fwd<HV, true>), blocks, NT, 0, S_, (const bf16_t *)x, (bf16_t *)P, (uint8_t *)arg, \
                     (bf16_t *)Y, N, Hin, Win, C, Ho, Wo, relu, sa, beta, knorm);                                    \
  else CXN_LAUNCH((pool_lrn_fwd<HV, false>), blocks, NT, 0, S_, (const bf16_t *)x, (bf16_t *)P, (uint8_t *)arg,  \
                  (bf16_t *)Y, N, Hin, Win, C, Ho, Wo, relu, sa, beta, knorm)
  switch (half) {
    case 0: CXN_PLF(0); break;
    case 1: CXN_PLF(1); break;
    case 2: CXN_PLF(2); break;
    case 3: CXN_PLF(3); break;
    default: CXN_PLF(4); break;
  }
#undef CXN_PLF
  RET;
}
// dbias_part: fp32 [blocks][C] per-block partial sums of the masked pooled gradient (null: no
// bias sum); part_rows < 0: only return the block count.  Returns the block count (>= 0), -1
// when not served, -4 when part_rows is too small.  det: the partial rows summed in one fixed
// order (else 256-row chunks added atomically).
CXN_API int cxn_lrn_pool_bwd(const void *P, const void *dY, const void *arg, void *dx, int N, int Hin, int Win, int C,
                             int Ho, int Wo, int relu_bit, int nsize, float alpha, float beta, float knorm,
                             float *dbias, float *dbias_part, long part_rows, int det, void *stream) {
  const int tpp = C / 8, half = nsize / 2;
  if (C % 8 || tpp > 64 || half > 4 || Hin < 3 || Win < 3 || N < 1) return -1;
  if (Ho != min(Hin - 2, Hin - 1) / 2 + 1 || Wo != min(Win - 2, Win - 1) / 2 + 1) return -1;
  const int HC = (Hin + 1) / 2, WC = (Win + 1) / 2;
  // cell rows per block: the band's windows (R + 1 rows: one row recomputed) staged in LDS as bf16
  // gradient + offset byte, within 56 KiB of dynamic LDS (the bias partials take 9 KiB more)
  const long row_bytes = static_cast<long>(Wo) * C * 3;
  static const int r_env = [] {  // CXN_LRN_POOL_R: probe override of the band height
    const char *e = std::getenv("CXN_LRN_POOL_R");
    return e != nullptr ? std::atoi(e) : 0;
  }();
  // 4 rows, 2 for wide-channel maps (AlexNet pool1 C = 96: R 4 70.4 us, R 2 77.1; pool2 C = 256:
  // R 4 56.8 us, R 2 51.0 -- profiles/r5_lrn_pool_bwd_band_probe.jsonl)
  int R = r_env > 0 ? r_env : (C >= 192 ? 2 : 4);
  while (R > 1 && (R + 1) * row_bytes > 56 * 1024) --R;
  if ((R + 1) * row_bytes > 56 * 1024) return -1;
  if (static_cast<long>(Hin) * Win * C >= (1L << 31)) return -1;  // 32-bit offsets inside an image
  const int nband = (HC + R - 1) / R;
  const long blocks_l = static_cast<long>(N) * nband;
  if (blocks_l >= (1L << 31)) return -1;
  const int blocks = static_cast<int>(blocks_l);
  if (part_rows < 0) return blocks;  // query
  const float sa = alpha / nsize;
  float *part = dbias != nullptr ? dbias_part : nullptr;
  if (dbias != nullptr && (part == nullptr || part_rows < blocks)) return -4;
  // (the bias partials reuse the window buffer: at least NT x 9 floats)
  const size_t lds = std::max(static_cast<size_t>((R + 1) * row_bytes), static_cast<size_t>(NT * 9 * 4));
#define CXN_PLB(HV) CXN_LAUNCH((lrn_pool_bwd<HV>), blocks, NT, lds, S_, (const bf16_t *)P, (const bf16_t *)dY,        \
                               (const uint8_t *)arg, (bf16_t *)dx, Hin, Win, C, Ho, Wo, HC, WC, R, nband, relu_bit, sa, \
                               beta, knorm, part)
  switch (half) {
    case 0: CXN_PLB(0); break;
    case 1: CXN_PLB(1); break;
    case 2: CXN_PLB(2); break;
    case 3: CXN_PLB(3); break;
    default: CXN_PLB(4); break;
  }
#undef CXN_PLB
  if (part != nullptr) {
    const int chunk = det ? blocks : 32;  // 4 rows per thread: latency-bound otherwise
    CXN_LAUNCH((part_rows_colsum), dim3((C + 31) / 32, (blocks + chunk - 1) / chunk), NT, 0, S_, part, blocks, C,
               dbias, chunk);
  }
  if (hipGetLastError() != hipSuccess) return -3;
  return blocks;
}
// LRN backward plus db += the column sums of the stored dx (lrn_bwd_db): the shuffle form's
// shapes (C % 8 == 0, C / 8 <= 64, local_size <= 9); -1 otherwise (nothing launched).  part (fp32,
// part_floats >= 4096 * C): up to 4096 blocks store per-block sums there and part_rows_colsum
// adds them up; without it 1024 blocks add theirs with one atomic each per channel.
CXN_API int cxn_lrn_bwd_db(const void *x, const void *dy, void *dx, long npix, int C, int nsize, float alpha,
                           float beta, float knorm, int mask_relu, float *db, float *part, long part_floats,
                           void *stream) {
  if (C % 8 != 0 || C / 8 > 64 || nsize / 2 > 4 || db == nullptr || npix <= 0) return -1;
  const int tpp = C / 8, half = nsize / 2;
  const long waves = (npix + 64 / tpp - 1) / (64 / tpp);
  const long ngroups = (waves + NT / 64 - 1) / (NT / 64);
  if (part != nullptr && part_floats < 4096L * C) part = nullptr;
  const int blocks = static_cast<int>(std::min<long>(ngroups, part != nullptr ? 4096 : 1024));
  const float sa = alpha / nsize;
#define CXN_LDB(HV) CXN_LAUNCH((lrn_bwd_db<HV>), blocks, NT, 0, S_, (const bf16_t *)x, (const bf16_t *)dy, (bf16_t *)dx, \
                               npix, C, sa, beta, knorm, mask_relu, ngroups, db, part)
  switch (half) {
    case 0: CXN_LDB(0); break;
    case 1: CXN_LDB(1); break;
    case 2: CXN_LDB(2); break;
    case 3: CXN_LDB(3); break;
    default: CXN_LDB(4); break;
  }
#undef CXN_LDB
  if (part != nullptr)
    CXN_LAUNCH((part_rows_colsum), dim3((C + 31) / 32, (blocks + 31) / 32), NT, 0, S_, part, blocks, C, db, 32);
  RET;
}
CXN_API int cxn_lrn_bwd(const void *x, const void *dy, void *dx, long npix, int C, int nsize, float alpha, float beta,
                        float knorm, int mask_relu, void *stream) {
  if (C % 8 != 0) return -1;
  const int half = nsize / 2;
  const int tpp = C / 8;  // threads per pixel
  if (tpp <= 64 && half <= 4) {  // shuffle form: whole pixels per wave
    const long waves = (npix + 64 / tpp - 1) / (64 / tpp);
    const int blocks = static_cast<int>((waves + NT / 64 - 1) / (NT / 64));
    const float sa = alpha / nsize;
    switch (half) {
      case 0: CXN_LAUNCH((lrn_bwd_shfl<0>), blocks, NT, 0, S_, (const bf16_t *)x, (const bf16_t *)dy, (bf16_t *)dx, npix, C, sa, beta, knorm, mask_relu); break;
      case 1: CXN_LAUNCH((lrn_bwd_shfl<1>), blocks, NT, 0, S_, (const bf16_t *)x, (const bf16_t *)dy, (bf16_t *)dx, npix, C, sa, beta, knorm, mask_relu); break;
      case 2: CXN_LAUNCH((lrn_bwd_shfl<2>), blocks, NT, 0, S_, (const bf16_t *)x, (const bf16_t *)dy, (bf16_t *)dx, npix, C, sa, beta, knorm, mask_relu); break;
      case 3: CXN_LAUNCH((lrn_bwd_shfl<3>), blocks, NT, 0, S_, (const bf16_t *)x, (const bf16_t *)dy, (bf16_t *)dx, npix, C, sa, beta, knorm, mask_relu); break;
      default: CXN_LAUNCH((lrn_bwd_shfl<4>), blocks, NT, 0, S_, (const bf16_t *)x, (const bf16_t *)dy, (bf16_t *)dx, npix, C, sa, beta, knorm, mask_relu); break;
    }
    RET;
  }
  if (tpp <= NT && (C + 2 * half) * 3 * 4 * (NT / tpp) <= 48 * 1024) {
    // LDS-staged form: each pixel row is read once, norm computed once per channel,
    // and dx may alias x (all reads of a pixel complete before its first write).
    const int ppb = NT / tpp;
    const int blocks = static_cast<int>((npix + ppb - 1) / ppb);
    const size_t smem = static_cast<size_t>(ppb) * (C + 2 * half) * 3 * sizeof(float);
    CXN_LAUNCH((lrn_bwd_lds), blocks, NT, smem, S_, (const bf16_t *)x, (const bf16_t *)dy, (bf16_t *)dx, npix, C, half,
                                          alpha / nsize, beta, knorm, mask_relu);
    RET;
  }
  if (half > 4 || x == dx) return -1;
  CXN_LAUNCH((lrn_bwd), nblocks(npix * C / 8), NT, 0, S_, (const bf16_t *)x, (const bf16_t *)dy, (bf16_t *)dx, npix, C,
                                                 half, alpha / nsize, beta, knorm, mask_relu);
  RET;
}
CXN_API int cxn_act_fwd(const void *x, void *y, void *y2, long n, int kind, float b, void *stream) {
  CXN_LAUNCH((act_fwd), nblocks(n / 8 + 1), NT, 0, S_, (const bf16_t *)x, (bf16_t *)y, (bf16_t *)y2, n, kind, b);
  RET;
}
CXN_API int cxn_act_bwd(const void *y, const void *dy, void *dx, long n, int kind, float b, void *stream) {
  CXN_LAUNCH((act_bwd), nblocks(n / 8 + 1), NT, 0, S_, (const bf16_t *)y, (const bf16_t *)dy, (bf16_t *)dx, n, kind, b);
  RET;
}
CXN_API int cxn_dropout(const void *x, void *y, long n, unsigned seed, const int *counter, float pkeep,
                        void *stream) {
  const double t = static_cast<double>(pkeep) * 4294967296.0;
  const uint32_t thresh = t >= 4294967295.0 ? 0xFFFFFFFFu : static_cast<uint32_t>(t);
  CXN_LAUNCH((dropout_apply), nblocks(n / 8 + 1), NT, 0, S_, (const bf16_t *)x, (bf16_t *)y, n, seed, counter, thresh, 1.0f / pkeep);
  RET;
}

// acc: float64 [nm] metric sums (+= this batch); part: fp32 workspace of >= 256*nm floats.
CXN_API int cxn_metric_eval(const float *p, int ldp, const float *lab, int ldl, int lw, int B, int K, int nm,
                            const int *kinds, const int *args, double *acc, float *part, void *stream) {
  if (nm < 1 || nm > 8 || B < 1) return nm < 1 || B < 1 ? 0 : -1;
  MetricSpec ms{};
  ms.nm = nm;
  for (int m = 0; m < nm; ++m) {
    ms.kind[m] = kinds[m];
    ms.arg[m] = args[m];
  }
  int nb = (B + 3) / 4;
  if (nb > 256) nb = 256;
  CXN_LAUNCH((metric_rows), nb, 256, 0, S_, p, ldp, lab, ldl, lw, B, K, ms, part);
  CXN_LAUNCH((metric_accum), 1, 64, 0, S_, part, nb, nm, acc);
  RET;
}

CXN_API int cxn_softmax(const void *x, void *y, float *pf, int rows, int K, void *stream) {
  if (rows <= 0) return 0;
  if (K <= 1024 && rows < (1 << 30)) {
    const bf16_t *xb = (const bf16_t *)x;
    bf16_t *yb = (bf16_t *)y;
    if (K <= 256) CXN_LAUNCH((softmax_rows_reg<4>), rows, 64, 0, S_, xb, yb, pf, K);
    else if (K <= 512) CXN_LAUNCH((softmax_rows_reg<8>), rows, 64, 0, S_, xb, yb, pf, K);
    else CXN_LAUNCH((softmax_rows_reg<16>), rows, 64, 0, S_, xb, yb, pf, K);
    RET;
  }
  CXN_LAUNCH((softmax_rows), cdiv(rows, 4), 256, 0, S_, (const bf16_t *)x, (bf16_t *)y, pf, rows, K);
  RET;
}
CXN_API int cxn_loss_grad(const float *p32, void *node, const float *label, int rows, int K, int lw, float scale,
                          int kind, void *stream) {
  CXN_LAUNCH((loss_grad), nblocks(static_cast<long>(rows) * K), NT, 0, S_, p32, (bf16_t *)node, label, rows, K, lw, scale, kind);
  RET;
}
CXN_API int cxn_colsum(const void *dy, float *db, long rows, int C, float *ws, long ws_elems, void *stream) {
  if (C % 8) {
    CXN_LAUNCH((colsum_scalar), cdiv(C, NT), NT, 0, S_, (const bf16_t *)dy, db, rows, C);
    RET;
  }
  const int CV = C / 8;
  int rpb = 512;
  // keep the partials within the caller's workspace
  while (static_cast<long>(cdiv(rows, rpb)) * C > ws_elems && rpb < (1 << 24)) rpb *= 2;
  // atomics straight into db: at most ~512 adders per channel (VGG conv1_2's 3.2M rows at 512
  // rows per block put 6272 atomics on each of 64 addresses and ran slower than two passes)
  if (!cxn_deterministic)
    while (cdiv(rows, rpb) > 512) rpb *= 2;
  if (static_cast<long>(cdiv(rows, rpb)) * C > ws_elems) return -2;
  dim3 grid(cdiv(rows, rpb), cdiv(CV, 64));
  if (!cxn_deterministic) {  // per-block atomics straight into db
    CXN_LAUNCH((colsum_bf16), grid, NT, 0, S_, (const bf16_t *)dy, ws, rows, C, rpb, db);
    RET;
  }
  CXN_LAUNCH((colsum_bf16), grid, NT, 0, S_, (const bf16_t *)dy, ws, rows, C, rpb, nullptr);
  CXN_LAUNCH((partials_reduce), partials_grid(static_cast<int>(grid.x), C), NT, 0, S_, ws, static_cast<int>(grid.x), C, db);
  RET;
}
// dys / dbs / rows / Cs: n deferred bias gradients (C % 8 == 0 each); masks: nullable array of
// nullable max-pool offset tensors (masked segments, see colsum_multi)
CXN_API int cxn_colsum_multi(const void *const *dys, float *const *dbs, const long *rows, const int *Cs,
                             const void *const *masks, int n, void *stream, const long *lds) {
  for (int base = 0; base < n; base += COLSUM_MAXSEG) {
    ColsumTable tab;
    const int cnt = n - base < COLSUM_MAXSEG ? n - base : COLSUM_MAXSEG;
    int nblk = 0;
    tab.n = cnt;
    for (int i = 0; i < cnt; ++i) {
      const int j = base + i;
      if (Cs[j] % 8) return -1;
      const long ld = lds ? lds[j] : Cs[j];
      if (ld % 8 || ld < Cs[j] || (masks && masks[j] && ld != Cs[j])) return -1;
      // <= 1024 blocks (adders per channel) per segment, >= 256 rows per block: the largest
      // segment (AlexNet conv1: 774k rows) needs ~4 blocks per CU to keep HBM busy
      long nb = cdiv(rows[j], 256L);
      int nchunk = 1;
      if (colsum_split) {
        // one block per (rows, chunk of <= 64 column vectors) reading ~96 KiB, >= 8 rows per
        // thread (one round of the 8-deep load batch): fc6 (256 x 4096) gets 24 blocks, not 1
        const int CV = Cs[j] / 8;
        nchunk = (CV + 63) / 64;
        const int CB = CV < 64 ? CV : 64;
        const long bpr = static_cast<long>(CB) * 8 * (masks && masks[j] ? 3 : 2);
        long want = 98304 / bpr;
        const long minr = (NT / CB) * 8L;
        if (want < minr) want = minr;
        nb = cdiv(rows[j], want);
      }
      if (nb > 1024) nb = 1024;
      if (nb < 1) nb = 1;
      const int rpb = rows[j] > 0 ? static_cast<int>(cdiv(rows[j], nb)) : 1;
      const int nrb = static_cast<int>(cdiv(rows[j], static_cast<long>(rpb)));
      tab.s[i] = ColsumSeg{static_cast<const bf16_t *>(dys[j]),
                           masks ? static_cast<const uint8_t *>(masks[j]) : nullptr, dbs[j], rows[j], ld, Cs[j], rpb,
                           nrb * nchunk, nchunk};
      tab.b0[i] = nblk;
      nblk += tab.s[i].nblk;
    }
    if (nblk > 0) CXN_LAUNCH((colsum_multi), nblk, NT, 0, S_, tab);
  }
  RET;
}
int cxn_deterministic = 0;
CXN_API int cxn_set_deterministic(int on) {
  cxn_deterministic = on ? 1 : 0;
  return 0;
}

CXN_API int cxn_splitk_accumulate(const float *ws, int nsplit, long slab, float *out, void *stream) {
  if ((reinterpret_cast<uintptr_t>(ws) | reinterpret_cast<uintptr_t>(out)) & 15 || slab % 4) return -1;
  long b = (slab / 4 + NT - 1) / NT;
  if (b > 4096) b = 4096;
  if (b < 1) b = 1;
  CXN_LAUNCH((splitk_accumulate), static_cast<int>(b), NT, 0, S_, ws, nsplit, slab, out);
  RET;
}

CXN_API int cxn_splitk_finalize(const float *ws, int nsplit, long slab, void *out, long rows, int cols,
                                const float *bias, int relu, int mask_relu, void *stream) {
  if (cols % 8) return -2;
  dim3 grid(cdiv(cols / 8, NT), static_cast<unsigned>(rows));
  CXN_LAUNCH((splitk_finalize<false>), grid, NT, 0, S_, ws, nsplit, slab, (bf16_t *)out, rows, cols, bias, relu,
             mask_relu, 0u, (const int *)nullptr, 0u, 1.f);
  RET;
}
// the same with the dropout of a fused fc -> relu -> dropout (mask as cxn_dropout)
CXN_API int cxn_splitk_finalize_dropout(const float *ws, int nsplit, long slab, void *out, long rows, int cols,
                                        const float *bias, int relu, unsigned seed, const int *counter, float pkeep,
                                        void *stream) {
  if (cols % 8 || static_cast<double>(rows) * cols >= 4294967296.0) return -2;
  dim3 grid(cdiv(cols / 8, NT), static_cast<unsigned>(rows));
  const double t = static_cast<double>(pkeep) * 4294967296.0;  // as cxn_dropout
  const uint32_t thresh = t >= 4294967295.0 ? 0xFFFFFFFFu : static_cast<uint32_t>(t);
  CXN_LAUNCH((splitk_finalize<true>), grid, NT, 0, S_, ws, nsplit, slab, (bf16_t *)out, rows, cols, bias, relu, 0,
             static_cast<uint32_t>(seed), counter, thresh, 1.f / pkeep);
  RET;
}
CXN_API int cxn_cast_f32_bf16(const float *x, void *y, long n, void *stream) {
  CXN_LAUNCH((cast_f32_bf16), nblocks(n), NT, 0, S_, x, (bf16_t *)y, n);
  RET;
}
CXN_API int cxn_add_bf16(const void *a, const void *b, void *y, long n, void *stream) {
  CXN_LAUNCH((add_bf16), nblocks(n / 8 + 1), NT, 0, S_, (const bf16_t *)a, (const bf16_t *)b, (bf16_t *)y, n);
  RET;
}
CXN_API int cxn_fanout_bf16(const void *src, void *d0, void *d1, void *d2, void *d3, int nd, long n, void *stream) {
  if (nd < 1 || nd > 4 || (n & 7) != 0) return -2;
  const long n8 = n / 8;
  CXN_LAUNCH((fanout_bf16), nblocks(n8), NT, 0, S_, (const uint4 *)src, (uint4 *)d0, (uint4 *)d1, (uint4 *)d2, (uint4 *)d3, nd,
                                          n8);
  RET;
}
CXN_API int cxn_sum_bf16(const void *s0, const void *s1, const void *s2, const void *s3, int ns, void *y, long n,
                         void *stream, int mask) {
  if (ns < 2 || ns > 4 || (n & 7) != 0) return -2;
  const long n8 = n / 8;
  CXN_LAUNCH((sum_bf16), nblocks(n8), NT, 0, S_, (const uint4 *)s0, (const uint4 *)s1, (const uint4 *)s2, (const uint4 *)s3, ns,
                                       (uint4 *)y, n8, mask);
  RET;
}
// ins[k] (NHWC, cs[k] channels, k < n <= 4) <-> out (Ct channels), npix pixels; bwd: out -> ins
CXN_API int cxn_concat(void *const *ins, const int *cs, int n, void *out, int Ct, long npix, int bwd, int mask,
                       void *stream) {
  if (n < 1 || n > 4 || Ct % 8) return -1;
  ConcatArgs a{};
  int off = 0;
  for (int k = 0; k < n; ++k) {
    if (cs[k] % 8) return -1;
    a.in[k] = static_cast<uint4 *>(ins[k]);
    a.c8[k] = cs[k] / 8;
    a.off8[k] = off / 8;
    off += cs[k];
  }
  if (off != Ct) return -1;
  const long total8 = npix * (Ct / 8);
  if (total8 >= (1L << 32)) return -1;
  CXN_LAUNCH((concat8), nblocks(total8), NT, 0, S_, a, n, static_cast<uint4 *>(out), Ct / 8, static_cast<uint32_t>(total8), bwd,
                                          mask);
  RET;
}
CXN_API int cxn_channel_copy(const void *src, int Cs, int soff, void *dst, int Cd, int doff, int Cc, long npix,
                             int accumulate, void *stream) {
  const long total8 = npix * (Cc / 8);
  if (((Cs | soff | Cd | doff | Cc) & 7) == 0 && ((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst)) & 15) == 0 &&
      total8 > 0 && total8 < (1L << 31)) {
    CXN_LAUNCH((channel_copy8), nblocks(total8), NT, 0, S_, (const uint4 *)src, Cs / 8, soff / 8, (uint4 *)dst, Cd / 8, doff / 8,
                                                  Cc / 8, static_cast<uint32_t>(total8), accumulate);
    RET;
  }
  CXN_LAUNCH((channel_copy), nblocks(npix * Cc), NT, 0, S_, (const bf16_t *)src, Cs, soff, (bf16_t *)dst, Cd, doff, Cc, npix,
                                                  accumulate);
  RET;
}

CXN_API int cxn_pad_interior(const void *src, void *dst, int N, int H, int W, int C, int H2, int W2, int py, int px,
                             void *stream) {
  const long npix = static_cast<long>(N) * H * W;
  const int bytes = C * 2;
  if (bytes % 8 == 0 && ((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst)) & 7) == 0) {
    CXN_LAUNCH((pad_interior<uint2>), nblocks(npix * (bytes / 8)), NT, 0, S_, (const uint2 *)src, (uint2 *)dst, npix, H, W,
               H2, W2, py, px, bytes / 8);
  } else {
    CXN_LAUNCH((pad_interior<bf16_t>), nblocks(npix * C), NT, 0, S_, (const bf16_t *)src, (bf16_t *)dst, npix, H, W, H2,
               W2, py, px, C);
  }
  RET;
}

CXN_API int cxn_add_rows_f32(const float *src, float *dst, long rows, int L, int Ls, void *stream) {
  if (rows <= 0 || L <= 0) return 0;
  CXN_LAUNCH((add_rows_f32), nblocks(rows * L), NT, 0, S_, src, dst, rows, L, Ls);
  RET;
}

CXN_API int cxn_pad_rows(const void *src, void *dst, long rows, int L, int Lp, void *stream) {
  CXN_LAUNCH((pad_rows), nblocks(rows * Lp), NT, 0, S_, (const bf16_t *)src, (bf16_t *)dst, rows, L, Lp);
  RET;
}
