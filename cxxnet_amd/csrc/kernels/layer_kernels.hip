// Kernels of the less common reference layers (all NHWC bf16 activations, fp32 statistics):
//   batch_norm            per-channel batch statistics, normalise, backward
//                         (reference src/layer/batch_norm_layer-inl.hpp:98-179)
//   prelu                 per-channel slope, optional multiplicative train-time noise
//                         (reference src/layer/prelu_layer-inl.hpp:111-152)
//   insanity              randomized leaky relu (reference src/layer/insanity_layer-inl.hpp:47-82)
//   insanity_max_pooling  max pooling over randomly shifted sources
//                         (reference src/layer/insanity_pooling_layer-inl.hpp:63-94, 170-205)
// Random draws are a counter hash of (element index, hash(step counter, layer seed)) --
// the same generator as dropout -- so backward regenerates forward's draws without storing a
// mask, and a captured HIP graph draws fresh values each replay (the counter lives on device).
#include "common.h"

namespace {

constexpr int NT = 256;

__device__ __forceinline__ uint32_t hash_u32(uint32_t x, uint32_t seed) {
  x ^= seed * 0x9E3779B9u;
  x ^= x >> 16; x *= 0x7FEB352Du;
  x ^= x >> 15; x *= 0x846CA68Bu;
  x ^= x >> 16;
  return x;
}
__device__ __forceinline__ uint32_t eff_seed(uint32_t seed, const int *counter) {
  return counter ? hash_u32(static_cast<uint32_t>(*counter), seed) : seed;
}
__device__ __forceinline__ float u01(uint32_t idx, uint32_t seed) {
  return static_cast<float>(hash_u32(idx, seed)) * 2.3283064365386963e-10f;  // [0, 1)
}

static inline int nblocks(long n, int cap = 256 * 16) {
  long b = (n + NT - 1) / NT;
  if (b < 1) b = 1;
  return static_cast<int>(b > cap ? cap : b);
}

// ------------------------------------------------------------------ parameter initialisation
// Random weight init on the device (reference LayerParam::RandInitWeight, src/layer/param.h:
// 114-138, draws on the host through mshadow's Random): element i takes the 24-bit uniforms
// of hash(2i, seed) and hash(2i+1, seed); dist 0 = uniform a + (b - a) u, dist 1 = normal
// a + b z with Box-Muller z = sqrt(-2 ln(1 - u1)) cos(2 pi u2).  ops.rand_fill's host path is
// the same integer hash with float32 math, so CPU and GPU models of one seed start alike (to a
// few ulps of logf/cosf); VGG-16's 138M parameters no longer go through a host RNG + copy.
__global__ void rand_fill(float *__restrict__ out, uint32_t n, uint32_t seed, int dist, float a, float b) {
  for (uint32_t i = blockIdx.x * NT + threadIdx.x; i < n; i += gridDim.x * NT) {
    const float u1 = static_cast<float>(hash_u32(2u * i, seed) >> 8) * 5.9604644775390625e-08f;
    if (dist == 0) {
      out[i] = a + (b - a) * u1;
    } else {
      const float u2 = static_cast<float>(hash_u32(2u * i + 1u, seed) >> 8) * 5.9604644775390625e-08f;
      out[i] = a + b * (sqrtf(-2.0f * logf(1.0f - u1)) * cosf(6.283185307179586f * u2));
    }
  }
}

// ------------------------------------------------------------------ per-channel reductions
// x, g: [rows][C] bf16.  out[q][c] += partial sums (caller zeroes out):
//   mode 0: out0 = sum x                 mode 1: out0 = sum (x - mean)^2
//   mode 2: out0 = sum (x - mean), out1 = sum g, out2 = sum g (x - mean)       (BN backward)
//   mode 3: out0 = sum min(x, 0) g                                            (PReLU slope grad)
// Block: 64 channels x 4 row lanes; grid.y over channel groups, grid.x over row chunks.
__global__ void chan_reduce(const bf16_t *__restrict__ x, const bf16_t *__restrict__ g,
                            const float *__restrict__ mean, float *__restrict__ out, long rows, int C, int mode,
                            int rows_per_block) {
  const int cl = threadIdx.x & 63, rl = threadIdx.x >> 6;
  const int c = blockIdx.y * 64 + cl;
  const long r0 = static_cast<long>(blockIdx.x) * rows_per_block;
  const long r1 = min(rows, r0 + rows_per_block);
  float a0 = 0.f, a1 = 0.f, a2 = 0.f;
  if (c < C) {
    const float m = mean ? mean[c] : 0.f;
    for (long r = r0 + rl; r < r1; r += 4) {
      const float xv = bf2f(x[r * C + c]);
      if (mode == 0) {
        a0 += xv;
      } else if (mode == 1) {
        const float d = xv - m;
        a0 += d * d;
      } else if (mode == 2) {
        const float d = xv - m, gv = bf2f(g[r * C + c]);
        a0 += d;
        a1 += gv;
        a2 += gv * d;
      } else {
        a0 += fminf(xv, 0.f) * bf2f(g[r * C + c]);
      }
    }
  }
  __shared__ float red[3][4][64];
  red[0][rl][cl] = a0;
  red[1][rl][cl] = a1;
  red[2][rl][cl] = a2;
  __syncthreads();
  if (rl == 0 && c < C) {
    const int nq = mode == 2 ? 3 : 1;
    for (int q = 0; q < nq; ++q) {
      const float s = red[q][0][cl] + red[q][1][cl] + red[q][2][cl] + red[q][3][cl];
      atomicAdd(out + q * C + c, s);
    }
  }
}

// ------------------------------------------------------------------ batch norm
// stats[0] = sum x -> mean; stats[1] = sum (x-mean)^2 -> inv = 1/sqrt(var + eps)
__global__ void bn_mean(const float *sum, float *mean, int C, float scale) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c < C) mean[c] = sum[c] * scale;
}
__global__ void bn_inv(const float *sq, float *inv, int C, float scale, float eps) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c < C) inv[c] = 1.f / sqrtf(sq[c] * scale + eps);
}
// y = (x - mean) inv slope + bias; xhat (nullable) = (x - mean) inv; xsave (nullable) = x
__global__ void bn_fwd(const bf16_t *x, bf16_t *y, bf16_t *xhat, bf16_t *xsave, const float *__restrict__ mean,
                       const float *__restrict__ inv, const float *__restrict__ slope,
                       const float *__restrict__ bias, long rows, int C) {
  const long n = rows * C;
  for (long i = blockIdx.x * static_cast<long>(blockDim.x) + threadIdx.x; i < n;
       i += static_cast<long>(gridDim.x) * blockDim.x) {
    const int c = static_cast<int>(i % C);
    const bf16_t xr = x[i];
    const float h = (bf2f(xr) - mean[c]) * inv[c];
    if (xsave) xsave[i] = xr;
    if (xhat) xhat[i] = f2bf(h);
    y[i] = f2bf(h * slope[c] + bias[c]);
  }
}
// reference backward (batch_norm_layer-inl.hpp:148-161) from the sums s0 = sum(x-mean),
// s1 = sum g, s2 = sum g (x-mean): gslope += s2 inv, gbias += s1, and the data-grad
// coefficients dx = g A + (x - mean) B + Cc.
__global__ void bn_bwd_coeffs(const float *__restrict__ sums, const float *__restrict__ inv,
                              const float *__restrict__ slope, float *gslope, float *gbias, float *coef, int C,
                              float scale) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const float s0 = sums[c], s1 = sums[C + c], s2 = sums[2 * C + c];
  const float iv = inv[c], sl = slope[c];
  const float ve = 1.f / (iv * iv);                        // var + eps
  const float gvar = sl * s2 * -0.5f * iv / ve;            // (var+eps)^-1.5 = inv / (var+eps)
  const float gexp = -sl * s1 * iv + gvar * scale * (-2.f * s0);
  gslope[c] += s2 * iv;
  gbias[c] += s1;
  coef[c] = sl * iv;
  coef[C + c] = gvar * scale * 2.f;
  coef[2 * C + c] = gexp * scale;
}
__global__ void bn_bwd(const bf16_t *g, const bf16_t *xsave, bf16_t *dx, const float *__restrict__ mean,
                       const float *__restrict__ coef, long rows, int C) {
  const long n = rows * C;
  for (long i = blockIdx.x * static_cast<long>(blockDim.x) + threadIdx.x; i < n;
       i += static_cast<long>(gridDim.x) * blockDim.x) {
    const int c = static_cast<int>(i % C);
    dx[i] = f2bf(bf2f(g[i]) * coef[c] + (bf2f(xsave[i]) - mean[c]) * coef[C + c] + coef[2 * C + c]);
  }
}

// ------------------------------------------------------------------ prelu
__device__ __forceinline__ float prelu_mask(float slope, uint32_t i, uint32_t seed, float rnd) {
  float m = slope;
  if (rnd > 0.f) m = slope * (1.f + u01(i, seed) * rnd * 2.f - rnd);
  return fminf(fmaxf(m, 0.f), 1.f);
}
// mode 0: y = x > 0 ? x : x m      mode 1: dx = x > 0 ? g : g m   (x, y/g [rows][C])
__global__ void prelu_apply(const bf16_t *x, const bf16_t *g, bf16_t *y, const float *__restrict__ slope,
                            long rows, int C, uint32_t seed0, const int *counter, float rnd, int mode) {
  const uint32_t seed = eff_seed(seed0, counter);
  const long n = rows * C;
  for (long i = blockIdx.x * static_cast<long>(blockDim.x) + threadIdx.x; i < n;
       i += static_cast<long>(gridDim.x) * blockDim.x) {
    const int c = static_cast<int>(i % C);
    const float xv = bf2f(x[i]);
    const float m = prelu_mask(slope[c], static_cast<uint32_t>(i), seed, rnd);
    const float v = mode == 0 ? xv : bf2f(g[i]);
    y[i] = f2bf(xv > 0.f ? v : v * m);
  }
}

// ------------------------------------------------------------------ insanity (randomized leaky relu)
// train: d ~ U[lb, ub) per element; test: d = (lb + ub) / 2.
// mode 0: y = x > 0 ? x : x / d (y2 optional second output)   mode 1: dx = y > 0 ? g : g / d
__global__ void insanity_apply(const bf16_t *x, const bf16_t *g, bf16_t *y, bf16_t *y2, long n, float lb, float ub,
                               int train, uint32_t seed0, const int *counter, int mode) {
  const uint32_t seed = eff_seed(seed0, counter);
  for (long i = blockIdx.x * static_cast<long>(blockDim.x) + threadIdx.x; i < n;
       i += static_cast<long>(gridDim.x) * blockDim.x) {
    const float d = train ? lb + u01(static_cast<uint32_t>(i), seed) * (ub - lb) : 0.5f * (lb + ub);
    const float xv = bf2f(x[i]);
    const float v = mode == 0 ? xv : bf2f(g[i]);
    const bf16_t o = f2bf(xv > 0.f ? v : v / d);
    y[i] = o;
    if (y2) y2[i] = o;
  }
}

// ------------------------------------------------------------------ insanity max pooling
// Source element (n, y, x, c) of the window is read from a neighbour chosen by its own
// uniform flag u: u < keep stays, then [keep, keep+d) y-1, [.., +2d) y+1, [.., +3d) x-1, else x+1
// (clamped at the border), d = (1 - keep) / 4.  Windows are ceil-mode, no padding.
__device__ __forceinline__ void shifted(int &yy, int &xx, float u, float keep, float d, int H, int W) {
  if (u < keep) return;
  if (u < keep + d) yy = yy > 0 ? yy - 1 : yy;
  else if (u < keep + 2.f * d) yy = yy + 1 < H ? yy + 1 : H - 1;
  else if (u < keep + 3.f * d) xx = xx > 0 ? xx - 1 : xx;
  else xx = xx + 1 < W ? xx + 1 : W - 1;
}
__global__ void ins_pool_fwd(const bf16_t *__restrict__ x, bf16_t *__restrict__ y, bf16_t *__restrict__ ysave,
                             int N, int H, int W, int C, int Ho, int Wo, int K, int S, float keep, uint32_t seed0,
                             const int *counter) {
  const uint32_t seed = eff_seed(seed0, counter);
  const float d = (1.f - keep) * 0.25f;
  const long n_out = static_cast<long>(N) * Ho * Wo * C;
  for (long i = blockIdx.x * static_cast<long>(blockDim.x) + threadIdx.x; i < n_out;
       i += static_cast<long>(gridDim.x) * blockDim.x) {
    const int c = static_cast<int>(i % C);
    long t = i / C;
    const int px = static_cast<int>(t % Wo);
    t /= Wo;
    const int py = static_cast<int>(t % Ho);
    const int n = static_cast<int>(t / Ho);
    const int y0 = py * S, y1 = min(y0 + K, H), x0 = px * S, x1 = min(x0 + K, W);
    float m = -INFINITY;
    for (int yy = y0; yy < y1; ++yy)
      for (int xx = x0; xx < x1; ++xx) {
        const long src = ((static_cast<long>(n) * H + yy) * W + xx) * C + c;
        int ly = yy, lx = xx;
        shifted(ly, lx, u01(static_cast<uint32_t>(src), seed), keep, d, H, W);
        m = fmaxf(m, bf2f(x[((static_cast<long>(n) * H + ly) * W + lx) * C + c]));
      }
    const bf16_t o = f2bf(m);
    y[i] = o;
    if (ysave) ysave[i] = o;
  }
}
// dx (distinct from x) for every source element: its shifted value compared with each
// covering window's max (value-compare unpool, every tie gets the gradient).
__global__ void ins_pool_bwd(const bf16_t *__restrict__ x, const bf16_t *__restrict__ ypool,
                             const bf16_t *__restrict__ gy, bf16_t *__restrict__ dx, int N, int H, int W, int C,
                             int Ho, int Wo, int K, int S, float keep, uint32_t seed0, const int *counter) {
  const uint32_t seed = eff_seed(seed0, counter);
  const float d = (1.f - keep) * 0.25f;
  const long n_in = static_cast<long>(N) * H * W * C;
  for (long i = blockIdx.x * static_cast<long>(blockDim.x) + threadIdx.x; i < n_in;
       i += static_cast<long>(gridDim.x) * blockDim.x) {
    const int c = static_cast<int>(i % C);
    long t = i / C;
    const int xx = static_cast<int>(t % W);
    t /= W;
    const int yy = static_cast<int>(t % H);
    const int n = static_cast<int>(t / H);
    int ly = yy, lx = xx;
    shifted(ly, lx, u01(static_cast<uint32_t>(i), seed), keep, d, H, W);
    const float vsrc = bf2f(x[((static_cast<long>(n) * H + ly) * W + lx) * C + c]);
    const int py0 = yy < K ? 0 : (yy - K + S) / S, px0 = xx < K ? 0 : (xx - K + S) / S;
    const int py1 = min((yy + S) / S, Ho), px1 = min((xx + S) / S, Wo);
    float acc = 0.f;
    for (int py = py0; py < py1; ++py)
      for (int px = px0; px < px1; ++px) {
        const long o = ((static_cast<long>(n) * Ho + py) * Wo + px) * C + c;
        if (vsrc == bf2f(ypool[o])) acc += bf2f(gy[o]);
      }
    dx[i] = f2bf(acc);
  }
}

}  // namespace

#define S_ static_cast<hipStream_t>(stream)
#define RET return hipGetLastError() == hipSuccess ? 0 : -3

// out must hold 3*C floats; it is zeroed here.
CXN_API int cxn_rand_fill(float *out, long n, unsigned seed, int dist, float a, float b, void *stream) {
  if (n < 0 || n > 0x7fffffffL) return -1;
  if (n == 0) return 0;
  CXN_LAUNCH((rand_fill), nblocks(n, 256 * 64), NT, 0, S_, out, static_cast<uint32_t>(n), seed, dist, a, b);
  RET;
}
CXN_API int cxn_chan_reduce(const void *x, const void *g, const float *mean, float *out, long rows, int C, int mode,
                            void *stream) {
  if (CXN_MEMSET(out, 0, sizeof(float) * 3 * C, S_) != hipSuccess) return -3;
  const int cg = (C + 63) / 64;
  int rb = static_cast<int>((rows + 255) / 256);
  if (rb > 1024 / cg + 1) rb = 1024 / cg + 1;
  if (cxn_deterministic) rb = 1;  // no cross-block atomics: one block per channel group
  const int rpb = static_cast<int>((rows + rb - 1) / rb);
  rb = static_cast<int>((rows + rpb - 1) / rpb);
  if (rb < 1) rb = 1;
  CXN_LAUNCH((chan_reduce), dim3(rb, cg), NT, 0, S_, (const bf16_t *)x, (const bf16_t *)g, mean, out, rows, C, mode, rpb);
  RET;
}
// stats: 3*C fp32 workspace; mean, inv: C fp32 outputs.  Two-pass (mean, then centred squares).
CXN_API int cxn_bn_stats(const void *x, float *stats, float *mean, float *inv, long rows, int C, float eps,
                         void *stream) {
  const float scale = 1.f / static_cast<float>(rows);
  int rc = cxn_chan_reduce(x, nullptr, nullptr, stats, rows, C, 0, stream);
  if (rc) return rc;
  CXN_LAUNCH((bn_mean), (C + NT - 1) / NT, NT, 0, S_, stats, mean, C, scale);
  rc = cxn_chan_reduce(x, nullptr, mean, stats, rows, C, 1, stream);
  if (rc) return rc;
  CXN_LAUNCH((bn_inv), (C + NT - 1) / NT, NT, 0, S_, stats, inv, C, scale, eps);
  RET;
}
CXN_API int cxn_bn_fwd(const void *x, void *y, void *xhat, void *xsave, const float *mean, const float *inv,
                       const float *slope, const float *bias, long rows, int C, void *stream) {
  CXN_LAUNCH((bn_fwd), nblocks(rows * C), NT, 0, S_, (const bf16_t *)x, (bf16_t *)y, (bf16_t *)xhat, (bf16_t *)xsave, mean, inv,
                                            slope, bias, rows, C);
  RET;
}
// sums/coef: 3*C fp32 workspaces.  dx may alias g.
CXN_API int cxn_bn_bwd(const void *g, const void *xsave, void *dx, const float *mean, const float *inv,
                       const float *slope, float *gslope, float *gbias, float *sums, float *coef, long rows, int C,
                       void *stream) {
  int rc = cxn_chan_reduce(xsave, g, mean, sums, rows, C, 2, stream);
  if (rc) return rc;
  CXN_LAUNCH((bn_bwd_coeffs), (C + NT - 1) / NT, NT, 0, S_, sums, inv, slope, gslope, gbias, coef, C,
                                                   1.f / static_cast<float>(rows));
  CXN_LAUNCH((bn_bwd), nblocks(rows * C), NT, 0, S_, (const bf16_t *)g, (const bf16_t *)xsave, (bf16_t *)dx, mean, coef, rows, C);
  RET;
}
CXN_API int cxn_prelu(const void *x, const void *g, void *y, const float *slope, long rows, int C, unsigned seed,
                      const int *counter, float rnd, int mode, void *stream) {
  CXN_LAUNCH((prelu_apply), nblocks(rows * C), NT, 0, S_, (const bf16_t *)x, (const bf16_t *)g, (bf16_t *)y, slope, rows, C,
                                                 seed, counter, rnd, mode);
  RET;
}
CXN_API int cxn_insanity(const void *x, const void *g, void *y, void *y2, long n, float lb, float ub, int train,
                         unsigned seed, const int *counter, int mode, void *stream) {
  CXN_LAUNCH((insanity_apply), nblocks(n), NT, 0, S_, (const bf16_t *)x, (const bf16_t *)g, (bf16_t *)y, (bf16_t *)y2, n, lb,
                                             ub, train, seed, counter, mode);
  RET;
}
CXN_API int cxn_ins_pool_fwd(const void *x, void *y, void *ysave, int N, int H, int W, int C, int Ho, int Wo, int K,
                             int S, float keep, unsigned seed, const int *counter, void *stream) {
  CXN_LAUNCH((ins_pool_fwd), nblocks(static_cast<long>(N) * Ho * Wo * C), NT, 0, S_, 
      (const bf16_t *)x, (bf16_t *)y, (bf16_t *)ysave, N, H, W, C, Ho, Wo, K, S, keep, seed, counter);
  RET;
}
CXN_API int cxn_ins_pool_bwd(const void *x, const void *ypool, const void *gy, void *dx, int N, int H, int W, int C,
                             int Ho, int Wo, int K, int S, float keep, unsigned seed, const int *counter,
                             void *stream) {
  CXN_LAUNCH((ins_pool_bwd), nblocks(static_cast<long>(N) * H * W * C), NT, 0, S_, 
      (const bf16_t *)x, (const bf16_t *)ypool, (const bf16_t *)gy, (bf16_t *)dx, N, H, W, C, Ho, Wo, K, S, keep,
      seed, counter);
  RET;
}
