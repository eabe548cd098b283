// Fused multi-tensor optimizer step over the flat parameter arena.
//
// One launch updates every parameter segment (weights and biases of every layer):
// fp32 master weight, fp32 gradient (zeroed after use, the reference's `dw = 0`),
// fp32 optimizer state, and the bf16 shadow copy the GEMM kernels consume.
//   SGD  (reference src/updater/sgd_updater-inl.hpp:73-84):
//        m = mu*m - lr*(clip(g) + wd*w);  w += m
//   NAG  (reference src/updater/nag_updater-inl.hpp:66-72):
//        old = m; m = mu*m - lr*(g + wd*w); w += (1+mu)*m - mu*old
//   Adam (reference src/updater/adam_updater-inl.hpp:74-82, incl. its `grad -= wd*w` sign):
//        g -= wd*w; m1 += d1*(g-m1); m2 += d2*(g^2-m2); w -= lr_t * m1/(sqrt(m2)+1e-8)
#include "common.h"

namespace {

constexpr int NT = 256;
constexpr int MAX_SEG = 48;

struct Seg {
  long off;
  long n;
  float lr, wd, mom, clip;
};
struct SegTable {
  Seg s[MAX_SEG];
};

__device__ __forceinline__ float clipg(float g, float c) {
  if (c == 0.f) return g;
  if (g != g) return 0.f;
  return fminf(fmaxf(g, -c), c);
}

// One element's step; returns the new weight.  m2 is used by adam only.
__device__ __forceinline__ float step1(int algo, const Seg &sg, float wv, float gv, float &m1, float &m2, float d1,
                                       float d2) {
  if (algo == 0) {
    // only the SGD updater clips (reference sgd_updater-inl.hpp:77-81); NAG and Adam
    // ignore clip_gradient
    gv = clipg(gv, sg.clip);
    // explicit fmas: the fc weight-gradient GEMM's fused step (gemm_glds.hip sgd_step) does
    // the same operations in the same order, so both give the same bits
    m1 = fmaf(sg.mom, m1, -sg.lr * fmaf(sg.wd, wv, gv));
    return wv + m1;
  }
  if (algo == 1) {
    const float old = m1;
    m1 = sg.mom * old - sg.lr * (gv + sg.wd * wv);
    return wv + (1.f + sg.mom) * m1 - sg.mom * old;
  }
  if (sg.wd > 0.f) gv -= sg.wd * wv;
  m1 += d1 * (gv - m1);
  m2 += d2 * (gv * gv - m2);
  return wv - sg.lr * (m1 / (sqrtf(m2) + 1e-8f));
}

// algo: 0 sgd, 1 nag, 2 adam.  st2 used by adam only.  wb may be null.
// Bandwidth-bound (22 B/param for SGD): four elements per thread through 16-byte loads and
// stores (8-byte bf16 shadow stores) for every segment whose offset is 4-aligned (all arena
// segments are 64-aligned); the < 4-element tail and unaligned slices go element-wise.
__global__ void __launch_bounds__(NT) fused_update(SegTable tab, float *__restrict__ w, float *__restrict__ g,
                                                   float *__restrict__ st1, float *__restrict__ st2,
                                                   bf16_t *__restrict__ wb, int algo_flags, float d1, float d2) {
  // algo_flags: bits 0-3 algorithm, bit 4 = zero the gradient after use (the reference's
  // `dw = 0`); without it the next step's first backprop overwrites/zeroes the gradient.
  const int algo = algo_flags & 15;
  const bool zero_g = (algo_flags & 16) != 0;
  const Seg sg = tab.s[blockIdx.y];
  const long stride = (long)gridDim.x * NT;
  long nvec = (sg.off & 3) == 0 ? sg.n >> 2 : 0;
  for (long q = blockIdx.x * (long)NT + threadIdx.x; q < nvec; q += stride) {
    const long k = sg.off + 4 * q;
    float4 wv = *reinterpret_cast<const float4 *>(w + k);
    const float4 gv = *reinterpret_cast<const float4 *>(g + k);
    float4 m1 = *reinterpret_cast<const float4 *>(st1 + k);
    float4 m2 = algo == 2 ? *reinterpret_cast<const float4 *>(st2 + k) : make_float4(0.f, 0.f, 0.f, 0.f);
    wv.x = step1(algo, sg, wv.x, gv.x, m1.x, m2.x, d1, d2);
    wv.y = step1(algo, sg, wv.y, gv.y, m1.y, m2.y, d1, d2);
    wv.z = step1(algo, sg, wv.z, gv.z, m1.z, m2.z, d1, d2);
    wv.w = step1(algo, sg, wv.w, gv.w, m1.w, m2.w, d1, d2);
    *reinterpret_cast<float4 *>(w + k) = wv;
    *reinterpret_cast<float4 *>(st1 + k) = m1;
    if (algo == 2) *reinterpret_cast<float4 *>(st2 + k) = m2;
    if (zero_g) *reinterpret_cast<float4 *>(g + k) = make_float4(0.f, 0.f, 0.f, 0.f);
    if (wb) *reinterpret_cast<uint2 *>(wb + k) = make_uint2(pack2(wv.x, wv.y), pack2(wv.z, wv.w));
  }
  for (long i = 4 * nvec + blockIdx.x * (long)NT + threadIdx.x; i < sg.n; i += stride) {
    const long k = sg.off + i;
    float m1 = st1[k], m2 = algo == 2 ? st2[k] : 0.f;
    const float wv = step1(algo, sg, w[k], g[k], m1, m2, d1, d2);
    st1[k] = m1;
    if (algo == 2) st2[k] = m2;
    w[k] = wv;
    if (zero_g) g[k] = 0.f;
    if (wb) wb[k] = f2bf(wv);
  }
}

// Non-finite check over a gradient range (failure detection): flag |= any(!isfinite).
__global__ void nonfinite_check(const float *__restrict__ g, long n, int *__restrict__ flag) {
  int bad = 0;
  for (long i = blockIdx.x * (long)NT + threadIdx.x; i < n; i += (long)gridDim.x * NT) {
    const float v = g[i];
    bad |= !(v - v == 0.f);
  }
  if (__any(bad) && (threadIdx.x & 63) == 0) atomicOr(flag, 1);
}

__global__ void scale_f32(float *__restrict__ x, long n, float s) {
  for (long i = blockIdx.x * (long)NT + threadIdx.x; i < n; i += (long)gridDim.x * NT) x[i] *= s;
}

}  // namespace

// segs: packed [nseg][6] doubles-as-floats: off, n, lr, wd, mom, clip
CXN_API int cxn_fused_update(const long *offs, const long *ns, const float *hyper /*[nseg][4]*/, int nseg, float *w,
                             float *g, float *st1, float *st2, void *wb, int algo, float d1, float d2, void *stream) {
  hipStream_t s = static_cast<hipStream_t>(stream);
  for (int base = 0; base < nseg; base += MAX_SEG) {
    SegTable tab;
    const int cnt = nseg - base < MAX_SEG ? nseg - base : MAX_SEG;
    long maxn = 1;
    for (int i = 0; i < cnt; ++i) {
      const int j = base + i;
      tab.s[i] = Seg{offs[j], ns[j], hyper[4 * j + 0], hyper[4 * j + 1], hyper[4 * j + 2], hyper[4 * j + 3]};
      if (ns[j] > maxn) maxn = ns[j];
    }
    long bx = (maxn + NT * 4 - 1) / (NT * 4);
    if (bx > 2048) bx = 2048;
    dim3 grid(static_cast<unsigned>(bx), cnt);
    CXN_LAUNCH((fused_update), grid, NT, 0, s, tab, w, g, st1, st2, static_cast<bf16_t *>(wb), algo, d1, d2);
  }
  return hipGetLastError() == hipSuccess ? 0 : -3;
}

CXN_API int cxn_nonfinite_check(const float *g, long n, int *flag, void *stream) {
  long b = (n + NT * 8 - 1) / (NT * 8);
  if (b > 1024) b = 1024;
  if (b < 1) b = 1;
  CXN_LAUNCH((nonfinite_check), b, NT, 0, static_cast<hipStream_t>(stream), g, n, flag);
  return hipGetLastError() == hipSuccess ? 0 : -3;
}

CXN_API int cxn_scale_f32(float *x, long n, float sc, void *stream) {
  long b = (n + NT * 8 - 1) / (NT * 8);
  if (b > 2048) b = 2048;
  if (b < 1) b = 1;
  CXN_LAUNCH((scale_f32), b, NT, 0, static_cast<hipStream_t>(stream), x, n, sc);
  return hipGetLastError() == hipSuccess ? 0 : -3;
}

// *p += v on the device (the step counter that dropout seeds and the updaters read): a library
// launch, so recorded launch lists and HIP graphs both advance it on every replay
__global__ void add_i32(int *p, int v) {
  if (threadIdx.x == 0) *p += v;
}
CXN_API int cxn_add_i32(int *p, int v, void *stream) {
  CXN_LAUNCH((add_i32), 1, 64, 0, static_cast<hipStream_t>(stream), p, v);
  return hipGetLastError() == hipSuccess ? 0 : -3;
}
