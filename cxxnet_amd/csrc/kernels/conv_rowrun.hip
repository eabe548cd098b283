// Direct forward convolution for few-channel, pad-0 first layers on kernel-row runs (AlexNet
// conv1: 3 channels on 228-pixel rows, 11x11 / 4, 96 outputs) for gfx950 -- reference
// src/layer/convolution_layer-inl.hpp:70-105 (im2col + GEMM).
//
// The implicit GEMM (gemm_glds K_ROWGATHER) gathers every output pixel's 11 kernel-row runs on
// its own: the 11x11 / 4 windows overlap ~7.6x, so at batch 256 it pulls 681 MB of runs through
// L2 for a 79 MB input and is load-bound (128 us, ~420 TFLOP/s).  Here a block walks output
// row groups (persistent grid) and stages the input rows a group needs ONCE in LDS:
//   * weights [Cout][KP] (row-padded runs, zero tails) are staged once per block;
//   * one work item = 4 output rows of one image; its S*3 + KH input rows are ONE contiguous
//     span of x (pad 0, rows back to back), copied global -> LDS with 1-KiB LDS-DMA
//     instructions (buffer_load ... lds) into a double buffer: item i+1's rows land while
//     item i's MFMAs run; past the tensor end the buffer descriptor returns zeros;
//   * k = (kernel row kh, position jj in the row's KW*C run padded to LP): a B fragment chunk
//     (8 consecutive k of one pixel) is 8 consecutive elements of a staged row, two
//     ds_read_b64 (8-byte aligned: pixel steps are S*C*2 bytes); the pad positions read the
//     next pixels' values, which meet zero weights;
//   * 8 waves, two per SIMD: wave (co half, output row) owns CFH x 16 output channels of one
//     row of 64 pixels: CFH x 4 accumulator tiles of v_mfma_f32_16x16x32_bf16; per k-step CFH A
//     reads (b128) and 8 B reads (b64) for 4 x CFH MFMAs, the next k-step's reads issued before
//     this one's MFMAs (the tap offset is arithmetic, no LDS table on the dependency chain);
//   * epilogue: bias + relu in fp32 -> bf16, transposed through LDS (the item's input buffer,
//     free by then) so each pixel's channels leave as 16-byte buffer stores; every store
//     instruction is issued (masked lanes store out of range), so the next item waits with a
//     counted s_waitcnt for its own DMAs only, not for these stores.
#include <cstdlib>
#include "common.h"

namespace {

constexpr int NT = 512;   // 8 waves, two per SIMD: one's LDS reads overlap the other's MFMAs
constexpr int RG = 4;     // output rows per work item (one per wave pair)
typedef __amdgpu_buffer_rsrc_t rsrc_t;
typedef __attribute__((address_space(3))) void lds_void;

__device__ __forceinline__ void wave_lds_handoff() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
}

template <int N_>
__device__ __forceinline__ void vm_wait_le() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N_) : "memory"); }
__device__ __forceinline__ void vm_wait(int n) {  // s_waitcnt vmcnt(n), n uniform, 0..15
  switch (n) {
    case 0: vm_wait_le<0>(); break;  case 1: vm_wait_le<1>(); break;  case 2: vm_wait_le<2>(); break;
    case 3: vm_wait_le<3>(); break;  case 4: vm_wait_le<4>(); break;  case 5: vm_wait_le<5>(); break;
    case 6: vm_wait_le<6>(); break;  case 7: vm_wait_le<7>(); break;  case 8: vm_wait_le<8>(); break;
    case 9: vm_wait_le<9>(); break;  case 10: vm_wait_le<10>(); break; case 11: vm_wait_le<11>(); break;
    case 12: vm_wait_le<12>(); break; case 13: vm_wait_le<13>(); break; case 14: vm_wait_le<14>(); break;
    default: vm_wait_le<15>(); break;
  }
}

template <int CFH>  // 16-channel output fragments per wave (Cout = 32 * CFH)
__global__ void __launch_bounds__(NT, 1)
conv_rowrun_fwd(const bf16_t *__restrict__ x, long x_bytes, const bf16_t *__restrict__ w, const float *__restrict__ bias,
                bf16_t *__restrict__ y, long y_bytes, int N, int H, int W, int C, int Ho, int Wo, int KH, int LP, FastDiv fd_lp, int S,
                int ldc, int relu, int KS, int XB, int ndma, int counted) {
  constexpr int COUT = 32 * CFH;
  constexpr int NWV = NT / 64;
  extern __shared__ __attribute__((aligned(1024))) char smem[];
  const int KP = KS * 32;                  // k padded to whole k-steps
  const int WPB = KP * 2 + 16;             // weight row pitch (bytes)
  const int pitch = W * C * 2;             // input row (bytes)
  const int K = KH * LP;
  char *sx0 = smem;                        // [2][XB] staged input spans
  char *sw = smem + 2 * XB;                // [COUT][WPB]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g4 = lane >> 4, l16 = lane & 15;
  const rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t *>(x), (short)0,
                                                      static_cast<int>(x_bytes), 0x00020000);

  const int groups_per_img = (Ho + RG - 1) / RG;
  const long items = static_cast<long>(N) * groups_per_img;
  auto issue = [&](long it, int buf) {  // one item's input span -> buffer buf (ndma 1-KiB DMAs)
    const int n = static_cast<int>(it / groups_per_img), grp = static_cast<int>(it - static_cast<long>(n) * groups_per_img);
    const long start = (static_cast<long>(n) * H + static_cast<long>(grp) * RG * S) * pitch;
    char *dst = sx0 + buf * XB;
    for (int q = wave; q < ndma; q += NWV) {
      const long off = start + q * 1024 + lane * 16;
      const uint32_t o = off < x_bytes ? static_cast<uint32_t>(off) : 0x80000000u;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rx, (lds_void *)(dst + q * 1024), 16, o, 0, 0, 0);
    }
  };
  const rsrc_t ry = __builtin_amdgcn_make_buffer_rsrc(y, (short)0, static_cast<int>(y_bytes), 0x00020000);
  long it = blockIdx.x;
  if (it < items) issue(it, 0);

  // weights, zero-padded to KP along k (they arrive row-padded to LP per kernel row)
  for (int e = tid; e < COUT * (KP / 8); e += NT) {
    const int co = e / (KP / 8), kc = e - co * (KP / 8);
    uint4 v = make_uint4(0, 0, 0, 0);
    if (kc * 8 < K) v = *reinterpret_cast<const uint4 *>(w + static_cast<long>(co) * K + kc * 8);
    *reinterpret_cast<uint4 *>(sw + co * WPB + kc * 16) = v;
  }
  float bv[CFH][4];
  const int ch = wave & 1, row = wave >> 1;  // co half, output row of the item
#pragma unroll
  for (int cf = 0; cf < CFH; ++cf)
#pragma unroll
    for (int j = 0; j < 4; ++j) bv[cf][j] = bias ? bias[(ch * CFH + cf) * 16 + 4 * g4 + j] : 0.f;
  const char *wrow = sw + (ch * CFH * 16 + l16) * WPB + 16 * g4;
  // the lane's k chunk of k-step s: byte offset in a span (pad chunks: offset 0, zero weights)
  auto tap = [&](int s) -> int {
    const int k = s * 32 + 8 * g4;
    const int kh = static_cast<int>(fdiv(static_cast<uint32_t>(k), fd_lp));
    return k < K ? kh * pitch + (k - kh * LP) * 2 : 0;
  };

  const int pxs = S * C * 2;  // bytes per output-pixel step in a staged row
  int pxo[4];                 // byte offset of this lane's pixel (column) in each of the wave's 4 fragments
#pragma unroll
  for (int pf = 0; pf < 4; ++pf) pxo[pf] = row * S * pitch + min(16 * pf + l16, Wo - 1) * pxs;
  int buf = 0;
  // this wave's epilogue stores of the previous item: every store instruction is issued (masked
  // stores go to an out-of-range offset), so the count is fixed and the wait below lets them
  // drain behind the next item's MFMAs (vector-memory operations retire in issue order)
  constexpr int NPASS = (16 * CFH * 2 + 63) / 64;
  const int npf = min(4, (Wo + 15) / 16);
  int nst = 0;
  for (; it < items; it += gridDim.x) {
    const int n = static_cast<int>(it / groups_per_img), grp = static_cast<int>(it - static_cast<long>(n) * groups_per_img);
    vm_wait(counted ? nst : 0);  // this item's span DMAs landed (only the last item's stores may be in flight)
    __syncthreads();  // ... for every wave; weights in; every wave done with the other buffer
    if (it + gridDim.x < items) issue(it + gridDim.x, buf ^ 1);
    const char *sx = sx0 + buf * XB;

    f32x4 acc[CFH][4];
#pragma unroll
    for (int cf = 0; cf < CFH; ++cf)
#pragma unroll
      for (int pf = 0; pf < 4; ++pf) acc[cf][pf] = f32x4{0.f, 0.f, 0.f, 0.f};
    // fragments of k-step s -> (a, b); the next step's reads are issued before this step's MFMAs
    auto load = [&](int s, bf16x8 (&a)[CFH], bf16x8 (&b)[4]) {
#pragma unroll
      for (int cf = 0; cf < CFH; ++cf) a[cf] = *reinterpret_cast<const bf16x8 *>(wrow + cf * 16 * WPB + s * 64);
      const char *p0 = sx + tap(s);
#pragma unroll
      for (int pf = 0; pf < 4; ++pf) {
        const uint2 lo = *reinterpret_cast<const uint2 *>(p0 + pxo[pf]);
        const uint2 hi = *reinterpret_cast<const uint2 *>(p0 + pxo[pf] + 8);
        b[pf] = __builtin_bit_cast(bf16x8, make_uint4(lo.x, lo.y, hi.x, hi.y));
      }
    };
    auto mma = [&](const bf16x8 (&a)[CFH], const bf16x8 (&b)[4]) {
#pragma unroll
      for (int pf = 0; pf < 4; ++pf)
#pragma unroll
        for (int cf = 0; cf < CFH; ++cf)
          acc[cf][pf] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[cf], b[pf], acc[cf][pf], 0, 0, 0);
    };
    bf16x8 a0[CFH], b0[4], a1[CFH], b1[4];
    load(0, a0, b0);
    for (int s = 0; s < KS; s += 2) {
      load(min(s + 1, KS - 1), a1, b1);
      mma(a0, b0);
      if (s + 1 >= KS) break;
      load(min(s + 2, KS - 1), a0, b0);
      mma(a1, b1);
    }
    __syncthreads();  // every wave is done reading the span: its buffer becomes epilogue staging

    // epilogue: per fragment, 16 pixels x (CFH*16) channels through this wave's staging rows
    constexpr int SPB = CFH * 32 + 16;  // staging row pitch (bytes)
    char *st = const_cast<char *>(sx) + wave * 16 * SPB;
    const int ho = grp * RG + row;
    nst = ho < Ho ? npf * NPASS : 0;
    if (ho < Ho) {  // wave-uniform
      const long yrow = (((static_cast<long>(n) * Ho + ho) * Wo) * static_cast<long>(ldc) + ch * CFH * 16) * 2;
#pragma unroll
      for (int pf = 0; pf < 4; ++pf) {
        const int col0 = 16 * pf;
        if (col0 >= Wo) break;  // wave-uniform
#pragma unroll
        for (int cf = 0; cf < CFH; ++cf) {
          float v[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            v[j] = acc[cf][pf][j] + bv[cf][j];
            if (relu) v[j] = fmaxf(v[j], 0.f);
          }
          *reinterpret_cast<uint2 *>(st + l16 * SPB + (cf * 16 + 4 * g4) * 2) =
              make_uint2(pack2(v[0], v[1]), pack2(v[2], v[3]));
        }
        wave_lds_handoff();
        constexpr int CH = CFH * 2;  // 16-byte chunks per pixel (of this wave's channels)
#pragma unroll
        for (int i = 0; i < NPASS; ++i) {
          const int c = min(lane + 64 * i, 16 * CH - 1);
          const int px = c / CH, part = c - px * CH;
          const int wo = col0 + px;
          const uint4 v = *reinterpret_cast<const uint4 *>(st + px * SPB + part * 16);
          const bool ok = lane + 64 * i < 16 * CH && wo < Wo;
          const uint32_t off = ok ? static_cast<uint32_t>(yrow + (static_cast<long>(wo) * ldc + part * 8) * 2) : 0x80000000u;
          typedef int v4i __attribute__((ext_vector_type(4)));
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4i, v), ry, off, 0, 0);
        }
        wave_lds_handoff();
      }
    }
    buf ^= 1;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// CXXNET_ROWRUN_COUNTED=0: drain every store of an item before the next one (s_waitcnt vmcnt(0))
static const int g_counted = [] {
  const char *e = getenv("CXXNET_ROWRUN_COUNTED");
  return e ? atoi(e) : 1;
}();

template <int CFH>
int launch(const bf16_t *x, long x_bytes, const bf16_t *w, const float *bias, bf16_t *y, int N, int H, int W, int C,
           int Ho, int Wo, int KH, int LP, int S, int ldc, int relu, hipStream_t s) {
  const long y_bytes = (static_cast<long>(N) * Ho * Wo * ldc) * 2;
  if (y_bytes >= (1L << 31)) return -1;
  const int K = KH * LP;
  const int KS = (K + 31) / 32;
  const int cout = 32 * CFH;
  const long span = static_cast<long>(S * (RG - 1) + KH) * W * C * 2 + 16;  // + the last run's pad reads
  const int ndma = static_cast<int>((span + 1023) / 1024);
  const int epi = (NT / 64) * 16 * (CFH * 32 + 16);  // epilogue staging reuses the item's buffer
  const int XB = (ndma * 1024 > epi ? ndma * 1024 : epi + 1023) / 1024 * 1024;
  const long lds = 2L * XB + static_cast<long>(cout) * (KS * 64 + 16);
  if (lds > 160 * 1024) return -1;
  static const hipError_t attr = hipFuncSetAttribute(reinterpret_cast<const void *>(conv_rowrun_fwd<CFH>),
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  if (attr != hipSuccess) return -1;  // once per instantiation (thread-safe static); -1: caller falls back
  const long items = static_cast<long>(N) * ((Ho + RG - 1) / RG);
  const int grid = static_cast<int>(items < 256 ? items : 256);
  CXN_LAUNCH(conv_rowrun_fwd<CFH>, dim3(grid), dim3(NT), static_cast<size_t>(lds), s, x, x_bytes, w, bias, y, y_bytes, N,
                     H, W, C, Ho, Wo, KH, LP, make_fastdiv(LP), S, ldc, relu, KS, XB, ndma, g_counted);
  return 0;
}


// (A direct weight-gradient over the staged kernel-row runs lived here until round 5: 169-189 us
// against the split-K GEMM's 159 on AlexNet conv1, profiles/r3_conv1_direct.md -- never shipped.)

}  // namespace

// x: NHWC [N][H][W][C] bf16 (pad 0; W is the row pitch in pixels, 8-byte aligned pixel steps);
// w: [Cout][KH][LP] bf16, each kernel row's KW*C run zero-padded to LP (% 8 == 0);
// y: [N][Ho][Wo] x ldc bf16.  Cout in {32, 64, 96, 128}, Wo <= 64.  -1: not served (GEMM path).
CXN_API int cxn_conv_rowrun_fwd(const void *x, long x_bytes, const void *w, const float *bias, void *y, int N, int H,
                                int W, int C, int Ho, int Wo, int Cout, int KH, int LP, int S, int ldc, int relu,
                                void *stream) {
  if (Cout % 32 || Cout > 128 || Wo > 64 || Wo < 1 || LP % 8 || ldc % 8 || ldc < Cout || S < 1) return -1;
  if ((S * C * 2) % 8 || (W * C * 2) % 8 || x_bytes >= (1L << 31)) return -1;
  if ((reinterpret_cast<uintptr_t>(y) & 15) || (reinterpret_cast<uintptr_t>(x) & 15) ||
      (reinterpret_cast<uintptr_t>(w) & 15) || (KH * LP) % 8)
    return -1;
  if ((Ho - 1) * S + KH > H) return -1;
  const bf16_t *xb = static_cast<const bf16_t *>(x);
  const bf16_t *wb = static_cast<const bf16_t *>(w);
  bf16_t *yb = static_cast<bf16_t *>(y);
  hipStream_t s = static_cast<hipStream_t>(stream);
  int rc = -1;
  switch (Cout / 32) {
    case 1: rc = launch<1>(xb, x_bytes, wb, bias, yb, N, H, W, C, Ho, Wo, KH, LP, S, ldc, relu, s); break;
    case 2: rc = launch<2>(xb, x_bytes, wb, bias, yb, N, H, W, C, Ho, Wo, KH, LP, S, ldc, relu, s); break;
    case 3: rc = launch<3>(xb, x_bytes, wb, bias, yb, N, H, W, C, Ho, Wo, KH, LP, S, ldc, relu, s); break;
    case 4: rc = launch<4>(xb, x_bytes, wb, bias, yb, N, H, W, C, Ho, Wo, KH, LP, S, ldc, relu, s); break;
    default: return -1;
  }
  if (rc != 0) return rc;
  return hipGetLastError() == hipSuccess ? 0 : -3;
}

