// Few-channel first-layer convolution forward (4-channel NHWC input, 8-byte pixels) for gfx950:
// VGG conv1_1 (3x3 / 1, pad 1), GoogLeNet conv1 (7x7 / 2, pad 3) -- reference
// src/layer/convolution_layer-inl.hpp:70-105 (im2col + GEMM per group).
//
// Why a kernel of its own: with 4 input channels the GEMM's K is tiny (36 / 196) and its
// output is wide (64 channels x every pixel), so the op is bound by writing y (VGG c1_1: 411 MB
// at batch 64) and by the per-tile fixed costs of the general LDS-DMA GEMM (one K-tile of
// loads, then a long epilogue, at one 128 KiB block per CU).  Here:
//   * a block stages the weights ONCE ([Cout][Kpad] bf16 in LDS) and then walks output rows
//     (persistent grid): per row it stages only the KH input rows it needs (KH x Wp pixels x
//     8 B, zero-padded borders, 5-13 KiB), so LDS stays small and 3-6 blocks share a CU --
//     one block's stores overlap another's loads and MFMAs;
//   * MFMA v_mfma_f32_16x16x32_bf16 with rows = output channels (A = weights from LDS,
//     ds_read_b128) and columns = 16 output pixels (B = two 4-channel taps per lane, gathered
//     from the staged rows with ds_read_b64 through a per-k-step tap table); each wave owns
//     up to 4 pixel columns of the row (64 pixels) and every output channel;
//   * epilogue: bias + relu in fp32, bf16, written through a per-wave LDS transpose so each
//     pixel's Cout channels leave as whole 16-byte chunks (a wave stores 16 pixels x Cout*2 B
//     per instruction pair instead of 8-byte pieces 128 B apart).
#include "common.h"

namespace {

constexpr int NT = 256;  // 4 waves

__device__ __forceinline__ void lds_handoff() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
}

// y[n][ho][wo][co] (row stride ldc) = relu?(bias[co] + sum_{ky,kx,c} w[co][ky][kx][c] x[n][ho*S-P+ky][wo*S-P+kx][c])
template <int CF>  // output channels / 16
__global__ void __launch_bounds__(NT) conv_fewc_fwd(const bf16_t *__restrict__ x, const bf16_t *__restrict__ w,
                                                    const float *__restrict__ bias, bf16_t *__restrict__ y, int N,
                                                    int H, int W, int Ho, int Wo, int KH, int KW, int S, int P,
                                                    int ldc, int relu, int KS) {
  constexpr int COUT = CF * 16;
  constexpr int SP = COUT * 2 + 16;  // epilogue staging row pitch (bytes): 16 B pad against bank conflicts
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int K = KH * KW * 4;
  const int KP = KS * 32;
  const int WP = KP * 2 + 16;         // weight row pitch (bytes)
  const int Wp = (Wo - 1) * S + KW;   // staged input row width (pixels)
  char *sw = smem;                                    // [COUT][WP]
  int *stap = reinterpret_cast<int *>(sw + COUT * WP);  // [KS * 8] tap byte offsets (-1: zero tap)
  char *sx = reinterpret_cast<char *>(stap + KS * 8);  // [KH][Wp] pixels x 8 B
  char *se = sx + ((KH * Wp * 8 + 15) & ~15);          // [4 waves][16][SP]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;

  // weights, zero-padded to KP along k; the tap table
  for (int e = tid; e < COUT * (KP / 4); e += NT) {  // one 4-channel tap (8 B) per element
    const int co = e / (KP / 4), kc = e - co * (KP / 4);
    uint2 v = make_uint2(0, 0);
    if (kc * 4 < K) v = *reinterpret_cast<const uint2 *>(w + static_cast<long>(co) * K + kc * 4);
    *reinterpret_cast<uint2 *>(sw + co * WP + kc * 8) = v;
  }
  for (int t = tid; t < KS * 8; t += NT) {
    const int ky = t / KW, kx = t - ky * KW;
    stap[t] = t < KH * KW ? (ky * Wp + kx) * 8 : -1;
  }
  float bv[CF][4];
#pragma unroll
  for (int cf = 0; cf < CF; ++cf)
#pragma unroll
    for (int j = 0; j < 4; ++j) bv[cf][j] = bias ? bias[cf * 16 + 4 * (lane >> 4) + j] : 0.f;

  const int nfr = (Wo + 15) / 16;          // 16-pixel columns of an output row
  const int passes = (nfr + 15) / 16;      // 4 waves x 4 columns per pass
  const long rows = static_cast<long>(N) * Ho;
  for (long r = blockIdx.x; r < rows; r += gridDim.x) {
    const int n = static_cast<int>(r / Ho), ho = static_cast<int>(r - static_cast<long>(n) * Ho);
    __syncthreads();  // previous row's readers of sx are done (and the weights / taps are in)
    // stage KH input rows, zero outside the image
    const int h0 = ho * S - P;
    for (int e = tid; e < KH * Wp; e += NT) {
      const int ky = e / Wp, c = e - ky * Wp;
      const int hi = h0 + ky, wi = c - P;
      uint2 v = make_uint2(0, 0);
      if (hi >= 0 && hi < H && wi >= 0 && wi < W)
        v = *reinterpret_cast<const uint2 *>(x + ((static_cast<long>(n) * H + hi) * W + wi) * 4);
      *reinterpret_cast<uint2 *>(sx + e * 8) = v;
    }
    __syncthreads();
    for (int pass = 0; pass < passes; ++pass) {
      f32x4 acc[CF][4];
#pragma unroll
      for (int cf = 0; cf < CF; ++cf)
#pragma unroll
        for (int pf = 0; pf < 4; ++pf) acc[cf][pf] = f32x4{0.f, 0.f, 0.f, 0.f};
      // this lane's pixel in each of the wave's columns (clamped: columns past Wo compute
      // garbage that is never stored)
      int pxo[4];
#pragma unroll
      for (int pf = 0; pf < 4; ++pf) {
        const int wo = min(16 * (pass * 16 + pf * 4 + wave) + (lane & 15), Wo - 1);
        pxo[pf] = wo * S * 8;
      }
      for (int s = 0; s < KS; ++s) {
        bf16x8 a[CF];
#pragma unroll
        for (int cf = 0; cf < CF; ++cf)
          a[cf] = *reinterpret_cast<const bf16x8 *>(sw + (cf * 16 + (lane & 15)) * WP + (s * 32 + 8 * (lane >> 4)) * 2);
        const int t0 = stap[s * 8 + 2 * (lane >> 4)], t1 = stap[s * 8 + 2 * (lane >> 4) + 1];
#pragma unroll
        for (int pf = 0; pf < 4; ++pf) {
          uint2 lo = make_uint2(0, 0), hi = make_uint2(0, 0);
          if (t0 >= 0) lo = *reinterpret_cast<const uint2 *>(sx + t0 + pxo[pf]);
          if (t1 >= 0) hi = *reinterpret_cast<const uint2 *>(sx + t1 + pxo[pf]);
          const uint4 q = make_uint4(lo.x, lo.y, hi.x, hi.y);
          const bf16x8 b = __builtin_bit_cast(bf16x8, q);
#pragma unroll
          for (int cf = 0; cf < CF; ++cf)
            acc[cf][pf] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[cf], b, acc[cf][pf], 0, 0, 0);
        }
      }
      // epilogue: per column, transpose through this wave's staging rows, 16-byte stores
      char *st = se + wave * 16 * SP;
      bf16_t *yrow = y + (static_cast<long>(n) * Ho + ho) * static_cast<long>(Wo) * ldc;
#pragma unroll
      for (int pf = 0; pf < 4; ++pf) {
        const int col0 = 16 * (pass * 16 + pf * 4 + wave);
        if (col0 >= Wo) break;  // wave-uniform
#pragma unroll
        for (int cf = 0; cf < CF; ++cf) {
          float v[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            v[j] = acc[cf][pf][j] + bv[cf][j];
            if (relu) v[j] = fmaxf(v[j], 0.f);
          }
          *reinterpret_cast<uint2 *>(st + (lane & 15) * SP + (cf * 16 + 4 * (lane >> 4)) * 2) =
              make_uint2(pack2(v[0], v[1]), pack2(v[2], v[3]));
        }
        lds_handoff();
        constexpr int CH = COUT / 8;  // 16-byte chunks per pixel
#pragma unroll
        for (int i = 0; i < (16 * CH + 63) / 64; ++i) {
          const int c = lane + 64 * i;
          if (c < 16 * CH) {
            const int px = c / CH, part = c - px * CH;
            const int wo = col0 + px;
            const uint4 v = *reinterpret_cast<const uint4 *>(st + px * SP + part * 16);
            if (wo < Wo) *reinterpret_cast<uint4 *>(yrow + static_cast<long>(wo) * ldc + part * 8) = v;
          }
        }
        lds_handoff();  // staging rows are rewritten by the next column
      }
    }
  }
}

template <int CF>
int launch(const bf16_t *x, const bf16_t *w, const float *bias, bf16_t *y, int N, int H, int W, int Ho, int Wo, int KH,
           int KW, int S, int P, int ldc, int relu, hipStream_t s) {
  const int K = KH * KW * 4;
  const int KS = (K + 31) / 32;
  const int Wp = (Wo - 1) * S + KW;
  const size_t lds = static_cast<size_t>(CF * 16) * (KS * 64 + 16) + KS * 8 * 4 + ((KH * Wp * 8 + 15) & ~15) +
                     4 * 16 * (CF * 32 + 16);
  if (lds > 96 * 1024) return -1;
  // once per instantiation (a thread-safe function-local static); if the attribute cannot be
  // set, decline (-1) so the caller runs the GEMM instead of failing the launch
  static const hipError_t attr = hipFuncSetAttribute(reinterpret_cast<const void *>(conv_fewc_fwd<CF>),
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024);
  if (attr != hipSuccess) return -1;
  const long rows = static_cast<long>(N) * Ho;
  // persistent: enough blocks for ~4 per CU, each walking output rows
  const int per_cu = lds <= 24 * 1024 ? 6 : lds <= 40 * 1024 ? 4 : lds <= 52 * 1024 ? 3 : 2;
  const long want = 256L * per_cu;
  const int grid = static_cast<int>(rows < want ? rows : want);
  CXN_LAUNCH(conv_fewc_fwd<CF>, dim3(grid), dim3(NT), lds, s, x, w, bias, y, N, H, W, Ho, Wo, KH, KW, S, P,
                     ldc, relu, KS);
  return 0;
}

}  // namespace

#define S_ static_cast<hipStream_t>(stream)

// 4-channel NHWC x (8-byte pixels, 8-byte aligned), w [Cout][KH][KW][4], Cout in {16, 32, 48, 64, 96,
// 128}, ldc % 8 == 0 (16-byte aligned output rows).  -1: shape not served (caller uses the GEMM).
CXN_API int cxn_conv_fewc_fwd(const void *x, const void *w, const float *bias, void *y, int N, int H, int W, int Ho,
                              int Wo, int Cout, int KH, int KW, int S, int P, int ldc, int relu, void *stream) {
  if (ldc % 8 || Cout % 16 || Cout > 128 || KH * KW * 4 > 256 || ldc < Cout || P < 0 || S < 1) return -1;
  if ((reinterpret_cast<uintptr_t>(y) & 15) || (reinterpret_cast<uintptr_t>(x) & 7)) return -1;
  const bf16_t *xb = static_cast<const bf16_t *>(x);
  const bf16_t *wb = static_cast<const bf16_t *>(w);
  bf16_t *yb = static_cast<bf16_t *>(y);
  int rc = -1;
  switch (Cout / 16) {
    case 1: rc = launch<1>(xb, wb, bias, yb, N, H, W, Ho, Wo, KH, KW, S, P, ldc, relu, S_); break;
    case 2: rc = launch<2>(xb, wb, bias, yb, N, H, W, Ho, Wo, KH, KW, S, P, ldc, relu, S_); break;
    case 3: rc = launch<3>(xb, wb, bias, yb, N, H, W, Ho, Wo, KH, KW, S, P, ldc, relu, S_); break;
    case 4: rc = launch<4>(xb, wb, bias, yb, N, H, W, Ho, Wo, KH, KW, S, P, ldc, relu, S_); break;
    case 6: rc = launch<6>(xb, wb, bias, yb, N, H, W, Ho, Wo, KH, KW, S, P, ldc, relu, S_); break;
    case 8: rc = launch<8>(xb, wb, bias, yb, N, H, W, Ho, Wo, KH, KW, S, P, ldc, relu, S_); break;
    default: return -1;
  }
  if (rc != 0) return rc;
  return hipGetLastError() == hipSuccess ? 0 : -3;
}
