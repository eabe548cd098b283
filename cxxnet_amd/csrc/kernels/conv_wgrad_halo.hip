// Direct 3x3 / stride-1 convolution WEIGHT gradient on resident LDS tiles (tiles 140-142), gfx950:
// dW[co][kh][kw][ci] += sum over pixels of dy[p][co] * x[p + (kh, kw) - pad][ci] for VGG-16's
// 3x3 layers.  Reference: src/layer/convolution_layer-inl.hpp:134-138 (im2col + gemm into gwmat).
//
// Why.  The split-K implicit GEMM (gemm_mfma.hip GATHER_MN x DIRECT_MN) rebuilds every pixel's
// im2col address per 16-byte load: at VGG conv3_2 it issues 3.7 VALU (and 1.2 SALU) per MFMA,
// and with two waves per SIMD the VALU issue port, not the matrix core, sets the pace -- 805
// TFLOP/s on conv3_2, 492 on conv1_2 (profiles/r4_wgrad_halo_probe.md).  Here a block owns one
// (64 output channels x 64 input channels) pair and streams 128-pixel patches through LDS:
//   * per patch two DMA sets with per-lane offsets fixed for the whole kernel (a few VALU per
//     patch): the input halo ((128/WT + 2) rows x (WT + 2) pixels x 64 channels) and the dy tile
//     (128 pixels x 64 channels); the nine taps are nine shifted windows of the same halo;
//   * K = pixels: a K-step is 32 pixels (one 32-wide patch row, or two 16-wide rows), 4 per
//     patch.  Both operands are pixel-major in LDS, so fragments are ds_read_b64_tr_b16 pairs;
//     every 128-byte pixel slot keeps its four 32-byte channel units XOR-permuted by bits 1-3
//     of the slot (key ((s >> 1) ^ ((s >> 3) << 1)) & 3, halo rows a multiple of 16 slots): the
//     8 slots a 32-lane half reads ({k..k+3, k+8..k+11} for any k) then land in 8 distinct bank
//     groups, and a tap shift moves a read by an immediate only;
//   * 4 waves (one per SIMD), wave w owns input channels 16w..16w+15 of the pair: per K-step
//     it reads 4 dy fragments and 9 halo fragments (one per tap) and issues 36 MFMAs into
//     4 x 9 accumulators pinned in AGPRs (144 registers) that live across all its patches;
//   * double-buffered: the next patch's 46 DMAs are issued (12 per wave, inline asm: see dma16w)
//     as a patch starts, one barrier per patch, at its end; fragment reads of K-step r + 1 ride on
//     the MFMAs of K-step r;
//   * persistent split over pixels: (pairs x splits) ~ one block per CU, consecutive blocks
//     (one XCD) share a pixel range so its x / dy bytes are fetched into that XCD's L2 once;
//   * epilogue: one fp32 atomic per accumulator element (the split-K kernels do the same).
#include "gemm_glds_common.h"

using namespace cxg;

namespace {

// One 1-KiB LDS-DMA (16 bytes per lane) as inline asm.  With the builtin, hipcc cannot tell the
// next patch's LDS bytes from the ones the current patch's ds_reads touch and puts a vmcnt(0)
// before the first ds_read after the DMAs: every patch then waited for all of the next patch's
// HBM loads at its first K-step instead of letting them land under its 144 MFMAs.  Completion
// is counted by hand (wait_vmcnt + barrier at the patch end).  M0 is saved and restored inside
// the statement (compiler-reserved).
__device__ __forceinline__ void dma16w(rsrc_t r, uint32_t lds_addr, uint32_t voff) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(voff), "s"(r), "s"(lds_addr) : "memory");
}

template <int N>
__device__ __forceinline__ void wait_lgkm_w() {
  asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(N) : "memory");
}

__device__ __forceinline__ void mfma_w(f32x4 &acc, const bf16x8 &a, const bf16x8 &b) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
}

// 32-byte unit permutation key of pixel slot s (bits 1-3 of s)
__host__ __device__ constexpr int wg_key(int s) { return ((s >> 1) ^ ((s >> 3) << 1)) & 3; }

// two transposed 8-byte reads (k-rows k and k + 4) -> one 16x16x32 operand fragment
__device__ __forceinline__ bf16x8 frag_tr(const char *p0, const char *p1) {
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4 *)(p0));
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4 *)(p1));
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  const s16x8 r = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, r);
}

template <int WT>
struct WgCfg {
  static constexpr int PR = 128 / WT;           // patch rows (4 or 8)
  static constexpr int KS = 4;                  // 32-pixel K-steps per patch
  static constexpr int P = WT == 32 ? 48 : 32;  // halo row pitch in slots (multiple of 16)
  static constexpr int CGR = (WT + 2 + 7) / 8;  // 8-slot DMA groups per halo row
  static constexpr int NGH = (PR + 2) * CGR;    // halo DMA groups
  static constexpr int HALO = (PR + 2) * P * 128;
  static constexpr int BUF = HALO + 128 * 128;  // halo + dy tile
  static constexpr int NG = NGH + 16;           // DMA groups per patch
  static constexpr int ND = (NG + 3) / 4;       // per wave
  static constexpr int NB = 2;  // patch buffers (three, with the barrier moved to the last K-step
                                // and the next patch's first reads riding on it: 3-4% slower,
                                // profiles/r4_wgrad_halo_probe.md)
  static constexpr int LDS = NB * BUF;
  static_assert(ND == 12 && NGH <= 32, "eight halo + four dy DMAs per wave");
  static_assert(LDS <= 160 * 1024, "LDS");
};

template <int WT>
__global__ void __launch_bounds__(256, 1)
conv_wgrad_halo(GOperand X, GOperand D, GEpi E, int npairs, int ncib, int per, int tiles_w, int tiles_h,
                int npatch) {
  using Cf = WgCfg<WT>;
  constexpr int P = Cf::P, KS = Cf::KS, ND = Cf::ND, NGH = Cf::NGH, BUF = Cf::BUF, NB = Cf::NB;
  __shared__ __attribute__((aligned(1024))) char smem[Cf::LDS];

  const uint32_t L = xcd_remap(blockIdx.x, gridDim.x);
  const int pair = static_cast<int>(L % static_cast<uint32_t>(npairs));
  const int split = static_cast<int>(L / static_cast<uint32_t>(npairs));
  const int cob = pair / ncib, cib = pair - cob * ncib;  // 64-channel output / input blocks
  const int pbeg = split * per, pend = min(npatch, pbeg + per);
  if (pbeg >= pend) return;  // whole block

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int l16 = lane & 15, g4 = lane >> 4;
  const int Hx = X.H, Wx = X.W, Ho = X.Ho, Wo = X.Wo;
  const rsrc_t rx = make_rsrc(X.ptr, X.nbytes), rd = make_rsrc(D.ptr, D.nbytes);
  const uint32_t xpb = static_cast<uint32_t>(X.C) * 2u, dpb = static_cast<uint32_t>(D.ld) * 2u;
  const uint32_t lds0 = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(reinterpret_cast<uintptr_t>((lds_void *)smem)));

  // this wave's DMA slots s: s < 8 halo group G = wave + 4 s (G < NGH), s >= 8 dy group
  // q = wave + 4 (s - 8).  Per lane only the column and the swizzled chunk offset are kept;
  // the group's row and LDS destination are recomputed in scalar registers at issue.
  int dcol[ND];
  uint32_t loff[ND];
#pragma unroll
  for (int s = 0; s < ND; ++s) {
    const int pc = lane & 7;
    int slot16, chan;
    if (s < 8) {
      const int G = wave + 4 * s;
      const int hr = G / Cf::CGR, cg = G - hr * Cf::CGR;
      const int col = 8 * cg + (lane >> 3);
      dcol[s] = col < WT + 2 ? col - X.pad_w : (1 << 24);
      slot16 = col & 15;
      chan = cib * 128;
    } else {
      const int px = 8 * (wave + 4 * (s - 8)) + (lane >> 3);
      dcol[s] = px % WT;
      slot16 = px & 15;
      chan = cob * 128;
    }
    loff[s] = static_cast<uint32_t>(chan + 16 * (2 * ((pc >> 1) ^ wg_key(slot16)) + (pc & 1)));
  }
  // patch p -> image and output origin
  auto decode = [&](int p, int &img, int &r0, int &c0) __attribute__((always_inline)) {
    const int tw = p % tiles_w, t2 = p / tiles_w;
    const int th = t2 % tiles_h;
    img = t2 / tiles_h;
    r0 = th * Cf::PR;
    c0 = tw * WT;
  };
  auto issue = [&](auto sc, int b, int img, int r0, int c0) __attribute__((always_inline)) {
    constexpr int s = decltype(sc)::value;
    int drow, dst, HH, WW;
    uint32_t pb;
    rsrc_t rs;
    if constexpr (s < 8) {
      const int G = wave + 4 * s;
      if (G >= NGH) return;
      const int hr = G / Cf::CGR, cg = G - hr * Cf::CGR;
      drow = hr - X.pad_h;
      dst = (hr * P + 8 * cg) * 128;
      HH = Hx; WW = Wx; pb = xpb; rs = rx;
    } else {
      const int q = wave + 4 * (s - 8);
      drow = (8 * q) / WT;
      dst = Cf::HALO + q * 1024;
      HH = Ho; WW = Wo; pb = dpb; rs = rd;
    }
    const int gr = r0 + drow, gc = c0 + dcol[s];
    const bool ok = static_cast<unsigned>(gr) < static_cast<unsigned>(HH) && static_cast<unsigned>(gc) < static_cast<unsigned>(WW);
    const uint32_t pix = static_cast<uint32_t>((img * HH + gr) * WW + gc);
    dma16w(rs, lds0 + static_cast<uint32_t>(b * BUF + dst), ok ? pix * pb + loff[s] : OOB);
  };

  // fragment read bases (bytes) per buffer: lane (l16, g4) reads k-rows pk and pk + 4
  int offA[NB][4][2], offB[NB][3][2];
#pragma unroll
  for (int hl = 0; hl < 2; ++hl) {
    const int pk = 8 * g4 + (l16 >> 2) + 4 * hl;
#pragma unroll
    for (int b = 0; b < NB; ++b) {
#pragma unroll
      for (int m = 0; m < 4; ++m) offA[b][m][hl] = b * BUF + Cf::HALO + pk * 128 + ((m ^ wg_key(pk)) << 5) + 8 * (l16 & 3);
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
        const int col = kw + (WT == 32 ? pk : (pk & 15));
        const int rowoff = WT == 32 ? 0 : (pk >> 4) * P;
        offB[b][kw][hl] = b * BUF + (rowoff + col) * 128 + ((wave ^ wg_key(col)) << 5) + 8 * (l16 & 3);
      }
    }
  }

  f32x4 acc[4][9];
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int t = 0; t < 9; ++t) acc[m][t] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 fa[2][4], fb[2][9];

  // fragment f (< 4: dy block f; else tap f - 4) of K-step r from buffer b into set `set`
  auto read = [&](int set, int f, int b, int r) __attribute__((always_inline)) {
    if (f < 4) {
      fa[set][f] = frag_tr(smem + offA[b][f][0] + r * 4096, smem + offA[b][f][1] + r * 4096);
    } else {
      const int t = f - 4, kh = t / 3, kw = t % 3;
      const int rr = (WT == 32 ? r : 2 * r) + kh;
      fb[set][t] = frag_tr(smem + offB[b][kw][0] + rr * P * 128, smem + offB[b][kw][1] + rr * P * 128);
    }
  };

  // prologue: the first patch
  {
    int img, r0, c0;
    decode(pbeg, img, r0, c0);
    static_for<ND>([&](auto sc) { issue(sc, 0, img, r0, c0); });
  }
  wait_vmcnt<0>();
  block_barrier();
#pragma unroll
  for (int f = 0; f < 13; ++f) read(0, f, 0, 0);
  __builtin_amdgcn_sched_barrier(0);

  // Patch p from buffer B (landed; its K-step-0 fragments are being read).  Its first K-step
  // issues all DMAs of patch p + 1 into buffer B ^ 1 (a whole patch to land under); the barrier
  // at its end publishes them and retires buffer B.
  auto patch = [&](auto bc, int p) __attribute__((always_inline)) {
    constexpr int B = decltype(bc)::value;
    const bool next = p + 1 < pend;
    int img = 0, r0 = 0, c0 = 0;
    if (next) decode(p + 1, img, r0, c0);
    static_for<KS>([&](auto rc) {
      constexpr int r = decltype(rc)::value;
      constexpr int cur = r & 1, nxt = cur ^ 1;
      wait_lgkm_w<0>();
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (r == 0) {
        if (next) static_for<ND>([&](auto sc) { issue(sc, B ^ 1, img, r0, c0); });
      }
      __builtin_amdgcn_sched_barrier(0);
      static_for<36>([&](auto uc) {
        constexpr int u = decltype(uc)::value;
        mfma_w(acc[u / 9][u % 9], fa[cur][u / 9], fb[cur][u % 9]);
        if constexpr (r + 1 < KS) {
          static_for<13>([&](auto jc) {
            constexpr int j = decltype(jc)::value;
            if constexpr ((j * 36) / 13 == u) read(nxt, j, B, r + 1);
          });
        }
        __builtin_amdgcn_sched_barrier(0);
      });
    });
    wait_vmcnt<0>();
    block_barrier();
    if (next) {
#pragma unroll
      for (int f = 0; f < 13; ++f) read(0, f, B ^ 1, 0);
    }
    __builtin_amdgcn_sched_barrier(0);
  };
  static_assert(KS % 2 == 0, "K-step 0 of every patch reads fragment set 0");
  // straight-line pairs (a conditional second patch would merge the accumulators through a
  // phi: ~140 AGPR copies per iteration), the odd last patch after the loop
  int p = pbeg;
  for (; p + 1 < pend; p += 2) {
    patch(std::integral_constant<int, 0>{}, p);
    patch(std::integral_constant<int, 1>{}, p + 1);
  }
  if (p < pend) patch(std::integral_constant<int, 0>{}, p);
  asm volatile("s_nop 15\n\ts_nop 15\n\ts_nop 15" ::: "memory");  // inline-asm MFMA results

  // acc[m][t] lane (l16, g4) element j: output channel 64 cob + 16 m + 4 g4 + j, tap t, input
  // channel 64 cib + 16 wave + l16
  float *out = static_cast<float *>(E.out);
  const int Cin = X.Cg;
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const long co = 64 * cob + 16 * m + 4 * g4 + j;
        atomicAdd(out + co * E.ldc + t * Cin + 64 * cib + 16 * wave + l16, acc[m][t][j] * E.alpha);
      }
}

int num_cu() {
  static const int n = [] {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0)
      v = 256;
    return v;
  }();
  return n;
}

template <int WT>
int launch_wg(const GOperand &X, const GOperand &D, const GEpi &E, hipStream_t s) {
  using Cf = WgCfg<WT>;
  const long hw = static_cast<long>(X.Ho) * X.Wo;
  const long N = X.kdim / hw;
  const int tiles_w = cdiv(X.Wo, WT), tiles_h = cdiv(X.Ho, Cf::PR);
  const long npatch = N * tiles_w * tiles_h;
  if (npatch >= (1L << 30)) return -1;
  const int ncib = X.Cg / 64, npairs = (D.rows / 64) * ncib;
  long nsplit = num_cu() / npairs;
  nsplit = nsplit < 1 ? 1 : (nsplit > npatch ? npatch : nsplit);
  const int per = cdiv(npatch, nsplit);
  nsplit = cdiv(npatch, per);
  CXN_LAUNCH((conv_wgrad_halo<WT>), dim3(static_cast<unsigned>(npairs * nsplit)), dim3(256), 0, s, X, D, E, npairs, ncib,
             per, tiles_w, tiles_h, static_cast<int>(npatch));
  return 0;
}

// share of computed pixels that are real output pixels for a patch width
double wg_util(int Ho, int Wo, int wt) {
  const int pr = 128 / wt;
  return static_cast<double>(Ho) * Wo / (static_cast<double>(cdiv(Ho, pr)) * pr * cdiv(Wo, wt) * wt);
}

}  // namespace

namespace cxg {
// 140: patch width chosen by pixel utilisation (32, or 16 when that wastes fewer), 141: 16,
// 142: 32.  Operands are those of the implicit-GEMM weight-gradient (A: MN_GATHER of the NHWC
// input x, rows 9 Cg; B: MN_DIRECT dy, rows Cout; fp32 atomic epilogue into dW [Cout][9 Cg]);
// served: one group, 3 x 3, stride 1, same-size output (any pad: x may be pre-padded), Cg and
// Cout multiples of 64.  -1 otherwise (the caller falls back).
int dispatch_wgrad_halo(int amode, int bmode, int epi, int tile, const GOperand &A, const GOperand &B, const GEpi &E,
                        int groups, hipStream_t s) {
  if (amode != MN_GATHER || bmode != MN_DIRECT || epi != EPI_F32_ATOMIC || groups != 1) return -1;
  if (A.KH != 3 || A.KW != 3 || A.stride != 1 || A.rows != 9 * A.Cg) return -1;
  if (A.Cg % 64 != 0 || B.rows % 64 != 0) return -1;
  if (A.H + 2 * A.pad_h != A.Ho + 2 || A.W + 2 * A.pad_w != A.Wo + 2 || A.pad_h > 2 || A.pad_w > 2) return -1;
  if (A.C % 8 != 0 || A.C < A.Cg || B.ld % 8 != 0 || B.ld < B.rows) return -1;
  const long hw = static_cast<long>(A.Ho) * A.Wo;
  if (hw <= 0 || A.kdim != B.kdim || A.kdim % hw != 0 || E.ldc < A.rows) return -1;
  int wt = 32;
  if (tile == 141) wt = 16;
  else if (tile == 140 && wg_util(A.Ho, A.Wo, 16) > wg_util(A.Ho, A.Wo, 32) + 1e-9) wt = 16;
  else if (tile != 140 && tile != 142) return -1;
  return wt == 16 ? launch_wg<16>(A, B, E, s) : launch_wg<32>(A, B, E, s);
}
}  // namespace cxg
