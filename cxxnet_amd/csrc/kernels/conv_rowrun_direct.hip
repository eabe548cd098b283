// Direct kernels for few-channel, strided first layers on kernel-row runs, gfx950: the weight
// gradient (conv_wgrad_rowrun) and the forward (conv_rowrun_fwd2).  Instances: AlexNet conv1
// (3 channels on 228-pixel rows, 11 x 11 / 4, pad 0, 96 outputs) and GoogLeNet conv1 (4-channel
// NHWC, 224 x 224, 7 x 7 / 2, pad 3, 64 outputs).  Reference: src/layer/convolution_layer-inl.hpp
// :70-105 (forward: im2col + GEMM per group) and :121-138 (weight gradient: im2col + GEMM into
// gwmat).
//
// Shared idea: for one output pixel the KW C input values of kernel row kh are CONTIGUOUS in
// the input row (2 S C bytes per output pixel), so im2col columns are read straight out of staged
// input rows with per-lane addresses  row(S oy_local + kh) + RUN0 + 2 S C ox + 8 j4  (j4: 4-element
// chunk of the run; runs padded to NCH chunks, pad elements meet zero weights or are dropped).  A
// work item is RG output rows of one image; its S (RG - 1) + KH input rows land by LDS-DMA in a
// double buffer while the previous item computes:
//   * pad 0 (AlexNet): the rows are ONE contiguous span of x, staged as is;
//   * pad > 0 (4 channels = 8 bytes per pixel, so a 16-byte DMA unit is two whole pixels): each
//     staged row gets LPX zero pixels in front and zeros behind, rows above / below the image are
//     zeros -- per-lane source offsets from a fixed table, validity checked per item.
// The item's RG Wo pixels form one flattened GEMM dimension and the (kh, chunk) pairs another, so
// the MFMA waste is 17 % for AlexNet (220 of 224 pixels, 99 chunks for 363 columns) instead of
// the 44 % of one 64-pixel row per wave with 40-element row-padded runs.
#include "direct_common.h"

using namespace cxg;
using namespace cxd;

namespace {

template <int KH_, int KW_, int C_, int S_, int PAD_, int W_, int WO_, int COUT_, int RG_>
struct RGeo {
  static constexpr int KH = KH_, KW = KW_, C = C_, S = S_, PAD = PAD_, W = W_, WO = WO_, COUT = COUT_, RG = RG_;
  static constexpr int SROWB = W * C * 2;                                   // source row bytes
  static constexpr int LPX = PAD == 0 ? 0 : (PAD + 1) / 2 * 2;             // staged zero pixels in front
  static constexpr int LW = PAD == 0 ? W : (LPX + W + PAD + 1) / 2 * 2;     // staged row pixels
  static constexpr int ROWB = LW * C * 2;                                   // staged row bytes
  static constexpr int RUN0 = (LPX - PAD) * C * 2;                          // output pixel 0's run
  static constexpr int XROWS = S * (RG - 1) + KH;                           // input rows per item
  static constexpr int NXQ = (XROWS * ROWB + 1023) / 1024, XB = NXQ * 1024;  // x DMA pieces, bytes
  static constexpr int PIX = RG * WO;                                       // output pixels per item
  static constexpr int NCH = (KW * C + 3) / 4, NCHK = KH * NCH;             // run chunks: per row, all
  static constexpr int MT = COUT / 16, MTW = MT / 2;                        // 16-channel tiles (per wave)
  static_assert(COUT % 32 == 0 && SROWB % 8 == 0 && (S * C * 2) % 8 == 0 && RUN0 % 8 == 0, "alignment");
  static_assert(PAD == 0 || (C * 2 == 8 && W % 2 == 0), "padded staging: two whole pixels per 16-byte unit");
  static_assert(RUN0 + S * C * 2 * (WO - 1) + 8 * NCH <= ROWB, "runs stay inside a staged row");
};

// x staging of one item.  vx[i]: pad 0 -- byte offset 1024 q + 16 lane of the span (piece q =
// wave + 8 i); pad > 0 -- the lane's source offset relative to image row 0 of the item's first
// row (-1: a pad column), xr[i]: its staged row.  offset(i) adds the item's first row.
template <class G, int NQW>
struct XStage {
  int vx[NQW], xr[NQW];
  __device__ __forceinline__ void init(int wave, int lane, int nxq) {
#pragma unroll
    for (int i = 0; i < NQW; ++i) {
      const int q = wave + 8 * i, b = 1024 * q + 16 * lane;
      if constexpr (G::PAD == 0) {
        vx[i] = b;
        xr[i] = 0;
      } else {
        const int rr = b / G::ROWB, px = (b - rr * G::ROWB) / (G::C * 2), spx = px - G::LPX;
        const bool ok = q < nxq && rr < G::XROWS && spx >= 0 && spx < G::W;
        vx[i] = ok ? (rr * G::W + spx) * G::C * 2 : -1;
        xr[i] = rr;
      }
    }
  }
  // the item's descriptor (pad 0: its span; else image n) and first input row (may be < 0)
  __device__ __forceinline__ rsrc_t rsrc(const bf16_t *x, int H, int n, int oy0, int &row0) const {
    row0 = G::S * oy0 - G::PAD;
    if constexpr (G::PAD == 0) {
      const long xrow = static_cast<long>(n) * H + row0;
      return make_rsrc(reinterpret_cast<const char *>(x) + xrow * G::SROWB, static_cast<uint32_t>((H - row0) * G::SROWB));
    } else {
      return make_rsrc(reinterpret_cast<const char *>(x) + static_cast<long>(n) * H * G::SROWB,
                       static_cast<uint32_t>(H * G::SROWB));
    }
  }
  __device__ __forceinline__ uint32_t offset(int i, int row0, int H) const {
    if constexpr (G::PAD == 0) {
      return static_cast<uint32_t>(vx[i]);
    } else {
      const int row = row0 + xr[i];
      return (vx[i] >= 0 && row >= 0 && row < H) ? static_cast<uint32_t>(vx[i] + row0 * G::SROWB) : OOB;
    }
  }
};

// dy staging rotation: pixel p's 16-byte channel chunks are stored rotated by rot(p) so that the 8
// pixels of a transposed read's half-wave (4 lanes x 8 bytes each) hit 8 distinct 8-bank groups.
// Pixel p starts at bank group (PB / 32) p mod 8, which repeats every P0 = 8 / gcd(PB / 32, 8)
// pixels; rotating by 2 chunks (one group) per repeat fills the other groups.
template <int PB>
struct DyRot {
  static constexpr int gcd(int a, int b) { return b == 0 ? a : gcd(b, a % b); }
  static constexpr int P0 = 8 / gcd((PB / 32) % 8 == 0 ? 8 : (PB / 32) % 8, 8), NCC = PB / 16;
  __device__ __forceinline__ static int rot(int p) { return 2 * ((p / P0) % (8 / P0)); }
  static_assert(PB % 32 == 0 && NCC >= 16 / P0, "rotation needs that many chunks per pixel");
};

// ---------------------------------------------------------------------------------------------
// Weight gradient  dW[co][kh][kw c] = sum_p dy[p][co] x[S oy + kh - PAD][S ox + kw - PAD][c].
// The GEMM's N index is (kernel row kh, position j of the row's KW C run).  A transposed LDS read
// (ds_read_b64_tr_b16) takes per lane one address of 4 consecutive N elements of one K row
// (pixel), so the B operand is read straight out of the staged rows.
//   * dy of the item's RG Wo pixels lands by LDS-DMA beside x ([pixel][COUT], chunks rotated,
//     DyRot); rows past the image read zeros (a short last row group).
//   * Block = 8 waves (2 per SIMD), tile = all COUT x all KH NCH 4 columns; wave (m half, n
//     quarter) holds MT/2 x ~NTN/4 accumulators.  Persistent: a block walks a contiguous item
//     range, stores its partial tile once; two fixed-order passes sum the partials into dW.
template <class G>
struct Rr {
  static constexpr int NK = (G::PIX + 31) / 32;                       // K-steps per item
  static constexpr int PB = G::COUT * 2;                              // dy bytes per pixel
  static constexpr int NDQ = (NK * 32 * PB + 1023) / 1024, DB = NDQ * 1024;
  static constexpr int BUF = G::XB + DB;
  static constexpr int NQ = G::NXQ + NDQ, NQW = (NQ + 7) / 8;         // DMA pieces (per wave)
  static constexpr int NTN = (G::NCHK + 3) / 4;                       // 16-column N tiles
  static constexpr int TPW = (NTN + 3) / 4;                           // N tiles per wave (max)
  static constexpr int SLAB = G::MT * NTN * 256;                      // floats per partial tile
  static_assert(PB % 16 == 0, "alignment");
  static_assert(2 * BUF <= 160 * 1024, "LDS");
  static_assert(NK >= 3, "DMA spread");
};

template <class G>
__global__ void __launch_bounds__(512, 1)
conv_wgrad_rowrun(const bf16_t *__restrict__ x, const bf16_t *__restrict__ dy, float *__restrict__ ws, int H, int Ho,
                  int ldy, int nitems, int per) {
  using R = Rr<G>;
  using Rot = DyRot<R::PB>;
  constexpr int NK = R::NK, BUF = R::BUF, XB = G::XB, NXQ = G::NXQ, NQ = R::NQ, NQW = R::NQW;
  constexpr int NCH = G::NCH, NTN = R::NTN, MTW = G::MTW, TPW = R::TPW, PB = R::PB, ROWB = G::ROWB;
  constexpr int S = G::S, C = G::C, WO = G::WO, RG = G::RG;
  __shared__ __attribute__((aligned(1024))) char smem[2 * BUF];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int mh = wave & 1, nq = wave >> 1;
  const int groups_per_img = (Ho + RG - 1) / RG;
  const int ib = blockIdx.x * per, ie = min(nitems, ib + per);
  const uint32_t lds0 = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(reinterpret_cast<uintptr_t>((lds_void *)smem)));

  // DMA: piece q = wave + 8 i; q < NXQ: x (XStage); else dy LDS bytes b = 1024 (q - NXQ) + 16
  // lane: pixel b / PB, stored chunk (b % PB) / 16 holding channel chunk (stored - rot) mod NCC
  XStage<G, NQW> xs;
  xs.init(wave, lane, NXQ);
  uint32_t vd[NQW];
#pragma unroll
  for (int i = 0; i < NQW; ++i) {
    const int q = wave + 8 * i;
    uint32_t v = OOB;
    if (q >= NXQ && q < NQ) {
      const int b = 1024 * (q - NXQ) + 16 * lane, pix = b / PB, st = (b % PB) / 16;
      const int cc = (st - Rot::rot(pix) + Rot::NCC) % Rot::NCC;
      if (pix < G::PIX) v = static_cast<uint32_t>((pix * ldy + 8 * cc) * 2);
    }
    vd[i] = v;
  }
  rsrc_t rx, rd;
  int row0 = 0;
  auto prep = [&](int it) __attribute__((always_inline)) {
    const int n = it / groups_per_img, oy0 = (it - n * groups_per_img) * RG;
    rx = xs.rsrc(x, H, n, oy0, row0);
    const long dpix = (static_cast<long>(n) * Ho + oy0) * WO;
    rd = make_rsrc(dy + dpix * ldy, static_cast<uint32_t>(static_cast<long>(Ho - oy0) * WO * ldy * 2));
  };
  auto issue_one = [&](int b, auto ic) __attribute__((always_inline)) {
    constexpr int i = decltype(ic)::value;
    const int q = wave + 8 * i;
    if (q < NXQ) dma16d(rx, lds0 + static_cast<uint32_t>(b * BUF + q * 1024), xs.offset(i, row0, H));
    else if (q < NQ) dma16d(rd, lds0 + static_cast<uint32_t>(b * BUF + XB + (q - NXQ) * 1024), vd[i]);
  };

  // fragment addresses: K row (pixel) of lane for read hl: sl (frag_d's permutation), columns 4 p..
  const int l16 = lane & 15, g4 = lane >> 4, p4 = l16 & 3;
  int pa[NK][2];  // x: row(S oy_local) + RUN0 + 2 S C ox of pixel 32 k + sl
#pragma unroll
  for (int k = 0; k < NK; ++k)
#pragma unroll
    for (int hl = 0; hl < 2; ++hl) {
      int pix = 32 * k + (((g4 >> 1) << 4) | (hl << 3) | ((g4 & 1) << 2) | (l16 >> 2));
      pix = pix < G::PIX ? pix : G::PIX - 1;  // pad pixels (zero dy) read any staged pixel
      const int oyl = pix / WO, ox = pix - oyl * WO;
      pa[k][hl] = S * oyl * ROWB + G::RUN0 + S * C * 2 * ox;
    }
  int ca[TPW];  // x: row(kh) + 8 j4 of the lane's chunk in N tile nq + 4 tt
#pragma unroll
  for (int tt = 0; tt < TPW; ++tt) {
    int c = 4 * (nq + 4 * tt) + p4;
    c = c < G::NCHK ? c : G::NCHK - 1;
    ca[tt] = (c / NCH) * ROWB + 8 * (c % NCH);
  }
  int da[MTW][2];  // dy: pixel sl, channel chunk (16 mt + 4 p4) / 8 rotated, half p4 & 1
#pragma unroll
  for (int j = 0; j < MTW; ++j)
#pragma unroll
    for (int hl = 0; hl < 2; ++hl) {
      const int sl = ((g4 >> 1) << 4) | (hl << 3) | ((g4 & 1) << 2) | (l16 >> 2);
      const int mt = mh * MTW + j, cc = (2 * mt + (p4 >> 1) + Rot::rot(sl)) % Rot::NCC;
      da[j][hl] = XB + sl * PB + cc * 16 + 8 * (p4 & 1);
    }
  const int ntn = nq + 4 * (TPW - 1) < NTN ? TPW : TPW - 1;  // this wave's N tiles

  f32x4 acc[MTW][TPW];
#pragma unroll
  for (int j = 0; j < MTW; ++j)
#pragma unroll
    for (int tt = 0; tt < TPW; ++tt) {
      acc[j][tt] = f32x4{0.f, 0.f, 0.f, 0.f};
      asm volatile("" : "+a"(acc[j][tt]));
    }
  bf16x8 fa[2][MTW], fb[2][TPW];
  constexpr int NR = MTW + TPW, NM = MTW * TPW, RS = NM / NR > 0 ? NM / NR : 1;
  auto read_one = [&](const char *buf, auto kc, auto sc, auto rc) __attribute__((always_inline)) {
    constexpr int k = decltype(kc)::value, st = decltype(sc)::value, r = decltype(rc)::value;
    if constexpr (r < MTW) {
      fa[st][r] = frag_d(buf + da[r][0] + 32 * k * PB, buf + da[r][1] + 32 * k * PB);
    } else {
      constexpr int tt = r - MTW;
      fb[st][tt] = frag_d(buf + pa[k][0] + ca[tt], buf + pa[k][1] + ca[tt]);
    }
  };

  if (ib < ie) {
    prep(ib);
    static_for<NQW>([&](auto ic) { issue_one(0, ic); });
  }
  for (int it = ib; it < ie; ++it) {
    const int b = (it - ib) & 1;
    wait_vmcnt<0>();
    block_barrier();
    const bool more = it + 1 < ie;
    if (more) prep(it + 1);
    const char *buf = smem + b * BUF;
    static_for<NR>([&](auto rc) { read_one(buf, std::integral_constant<int, 0>{}, std::integral_constant<int, 0>{}, rc); });
    static_for<NK>([&](auto kc) {
      constexpr int k = decltype(kc)::value, s0 = k & 1;
      static_for<NM>([&](auto qc) {
        constexpr int q = decltype(qc)::value;
        constexpr int tt = q / MTW, j = q % MTW;
        __builtin_amdgcn_sched_barrier(0);
        if (tt < ntn) mfma_d<true>(acc[j][tt], fa[s0][j], fb[s0][tt]);
        static_for<NQW>([&](auto ic) {
          constexpr int i = decltype(ic)::value;
          // the next item's DMAs go out during the first K-step (one after each MFMA): its
          // compute is short against their latency (AlexNet b256 1.814 / 1.819 -> 1.800 / 1.806 ms
          // against spreading them over the K-steps; GoogLeNet b128 unchanged)
          if constexpr (k == 0 && q == i % NM) {
            if (more) issue_one(b ^ 1, ic);
          }
        });
        if constexpr (k + 1 < NK) {
          if constexpr (q % RS == RS - 1 && q / RS < NR)
            read_one(buf, std::integral_constant<int, k + 1>{}, std::integral_constant<int, s0 ^ 1>{},
                     std::integral_constant<int, q / RS>{});
          if constexpr (q == NM - 1 && NM / RS < NR)
            static_for<NR - NM / RS>([&](auto rc) {
              read_one(buf, std::integral_constant<int, k + 1>{}, std::integral_constant<int, s0 ^ 1>{},
                       std::integral_constant<int, NM / RS + decltype(rc)::value>{});
            });
        }
      });
      __builtin_amdgcn_sched_barrier(0);
    });
  }
  asm volatile("s_nop 15\n\ts_nop 15\n\ts_nop 15" ::: "memory");
#pragma unroll
  for (int j = 0; j < MTW; ++j)
#pragma unroll
    for (int tt = 0; tt < TPW; ++tt) pin_d<true>(acc[j][tt]);
  // partial tile: ws[block][mt][nt][lane] (f32x4)
  float *out = ws + static_cast<long>(blockIdx.x) * R::SLAB + 4 * lane;
#pragma unroll
  for (int tt = 0; tt < TPW; ++tt)
    if (tt < ntn) {
#pragma unroll
      for (int j = 0; j < MTW; ++j)
        *reinterpret_cast<f32x4 *>(out + ((mh * MTW + j) * NTN + nq + 4 * tt) * 256) = acc[j][tt];
    }
}

// fixed-order sums of the partial tiles: pass 1 (final == 0) sums groups of GS slabs into
// out[group]; pass 2 sums the groups and adds alpha x the (kh, j < KW C) columns into dW
template <int KH, int KW, int C, int MT, int NTN>
__global__ void __launch_bounds__(256)
conv_wgrad_rowrun_reduce(const float *__restrict__ in, int nslab, int gs, float *__restrict__ out, float *__restrict__ dw,
                         float alpha, int final) {
  constexpr int NCH = (KW * C + 3) / 4, NE = MT * NTN * 64;  // f32x4 units per slab
  constexpr long SLAB = static_cast<long>(NE) * 4;
  const long tid = static_cast<long>(blockIdx.x) * 256 + threadIdx.x;
  const int grp = static_cast<int>(tid / NE), e = static_cast<int>(tid - static_cast<long>(grp) * NE);
  if (grp * gs >= nslab) return;
  const int s1 = min(nslab, grp * gs + gs);
  f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int sl = grp * gs; sl < s1; ++sl) acc += *reinterpret_cast<const f32x4 *>(in + sl * SLAB + 4L * e);
  if (!final) {
    *reinterpret_cast<f32x4 *>(out + grp * SLAB + 4L * e) = acc;
    return;
  }
  const int lane = e & 63, t = e >> 6, mt = t / NTN, nt = t - mt * NTN;
  const int c = 4 * nt + (lane & 15) / 4, jj = 4 * (c % NCH) + (lane & 3), kh = c / NCH;
  if (kh >= KH || jj >= KW * C) return;
  const int co = 16 * mt + 4 * (lane >> 4);
#pragma unroll
  for (int i = 0; i < 4; ++i) dw[static_cast<long>(co + i) * KH * KW * C + kh * KW * C + jj] += alpha * acc[i];
}

template <class G>
struct RrLaunch {
  using R = Rr<G>;
  static constexpr int GS = 16;
  static void plan(int N, int Ho, int &nitems, int &per, int &nblk) {
    nitems = N * ((Ho + G::RG - 1) / G::RG);
    per = (nitems + 255) / 256;
    nblk = (nitems + per - 1) / per;
  }
  static long ws(int N, int Ho) {
    int nitems, per, nblk;
    plan(N, Ho, nitems, per, nblk);
    return static_cast<long>(nblk + (nblk + GS - 1) / GS) * R::SLAB;
  }
  static int run(const bf16_t *x, const bf16_t *dy, float *dw, float *ws_, long ws_floats, int N, int H, int Ho, int ldy,
                 float alpha, hipStream_t s) {
    int nitems, per, nblk;
    plan(N, Ho, nitems, per, nblk);
    const int ngrp = (nblk + GS - 1) / GS;
    if (ws_floats < static_cast<long>(nblk + ngrp) * R::SLAB) return -4;
    CXN_LAUNCH((conv_wgrad_rowrun<G>), dim3(static_cast<unsigned>(nblk)), dim3(512), 0, s, x, dy, ws_, H, Ho, ldy, nitems,
               per);
    float *part = ws_ + static_cast<long>(nblk) * R::SLAB;
    constexpr int NE = G::MT * R::NTN * 64;
    CXN_LAUNCH((conv_wgrad_rowrun_reduce<G::KH, G::KW, G::C, G::MT, R::NTN>),
               dim3(static_cast<unsigned>((ngrp * NE + 255) / 256)), dim3(256), 0, s, ws_, nblk, GS, part, nullptr, 0.f, 0);
    CXN_LAUNCH((conv_wgrad_rowrun_reduce<G::KH, G::KW, G::C, G::MT, R::NTN>), dim3(static_cast<unsigned>((NE + 255) / 256)),
               dim3(256), 0, s, part, ngrp, ngrp, nullptr, dw, alpha, 1);
    return 0;
  }
};

// ---------------------------------------------------------------------------------------------
// Forward  y[p][co] = relu(bias[co] + sum_{kh, j} W[co][kh][j] x[S oy + kh - PAD][S C ox + j - PAD C]).
//   * GEMM: A = W (M = co), B = the pixels' row runs (N = pixel, K = (kh, 4-element chunk)).
//     The lane's 8 K values of a 16x16x32 B fragment are two chunks = two ds_read_b64 at
//     pixel address + chunk address (K-step k, lane group g4: chunks 8 k + 2 g4, + 1).
//   * W is staged once per block as [co][NK * 8 chunks] (+16 B row pad: conflict-free
//     ds_read_b128 of the A fragment = chunks 8 k + 2 g4 .. + 1 of one co row).  When a wave's
//     share of it fits 64 registers (GoogLeNet: 2 tiles x 7 K-steps) it is read into VGPRs once
//     and the K loop reads only B.
//   * Block = 8 waves (2 per SIMD); wave (m half, n quarter): MT/2 x ~NTN/4 accumulator tiles
//     in AGPRs, zeroed by the item's first MFMA (C operand 0).  Per K-step a wave reads its
//     fragments one ahead of the MFMAs and issues a share of the next item's DMAs.
//   * Epilogue: bias + relu, 4 consecutive co of one pixel per lane -> one 8-byte buffer store;
//     every store instruction is issued (masked lanes use out-of-range offsets), so the next
//     item waits with a counted vmcnt for its own DMAs only (vector memory retires in order).
template <class G>
struct Rf {
  static constexpr int NQW = (G::NXQ + 7) / 8;
  static constexpr int NTN = (G::PIX + 15) / 16, TPW = (NTN + 3) / 4;
  static constexpr int NK = (G::NCHK + 7) / 8;                    // K-steps
  static constexpr int WROW = NK * 64 + 16, WB = (G::COUT * WROW + 1023) / 1024 * 1024;
  static constexpr int NST = G::MTW * TPW;                        // epilogue stores per wave and item
  static constexpr bool WREG = G::MTW * NK * 4 <= 64;             // the wave's W fragments in VGPRs
  static_assert(WB + 2 * G::XB <= 160 * 1024, "LDS");
  static_assert(NK >= 3 && NST <= 60, "pipeline");
};

__device__ __forceinline__ void mfma_z(f32x4 &acc, const bf16x8 &a, const bf16x8 &b) {  // acc = a b
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, 0" : "=a"(acc) : "v"(a), "v"(b));
}

template <class G>
__global__ void __launch_bounds__(512, 1)
conv_rowrun_fwd2(const bf16_t *__restrict__ x, const bf16_t *__restrict__ w, const float *__restrict__ bias,
                 bf16_t *__restrict__ y, int H, int Ho, int ldc, int relu, int nitems, int per) {
  using F = Rf<G>;
  constexpr int NK = F::NK, XB = G::XB, WB = F::WB, NXQ = G::NXQ, NQW = F::NQW, NCH = G::NCH, NCHK = G::NCHK;
  constexpr int MTW = G::MTW, TPW = F::TPW, ROWB = G::ROWB, WROW = F::WROW, PIX = G::PIX;
  constexpr int S = G::S, C = G::C, WO = G::WO, RG = G::RG, KH = G::KH, KRUN = G::KW * G::C;
  constexpr bool WREG = F::WREG;
  __shared__ __attribute__((aligned(1024))) char smem[WB + 2 * XB];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int mh = wave & 1, nq = wave >> 1;
  const int gpi = (Ho + RG - 1) / RG;
  const int ib = blockIdx.x * per, ie = min(nitems, ib + per);
  const uint32_t lds0 = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(reinterpret_cast<uintptr_t>((lds_void *)smem)));

  XStage<G, NQW> xs;
  xs.init(wave, lane, NXQ);
  rsrc_t rx, ry;
  int row0 = 0;
  auto prep = [&](int it) __attribute__((always_inline)) {
    const int n = it / gpi, oy0 = (it - n * gpi) * RG;
    rx = xs.rsrc(x, H, n, oy0, row0);
  };
  auto prep_y = [&](int it) __attribute__((always_inline)) {
    const int n = it / gpi, oy0 = (it - n * gpi) * RG;
    const long p0 = (static_cast<long>(n) * Ho + oy0) * WO;
    ry = make_rsrc(y + p0 * ldc, static_cast<uint32_t>(static_cast<long>(Ho - oy0) * WO * ldc * 2));
  };
  auto issue_one = [&](int b, auto ic) __attribute__((always_inline)) {
    constexpr int i = decltype(ic)::value;
    const int q = wave + 8 * i;
    if (q < NXQ) dma16d(rx, lds0 + static_cast<uint32_t>(WB + b * XB + q * 1024), xs.offset(i, row0, H));
  };
  if (ib < ie) {
    prep(ib);
    static_for<NQW>([&](auto ic) { issue_one(0, ic); });
  }
  // weights -> [co][chunk] image (zero chunks past a run / past the last kernel row)
  for (int e = tid; e < G::COUT * NK * 8; e += 512) {
    const int co = e / (NK * 8), c = e - co * (NK * 8);
    const int kh = c / NCH, j0 = 4 * (c - kh * NCH);
    typedef short s16x4_ __attribute__((ext_vector_type(4)));
    s16x4_ v = {0, 0, 0, 0};
    if (c < NCHK) {
      const short *src = reinterpret_cast<const short *>(w) + static_cast<long>(co) * KH * KRUN + kh * KRUN + j0;
#pragma unroll
      for (int t = 0; t < 4; ++t) v[t] = j0 + t < KRUN ? src[t] : static_cast<short>(0);
    }
    *reinterpret_cast<s16x4_ *>(smem + co * WROW + c * 8) = v;
  }

  const int l16 = lane & 15, g4 = lane >> 4;
  float bv[MTW][4];
#pragma unroll
  for (int j = 0; j < MTW; ++j)
#pragma unroll
    for (int t = 0; t < 4; ++t) bv[j][t] = bias ? bias[16 * (mh * MTW + j) + 4 * g4 + t] : 0.f;
  int wa[MTW];  // A: co row 16 mt + l16, chunks 2 g4 .. (+ 64 k)
#pragma unroll
  for (int j = 0; j < MTW; ++j) wa[j] = (16 * (mh * MTW + j) + l16) * WROW + 16 * g4;
  int pa[TPW];  // B: pixel 16 (nq + 4 tt) + l16 of the item
#pragma unroll
  for (int tt = 0; tt < TPW; ++tt) {
    int p = 16 * (nq + 4 * tt) + l16;
    p = p < PIX ? p : PIX - 1;
    const int oyl = p / WO, ox = p - oyl * WO;
    pa[tt] = WB + S * oyl * ROWB + G::RUN0 + S * C * 2 * ox;
  }
  int ca[NK][2];  // B: chunk 8 k + 2 g4 + h
#pragma unroll
  for (int k = 0; k < NK; ++k)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      int c = 8 * k + 2 * g4 + h;
      c = c < NCHK ? c : NCHK - 1;  // (zero weights)
      ca[k][h] = (c / NCH) * ROWB + 8 * (c % NCH);
    }
  uint32_t so[TPW];  // store offsets of the lane's pixels (4 co of 16 mt + 4 g4 added per tile)
#pragma unroll
  for (int tt = 0; tt < TPW; ++tt) {
    const int p = 16 * (nq + 4 * tt) + l16;
    so[tt] = p < PIX ? static_cast<uint32_t>(p * ldc * 2 + 8 * g4) : OOB;
  }

  f32x4 acc[MTW][TPW];
  bf16x8 fa[2][MTW], fb[2][TPW];
  bf16x8 wr[WREG ? MTW : 1][WREG ? NK : 1];
  constexpr int NRA = WREG ? 0 : MTW;  // A reads per K-step
  constexpr int NR = NRA + TPW, NM = MTW * TPW, RS = NM / NR > 0 ? NM / NR : 1;
  auto read_one = [&](const char *bx, auto kc, auto sc, auto rc) __attribute__((always_inline)) {
    constexpr int k = decltype(kc)::value, st = decltype(sc)::value, r = decltype(rc)::value;
    if constexpr (r < NRA) {
      fa[st][r] = *reinterpret_cast<const bf16x8 *>(smem + wa[r] + 64 * k);
    } else {
      constexpr int tt = r - NRA;
      typedef short s16x4_ __attribute__((ext_vector_type(4)));
      typedef short s16x8_ __attribute__((ext_vector_type(8)));
      const s16x4_ lo = *reinterpret_cast<const s16x4_ *>(bx + pa[tt] + ca[k][0]);
      const s16x4_ hi = *reinterpret_cast<const s16x4_ *>(bx + pa[tt] + ca[k][1]);
      const s16x8_ v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      fb[st][tt] = __builtin_bit_cast(bf16x8, v);
    }
  };
  auto afrag = [&](auto kc, auto sc, auto jc) __attribute__((always_inline)) -> const bf16x8 & {
    constexpr int k = decltype(kc)::value, st = decltype(sc)::value, j = decltype(jc)::value;
    if constexpr (WREG) return wr[j][k];
    else return fa[st][j];
  };

  for (int it = ib; it < ie; ++it) {
    const int b = (it - ib) & 1;
    wait_vmcnt<F::NST>();  // this item's DMAs landed (the previous item's stores may still drain)
    block_barrier();
    if constexpr (WREG) {
      if (it == ib) {  // the weight image is complete after the first barrier
#pragma unroll
        for (int j = 0; j < MTW; ++j)
#pragma unroll
          for (int k = 0; k < NK; ++k) wr[j][k] = *reinterpret_cast<const bf16x8 *>(smem + wa[j] + 64 * k);
      }
    }
    const bool more = it + 1 < ie;
    if (more) prep(it + 1);
    prep_y(it);
    const char *bx = smem + b * XB;
    static_for<NR>([&](auto rc) { read_one(bx, std::integral_constant<int, 0>{}, std::integral_constant<int, 0>{}, rc); });
    static_for<NK>([&](auto kc) {
      constexpr int k = decltype(kc)::value, s0 = k & 1;
      static_for<NM>([&](auto qc) {
        constexpr int q = decltype(qc)::value;
        constexpr int tt = q / MTW, j = q % MTW;
        __builtin_amdgcn_sched_barrier(0);
        const bf16x8 &av = afrag(kc, std::integral_constant<int, s0>{}, std::integral_constant<int, j>{});
        if constexpr (k == 0) mfma_z(acc[j][tt], av, fb[s0][tt]);
        else mfma_d<true>(acc[j][tt], av, fb[s0][tt]);
        static_for<NQW>([&](auto ic) {
          constexpr int i = decltype(ic)::value;
          // the next item's DMAs go out during the first K-step (one after each MFMA): its
          // compute is short against their latency (AlexNet b256 1.814 / 1.819 -> 1.800 / 1.806 ms
          // against spreading them over the K-steps; GoogLeNet b128 unchanged)
          if constexpr (k == 0 && q == i % NM) {
            if (more) issue_one(b ^ 1, ic);
          }
        });
        if constexpr (k + 1 < NK) {
          if constexpr (q % RS == RS - 1 && q / RS < NR)
            read_one(bx, std::integral_constant<int, k + 1>{}, std::integral_constant<int, s0 ^ 1>{},
                     std::integral_constant<int, q / RS>{});
          if constexpr (q == NM - 1 && NM / RS < NR)
            static_for<NR - NM / RS>([&](auto rc) {
              read_one(bx, std::integral_constant<int, k + 1>{}, std::integral_constant<int, s0 ^ 1>{},
                       std::integral_constant<int, NM / RS + decltype(rc)::value>{});
            });
        }
      });
      __builtin_amdgcn_sched_barrier(0);
    });
    asm volatile("s_nop 15\n\ts_nop 15\n\ts_nop 15" ::: "memory");
#pragma unroll
    for (int tt = 0; tt < TPW; ++tt)
#pragma unroll
      for (int j = 0; j < MTW; ++j) {
        pin_d<true>(acc[j][tt]);
        float f[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          f[t] = acc[j][tt][t] + bv[j][t];
          if (relu) f[t] = fmaxf(f[t], 0.f);
        }
        typedef int v2i __attribute__((ext_vector_type(2)));
        const v2i pk = {static_cast<int>(pack2(f[0], f[1])), static_cast<int>(pack2(f[2], f[3]))};
        const uint32_t off = so[tt] == OOB ? OOB : so[tt] + static_cast<uint32_t>(32 * (mh * MTW + j));
        __builtin_amdgcn_raw_buffer_store_b64(pk, ry, off, 0, 0);
      }
  }
}

template <class G>
int launch_fwd2(const bf16_t *x, const bf16_t *w, const float *bias, bf16_t *y, int N, int H, int Ho, int ldc, int relu,
                hipStream_t s) {
  const int nitems = N * ((Ho + G::RG - 1) / G::RG);
  const int per = (nitems + 255) / 256, nblk = (nitems + per - 1) / per;
  CXN_LAUNCH((conv_rowrun_fwd2<G>), dim3(static_cast<unsigned>(nblk)), dim3(512), 0, s, x, w, bias, y, H, Ho, ldc, relu,
             nitems, per);
  return 0;
}

// the served geometries
using GAlex = RGeo<11, 11, 3, 4, 0, 228, 55, 96, 4>;    // AlexNet conv1 (rows padded to 228 pixels)
using GGoog = RGeo<7, 7, 4, 2, 3, 224, 112, 64, 2>;     // GoogLeNet conv1 (4-channel NHWC input)

// 0: AlexNet, 1: GoogLeNet, -1: not served
int pick_geo(int H, int W, int C, int Ho, int Wo, int Cout, int KH, int KW, int stride, int pad) {
  if (C == 3 && W == 228 && Wo == 55 && Cout == 96 && KH == 11 && KW == 11 && stride == 4 && pad == 0 &&
      Ho > 0 && H >= 4 * (Ho - 1) + 11)
    return 0;
  if (C == 4 && W == 224 && Wo == 112 && Cout == 64 && KH == 7 && KW == 7 && stride == 2 && pad == 3 && Ho > 0 &&
      H + 6 >= 2 * (Ho - 1) + 7)
    return 1;
  return -1;
}

}  // namespace

// Few-channel first layer weight gradient (conv_wgrad_rowrun).  Served: the AlexNet conv1 class
// (3 channels on rows of 228 pixels, 11 x 11 / 4, pad 0, 55 output columns, 96 outputs) and the
// GoogLeNet conv1 class (4 channels on 224-pixel rows, 7 x 7 / 2, pad 3, 112 output columns, 64
// outputs); one group, x contiguous [N][H][W][C], dy pixel stride ldy a multiple of 8.  dw fp32
// [Cout][KH][KW][C] += alpha * gradient.  ws == nullptr: workspace floats (0: not served); else
// -1 not served, -4 workspace too small.
CXN_API long cxn_conv_wgrad_rowrun(const void *x, const void *dy, float *dw, float *ws, long ws_floats, int N, int H,
                                   int W, int C, int Ho, int Wo, int Cout, int ldy, int KH, int KW, int stride, int pad,
                                   float alpha, void *stream) {
  const int geo = pick_geo(H, W, C, Ho, Wo, Cout, KH, KW, stride, pad);
  const bool ok = geo >= 0 && N > 0 && ldy >= Cout && ldy % 8 == 0 && static_cast<long>(H) * W * C * 2 < (1L << 31) &&
                  static_cast<long>(Ho) * Wo * ldy * 2 < (1L << 31);
  if (!ok) return ws ? -1 : 0;
  if (!ws) return geo == 0 ? RrLaunch<GAlex>::ws(N, Ho) : RrLaunch<GGoog>::ws(N, Ho);
  const bf16_t *xb = static_cast<const bf16_t *>(x), *dyb = static_cast<const bf16_t *>(dy);
  hipStream_t s = static_cast<hipStream_t>(stream);
  const int rc = geo == 0 ? RrLaunch<GAlex>::run(xb, dyb, dw, ws, ws_floats, N, H, Ho, ldy, alpha, s)
                          : RrLaunch<GGoog>::run(xb, dyb, dw, ws, ws_floats, N, H, Ho, ldy, alpha, s);
  if (rc != 0) return rc;
  return hipGetLastError() == hipSuccess ? 0 : -3;
}

// Few-channel first layer forward (conv_rowrun_fwd2).  Served: the geometries of
// cxn_conv_wgrad_rowrun; w bf16 [Cout][KH][KW][C] (not row-padded), bias fp32 or null, y bf16
// with pixel stride ldc (a multiple of 4, >= Cout).  -1: not served.
CXN_API int cxn_conv_rowrun_fwd2(const void *x, const void *w, const float *bias, void *y, int N, int H, int W, int C,
                                 int Ho, int Wo, int Cout, int ldc, int KH, int KW, int stride, int pad, int relu,
                                 void *stream) {
  const int geo = pick_geo(H, W, C, Ho, Wo, Cout, KH, KW, stride, pad);
  const bool ok = geo >= 0 && N > 0 && ldc >= Cout && ldc % 4 == 0 && static_cast<long>(H) * W * C * 2 < (1L << 31) &&
                  static_cast<long>(Ho) * Wo * ldc * 2 < (1L << 31);
  if (!ok) return -1;
  const bf16_t *xb = static_cast<const bf16_t *>(x), *wb = static_cast<const bf16_t *>(w);
  bf16_t *yb = static_cast<bf16_t *>(y);
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (geo == 0) launch_fwd2<GAlex>(xb, wb, bias, yb, N, H, Ho, ldc, relu, s);
  else launch_fwd2<GGoog>(xb, wb, bias, yb, N, H, Ho, ldc, relu, s);
  return hipGetLastError() == hipSuccess ? 0 : -3;
}
