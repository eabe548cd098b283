// Direct stride-1 "same" convolution WEIGHT gradient for small maps (AlexNet conv3-5: 13 x 13,
// 3 x 3, grouped; conv2: 27 x 27, 5 x 5, grouped, tap-split form below), gfx950:  dW[co][kh][kw][ci] += sum_p dy[p][co] * x[p + (kh, kw) - pad][ci].
// Reference: src/layer/convolution_layer-inl.hpp:121-138 (im2col + gemm into gwmat per group).
//
// Why.  The split-K implicit GEMM (gemm_mfma.hip GATHER_MN) rebuilds every pixel's im2col address
// per 16-byte load (3.66 VALU per MFMA) and meets its K slices in fp32 atomics; on AlexNet's
// 13 x 13 layers it ran 455-635 TFLOP/s (profiles/r4_alexnet_b256_kernels_final.md).  The VGG
// halo kernel (conv_wgrad_halo.hip) tiles 2-D patches of 16-32 columns, which waste a third of
// the MFMAs on a 13-wide map.  Here:
//   * Pixel "slots": every image row is followed by a P-wide zero gap (pitch PW = W + P), and
//     images of a stage are stacked with P zero separator rows.  In that linear slot space the
//     input pixel under tap (kh, kw) of output slot s is slot s + kh * PW + kw of the staged x
//     image, for EVERY slot: a tap is a constant shift, zero padding falls on gap / separator
//     slots (zeros), and the K walk over output slots has no per-pixel index arithmetic.  The dy
//     gap slots are zero, so they add nothing (13 x 13: 169 of 192 walked slots are pixels).
//   * A stage = IPS whole images; one block streams its images' x (32 channels) and dy (64
//     channels) through a double-buffered LDS pair by LDS-DMA.  Every lane's DMA source offsets
//     within a stage are fixed for the whole kernel (computed once); per stage only the buffer
//     descriptors move, and slots outside the map read as zeros through out-of-range offsets.
//   * LDS images are channel-unit-major ([16-channel unit][slot][16 ch], 32 B per slot-unit).
//     An MFMA k-index -> slot permutation makes each 32-lane half of a ds_read_b64_tr_b16 read 8
//     consecutive slots (256 contiguous bytes): conflict-free for dy and for every tap shift.
//   * Block tile 64 co x 32 ci x all taps.  The four waves (one per SIMD) each accumulate the
//     WHOLE tile (4 x 2 x 9 f32x4 = 288 AGPRs) over every fourth K-step, so per K-step a wave
//     reads 4 dy + 18 x fragments for 72 MFMAs (0.31 reads per MFMA) with constant addresses.
//     The four partial tiles meet through LDS after the loop.
//   * Split over images: (pairs x splits) ~ one block per CU, XCD-contiguous so the blocks that
//     read the same images share an L2.  No atomics: each block stores its partial tile with
//     plain coalesced 16-byte stores into a workspace, and conv_wgrad_direct_reduce sums the
//     splits in a fixed order into dW (+=), so the result is bitwise reproducible.
#include "direct_common.h"

using namespace cxg;
using namespace cxd;

namespace {

constexpr int NAGPR_ACC = 56;  // f32x4 accumulators kept in AGPRs (224 of the 256)


template <int H, int W, int KS, int IPS>
struct Wd {
  static constexpr int P = (KS - 1) / 2;
  static constexpr int T = KS * KS;
  static constexpr int PW = W + P;                       // slot pitch
  static constexpr int VR = H + P;                       // virtual rows per image
  static constexpr int WALK = (IPS * VR - P) * PW;       // output slots that can hold pixels
  static constexpr int NK = (WALK + 127) / 128 * 4;      // K-steps per stage, a multiple of 4
  static constexpr int KW4 = NK / 4;                     // K-steps per wave per stage
  static constexpr int NKS = NK * 32;                    // dy slots per stage
  static constexpr int NX = (NKS + (KS - 1) * (PW + 1) + 31) / 32;  // x slot groups of 32
  static constexpr int NXS = NX * 32;
  static constexpr int XLEAD = P * PW + P;               // x slot of linear position 0
  static constexpr int CO_U = 4, CI_U = 2;               // 64 co x 32 ci per block
  static constexpr int DYB = CO_U * NKS * 32;            // dy bytes per buffer
  static constexpr int XB = CI_U * NXS * 32;
  static constexpr int BUF = DYB + XB;
  static constexpr int NQD = CO_U * NK / 4;              // dy DMA instructions per wave
  static constexpr int NQX = (CI_U * NX + 3) / 4;        // x DMA instructions per wave (last maybe idle)
  static constexpr int NACC = CO_U * CI_U * T;           // f32x4 accumulators per wave
  static_assert(2 * BUF <= 160 * 1024, "LDS");  // (the epilogue's chunked combine checks its own fit)
};

// (image, row, col) of a linear position in a stage's virtual slot space; -1 when it is padding
template <int H, int W, int KS, int IPS>
__device__ __forceinline__ int slot_pixel(int lin) {
  using G = Wd<H, W, KS, IPS>;
  const int vrow = fdiv_floor(lin, G::PW);
  const int col = lin - vrow * G::PW;
  const int img = fdiv_floor(vrow, G::VR);
  const int row = vrow - img * G::VR;
  if (img < 0 || img >= IPS || row >= H || col >= W) return -1;
  return (img * H + row) * W + col;
}

template <int H, int W, int KS, int IPS, int V>
__global__ void __launch_bounds__(256, 1)
conv_wgrad_direct(const bf16_t *__restrict__ x, const bf16_t *__restrict__ dy, float *__restrict__ ws, int N, int C,
                  int ldy, int Cg, int Cog, int npairs, int nci_b, int nco_b, int per, int nstages, int want_db) {
  using G = Wd<H, W, KS, IPS>;
  constexpr int T = G::T, NK = G::NK, KW4 = G::KW4, NKS = G::NKS, NX = G::NX, NXS = G::NXS, PW = G::PW;
  constexpr int CO_U = G::CO_U, CI_U = G::CI_U, BUF = G::BUF, DYB = G::DYB, NQD = G::NQD, NQX = G::NQX;
  constexpr int HW = H * W;
  __shared__ __attribute__((aligned(1024))) char smem[2 * BUF];

  const uint32_t L = xcd_remap(blockIdx.x, gridDim.x);
  const int pair = static_cast<int>(L % static_cast<uint32_t>(npairs));
  const int split = static_cast<int>(L / static_cast<uint32_t>(npairs));
  const int per_g = nco_b * nci_b;
  const int g = pair / per_g, rem = pair - g * per_g;
  const int cob = rem / nci_b, cib = rem - cob * nci_b;
  const int ci0 = g * Cg + cib * 16 * CI_U, co0 = g * Cog + cob * 16 * CO_U;
  const int sb = split * per, se = min(nstages, sb + per);

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);

  const uint32_t lds0 = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(reinterpret_cast<uintptr_t>((lds_void *)smem)));
  // ---- per-lane DMA source offsets within a stage (fixed for the whole kernel)
  uint32_t vd[NQD], vx[NQX];
#pragma unroll
  for (int i = 0; i < NQD; ++i) {
    const int q = wave + 4 * i;
    const int u = q / NK, sg = q - u * NK;
    const int pix = slot_pixel<H, W, KS, IPS>(32 * sg + (lane >> 1));
    vd[i] = pix >= 0 ? static_cast<uint32_t>((pix * ldy + 16 * u + 8 * (lane & 1)) * 2) : OOB;
  }
#pragma unroll
  for (int i = 0; i < NQX; ++i) {
    const int q = wave + 4 * i;
    const int u = q / NX, sg = q - u * NX;
    const int pix = slot_pixel<H, W, KS, IPS>(32 * sg + (lane >> 1) - G::XLEAD);
    vx[i] = (q < CI_U * NX && pix >= 0) ? static_cast<uint32_t>((pix * C + 16 * u + 8 * (lane & 1)) * 2) : OOB;
  }
  // stage st -> buffer b: the DMAs of this wave (descriptors cover the stage's whole images; a
  // missing last image is out of range, so its slots read as zeros).  DMA i < NQD is dy
  // instruction wave + 4 i, the rest x instructions.
  constexpr int NDMA = NQD + NQX;
  rsrc_t rd, rx;
  auto prep = [&](int st) __attribute__((always_inline)) {
    const int n0 = st * IPS;
    const int nimg = min(IPS, N - n0);
    const long pd = static_cast<long>(n0) * HW;
    rd = make_rsrc(dy + pd * ldy + co0, static_cast<uint32_t>((nimg * HW * static_cast<long>(ldy) - co0) * 2));
    rx = make_rsrc(x + pd * C + ci0, static_cast<uint32_t>((nimg * HW * static_cast<long>(C) - ci0) * 2));
  };
  auto issue_one = [&](auto ic, int b) __attribute__((always_inline)) {
    constexpr int i = decltype(ic)::value;
    const uint32_t base = lds0 + b * BUF + wave * 1024;  // wave-uniform LDS byte address
    if constexpr (i < NQD) {
      dma16d(rd, base + i * 4096, vd[i]);
    } else {
      constexpr int k = i - NQD;
      if (wave + 4 * k < CI_U * NX) dma16d(rx, base + DYB + k * 4096, vx[k]);
    }
  };
  auto issue = [&](int st, int b) __attribute__((always_inline)) {
    prep(st);
    static_for<NDMA>([&](auto ic) { issue_one(ic, b); });
  };

  // ---- fragment read bases: lane (l16, g4) = (4 q + p, g4) reads slot sl(hl) bytes 8p..8p+7
  const int l16 = lane & 15, g4 = lane >> 4;
  int bd[2][2], bx[2][2];  // [buffer][hl]
#pragma unroll
  for (int hl = 0; hl < 2; ++hl) {
    const int sl = ((g4 >> 1) << 4) | (hl << 3) | ((g4 & 1) << 2) | (l16 >> 2);
    const int o = (sl + 32 * wave) * 32 + 8 * (l16 & 3);  // this wave's first K-step
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      bd[b][hl] = b * BUF + o;
      bx[b][hl] = b * BUF + DYB + o;
    }
  }

  // accumulator i = (m CI_U + u) T + t
  f32x4 acc[G::NACC];
#pragma unroll
  for (int i = 0; i < G::NACC; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 fa[2][CO_U], fb[3][CI_U];
  // bias gradient (want_db): db[co] = sum over pixels of dy, as MFMAs of the dy fragments with a
  // ones operand.  K-step k (= wave + 4 j of every stage) of co block cob is summed by the block
  // with ci block k % nci_b, so each pixel counts once and the extra MFMAs (4 per summed K-step)
  // are spread over the ci blocks (< 1 % of the MFMAs).
  f32x4 accb[CO_U];
#pragma unroll
  for (int m = 0; m < CO_U; ++m) accb[m] = f32x4{0.f, 0.f, 0.f, 0.f};
  bool dbj[KW4];
#pragma unroll
  for (int j = 0; j < KW4; ++j) dbj[j] = want_db && (wave + 4 * j) % nci_b == cib;
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  bf16x8 ones = __builtin_bit_cast(bf16x8, s16x8{0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80});
  asm volatile("" : "+v"(ones));  // opaque: not re-materialised next to its MFMAs

  // K-step j (0..KW4-1) of this wave in buffer b: slots 32 (wave + 4 j) ..
  auto read_a = [&](int set, int b, int j) __attribute__((always_inline)) {
#pragma unroll
    for (int m = 0; m < CO_U; ++m) {
      const int off = (m * NKS + 128 * j) * 32;
      fa[set][m] = frag_d(smem + bd[b][0] + off, smem + bd[b][1] + off);
    }
  };
  auto read_bu = [&](int set, int b, int j, int t, int u) __attribute__((always_inline)) {
    const int kh = t / KS, kw = t - kh * KS;
    const int off = (u * NXS + 128 * j + kh * PW + kw) * 32;
    fb[set][u] = frag_d(smem + bx[b][0] + off, smem + bx[b][1] + off);
  };
  auto read_b = [&](int set, int b, int j, int t) __attribute__((always_inline)) {
#pragma unroll
    for (int u = 0; u < CI_U; ++u) read_bu(set, b, j, t, u);
  };

  // prologue: stage sb
  issue(sb, 0);
  wait_vmcnt<0>();
  block_barrier();
  read_a(0, 0, 0);
  read_b(0, 0, 0, 0);
  read_b(1, 0, 0, 1);
  __builtin_amdgcn_sched_barrier(0);

  // One stage from buffer B (landed; K-step 0's dy and taps 0-1 are being read).  KW4 K-steps of
  // T taps; during tap t the reads of tap t + 2 (or of the next K-step's dy / taps 0-1) are
  // issued between the MFMAs.  Set indices are compile-time over a pair of stages: KW4 * T taps
  // per stage is a multiple of 3 (T = 9), and fa alternates per K-step.
  auto stage = [&](auto bc, int st) __attribute__((always_inline)) {
    constexpr int B = decltype(bc)::value;
    const bool next = st + 1 < se;
    if constexpr (V & 1) {
      if (next) prep(st + 1);  // the DMAs ride on K-step 0's taps
    } else {
      if (next) issue(st + 1, B ^ 1);
    }
    __builtin_amdgcn_sched_barrier(0);
    static_for<KW4>([&](auto jc) {
      constexpr int j = decltype(jc)::value;
      constexpr int ja = (B * KW4 + j) & 1;  // fa set of this K-step
      constexpr bool more = j + 1 < KW4;
      static_for<T>([&](auto tc) {
        constexpr int t = decltype(tc)::value;
        constexpr int gt = B * KW4 * T + j * T + t;  // running tap index over the stage pair
        constexpr int sb3 = gt % 3;
        // wait for tap t (and at t = 0 the K-step's dy): what may stay in flight is the reads
        // issued after them
        if constexpr (t == T - 1) {
          if constexpr (more) wait_lgkm_d<2 * CI_U + 2 * CO_U>();
          else wait_lgkm_d<0>();
        } else if constexpr (t == T - 2 && !more) {
          wait_lgkm_d<2 * CI_U>();
        } else {
          wait_lgkm_d<2 * CI_U>();
        }
        __builtin_amdgcn_sched_barrier(0);
        static_for<CO_U * CI_U>([&](auto uc) {
          constexpr int q = decltype(uc)::value;
          constexpr int m = q / CI_U, u = q % CI_U;
          constexpr int ai = (m * CI_U + u) * T + t;
          mfma_d<(ai < NAGPR_ACC)>(acc[ai], fa[ja][m], fb[sb3][u]);
          if constexpr ((V & 1) && j == 0 && q == 4) {
            static_for<NDMA>([&](auto ic) {
              constexpr int i = decltype(ic)::value;
              if constexpr (i * T / NDMA == t) {
                if (next) issue_one(ic, B ^ 1);
              }
            });
          }
          // the next reads: both x fragments of tap t + 2 after MFMA 1 (64: one after MFMA 1, one
          // after MFMA 3 -- at most two ds_reads per MFMA gap)
          constexpr int q0 = (V & 2) ? 5 : 1;
          if constexpr ((V & 64) ? (q == q0 || q == q0 + 2) : q == q0) {
            constexpr int uu = (V & 64) ? (q - q0) / 2 : -1;
            auto rd = [&](int jj, int tt) __attribute__((always_inline)) {
              if constexpr (uu < 0) read_b((gt + 2) % 3, B, jj, tt);
              else read_bu((gt + 2) % 3, B, jj, tt, uu);
            };
            if constexpr (t + 2 < T) rd(j, t + 2);
            else if (more) rd(j + 1, t + 2 - T);
          }
          if constexpr (q == 3 && t == T - 2) {
            if (more) read_a(ja ^ 1, B, j + 1);
          }
          if constexpr (q == CO_U * CI_U - 1 && t == T - 1) {
            if (dbj[j]) {
#pragma unroll
              for (int mm = 0; mm < CO_U; ++mm) mfma_db(accb[mm], fa[ja][mm], ones);
            }
          }
          __builtin_amdgcn_sched_barrier(0);
        });
      });
    });
    wait_vmcnt<0>();
    block_barrier();
    if (next) {
      constexpr int gt0 = ((B ^ 1) * KW4 * T) % 3;
      read_a(((B ^ 1) * KW4) & 1, B ^ 1, 0);
      read_b(gt0, B ^ 1, 0, 0);
      read_b((gt0 + 1) % 3, B ^ 1, 0, 1);
    }
    __builtin_amdgcn_sched_barrier(0);
  };
  static_assert((2 * G::KW4 * G::T) % 3 == 0 && (2 * G::KW4) % 2 == 0, "set indices repeat over a stage pair");
  int st = sb;
  for (; st + 1 < se; st += 2) {
    stage(std::integral_constant<int, 0>{}, st);
    stage(std::integral_constant<int, 1>{}, st + 1);
  }
  if (st < se) stage(std::integral_constant<int, 0>{}, st);
  asm volatile("s_nop 15\n\ts_nop 15\n\ts_nop 15" ::: "memory");  // inline-asm MFMA results
  static_for<G::NACC>([&](auto ic) {
    constexpr int i = decltype(ic)::value;
    pin_d<(i < NAGPR_ACC)>(acc[i]);
  });
#pragma unroll
  for (int m = 0; m < CO_U; ++m) pin_d<false>(accb[m]);

  // ---- the four waves' partial tiles meet through LDS (both stage buffers are free: the last
  // stage ended with a barrier), CH accumulators at a time so that no more than a few sums are
  // live in VGPRs: every wave writes its CH accumulators (lane l's f32x4 of accumulator i at
  // byte (i - c0) * 1024 + 16 l of the wave's region), then wave w sums accumulators
  // c0 + CH/4 w .. over the four regions and stores them (coalesced 1-KiB rows).
  constexpr int NACC = G::NACC, CH = 24, NCH = NACC / CH, Q = CH / 4, RB = CH * 1024;
  static_assert(NACC % CH == 0 && 4 * RB <= 2 * BUF, "epilogue chunks");
  float *out = ws + (static_cast<long>(split) * npairs + pair) * (NACC * 256) + 4 * lane;
  static_for<NCH>([&](auto cc) {
    constexpr int c0 = decltype(cc)::value * CH;
    static_for<CH>([&](auto ic) {
      constexpr int i = decltype(ic)::value;
      *reinterpret_cast<f32x4 *>(smem + wave * RB + i * 1024 + 16 * lane) = acc[c0 + i];
    });
    block_barrier();
#pragma unroll
    for (int k = 0; k < Q; ++k) {
      const int i = Q * wave + k;
      f32x4 v = *reinterpret_cast<const f32x4 *>(smem + i * 1024 + 16 * lane);
#pragma unroll
      for (int w = 1; w < 4; ++w) v += *reinterpret_cast<const f32x4 *>(smem + w * RB + i * 1024 + 16 * lane);
      *reinterpret_cast<f32x4 *>(out + (c0 + i) * 256) = v;
    }
    block_barrier();
  });
  if (want_db) {
    // every column of the ones-product holds the row sum: lanes of column 0 hand over their 16
    // channels (16 m + 4 g4 + j) per wave, wave 0 sums the four waves and stores 64 partials
    float *sdb = reinterpret_cast<float *>(smem);
    if (l16 == 0) {
#pragma unroll
      for (int m = 0; m < CO_U; ++m)
#pragma unroll
        for (int j = 0; j < 4; ++j) sdb[wave * 64 + 16 * m + 4 * g4 + j] = accb[m][j];
    }
    block_barrier();
    if (wave == 0) {
      const float v = sdb[lane] + sdb[64 + lane] + sdb[128 + lane] + sdb[192 + lane];
      ws[static_cast<long>(gridDim.x) * (NACC * 256) + (static_cast<long>(split) * npairs + pair) * 64 + lane] = v;
    }
  }
}

// dW[co][t][ci] += sum over splits of the partial tiles (fixed order).  Thread = (pair, acc i,
// lane): its f32x4 holds output channels co0 + 16 m + 4 (lane >> 4) + j, input channel ci0 + 16 u +
// (lane & 15), tap t, with i = (m CI_U + u) T + t.
template <int T>
__global__ void __launch_bounds__(256)
conv_wgrad_direct_reduce(const float *__restrict__ ws, float *__restrict__ dw, float *__restrict__ db, int nsplit,
                         int npairs, int nci_b, int nco_b, int Cg, int Cog, float alpha) {
  constexpr int CO_U = 4, CI_U = 2, NACC = CO_U * CI_U * T;
  // the bias-gradient blocks come first (they start with the grid instead of trailing it)
  const int nbb = db != nullptr ? (npairs / nci_b + 3) / 4 : 0;
  if (static_cast<int>(blockIdx.x) < nbb) {
    // bias gradient: wave = (co block of a group); lane = channel; the nsplit x nci_b partial
    // rows are summed in a fixed order with eight loads in flight
    const int gcb = static_cast<int>(blockIdx.x) * 4 + static_cast<int>(threadIdx.x >> 6);  // g * nco_b + cob
    if (gcb >= npairs / nci_b) return;
    const int cl = threadIdx.x & 63;
    const float *pdb = ws + static_cast<long>(nsplit) * npairs * NACC * 256 + static_cast<long>(gcb) * nci_b * 64 + cl;
    const int nr = nsplit * nci_b;  // partial row r = (split r / nci_b, ci block r % nci_b)
    auto row = [&](int r) { return pdb[(static_cast<long>(r / nci_b) * npairs + r % nci_b) * 64]; };
    float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    int r = 0;
    for (; r + 8 <= nr; r += 8) {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] += row(r + e);
    }
    for (int e = 0; r < nr; ++r, ++e) v[e] += row(r);
    const float tot = ((v[0] + v[1]) + (v[2] + v[3])) + ((v[4] + v[5]) + (v[6] + v[7]));
    const int g = gcb / nco_b, cob = gcb - g * nco_b;
    db[g * Cog + cob * 64 + cl] += alpha * tot;
    return;
  }
  const long tid = static_cast<long>(blockIdx.x - nbb) * 256 + threadIdx.x;
  const long total = static_cast<long>(npairs) * NACC * 64;
  if (tid >= total) return;
  const int lane = static_cast<int>(tid & 63);
  const long r = tid >> 6;
  const int i = static_cast<int>(r % NACC);
  const int pair = static_cast<int>(r / NACC);
  f32x4 s = f32x4{0.f, 0.f, 0.f, 0.f};
  const long slab = static_cast<long>(npairs) * NACC * 256;
  const float *p = ws + (static_cast<long>(pair) * NACC + i) * 256 + 4 * lane;
  for (int k = 0; k < nsplit; ++k) s += *reinterpret_cast<const f32x4 *>(p + k * slab);
  const int per_g = nco_b * nci_b;
  const int g = pair / per_g, rem = pair - g * per_g;
  const int cob = rem / nci_b, cib = rem - cob * nci_b;
  const int t = i % T, mu = i / T;
  const int m = mu / CI_U, u = mu - m * CI_U;
  const int ci = cib * 16 * CI_U + 16 * u + (lane & 15);
  const int co = g * Cog + cob * 16 * CO_U + 16 * m + 4 * (lane >> 4);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    float *d = dw + (static_cast<long>(co + j) * T + t) * Cg + ci;
    *d += alpha * s[j];
  }
}

template <int H, int W, int KS, int IPS>
int launch_wd(const bf16_t *x, const bf16_t *dy, float *dw, float *db, float *ws, long ws_floats, int N, int C, int ldy,
              int Cg, int Cog, int groups, int splits, float alpha, hipStream_t s) {
  using G = Wd<H, W, KS, IPS>;
  const int nci_b = Cg / 32, nco_b = Cog / 64;
  const int npairs = groups * nci_b * nco_b;
  const int nstages = (N + IPS - 1) / IPS;
  int S = splits > 0 ? splits : 256 / npairs;
  S = S < 1 ? 1 : (S > nstages ? nstages : S);
  const int per = (nstages + S - 1) / S;
  S = (nstages + per - 1) / per;  // every split holds at least one stage
  const long need = static_cast<long>(S) * npairs * (G::NACC * 256 + 64);
  if (ws_floats < need) return -4;
  // schedule 65 (bits: 1 = the next stage's DMAs ride on K-step 0's taps, 64 = the two x
  // fragments of tap t + 2 issued after MFMAs 1 and 3 of tap t); measured against the plain
  // schedule (DMAs at the stage start, 101.6 -> ~100 / 112 -> 101 us on conv3, r5_wgrad_direct_*)
  CXN_LAUNCH((conv_wgrad_direct<H, W, KS, IPS, 65>), dim3(static_cast<unsigned>(npairs * S)), dim3(256), 0, s, x, dy,
             ws, N, C, ldy, Cg, Cog, npairs, nci_b, nco_b, per, nstages, db != nullptr ? 1 : 0);
  const long blocks = (static_cast<long>(npairs) * G::NACC * 64 + 255) / 256 + (db != nullptr ? (npairs / nci_b + 3) / 4 : 0);
  CXN_LAUNCH((conv_wgrad_direct_reduce<G::T>), dim3(static_cast<unsigned>(blocks)), dim3(256), 0, s, ws, dw, db, S,
             npairs, nci_b, nco_b, Cg, Cog, alpha);
  return 0;
}

// workspace floats for a launch (0 when the shape is not served)
template <int H, int W, int KS, int IPS>
long ws_wd(int N, int Cg, int Cog, int groups, int splits) {
  using G = Wd<H, W, KS, IPS>;
  const int npairs = groups * (Cg / 32) * (Cog / 64);
  const int nstages = (N + IPS - 1) / IPS;
  int S = splits > 0 ? splits : 256 / npairs;
  S = S < 1 ? 1 : (S > nstages ? nstages : S);
  const int per = (nstages + S - 1) / S;
  S = (nstages + per - 1) / per;
  return static_cast<long>(S) * npairs * (G::NACC * 256 + 64);
}

// ---------------------------------------------------------------------------------------------
// Tap-split form for larger maps / kernels (AlexNet conv2: 27 x 27, 5 x 5, 48 input channels
// per group): 25 taps x 64 output channels x 32 input channels would be 200 accumulators per
// wave.  Here a block tile is 16 CO_U output channels x 16 input channels x all taps, and the
// four waves split the TAPS (wave w: taps w, w + 4, ...; 7 / 6 / 6 / 6 of 25) while each walks
// every K-step, so a wave holds CO_U x 7 accumulators and reads CO_U dy + 7 x fragments per
// K-step for 7 CO_U MFMAs.  A stage is a band of R output rows of one image (two bands for
// 27 rows): dy rows of the band (rows past it read zeros, so a band's slots never count a
// neighbour's pixels), x rows of the band plus the halo (rows off the map read zeros: two
// per-lane offset sets, one per band).  LDS images and fragment reads as above
// ([unit][slot][16 ch], ds_read_b64_tr_b16 pairs with the slot permutation of frag_d).
template <int H, int W, int KS, int R, int CO_U, int NWV>
struct Wt {
  static constexpr int P = (KS - 1) / 2, T = KS * KS, PW = W + P;
  static constexpr int NB = (H + R - 1) / R;
  static constexpr int NK = (R * PW + 31) / 32;                    // K-steps per stage
  static constexpr int NKS = NK * 32;
  static constexpr int NX = (NKS + (KS - 1) * (PW + 1) + 31) / 32;
  static constexpr int NXS = NX * 32;
  static constexpr int XLEAD = P * PW + P;
  static constexpr int DYB = CO_U * NKS * 32, XB = NXS * 32, BUF = DYB + XB;
  static constexpr int NQD = CO_U * NK, NQ = NQD + NX, NQW = (NQ + NWV - 1) / NWV;  // DMA pieces
  static constexpr int TPW = (T + 3) / 4;                          // taps per wave
  static constexpr int NP = NWV / 4;                               // K-step interleave (wave groups)
  static constexpr int NJ = (NK + NP - 1) / NP;                    // K-steps per wave and stage
  static constexpr int NACC = CO_U * T;                            // accumulators of a block tile
  static_assert(NWV == 4 || NWV == 8, "waves");
  static_assert(2 * BUF <= 160 * 1024, "LDS");
  static_assert(NB <= 2, "x offset sets");
  static_assert(NJ >= 2, "DMA spread");
};

// NWV = 8: two waves per SIMD; waves w and w + 4 hold the same taps and take alternate K-steps
// (summed through LDS at the end).  A stage's DMAs for the next one are spread over
// this stage's K-steps (one or two after an MFMA) instead of a burst at the stage start.
template <int H, int W, int KS, int R, int CO_U, int NWV>
__global__ void __launch_bounds__(NWV * 64, 1)
conv_wgrad_taps(const bf16_t *__restrict__ x, const bf16_t *__restrict__ dy, float *__restrict__ ws, int N, int C,
                int ldy, int Cg, int Cog, int npairs, int nciu, int ncob, int per, int nstages) {
  using G = Wt<H, W, KS, R, CO_U, NWV>;
  constexpr int T = G::T, NK = G::NK, NKS = G::NKS, PW = G::PW, P = G::P, NP = G::NP, NJ = G::NJ;
  constexpr int BUF = G::BUF, DYB = G::DYB, NQD = G::NQD, NQ = G::NQ, NQW = G::NQW, TPW = G::TPW, NB = G::NB;
  constexpr int HW = H * W;
  __shared__ __attribute__((aligned(1024))) char smem[2 * BUF];
  const uint32_t L = xcd_remap(blockIdx.x, gridDim.x);
  const int pair = static_cast<int>(L % static_cast<uint32_t>(npairs));
  const int split = static_cast<int>(L / static_cast<uint32_t>(npairs));
  const int per_g = ncob * nciu;
  const int g = pair / per_g, rem = pair - g * per_g;
  const int cob = rem / nciu, ciu = rem - cob * nciu;
  const int ci0 = g * Cg + ciu * 16, co0 = g * Cog + cob * 16 * CO_U;
  const int sb = split * per, se = min(nstages, sb + per);
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int tg = wave & 3, kpar = wave >> 2;
  const uint32_t lds0 = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(reinterpret_cast<uintptr_t>((lds_void *)smem)));

  // per-lane DMA offsets: piece q = wave + NWV i; q < NQD: dy unit q / NK, slots 32 (q % NK) ..;
  // else x slots 32 (q - NQD) .. (minus the lead); lane: slot lane >> 1, channels 8 (lane & 1) ..
  // x rows are relative to the band's first halo row (band 1) or row 0 (band 0: rows above read 0)
  uint32_t vq[NB][NQW];
#pragma unroll
  for (int bb = 0; bb < NB; ++bb)
#pragma unroll
    for (int i = 0; i < NQW; ++i) {
      const int q = wave + NWV * i;
      uint32_t v = OOB;
      if (q < NQD) {
        const int u = q / NK, sg = q - u * NK;
        const int o = 32 * sg + (lane >> 1), vrow = o / PW, col = o - vrow * PW;
        if (vrow < R && col < W) v = static_cast<uint32_t>(((vrow * W + col) * ldy + 16 * u + 8 * (lane & 1)) * 2);
      } else if (q < NQ) {
        const int lin = 32 * (q - NQD) + (lane >> 1) - G::XLEAD;
        const int vrow = fdiv_floor(lin, PW), col = lin - vrow * PW;
        const int rrel = bb == 0 ? vrow : vrow + P;  // row relative to the x base of this band
        if (rrel >= 0 && col < W) v = static_cast<uint32_t>(((rrel * W + col) * C + 8 * (lane & 1)) * 2);
      }
      vq[bb][i] = v;
    }
  rsrc_t rd, rx;
  int bsel = 0;
  auto prep = [&](int st) __attribute__((always_inline)) {
    const int n = st / NB, band = st - n * NB, r0 = band * R;
    const int xr0 = band == 0 ? 0 : r0 - P;
    const long pd = static_cast<long>(n) * HW + static_cast<long>(r0) * W;
    rd = make_rsrc(dy + pd * ldy + co0, static_cast<uint32_t>((static_cast<long>(H - r0) * W * ldy - co0) * 2));
    const long px = static_cast<long>(n) * HW + static_cast<long>(xr0) * W;
    rx = make_rsrc(x + px * C + ci0, static_cast<uint32_t>((static_cast<long>(H - xr0) * W * C - ci0) * 2));
    bsel = band;
  };
  auto issue_one = [&](int b, auto ic) __attribute__((always_inline)) {
    constexpr int i = decltype(ic)::value;
    const int q = wave + NWV * i;
    const uint32_t off = (NB == 2 && bsel == 1) ? vq[NB - 1][i] : vq[0][i];
    if (q < NQD) dma16d(rd, lds0 + static_cast<uint32_t>(b * BUF + q * 1024), off);
    else if (q < NQ) dma16d(rx, lds0 + static_cast<uint32_t>(b * BUF + DYB + (q - NQD) * 1024), off);
  };

  // fragment read bases (frag_d's slot permutation); A = dy unit m at K-step k: (m NKS + 32 k) 32,
  // B = x at K-step k under tap t: DYB + (32 k + shift(t)) 32
  const int l16 = lane & 15, g4 = lane >> 4;
  int bo[2];
#pragma unroll
  for (int hl = 0; hl < 2; ++hl) {
    const int sl = ((g4 >> 1) << 4) | (hl << 3) | ((g4 & 1) << 2) | (l16 >> 2);
    bo[hl] = sl * 32 + 8 * (l16 & 3);
  }
  f32x4 acc[CO_U][TPW];
#pragma unroll
  for (int m = 0; m < CO_U; ++m)
#pragma unroll
    for (int tt = 0; tt < TPW; ++tt) {
      acc[m][tt] = f32x4{0.f, 0.f, 0.f, 0.f};
      asm volatile("" : "+a"(acc[m][tt]));
    }
  const int ntap = tg + 4 * (TPW - 1) < T ? TPW : TPW - 1;  // this wave's tap count
  bf16x8 fa[2][CO_U], fb[2][TPW];
  constexpr int NR = CO_U + TPW, NM = CO_U * TPW, RS = NM / NR > 0 ? NM / NR : 1;
  auto read_one = [&](const char *buf, int k, auto sc, auto rc) __attribute__((always_inline)) {
    constexpr int st = decltype(sc)::value, r = decltype(rc)::value;
    if constexpr (r < CO_U) {
      const int off = (r * NKS + 32 * k) * 32;
      fa[st][r] = frag_d(buf + bo[0] + off, buf + bo[1] + off);
    } else {
      constexpr int tt = r - CO_U;
      const int t = tg + 4 * tt < T ? tg + 4 * tt : tg;  // (a missing tap reads anything finite)
      const int off = DYB + (32 * k + (t / KS) * PW + (t % KS)) * 32;
      fb[st][tt] = frag_d(buf + bo[0] + off, buf + bo[1] + off);
    }
  };

  if (sb < se) {
    prep(sb);
    static_for<NQW>([&](auto ic) { issue_one(0, ic); });
  }
  for (int st = sb; st < se; ++st) {
    const int b = (st - sb) & 1;
    wait_vmcnt<0>();
    block_barrier();
    const bool more = st + 1 < se;  // the next stage's DMAs land under this one
    if (more) prep(st + 1);
    const char *buf = smem + b * BUF;
    static_for<NR>([&](auto rc) { read_one(buf, kpar, std::integral_constant<int, 0>{}, rc); });
    // this wave's K-steps k = kpar + NP j; register sets alternate with j; DMA piece i goes out in
    // step i (NJ - 1) / NQW (never the last: a wave may have one step fewer)
    static_for<NJ>([&](auto jc) {
      constexpr int j = decltype(jc)::value, s0 = j & 1;
      const int k = kpar + NP * j;
      const bool valid = j < NJ - 1 || k < NK;
      static_for<NM>([&](auto qc) {
        constexpr int q = decltype(qc)::value;
        constexpr int tt = q / CO_U, m = q % CO_U;
        __builtin_amdgcn_sched_barrier(0);
        if (valid && tt < ntap) mfma_d<true>(acc[m][tt], fa[s0][m], fb[s0][tt]);
        static_for<NQW>([&](auto ic) {
          constexpr int i = decltype(ic)::value;
          constexpr int js = i * (NJ - 1) / NQW, first = (js * NQW + NJ - 2) / (NJ - 1);
          if constexpr (js == j && q == 2 * (i - first) + 1) {
            if (more) issue_one(b ^ 1, ic);
          }
        });
        if constexpr (q % RS == RS - 1 && q / RS < NR) {
          if (k + NP < NK) read_one(buf, k + NP, std::integral_constant<int, s0 ^ 1>{}, std::integral_constant<int, q / RS>{});
        }
        if constexpr (q == NM - 1 && NM / RS < NR) {
          if (k + NP < NK)
            static_for<NR - NM / RS>([&](auto rc) {
              read_one(buf, k + NP, std::integral_constant<int, s0 ^ 1>{},
                       std::integral_constant<int, NM / RS + decltype(rc)::value>{});
            });
        }
      });
      __builtin_amdgcn_sched_barrier(0);
    });
    // (no barrier here: the next stage's starts with one, after which its DMAs go into this buffer)
  }
  asm volatile("s_nop 15\n\ts_nop 15\n\ts_nop 15" ::: "memory");
#pragma unroll
  for (int m = 0; m < CO_U; ++m)
#pragma unroll
    for (int tt = 0; tt < TPW; ++tt) pin_d<true>(acc[m][tt]);
  if constexpr (NP == 2) {  // the odd-K-step waves hand their sums to the even ones through LDS
    static_assert(4 * TPW * CO_U * 1024 <= 2 * BUF, "LDS combine");
    block_barrier();  // every wave is done with the stage buffers
    char *cb = smem + (tg * TPW * CO_U) * 1024 + 16 * lane;
    if (kpar == 1) {
#pragma unroll
      for (int tt = 0; tt < TPW; ++tt)
#pragma unroll
        for (int m = 0; m < CO_U; ++m) *reinterpret_cast<f32x4 *>(cb + (tt * CO_U + m) * 1024) = acc[m][tt];
    }
    block_barrier();
    if (kpar == 1) return;
#pragma unroll
    for (int tt = 0; tt < TPW; ++tt)
#pragma unroll
      for (int m = 0; m < CO_U; ++m) acc[m][tt] += *reinterpret_cast<const f32x4 *>(cb + (tt * CO_U + m) * 1024);
  }
  // partial tile: ws[(split npairs + pair)][t][m][lane] (f32x4), this wave's taps
  float *out = ws + (static_cast<long>(split) * npairs + pair) * (G::NACC * 256) + 4 * lane;
#pragma unroll
  for (int tt = 0; tt < TPW; ++tt) {
    const int t = tg + 4 * tt;
    if (t < T) {
#pragma unroll
      for (int m = 0; m < CO_U; ++m) *reinterpret_cast<f32x4 *>(out + (t * CO_U + m) * 256) = acc[m][tt];
    }
  }
}

// dW[co][t][ci] += alpha * sum over split slabs (fixed order); thread = (pair, t, m, lane)
template <int T, int CO_U>
__global__ void __launch_bounds__(256)
conv_wgrad_taps_reduce(const float *__restrict__ ws, float *__restrict__ dw, int nsplit, int npairs, int nciu, int ncob,
                       int Cg, int Cog, float alpha) {
  constexpr int NACC = CO_U * T;
  const long tid = static_cast<long>(blockIdx.x) * 256 + threadIdx.x;
  if (tid >= static_cast<long>(npairs) * NACC * 64) return;
  const int lane = static_cast<int>(tid & 63);
  const long r = tid >> 6;
  const int i = static_cast<int>(r % NACC), pair = static_cast<int>(r / NACC);
  const long slab = static_cast<long>(npairs) * NACC * 256;
  const float *p = ws + (static_cast<long>(pair) * NACC + i) * 256 + 4 * lane;
  f32x4 s = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int k = 0; k < nsplit; ++k) s += *reinterpret_cast<const f32x4 *>(p + k * slab);
  const int per_g = ncob * nciu;
  const int g = pair / per_g, rem = pair - g * per_g;
  const int cob = rem / nciu, ciu = rem - cob * nciu;
  const int t = i / CO_U, m = i - t * CO_U;
  const int ci = ciu * 16 + (lane & 15);
  const int co = g * Cog + cob * 16 * CO_U + 16 * m + 4 * (lane >> 4);
#pragma unroll
  for (int j = 0; j < 4; ++j) dw[(static_cast<long>(co + j) * T + t) * Cg + ci] += alpha * s[j];
}

// splits S (stage ranges) from the request (0: fill ~256 CUs); returns stages per split
template <int H, int W, int KS, int R, int CO_U, int NWV>
int wt_splits(int N, int npairs, int splits, int &S) {
  using G = Wt<H, W, KS, R, CO_U, NWV>;
  const int nstages = N * G::NB;
  S = splits > 0 ? splits : 256 / npairs;
  S = S < 1 ? 1 : (S > nstages ? nstages : S);
  const int per = (nstages + S - 1) / S;
  S = (nstages + per - 1) / per;
  return per;
}

template <int H, int W, int KS, int R, int CO_U, int NWV>
long ws_wt(int N, int Cg, int Cog, int groups, int splits) {
  using G = Wt<H, W, KS, R, CO_U, NWV>;
  const int npairs = groups * (Cg / 16) * (Cog / (16 * CO_U));
  int S;
  wt_splits<H, W, KS, R, CO_U, NWV>(N, npairs, splits, S);
  return static_cast<long>(S) * npairs * G::NACC * 256;
}

template <int H, int W, int KS, int R, int CO_U, int NWV>
int launch_wt(const bf16_t *x, const bf16_t *dy, float *dw, float *ws, long ws_floats, int N, int C, int ldy, int Cg,
              int Cog, int groups, int splits, float alpha, hipStream_t s) {
  using G = Wt<H, W, KS, R, CO_U, NWV>;
  const int nciu = Cg / 16, ncob = Cog / (16 * CO_U);
  const int npairs = groups * nciu * ncob;
  int S;
  const int per = wt_splits<H, W, KS, R, CO_U, NWV>(N, npairs, splits, S);
  if (ws_floats < static_cast<long>(S) * npairs * G::NACC * 256) return -4;
  CXN_LAUNCH((conv_wgrad_taps<H, W, KS, R, CO_U, NWV>), dim3(static_cast<unsigned>(npairs * S)), dim3(NWV * 64), 0, s,
             x, dy, ws, N, C, ldy, Cg, Cog, npairs, nciu, ncob, per, N * G::NB);
  const long blocks = (static_cast<long>(npairs) * G::NACC * 64 + 255) / 256;
  CXN_LAUNCH((conv_wgrad_taps_reduce<G::T, CO_U>), dim3(static_cast<unsigned>(blocks)), dim3(256), 0, s, ws, dw, S,
             npairs, nciu, ncob, Cg, Cog, alpha);
  return 0;
}


}  // namespace

// Served: stride 1, "same" padding (pad = (K - 1) / 2); K = 3 on 13 x 13 or 14 x 14 maps with input channels
// per group a multiple of 32, or K = 5 on 27 x 27 maps (no db) with a multiple of 16; output
// channels per group a multiple of 64; x / dy pixel strides (C,
// ldy) multiples of 8.  ws == nullptr: returns the workspace size in floats (0: not served).
// Otherwise launches the kernel and the split reduction into dw (fp32 [Cout][K][K][Cg], +=
// alpha * gradient) and, when db is given, the bias gradient (fp32 [Cout], += alpha * sum of dy
// over pixels); -1 when not served, -4 when ws is too small.
CXN_API long cxn_conv_wgrad_direct(const void *x, const void *dy, float *dw, float *db, float *ws, long ws_floats,
                                   int N, int H,
                                   int W, int C, int ldy, int Cg, int Cog, int groups, int KH, int KW, int pad_h,
                                   int pad_w, int stride, int splits, float alpha, void *stream) {
  if (stride != 1 || KH != KW || pad_h != pad_w || pad_h != (KH - 1) / 2) return ws ? -1 : 0;
  if (Cg % 16 || Cog % 64 || C % 8 || ldy % 8 || groups < 1 || C < groups * Cg || ldy < groups * Cog) return ws ? -1 : 0;
  if (KH == 3 && Cg % 32) return ws ? -1 : 0;
  if (static_cast<long>(N) * H * W * (C > ldy ? C : ldy) >= (1L << 30)) return ws ? -1 : 0;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const bf16_t *xb = static_cast<const bf16_t *>(x), *dyb = static_cast<const bf16_t *>(dy);
  if (KH == 5 && H == 27 && W == 27 && db == nullptr && Cg % 16 == 0 && Cog % 64 == 0) {  // tap-split form (conv2)
    // eight waves (2 per SIMD, K-steps alternating) over four: 119 vs 141 us at AlexNet b256
    if (!ws) return ws_wt<27, 27, 5, 14, 4, 8>(N, Cg, Cog, groups, splits);
    const int rc = launch_wt<27, 27, 5, 14, 4, 8>(xb, dyb, dw, ws, ws_floats, N, C, ldy, Cg, Cog, groups, splits, alpha, s);
    if (rc != 0) return rc;
    return hipGetLastError() == hipSuccess ? 0 : -3;
  }
  if (KH == 3 && H == 13 && W == 13) {
    if (!ws) return ws_wd<13, 13, 3, 2>(N, Cg, Cog, groups, splits);
    const int rc = launch_wd<13, 13, 3, 2>(xb, dyb, dw, db, ws, ws_floats, N, C, ldy, Cg, Cog, groups, splits, alpha, s);
    if (rc != 0) return rc;
    return hipGetLastError() == hipSuccess ? 0 : -3;
  }
  if (KH == 3 && H == 14 && W == 14) {  // (VGG-16 conv5_x, GoogLeNet 4c / 4e): one image per stage
    if (!ws) return ws_wd<14, 14, 3, 1>(N, Cg, Cog, groups, splits);
    const int rc = launch_wd<14, 14, 3, 1>(xb, dyb, dw, db, ws, ws_floats, N, C, ldy, Cg, Cog, groups, splits, alpha, s);
    if (rc != 0) return rc;
    return hipGetLastError() == hipSuccess ? 0 : -3;
  }
  return ws ? -1 : 0;
}

