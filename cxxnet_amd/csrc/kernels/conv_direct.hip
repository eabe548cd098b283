// Direct stride-1 "same" convolution for small maps on the gap-slot layout, gfx950: the forward
// y[p][co] = f(sum_{t, ci} W[co][t][ci] x[p + shift(t)][ci] + b[co]), and the data gradient as the
// same forward over dy with the flipped weights (conv_weight_flip), its epilogue applying the relu'
// mask of the node it writes and summing that node's bias gradient.
// Reference: src/layer/convolution_layer-inl.hpp:70-101 (forward: im2col + gemm per group) and
// :139-155 (backward data: gemm + col2im).
//
// Why.  The implicit GEMMs (gemm_glds.hip K_GATHER) rebuild each pixel's im2col address per
// 16-byte load -- 3.5-6 VALU per MFMA on AlexNet conv2-5 (profiles/r5_pmc_alexnet_ops.md) -- and
// fetch every input pixel once per tap through L2.  Here the taps are constant LDS offsets:
//   * Gap slots (as conv_wgrad_direct.hip): every image row is followed by a P-wide zero gap
//     (pitch PW = W + P) and the images of a block are stacked with P zero separator rows.  In
//     that slot space the input under tap (kh, kw) of output slot o is staged slot
//     o + kh * PW + kw, for every slot: padding falls on gap slots, which are zeros.
//   * A block item = IPB whole images x 16 NF output channels of one group.  Its K loop walks
//     the input channels in stages of 32: per stage the block stages the x halo of its images
//     (32 channels, four 8-channel planes [plane][slot][8 ch], 16 B per slot) and the weights of
//     all taps for its channels (one 1-KiB operand image per (tap, 16 channels), lane l's 16 B at
//     16 l), both by LDS-DMA with per-lane source offsets fixed for the whole kernel: per stage
//     only the buffer descriptors move, and slots off the map read zeros through out-of-range
//     offsets.  Every fragment read is one ds_read_b128 at a constant offset from a per-lane base,
//     conflict-free for any tap shift (16 consecutive slots of one plane per 16 lanes).
//   * MFMA v_mfma_f32_16x16x32_bf16 with the weights as A (rows = output channels) and the
//     shifted slots as B (columns = slots), so each lane's accumulator holds 4 consecutive output
//     channels of one slot: the epilogue stores 8 bytes per lane straight from registers (no LDS
//     staging), skipping gap / separator slots.
//   * Four waves, one per SIMD; wave w owns M fragments w * WMF .. of the item's slots and all NF
//     channel fragments: per tap WMF + NF reads for WMF * NF MFMAs.
//   * Persistent: one block per CU walks items L, L + grid, ... (L = XCD-contiguous remap of the
//     block id, so the blocks sharing an item's x or weights share an L2), as one continuous
//     stream of stages: the next stage's DMAs -- the next item's first stage included -- ride on
//     the current stage's taps, and an item's epilogue runs while its successor's first stage
//     lands.
#include "gemm_glds_common.h"

#include <cstdlib>

using namespace cxg;

namespace cxg {
void launch_db_reduce(const GEpi &E, int rows, hipStream_t s);
}

namespace {

// One 1-KiB LDS-DMA (16 bytes per lane), inline asm so that hipcc neither waits for it before the
// current stage's ds_reads nor reorders LDS reads across it; completion is counted by hand
// (wait_vmcnt + barrier at the end of each stage).  M0 is saved and restored in the statement.
__device__ __forceinline__ void dma16c(rsrc_t r, uint32_t lds_addr, uint32_t voff) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(voff), "s"(r), "s"(lds_addr) : "memory");
}

// MFMA on an accumulator pinned to AGPRs: with the builtin, hipcc kept the loop-carried tile in
// VGPRs and copied all of it into AGPRs and back every stage (2 x 96 v_accvgpr moves per stage)
__device__ __forceinline__ void mfma_acc(f32x4 &acc, const bf16x8 &a, const bf16x8 &b) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
}

constexpr int cd_fdiv(int a, int b) { return a >= 0 ? a / b : -((-a + b - 1) / b); }

template <int H, int W, int KS, int IPB, int NF, int NW>
struct Cd {
  static constexpr int P = (KS - 1) / 2, T = KS * KS, PW = W + P, VR = H + P;
  static constexpr int IMG = VR * PW;                             // slots per image
  static constexpr int OS = (IPB * VR - P) * PW;                  // output slots that can hold pixels
  static constexpr int WMF = ((OS + 15) / 16 + NW - 1) / NW;      // M fragments per wave
  static constexpr int MS = 16 * NW * WMF;                        // output slots computed
  static constexpr int NXS = (MS + (KS - 1) * (PW + 1) + 16 * NW - 1) / (16 * NW) * (16 * NW);  // staged x slots
  static constexpr int NXP = NXS / 16;                            // x DMA pieces: 16 slots x 4 planes each
  static constexpr int XB = NXP * 1024;                           // x image bytes
  static constexpr int WB = T * NF * 1024;                        // weight image bytes
  static constexpr int BUF = XB + WB;
  static constexpr int NDX = NXP, ND = NDX + T * NF, NDPW = (ND + NW - 1) / NW;
  static constexpr int XLEAD = P * PW + P;                        // staged slot of linear position 0
  static_assert(2 * BUF <= 160 * 1024, "LDS");
};

// pixel (image-relative: (img H + row) W + col) of a linear slot position, -1 on gap / separator
template <int H, int W, int KS, int IPB>
__device__ __forceinline__ int cd_pixel(int lin) {
  constexpr int P = (KS - 1) / 2, PW = W + P, VR = H + P;
  const int vrow = cd_fdiv(lin, PW) ;
  const int col = lin - vrow * PW;
  const int img = cd_fdiv(vrow, VR);
  const int row = vrow - img * VR;
  if (lin < 0 || img >= IPB || row >= H || col >= W) return -1;
  return (img * H + row) * W + col;
}

struct CdArgs {
  const bf16_t *x;    // NHWC input (pixel stride ldx), group g's channels at g * Cg
  const bf16_t *w;    // [groups * Cog][KS][KS][Cg]
  const float *bias;  // EPI 0: [groups * Cog] or null
  bf16_t *y;          // NHWC output (pixel stride ldy), group g's channels at g * Cog
  float *dbp;         // EPI 2: bias-gradient partial rows [nig * NW][dbp_ld]
  int N, ldx, ldy, Cg, Cog, groups, ncob, nitems, nst, relu, dbp_ld;
};

// EPI 0: + bias, optional relu (a.relu).  EPI 1: data gradient; with a.relu, y *= (y_old > 0)
// (y holds relu(z) on entry).  EPI 2: EPI 1 plus the column sums of the stored values as partial
// rows.
// SB = 0: persistent blocks (one per CU), two LDS stage buffers, the next stage's DMAs under the
// current stage.  SB = 1: one block per item, one stage buffer (64 KiB), two blocks per CU: the
// co-resident block's MFMAs cover a block's DMA waits, barriers, first-tap reads and epilogue.
// NL > 0: NL more waves per block only issue the LDS-DMAs (an LDS-DMA costs its issuing wave
// ~60-185 cycles of issue; on the MFMA waves that was ~17 % of the forward), the NW MFMA waves
// only compute; both kinds meet at the one barrier per stage.
// DBG: compile-time ablation bits used while tuning (1 / 2: skip the x / weight DMAs, 8: skip the
// fragment reads, 16 / 32: skip the MFMAs / epilogue, 64-256: DMA tap spread); 0 in every launch.
template <int H, int W, int KS, int IPB, int NF, int NW, int EPI, int DBG = 0, bool SB = false, int NL = 0>
__global__ void __launch_bounds__(64 * (NW + NL), (SB || NW + NL == 8) ? 2 : 1) conv_direct(CdArgs a) {
  using G = Cd<H, W, KS, IPB, NF, NW>;
  constexpr int T = G::T, WMF = G::WMF, XB = G::XB, BUF = G::BUF;
  constexpr int NDX = G::NDX, ND = G::ND, PW = G::PW, IMG = G::IMG, HW = H * W;
  constexpr int DW = NL > 0 ? NL : NW;  // waves that issue DMAs
  constexpr int NDPW = (ND + DW - 1) / DW;
  static_assert(NDX % DW == 0, "x pieces per wave");
  __shared__ __attribute__((aligned(1024))) char smem[SB ? BUF : 2 * BUF];

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t lds0 =
      __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(reinterpret_cast<uintptr_t>((lds_void *)smem)));
  const int nb = static_cast<int>(gridDim.x);
  const int L = static_cast<int>(xcd_remap(blockIdx.x, gridDim.x));
  const int nmine = SB ? 1 : (L < a.nitems ? (a.nitems - L + nb - 1) / nb : 0);
  const int K = nmine * a.nst;  // stages of this block
  if (K == 0) return;

  const int dwave = NL > 0 ? wave - NW : wave;  // DMA wave index
  // ---- per-lane DMA source offsets (bytes from the stage's descriptor base), fixed for the kernel
  uint32_t voff[NDPW];
#pragma unroll
  for (int i = 0; i < NDPW; ++i) {
    const int q = dwave + DW * i;
    uint32_t v = OOB;
    if (q < NDX) {  // slots 16 q .. 16 q + 15, lane (plane lane >> 4, slot lane & 15)
      const int pix = cd_pixel<H, W, KS, IPB>(16 * q + (lane & 15) - G::XLEAD);
      if (pix >= 0) v = static_cast<uint32_t>((pix * a.ldx + 8 * (lane >> 4)) * 2);
    } else if (q < ND) {
      const int qw = q - NDX, t = qw / NF, f = qw - t * NF;
      v = static_cast<uint32_t>((((16 * f + (lane & 15)) * T + t) * a.Cg + 8 * (lane >> 4)) * 2);
    }
    voff[i] = v;
  }

  auto item_of = [&](int k, int &ig, int &g, int &cob, int &s) __attribute__((always_inline)) {
    const int j = k / a.nst;
    s = k - j * a.nst;
    const int it = L + j * nb;
    const int r = it / a.ncob;
    cob = it - r * a.ncob;
    ig = r / a.groups;
    g = r - ig * a.groups;
  };
  rsrc_t rx, rw;
  // descriptors of stage k; past the last stage (k == K) empty ranges: the DMAs issued for it
  // write zeros into the idle buffer, so the issue needs no branch
  auto prep = [&](int k) __attribute__((always_inline)) {
    if (k >= K) {
      rx = make_rsrc(a.x, 0u);
      rw = make_rsrc(a.w, 0u);
      return;
    }
    int ig, g, cob, s;
    item_of(k, ig, g, cob, s);
    const int n0 = ig * IPB;
    const int nimg = min(IPB, a.N - n0);
    const long cx = static_cast<long>(g) * a.Cg + 32 * s;
    rx = make_rsrc(a.x + static_cast<long>(n0) * HW * a.ldx + cx,
                   static_cast<uint32_t>((static_cast<long>(nimg) * HW * a.ldx - cx) * 2));
    const long co = static_cast<long>(g) * a.Cog + cob * 16 * NF;
    rw = make_rsrc(a.w + co * T * a.Cg + 32 * s, static_cast<uint32_t>((16L * NF * T * a.Cg - 32 * s) * 2));
  };
  // DMA i of this wave is piece q = dwave + DW i: x pieces for i < NDX / DW (NDX is a multiple of
  // DW), weight pieces after them (only the last i may run past ND, for some waves)
  auto issue_one = [&](auto ic, int b) __attribute__((always_inline)) {
    constexpr int i = decltype(ic)::value;
    const int q = dwave + DW * i;
    const uint32_t dst = lds0 + static_cast<uint32_t>(b * BUF + q * 1024);
    if constexpr (i < NDX / DW) {
      if constexpr (!(DBG & 1)) dma16c(rx, dst, voff[i]);
    } else if constexpr (DW * (i + 1) <= ND) {
      if constexpr (!(DBG & 2)) dma16c(rw, dst, voff[i]);
    } else {
      if constexpr (!(DBG & 2)) if (q < ND) dma16c(rw, dst, voff[i]);
    }
  };

  // fragment read bases.  x image: 1-KiB slot groups [16 slots of plane 0][.. plane 1][.. 2][.. 3],
  // 16 B per (slot, plane); lane (plane p = lane >> 4, l16 = lane & 15) of M fragment mi under a
  // tap shift sh = 16 h + r reads slot s = 16 (mi + h) + l16 + r, at byte
  // 1024 (mi + h + ((l16 + r) >> 4)) + 256 p + 16 ((l16 + r) & 15): per-lane offsets for the 16
  // values of r, everything else an immediate.  Weight image (t, f): 16 bytes per lane.
  const int l16 = lane & 15;
  const int xrd = 1024 * wave * WMF + 256 * (lane >> 4);
  auto xoff = [&](int r) __attribute__((always_inline)) {
    return xrd + 1024 * ((l16 + r) >> 4) + 16 * ((l16 + r) & 15);
  };
  const int wrd = XB + 16 * lane;

  f32x4 acc[WMF][NF];
#pragma unroll
  for (int i = 0; i < WMF; ++i)
#pragma unroll
    for (int f = 0; f < NF; ++f) acc[i][f] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto epilogue = [&](int k) __attribute__((always_inline)) {
    int ig, g, cob, s;
    item_of(k, ig, g, cob, s);
    const int n0 = ig * IPB;
    const int c0 = g * a.Cog + cob * 16 * NF + 4 * (lane >> 4);
    int po[WMF];  // element offsets (< 2^30: cxn_conv_direct checks the extent)
    bool ok[WMF];
#pragma unroll
    for (int i = 0; i < WMF; ++i) {
      const int o = 16 * (wave * WMF + i) + (lane & 15);
      const int img = o / IMG, ro = o - img * IMG;
      const int r = ro / PW, c = ro - r * PW;
      ok[i] = img < IPB && r < H && c < W && n0 + img < a.N;
      po[i] = ((n0 + img) * HW + r * W + c) * a.ldy + c0;
    }
    if constexpr (EPI == 0) {
      f32x4 bv[NF];
#pragma unroll
      for (int f = 0; f < NF; ++f)
        bv[f] = a.bias ? f32x4{a.bias[c0 + 16 * f], a.bias[c0 + 16 * f + 1], a.bias[c0 + 16 * f + 2],
                               a.bias[c0 + 16 * f + 3]}
                       : f32x4{0.f, 0.f, 0.f, 0.f};  // (the bias may sit at any offset of the arena)
#pragma unroll
      for (int i = 0; i < WMF; ++i) {
#pragma unroll
        for (int f = 0; f < NF; ++f) {
          f32x4 v = acc[i][f] + bv[f];
          if (a.relu) {
#pragma unroll
            for (int j = 0; j < 4; ++j) v[j] = fmaxf(v[j], 0.f);
          }
          if (ok[i]) *reinterpret_cast<uint2 *>(a.y + po[i] + 16 * f) = make_uint2(pack2(v[0], v[1]), pack2(v[2], v[3]));
        }
      }
    } else {
      f32x4 sum[NF];
#pragma unroll
      for (int f = 0; f < NF; ++f) sum[f] = f32x4{0.f, 0.f, 0.f, 0.f};
      // in halves of the M fragments: each half's old values are all loaded before its first store
      constexpr int HM = (WMF + 1) / 2;
#pragma unroll
      for (int h = 0; h < WMF; h += HM) {
        uint2 old[HM][NF];
#pragma unroll
        for (int i = 0; i < HM; ++i)
#pragma unroll
          for (int f = 0; f < NF; ++f)
            old[i][f] = (a.relu && h + i < WMF && ok[h + i])
                            ? *reinterpret_cast<const uint2 *>(a.y + po[h + i] + 16 * f)
                            : make_uint2(0x3f803f80u, 0x3f803f80u);  // (no mask: all ones)
#pragma unroll
        for (int i = 0; i < HM; ++i) {
          if (h + i >= WMF) continue;
#pragma unroll
          for (int f = 0; f < NF; ++f) {
            const uint2 o2 = old[i][f];
            // relu'(z) from relu(z) > 0: bf16 bits > 0 as signed shorts
            const bool m0 = static_cast<short>(o2.x & 0xffffu) > 0, m1 = static_cast<short>(o2.x >> 16) > 0;
            const bool m2 = static_cast<short>(o2.y & 0xffffu) > 0, m3 = static_cast<short>(o2.y >> 16) > 0;
            const f32x4 v = acc[h + i][f];
            const uint2 pk =
                make_uint2(pack2(m0 ? v[0] : 0.f, m1 ? v[1] : 0.f), pack2(m2 ? v[2] : 0.f, m3 ? v[3] : 0.f));
            if (ok[h + i]) *reinterpret_cast<uint2 *>(a.y + po[h + i] + 16 * f) = pk;
            if constexpr (EPI == 2) {
              if (ok[h + i]) {
                sum[f][0] += __uint_as_float(pk.x << 16);
                sum[f][1] += __uint_as_float(pk.x & 0xffff0000u);
                sum[f][2] += __uint_as_float(pk.y << 16);
                sum[f][3] += __uint_as_float(pk.y & 0xffff0000u);
              }
            }
          }
        }
      }
      if constexpr (EPI == 2) {
        // sum over the 16 slots of a lane group (lane & 15), then lane (lane & 15) == 0 writes the
        // wave's partial row (row = image group x wave, every column written exactly once)
#pragma unroll
        for (int f = 0; f < NF; ++f)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            float v = sum[f][j];
            v += __shfl_xor(v, 1);
            v += __shfl_xor(v, 2);
            v += __shfl_xor(v, 4);
            v += __shfl_xor(v, 8);
            sum[f][j] = v;
          }
        if ((lane & 15) == 0) {
          float *row = a.dbp + static_cast<long>(ig * NW + wave) * a.dbp_ld + c0;
#pragma unroll
          for (int f = 0; f < NF; ++f) *reinterpret_cast<f32x4 *>(row + 16 * f) = sum[f];
        }
      }
    }
  };

  // prologue: the first stage
  if (NL == 0 || wave >= NW) {
    prep(0);
    static_for<NDPW>([&](auto ic) {
      constexpr int i = decltype(ic)::value;
      const int q = dwave + DW * i;
      if (q < ND) dma16c(i < NDX / DW ? rx : rw, lds0 + static_cast<uint32_t>(q * 1024), voff[i]);
    });
  }
  wait_vmcnt<0>();
  block_barrier();
  if constexpr (NL > 0) {
    if (wave >= NW) {  // loader waves: stage k + 1's DMAs during stage k, one barrier per stage
      for (int k = 0; k < K; ++k) {
        if (k + 1 < K) {
          prep(k + 1);
          static_for<NDPW>([&](auto ic) { issue_one(ic, (k + 1) & 1); });
        }
        wait_vmcnt<0>();
        block_barrier();
      }
      return;
    }
  }

  // Per stage: tap t's fragments were read one tap ahead (register sets alternate by tap
  // parity); the reads of tap t + 1 are issued before tap t's MFMAs, and sched_barriers keep the
  // two groups apart, so each tap's 24 MFMAs cover the next tap's LDS latency.  The next stage's
  // DMAs are issued over the first taps and land under the rest of the stage.
  constexpr int DMA_TAPS = (DBG & 64) ? 1 : (DBG & 128) ? 2 : (DBG & 256) ? 6 : (T < 4 ? T : 4);
  bf16x8 xf[2][WMF], wf[2][NF];
  // fragment r of tap t into register set st: r < NF the weight fragment r (every MFMA of the
  // next tap's first row needs them), else the x fragment of M fragment r - NF, in MFMA order
  auto read_one = [&](const char *buf, auto tc, auto sc, auto rc) __attribute__((always_inline)) {
    constexpr int t = decltype(tc)::value, st = decltype(sc)::value, r = decltype(rc)::value;
    constexpr int kh = t / KS, kw = t - kh * KS;
    constexpr int sh = kh * PW + kw;
    if constexpr (r < NF) {
      wf[st][r] = *reinterpret_cast<const bf16x8 *>(buf + wrd + (t * NF + r) * 1024);
    } else {
      xf[st][r - NF] = *reinterpret_cast<const bf16x8 *>(buf + xoff(sh & 15) + 1024 * (r - NF + (sh >> 4)));
    }
  };
  constexpr int NR = WMF + NF;  // fragment reads per tap
  auto stage = [&](int k) __attribute__((always_inline)) {
    const int b = SB ? 0 : (k & 1);
    if constexpr (!SB && NL == 0) prep(k + 1);
    const char *buf = smem + b * BUF;
    static_for<NR>([&](auto rc) { read_one(buf, std::integral_constant<int, 0>{}, std::integral_constant<int, 0>{}, rc); });
    static_for<T>([&](auto tc) {
      constexpr int t = decltype(tc)::value;
      constexpr int st = t & 1;
      // tap t's MFMAs with the NR reads of tap t + 1 spread between them (one per RS MFMAs):
      // clumped, each wave's read burst held its MFMA pipe idle while four waves queued at the LDS
      constexpr int NM = WMF * NF, RS = NM / NR > 0 ? NM / NR : 1;
      static_for<NM>([&](auto qc) {
        constexpr int q = decltype(qc)::value;
        constexpr int i = q / NF, f = q % NF;
        __builtin_amdgcn_sched_barrier(0);
        mfma_acc(acc[i][f], wf[st][f], xf[st][i]);
        if constexpr (!(DBG & 8) && t + 1 < T && q % RS == RS - 1 && q / RS < NR) {
          read_one(buf, std::integral_constant<int, t + 1>{}, std::integral_constant<int, st ^ 1>{},
                   std::integral_constant<int, q / RS>{});
        }
        if constexpr (!(DBG & 8) && t + 1 < T && q == NM - 1 && NM / RS < NR) {  // reads left over
          static_for<NR - NM / RS>([&](auto rc) {
            read_one(buf, std::integral_constant<int, t + 1>{}, std::integral_constant<int, st ^ 1>{},
                     std::integral_constant<int, NM / RS + decltype(rc)::value>{});
          });
        }
      });
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (!SB && NL == 0) {
        static_for<NDPW>([&](auto ic) {
          constexpr int i = decltype(ic)::value;
          if constexpr (i * DMA_TAPS / NDPW == t) issue_one(ic, b ^ 1);
        });
      }
    });
    if constexpr (SB) {  // reload the one buffer once every wave has read it
      if (k + 1 < K) {
        block_barrier();
        prep(k + 1);
        static_for<NDPW>([&](auto ic) { issue_one(ic, 0); });
      }
    }
    if constexpr (!(DBG & 16)) {
      wait_vmcnt<0>();
      asm volatile("" ::: "memory");
      block_barrier();
      asm volatile("" ::: "memory");
    }
  };
  // items outer, stages inner: the accumulators stay in AGPRs across the stage loop (one flat
  // loop with a conditional epilogue made hipcc carry them in VGPRs and copy them every stage)
  for (int j = 0, k = 0; j < nmine; ++j) {
#pragma unroll
    for (int i = 0; i < WMF; ++i)
#pragma unroll
      for (int f = 0; f < NF; ++f) {
        acc[i][f] = f32x4{0.f, 0.f, 0.f, 0.f};
        asm volatile("" : "+a"(acc[i][f]));
      }
    for (int s = 0; s < a.nst; ++s, ++k) stage(k);
    asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");  // the last inline-asm MFMAs' results
#pragma unroll
    for (int i = 0; i < WMF; ++i)
#pragma unroll
      for (int f = 0; f < NF; ++f) asm volatile("" : "+a"(acc[i][f]));
    if constexpr (!(DBG & 32)) epilogue(k - 1);
    else if (a.N < 0) epilogue(k - 1);  // (never: keeps the accumulators live)
  }
}

template <int H, int W, int KS, int IPB, int NF, int NW>
int launch_cd(CdArgs a, int epi, int variant, float *db, hipStream_t s) {
  using G = Cd<H, W, KS, IPB, NF, NW>;
  (void)sizeof(G);
  if (a.Cog % (16 * NF) || a.Cg % 32) return -1;
  const int nig = (a.N + IPB - 1) / IPB;
  a.ncob = a.Cog / (16 * NF);
  a.nitems = nig * a.groups * a.ncob;
  a.nst = a.Cg / 32;
  const int sb = variant == 1;
  const int grid = a.nitems < 256 ? a.nitems : 256;
  const dim3 blk(64 * NW);
  if (variant == 2 && NW == 4) {
    const dim3 b8(64 * (NW + 4));
    if (epi == 0) CXN_LAUNCH((conv_direct<H, W, KS, IPB, NF, NW, 0, 0, false, 4>), dim3(grid), b8, 0, s, a);
    else if (epi == 1) CXN_LAUNCH((conv_direct<H, W, KS, IPB, NF, NW, 1, 0, false, 4>), dim3(grid), b8, 0, s, a);
    else CXN_LAUNCH((conv_direct<H, W, KS, IPB, NF, NW, 2, 0, false, 4>), dim3(grid), b8, 0, s, a);
  } else if (sb && NW == 4) {
    const dim3 g1(a.nitems);
    if (epi == 0) CXN_LAUNCH((conv_direct<H, W, KS, IPB, NF, NW, 0, 0, true>), g1, blk, 0, s, a);
    else if (epi == 1) CXN_LAUNCH((conv_direct<H, W, KS, IPB, NF, NW, 1, 0, true>), g1, blk, 0, s, a);
    else CXN_LAUNCH((conv_direct<H, W, KS, IPB, NF, NW, 2, 0, true>), g1, blk, 0, s, a);
  } else if (epi == 0) {
    CXN_LAUNCH((conv_direct<H, W, KS, IPB, NF, NW, 0>), dim3(grid), blk, 0, s, a);
  } else if (epi == 1) {
    CXN_LAUNCH((conv_direct<H, W, KS, IPB, NF, NW, 1>), dim3(grid), blk, 0, s, a);
  } else {
    CXN_LAUNCH((conv_direct<H, W, KS, IPB, NF, NW, 2>), dim3(grid), blk, 0, s, a);
  }
  if (epi == 2) {
    GEpi E{};
    E.dbias = a.dbp;
    E.part_ld = a.dbp_ld;
    E.dbias_final = db;
    launch_db_reduce(E, nig * NW, s);
  }
  return 0;
}

// ---------------------------------------------------------------------------------------------
// Paired-tap form for larger maps and kernels (AlexNet conv2: 27 x 27, 5 x 5, 48 input channels
// per group).  The K loop walks the input channels in stages of 16 and each MFMA's K = 32 holds
// two (tap, 16 channels) halves: lanes 0-31 read tap 2p, lanes 32-63 tap 2p + 1 (a missing last
// tap reads zero weights), so a stage is ceil(T / 2) MFMA K-steps and any channel count that is a
// multiple of 16 is served.  A block item is a band of R output rows of one image (the halo rows
// above / below come from the same image, rows off the map read zeros) x 16 NF output channels;
// one block per item and one stage buffer, two blocks per CU (as variant 1 above).
//   x image: 16-slot groups [plane 0: 16 slots][plane 1: 16 slots] x 16 B (512 B); one 1-KiB
//     DMA piece fills two groups.  Lane (half h, plane p, l16) of M fragment i under pair q
//     reads slot s = 16 (mi) + l16 + shift(2q + h): byte 512 (mi + (u >> 4)) + 256 p + 16 (u & 15),
//     u = l16 + shift -- a per-lane offset per pair, the fragment index an immediate.
//   weight image (q, f): 1 KiB, lane l's 16 B at 16 l: W[co 16 f + l16][tap 2q + h][8 p ..].
template <int H, int W, int KS, int R, int NF>
struct Cp {
  static constexpr int P = (KS - 1) / 2, T = KS * KS, NPR = (T + 1) / 2, PW = W + P;
  static constexpr int NB = (H + R - 1) / R;                       // bands per image
  static constexpr int OS = R * PW;                                // output slots of a full band
  static constexpr int WMF = ((OS + 15) / 16 + 3) / 4;             // M fragments per wave
  static constexpr int MS = 64 * WMF;
  static constexpr int NXS = (MS + (KS - 1) * (PW + 1) + 31) / 32 * 32;
  static constexpr int NDX = NXS / 32;                             // x DMA pieces
  static constexpr int XB = NXS * 32;
  static constexpr int WB = NPR * NF * 1024;
  static constexpr int BUF = XB + WB;
  static constexpr int ND = NDX + NPR * NF, NDPW = (ND + 3) / 4;
  static constexpr int XLEAD = P * PW + P;
  static_assert(BUF <= 80 * 1024, "two blocks per CU");
};

template <int H, int W, int KS, int R, int NF, int EPI>
__global__ void __launch_bounds__(256, 2) conv_direct_pair(CdArgs a) {
  using G = Cp<H, W, KS, R, NF>;
  constexpr int T = G::T, NPR = G::NPR, WMF = G::WMF, XB = G::XB, BUF = G::BUF, PW = G::PW, P = G::P;
  constexpr int NDX = G::NDX, ND = G::ND, NDPW = G::NDPW, HW = H * W;
  __shared__ __attribute__((aligned(1024))) char smem[BUF];
  const int lane = threadIdx.x & 63, l16 = lane & 15, hl = lane >> 5, pl = (lane >> 4) & 1;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t lds0 =
      __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(reinterpret_cast<uintptr_t>((lds_void *)smem)));
  // item = ((n NB + band) groups + g) ncob + cob
  const int it = static_cast<int>(xcd_remap(blockIdx.x, gridDim.x));
  const int cob = it % a.ncob, r1 = it / a.ncob;
  const int g = r1 % a.groups, r2 = r1 / a.groups;
  const int band = r2 % G::NB, n = r2 / G::NB;
  const int r0 = band * R, nr = min(R, H - r0);

  uint32_t voff[NDPW];
#pragma unroll
  for (int i = 0; i < NDPW; ++i) {
    const int q = wave + 4 * i;
    uint32_t v = OOB;
    if (q < NDX) {
      const int lin = 32 * q + 16 * hl + l16 - G::XLEAD;
      const int vrow = cd_fdiv(lin, PW), col = lin - vrow * PW, row = r0 + vrow;
      if (row >= 0 && row < H && col < W) v = static_cast<uint32_t>(((row * W + col) * a.ldx + 8 * pl) * 2);
    } else if (q < ND) {
      const int qw = q - NDX, pr = qw / NF, f = qw - pr * NF, t = 2 * pr + hl;
      if (t < T) v = static_cast<uint32_t>((((16 * f + l16) * T + t) * a.Cg + 8 * pl) * 2);
    }
    voff[i] = v;
  }
  rsrc_t rx, rw;
  auto prep = [&](int s) __attribute__((always_inline)) {
    const long cx = static_cast<long>(g) * a.Cg + 16 * s;
    rx = make_rsrc(a.x + static_cast<long>(n) * HW * a.ldx + cx, static_cast<uint32_t>((static_cast<long>(HW) * a.ldx - cx) * 2));
    const long co = static_cast<long>(g) * a.Cog + cob * 16 * NF;
    rw = make_rsrc(a.w + co * T * a.Cg + 16 * s, static_cast<uint32_t>((16L * NF * T * a.Cg - 16 * s) * 2));
  };
  auto issue_all = [&]() __attribute__((always_inline)) {
    static_for<NDPW>([&](auto ic) {
      constexpr int i = decltype(ic)::value;
      const int q = wave + 4 * i;
      const uint32_t dst = lds0 + static_cast<uint32_t>(q * 1024);
      if (q < NDX) dma16c(rx, dst, voff[i]);
      else if (q < ND) dma16c(rw, dst, voff[i]);
    });
  };
  auto shift = [](int t) { return (t / KS) * PW + (t % KS); };
  // per-lane x read offset of pair pr (fragment 0 of this wave)
  auto xoffp = [&](int pr) __attribute__((always_inline)) {
    const int t0 = 2 * pr, t1 = 2 * pr + 1 < T ? 2 * pr + 1 : 2 * pr;
    const int u = l16 + (hl ? shift(t1) : shift(t0));
    return 512 * (wave * WMF + (u >> 4)) + 256 * pl + 16 * (u & 15);
  };
  const int wrd = XB + 16 * lane;

  f32x4 acc[WMF][NF];
#pragma unroll
  for (int i = 0; i < WMF; ++i)
#pragma unroll
    for (int f = 0; f < NF; ++f) {
      acc[i][f] = f32x4{0.f, 0.f, 0.f, 0.f};
      asm volatile("" : "+a"(acc[i][f]));
    }
  bf16x8 xf[2][WMF], wf[2][NF];
  auto read_one = [&](auto pc, auto sc, auto rc) __attribute__((always_inline)) {
    constexpr int pr = decltype(pc)::value, st = decltype(sc)::value, r = decltype(rc)::value;
    if constexpr (r < NF) {
      wf[st][r] = *reinterpret_cast<const bf16x8 *>(smem + wrd + (pr * NF + r) * 1024);
    } else {
      xf[st][r - NF] = *reinterpret_cast<const bf16x8 *>(smem + xoffp(pr) + 512 * (r - NF));
    }
  };
  constexpr int NR = WMF + NF, NM = WMF * NF, RS = NM / NR > 0 ? NM / NR : 1;

  prep(0);
  issue_all();
  for (int s = 0; s < a.nst; ++s) {
    wait_vmcnt<0>();
    block_barrier();
    static_for<NR>([&](auto rc) { read_one(std::integral_constant<int, 0>{}, std::integral_constant<int, 0>{}, rc); });
    static_for<NPR>([&](auto pc) {
      constexpr int pr = decltype(pc)::value, st = pr & 1;
      static_for<NM>([&](auto qc) {
        constexpr int q = decltype(qc)::value;
        constexpr int i = q / NF, f = q % NF;
        __builtin_amdgcn_sched_barrier(0);
        mfma_acc(acc[i][f], wf[st][f], xf[st][i]);
        if constexpr (pr + 1 < NPR && q % RS == RS - 1 && q / RS < NR) {
          read_one(std::integral_constant<int, pr + 1>{}, std::integral_constant<int, st ^ 1>{},
                   std::integral_constant<int, q / RS>{});
        }
        if constexpr (pr + 1 < NPR && q == NM - 1 && NM / RS < NR) {
          static_for<NR - NM / RS>([&](auto rc) {
            read_one(std::integral_constant<int, pr + 1>{}, std::integral_constant<int, st ^ 1>{},
                     std::integral_constant<int, NM / RS + decltype(rc)::value>{});
          });
        }
      });
      __builtin_amdgcn_sched_barrier(0);
    });
    if (s + 1 < a.nst) {  // reload the one buffer once every wave has read it
      block_barrier();
      prep(s + 1);
      issue_all();
    }
  }
  asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");
#pragma unroll
  for (int i = 0; i < WMF; ++i)
#pragma unroll
    for (int f = 0; f < NF; ++f) asm volatile("" : "+a"(acc[i][f]));

  // ---- epilogue (as conv_direct): 4 consecutive output channels of one slot per lane
  const int c0 = g * a.Cog + cob * 16 * NF + 4 * (lane >> 4);
  int po[WMF];
  bool ok[WMF];
#pragma unroll
  for (int i = 0; i < WMF; ++i) {
    const int o = 16 * (wave * WMF + i) + l16;
    const int r = o / PW, c = o - r * PW;
    ok[i] = r < nr && c < W;
    po[i] = ((n * H + r0 + r) * W + c) * a.ldy + c0;
  }
  if constexpr (EPI == 0) {
    f32x4 bv[NF];
#pragma unroll
    for (int f = 0; f < NF; ++f)
      bv[f] = a.bias ? f32x4{a.bias[c0 + 16 * f], a.bias[c0 + 16 * f + 1], a.bias[c0 + 16 * f + 2], a.bias[c0 + 16 * f + 3]}
                     : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < WMF; ++i)
#pragma unroll
      for (int f = 0; f < NF; ++f) {
        f32x4 v = acc[i][f] + bv[f];
        if (a.relu) {
#pragma unroll
          for (int j = 0; j < 4; ++j) v[j] = fmaxf(v[j], 0.f);
        }
        if (ok[i]) *reinterpret_cast<uint2 *>(a.y + po[i] + 16 * f) = make_uint2(pack2(v[0], v[1]), pack2(v[2], v[3]));
      }
  } else {
    f32x4 sum[NF];
#pragma unroll
    for (int f = 0; f < NF; ++f) sum[f] = f32x4{0.f, 0.f, 0.f, 0.f};
    constexpr int HM = (WMF + 1) / 2;
#pragma unroll
    for (int h = 0; h < WMF; h += HM) {
      uint2 old[HM][NF];
#pragma unroll
      for (int i = 0; i < HM; ++i)
#pragma unroll
        for (int f = 0; f < NF; ++f)
          old[i][f] = (a.relu && h + i < WMF && ok[h + i]) ? *reinterpret_cast<const uint2 *>(a.y + po[h + i] + 16 * f)
                                                          : make_uint2(0x3f803f80u, 0x3f803f80u);
#pragma unroll
      for (int i = 0; i < HM; ++i) {
        if (h + i >= WMF) continue;
#pragma unroll
        for (int f = 0; f < NF; ++f) {
          const uint2 o2 = old[i][f];
          const bool m0 = static_cast<short>(o2.x & 0xffffu) > 0, m1 = static_cast<short>(o2.x >> 16) > 0;
          const bool m2 = static_cast<short>(o2.y & 0xffffu) > 0, m3 = static_cast<short>(o2.y >> 16) > 0;
          const f32x4 v = acc[h + i][f];
          const uint2 pk = make_uint2(pack2(m0 ? v[0] : 0.f, m1 ? v[1] : 0.f), pack2(m2 ? v[2] : 0.f, m3 ? v[3] : 0.f));
          if (ok[h + i]) *reinterpret_cast<uint2 *>(a.y + po[h + i] + 16 * f) = pk;
          if constexpr (EPI == 2) {
            if (ok[h + i]) {
              sum[f][0] += __uint_as_float(pk.x << 16);
              sum[f][1] += __uint_as_float(pk.x & 0xffff0000u);
              sum[f][2] += __uint_as_float(pk.y << 16);
              sum[f][3] += __uint_as_float(pk.y & 0xffff0000u);
            }
          }
        }
      }
    }
    if constexpr (EPI == 2) {
#pragma unroll
      for (int f = 0; f < NF; ++f)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          float v = sum[f][j];
          v += __shfl_xor(v, 1);
          v += __shfl_xor(v, 2);
          v += __shfl_xor(v, 4);
          v += __shfl_xor(v, 8);
          sum[f][j] = v;
        }
      if (l16 == 0) {
        float *row = a.dbp + static_cast<long>((n * G::NB + band) * 4 + wave) * a.dbp_ld + c0;
#pragma unroll
        for (int f = 0; f < NF; ++f) *reinterpret_cast<f32x4 *>(row + 16 * f) = sum[f];
      }
    }
  }
}

template <int H, int W, int KS, int R, int NF>
int launch_cp(CdArgs a, int epi, float *db, hipStream_t s) {
  using G = Cp<H, W, KS, R, NF>;
  if (a.Cog % (16 * NF) || a.Cg % 16) return -1;
  a.ncob = a.Cog / (16 * NF);
  a.nitems = a.N * G::NB * a.groups * a.ncob;
  a.nst = a.Cg / 16;
  const dim3 grid(a.nitems), blk(256);
  if (epi == 0) CXN_LAUNCH((conv_direct_pair<H, W, KS, R, NF, 0>), grid, blk, 0, s, a);
  else if (epi == 1) CXN_LAUNCH((conv_direct_pair<H, W, KS, R, NF, 1>), grid, blk, 0, s, a);
  else {
    CXN_LAUNCH((conv_direct_pair<H, W, KS, R, NF, 2>), grid, blk, 0, s, a);
    GEpi E{};
    E.dbias = a.dbp;
    E.part_ld = a.dbp_ld;
    E.dbias_final = db;
    launch_db_reduce(E, a.N * G::NB * 4, s);
  }
  return 0;
}

// ---------------------------------------------------------------------------------------------
// Version 2 (tile 203): the paired-tap K walk of conv_direct_pair on persistent blocks of eight
// waves -- two per SIMD, so one wave's LDS-read and DMA-issue stalls are covered by its partner's
// MFMAs (a calibration loop with this fragment pattern: 75 % of the MFMA peak at one wave per
// SIMD, 98 % at two) -- and double-buffered stages, so the next stage's DMAs land under the
// current stage and an item's first stage lands under its predecessor's last.
//   * Waves WM (along the slots) x WN (along the output channels); wave tile WMF x NFW fragments.
//   * An item = IPB images stacked with separator rows (13 x 13) or a band of R virtual rows of
//     one image (27 x 27) x 16 NFW WN output channels of one group.
//   * Stage = (16-channel chunk, group of PPG tap pairs); the chunk's x image stays in its own
//     double buffer for the chunk's NPG stages, the weight image of a stage in a second one.
template <int H, int W, int KS, int IPB, int R, int WM, int WN, int NFW>
struct C2 {
  static constexpr int P = (KS - 1) / 2, T = KS * KS, NPR = (T + 1) / 2, PW = W + P, VR = H + P;
  static constexpr int NB = (IPB * VR - P + R - 1) / R;           // bands per item stack
  static constexpr int MF = (R * PW + 15) / 16;
  static constexpr int WMF = (MF + WM - 1) / WM;
  static constexpr int MS = 16 * WM * WMF;
  static constexpr int NXS = (MS + (KS - 1) * (PW + 1) + 31) / 32 * 32;
  static constexpr int NDX = NXS / 32;                             // x DMA pieces per chunk
  static constexpr int XB = NXS * 32;
  static constexpr int NFB = NFW * WN;                             // channel fragments per block
  static constexpr int PPG_MAX = (160 * 1024 - 2 * XB) / (2 * NFB * 1024);
  static constexpr int NPG = (NPR + PPG_MAX - 1) / PPG_MAX;        // pair groups (stages) per chunk
  static constexpr int PPG = (NPR + NPG - 1) / NPG;                // pairs per stage
  static constexpr int WBF = PPG * NFB * 1024;
  static constexpr int NDW = PPG * NFB;                            // weight DMA pieces per stage
  static constexpr int XLEAD = P * PW + P;
  static constexpr int NDXW = (NDX + 7) / 8, NDWW = (NDW + 7) / 8; // per wave (8 waves)
  static_assert(WM * WN == 8, "eight waves");
  static_assert(PPG_MAX >= 1 && 2 * XB + 2 * WBF <= 160 * 1024, "LDS");
};

template <int H, int W, int KS, int IPB, int R, int WM, int WN, int NFW, int EPI>
__global__ void __launch_bounds__(512, 2) conv_direct2(CdArgs a) {
  using G = C2<H, W, KS, IPB, R, WM, WN, NFW>;
  constexpr int T = G::T, NPR = G::NPR, WMF = G::WMF, XB = G::XB, WBF = G::WBF, PW = G::PW, VR = G::VR;
  constexpr int NPG = G::NPG, PPG = G::PPG, NFB = G::NFB, NDX = G::NDX, NDW = G::NDW, NB = G::NB;
  constexpr int HW = H * W;
  __shared__ __attribute__((aligned(1024))) char smem[2 * XB + 2 * WBF];
  const int lane = threadIdx.x & 63, l16 = lane & 15, hl = lane >> 5, pl = (lane >> 4) & 1;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave % WM, wn = wave / WM;
  const uint32_t lds0 =
      __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(reinterpret_cast<uintptr_t>((lds_void *)smem)));
  const int nb = static_cast<int>(gridDim.x);
  const int L = static_cast<int>(xcd_remap(blockIdx.x, gridDim.x));
  const int nmine = L < a.nitems ? (a.nitems - L + nb - 1) / nb : 0;
  const int SPI = a.nst * NPG;  // stages per item
  const int K = nmine * SPI;
  if (K == 0) return;

  // item = ((ig NB + band) groups + g) ncob + cob
  auto item_of = [&](int j, int &ig, int &band, int &g, int &cob) __attribute__((always_inline)) {
    const int it = L + j * nb;
    cob = it % a.ncob;
    const int r1 = it / a.ncob;
    g = r1 % a.groups;
    const int r2 = r1 / a.groups;
    band = r2 % NB;
    ig = r2 / NB;
  };
  // x DMA offsets per band (NB <= 2: two sets), weight offsets of a stage's pairs (group 0)
  static_assert(NB <= 2, "x offset sets");
  uint32_t vx[NB][G::NDXW], vw[G::NDWW];
#pragma unroll
  for (int bb = 0; bb < NB; ++bb)
#pragma unroll
    for (int i = 0; i < G::NDXW; ++i) {
      const int q = wave + 8 * i;
      uint32_t v = OOB;
      if (q < NDX) {
        const int lin = 32 * q + 16 * hl + l16 - G::XLEAD;
        const int vrow = cd_fdiv(lin, PW), col = lin - vrow * PW;
        const int gv = bb * R + vrow, img = cd_fdiv(gv, VR), row = gv - img * VR;
        if (img >= 0 && img < IPB && row < H && col < W)
          v = static_cast<uint32_t>((((img * H + row) * W + col) * a.ldx + 8 * pl) * 2);
      }
      vx[bb][i] = v;
    }
#pragma unroll
  for (int i = 0; i < G::NDWW; ++i) {
    const int q = wave + 8 * i;
    const int pp = q / NFB, f = q - pp * NFB;
    vw[i] = q < NDW ? static_cast<uint32_t>((((16 * f + l16) * T + 2 * pp + hl) * a.Cg + 8 * pl) * 2) : OOB;
  }

  rsrc_t rx, rw;
  int band_n = 0, npp_n = PPG, pr0_n = 0;  // of the stage being loaded
  bool newx = true;
  auto prep = [&](int k) __attribute__((always_inline)) {
    const int j = k / SPI, r = k - j * SPI, c = r / NPG, h = r - c * NPG;
    int ig, band, g, cob;
    item_of(j, ig, band, g, cob);
    const int n0 = ig * IPB, nimg = min(IPB, a.N - n0);
    const long cx = static_cast<long>(g) * a.Cg + 16 * c;
    rx = make_rsrc(a.x + static_cast<long>(n0) * HW * a.ldx + cx,
                   static_cast<uint32_t>((static_cast<long>(nimg) * HW * a.ldx - cx) * 2));
    const long co = static_cast<long>(g) * a.Cog + cob * 16 * NFB;
    const long wofs = co * T * a.Cg + 16 * c + static_cast<long>(2 * h * PPG) * a.Cg;
    rw = make_rsrc(a.w + wofs, static_cast<uint32_t>((static_cast<long>(16 * NFB) * T * a.Cg - (wofs - co * T * a.Cg)) * 2));
    band_n = band;
    pr0_n = h * PPG;
    npp_n = min(PPG, NPR - h * PPG);
    newx = h == 0;
  };
  // DMAs of stage k (prep'd) into W buffer wb and, at a chunk's first stage, x buffer xb
  auto issue = [&](int wb, int xb) __attribute__((always_inline)) {
    if (newx) {
#pragma unroll
      for (int i = 0; i < G::NDXW; ++i) {
        const int q = wave + 8 * i;
        if (q < NDX) {
          const uint32_t off = (NB == 2 && band_n == 1) ? vx[NB - 1][i] : vx[0][i];
          dma16c(rx, lds0 + static_cast<uint32_t>(xb * XB + q * 1024), off);
        }
      }
    }
#pragma unroll
    for (int i = 0; i < G::NDWW; ++i) {
      const int q = wave + 8 * i;
      const int pp = q / NFB;
      if (q < NDW && pp < npp_n) {
        // the second half of an odd tap count's last pair reads zeros
        const uint32_t off = (2 * (pr0_n + pp) + 1 >= T && hl) ? OOB : vw[i];
        dma16c(rw, lds0 + static_cast<uint32_t>(2 * XB + wb * WBF + q * 1024), off);
      }
    }
  };

  auto shift = [](int t) { return (t / KS) * PW + (t % KS); };
  f32x4 acc[WMF][NFW];
  bf16x8 xf[2][WMF], wf[2][NFW];
  constexpr int NR = WMF + NFW, NM = WMF * NFW, RS = NM / NR > 0 ? NM / NR : 1;

  auto epilogue = [&](int j) __attribute__((always_inline)) {
    int ig, band, g, cob;
    item_of(j, ig, band, g, cob);
    const int n0 = ig * IPB, r0 = band * R;
    const int c0 = g * a.Cog + cob * 16 * NFB + wn * 16 * NFW + 4 * (lane >> 4);
    int po[WMF];
    bool ok[WMF];
#pragma unroll
    for (int i = 0; i < WMF; ++i) {
      const int o = 16 * (wm * WMF + i) + l16;
      const int vrow = o / PW, c = o - vrow * PW;
      const int gv = r0 + vrow, img = gv / VR, row = gv - img * VR;
      ok[i] = vrow < R && img < IPB && n0 + img < a.N && row < H && c < W;
      po[i] = (((n0 + img) * H + row) * W + c) * a.ldy + c0;
    }
    if constexpr (EPI == 0) {
      f32x4 bv[NFW];
#pragma unroll
      for (int f = 0; f < NFW; ++f)
        bv[f] = a.bias ? f32x4{a.bias[c0 + 16 * f], a.bias[c0 + 16 * f + 1], a.bias[c0 + 16 * f + 2],
                               a.bias[c0 + 16 * f + 3]}
                       : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int i = 0; i < WMF; ++i)
#pragma unroll
        for (int f = 0; f < NFW; ++f) {
          f32x4 v = acc[i][f] + bv[f];
          if (a.relu) {
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e], 0.f);
          }
          if (ok[i]) *reinterpret_cast<uint2 *>(a.y + po[i] + 16 * f) = make_uint2(pack2(v[0], v[1]), pack2(v[2], v[3]));
        }
    } else {
      f32x4 sum[NFW];
#pragma unroll
      for (int f = 0; f < NFW; ++f) sum[f] = f32x4{0.f, 0.f, 0.f, 0.f};
      constexpr int HM = 2;  // (two M fragments at a time: registers)
#pragma unroll
      for (int hh = 0; hh < WMF; hh += HM) {
        uint2 old[HM][NFW];
#pragma unroll
        for (int i = 0; i < HM; ++i)
#pragma unroll
          for (int f = 0; f < NFW; ++f)
            old[i][f] = (a.relu && hh + i < WMF && ok[hh + i])
                            ? *reinterpret_cast<const uint2 *>(a.y + po[hh + i] + 16 * f)
                            : make_uint2(0x3f803f80u, 0x3f803f80u);
#pragma unroll
        for (int i = 0; i < HM; ++i) {
          if (hh + i >= WMF) continue;
#pragma unroll
          for (int f = 0; f < NFW; ++f) {
            const uint2 o2 = old[i][f];
            const bool m0 = static_cast<short>(o2.x & 0xffffu) > 0, m1 = static_cast<short>(o2.x >> 16) > 0;
            const bool m2 = static_cast<short>(o2.y & 0xffffu) > 0, m3 = static_cast<short>(o2.y >> 16) > 0;
            const f32x4 v = acc[hh + i][f];
            const uint2 pk =
                make_uint2(pack2(m0 ? v[0] : 0.f, m1 ? v[1] : 0.f), pack2(m2 ? v[2] : 0.f, m3 ? v[3] : 0.f));
            if (ok[hh + i]) *reinterpret_cast<uint2 *>(a.y + po[hh + i] + 16 * f) = pk;
            if constexpr (EPI == 2) {
              if (ok[hh + i]) {
                sum[f][0] += __uint_as_float(pk.x << 16);
                sum[f][1] += __uint_as_float(pk.x & 0xffff0000u);
                sum[f][2] += __uint_as_float(pk.y << 16);
                sum[f][3] += __uint_as_float(pk.y & 0xffff0000u);
              }
            }
          }
        }
      }
      if constexpr (EPI == 2) {
#pragma unroll
        for (int f = 0; f < NFW; ++f)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            float v = sum[f][e];
            v += __shfl_xor(v, 1);
            v += __shfl_xor(v, 2);
            v += __shfl_xor(v, 4);
            v += __shfl_xor(v, 8);
            sum[f][e] = v;
          }
        if (l16 == 0) {  // row = (image group, band) x wave along the slots
          float *row = a.dbp + static_cast<long>((ig * NB + band) * WM + wm) * a.dbp_ld + c0;
#pragma unroll
          for (int f = 0; f < NFW; ++f) *reinterpret_cast<f32x4 *>(row + 16 * f) = sum[f];
        }
      }
    }
  };

  // prologue: stage 0 into W buffer 0 / x buffer 0
  prep(0);
  issue(0, 0);
  wait_vmcnt<0>();
  block_barrier();
  const int wrd = 16 * lane;
  int xbuf = 0;
  for (int j = 0, k = 0; j < nmine; ++j) {
#pragma unroll
    for (int i = 0; i < WMF; ++i)
#pragma unroll
      for (int f = 0; f < NFW; ++f) {
        acc[i][f] = f32x4{0.f, 0.f, 0.f, 0.f};
        asm volatile("" : "+a"(acc[i][f]));
      }
    for (int r = 0; r < SPI; ++r, ++k) {
      const int h = r % NPG;
      const int wb = k & 1;
      if (k + 1 < K) {  // the next stage's DMAs land under this one
        prep(k + 1);
        issue(wb ^ 1, newx ? (xbuf ^ 1) : xbuf);
      }
      const char *xs = smem + xbuf * XB + 512 * (wm * WMF);
      const char *ws = smem + 2 * XB + wb * WBF + wn * NFW * 1024 + wrd;
      const int pr0 = h * PPG, npp = min(PPG, NPR - pr0);
      auto read_one = [&](int pr, int pp, auto sc, auto rc) __attribute__((always_inline)) {
        constexpr int st = decltype(sc)::value, rr = decltype(rc)::value;
        if constexpr (rr < NFW) {
          wf[st][rr] = *reinterpret_cast<const bf16x8 *>(ws + (pp * NFB + rr) * 1024);
        } else {
          const int t0 = 2 * pr, t1 = 2 * pr + 1 < T ? 2 * pr + 1 : 2 * pr;
          const int u = l16 + (hl ? shift(t1) : shift(t0));
          xf[st][rr - NFW] = *reinterpret_cast<const bf16x8 *>(xs + 512 * (rr - NFW + (u >> 4)) + 256 * pl + 16 * (u & 15));
        }
      };
      static_for<NR>([&](auto rc) { read_one(pr0, 0, std::integral_constant<int, 0>{}, rc); });
      // pairs of this stage, two at a time (register sets alternate)
      static_for<PPG>([&](auto pc) {
        constexpr int pp = decltype(pc)::value, st = pp & 1;
        if (pp < npp) {
          static_for<NM>([&](auto qc) {
            constexpr int q = decltype(qc)::value;
            constexpr int i = q / NFW, f = q % NFW;
            __builtin_amdgcn_sched_barrier(0);
            mfma_acc(acc[i][f], wf[st][f], xf[st][i]);
            if constexpr (q % RS == RS - 1 && q / RS < NR) {
              if (pp + 1 < npp)
                read_one(pr0 + pp + 1, pp + 1, std::integral_constant<int, st ^ 1>{}, std::integral_constant<int, q / RS>{});
            }
            if constexpr (q == NM - 1 && NM / RS < NR) {
              if (pp + 1 < npp)
                static_for<NR - NM / RS>([&](auto rc) {
                  read_one(pr0 + pp + 1, pp + 1, std::integral_constant<int, st ^ 1>{},
                           std::integral_constant<int, NM / RS + decltype(rc)::value>{});
                });
            }
          });
          __builtin_amdgcn_sched_barrier(0);
        }
      });
      wait_vmcnt<0>();
      asm volatile("" ::: "memory");
      block_barrier();
      asm volatile("" ::: "memory");
      if (h == NPG - 1) xbuf ^= 1;  // the next chunk's x image
    }
    asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");
#pragma unroll
    for (int i = 0; i < WMF; ++i)
#pragma unroll
      for (int f = 0; f < NFW; ++f) asm volatile("" : "+a"(acc[i][f]));
    epilogue(j);
  }
}

template <int H, int W, int KS, int IPB, int R, int WM, int WN, int NFW>
int launch_c2(CdArgs a, int epi, float *db, hipStream_t s) {
  using G = C2<H, W, KS, IPB, R, WM, WN, NFW>;
  if (a.Cog % (16 * G::NFB) || a.Cg % 16) return -1;
  const int nig = (a.N + IPB - 1) / IPB;
  a.ncob = a.Cog / (16 * G::NFB);
  a.nitems = nig * G::NB * a.groups * a.ncob;
  a.nst = a.Cg / 16;
  const int grid = a.nitems < 256 ? a.nitems : 256;
  if (epi == 0) CXN_LAUNCH((conv_direct2<H, W, KS, IPB, R, WM, WN, NFW, 0>), dim3(grid), dim3(512), 0, s, a);
  else if (epi == 1) CXN_LAUNCH((conv_direct2<H, W, KS, IPB, R, WM, WN, NFW, 1>), dim3(grid), dim3(512), 0, s, a);
  else {
    CXN_LAUNCH((conv_direct2<H, W, KS, IPB, R, WM, WN, NFW, 2>), dim3(grid), dim3(512), 0, s, a);
    GEpi E{};
    E.dbias = a.dbp;
    E.part_ld = a.dbp_ld;
    E.dbias_final = db;
    launch_db_reduce(E, nig * G::NB * WM, s);
  }
  return 0;
}

}  // namespace

// Served: stride 1, "same" padding, K = 3 on 13 x 13 maps with Cg (input channels per group) a
// multiple of 32 and Cog (output channels per group) a multiple of 64; K = 5 on 27 x 27 maps (the
// paired-tap form, every variant id) with Cg a multiple of 16 and Cog a multiple of 64 or 48.
// Pixel strides multiples of 8.
// variant: 0 persistent blocks with two stage buffers, 1 one block per item with one stage
// buffer (two blocks per CU), 2 as 0 with four more waves per block that only issue the LDS-DMAs.
// epi 0: y = conv(x, w) + bias (relu optional).  epi 1: data gradient (x = dy, w = flipped
// weights), with relu = 1 y *= relu'(y_old).  epi 2: epi 1 and db += column sums of the stored y (dbp: a
// workspace of at least dbp_elems floats, db the fp32 bias gradient).  dbp == nullptr with
// epi 2 asks for the workspace size (floats).  Returns -1 when the shape is not served.
CXN_API long cxn_conv_direct(const void *x, int ldx, const void *w, const float *bias, void *y, int ldy, float *dbp,
                             long dbp_elems, float *db, int N, int H, int W, int Cg, int Cog, int groups, int KS,
                             int relu, int epi, int variant, void *stream) {
  const bool pair = KS == 5 && H == 27 && W == 27;  // paired-tap form (AlexNet conv2)
  const bool m14 = KS == 3 && H == 14 && W == 14;    // VGG-16 conv5, GoogLeNet's 14 x 14 3 x 3 convs
  if (!pair && !m14 && (KS != 3 || H != 13 || W != 13)) return -1;
  if (ldx % 8 || ldy % 8 || groups < 1 || ldx < groups * Cg || ldy < groups * Cog) return -1;
  if (pair ? (Cg % 16 || (Cog % 64 && Cog % 48)) : (Cg % 32 || Cog % 64)) return -1;
  if (static_cast<long>(N) * H * W * (ldx > ldy ? ldx : ldy) >= (1L << 30)) return -1;
  constexpr int IPB = 2;
  const long need = pair ? static_cast<long>(N) * 2 * 8 * groups * Cog  // (rows: image band x wave)
                         : static_cast<long>((N + IPB - 1) / IPB) * 8 * groups * Cog;  // (image group x wave)
  if (epi == 2 && dbp == nullptr) return need;
  if (epi == 2 && dbp_elems < need) return -4;
  CdArgs a{};
  a.x = static_cast<const bf16_t *>(x);
  a.w = static_cast<const bf16_t *>(w);
  a.bias = bias;
  a.y = static_cast<bf16_t *>(y);
  a.dbp = dbp;
  a.N = N;
  a.ldx = ldx;
  a.ldy = ldy;
  a.Cg = Cg;
  a.Cog = Cog;
  a.groups = groups;
  a.relu = relu;
  a.dbp_ld = groups * Cog;
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (variant < 0 || variant > 3) return -1;
  int rc;
  if (m14) {
    if (variant == 3) return -1;
    rc = launch_cd<14, 14, 3, IPB, 4, 4>(a, epi, variant, db, s);
  } else if (variant == 3) {  // version 2: eight waves, paired taps, persistent double-buffered stages
    if (pair) {
      rc = Cog % 128 == 0 ? launch_c2<27, 27, 5, 1, 14, 4, 2, 4>(a, epi, db, s)
         : Cog % 48 == 0  ? launch_c2<27, 27, 5, 1, 14, 8, 1, 3>(a, epi, db, s)
                          : -1;
    } else {
      rc = Cog % 128 == 0 ? launch_c2<13, 13, 3, 2, 27, 4, 2, 4>(a, epi, db, s)
         : Cog % 96 == 0  ? launch_c2<13, 13, 3, 2, 27, 4, 2, 3>(a, epi, db, s)
                          : -1;
    }
  } else if (pair) {
    rc = Cog % 64 == 0 ? launch_cp<27, 27, 5, 14, 4>(a, epi, db, s) : launch_cp<27, 27, 5, 14, 3>(a, epi, db, s);
  } else {
    rc = launch_cd<13, 13, 3, IPB, 4, 4>(a, epi, variant, db, s);
  }
  if (rc != 0) return rc;
  return hipGetLastError() == hipSuccess ? 0 : -3;
}
