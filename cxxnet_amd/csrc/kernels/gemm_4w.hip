// One-wave-per-SIMD bf16 MFMA GEMM for gfx950 with address-free DMA issue (tile ids 110-115).
//
// Same contract as gemm_glds.hip: C[j][i] (+)= alpha * sum_k A(i,k) B(j,k), A K-major (weights,
// fc operands), B K-major or an implicit-im2col gather of an NHWC activation (conv forward /
// stride-1 data-gradient).
//
// Why this kernel.  The 8-wave tiles park a third of their wave cycles at barriers (two waves
// per SIMD meet at every one), and round 3's one-wave-per-SIMD tile still issued 62 VALU per 128
// MFMAs: every LDS-DMA recomputed its global address (add + bounds select) and all 16 row
// offsets were bumped each K-tile.  A 16x16x32 MFMA holds the SIMD's issue for 8 of its 16
// cycles, so that address math competes with the MFMAs.  Here the loop issues NO vector
// arithmetic for its DMAs:
//   * every lane's DMA offsets are fixed for the whole K loop (row * ld + swizzled chunk, or an
//     out-of-range sentinel for rows past the operand), computed once;
//   * the K-tile advance moves the buffer DESCRIPTOR: its base steps by 128 bytes per K-tile
//     and its record count shrinks by the same amount (scalar arithmetic); K-tiles past the
//     slice get a zero-record descriptor, so their DMAs are dummies that read zeros and keep
//     the vmcnt bookkeeping constant;
//   * gathers (conv): with Cg % 64 == 0 a K-tile lies inside ONE kernel tap (kh, kw) and one
//     64-channel block, both wave-uniform: the tap's pixel shift goes into the descriptor base,
//     and the per-row padding test is one bit of a per-row tap mask computed once
//     (2 VALU per DMA: extract the bit, or it into bit 31 of the offset);
//   * the loop body is unrolled over the two LDS stages, so every ds_read address is a fixed
//     base register plus an immediate.
// Schedule of one K-tile t (stage S = t & 1; F0 / F1 = fragments of k-steps 0 / 1; the DMAs of
// tile t+1 were issued one K-tile earlier into stage S^1):
//   [A] k-step-0 MFMAs, the first NF carrying one ds_read of F1 (stage S) each
//       lgkmcnt(0), barrier                       -> every wave is done reading stage S
//   [B] the remaining k-step-0 and most k-step-1 MFMAs, with the DMAs of tile t+2 into stage S
//       spread evenly over them
//       vmcnt(NA + NB), barrier                   -> tile t+1 landed in stage S^1 for every wave
//   [C] the last k-step-1 MFMAs, the first NF carrying one ds_read of F0 of tile t+1 (stage S^1)
// so a DMA has ~one K-tile of MFMAs to land, and each fragment set is read one k-step ahead.
// MF = 32 selects v_mfma_f32_32x32x16_bf16 (four k-steps of 16 per K-tile, f32x16 accumulators)
// instead of 16x16x32.
// Reference: src/layer/convolution_layer-inl.hpp:70-155, src/layer/fullc_layer-inl.hpp:101-130.
#include "gemm_glds_common.h"

using namespace cxg;

namespace {

// One 1-KiB LDS-DMA (16 bytes per lane) through a descriptor built from (base, records).  A free
// function on purpose: with the builtin called directly inside the kernel's lambdas, hipcc's host
// pass silently dropped the kernel's launch stub (undefined __device_stub__ at load time).
__device__ __forceinline__ void lds_dma16(const char *p, uint32_t n, char *dst, uint32_t voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(make_rsrc(p, n), (lds_void *)dst, 16, voff, 0, 0, 0);
}

template <int N>
__device__ __forceinline__ void wait_lgkm() {
  asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(N) : "memory");
}

// MFMA with the accumulator pinned in its AGPRs ("+a"): the builtin let hipcc rotate the
// loop-carried accumulators through other registers.  Hazards hipcc does not pad for inline asm:
// the A/B operands come only from ds_read (waited with lgkmcnt; benchmarks/asm_audit.py checks
// that no VALU writes them in the loop); the reads of the accumulators after the loop are padded.
__device__ __forceinline__ void mfma16(f32x4 &acc, const bf16x8 &a, const bf16x8 &b) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
}
__device__ __forceinline__ void mfma32(f32x16 &acc, const bf16x8 &a, const bf16x8 &b) {
  asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
}

template <int MF>
struct Acc;
template <>
struct Acc<16> {
  typedef f32x4 T;
};
template <>
struct Acc<32> {
  typedef f32x16 T;
};

template <int BM, int BN, int BMODE, int EPI, int MF>
__global__ void __launch_bounds__(256, 1)
gemm_4f(GOperand A, GOperand B, GEpi E, int tiles_i, int tiles_j, int ksplit_tiles, int ktiles_total) {
  constexpr int NW = 4, WM = BM / 2, WN = BN / 2;
  constexpr int MR = WM / MF, NR = WN / MF;  // MFMA blocks per wave
  constexpr int KS = 64 / (MF == 16 ? 32 : 16);  // k-steps per K-tile
  constexpr int NA = BM / 32, NB = BN / 32;       // 1-KiB DMAs per wave per K-tile
  constexpr int NQ = NA + NB;
  constexpr int A_BYTES = BM * 128, STAGE = (BM + BN) * 128;
  constexpr int PER = MR * NR;      // MFMAs per k-step
  constexpr int T = KS * PER;       // MFMAs per K-tile
  constexpr int NF = MR + NR;       // fragment reads per k-step
  // [A] / [C] lengths: the reads of one k-step one per MFMA plus a tail for them to land
  constexpr int LA = NF + 10 < PER ? NF + 10 : PER;
  constexpr int LC = NF + 6 < PER ? NF + 6 : PER;
  constexpr int LB = T - LA - LC;
  static_assert(NF <= LA && NF <= LC && LA + LC <= T, "schedule");
  // DMA q of tile t+2 rides in front of MFMA dslot(q): spread over [B] when it has an MFMA per
  // DMA (the large tiles), else over [B] and [C] (small tiles: stage S is free from the first
  // barrier on); the second barrier then waits for tile t+1 with vmcnt(NQB), the DMAs of tile
  // t+2 issued before it
  constexpr int DSPAN = LB >= NQ ? LB : T - LA;
  constexpr int NQB = [&]() constexpr {
    int n = 0;
    for (int q = 0; q < NQ; ++q) n += (LA + q * DSPAN / NQ) < T - LC;
    return n;
  }();
  static_assert(NW * MF * (WM + 4) * 4 <= 2 * STAGE, "epilogue staging fits");
  using AccT = typename Acc<MF>::T;
  __shared__ __attribute__((aligned(1024))) char smem[2 * STAGE];

  const uint32_t ntile = static_cast<uint32_t>(tiles_i) * tiles_j;
  const GemmBlock wb = gemm_block(ntile);
  const int g = wb.g;
  int ti, tj;
  tile_ij(wb.tile, tiles_i, tiles_j, E.group_i, ti, tj);
  const int i0 = ti * BM, j0 = tj * BN;
  const int kt_beg = wb.slice * ksplit_tiles;
  const int kt_end = min(kt_beg + ksplit_tiles, ktiles_total);
  if (kt_beg >= kt_end) return;
  const int nt = kt_end - kt_beg;

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wave >> 1, wc = wave & 1;
  // DMA s of a wave fills LDS rows 8 (wave + 4 s) + lane / 8 of the operand tile; the 16-byte
  // chunk lane & 7 of that row holds logical chunk lchunk (XOR swizzle, applied at the source)
  const int lchunk = (lane & 7) ^ (((wave & 1) << 2) + (lane >> 4));
  const uint32_t goA = static_cast<uint32_t>(g * A.gstride) * 2u;
  const uint32_t goB = static_cast<uint32_t>(g * B.gstride) * 2u;

  uint32_t offA[NA], offB[NB], invB[NB];
#pragma unroll
  for (int s = 0; s < NA; ++s) {
    const int r = i0 + 8 * (wave + 4 * s) + (lane >> 3);
    offA[s] = r < A.rows ? goA + static_cast<uint32_t>(r * A.ld) * 2u + lchunk * 16u : OOB;
  }
#pragma unroll
  for (int s = 0; s < NB; ++s) {
    const int r = j0 + 8 * (wave + 4 * s) + (lane >> 3);
    if constexpr (BMODE == K_DIRECT) {
      offB[s] = r < B.rows ? goB + static_cast<uint32_t>(r * B.ld) * 2u + lchunk * 16u : OOB;
      invB[s] = 0;
    } else {
      uint32_t off = OOB, inv = 0xffffffffu;
      if (r < B.rows) {
        const uint32_t n = fdiv(static_cast<uint32_t>(r), B.fd_hw);
        const uint32_t rem = static_cast<uint32_t>(r) - n * static_cast<uint32_t>(B.Ho * B.Wo);
        const uint32_t ho = fdiv(rem, B.fd_wo);
        const uint32_t wo = rem - ho * B.Wo;
        const int hb = static_cast<int>(ho) * B.stride, wbse = static_cast<int>(wo) * B.stride;
        off = goB + static_cast<uint32_t>(((static_cast<int>(n) * B.H + hb) * B.W + wbse) * B.C) * 2u + lchunk * 16u;
        // bit (kh * KW + kw) clear <=> input pixel (hb - pad_h + kh, wb - pad_w + kw) inside the image
        for (int kh = 0, tap = 0; kh < B.KH; ++kh) {
          const bool hin = static_cast<unsigned>(hb - B.pad_h + kh) < static_cast<unsigned>(B.H);
          for (int kw = 0; kw < B.KW; ++kw, ++tap) {
            const bool in = hin && static_cast<unsigned>(wbse - B.pad_w + kw) < static_cast<unsigned>(B.W);
            if (in) inv &= ~(1u << tap);
          }
        }
      }
      offB[s] = off;
      invB[s] = inv;
    }
  }

  // Descriptor of K-tile t (relative to the slice): base and record count, scalar arithmetic only
  struct Desc {
    const char *p;
    uint32_t n;
    uint32_t tap;  // gather: the K-tile's tap index kh * KW + kw
  };
  auto descA = [&](int t) __attribute__((always_inline)) -> Desc {
    const int kt = kt_beg + t;
    const bool in = kt < kt_end;
    const uint32_t step = in ? static_cast<uint32_t>(kt) * 128u : 0u;
    return {reinterpret_cast<const char *>(A.ptr) + step, in ? A.nbytes - step : 0u, 0u};
  };
  // B: K_DIRECT as A; gather: the tap and channel block of the K-tile (Cg % 64 == 0)
  auto descB = [&](int t) __attribute__((always_inline)) -> Desc {
    const int kt = kt_beg + t;
    const bool in = kt < kt_end;
    if constexpr (BMODE == K_DIRECT) {
      const uint32_t step = in ? static_cast<uint32_t>(kt) * 128u : 0u;
      return {reinterpret_cast<const char *>(B.ptr) + step, in ? B.nbytes - step : 0u, 0u};
    } else {
      const uint32_t k0 = in ? static_cast<uint32_t>(kt) * 64u : 0u;
      const uint32_t q = fdiv(k0, B.fd_cg);  // tap index kh * KW + kw
      const int c0 = static_cast<int>(k0 - q * static_cast<uint32_t>(B.Cg));
      const uint32_t kh = fdiv(q, B.fd_kw);
      const int kw = static_cast<int>(q - kh * static_cast<uint32_t>(B.KW));
      const int shift = (((static_cast<int>(kh) - B.pad_h) * B.W + (kw - B.pad_w)) * B.C + c0) * 2;
      return {reinterpret_cast<const char *>(B.ptr) + shift,
              in ? static_cast<uint32_t>(static_cast<int>(B.nbytes) - shift) : 0u, q};
    }
  };
  auto voffB = [&](int s, uint32_t tap) __attribute__((always_inline)) -> uint32_t {
    if constexpr (BMODE == K_DIRECT) {
      return offB[s];
    } else {
      return offB[s] | (((invB[s] >> tap) & 1u) << 31);
    }
  };
  auto dmaA = [&](const char *p, uint32_t n, int stage, int s) __attribute__((always_inline)) {
    lds_dma16(p, n, smem + stage * STAGE + (wave + NW * s) * 1024, offA[s]);
  };
  auto dmaB = [&](const char *p, uint32_t n, uint32_t tap, int stage, int s) __attribute__((always_inline)) {
    lds_dma16(p, n, smem + stage * STAGE + A_BYTES + (wave + NW * s) * 1024, voffB(s, tap));
  };

  // fragment read bases: row (lane & 15) [16x16x32] or (lane & 31) [32x32x16] of a fragment
  // block, swizzled chunk of k-step kk
  const char *pa = smem + wr * WM * 128;
  const char *pb = smem + A_BYTES + wc * WN * 128;
  auto frag_off = [&](int kk) __attribute__((always_inline)) -> int {
    if constexpr (MF == 16) {
      const int row = lane & 15;
      const int ch = ((kk >> 3) + (lane >> 4)) ^ (row >> 1);
      return row * 128 + ch * 16;
    } else {
      const int row = lane & 31;
      const int ch = ((kk >> 3) + (lane >> 5)) ^ ((row >> 1) & 7);
      return row * 128 + ch * 16;
    }
  };

  AccT acc[MR][NR];
#pragma unroll
  for (int m = 0; m < MR; ++m)
#pragma unroll
    for (int n = 0; n < NR; ++n) acc[m][n] = AccT{};

  // one fragment set per k-step (16x16x32: 2 sets of 16 fragments; 32x32x16: 4 sets of 8)
  bf16x8 fa[KS][MR], fb[KS][NR];
  auto read_frag = [&](int set, int f, int stage, int kk) __attribute__((always_inline)) {
    const int o = frag_off(kk);
    if (f < MR)
      fa[set][f] = *reinterpret_cast<const bf16x8 *>(pa + stage * STAGE + f * MF * 128 + o);
    else
      fb[set][f - MR] = *reinterpret_cast<const bf16x8 *>(pb + stage * STAGE + (f - MR) * MF * 128 + o);
  };
  auto mma = [&](int set, int u) __attribute__((always_inline)) {
    const int m = u / NR, n = u % NR;
    if constexpr (MF == 16)
      mfma16(acc[m][n], fa[set][m], fb[set][n]);
    else
      mfma32(acc[m][n], fa[set][m], fb[set][n]);
  };

  // prologue: tiles 0 and 1 in flight, tile 0 landed everywhere, k-step 0 of tile 0 read
  {
    const Desc a0 = descA(0), b0 = descB(0), a1 = descA(1), b1 = descB(1);
#pragma unroll
    for (int s = 0; s < NA; ++s) dmaA(a0.p, a0.n, 0, s);
#pragma unroll
    for (int s = 0; s < NB; ++s) dmaB(b0.p, b0.n, b0.tap, 0, s);
#pragma unroll
    for (int s = 0; s < NA; ++s) dmaA(a1.p, a1.n, 1, s);
#pragma unroll
    for (int s = 0; s < NB; ++s) dmaB(b1.p, b1.n, b1.tap, 1, s);
  }
  wait_vmcnt<NQ>();
  block_barrier();
#pragma unroll
  for (int f = 0; f < NF; ++f) read_frag(0, f, 0, 0);
  __builtin_amdgcn_sched_barrier(0);

  // One K-tile in stage ST.  MFMA number v of the tile (0 .. T-1) is k-step v / PER, block v % PER.
  // [A] carries the reads of k-steps 1 .. KS-1 (NRA of them), spread over its first LA - TA MFMAs
  // (TA MFMAs left for the last ones to land); [C] carries the NF reads of k-step 0 of tile t+1.
  constexpr int NRA = (KS - 1) * NF;
  constexpr int TA = MF == 16 ? 8 : 4;
  auto ktile = [&](auto stc, int t) __attribute__((always_inline)) {
    constexpr int ST = decltype(stc)::value;
    wait_lgkm<0>();  // fragments of k-step 0
    __builtin_amdgcn_sched_barrier(0);
    static_for<T>([&](auto vc) {
      constexpr int v = decltype(vc)::value;
      constexpr int ks = v / PER, u = v % PER;
      if constexpr (v == LA) {
        // [A] -> [B]: the reads of k-step 1 are in; every wave is done with stage ST
        wait_lgkm<0>();
        block_barrier();
      }
      if constexpr (v == T - LC) {
        // [B] -> [C]: this wave's DMAs of tile t+1 (older than the NQB of tile t+2) have landed
        wait_vmcnt<NQB>();
        block_barrier();
      }
      if constexpr (v >= LA) {
        // DMA q of tile t+2 in front of MFMA dslot(q)
        static_for<NQ>([&](auto qc) {
          constexpr int q = decltype(qc)::value;
          if constexpr (v == LA + q * DSPAN / NQ) {
            if constexpr (q < NA) {
              const Desc d = descA(t + 2);
              dmaA(d.p, d.n, ST, q);
            } else {
              const Desc d = descB(t + 2);
              dmaB(d.p, d.n, d.tap, ST, q - NA);
            }
          }
        });
      }
      mma(ks, u);
      // reads riding on this MFMA
      if constexpr (v < LA) {
        static_for<NRA>([&](auto rc) {
          constexpr int r = decltype(rc)::value;
          if constexpr (r * (LA - TA) / NRA == v)
            read_frag(1 + r / NF, r % NF, ST, (1 + r / NF) * (64 / KS));  // [A]: k-steps 1.. of tile t
        });
      } else if constexpr (v >= T - LC && v < T - LC + NF) {
        read_frag(0, v - (T - LC), ST ^ 1, 0);  // [C]: k-step 0 of tile t+1
      }
      __builtin_amdgcn_sched_barrier(0);
    });
  };

  // two K-tiles (both stages) per trip, so every LDS address is a base register + an immediate;
  // an odd last K-tile runs after the loop (a branch inside the loop made hipcc spill the
  // accumulators at the join)
  int t = 0;
  for (; t + 1 < nt; t += 2) {
    ktile(std::integral_constant<int, 0>{}, t);
    ktile(std::integral_constant<int, 1>{}, t + 1);
  }
  if (t < nt) ktile(std::integral_constant<int, 0>{}, t);
  // results of the last MFMAs are read by compiler code below: XDL passes -> wait states
  asm volatile("s_nop 15\n\ts_nop 15\n\ts_nop 15" ::: "memory");
  wait_vmcnt<0>();
  wait_lgkm<0>();
  __syncthreads();  // the epilogue reuses the stage buffers

  if constexpr (MF == 16) {
    seg_epilogue<EPI, MR, NR, WM>(acc, smem, E, g, wb.slice, A.rows, B.rows, i0 + wr * WM, j0 + wc * WN, wave, lane);
  } else {
    // 32x32 block (m, n): the lane holds output column j = lane & 31 and rows i = 8 b + 4 (lane / 32)
    // + e of register 4 b + e: stage 32 j-rows x WM i-columns per n, then write whole rows
    float *ep = reinterpret_cast<float *>(smem) + wave * 32 * (WM + 4);
    float bv8[8];
    staged_bias<WM>(E, g, A.rows, i0 + wr * WM, lane, bv8);
#pragma unroll
    for (int n = 0; n < NR; ++n) {
#pragma unroll
      for (int m = 0; m < MR; ++m)
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          const f32x4 v = {acc[m][n][4 * b], acc[m][n][4 * b + 1], acc[m][n][4 * b + 2], acc[m][n][4 * b + 3]};
          *reinterpret_cast<f32x4 *>(ep + (lane & 31) * (WM + 4) + m * 32 + 8 * b + 4 * (lane >> 5)) = v;
        }
      wait_lgkm<0>();
      wave_lds_handoff<true>();
      write_staged<EPI, 32, WM>(ep, E, g, wb.slice, A.rows, B.rows, i0 + wr * WM, j0 + wc * WN + n * 32, lane, bv8);
      wait_lgkm<0>();
      wave_lds_handoff<true>();
    }
  }
}

template <int BM, int BN, int BMODE, int EPI, int MF>
void launch_4f(const GOperand &A, const GOperand &B, const GEpi &E, int groups, int ksplit, hipStream_t s) {
  const int ti = cdiv(A.rows, BM), tj = cdiv(B.rows, BN);
  const int ktiles = cdiv(A.kdim, BK);
  ksplit = ksplit < 1 ? 1 : (ksplit > ktiles ? ktiles : ksplit);
  const int per = cdiv(ktiles, ksplit);
  ksplit = cdiv(ktiles, per);
  dim3 grid(ti * tj, ksplit, groups);
  CXN_LAUNCH((gemm_4f<BM, BN, BMODE, EPI, MF>), grid, dim3(256), 0, s, A, B, E, ti, tj, per, ktiles);
}

}  // namespace

namespace cxg {
// Operands the address-free loop supports: whole K-tiles (kdim % 64 == 0: no partial tile to
// mask), gathers with whole 64-channel blocks per tap (Cg % 64 == 0), at most 32 taps, unit
// dilation; descriptor ranges that stay below 2^31 after the tap shifts.
static bool fast_ok(int bmode, const GOperand &A, const GOperand &B) {
  if (A.kdim % 64 != 0) return false;
  if (bmode == K_GATHER) {
    if (B.Cg % 64 != 0 || B.KH * B.KW > 32 || B.KH * B.KW * B.Cg != B.kdim) return false;
    const long span = (static_cast<long>(B.KH + B.pad_h) * B.W + B.KW + B.pad_w) * B.C * 2;
    if (static_cast<long>(B.nbytes) + span >= (1L << 31)) return false;
  }
  return true;
}

// 114: 128x128 (16x16x32 MFMA), conv forward / data-gradient gathers
int dispatch_4w(int amode, int bmode, int epi, int tile, const GOperand &A, const GOperand &B, const GEpi &E,
                int groups, int ksplit, hipStream_t s) {
  if (amode != K_DIRECT || !fast_ok(bmode, A, B)) return -1;
#define CX4(BMV, EPV)                                                                \
  if (bmode == BMV && epi == EPV) {                                                  \
    switch (tile) {                                                                  \
      case 114: launch_4f<128, 128, BMV, EPV, 16>(A, B, E, groups, ksplit, s); return 0; \
      default: return -1;                                                            \
    }                                                                                \
  }
  // (tiles 110-113 / 115 -- 256x256 in 16x16x32 and 32x32x16 form, 256x128, 128x256, 64x256 -- and
  // the K_DIRECT instantiations were measured and retired: no table entry uses them,
  // docs/performance.md "MFMA shape")
  CX4(K_GATHER, EPI_BF16)  // conv fwd / dgrad
#undef CX4
  return -1;
}
}  // namespace cxg
