// One-wave-per-SIMD bf16 MFMA GEMM tiles for gfx950: 4 waves, each owning a (BM/2) x (BN/2)
// block of the output (256 x 256 tile: 128 x 128 per wave, 256 accumulator registers), with
// the fragment reads of the next k-step and the LDS-DMA of the K-tile after next issued in the
// shadow of the current k-step's MFMAs.
//
// Same contract and operand loaders as gemm_glds.hip (C[j][i] (+)= alpha * sum_k A(i,k) B(j,k),
// K-major A and B); tile ids 92-97.
//
// Why this shape: PMC on 8192^3 (profiles/r3_pmc_square_gemm.md) shows hipBLASLt's
// MT256x256x64 kernel at 86 % MFMA utilisation with waves parked 5 % of their cycles, against
// 57 % / 36 % for our 8-wave (two per SIMD) 256 x 256 tile: two co-resident waves that meet at
// every barrier leave the SIMD's matrix pipe idle while both wait.  With one wave per SIMD the
// wave's own instruction stream has to hide every latency, so the loop is software-pipelined:
//   iteration t (K-tile t in LDS buffer t & 1; fragments F0 = k-step 0 of tile t in registers):
//     [A]  ds_read F1 = k-step 1 of tile t           | 64 (MR x NR) MFMAs on F0
//          lgkmcnt(0) (F1 read, so buffer t & 1 is free for this wave), vmcnt(0) (tile t+1's
//          DMAs, issued one half-iteration ago, have landed), s_barrier
//     [B]  ds_read F0 = k-step 0 of tile t+1 (buffer (t+1) & 1)
//          LDS-DMA of tile t+2 into buffer t & 1   | MFMAs on F1
//   so one barrier per K-tile, no wait on an LDS read in front of an MFMA, and a DMA has
//   [B] + [A] (two k-steps of MFMAs) to land.  Past the K slice the DMAs are all-OOB dummies.
// The order is pinned with sched_barrier (hipcc otherwise sinks the reads and DMAs to the end of
// each k-step, where their latency is exposed).  SCHED = 0: [B]'s DMAs are spread evenly over its
// MFMAs; SCHED = 1: one in front of each of the first MFMAs (a burst: more time to land).
// Reference: src/layer/convolution_layer-inl.hpp:70-155, src/layer/fullc_layer-inl.hpp:101-130.
#include "gemm_glds_common.h"

using namespace cxg;

namespace {

// One MFMA row (8 accumulators) as inline asm: with the builtin, hipcc rotated the 256 loop-carried
// accumulators through other AGPRs / VGPRs (352 v_accvgpr_* per 128 MFMAs); the "+a" operand pins
// each accumulator in place.  Hazards hipcc no longer pads (cdna guide 5.7 item 2): the chain
// MFMA D -> next MFMA's C needs none; the A/B operands are written only by ds_read (the loop is
// audited for VALU writes of them: benchmarks/asm_audit.py); the reads of D after the main loop
// are padded there.
__device__ __forceinline__ void mfma_asm(f32x4 &acc, const bf16x8 &a, const bf16x8 &b) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
}

template <int NR>
__device__ __forceinline__ void mfma_row_asm(f32x4 (&acc)[NR], const bf16x8 &a, const bf16x8 (&fb)[NR]) {
#pragma unroll
  for (int n = 0; n < NR; ++n)
    asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc[n]) : "v"(a), "v"(fb[n]));
}

template <int BM, int BN, int AMODE, int BMODE, int EPI, int SCHED>
__global__ void __launch_bounds__(256, 1)
gemm_4w(GOperand A, GOperand B, GEpi E, int tiles_i, int tiles_j, int ksplit_tiles, int ktiles_total) {
  constexpr int NW = 4, WM = BM / 2, WN = BN / 2, MR = WM / 16, NR = WN / 16;
  using OA = Op<AMODE, BM, NW>;
  using OB = Op<BMODE, BN, NW>;
  constexpr int A_BYTES = BM * 128, STAGE = (BM + BN) * 128;
  constexpr int NPT = OA::NI + OB::NI;  // DMA instructions per wave per K-tile
  static_assert(NPT <= (MR - 1) * NR, "every DMA gets an MFMA slot in rows 1.. of [B]");
  static_assert(NW * 16 * (WM + 4) * 4 <= 2 * STAGE, "epilogue staging fits");
  __shared__ __attribute__((aligned(1024))) char smem[2 * STAGE];

  const uint32_t ntile = static_cast<uint32_t>(tiles_i) * tiles_j;
  const GemmBlock wb = gemm_block(ntile);
  const int g = wb.g;
  const uint32_t tile = wb.tile;
  int ti, tj;
  tile_ij(tile, tiles_i, tiles_j, E.group_i, ti, tj);
  const int i0 = ti * BM, j0 = tj * BN;
  const int kt_beg = wb.slice * ksplit_tiles;
  const int kt_end = min(kt_beg + ksplit_tiles, ktiles_total);
  if (kt_beg >= kt_end) return;
  const int nt = kt_end - kt_beg;

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wave >> 1, wc = wave & 1;
  const rsrc_t rA = make_rsrc(A.ptr, A.nbytes);
  const rsrc_t rB = make_rsrc(B.ptr, B.nbytes);
  const uint32_t goA = static_cast<uint32_t>(g * A.gstride) * 2u;
  const uint32_t goB = static_cast<uint32_t>(g * B.gstride) * 2u;
  OA oa;
  OB ob;
  oa.init(A, i0, goA, wave, lane);
  ob.init(B, j0, goB, wave, lane);
  // K_DIRECT operands: DMA s reads rows 32 s further than DMA 0 -- one base register and a
  // stride instead of one row offset per DMA (rows past the operand read zeros (outside the
  // buffer) or rows of the next group, which only feed output rows the epilogue never stores)
  const uint32_t rsA = 32u * static_cast<uint32_t>(A.ld) * 2u, rsB = 32u * static_cast<uint32_t>(B.ld) * 2u;
  const uint32_t baseA = goA + static_cast<uint32_t>((i0 + 8 * wave + (lane >> 3)) * A.ld) * 2u;
  const uint32_t baseB = goB + static_cast<uint32_t>((j0 + 8 * wave + (lane >> 3)) * B.ld) * 2u;
  auto offA = [&](auto sc, const typename OA::Prep &p) __attribute__((always_inline)) -> uint32_t {
    constexpr int s = decltype(sc)::value;
    if constexpr (AMODE == K_DIRECT) {
      uint32_t off = p.kin ? baseA + static_cast<uint32_t>(p.k) * 2u + s * rsA : OOB;
      asm volatile("" : "+v"(off));
      return off;
    } else {
      return oa.template offset<s>(A, p, wave, lane);
    }
  };
  auto offB = [&](auto sc, const typename OB::Prep &p) __attribute__((always_inline)) -> uint32_t {
    constexpr int s = decltype(sc)::value;
    if constexpr (BMODE == K_DIRECT) {
      uint32_t off = p.kin ? baseB + static_cast<uint32_t>(p.k) * 2u + s * rsB : OOB;
      asm volatile("" : "+v"(off));
      return off;
    } else {
      return ob.template offset<s>(B, p, wave, lane);
    }
  };

  // DMA instruction q (0 .. NPT-1) of K-tile t into buffer t & 1: A's NI first, then B's
  auto dma = [&](auto qc, int t, const typename OA::Prep &pa, const typename OB::Prep &pb)
      __attribute__((always_inline)) -> void {
    constexpr int q = decltype(qc)::value;
    char *sa = smem + (t & 1) * STAGE;
    if constexpr (q < OA::NI) {
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rA, (lds_void *)(sa + (wave + NW * q) * 1024), 16,
                                               offA(std::integral_constant<int, q>{}, pa), 0, 0, 0);
    } else {
      constexpr int s = q - OA::NI;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rB, (lds_void *)(sa + A_BYTES + (wave + NW * s) * 1024), 16,
                                               offB(std::integral_constant<int, s>{}, pb), 0, 0, 0);
    }
  };
  auto issue = [&](int t) __attribute__((always_inline)) {
    const int kt = kt_beg + t;
    const typename OA::Prep pa = oa.prep(A, kt, kt_end, goA);
    const typename OB::Prep pb = ob.prep(B, kt, kt_end, goB);
    static_for<NPT>([&](auto qc) { dma(qc, t, pa, pb); });
  };

  f32x4 acc[MR][NR];
#pragma unroll
  for (int m = 0; m < MR; ++m)
#pragma unroll
    for (int n = 0; n < NR; ++n) acc[m][n] = f32x4{0.f, 0.f, 0.f, 0.f};

  // Fragment registers: one A set, refilled row by row right behind its last MFMA, and two B
  // sets that alternate between k-steps (B fragments are used by every MFMA row, so the next
  // k-step's B needs registers of its own): 96 fragment VGPRs next to the 256 accumulators.
  bf16x8 fa[MR], fb0[NR], fb1[NR];
  auto read_a = [&](auto mc, int t, int kk) __attribute__((always_inline)) -> void {
    constexpr int m = decltype(mc)::value;
    fa[m] = frag<K_DIRECT>(smem + (t & 1) * STAGE, wr * WM + m * 16, kk, lane);
  };
  auto read_b = [&](int t, int kk, bf16x8 (&fb)[NR]) __attribute__((always_inline)) -> void {
    const char *sb = smem + (t & 1) * STAGE + A_BYTES;
#pragma unroll
    for (int n = 0; n < NR; ++n) fb[n] = frag<K_DIRECT>(sb, wc * WN + n * 16, kk, lane);
  };
  auto read_b1 = [&](auto nc, int t, int kk, bf16x8 (&fb)[NR]) __attribute__((always_inline)) -> void {
    constexpr int n = decltype(nc)::value;
    fb[n] = frag<K_DIRECT>(smem + (t & 1) * STAGE + A_BYTES, wc * WN + n * 16, kk, lane);
  };
  auto mfma_row = [&](auto mc, const bf16x8 (&fb)[NR]) __attribute__((always_inline)) -> void {
    constexpr int m = decltype(mc)::value;
    mfma_row_asm<NR>(acc[m], fa[m], fb);
  };

  // prologue: tiles 0 and 1 in flight, tile 0 landed for every wave, k-step 0 of tile 0 read
  issue(0);
  issue(1);
  wait_vmcnt<NPT>();
  block_barrier();
  static_for<MR>([&](auto mc) { read_a(mc, 0, 0); });
  read_b(0, 0, fb0);
  // retire them here: left pending into the loop, hipcc's wait for them lands in front of the
  // first MFMA of EVERY iteration (it merges the loop-entry state at the header)
  __builtin_amdgcn_s_waitcnt(0xc07f);
  __builtin_amdgcn_sched_barrier(0);

  for (int t = 0; t < nt; ++t) {
    // [A] k-step 0 of tile t (fa, fb0); reads of k-step 1: fb1 first, fa row by row
    // [A] k-step 0 of tile t (fa, fb0); reads of k-step 1: fb1 one per MFMA of row 0, fa row by
    // row behind each row's last MFMA
    static_for<MR>([&](auto mc) {
      constexpr int m = decltype(mc)::value;
      static_for<NR>([&](auto nc) {
        constexpr int n = decltype(nc)::value;
        mfma_asm(acc[m][n], fa[m], fb0[n]);
        if constexpr (m == 0) read_b1(nc, t, 32, fb1);
        __builtin_amdgcn_sched_barrier(0);
      });
      read_a(mc, t, 32);
      __builtin_amdgcn_sched_barrier(0);
    });
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's reads of buffer t & 1 are done
    wait_vmcnt<0>();                     // tile t + 1 has landed (this wave's DMAs)
    block_barrier();
    // [B] k-step 1 of tile t (fa, fb1); reads of k-step 0 of tile t+1 (fb0 one per MFMA of row 0,
    // fa row by row) and the DMAs of tile t+2 into buffer t & 1 over the remaining MFMAs
    {
      const int kt = kt_beg + t + 2;
      const typename OA::Prep pa = oa.prep(A, kt, kt_end, goA);
      const typename OB::Prep pb = ob.prep(B, kt, kt_end, goB);
      // DMA q goes in front of MFMA number slot(q) of [B] (rows 1..MR-1): spread evenly
      // (SCHED 0) or one per MFMA from the first (SCHED 1)
      static_for<MR>([&](auto mc) {
        constexpr int m = decltype(mc)::value;
        static_for<NR>([&](auto nc) {
          constexpr int n = decltype(nc)::value, u = m * NR + n;
          static_for<NPT>([&](auto qc) {
            constexpr int q = decltype(qc)::value;
            constexpr int slot = NR + (SCHED == 1 ? q : q * ((MR - 1) * NR) / NPT);
            if constexpr (slot == u) {
              char *sa = smem + (t & 1) * STAGE;
              if constexpr (q < OA::NI) {
                __builtin_amdgcn_raw_ptr_buffer_load_lds(rA, (lds_void *)(sa + (wave + NW * q) * 1024), 16,
                                                         offA(std::integral_constant<int, q>{}, pa), 0, 0, 0);
              } else {
                __builtin_amdgcn_raw_ptr_buffer_load_lds(
                    rB, (lds_void *)(sa + A_BYTES + (wave + NW * (q - OA::NI)) * 1024), 16,
                    offB(std::integral_constant<int, q - OA::NI>{}, pb), 0, 0, 0);
              }
            }
          });
          mfma_asm(acc[m][n], fa[m], fb1[n]);
          if constexpr (m == 0) read_b1(nc, t + 1, 0, fb0);
          __builtin_amdgcn_sched_barrier(0);
        });
        read_a(mc, t + 1, 0);
        __builtin_amdgcn_sched_barrier(0);
      });
    }
    // retire tile t+1's k-step 0 reads behind [B]'s MFMAs: the next [A] then waits on nothing
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_sched_barrier(0);
  }
  // the last MFMAs' results are read by compiler code below: 8-pass XDL -> 12 wait states
  asm volatile("s_nop 15\n\ts_nop 15" ::: "memory");
  wait_vmcnt<0>();
  __syncthreads();  // the epilogue reuses the stage buffers

  seg_epilogue<EPI, MR, NR, WM>(acc, smem, E, g, wb.slice, A.rows, B.rows, i0 + wr * WM, j0 + wc * WN, wave, lane);
}

template <int BM, int BN, int AMODE, int BMODE, int EPI, int SCHED>
void launch_4w(const GOperand &A, const GOperand &B, const GEpi &E, int groups, int ksplit, hipStream_t s) {
  const int ti = cdiv(A.rows, BM), tj = cdiv(B.rows, BN);
  const int ktiles = cdiv(A.kdim, BK);
  ksplit = ksplit < 1 ? 1 : (ksplit > ktiles ? ktiles : ksplit);
  const int per = cdiv(ktiles, ksplit);
  ksplit = cdiv(ktiles, per);
  dim3 grid(ti * tj, ksplit, groups);
  hipLaunchKernelGGL((gemm_4w<BM, BN, AMODE, BMODE, EPI, SCHED>), grid, dim3(256), 0, s, A, B, E, ti, tj, per, ktiles);
}

}  // namespace

namespace cxg {
// 92: 256x256, 94: 128x256, 95: 256x128, 98: 96x256 (DMAs spread over [B]); 93 / 96 / 97 / 100: the same
// with the DMAs in a burst
int dispatch_4w(int amode, int bmode, int epi, int tile, const GOperand &A, const GOperand &B, const GEpi &E,
                int groups, int ksplit, hipStream_t s) {
#define CX4(AMV, BMV, EPV)                                                                                 \
  if (amode == AMV && bmode == BMV && epi == EPV) {                                                        \
    switch (tile) {                                                                                        \
      case 92: launch_4w<256, 256, AMV, BMV, EPV, 0>(A, B, E, groups, ksplit, s); return 0;                \
      case 93: launch_4w<256, 256, AMV, BMV, EPV, 1>(A, B, E, groups, ksplit, s); return 0;                \
      case 94: launch_4w<128, 256, AMV, BMV, EPV, 0>(A, B, E, groups, ksplit, s); return 0;                \
      case 95: launch_4w<256, 128, AMV, BMV, EPV, 0>(A, B, E, groups, ksplit, s); return 0;                \
      case 96: launch_4w<128, 256, AMV, BMV, EPV, 1>(A, B, E, groups, ksplit, s); return 0;                \
      case 97: launch_4w<256, 128, AMV, BMV, EPV, 1>(A, B, E, groups, ksplit, s); return 0;                \
      case 98: launch_4w<96, 256, AMV, BMV, EPV, 0>(A, B, E, groups, ksplit, s); return 0;                 \
      case 100: launch_4w<96, 256, AMV, BMV, EPV, 1>(A, B, E, groups, ksplit, s); return 0;                \
      default: return -1;                                                                                  \
    }                                                                                                      \
  }
  CX4(K_DIRECT, K_GATHER, EPI_BF16)     // conv fwd / dgrad
  CX4(K_DIRECT, K_ROWGATHER, EPI_BF16)  // conv fwd, few input channels (AlexNet conv1)
  CX4(K_DIRECT, K_DIRECT, EPI_BF16)  // fc fwd, square GEMMs
  CX4(K_DIRECT, K_DIRECT, EPI_F32)   // fc fwd split-K
#undef CX4
  return -1;
}
}  // namespace cxg
