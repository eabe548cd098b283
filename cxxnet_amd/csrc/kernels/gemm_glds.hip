// LDS-DMA pipelined bf16 MFMA GEMM for gfx950 (K-major operands).
//
// Serves the GEMMs whose two operands are both K-contiguous:
//   conv forward    A = weights [Cout][KH][KW][Cg],  B = implicit im2col of NHWC x   (reference K1-K4)
//   conv data-grad  A = flipped weights,             B = implicit im2col of NHWC dy  (reference K7+K8)
//   fc forward      A = weights [nout][nin],         B = activations [batch][nin]     (reference K9)
// (reference: src/layer/convolution_layer-inl.hpp:70-155, src/layer/fullc_layer-inl.hpp:101-112).
//
// Design (MI355X-first; see gemm_mfma.hip for the register-staged generic kernel):
//   * both tiles go global -> LDS with `buffer_load_dwordx4 ... lds` (LDS-DMA): no VGPR
//     staging, no ds_write pass, out-of-range rows / padding taps become buffer-OOB loads
//     that land as zeros;
//   * LDS image is lane-linear per wave-instruction (8 rows x 128 B) with an XOR swizzle
//     on the 16-byte chunk (chunk ^ ((row >> 1) & 7)) applied on the SOURCE address, so the
//     16x16x32 fragment reads (ds_read_b128) are bank-conflict free;
//   * STAGES-deep ring of LDS buffers; each wave waits only for its own loads of the tile
//     about to be read (counted `s_waitcnt vmcnt(N)`), then a raw s_barrier -- the DMAs of
//     the next tiles stay in flight across it;
//   * 4 waves, wave grid WGM x WGN, v_mfma_f32_16x16x32_bf16 with fp32 accumulators;
//   * implicit-GEMM gather: per tile each lane decodes ONE k offset (its 16-byte chunk is
//     fixed by the swizzle), the per-row pixel geometry is precomputed once;
//   * epilogue: bias / relu / relu'-mask / alpha, staged per wave through LDS so every
//     global store is a full 16-byte vector of a contiguous output row; or fp32 split-K
//     slabs (EPI_F32) reduced by splitk_finalize.
#include <utility>
#include "common.h"

namespace {

constexpr int BK = 64;
constexpr int NT = 256;
constexpr uint32_t OOB = 0x80000000u;  // >= num_records: the load returns zeros
typedef __amdgpu_buffer_rsrc_t rsrc_t;
typedef __attribute__((address_space(3))) void lds_void;

enum { B_DIRECT = 0, B_GATHER = 1 };
enum { EPI_BF16 = 0, EPI_F32 = 1 };

struct GOperand {
  const bf16_t *ptr;
  long gstride;     // per-group element offset
  uint32_t nbytes;  // descriptor range (all groups)
  int ld, rows, kdim;
  int H, W, C, Ho, Wo, KW, stride, pad_h, pad_w, Cg;  // gather geometry (NHWC source)
  FastDiv fd_cg, fd_kw, fd_hw, fd_wo;
};

struct GEpi {
  void *out;
  long gstride;
  int ldc;
  float alpha;
  const float *bias;
  long bias_gstride;
  int relu, mask_relu;
  long kstride;
};

__device__ __forceinline__ rsrc_t make_rsrc(const void *p, uint32_t nbytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), (short)0, static_cast<int>(nbytes), 0x00020000);
}

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

template <typename F, int... I>
__device__ __forceinline__ void static_for_impl(F &&f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
// f(std::integral_constant<int, i>) for i = 0..N-1, fully unrolled with constant indices
template <int N, typename F>
__device__ __forceinline__ void static_for(F &&f) {
  static_for_impl(f, std::make_integer_sequence<int, N>{});
}

__device__ __forceinline__ void block_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

template <int BM, int BN, int WGM, int WGN, int STAGES, int BMODE, int EPI>
__global__ void __launch_bounds__(NT, 1)
gemm_glds(GOperand A, GOperand B, GEpi E, int tiles_i, int tiles_j, int ksplit_tiles, int ktiles_total) {
  static_assert(WGM * WGN == 4, "4 waves");
  static_assert(BM % 32 == 0 && BN % 32 == 0, "tile rows must be a multiple of 32 (8 rows per DMA x 4 waves)");
  constexpr int WM = BM / WGM, WN = BN / WGN;
  static_assert(WM % 16 == 0 && WN % 16 == 0, "wave tile must be a multiple of 16");
  constexpr int MR = WM / 16, NR = WN / 16;
  constexpr int NIA = BM / 32, NIB = BN / 32;  // DMA instructions per wave per tile
  constexpr int NPT = NIA + NIB;
  constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2;
  constexpr int STAGE_BYTES = A_BYTES + B_BYTES;
  constexpr int EPI_BYTES = 4 * 16 * (WM + 4) * 4;
  constexpr int SMEM = STAGES * STAGE_BYTES > EPI_BYTES ? STAGES * STAGE_BYTES : EPI_BYTES;
  __shared__ __attribute__((aligned(1024))) char smem[SMEM];

  const int g = blockIdx.z;
  const uint32_t ntile = static_cast<uint32_t>(tiles_i) * tiles_j;
  const uint32_t tile = xcd_remap(blockIdx.x, ntile);
  const int ti = tile % tiles_i, tj = tile / tiles_i;  // i fastest: neighbours share the B panel
  const int i0 = ti * BM, j0 = tj * BN;
  const int kt_beg = blockIdx.y * ksplit_tiles;
  const int kt_end = min(kt_beg + ksplit_tiles, ktiles_total);
  if (kt_beg >= kt_end) return;
  const int nt = kt_end - kt_beg;

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const rsrc_t rA = make_rsrc(A.ptr, A.nbytes);
  const rsrc_t rB = make_rsrc(B.ptr, B.nbytes);
  const uint32_t goA = static_cast<uint32_t>(g * A.gstride) * 2u;
  const uint32_t goB = static_cast<uint32_t>(g * B.gstride) * 2u;

  // This lane's logical 16-byte chunk inside its 128-byte row, identical for every DMA
  // the wave issues (rows 8q + lane/8 with q = wave + 4s): chunk ^ ((row >> 1) & 7).
  const int lchunk = (lane & 7) ^ (((wave & 1) << 2) + (lane >> 4));
  const int lrow = lane >> 3;

  // ---- per-row source geometry, fixed across K
  uint32_t rowA[NIA];
#pragma unroll
  for (int s = 0; s < NIA; ++s) {
    const int r = i0 + 8 * (wave + 4 * s) + lrow;
    rowA[s] = r < A.rows ? goA + static_cast<uint32_t>(r * A.ld) * 2u : OOB;
  }
  int bbase[NIB], bh[NIB], bw[NIB];
#pragma unroll
  for (int s = 0; s < NIB; ++s) {
    const int p = j0 + 8 * (wave + 4 * s) + lrow;
    if constexpr (BMODE == B_GATHER) {
      if (p < B.rows) {
        const uint32_t n = fdiv(static_cast<uint32_t>(p), B.fd_hw);
        const uint32_t rem = static_cast<uint32_t>(p) - n * static_cast<uint32_t>(B.Ho * B.Wo);
        const uint32_t ho = fdiv(rem, B.fd_wo);
        const uint32_t wo = rem - ho * B.Wo;
        bbase[s] = static_cast<int>(n) * B.H * B.W * B.C;
        bh[s] = static_cast<int>(ho) * B.stride - B.pad_h;
        bw[s] = static_cast<int>(wo) * B.stride - B.pad_w;
      } else {
        bbase[s] = -1;
        bh[s] = 0;
        bw[s] = 0;
      }
    } else {
      bbase[s] = p < B.rows ? static_cast<int>(goB) + p * B.ld * 2 : -1;
      bh[s] = bw[s] = 0;
    }
  }

  // ---- DMAs of one K-tile: prep() decodes this lane's k once, issue_one<q>() sends
  // DMA instruction q (A rows for q < NIA, then B rows) into stage buffer `st`.  The
  // pieces are interleaved with the previous tile's MFMAs by compute().
  struct Prep {
    uint32_t ka;   // byte offset of k in an A row, or OOB
    uint32_t kb;   // direct B: byte offset of k; gather B: channel byte offset (+ group)
    int kh, kw;
    bool kin;
  };
  auto prep = [&](int kt) {
    Prep p;
    const int k = kt * BK + lchunk * 8;
    p.kin = kt < kt_end && k < A.kdim;
    p.ka = p.kin ? static_cast<uint32_t>(k) * 2u : OOB;
    if constexpr (BMODE == B_GATHER) {
      const uint32_t r = fdiv(static_cast<uint32_t>(k), B.fd_cg);
      const int c = k - static_cast<int>(r) * B.Cg;
      const uint32_t kh = fdiv(r, B.fd_kw);
      p.kh = p.kin ? static_cast<int>(kh) : -(1 << 20);  // out of range -> every row OOB
      p.kw = static_cast<int>(r - kh * B.KW);
      p.kb = goB + static_cast<uint32_t>(c) * 2u;
    } else {
      p.kb = p.ka;
      p.kh = p.kw = 0;
    }
    return p;
  };
  auto issue_one = [&](const Prep &p, int st, auto qc) {
    constexpr int q = decltype(qc)::value;
    char *sa = smem + st * STAGE_BYTES;
    uint32_t off;
    if constexpr (q < NIA) {
      off = (p.ka != OOB && rowA[q] != OOB) ? rowA[q] + p.ka : OOB;
      asm volatile("" : "+v"(off));  // keep the select: no per-lane branch around the DMA
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rA, (lds_void *)(sa + (wave + 4 * q) * 1024), 16, off, 0, 0, 0);
    } else {
      constexpr int s = q - NIA;
      if constexpr (BMODE == B_GATHER) {
        const int hi = bh[s] + p.kh, wi = bw[s] + p.kw;
        const bool ok = bbase[s] >= 0 && static_cast<unsigned>(hi) < static_cast<unsigned>(B.H) &&
                        static_cast<unsigned>(wi) < static_cast<unsigned>(B.W);
        off = ok ? p.kb + static_cast<uint32_t>(bbase[s] + (hi * B.W + wi) * B.C) * 2u : OOB;
      } else {
        off = (p.kin && bbase[s] >= 0) ? static_cast<uint32_t>(bbase[s]) + p.kb : OOB;
      }
      asm volatile("" : "+v"(off));
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rB, (lds_void *)(sa + A_BYTES + (wave + 4 * s) * 1024), 16, off, 0,
                                               0, 0);
    }
  };
  auto issue_all = [&](int kt, int st) {
    const Prep p = prep(kt);
    static_for<NPT>([&](auto qc) { issue_one(p, st, qc); });
  };

  const int wi_ = wave % WGM, wj_ = wave / WGM;
  f32x4 acc[MR][NR];
#pragma unroll
  for (int m = 0; m < MR; ++m)
#pragma unroll
    for (int n = 0; n < NR; ++n) acc[m][n] = f32x4{0.f, 0.f, 0.f, 0.f};

  // fragment addressing: rows base16 + (lane & 15); (row >> 1) & 7 == (lane & 15) >> 1
  const int frow = (lane & 15) * 128;
  const int fx0 = ((0 + (lane >> 4)) ^ ((lane & 15) >> 1)) << 4;
  const int fx1 = ((4 + (lane >> 4)) ^ ((lane & 15) >> 1)) << 4;
  // compute one staged tile; the DMAs of the tile STAGES-1 ahead are issued first, ahead
  // of the fragment reads (issue-before-read: their latency hides under this tile's MFMAs).
  // Interleaving them between MFMA rows measured worse codegen: the live ranges pushed the
  // loop past 256 VGPRs and hipcc copied the accumulators AGPR<->VGPR every iteration.
  auto compute = [&](int st, const Prep &p, int st_w) {
    const char *sa = smem + st * STAGE_BYTES + wi_ * WM * 128 + frow;
    const char *sb = smem + st * STAGE_BYTES + A_BYTES + wj_ * WN * 128 + frow;
    static_for<2>([&](auto kkc) {
      constexpr int kk = decltype(kkc)::value;
      const int fx = kk ? fx1 : fx0;
      if constexpr (kk == 0) static_for<NPT>([&](auto qc) { issue_one(p, st_w, qc); });
      bf16x8 fa[MR], fb[NR];
#pragma unroll
      for (int m = 0; m < MR; ++m) fa[m] = *reinterpret_cast<const bf16x8 *>(sa + m * 16 * 128 + fx);
#pragma unroll
      for (int n = 0; n < NR; ++n) fb[n] = *reinterpret_cast<const bf16x8 *>(sb + n * 16 * 128 + fx);
      static_for<MR>([&](auto mc) {
        constexpr int m = decltype(mc)::value;
#pragma unroll
        for (int n = 0; n < NR; ++n)
          acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[m], fb[n], acc[m][n], 0, 0, 0);

      });
    });
  };

  // ---- main loop: STAGES-deep DMA ring
#pragma unroll
  for (int s = 0; s < STAGES - 1; ++s) issue_all(kt_beg + s, s);  // (all-OOB dummies past the slice)
  int st_read = 0, st_write = STAGES - 1;
  for (int t = 0; t < nt; ++t) {
    // Every iteration issues one tile's DMAs (past the slice: all-OOB dummies that write
    // zeros into the buffer of the already-consumed tile t-1), so exactly STAGES-2 tiles
    // of this wave's DMAs may stay in flight beyond tile t -- a branch-free loop body.
    wait_vmcnt<NPT * (STAGES - 2)>();
    block_barrier();  // every wave's DMAs of tile t have landed; every wave is done reading tile t-1
    const Prep p = prep(kt_beg + t + STAGES - 1);
    compute(st_read, p, st_write);
    st_read = st_read + 1 == STAGES ? 0 : st_read + 1;
    st_write = st_write + 1 == STAGES ? 0 : st_write + 1;
  }
  wait_vmcnt<0>();
  __syncthreads();  // stage buffers are reused by the epilogue

  // ---- epilogue
  const int Mi = A.rows, Nj = B.rows;
  const int ibase = i0 + wi_ * WM, jbase = j0 + wj_ * WN;
  if constexpr (EPI == EPI_F32) {
    float *out = reinterpret_cast<float *>(E.out) + g * E.gstride + blockIdx.y * E.kstride;
#pragma unroll
    for (int m = 0; m < MR; ++m)
#pragma unroll
      for (int n = 0; n < NR; ++n) {
        const int i = ibase + m * 16 + (lane >> 4) * 4;
        const int j = jbase + n * 16 + (lane & 15);
        if (j < Nj && i < Mi) {
          f32x4 v = acc[m][n] * E.alpha;
          float *dst = out + static_cast<long>(j) * E.ldc + i;
          if (i + 4 <= Mi && (E.ldc & 3) == 0) {
            *reinterpret_cast<f32x4 *>(dst) = v;
          } else {
            for (int e = 0; e < 4 && i + e < Mi; ++e) dst[e] = v[e];
          }
        }
      }
  } else {
    float *ep = reinterpret_cast<float *>(smem) + wave * 16 * (WM + 4);
    bf16_t *out = reinterpret_cast<bf16_t *>(E.out) + g * E.gstride;
    const float *bias = E.bias ? E.bias + g * E.bias_gstride : nullptr;
    constexpr int LPR = WM / 8;   // lanes per output row (8 bf16 per lane)
    constexpr int RPI = 64 / LPR; // rows per pass
    const int il = (lane % LPR) * 8;
    const int i = ibase + il;
    float bv[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) bv[e] = (bias && i + e < Mi) ? bias[i + e] : 0.f;
    const bool vec_store = ((E.ldc & 7) == 0) && (i + 8 <= Mi);
#pragma unroll
    for (int n = 0; n < NR; ++n) {
#pragma unroll
      for (int m = 0; m < MR; ++m)
        *reinterpret_cast<f32x4 *>(ep + (lane & 15) * (WM + 4) + m * 16 + (lane >> 4) * 4) = acc[m][n];
      __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the wave's LDS writes are visible to its reads
#pragma unroll
      for (int jl = lane / LPR; jl < 16; jl += RPI) {
        const int j = jbase + n * 16 + jl;
        if (j < Nj && i < Mi) {
          const f32x4 x0 = *reinterpret_cast<const f32x4 *>(ep + jl * (WM + 4) + il);
          const f32x4 x1 = *reinterpret_cast<const f32x4 *>(ep + jl * (WM + 4) + il + 4);
          float f[8] = {x0[0], x0[1], x0[2], x0[3], x1[0], x1[1], x1[2], x1[3]};
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            f[e] = f[e] * E.alpha + bv[e];
            if (E.relu) f[e] = fmaxf(f[e], 0.f);
          }
          bf16_t *dst = out + static_cast<long>(j) * E.ldc + i;
          if (vec_store) {
            if (E.mask_relu) {
              float old[8];
              unpack8(*reinterpret_cast<const uint4 *>(dst), old);
#pragma unroll
              for (int e = 0; e < 8; ++e) f[e] = old[e] > 0.f ? f[e] : 0.f;
            }
            *reinterpret_cast<uint4 *>(dst) = pack8(f);
          } else {
            for (int e = 0; e < 8 && i + e < Mi; ++e) {
              if (E.mask_relu && !(bf2f(dst[e]) > 0.f)) f[e] = 0.f;
              dst[e] = f2bf(f[e]);
            }
          }
        }
      }
      __builtin_amdgcn_s_waitcnt(0xc07f);
    }
  }
}

template <int BM, int BN, int WGM, int WGN, int STAGES, int BMODE, int EPI>
void launch(const GOperand &A, const GOperand &B, const GEpi &E, int groups, int ksplit, hipStream_t s) {
  const int ti = cdiv(A.rows, BM), tj = cdiv(B.rows, BN);
  const int ktiles = cdiv(A.kdim, BK);
  ksplit = ksplit < 1 ? 1 : (ksplit > ktiles ? ktiles : ksplit);
  const int per = cdiv(ktiles, ksplit);
  ksplit = cdiv(ktiles, per);
  dim3 grid(ti * tj, ksplit, groups);
  hipLaunchKernelGGL((gemm_glds<BM, BN, WGM, WGN, STAGES, BMODE, EPI>), grid, dim3(NT), 0, s, A, B, E, ti, tj, per,
                     ktiles);
}

// Tile ids (BM x BN, wave grid, stages):
//   0: 128x256 (1x4) 3 stages   1: 128x128 (1x4) 2 stages   2: 128x128 (2x2) 3 stages
//   4: 192x256 (1x4) 2 stages   5: 64x256 (1x4) 3 stages
//   6: 256x128 (4x1) 3 stages   7: 64x128 (1x4) 2 stages    8: 192x128 (1x4) 2 stages
//   9: 96x128 (1x4) 2 stages    10: 128x64 (2x2) 2 stages   11: 64x128 (1x4) 3 stages
//  12: 64x128 (1x4) 4 stages   13: 128x128 (1x4) 3 stages  14: 128x64 (2x2) 3 stages
//  15: 64x64 (2x2) 3 stages    16: 192x64 (2x2) 3 stages
#define CXG_TILES(BMODE, EPI)                                                               \
  switch (tile) {                                                                           \
    case 0: launch<128, 256, 1, 4, 3, BMODE, EPI>(A, B, E, groups, ksplit, s); return 0;    \
    case 1: launch<128, 128, 1, 4, 2, BMODE, EPI>(A, B, E, groups, ksplit, s); return 0;    \
    case 2: launch<128, 128, 2, 2, 3, BMODE, EPI>(A, B, E, groups, ksplit, s); return 0;    \
    case 4: launch<192, 256, 1, 4, 2, BMODE, EPI>(A, B, E, groups, ksplit, s); return 0;    \
    case 5: launch<64, 256, 1, 4, 3, BMODE, EPI>(A, B, E, groups, ksplit, s); return 0;     \
    case 6: launch<256, 128, 4, 1, 3, BMODE, EPI>(A, B, E, groups, ksplit, s); return 0;    \
    case 7: launch<64, 128, 1, 4, 2, BMODE, EPI>(A, B, E, groups, ksplit, s); return 0;     \
    case 8: launch<192, 128, 1, 4, 2, BMODE, EPI>(A, B, E, groups, ksplit, s); return 0;    \
    case 9: launch<96, 128, 1, 4, 2, BMODE, EPI>(A, B, E, groups, ksplit, s); return 0;     \
    case 10: launch<128, 64, 2, 2, 2, BMODE, EPI>(A, B, E, groups, ksplit, s); return 0;    \
    case 11: launch<64, 128, 1, 4, 3, BMODE, EPI>(A, B, E, groups, ksplit, s); return 0;    \
    case 12: launch<64, 128, 1, 4, 4, BMODE, EPI>(A, B, E, groups, ksplit, s); return 0;    \
    case 13: launch<128, 128, 1, 4, 3, BMODE, EPI>(A, B, E, groups, ksplit, s); return 0;   \
    case 14: launch<128, 64, 2, 2, 3, BMODE, EPI>(A, B, E, groups, ksplit, s); return 0;    \
    case 15: launch<64, 64, 2, 2, 3, BMODE, EPI>(A, B, E, groups, ksplit, s); return 0;     \
    case 16: launch<192, 64, 2, 2, 3, BMODE, EPI>(A, B, E, groups, ksplit, s); return 0;    \
    default: return -1;                                                                     \
  }

int dispatch(int bmode, int epi, int tile, const GOperand &A, const GOperand &B, const GEpi &E, int groups, int ksplit,
             hipStream_t s) {
  if (bmode == B_GATHER && epi == EPI_BF16) { CXG_TILES(B_GATHER, EPI_BF16) }
  if (bmode == B_DIRECT && epi == EPI_BF16) { CXG_TILES(B_DIRECT, EPI_BF16) }
  if (bmode == B_DIRECT && epi == EPI_F32) { CXG_TILES(B_DIRECT, EPI_F32) }
  return -1;
}
#undef CXG_TILES

}  // namespace

// Same operand record as cxn_gemm (gemm_mfma.hip).
struct CxnOperandG {
  const void *ptr;
  long gstride;
  long nbytes;
  int ld, rows, kdim;
  int H, W, C, Ho, Wo, KH, KW, stride, pad_h, pad_w, dil, Cg;
};

// Returns 0 on success, -1 unsupported configuration (the caller falls back), -3 launch error.
// Requirements: kdim % 8 == 0, 16-byte aligned rows (ld % 8 == 0), gather: Cg % 8 == 0 and
// dil == 1, every buffer < 2 GiB.
CXN_API int cxn_gemm_glds(const CxnOperandG *a, const CxnOperandG *b, int bmode, void *out, long out_gstride, int ldc,
                          float alpha, const float *bias, long bias_gstride, int relu, int mask_relu, int epi,
                          int tile, int groups, int ksplit, long kstride, void *stream) {
  if (a->kdim != b->kdim || a->kdim % 8 != 0) return -1;
  if (a->nbytes >= (1L << 31) || b->nbytes >= (1L << 31)) return -1;
  if (a->ld % 8 != 0 || a->gstride % 8 != 0 || (reinterpret_cast<uintptr_t>(a->ptr) & 15)) return -1;
  if (reinterpret_cast<uintptr_t>(b->ptr) & 15) return -1;
  if (bmode == B_GATHER && (b->Cg % 8 != 0 || b->C % 8 != 0 || b->dil > 1 || b->gstride % 8 != 0)) return -1;
  if (bmode == B_DIRECT && (b->ld % 8 != 0 || b->gstride % 8 != 0)) return -1;
  if (a->rows <= 0 || b->rows <= 0 || a->kdim <= 0) return 0;
  GOperand A{}, B{};
  A.ptr = static_cast<const bf16_t *>(a->ptr);
  A.gstride = a->gstride;
  A.nbytes = static_cast<uint32_t>(a->nbytes);
  A.ld = a->ld; A.rows = a->rows; A.kdim = a->kdim;
  B.ptr = static_cast<const bf16_t *>(b->ptr);
  B.gstride = b->gstride;
  B.nbytes = static_cast<uint32_t>(b->nbytes);
  B.ld = b->ld; B.rows = b->rows; B.kdim = b->kdim;
  if (bmode == B_GATHER) {
    B.H = b->H; B.W = b->W; B.C = b->C; B.Ho = b->Ho; B.Wo = b->Wo; B.KW = b->KW;
    B.stride = b->stride; B.pad_h = b->pad_h; B.pad_w = b->pad_w; B.Cg = b->Cg;
    B.fd_cg = make_fastdiv(b->Cg);
    B.fd_kw = make_fastdiv(b->KW > 0 ? b->KW : 1);
    B.fd_hw = make_fastdiv(b->Ho * b->Wo > 0 ? b->Ho * b->Wo : 1);
    B.fd_wo = make_fastdiv(b->Wo > 0 ? b->Wo : 1);
  }
  GEpi E{out, out_gstride, ldc, alpha, bias, bias_gstride, relu, mask_relu, kstride};
  hipStream_t s = static_cast<hipStream_t>(stream);
  const int rc = dispatch(bmode, epi, tile, A, B, E, groups < 1 ? 1 : groups, ksplit < 1 ? 1 : ksplit, s);
  if (rc != 0) return rc;
  return hipGetLastError() == hipSuccess ? 0 : -3;
}
