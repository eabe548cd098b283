// LDS-DMA pipelined bf16 MFMA GEMM for gfx950.
//
// Computes, per group g = blockIdx.z:   C[j][i] (+)= alpha * sum_k A(i, k) * B(j, k)
// with each operand loaded by one of four loaders:
//   K_DIRECT  : elem(row,k) = p[row*ld + k]          (k contiguous)
//   K_GATHER  : rows = output pixels, k = (kh,kw,c)   implicit im2col of an NHWC tensor
//   K_ROWGATHER: rows = output pixels, k = (kh, j)   j over a kernel row's KW*C contiguous
//               elements, zero-padded to 8 (few-channel convs: conv1's 11x11x4 runs of 44)
//   MN_DIRECT : elem(row,k) = p[k*ld + row]          (row contiguous)
//   MN_GATHER : rows = (kh,kw,c), k = output pixels   transposed implicit im2col
// It serves the GEMM-shaped ops of AlexNet-class nets:
//   conv forward     A K_DIRECT (weights)        B K_GATHER (x)          bf16 out   (reference K1-K4)
//   conv1 forward    A K_DIRECT (row-padded w)   B K_ROWGATHER (x)       bf16 out
//   conv data-grad   A K_DIRECT (flipped w)      B K_GATHER (dy)         bf16 out   (reference K7+K8)
//   conv weight-grad A MN_GATHER (x)             B MN_DIRECT (dy)        fp32 atomics, split-K (K5/K6)
//   fc forward       A K_DIRECT (W)              B K_DIRECT (x)          bf16 / split-K slabs (K9)
//   fc data-grad     A MN_DIRECT (W)             B K_DIRECT (dy)         bf16 / split-K slabs (K12)
//   fc weight-grad   A MN_DIRECT (x)             B MN_DIRECT (dy)        fp32 store / += (K10)
// (reference: src/layer/convolution_layer-inl.hpp:70-155, src/layer/fullc_layer-inl.hpp:101-130,
//  which do these as im2col + cuBLAS sgemm).
//
// Design (MI355X-first):
//   * both tiles go global -> LDS with `buffer_load_dwordx4 ... lds` (LDS-DMA): no VGPR
//     staging, no ds_write pass; out-of-range rows, K tails and padding taps are buffer-OOB
//     loads that land as zeros;
//   * the LDS image is lane-linear per DMA instruction (1 KiB) with an XOR swizzle of the
//     16-byte chunks applied on the SOURCE address, so the fragment reads are bank-conflict
//     free: K-major tiles [rows][64] are read with ds_read_b128 (chunk ^ ((row>>1)&7)),
//     MN-major tiles [64][128] with ds_read_b64_tr_b16 (chunk ^ 2*((k&3) | ((k>>3)&1)<<2));
//   * each lane's 16-byte chunk is fixed by the swizzle, so per K-tile a lane decodes one k
//     (K-major) or one pixel per DMA (MN-major); row geometry is precomputed once;
//   * STAGES-deep LDS ring; every iteration issues one tile of DMAs (all-OOB dummies past the
//     K slice) so each wave waits with one constant `s_waitcnt vmcnt(N)` for its own loads of
//     the tile to read, then a raw s_barrier: DMAs of later tiles stay in flight across it;
//   * 4 waves (wave grid WGM x WGN) of v_mfma_f32_16x16x32_bf16; small-LDS 2-stage tiles run
//     2-5 blocks per CU, which is what hides the DMA latency best (profiles/early-r14_glds_tiles.jsonl);
//   * epilogues staged per wave through LDS so every global access is a contiguous row
//     segment: bf16 (+bias, relu, relu'-mask of the old value), fp32 split-K slab, fp32 +=,
//     fp32 atomics.
#include <cstdlib>
#include "gemm_glds_common.h"

using namespace cxg;

namespace {


// ---------------------------------------------------------------------------------- kernel
// PIPE bit 0: s_setprio(1) around each MFMA cluster (hipcc then keeps the cluster between the
//             barriers instead of spreading it among the DMA issue -- cdna guide T5);
// PIPE bit 1: both k-steps' fragments are read before the first MFMA (the k=32 reads are in
//             flight under the k=0 MFMAs).
// BMC (<= BM): A rows COMPUTED per block when it differs from the BM rows staged in LDS -- a
// 48-row tile stages 64 rows (the DMA granularity is 8 rows x waves) but runs MFMAs and the
// epilogue on 48 and steps i by 48 (AlexNet conv2's data-gradient onto 48 channels per group).
template <int BM, int BN, int WGM, int WGN, int STAGES, int AMODE, int BMODE, int EPI, int PIPE = 0, int BMC = BM>
__global__ void __launch_bounds__(64 * WGM * WGN, 1)
gemm_glds(GOperand A, GOperand B, GEpi E, int tiles_i, int tiles_j, int ksplit_tiles, int ktiles_total) {
  constexpr int NW = WGM * WGN;  // 4 waves, or 8 (two per SIMD) for the large tiles
  static_assert(NW == 4 || NW == 8, "4 or 8 waves");
  static_assert(BM % (8 * NW) == 0 && BN % (8 * NW) == 0, "tile rows: a multiple of 8 rows per DMA x waves");
  static_assert(BMC <= BM && BMC % (16 * WGM) == 0, "computed rows: whole 16-row fragments per wave");
  constexpr int WM = BMC / WGM, WN = BN / WGN;
  static_assert(WM % 16 == 0 && WN % 16 == 0, "wave tile must be a multiple of 16");
  constexpr int MR = WM / 16, NR = WN / 16;
  using OA = Op<AMODE, BM, NW>;
  using OB = Op<BMODE, BN, NW>;
  constexpr int NPT = OA::NI + OB::NI;  // DMA instructions per wave per tile
  constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2;
  constexpr int STAGE_BYTES = A_BYTES + B_BYTES;
  constexpr int EPI_BYTES = NW * 16 * (WM + 4) * 4;
  constexpr int SMEM = STAGES * STAGE_BYTES > EPI_BYTES ? STAGES * STAGE_BYTES : EPI_BYTES;
  __shared__ __attribute__((aligned(1024))) char smem[SMEM];

  const uint32_t ntile = static_cast<uint32_t>(tiles_i) * tiles_j;
  const GemmBlock wb = gemm_block(ntile);
  const int g = wb.g;
  const uint32_t tile = wb.tile;
  int ti, tj;
  tile_ij(tile, tiles_i, tiles_j, E.group_i, ti, tj);
  const int i0 = ti * BMC, j0 = tj * BN;
  const int kt_beg = wb.slice * ksplit_tiles;
  const int kt_end = min(kt_beg + ksplit_tiles, ktiles_total);
  if (kt_beg >= kt_end) return;
  const int nt = kt_end - kt_beg;

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const rsrc_t rA = make_rsrc(A.ptr, A.nbytes);
  const rsrc_t rB = make_rsrc(B.ptr, B.nbytes);
  const uint32_t goA = static_cast<uint32_t>(g * A.gstride) * 2u;
  const uint32_t goB = static_cast<uint32_t>(g * B.gstride) * 2u;
  OA oa;
  OB ob;
  oa.init(A, i0, goA, wave, lane);
  ob.init(B, j0, goB, wave, lane);

  // issue every DMA of K-tile kt into stage buffer st (dummies past the slice)
  auto issue = [&](int kt, int st) {
    const typename OA::Prep pa = oa.prep(A, kt, kt_end, goA);
    const typename OB::Prep pb = ob.prep(B, kt, kt_end, goB);
    char *sa = smem + st * STAGE_BYTES;
    static_for<OA::NI>([&](auto sc) {
      constexpr int s = decltype(sc)::value;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rA, (lds_void *)(sa + (wave + NW * s) * 1024), 16,
                                               oa.template offset<s>(A, pa, wave, lane), 0, 0, 0);
    });
    static_for<OB::NI>([&](auto sc) {
      constexpr int s = decltype(sc)::value;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rB, (lds_void *)(sa + A_BYTES + (wave + NW * s) * 1024), 16,
                                               ob.template offset<s>(B, pb, wave, lane), 0, 0, 0);
    });
  };

  const int wi_ = wave % WGM, wj_ = wave / WGM;
  f32x4 acc[MR][NR];
#pragma unroll
  for (int m = 0; m < MR; ++m)
#pragma unroll
    for (int n = 0; n < NR; ++n) acc[m][n] = f32x4{0.f, 0.f, 0.f, 0.f};

  // One staged tile: the DMAs of the tile STAGES-1 ahead are issued first, ahead of the
  // fragment reads (their latency hides under this tile's MFMAs).  Interleaving them between
  // MFMA rows measured worse: the live ranges pushed the loop past 256 VGPRs and hipcc copied
  // the accumulators AGPR<->VGPR every iteration.
  auto compute = [&](int st) {
    const char *sa = smem + st * STAGE_BYTES;
    const char *sb = sa + A_BYTES;
    if constexpr ((PIPE & 2) != 0) {
      bf16x8 fa0[MR], fb0[NR], fa1[MR], fb1[NR];
#pragma unroll
      for (int m = 0; m < MR; ++m) fa0[m] = frag<AMODE>(sa, wi_ * WM + m * 16, 0, lane);
#pragma unroll
      for (int n = 0; n < NR; ++n) fb0[n] = frag<BMODE>(sb, wj_ * WN + n * 16, 0, lane);
#pragma unroll
      for (int m = 0; m < MR; ++m) fa1[m] = frag<AMODE>(sa, wi_ * WM + m * 16, 32, lane);
#pragma unroll
      for (int n = 0; n < NR; ++n) fb1[n] = frag<BMODE>(sb, wj_ * WN + n * 16, 32, lane);
      if constexpr ((PIPE & 1) != 0) __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int m = 0; m < MR; ++m)
#pragma unroll
        for (int n = 0; n < NR; ++n)
          acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa0[m], fb0[n], acc[m][n], 0, 0, 0);
#pragma unroll
      for (int m = 0; m < MR; ++m)
#pragma unroll
        for (int n = 0; n < NR; ++n)
          acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa1[m], fb1[n], acc[m][n], 0, 0, 0);
      if constexpr ((PIPE & 1) != 0) __builtin_amdgcn_s_setprio(0);
      return;
    }
    static_for<2>([&](auto kkc) {
      constexpr int kk = decltype(kkc)::value * 32;
      bf16x8 fa[MR], fb[NR];
#pragma unroll
      for (int m = 0; m < MR; ++m) fa[m] = frag<AMODE>(sa, wi_ * WM + m * 16, kk, lane);
#pragma unroll
      for (int n = 0; n < NR; ++n) fb[n] = frag<BMODE>(sb, wj_ * WN + n * 16, kk, lane);
      if constexpr ((PIPE & 1) != 0) __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int m = 0; m < MR; ++m)
#pragma unroll
        for (int n = 0; n < NR; ++n)
          acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[m], fb[n], acc[m][n], 0, 0, 0);
      if constexpr ((PIPE & 1) != 0) __builtin_amdgcn_s_setprio(0);
    });
  };

  // ---- main loop: STAGES-deep DMA ring
#pragma unroll
  for (int s = 0; s < STAGES - 1; ++s) issue(kt_beg + s, s);
  int st_read = 0, st_write = STAGES - 1;
  for (int t = 0; t < nt; ++t) {
    // exactly STAGES-2 tiles of this wave's DMAs may stay in flight beyond tile t
    wait_vmcnt<NPT * (STAGES - 2)>();
    block_barrier();  // every wave's DMAs of tile t have landed; every wave is done reading tile t-1
    issue(kt_beg + t + STAGES - 1, st_write);
    compute(st_read);
    st_read = st_read + 1 == STAGES ? 0 : st_read + 1;
    st_write = st_write + 1 == STAGES ? 0 : st_write + 1;
  }
  wait_vmcnt<0>();
  __syncthreads();  // stage buffers are reused by the epilogue

  // ---- epilogue: each wave stages 16 output rows (j) x WM columns (i) in LDS, then writes rows
  const int Mi = A.rows, Nj = B.rows;
  const int ibase = i0 + wi_ * WM, jbase = j0 + wj_ * WN;
  float *ep = reinterpret_cast<float *>(smem) + wave * 16 * (WM + 4);
  const float *bias = E.bias ? E.bias + g * E.bias_gstride : nullptr;
  // bf16 epilogue: a lane always serves the same 8 output columns (i), so their bias values
  // are loaded once here instead of once per output row
  constexpr int LPR_B = WM / 8;  // lanes per output row (8 bf16 per lane)
  const int il_b = (lane % LPR_B) * 8;
  constexpr bool BF = EPI == EPI_BF16 || EPI == EPI_BF16_DB || EPI == EPI_BF16_ADD;
  constexpr bool ADD = EPI == EPI_BF16_ADD;
  float bias8[8], bsum[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) bsum[e] = 0.f;
  if constexpr (BF) {
#pragma unroll
    for (int e = 0; e < 8; ++e) bias8[e] = (bias && ibase + il_b + e < Mi) ? bias[ibase + il_b + e] : 0.f;
  }
#pragma unroll
  for (int n = 0; n < NR; ++n) {
#pragma unroll
    for (int m = 0; m < MR; ++m)
      *reinterpret_cast<f32x4 *>(ep + (lane & 15) * (WM + 4) + m * 16 + (lane >> 4) * 4) = acc[m][n];
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
    constexpr bool kPartialLanes = (64 / (WM / 8)) * (WM / 8) < 64 || (64 / (WM / 4)) * (WM / 4) < 64;
    wave_lds_handoff<kPartialLanes>();
    if constexpr (BF) {
      bf16_t *out = reinterpret_cast<bf16_t *>(E.out) + g * E.gstride;
      constexpr int LPR = LPR_B;
      constexpr int RPI = 64 / LPR;  // rows per pass
      const int il = il_b;
      const int i = ibase + il;
      const bool vec_store = ((E.ldc & 7) == 0) && (i + 8 <= Mi);
      // second destination (E.out2): this lane's 8 columns lie on one side of split_i
      int ldc = E.ldc, ic = i;
      if (E.out2 != nullptr && i >= E.split_i) {
        out = reinterpret_cast<bf16_t *>(E.out2);
        ldc = E.ldc2;
        ic = i - E.split_i;
      }
      // relu'-mask: the fragment's old values are all loaded before its first store (a load
      // issued after a store waits for it: vmcnt counts both in issue order)
      constexpr int NIT = (16 + RPI - 1) / RPI;
      const int jl0 = lane < LPR * RPI ? lane / LPR : 16;
      uint4 oldv[NIT], addv[ADD ? NIT : 1];
      if (E.mask_relu && vec_store) {
#pragma unroll
        for (int k = 0; k < NIT; ++k) {
          const int jl = jl0 + k * RPI;
          if (jl < 16 && jbase + n * 16 + jl < Nj && i < Mi)
            oldv[k] = *reinterpret_cast<const uint4 *>(out + static_cast<long>(jbase + n * 16 + jl) * ldc + ic);
        }
      }
      const bf16_t *addp = ADD ? E.add + g * E.gstride : nullptr;
      if (ADD && vec_store) {
#pragma unroll
        for (int k = 0; k < NIT; ++k) {
          const int jl = jl0 + k * RPI;
          if (jl < 16 && jbase + n * 16 + jl < Nj && i < Mi)
            addv[k] = *reinterpret_cast<const uint4 *>(addp + static_cast<long>(jbase + n * 16 + jl) * ldc + ic);
        }
      }
#pragma unroll
      for (int k = 0; k < NIT; ++k) {  // WM = 96: 4 lanes idle
        const int jl = jl0 + k * RPI;
        const int j = jbase + n * 16 + jl;
        if (jl < 16 && j < Nj && i < Mi) {
          const f32x4 x0 = *reinterpret_cast<const f32x4 *>(ep + jl * (WM + 4) + il);
          const f32x4 x1 = *reinterpret_cast<const f32x4 *>(ep + jl * (WM + 4) + il + 4);
          float f[8] = {x0[0], x0[1], x0[2], x0[3], x1[0], x1[1], x1[2], x1[3]};
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            f[e] = f[e] * E.alpha + bias8[e];
            if (E.relu) f[e] = fmaxf(f[e], 0.f);
          }
          bf16_t *dst = out + static_cast<long>(j) * ldc + ic;
          if (vec_store) {
            if constexpr (ADD) {
              float a8[8];
              unpack8(addv[k], a8);
#pragma unroll
              for (int e = 0; e < 8; ++e) f[e] += a8[e];
            }
            if (E.mask_relu) {
              float old[8];
              unpack8(oldv[k], old);
#pragma unroll
              for (int e = 0; e < 8; ++e) f[e] = old[e] > 0.f ? f[e] : 0.f;
            }
            const uint4 packed = pack8(f);
            *reinterpret_cast<uint4 *>(dst) = packed;
            if constexpr (EPI == EPI_BF16_DB) {  // sum what was stored (bf16), as a separate pass would
              float r[8];
              unpack8(packed, r);
#pragma unroll
              for (int e = 0; e < 8; ++e) bsum[e] += r[e];
            }
          } else {
            for (int e = 0; e < 8 && i + e < Mi; ++e) {
              if constexpr (ADD) f[e] += bf2f(addp[static_cast<long>(j) * ldc + ic + e]);
              if (E.mask_relu && !(bf2f(dst[e]) > 0.f)) f[e] = 0.f;
              dst[e] = f2bf(f[e]);
              if constexpr (EPI == EPI_BF16_DB) bsum[e] += bf2f(dst[e]);
            }
          }
        }
      }
    } else if constexpr (EPI == EPI_F32_ATOMIC) {
      // one float per lane: every atomic instruction covers 64 consecutive floats of a row
      float *out = reinterpret_cast<float *>(E.out) + g * E.gstride;
#pragma unroll 4
      for (int jl = 0; jl < 16; ++jl) {
        const int j = jbase + n * 16 + jl;
#pragma unroll
        for (int u = 0; u < (WM + 63) / 64; ++u) {
          const int il = u * 64 + lane;
          const int i = ibase + il;
          if (j < Nj && il < WM && i < Mi)
            atomicAdd(out + static_cast<long>(j) * E.ldc + i, ep[jl * (WM + 4) + il] * E.alpha);
        }
      }
    } else if constexpr (EPI == EPI_F32_SGD) {
      // The fused SGD step is a memory stream (18 bytes per parameter: w and m read and written,
      // the bf16 shadow written).  All of this lane's w / m loads of the fragment are issued
      // before any store: loop iterations that store to w and m cannot be reordered by the
      // compiler (it cannot prove the rows distinct), so a load-compute-store loop kept one
      // HBM round trip in flight per lane (AlexNet fc6 at b32: 172 us for 680 MB).
      const SgdHyp hy = sgd_hyper(E);
      constexpr int LPR = WM / 4;
      constexpr int RPI = 64 / LPR;
      constexpr int NJL = (16 + RPI - 1) / RPI;
      const int il = (lane % LPR) * 4;
      const int i = ibase + il;
      const int jl0 = lane < LPR * RPI ? lane / LPR : 16;
      if (((E.ldc & 3) == 0) && (i + 4 <= Mi)) {
        f32x4 wv[NJL], mv[NJL];
#pragma unroll
        for (int r = 0; r < NJL; ++r) {
          const int jl = jl0 + r * RPI, j = jbase + n * 16 + jl;
          if (jl < 16 && j < Nj) {
            const long idx = static_cast<long>(j) * E.ldc + i;
            wv[r] = *reinterpret_cast<const f32x4 *>(E.sgd_w + idx);
            mv[r] = *reinterpret_cast<const f32x4 *>(E.sgd_m + idx);
          }
        }
#pragma unroll
        for (int r = 0; r < NJL; ++r) {
          const int jl = jl0 + r * RPI, j = jbase + n * 16 + jl;
          if (jl < 16 && j < Nj) {
            const long idx = static_cast<long>(j) * E.ldc + i;
            const f32x4 v = *reinterpret_cast<const f32x4 *>(ep + jl * (WM + 4) + il) * E.alpha;
            f32x4 w4 = wv[r], m4 = mv[r];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              float mm = m4[e];
              w4[e] = sgd_step(hy, v[e], mm, w4[e]);
              m4[e] = mm;
            }
            *reinterpret_cast<f32x4 *>(E.sgd_w + idx) = w4;
            *reinterpret_cast<f32x4 *>(E.sgd_m + idx) = m4;
            *reinterpret_cast<uint2 *>(E.sgd_wb + idx) = make_uint2(pack2(w4[0], w4[1]), pack2(w4[2], w4[3]));
          }
        }
      } else {
        for (int jl = jl0; jl < 16; jl += RPI) {
          const int j = jbase + n * 16 + jl;
          if (j < Nj && i < Mi) {
            const f32x4 v = *reinterpret_cast<const f32x4 *>(ep + jl * (WM + 4) + il) * E.alpha;
            const long idx = static_cast<long>(j) * E.ldc + i;
            for (int e = 0; e < 4 && i + e < Mi; ++e) {
              float mm = E.sgd_m[idx + e];
              const float wn = sgd_step(hy, v[e], mm, E.sgd_w[idx + e]);
              E.sgd_m[idx + e] = mm;
              E.sgd_w[idx + e] = wn;
              E.sgd_wb[idx + e] = f2bf(wn);
            }
          }
        }
      }
    } else {
      float *out = reinterpret_cast<float *>(E.out) + g * E.gstride;
      if constexpr (EPI == EPI_F32) out += wb.slice * E.kstride;
      constexpr int LPR = WM / 4;    // lanes per row, 4 floats per lane (16-byte accesses)
      constexpr int RPI = 64 / LPR;
      const int il = (lane % LPR) * 4;
      const int i = ibase + il;
      const bool vec = ((E.ldc & 3) == 0) && (i + 4 <= Mi);
#pragma unroll
      for (int jl = lane < LPR * RPI ? lane / LPR : 16; jl < 16; jl += RPI) {
        const int j = jbase + n * 16 + jl;
        if (j < Nj && i < Mi) {
          f32x4 v = *reinterpret_cast<const f32x4 *>(ep + jl * (WM + 4) + il) * E.alpha;
          {
            float *dst = out + static_cast<long>(j) * E.ldc + i;
            if (vec) {
              if constexpr (EPI == EPI_F32_ACC) v += *reinterpret_cast<const f32x4 *>(dst);
              *reinterpret_cast<f32x4 *>(dst) = v;
            } else {
              for (int e = 0; e < 4 && i + e < Mi; ++e) dst[e] = (EPI == EPI_F32_ACC ? dst[e] : 0.f) + v[e];
            }
          }
        }
      }
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);
    wave_lds_handoff<kPartialLanes>();
  }
  if constexpr (EPI == EPI_BF16_DB) {
    // lanes l and l + k * LPR_B served the same 8 columns: their sums meet in this wave's (now
    // free) staging area, then one fp32 atomic per column per wave
    static_assert(16 * (WM + 4) >= 64 * 9, "staging area holds the lane sums");
    constexpr int RPI_B = 64 / LPR_B;
#pragma unroll
    for (int e = 0; e < 8; ++e) ep[lane * 9 + e] = bsum[e];
    __builtin_amdgcn_s_waitcnt(0xc07f);
    wave_lds_handoff<true>();
    if (lane < LPR_B) {
      float *row = E.dbias + static_cast<long>(tj * WGN + wj_) * E.part_ld + g * E.bias_gstride;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float t = 0.f;
#pragma unroll
        for (int q = 0; q < RPI_B; ++q) t += ep[(lane + q * LPR_B) * 9 + e];
        const int i = ibase + lane * 8 + e;
        if (i < Mi) row[i] = t;
      }
    }
  }
}

// db[c] += sum_r part[r][c] (r < nrows, row stride ld): 32 columns x 8 row groups per block over
// one chunk of rows, one atomic per column per chunk (~10^3 adders per address at most)
__global__ void db_partials_reduce(const float *__restrict__ part, int nrows, int ld, float *__restrict__ db) {
  const int c = blockIdx.x * 32 + (threadIdx.x & 31);
  const int rg = threadIdx.x >> 5;
  const int per = (nrows + gridDim.y - 1) / gridDim.y;
  const int r0 = blockIdx.y * per, r1 = min(nrows, r0 + per);
  float acc = 0.f;
  if (c < ld)
    for (int r = r0 + rg; r < r1; r += 8) acc += part[static_cast<long>(r) * ld + c];
  __shared__ float red[8][33];
  red[rg][threadIdx.x & 31] = acc;
  __syncthreads();
  if (rg == 0 && c < ld) {
    float t = 0.f;
#pragma unroll
    for (int q = 0; q < 8; ++q) t += red[q][threadIdx.x & 31];
    atomicAdd(db + c, t);
  }
}

}  // namespace
namespace cxg {
// db[c] += column sums of the partial rows an EPI_BF16_DB epilogue wrote (conv_halo.hip uses it)
void launch_db_reduce(const GEpi &E, int rows, hipStream_t s) {
  const int chunks = (rows + 255) / 256;
  CXN_LAUNCH(db_partials_reduce, dim3((E.part_ld + 31) / 32, chunks), dim3(256), 0, s, E.dbias, rows, E.part_ld,
             E.dbias_final);
}
}  // namespace cxg
namespace {

template <int BM, int BN, int WGM, int WGN, int STAGES, int AMODE, int BMODE, int EPI, int PIPE = 0, int BMC = BM>
int launch(const GOperand &A, const GOperand &B, const GEpi &E, int groups, int ksplit, hipStream_t s) {
  const int ti = cdiv(A.rows, BMC), tj = cdiv(B.rows, BN);
  const int ktiles = cdiv(A.kdim, BK);
  ksplit = ksplit < 1 ? 1 : (ksplit > ktiles ? ktiles : ksplit);
  const int per = cdiv(ktiles, ksplit);
  ksplit = cdiv(ktiles, per);
  dim3 grid(ti * tj, ksplit, groups);
  if constexpr (EPI == EPI_BF16_DB) {
    const long rows = static_cast<long>(tj) * WGN;
    if (rows * E.part_ld > E.part_elems) return -1;  // workspace too small: the caller sums dx itself
  }
  CXN_LAUNCH((gemm_glds<BM, BN, WGM, WGN, STAGES, AMODE, BMODE, EPI, PIPE, BMC>), grid, dim3(64 * WGM * WGN), 0, s,
                     A, B, E, ti, tj, per, ktiles);
  if constexpr (EPI == EPI_BF16_DB) {
    const int rows = tj * WGN;
    const int chunks = (rows + 255) / 256;  // 256 rows per block: <= ~10^3 adders per address
    CXN_LAUNCH(db_partials_reduce, dim3((E.part_ld + 31) / 32, chunks), dim3(256), 0, s, E.dbias, rows,
                       E.part_ld, E.dbias_final);
  }
  return 0;
}




// Tile ids (BM x BN, wave grid, stages): only the tiles some shipped table entry uses
// (ops/glds_tune_gfx950.json) or a default pick (ops.gemm._pick_glds: 1 / 7 / 10 / 15; fc
// weight-grad 1) are compiled -- tests/test_tile_table_cpu.py checks both directions.
//   1: 128x128 (1x4) 2      2: 128x128 (2x2) 3      7: 64x128 (1x4) 2       10: 128x64 (2x2) 2
//  15: 64x64 (2x2) 3       17: 128x128 (2x2) 2
// 8 waves, two per SIMD: 21: 256x256 (2x4) 2   23: 128x128 (2x4) 3   25: 64x512 (1x8) 2
// PIPE variants (setprio around the MFMA clusters, both k-steps' fragments read ahead): 30, 31, 34,
// 37-41; 96-row 72 (96x128) / 96-column 75 (64x96); 32-row 76-78; 48 of 64 staged rows 79 (AlexNet
// conv2's 48-channel data-gradient); 82: 256x192 against wave quantisation (AlexNet conv3 dgrad).
// Tiles measured and retired (no table entry, rounds 2-4): 0, 13, 20, 33, 35, 36, 70, 71, 73, 74,
// 80, 81, 83, the segmented (50 / 51) and ping-pong (60 / 61) 8-wave pipelines, the MN-major 4w
// weight-gradient (120), 4w tiles 110-113 / 115 and the persistent 64-channel halo (132).
#define CXG_T(ID, BM, BN, WGM, WGN, ST) \
  case ID: return launch<BM, BN, WGM, WGN, ST, AM, BMo, EP>(A, B, E, groups, ksplit, s);
#define CXG_TP(ID, BM, BN, WGM, WGN, ST, PIPE) \
  case ID: return launch<BM, BN, WGM, WGN, ST, AM, BMo, EP, PIPE>(A, B, E, groups, ksplit, s);
#define CXG_TC(ID, BM, BMC, BN, WGM, WGN, ST) \
  case ID: return launch<BM, BN, WGM, WGN, ST, AM, BMo, EP, 0, BMC>(A, B, E, groups, ksplit, s);
#define CXG_KK_TILES                                                                                      \
  switch (tile) {                                                                                         \
    CXG_T(1, 128, 128, 1, 4, 2) CXG_T(7, 64, 128, 1, 4, 2) CXG_T(10, 128, 64, 2, 2, 2)                    \
    CXG_T(15, 64, 64, 2, 2, 3) CXG_T(21, 256, 256, 2, 4, 2) CXG_T(25, 64, 512, 1, 8, 2)                   \
    CXG_TP(30, 128, 256, 2, 4, 3, 0) CXG_TP(31, 128, 256, 2, 4, 3, 3) CXG_TP(34, 256, 256, 2, 4, 2, 3)    \
    CXG_TP(37, 64, 128, 1, 4, 2, 3) CXG_TP(38, 128, 256, 2, 4, 2, 3) CXG_TP(39, 64, 256, 2, 4, 3, 3)      \
    CXG_TP(72, 96, 128, 2, 2, 2, 0) CXG_TP(75, 64, 96, 2, 2, 2, 0)                                        \
    CXG_T(76, 32, 128, 1, 4, 2) CXG_T(77, 32, 64, 1, 4, 3) CXG_T(78, 32, 256, 1, 4, 2)                    \
    CXG_TC(79, 64, 48, 128, 1, 4, 2) CXG_TP(82, 256, 192, 2, 4, 2, 3)                                     \
    default: return -1;                                                                                   \
  }
#define CXG_MM_TILES  /* both MN-major (128 x 128) */                                                     \
  switch (tile) {                                                                                         \
    CXG_T(1, 128, 128, 1, 4, 2) CXG_T(2, 128, 128, 2, 2, 3) CXG_T(17, 128, 128, 2, 2, 2)                  \
    CXG_T(23, 128, 128, 2, 4, 3) CXG_TP(40, 128, 128, 1, 4, 2, 3) CXG_TP(41, 128, 128, 2, 2, 2, 3)        \
    default: return -1;                                                                                   \
  }
#define CXG_CASE(AMV, BMV, EPV, TILES)                       \
  if (amode == AMV && bmode == BMV && epi == EPV) {          \
    constexpr int AM = AMV, BMo = BMV, EP = EPV;             \
    TILES                                                    \
  }

int dispatch(int amode, int bmode, int epi, int tile, const GOperand &A, const GOperand &B, const GEpi &E,
             int groups, int ksplit, hipStream_t s) {
  if (tile == 114) return cxg::dispatch_4w(amode, bmode, epi, tile, A, B, E, groups, ksplit, s);
  if (tile >= 130 && tile <= 133) return cxg::dispatch_halo(amode, bmode, epi, tile, A, B, E, groups, ksplit, s);
  if (tile >= 140 && tile <= 142) return cxg::dispatch_wgrad_halo(amode, bmode, epi, tile, A, B, E, groups, s);
  CXG_CASE(K_DIRECT, K_GATHER, EPI_BF16, CXG_KK_TILES)    // conv fwd / dgrad
  CXG_CASE(K_DIRECT, K_GATHER, EPI_BF16_DB, CXG_KK_TILES)  // conv dgrad + the lower conv's bias gradient
  CXG_CASE(K_DIRECT, K_GATHER, EPI_BF16_ADD, CXG_KK_TILES)  // conv dgrad + a second gradient (split sum)
  CXG_CASE(K_DIRECT, K_ROWGATHER, EPI_BF16, CXG_KK_TILES)  // conv fwd, few input channels (conv1)
  CXG_CASE(K_DIRECT, K_DIRECT, EPI_BF16, CXG_KK_TILES)    // fc fwd
  CXG_CASE(K_DIRECT, K_DIRECT, EPI_F32, CXG_KK_TILES)     // fc fwd split-K
  CXG_CASE(MN_GATHER, MN_DIRECT, EPI_F32_ATOMIC, CXG_MM_TILES)  // conv wgrad
  CXG_CASE(MN_DIRECT, MN_DIRECT, EPI_F32, CXG_MM_TILES)   // fc wgrad (store)
  CXG_CASE(MN_DIRECT, MN_DIRECT, EPI_F32_ACC, CXG_MM_TILES)  // fc wgrad (+=)
  CXG_CASE(MN_DIRECT, MN_DIRECT, EPI_F32_SGD, CXG_MM_TILES)  // fc wgrad fused with the SGD step
  return -1;
}
#undef CXG_CASE
#undef CXG_MM_TILES
#undef CXG_KK_TILES
#undef CXG_T
#undef CXG_TC
#undef CXG_TP

}  // namespace

int cxg::g_gemm_group_i = 8;  // +7 % on 8192^3 (profiles/r3_gemm_tile_order.jsonl), neutral on the model steps

// Tile order of the LDS-DMA GEMM kernels: 0 = i fastest over all i-tiles; n > 0 = i fastest in
// groups of n i-tiles (common.h tile_ij).  Returns the previous setting.
CXN_API int cxn_gemm_set_group(int group_i) {
  const int old = cxg::g_gemm_group_i;
  cxg::g_gemm_group_i = group_i < 0 ? 0 : group_i;
  return old;
}

// Same operand record as cxn_gemm (gemm_mfma.hip).
struct CxnOperandG {
  const void *ptr;
  long gstride;
  long nbytes;
  int ld, rows, kdim;
  int H, W, C, Ho, Wo, KH, KW, stride, pad_h, pad_w, dil, Cg;
};

namespace {
// Byte alignment the kernel-row runs of the row gathers need (their 16-byte DMAs start at a
// pixel's first element): every image row (W*C*2 bytes) and every output-pixel step
// (stride*C*2) must be a multiple of it.  8: NHWC4 input (C = 4); CXXNET_ROWRUN_ALIGN overrides
// for probing (benchmarks/conv1_c3_probe.py).
static const int g_rowrun_align = [] {
  const char *e = getenv("CXXNET_ROWRUN_ALIGN");
  const int v = e ? atoi(e) : 8;
  return v > 0 ? v : 8;
}();
bool rowrun_aligned(const CxnOperandG *o) {
  return (o->W * o->C * 2) % g_rowrun_align == 0 && (o->stride * o->C * 2) % g_rowrun_align == 0;
}
bool supported(const CxnOperandG *o, int mode) {
  if (o->nbytes >= (1L << 31) || (reinterpret_cast<uintptr_t>(o->ptr) & 15) || o->gstride % 8 != 0) return false;
  if (mode == K_DIRECT || mode == MN_DIRECT) return o->ld % 8 == 0 && (mode == K_DIRECT || o->rows % 8 == 0);
  if (mode == K_ROWGATHER)  // whole kernel rows read as runs: no padding, one group, aligned pixels
    return o->pad_h == 0 && o->pad_w == 0 && o->Cg == o->C && rowrun_aligned(o) && o->dil <= 1 &&
           o->kdim == o->KH * ((o->KW * o->C + 7) / 8) * 8;
  if (o->Cg % 8 != 0 || o->dil > 1) return false;
  // MN gather over whole kernel rows (few-channel weight-grad, conv1): KW = 1 and Cg = a kernel row's
  // KW*C elements padded to 8, so a 16-byte chunk runs across pixels (aligned as the runs above)
  const bool row_runs = mode == MN_GATHER && o->KW == 1 && o->pad_h == 0 && o->pad_w == 0 && rowrun_aligned(o);
  if (o->C % 8 != 0 && !row_runs) return false;
  return mode == K_GATHER || o->rows % 8 == 0;
}
void fill(GOperand &r, const CxnOperandG *o, int mode) {
  r.ptr = static_cast<const bf16_t *>(o->ptr);
  r.gstride = o->gstride;
  r.nbytes = static_cast<uint32_t>(o->nbytes);
  r.ld = o->ld; r.rows = o->rows; r.kdim = o->kdim;
  if (mode == K_GATHER || mode == MN_GATHER) {
    r.H = o->H; r.W = o->W; r.C = o->C; r.Ho = o->Ho; r.Wo = o->Wo; r.KW = o->KW; r.KH = o->KH;
    r.stride = o->stride; r.pad_h = o->pad_h; r.pad_w = o->pad_w; r.Cg = o->Cg;
    r.fd_cg = make_fastdiv(o->Cg);
    r.fd_kw = make_fastdiv(o->KW > 0 ? o->KW : 1);
    r.fd_hw = make_fastdiv(o->Ho * o->Wo > 0 ? o->Ho * o->Wo : 1);
    r.fd_wo = make_fastdiv(o->Wo > 0 ? o->Wo : 1);
  }
  if (mode == K_ROWGATHER) {
    r.H = o->H; r.W = o->W; r.C = o->C; r.Ho = o->Ho; r.Wo = o->Wo; r.KW = o->KW; r.KH = o->KH;
    r.stride = o->stride; r.pad_h = r.pad_w = 0; r.Cg = o->Cg;
    r.rlc = (o->KW * o->C + 7) / 8;
    r.fd_rlc = make_fastdiv(r.rlc);
    r.fd_hw = make_fastdiv(o->Ho * o->Wo > 0 ? o->Ho * o->Wo : 1);
    r.fd_wo = make_fastdiv(o->Wo > 0 ? o->Wo : 1);
  }
}
}  // namespace

// Returns 0 on success, -1 unsupported configuration (the caller falls back), -3 launch error.
// Requirements: kdim % 8 == 0; 16-byte aligned rows; MN-major operands: rows % 8 == 0;
// gathers: Cg % 8 == 0 and dil == 1; every buffer < 2 GiB.
CXN_API int cxn_gemm_glds(const CxnOperandG *a, const CxnOperandG *b, int amode, int bmode, void *out,
                          long out_gstride, int ldc, float alpha, const float *bias, long bias_gstride, int relu,
                          int mask_relu, int epi, int tile, int groups, int ksplit, long kstride, float *dbias,
                          float *dws, long dws_elems, int dws_ld, void *stream) {
  if (a->kdim != b->kdim) return -1;
  if (epi == EPI_BF16_DB && (dbias == nullptr || dws == nullptr || ksplit > 1 || bias != nullptr)) return -1;
  if ((kmajor(amode) || kmajor(bmode)) && a->kdim % 8 != 0) return -1;
  if (!supported(a, amode) || !supported(b, bmode)) return -1;
  if (a->rows <= 0 || b->rows <= 0 || a->kdim <= 0) return 0;
  GOperand A{}, B{};
  fill(A, a, amode);
  fill(B, b, bmode);
  if (epi == EPI_F32_SGD) return -1;  // only through cxn_gemm_glds_sgd
  GEpi E{out, out_gstride, ldc, alpha, bias, bias_gstride, relu, mask_relu, kstride,
         nullptr, nullptr, nullptr, 0.f, 0.f, 0.f, 0.f, dws, dws_ld, dws_elems, dbias, g_gemm_group_i};
  hipStream_t s = static_cast<hipStream_t>(stream);
  const int rc = dispatch(amode, bmode, epi, tile, A, B, E, groups < 1 ? 1 : groups, ksplit < 1 ? 1 : ksplit, s);
  if (rc != 0) return rc;
  return hipGetLastError() == hipSuccess ? 0 : -3;
}

// cxn_gemm_glds with a second bf16 source added in the epilogue: out = mask(acc + add), add laid out
// like out (row stride ldc, group stride out_gstride).  The gemm_glds tiles of the dispatch switch
// only (not 114 / 130-142, whose epilogues do not read it); conv data-gradient operands (K_DIRECT
// weights x K_GATHER dy), no bias, no split-K.
CXN_API int cxn_gemm_glds_add(const CxnOperandG *a, const CxnOperandG *b, int amode, int bmode, void *out,
                              long out_gstride, int ldc, const void *add, int mask_relu, int tile, int groups,
                              void *stream) {
  if (a->kdim != b->kdim || add == nullptr || (ldc & 7) || tile == 114 || (tile >= 130 && tile <= 142)) return -1;
  if ((kmajor(amode) || kmajor(bmode)) && a->kdim % 8 != 0) return -1;
  if (!supported(a, amode) || !supported(b, bmode)) return -1;
  if (a->rows <= 0 || b->rows <= 0 || a->kdim <= 0) return 0;
  GOperand A{}, B{};
  fill(A, a, amode);
  fill(B, b, bmode);
  GEpi E{out, out_gstride, ldc, 1.f, nullptr, 0, 0, mask_relu, 0,
         nullptr, nullptr, nullptr, 0.f, 0.f, 0.f, 0.f, nullptr, 0, 0, nullptr, g_gemm_group_i};
  E.add = static_cast<const bf16_t *>(add);
  if (amode != K_DIRECT || bmode != K_GATHER) return -1;  // the one instantiated form
  const int rc = dispatch(amode, bmode, EPI_BF16_ADD, tile, A, B, E, groups < 1 ? 1 : groups, 1,
                          static_cast<hipStream_t>(stream));
  if (rc != 0) return rc;
  return hipGetLastError() == hipSuccess ? 0 : -3;
}

// cxn_gemm_glds with two bf16 destinations: output columns [0, split_i) to out (row stride
// ldc), [split_i, rows of A) to out2 (row stride ldc2) -- the sibling 1x1 convs of an inception
// module as one GEMM (NeuralNet._fuse_siblings).  Only the gemm_glds tiles of the dispatch switch
// (not 114 / 130-142, whose epilogues have one destination); EPI_BF16, no split-K.
CXN_API int cxn_gemm_glds_split(const CxnOperandG *a, const CxnOperandG *b, int amode, int bmode, void *out, int ldc,
                                void *out2, int ldc2, int split_i, const float *bias, int relu, int tile,
                                void *stream) {
  if (a->kdim != b->kdim || split_i <= 0 || split_i % 8 != 0 || split_i >= a->rows || (ldc & 7) || (ldc2 & 7))
    return -1;
  if (tile == 114 || (tile >= 130 && tile <= 142)) return -1;
  if ((kmajor(amode) || kmajor(bmode)) && a->kdim % 8 != 0) return -1;
  if (!supported(a, amode) || !supported(b, bmode)) return -1;
  if (b->rows <= 0 || a->kdim <= 0) return 0;
  GOperand A{}, B{};
  fill(A, a, amode);
  fill(B, b, bmode);
  GEpi E{out, 0, ldc, 1.f, bias, 0, relu, 0, 0,
         nullptr, nullptr, nullptr, 0.f, 0.f, 0.f, 0.f, nullptr, 0, 0, nullptr, g_gemm_group_i};
  E.out2 = out2;
  E.ldc2 = ldc2;
  E.split_i = split_i;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const int rc = dispatch(amode, bmode, EPI_BF16, tile, A, B, E, 1, 1, s);
  if (rc != 0) return rc;
  return hipGetLastError() == hipSuccess ? 0 : -3;
}

// fc weight-grad fused with the SGD step (single GPU, update_period 1): for every element of
// dw = alpha * B^T A (MN-major x and dy, ldc = nin) the epilogue applies
//   g = clip(dw); m = mom*m - lr*(g + wd*w); w += m; wb = bf16(w)
// to the layer's master / momentum / shadow slices instead of storing dw.
CXN_API int cxn_gemm_glds_sgd(const CxnOperandG *a, const CxnOperandG *b, int ldc, float alpha, float *w, float *m,
                              void *wb, float lr, float wd, float mom, float clip, const float *hyp, int tile,
                              void *stream) {
  if (a->kdim != b->kdim) return -1;
  if (!supported(a, MN_DIRECT) || !supported(b, MN_DIRECT)) return -1;
  if (a->rows % 4 != 0 || ldc % 4 != 0 || (reinterpret_cast<uintptr_t>(w) & 15) || (reinterpret_cast<uintptr_t>(m) & 15) ||
      (reinterpret_cast<uintptr_t>(wb) & 7))
    return -1;
  if (a->rows <= 0 || b->rows <= 0 || a->kdim <= 0) return 0;
  GOperand A{}, B{};
  fill(A, a, MN_DIRECT);
  fill(B, b, MN_DIRECT);
  GEpi E{nullptr, 0, ldc, alpha, nullptr, 0, 0, 0, 0, w, m, static_cast<bf16_t *>(wb), lr, wd, mom, clip, nullptr, 0, 0, nullptr,
         g_gemm_group_i, hyp};
  hipStream_t s = static_cast<hipStream_t>(stream);
  const int rc = dispatch(MN_DIRECT, MN_DIRECT, EPI_F32_SGD, tile, A, B, E, 1, 1, s);
  if (rc != 0) return rc;
  return hipGetLastError() == hipSuccess ? 0 : -3;
}
