// 256 x 256 bf16 MFMA GEMM tile with an 8-phase (two K-tiles) LDS-DMA pipeline for gfx950.
//
// Same contract and operand loaders as gemm_glds.hip (C[j][i] (+)= alpha * sum_k A(i,k) B(j,k),
// K-major A and B: weights / implicit-im2col gathers / fc operands); tile ids 90-95.
//
// Structure (the cdna guide's 256^2 8-phase template, adapted to this library's loaders):
//   * 8 waves (2 x 4), wave (wr, wc) owns output rows i0 + 128 wr .. +128 and columns
//     j0 + 64 wc .. +64: acc[8][4] of 16 x 16 fragments (128 accumulator registers);
//   * a K-tile (BK = 64) is staged as four HALF-TILES of 128 rows x 128 B (16 KiB, two 1-KiB
//     DMAs per wave), ordered by the phase that first reads them:
//       h0 = A rows of both wave rows' first 64-row halves (mh0)   read in phase 0
//       h1 = B rows of every wave column's first 32 rows (nh0)     read in phase 0
//       h2 = B rows nh1                                            read in phase 1
//       h3 = A rows mh1                                            read in phase 2
//     two K-tile buffers: 128 KiB of LDS, one block per CU;
//   * phase q of K-tile t reads its fragments, issues ONE half-tile of DMAs, waits with a
//     constant `s_waitcnt vmcnt(10)` (the 5 most recent half-tiles stay in flight), crosses a
//     barrier and runs 16 MFMAs (one 64 x 32 quadrant of the wave's tile, K = 64):
//       q   reads        MFMA quadrant   issues
//       0   A mh0, B nh0 (mh0, nh0)      h3 of K-tile t+1  (buffer t+1; its h3 was last read at t-1)
//       1   B nh1        (mh0, nh1)      h0 of K-tile t+2  (buffer t: h0 last read in phase 0)
//       2   A mh1        (mh1, nh1)      h1 of K-tile t+2  (h1 last read in phase 0; B nh0 in registers)
//       3   --           (mh1, nh0)      h2 of K-tile t+2  (h2 last read in phase 1)
//     so every DMA targets a half-tile whose readers all passed the barrier behind their reads,
//     and every half-tile is retired by a wait one phase before its first read;
//   * V = 0: a second barrier after the MFMAs (the template as written); V = 1: one barrier per
//     phase (the reads of phase q + 1 follow the MFMAs of phase q without a barrier; the
//     lgkmcnt(0) in front of each barrier keeps the WAR order);
//   * past the K slice the DMAs are all-OOB dummies (zeros), so the count never changes.
// Reference: src/layer/convolution_layer-inl.hpp:70-155, src/layer/fullc_layer-inl.hpp:101-130.
#include "gemm_glds_common.h"

using namespace cxg;

namespace {

template <int AMODE, int BMODE, int EPI, int V>
__global__ void __launch_bounds__(512, 1)
gemm_8p(GOperand A, GOperand B, GEpi E, int tiles_i, int tiles_j, int ksplit_tiles, int ktiles_total) {
  constexpr int NW = 8, WM = 128, WN = 64, MR = 8, NR = 4;
  constexpr int HALF = 128 * 128, BUF = 4 * HALF;
  static_assert(NW * 16 * (WM + 4) * 4 <= 2 * BUF, "epilogue staging fits");
  __shared__ __attribute__((aligned(1024))) char smem[2 * BUF];

  const uint32_t ntile = static_cast<uint32_t>(tiles_i) * tiles_j;
  const GemmBlock wb = gemm_block(ntile);
  const int g = wb.g;
  const uint32_t tile = wb.tile;
  int ti, tj;
  tile_ij(tile, tiles_i, tiles_j, E.group_i, ti, tj);
  const int i0 = ti * 256, j0 = tj * 256;
  const int kt_beg = wb.slice * ksplit_tiles;
  const int kt_end = min(kt_beg + ksplit_tiles, ktiles_total);
  if (kt_beg >= kt_end) return;
  const int nt = kt_end - kt_beg;

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wave >> 2, wc = wave & 3;
  const rsrc_t rA = make_rsrc(A.ptr, A.nbytes);
  const rsrc_t rB = make_rsrc(B.ptr, B.nbytes);
  const uint32_t goA = static_cast<uint32_t>(g * A.gstride) * 2u;
  const uint32_t goB = static_cast<uint32_t>(g * B.gstride) * 2u;

  // half-tile loaders: DMA s of a wave fills LDS rows lr = 8 (wave + 8 s) + lane/8 of its half
  using OA = Op<AMODE, 128, NW>;
  using OB = Op<BMODE, 128, NW>;
  static_assert(OA::NI == 2 && OB::NI == 2, "two DMAs per wave per half-tile");
  OA a0, a1;  // h0 (mh0 rows), h3 (mh1 rows)
  OB b0, b1;  // h1 (nh0 rows), h2 (nh1 rows)
  {
    const int lc = (lane & 7) ^ (((wave & 1) << 2) + (lane >> 4));
    a0.lchunk = a1.lchunk = b0.lchunk = b1.lchunk = lc;
    static_for<2>([&](auto sc) {
      constexpr int s = decltype(sc)::value;
      const int lr = 8 * (wave + NW * s) + (lane >> 3);
      // A: LDS rows 0-63 <- wave row 0's 64-row half, 64-127 <- wave row 1's (i0 + 128 + ...)
      a0.set_row(A, s, i0 + lr + 64 * s, goA);
      a1.set_row(A, s, i0 + 64 + lr + 64 * s, goA);
      // B: LDS rows 32 c .. 32 c + 31 <- wave column c's first (h1) / second (h2) 32 rows
      const int jb = j0 + (lr >> 5) * 64 + (lr & 31);
      b0.set_row(B, s, jb, goB);
      b1.set_row(B, s, jb + 32, goB);
    });
  }

  // every DMA of half-tile h of local K-tile t (buffer t & 1); dummies past the slice
  auto issue = [&](auto hc, int t) __attribute__((always_inline)) {
    constexpr int h = decltype(hc)::value;
    char *dst = smem + (t & 1) * BUF + h * HALF;
    const int kt = kt_beg + t;
    // (the loader is chosen with if constexpr: selecting a reference to one of two loader structs
    // made hipcc keep them in private memory, promoted to LDS)
    auto dma = [&](const auto &o, const GOperand &op, rsrc_t rs, uint32_t goff) __attribute__((always_inline)) {
      const auto p = o.prep(op, kt, kt_end, goff);
      static_for<2>([&](auto sc) {
        constexpr int s = decltype(sc)::value;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void *)(dst + (wave + NW * s) * 1024), 16,
                                                 o.template offset<s>(op, p, wave, lane), 0, 0, 0);
      });
    };
    if constexpr (h == 0) dma(a0, A, rA, goA);
    if constexpr (h == 3) dma(a1, A, rA, goA);
    if constexpr (h == 1) dma(b0, B, rB, goB);
    if constexpr (h == 2) dma(b1, B, rB, goB);
  };

  f32x4 acc[MR][NR];
#pragma unroll
  for (int m = 0; m < MR; ++m)
#pragma unroll
    for (int n = 0; n < NR; ++n) acc[m][n] = f32x4{0.f, 0.f, 0.f, 0.f};

  bf16x8 fa[4][2], fb0[2][2], fb1[2][2];
  auto read_a = [&](const char *half) __attribute__((always_inline)) {
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int k = 0; k < 2; ++k) fa[m][k] = frag<K_DIRECT>(half, wr * 64 + m * 16, 32 * k, lane);
  };
  auto read_b = [&](const char *half, bf16x8 (&fb)[2][2]) __attribute__((always_inline)) {
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
      for (int k = 0; k < 2; ++k) fb[n][k] = frag<K_DIRECT>(half, wc * 32 + n * 16, 32 * k, lane);
  };
  auto mfma_q = [&](int mb, int nb, const bf16x8 (&fb)[2][2]) __attribute__((always_inline)) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int k = 0; k < 2; ++k)
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int n = 0; n < 2; ++n)
          acc[mb + m][nb + n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[m][k], fb[n][k], acc[mb + m][nb + n], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };
  auto sync_in = [&]() {
    wait_vmcnt<10>();                      // half-tiles older than the 5 most recent have landed
    if constexpr (V == 1) __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this phase's reads done
    block_barrier();
  };
  auto sync_out = [&]() {
    if constexpr (V == 0) block_barrier();
  };

  // prologue: K-tile 0 whole, K-tile 1 h0-h2
  issue(std::integral_constant<int, 0>{}, 0);
  issue(std::integral_constant<int, 1>{}, 0);
  issue(std::integral_constant<int, 2>{}, 0);
  issue(std::integral_constant<int, 3>{}, 0);
  issue(std::integral_constant<int, 0>{}, 1);
  issue(std::integral_constant<int, 1>{}, 1);
  issue(std::integral_constant<int, 2>{}, 1);
  wait_vmcnt<10>();
  block_barrier();

  for (int t = 0; t < nt; ++t) {
    const char *buf = smem + (t & 1) * BUF;
    // phase 0
    read_a(buf);
    read_b(buf + HALF, fb0);
    issue(std::integral_constant<int, 3>{}, t + 1);
    sync_in();
    mfma_q(0, 0, fb0);
    sync_out();
    // phase 1
    read_b(buf + 2 * HALF, fb1);
    issue(std::integral_constant<int, 0>{}, t + 2);
    sync_in();
    mfma_q(0, 2, fb1);
    sync_out();
    // phase 2
    read_a(buf + 3 * HALF);
    issue(std::integral_constant<int, 1>{}, t + 2);
    sync_in();
    mfma_q(4, 2, fb1);
    sync_out();
    // phase 3
    issue(std::integral_constant<int, 2>{}, t + 2);
    sync_in();
    mfma_q(4, 0, fb0);
    sync_out();
  }
  wait_vmcnt<0>();
  __syncthreads();  // the epilogue reuses the stage buffers

  seg_epilogue<EPI, MR, NR, WM>(acc, smem, E, g, wb.slice, A.rows, B.rows, i0 + wr * WM, j0 + wc * WN, wave, lane);
}

template <int AMODE, int BMODE, int EPI, int V>
void launch_8p(const GOperand &A, const GOperand &B, const GEpi &E, int groups, int ksplit, hipStream_t s) {
  const int ti = cdiv(A.rows, 256), tj = cdiv(B.rows, 256);
  const int ktiles = cdiv(A.kdim, BK);
  ksplit = ksplit < 1 ? 1 : (ksplit > ktiles ? ktiles : ksplit);
  const int per = cdiv(ktiles, ksplit);
  ksplit = cdiv(ktiles, per);
  dim3 grid(ti * tj, ksplit, groups);
  hipLaunchKernelGGL((gemm_8p<AMODE, BMODE, EPI, V>), grid, dim3(512), 0, s, A, B, E, ti, tj, per, ktiles);
}

}  // namespace

namespace cxg {
// tiles 90 (template: two barriers per phase) and 91 (one barrier per phase)
int dispatch_8p(int amode, int bmode, int epi, int tile, const GOperand &A, const GOperand &B, const GEpi &E,
                int groups, int ksplit, hipStream_t s) {
#define CX8(AMV, BMV, EPV)                                                                       \
  if (amode == AMV && bmode == BMV && epi == EPV) {                                              \
    if (tile == 90) { launch_8p<AMV, BMV, EPV, 0>(A, B, E, groups, ksplit, s); return 0; }       \
    if (tile == 91) { launch_8p<AMV, BMV, EPV, 1>(A, B, E, groups, ksplit, s); return 0; }       \
  }
  CX8(K_DIRECT, K_GATHER, EPI_BF16)  // conv fwd / dgrad
  CX8(K_DIRECT, K_DIRECT, EPI_BF16)  // fc fwd, square GEMMs
  CX8(K_DIRECT, K_DIRECT, EPI_F32)   // fc fwd split-K
#undef CX8
  return -1;
}
}  // namespace cxg
