// Direct 3x3 / stride-1 / pad-1 convolution on a resident input halo (tile ids 130-133) for
// gfx950: VGG-16's high-resolution layers (conv1_2, conv2_x: 224^2 / 112^2 maps, 64-128
// channels), forward and stride-1 data-gradient (the same product with the flipped weights).
// Reference: src/layer/convolution_layer-inl.hpp:70-155 (im2col + GEMM).
//
// Why.  The implicit GEMM (gemm_glds / gemm_4w K_GATHER) fetches every output pixel's 9 taps on
// its own, so each input pixel crosses L2 -> LDS nine times per 64-channel block, and on these
// maps (few channels, 800k-3.2M pixels) that traffic, not the MFMAs, bounds the kernel: VGG
// conv1_2 forward ran at 27 % MFMA busy with 7.7 VALU per MFMA (profiles/r3_pmc_vgg16_ops.md).
// Here a block owns an R x WT patch of output pixels (256 pixels) x BM output channels and
// stages the (R + 2) x (WT + 2) input halo of one 64-channel block ONCE in LDS; the nine taps
// are nine shifted reads of the same halo:
//   * K loop: channel block cb (runtime) x tap (unrolled): one K-tile = the 64 channels of cb at
//     one tap.  The weights of a K-tile (BM x 64) stream through a 3-stage LDS ring by LDS-DMA
//     with fixed per-lane offsets (the K advance moves the buffer descriptor, as gemm_4w.hip);
//     9 taps per channel block make the stage tap % 3 a compile-time constant;
//   * halo rows are P = roundup8(WT + 2) pixel slots of 128 bytes; the 16-byte chunk c of slot s
//     holds logical chunk c ^ (s & 7).  P % 8 == 0 makes the key the slot's column & 7, so a
//     fragment read at tap (kh, kw) is a fixed per-lane base for (kw, k-step) plus an
//     immediate for (kh, fragment): no address arithmetic in the loop, and the b128 reads of 16
//     consecutive pixels hit 16 distinct bank slots for every kw (the key follows the column);
//   * with more than one channel block the halo is double-buffered: the next block's halo DMAs
//     ride two per wave on the first seven K-tiles of the current one (wait counts are
//     compile-time per tap; past the last block they are zero-range dummies into a 1-KiB sink);
//   * one barrier per K-tile: [A] k-step-0 MFMAs carrying the k-step-1 reads and the DMAs of
//     K-tile t+2; wait for t+1's weights; barrier; [B] k-step-1 MFMAs carrying the reads of
//     k-step 0 of t+1 (whose weights sit in a stage nobody reads any more, hence three stages);
//   * 4 waves (one per SIMD): BM = 64 -> 1 x 4 waves of 64 channels x 64 pixels; BM = 128 ->
//     2 x 2 waves of 64 x 128; accumulators pinned in AGPRs (inline-asm MFMA as gemm_4w.hip);
//   * epilogue: the 8-wave kernels' staged writer (bias, relu, relu'-mask of the old value),
//     one 16-pixel fragment (one row segment of the patch) at a time.
#include "gemm_glds_common.h"

using namespace cxg;

namespace cxg {
void launch_db_reduce(const GEpi &E, int rows, hipStream_t s);  // gemm_glds.hip
}

namespace {

__device__ __forceinline__ void lds_dma16h(const char *p, uint32_t n, char *dst, uint32_t voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(make_rsrc(p, n), (lds_void *)dst, 16, voff, 0, 0, 0);
}

template <int N>
__device__ __forceinline__ void wait_lgkm_h() {
  asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(N) : "memory");
}

__device__ __forceinline__ void mfma_h(f32x4 &acc, const bf16x8 &a, const bf16x8 &b) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
}

// an empty volatile asm that "rewrites" every accumulator: register code reading or writing
// them cannot move across it, and it keeps its order with the other volatile asm
template <int MR, int NR>
__device__ __forceinline__ void pin_acc(f32x4 (&acc)[MR][NR]) {
#pragma unroll
  for (int m = 0; m < MR; ++m)
#pragma unroll
    for (int n = 0; n < NR; ++n) asm volatile("" : "+a"(acc[m][n]));
}

constexpr int halo_pitch(int wt) { return (wt + 2 + 7) / 8 * 8; }

template <int BM, int WT, bool DBL>
struct HaloCfg {
  static constexpr int R = 256 / WT;                 // patch rows
  static constexpr int P = halo_pitch(WT);           // halo slots per row
  static constexpr int HR = R + 2;                   // halo rows
  static constexpr int HALO = HR * P * 128;          // bytes per halo buffer
  static constexpr int NG = HR * P / 8;              // 1-KiB DMA groups per halo
  static constexpr int NHD = (NG + 3) / 4;           // halo DMAs per wave
  static constexpr int NHB = DBL ? 2 : 1;            // halo buffers
  static constexpr int ASTAGE = BM * 128;            // weight K-tile
  static constexpr int A_OFF = NHB * HALO;
  static constexpr int SINK = A_OFF + 3 * ASTAGE;    // 1 KiB for dummy DMAs
  static constexpr int LDS = SINK + 1024;
  static constexpr int WGM = BM / 64, WGN = 4 / WGM;
  static constexpr int WM = 64, WN = 256 / WGN;
  static constexpr int MR = WM / 16, NR = WN / 16;
  static constexpr int NA = BM / 32;                 // weight DMAs per wave per K-tile
  static constexpr int NHK = DBL ? 2 : 0;            // next-halo DMAs per wave per K-tile (taps 0-6)
  static_assert(!DBL || 7 * NHK >= NHD, "next halo fits in seven K-tiles");
  static_assert(LDS <= 160 * 1024, "LDS");
  static_assert(WN % WT == 0, "a wave owns whole patch rows");
};

template <int BM, int WT, bool DBL, int EPI = EPI_BF16>
__global__ void __launch_bounds__(256, 1)
conv_halo(GOperand A, GOperand B, GEpi E, int tiles_o, int tiles_w, int tiles_h, int ncb) {
  using Cf = HaloCfg<BM, WT, DBL>;
  constexpr int P = Cf::P, HALO = Cf::HALO, NHD = Cf::NHD, NG = Cf::NG;
  constexpr int WM = Cf::WM, WN = Cf::WN, MR = Cf::MR, NR = Cf::NR, NA = Cf::NA, NHK = Cf::NHK;
  constexpr int PER = MR * NR, NF = MR + NR;
  __shared__ __attribute__((aligned(1024))) char smem[Cf::LDS];

  const uint32_t ntile = static_cast<uint32_t>(tiles_o) * tiles_w * tiles_h * B.Ho;  // B.Ho carries N
  const GemmBlock gb = gemm_block(ntile);
  uint32_t r = gb.tile;
  const int to = static_cast<int>(r % tiles_o); r /= tiles_o;
  const int tw = static_cast<int>(r % tiles_w); r /= tiles_w;
  const int th = static_cast<int>(r % tiles_h);
  const int img = static_cast<int>(r / tiles_h);
  const int H = B.H, W = B.W;
  const int h0 = th * Cf::R, w0 = tw * WT, i0 = to * BM;

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wave / Cf::WGN, wc = wave % Cf::WGN;
  const int l16 = lane & 15, g4 = lane >> 4;

  // weight DMAs: rows i0 + 8 (wave + 4 s) + lane / 8, swizzled chunk (as gemm_4w.hip)
  const int lchunk = (lane & 7) ^ (((wave & 1) << 2) + (lane >> 4));
  uint32_t offA[NA];
#pragma unroll
  for (int s = 0; s < NA; ++s) {
    const int row = i0 + 8 * (wave + 4 * s) + (lane >> 3);
    offA[s] = row < A.rows ? static_cast<uint32_t>(row * A.ld) * 2u + lchunk * 16u : OOB;
  }
  // halo DMAs: group q = wave + 4 s covers slots 8q .. 8q + 7; lane -> slot 8q + lane / 8,
  // physical chunk lane & 7 <- logical chunk (lane & 7) ^ (lane / 8)
  uint32_t offH[NHD];
#pragma unroll
  for (int s = 0; s < NHD; ++s) {
    const int q = wave + 4 * s;
    const int slot = 8 * q + (lane >> 3);
    const int hr = slot / P, hc = slot - hr * P;
    const int gh = h0 - 1 + hr, gw = w0 - 1 + hc;
    const bool ok = q < NG && hc < WT + 2 && static_cast<unsigned>(gh) < static_cast<unsigned>(H) &&
                    static_cast<unsigned>(gw) < static_cast<unsigned>(W);
    offH[s] = ok ? static_cast<uint32_t>(((img * H + gh) * W + gw) * B.C) * 2u + (((lane & 7) ^ (lane >> 3)) * 16u) : OOB;
  }
  auto halo_dst = [&](int buf, int s) -> char * {
    const int q = wave + 4 * s;
    return q < NG ? smem + buf * HALO + q * 1024 : smem + Cf::SINK;
  };
  // weight K-tile t = cb * 9 + tap: columns tap * C + 64 cb; past the last block: no records
  auto descA = [&](int cb, int tap, const char *&p, uint32_t &n) __attribute__((always_inline)) {
    const bool in = cb < ncb;
    const uint32_t step = in ? static_cast<uint32_t>(tap * B.Cg + 64 * cb) * 2u : 0u;
    p = reinterpret_cast<const char *>(A.ptr) + step;
    n = in ? A.nbytes - step : 0u;
  };
  auto issue_A = [&](int cb, int tap, int stage) __attribute__((always_inline)) {
    const char *p;
    uint32_t n;
    descA(cb, tap, p, n);
#pragma unroll
    for (int s = 0; s < NA; ++s) lds_dma16h(p, n, smem + Cf::A_OFF + stage * Cf::ASTAGE + (wave + 4 * s) * 1024, offA[s]);
  };
  auto halo_desc = [&](int cb, const char *&p, uint32_t &n) __attribute__((always_inline)) {
    const bool in = cb < ncb;
    p = reinterpret_cast<const char *>(B.ptr) + (in ? 128 * cb : 0);
    n = in ? B.nbytes - 128u * cb : 0u;
  };

  // per-lane fragment read bases.  A: row l16 of a 16-row block, chunk ((kk >> 3) + g4) ^ (row >> 1)
  const char *pa = smem + Cf::A_OFF + wr * WM * 128;
  const int fa_off0 = l16 * 128 + ((0 + g4) ^ (l16 >> 1)) * 16;
  const int fa_off1 = l16 * 128 + ((4 + g4) ^ (l16 >> 1)) * 16;
  // B: column l16 + kw of the patch row, logical chunk 4 kk + g4 at physical ^ ((l16 + kw) & 7)
  int fb_off[3][2];
#pragma unroll
  for (int kw = 0; kw < 3; ++kw)
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
      fb_off[kw][kk] = (l16 + kw) * 128 + (((4 * kk + g4) ^ ((l16 + kw) & 7)) * 16) + wc * (WN / WT) * P * 128;

  f32x4 acc[MR][NR];
#pragma unroll
  for (int m = 0; m < MR; ++m)
#pragma unroll
    for (int n = 0; n < NR; ++n) acc[m][n] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 fa[2][MR], fb[2][NR];

  // fragment f (< MR: weights of block f; else patch fragment f - MR) of k-step kk of K-tile
  // (tap, A stage st, halo buffer hb)
  auto read_frag = [&](int set, int f, int st, int hb, int tap, int kk) __attribute__((always_inline)) {
    if (f < MR) {
      fa[set][f] = *reinterpret_cast<const bf16x8 *>(pa + st * Cf::ASTAGE + f * 16 * 128 + (kk ? fa_off1 : fa_off0));
    } else {
      const int n = f - MR;
      const int kh = tap / 3, kw = tap % 3;
      const int rr = (16 * n) / WT, c0 = (16 * n) % WT;
      fb[set][n] = *reinterpret_cast<const bf16x8 *>(smem + hb * HALO + ((rr + kh) * P + c0) * 128 + fb_off[kw][kk]);
    }
  };

  // prologue: halo of block 0, weights of K-tiles 0 and 1
  {
    const char *p;
    uint32_t n;
    halo_desc(0, p, n);
#pragma unroll
    for (int s = 0; s < NHD; ++s) lds_dma16h(p, n, halo_dst(0, s), offH[s]);
    issue_A(0, 0, 0);
    issue_A(0, 1, 1);
  }
  wait_vmcnt<NA>();
  block_barrier();
#pragma unroll
  for (int f = 0; f < NF; ++f) read_frag(0, f, 0, 0, 0, 0);
  __builtin_amdgcn_sched_barrier(0);

  for (int cb = 0; cb < ncb; ++cb) {
    const int hb = DBL ? (cb & 1) : 0;
    const char *hp;
    uint32_t hn;
    halo_desc(cb + 1, hp, hn);  // next block's halo (zero-range past the last one)
    static_for<9>([&](auto tc) {
      constexpr int tap = decltype(tc)::value;
      constexpr int st = tap % 3;
      // DMAs riding on [A]: the weights of K-tile t + 2, then (taps 0-6) NHK of the next halo's
      constexpr int NQ = NA + (tap < 7 ? NHK : 0);
      wait_lgkm_h<0>();  // k-step-0 fragments of this K-tile
      __builtin_amdgcn_sched_barrier(0);
      static_for<PER>([&](auto uc) {
        constexpr int u = decltype(uc)::value;
        if constexpr (u == 0) {  // the weights of K-tile t + 2 (into the stage t - 1 used)
          const char *p;
          uint32_t n;
          descA(cb + (tap + 2) / 9, (tap + 2) % 9, p, n);
#pragma unroll
          for (int s = 0; s < NA; ++s)
            lds_dma16h(p, n, smem + Cf::A_OFF + ((tap + 2) % 3) * Cf::ASTAGE + (wave + 4 * s) * 1024, offA[s]);
        }
        if constexpr (NQ > NA) {  // then this K-tile's share of the next block's halo, spread out
          static_for<NHK>([&](auto jc) {
            constexpr int j = decltype(jc)::value;
            if constexpr (u == (j + 1) * PER / (NHK + 1)) {
              constexpr int hs = tap * NHK + j;  // this wave's halo DMA index
              if constexpr (hs < NHD) {
                lds_dma16h(hp, hn, halo_dst(hb ^ 1, hs), offH[hs]);
              } else {
                lds_dma16h(hp, 0u, smem + Cf::SINK, OOB);  // keeps the count fixed
              }
            }
          });
        }
        mfma_h(acc[u / NR][u % NR], fa[0][u / NR], fb[0][u % NR]);
        if constexpr (u < NF) read_frag(1, u, st, hb, tap, 1);
        __builtin_amdgcn_sched_barrier(0);
      });
      // [A] -> [B]: the weights of K-tile t + 1 (and, at tap 8, the next block's halo, issued
      // before them) have landed for this wave; the barrier makes them landed for every wave
      wait_lgkm_h<0>();
      wait_vmcnt<NQ>();
      block_barrier();
      static_for<PER>([&](auto uc) {
        constexpr int u = decltype(uc)::value;
        mfma_h(acc[u / NR][u % NR], fa[1][u / NR], fb[1][u % NR]);
        if constexpr (u < NF) {
          if constexpr (tap < 8) {
            read_frag(0, u, (tap + 1) % 3, hb, tap + 1, 0);
          } else {
            read_frag(0, u, 0, DBL ? (hb ^ 1) : 0, 0, 0);  // block cb + 1, tap 0 (stage 9 % 3)
          }
        }
        __builtin_amdgcn_sched_barrier(0);
      });
    });
  }
  asm volatile("s_nop 15\n\ts_nop 15\n\ts_nop 15" ::: "memory");
  wait_vmcnt<0>();
  wait_lgkm_h<0>();
  __syncthreads();  // the epilogue stages through the halo buffers

  // epilogue: one 16-pixel fragment (one patch-row segment) at a time
  float *ep = reinterpret_cast<float *>(smem) + wave * 16 * (WM + 4);
  float bv8[8];
  staged_bias<WM>(E, 0, A.rows, i0 + wr * WM, lane, bv8);
  float bsum[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int n = 0; n < NR; ++n) {
#pragma unroll
    for (int m = 0; m < MR; ++m)
      *reinterpret_cast<f32x4 *>(ep + l16 * (WM + 4) + m * 16 + g4 * 4) = acc[m][n];
    wait_lgkm_h<0>();
    const int p0 = wc * WN + 16 * n;
    const int h = h0 + p0 / WT, w = w0 + p0 % WT;
    const int valid = h < H ? min(16, W - w) : 0;
    const int jrow0 = (img * H + h) * W + w;
    write_staged<EPI_BF16, 16, WM>(ep, E, 0, 0, A.rows, jrow0 + max(valid, 0), i0 + wr * WM, jrow0, lane, bv8,
                                   EPI == EPI_BF16_DB ? bsum : nullptr);
    wait_lgkm_h<0>();
  }
  if constexpr (EPI == EPI_BF16_DB) {
    // the lower conv's bias gradient: lanes l, l + 8, ... summed the same 8 channels; their sums
    // meet in the wave's staging area and one row of the partials workspace per (patch, wave
    // column) takes them (rows: patch x WGN; db_partials_reduce adds the rows)
    constexpr int LPR = WM / 8, RPI = 64 / LPR;
    static_assert(16 * (WM + 4) >= 64 * 9, "staging area holds the lane sums");
#pragma unroll
    for (int e = 0; e < 8; ++e) ep[lane * 9 + e] = bsum[e];
    wait_lgkm_h<0>();
    if (lane < LPR) {
      float *row = E.dbias + static_cast<long>(gb.tile / static_cast<uint32_t>(tiles_o) * Cf::WGN + wc) * E.part_ld;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float t = 0.f;
#pragma unroll
        for (int q = 0; q < RPI; ++q) t += ep[(lane + q * LPR) * 9 + e];
        const int i = i0 + wr * WM + lane * 8 + e;
        if (i < A.rows) row[i] = t;
      }
    }
  }
}

template <int BM, int WT, bool DBL, int EPI = EPI_BF16>
int launch_halo(const GOperand &A, const GOperand &B, const GEpi &E, hipStream_t s) {
  const int N = B.Ho;
  const int tiles_o = cdiv(A.rows, BM), tiles_w = cdiv(B.W, WT), tiles_h = cdiv(B.H, HaloCfg<BM, WT, DBL>::R);
  const int ncb = B.Cg / 64;
  const long nt = static_cast<long>(tiles_o) * tiles_w * tiles_h * N;
  if (nt >= (1L << 31)) return -1;
  const long rows = nt / tiles_o * HaloCfg<BM, WT, DBL>::WGN;  // EPI_BF16_DB partial rows
  if (EPI == EPI_BF16_DB && rows * E.part_ld > E.part_elems) return -1;  // the caller sums dx itself
  CXN_LAUNCH((conv_halo<BM, WT, DBL, EPI>), dim3(static_cast<unsigned>(nt)), dim3(256), 0, s, A, B, E, tiles_o,
             tiles_w, tiles_h, ncb);
  if (EPI == EPI_BF16_DB) launch_db_reduce(E, static_cast<int>(rows), s);
  return 0;
}

// Persistent form for ONE output-channel block (tile 133: VGG conv1_2 forward / data-
// gradient, conv2_1 forward, conv2_2).  With one or two channel blocks the kernel above stages
// its first halo, runs its K-tiles and writes out with nothing overlapping the first halo's HBM
// fetch or the epilogue inside the block; conv1_2 ran at ~590 TFLOP/s against ~1,000 for the
// conv3-4 layers with 4-8 blocks.  Here one block per CU walks work items (patch, channel
// block) over an XCD-contiguous patch range (the patches an XCD runs together are neighbours and
// share halo rows in its L2).  The NEXT item's halo -- the next channel block of this patch, or
// block 0 of the next patch -- rides on the current item's K-tiles exactly as in the kernel
// above, and so do the next item's first two weight K-tiles (taps 7-8: the ring's t + 2 records;
// one output-channel block, so every patch uses the same weights).  After a patch's last channel
// block the epilogue stages through that item's halo buffer (no wave reads it after the tap-8
// barrier) and a barrier closes it before the item after next streams into that buffer.
template <int BM, int WT>
__global__ void __launch_bounds__(256, 1)
conv_halo_ps(GOperand A, GOperand B, GEpi E, int tiles_w, int tiles_h, uint32_t ntile, int ncb) {
  using Cf = HaloCfg<BM, WT, true>;
  constexpr int P = Cf::P, HALO = Cf::HALO, NHD = Cf::NHD, NG = Cf::NG;
  constexpr int WM = Cf::WM, WN = Cf::WN, MR = Cf::MR, NR = Cf::NR, NA = Cf::NA, NHK = Cf::NHK;
  constexpr int PER = MR * NR, NF = MR + NR;
  __shared__ __attribute__((aligned(1024))) char smem[Cf::LDS];

  // block b runs on XCD b % 8; XCD x owns patches [x ntile / 8, (x + 1) ntile / 8)
  const uint32_t g8 = gridDim.x / 8, xcd = blockIdx.x % 8;
  const uint32_t lo = static_cast<uint32_t>(static_cast<uint64_t>(ntile) * xcd / 8);
  const uint32_t hi = static_cast<uint32_t>(static_cast<uint64_t>(ntile) * (xcd + 1) / 8);
  uint32_t t = lo + blockIdx.x / 8;
  if (t >= hi) return;  // whole block, before any barrier
  const int H = B.H, W = B.W;
  auto coords = [&](uint32_t tt, int &h0, int &w0, int &img) {
    const int tw = static_cast<int>(tt % static_cast<uint32_t>(tiles_w));
    tt /= static_cast<uint32_t>(tiles_w);
    const int th = static_cast<int>(tt % static_cast<uint32_t>(tiles_h));
    img = static_cast<int>(tt / static_cast<uint32_t>(tiles_h));
    h0 = th * Cf::R;
    w0 = tw * WT;
  };

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wave / Cf::WGN, wc = wave % Cf::WGN;
  const int l16 = lane & 15, g4 = lane >> 4;

  const int lchunk = (lane & 7) ^ (((wave & 1) << 2) + (lane >> 4));
  uint32_t offA[NA];
#pragma unroll
  for (int s = 0; s < NA; ++s) {
    const int row = 8 * (wave + 4 * s) + (lane >> 3);
    offA[s] = row < A.rows ? static_cast<uint32_t>(row * A.ld) * 2u + lchunk * 16u : OOB;
  }
  // bias of the lane's accumulator rows (channel wr 64 + 16 m + 4 g4 + j), loaded once
  float bv[MR][4];
#pragma unroll
  for (int m = 0; m < MR; ++m)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int ch = wr * WM + 16 * m + 4 * g4 + j;
      bv[m][j] = (E.bias != nullptr && ch < A.rows) ? E.bias[ch] : 0.f;
    }
  // halo DMA offsets of the current patch (offH) and of the next item's halo (offN)
  uint32_t offH[NHD], offN[NHD];
  auto set_halo = [&](uint32_t (&off)[NHD], bool valid, int h0, int w0, int img) {
#pragma unroll
    for (int s = 0; s < NHD; ++s) {
      const int q = wave + 4 * s;
      const int slot = 8 * q + (lane >> 3);
      const int hr = slot / P, hc = slot - hr * P;
      const int gh = h0 - 1 + hr, gw = w0 - 1 + hc;
      const bool ok = valid && q < NG && hc < WT + 2 && static_cast<unsigned>(gh) < static_cast<unsigned>(H) &&
                      static_cast<unsigned>(gw) < static_cast<unsigned>(W);
      off[s] = ok ? static_cast<uint32_t>(((img * H + gh) * W + gw) * B.C) * 2u + (((lane & 7) ^ (lane >> 3)) * 16u) : OOB;
    }
  };
  auto halo_dst = [&](int buf, int s) -> char * {
    const int q = wave + 4 * s;
    return q < NG ? smem + buf * HALO + q * 1024 : smem + Cf::SINK;
  };
  const char *const wptr = reinterpret_cast<const char *>(A.ptr);
  // weight K-tile (cb, tap): columns tap * Cg + 64 cb; in = false: no records
  auto issue_A = [&](bool in, int cb, int tap, int stage) __attribute__((always_inline)) {
    const uint32_t step = in ? static_cast<uint32_t>(tap * B.Cg + 64 * cb) * 2u : 0u;
    const uint32_t n = in ? A.nbytes - step : 0u;
#pragma unroll
    for (int s = 0; s < NA; ++s)
      lds_dma16h(wptr + step, n, smem + Cf::A_OFF + stage * Cf::ASTAGE + (wave + 4 * s) * 1024, offA[s]);
  };

  const char *pa = smem + Cf::A_OFF + wr * WM * 128;
  const int fa_off0 = l16 * 128 + ((0 + g4) ^ (l16 >> 1)) * 16;
  const int fa_off1 = l16 * 128 + ((4 + g4) ^ (l16 >> 1)) * 16;
  int fb_off[3][2];
#pragma unroll
  for (int kw = 0; kw < 3; ++kw)
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
      fb_off[kw][kk] = (l16 + kw) * 128 + (((4 * kk + g4) ^ ((l16 + kw) & 7)) * 16) + wc * (WN / WT) * P * 128;

  f32x4 acc[MR][NR];
  bf16x8 fa[2][MR], fb[2][NR];
  auto read_frag = [&](int set, int f, int st, int hb, int tap, int kk) __attribute__((always_inline)) {
    if (f < MR) {
      fa[set][f] = *reinterpret_cast<const bf16x8 *>(pa + st * Cf::ASTAGE + f * 16 * 128 + (kk ? fa_off1 : fa_off0));
    } else {
      const int n = f - MR;
      const int kh = tap / 3, kw = tap % 3;
      const int rr = (16 * n) / WT, c0 = (16 * n) % WT;
      fb[set][n] = *reinterpret_cast<const bf16x8 *>(smem + hb * HALO + ((rr + kh) * P + c0) * 128 + fb_off[kw][kk]);
    }
  };

  int h0, w0, img;
  coords(t, h0, w0, img);
  set_halo(offH, true, h0, w0, img);
  const char *const hp = reinterpret_cast<const char *>(B.ptr);
#pragma unroll
  for (int s = 0; s < NHD; ++s) lds_dma16h(hp, B.nbytes, halo_dst(0, s), offH[s]);
  issue_A(true, 0, 0, 0);
  issue_A(true, 0, 1, 1);
  wait_vmcnt<NA>();
  block_barrier();
#pragma unroll
  for (int f = 0; f < NF; ++f) read_frag(0, f, 0, 0, 0, 0);
  __builtin_amdgcn_sched_barrier(0);

  int hb = 0, cb = 0;
  uint32_t tn = t;
  int h0n = h0, w0n = w0, imgn = img;
  for (;;) {
    const bool last_cb = cb == ncb - 1;
    bool more = true;
    int cbn = cb + 1;
    if (last_cb) {  // the next item is block 0 of the next patch (if any)
      tn = t + g8;
      more = tn < hi;
      cbn = 0;
      if (more) coords(tn, h0n, w0n, imgn);
      set_halo(offN, more, h0n, w0n, imgn);
    } else {
#pragma unroll
      for (int s = 0; s < NHD; ++s) offN[s] = offH[s];
    }
    const uint32_t hstep = more ? 128u * cbn : 0u;
    const char *const hpn = hp + hstep;
    const uint32_t hn = more ? B.nbytes - hstep : 0u;
    if (cb == 0) {
#pragma unroll
      for (int m = 0; m < MR; ++m)
#pragma unroll
        for (int n = 0; n < NR; ++n) acc[m][n] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    // accumulator writes, then wait states, then the first inline-asm MFMA.  The empty asm
    // statements pin the register writes above the s_nop (volatile asm keeps its order; plain
    // register code does not)
    pin_acc(acc);
    asm volatile("s_nop 7" ::: "memory");
    static_for<9>([&](auto tc) {
      constexpr int tap = decltype(tc)::value;
      constexpr int st = tap % 3;
      constexpr int NQ = NA + (tap < 7 ? NHK : 0);
      wait_lgkm_h<0>();
      __builtin_amdgcn_sched_barrier(0);
      static_for<PER>([&](auto uc) {
        constexpr int u = decltype(uc)::value;
        if constexpr (u == 0) {  // weights of K-tile t + 2: this item's, or taps 0-1 of the next
          if constexpr (tap + 2 < 9) issue_A(true, cb, tap + 2, (tap + 2) % 3);
          else issue_A(more, cbn, tap + 2 - 9, (tap + 2) % 3);
        }
        static_for<NHK>([&](auto jc) {
          constexpr int j = decltype(jc)::value;
          if constexpr (tap < 7 && u == (j + 1) * PER / (NHK + 1)) {
            constexpr int hs = tap * NHK + j;
            if constexpr (hs < NHD) {
              lds_dma16h(hpn, hn, halo_dst(hb ^ 1, hs), offN[hs]);
            } else {
              lds_dma16h(hp, 0u, smem + Cf::SINK, OOB);
            }
          }
        });
        mfma_h(acc[u / NR][u % NR], fa[0][u / NR], fb[0][u % NR]);
        if constexpr (u < NF) read_frag(1, u, st, hb, tap, 1);
        __builtin_amdgcn_sched_barrier(0);
      });
      wait_lgkm_h<0>();
      wait_vmcnt<NQ>();  // all but this tap's DMAs
      block_barrier();
      static_for<PER>([&](auto uc) {
        constexpr int u = decltype(uc)::value;
        mfma_h(acc[u / NR][u % NR], fa[1][u / NR], fb[1][u % NR]);
        if constexpr (u < NF) {
          if constexpr (tap < 8) {
            read_frag(0, u, (tap + 1) % 3, hb, tap + 1, 0);
          } else {
            read_frag(0, u, 0, hb ^ 1, 0, 0);  // next item, tap 0 (garbage past the last: unused)
          }
        }
        __builtin_amdgcn_sched_barrier(0);
      });
    });
    if (last_cb) {
      // MFMA results land after the wait states; pin_acc keeps every accumulator read below them
      // (without it hipcc hoisted the epilogue's AGPR reads and arithmetic above the s_nop and read
      // accumulators the last MFMAs had not written yet)
      asm volatile("s_nop 15\n\ts_nop 15\n\ts_nop 15" ::: "memory");
      pin_acc(acc);
      wait_lgkm_h<0>();
      // Epilogue.  alpha, bias and relu are applied in registers; the wave's bf16 [pixel][channel]
      // image of 64 pixels (16-byte chunk c of pixel p at c ^ (p & 7)) is staged in this item's
      // dead halo buffer and leaves as 16-byte row segments.  The 8-wave kernels' staged writer
      // loads the bias (and the relu'-mask's old value) next to every store, and in-order vmcnt
      // then makes each of those loads wait for the stores before it; here the bias sits in
      // registers and a half's mask loads are all issued before its first store.
      char *eb = smem + hb * HALO + wave * 8192;
      bf16_t *const out = reinterpret_cast<bf16_t *>(E.out);
      const int ic = wr * WM + (lane & 7) * 8;
      static_for<NR / 4>([&](auto hc) {
        constexpr int half = decltype(hc)::value;
#pragma unroll
        for (int n4 = 0; n4 < 4; ++n4) {
          const int pix = n4 * 16 + l16;
#pragma unroll
          for (int m = 0; m < MR; ++m) {
            const f32x4 v = acc[m][half * 4 + n4];
            float f[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              f[j] = v[j] * E.alpha + bv[m][j];
              if (E.relu) f[j] = fmaxf(f[j], 0.f);
            }
            const int c16 = 2 * m + (g4 >> 1);
            *reinterpret_cast<uint2 *>(eb + pix * 128 + ((c16 ^ (pix & 7)) * 16) + (g4 & 1) * 8) =
                make_uint2(pack2(f[0], f[1]), pack2(f[2], f[3]));
          }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        uint4 q[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const int pix = (lane >> 3) + 8 * k;
          q[k] = *reinterpret_cast<const uint4 *>(eb + pix * 128 + (((lane & 7) ^ (pix & 7)) * 16));
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // (the next half rewrites the image)
        long row[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const int pp = wc * WN + half * 64 + (lane >> 3) + 8 * k;
          const int h = h0 + pp / WT, w = w0 + pp % WT;
          row[k] = (h < H && w < W && ic < A.rows) ? (static_cast<long>(img * H + h) * W + w) * E.ldc + ic : -1;
        }
        if (E.mask_relu) {
          uint4 old[8];
#pragma unroll
          for (int k = 0; k < 8; ++k)
            if (row[k] >= 0) old[k] = *reinterpret_cast<const uint4 *>(out + row[k]);
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            if (row[k] >= 0) {
              float o[8], f[8];
              unpack8(old[k], o);
              unpack8(q[k], f);
#pragma unroll
              for (int e = 0; e < 8; ++e) f[e] = o[e] > 0.f ? f[e] : 0.f;
              q[k] = pack8(f);
            }
          }
        }
#pragma unroll
        for (int k = 0; k < 8; ++k)
          if (row[k] >= 0) *reinterpret_cast<uint4 *>(out + row[k]) = q[k];
      });
      block_barrier();  // staging reads done before the item after next streams into this buffer
      if (!more) break;
      t = tn;
      h0 = h0n;
      w0 = w0n;
      img = imgn;
#pragma unroll
      for (int s = 0; s < NHD; ++s) offH[s] = offN[s];
    }
    cb = cbn;
    hb ^= 1;
  }
  wait_vmcnt<0>();
}

int num_cu_h() {
  static const int n = [] {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0)
      v = 256;
    return v;
  }();
  return n;
}

template <int BM, int WT>
int launch_halo_ps(const GOperand &A, const GOperand &B, const GEpi &E, hipStream_t s) {
  const int N = B.Ho;
  const int tiles_w = cdiv(B.W, WT), tiles_h = cdiv(B.H, HaloCfg<BM, WT, true>::R);
  const long nt = static_cast<long>(tiles_w) * tiles_h * N;
  if (nt >= (1L << 31)) return -1;
  // one block per CU, a multiple of 8 (one share per XCD), no more than 8 x the patches per XCD
  long g = num_cu_h() / 8 * 8;
  const long per_xcd = (nt + 7) / 8;
  if (g / 8 > per_xcd) g = per_xcd * 8;
  if (g < 8) g = 8;
  CXN_LAUNCH((conv_halo_ps<BM, WT>), dim3(static_cast<unsigned>(g)), dim3(256), 0, s, A, B, E, tiles_w, tiles_h,
             static_cast<uint32_t>(nt), B.Cg / 64);
  return 0;
}

}  // namespace

namespace cxg {
// 130: 64 output channels per block, 131: 128; 133: the persistent form of 131 (one
// output-channel block only; its 64-channel form 132 was measured and retired).  The operands are the implicit-GEMM ones of a
// conv forward or stride-1 data-gradient (A: weights [rows][9 Cg], B: K_GATHER of an NHWC map);
// served: one group, 3 x 3, stride 1, pad 1, same-size output, Cg % 64 == 0, whole pixels of the
// B map addressable in 31 bits.  -1 otherwise (the caller falls back).
int dispatch_halo(int amode, int bmode, int epi, int tile, GOperand A, GOperand B, const GEpi &E, int groups, int ksplit,
                  hipStream_t s) {
  if (amode != K_DIRECT || bmode != K_GATHER || (epi != EPI_BF16 && epi != EPI_BF16_DB) || groups != 1 || ksplit > 1)
    return -1;
  const bool db = epi == EPI_BF16_DB;  // 130 / 131 only: + the lower conv's bias gradient
  if (B.KH != 3 || B.KW != 3 || B.stride != 1 || B.pad_h != 1 || B.pad_w != 1) return -1;
  if (B.Cg % 64 != 0 || B.kdim != 9 * B.Cg || A.kdim != B.kdim || A.ld < A.kdim) return -1;
  if (B.Ho != B.H || B.Wo != B.W) return -1;  // pad 1, stride 1: the output has the input's size
  const long pix = static_cast<long>(B.rows);
  if (pix % (static_cast<long>(B.H) * B.W) != 0) return -1;
  B.Ho = static_cast<int>(pix / (static_cast<long>(B.H) * B.W));  // images (the launcher's N)
  if (B.C % 8 != 0 || B.C < B.Cg || (E.ldc & 7) != 0) return -1;
  const bool wide = B.W % 32 == 0 || B.W % 16 != 0;
  const bool dbl = B.Cg > 64;
  if (db && (E.dbias == nullptr || E.dbias_final == nullptr || E.bias != nullptr)) return -1;
  if (db && tile == 130) {
    if (wide)
      return dbl ? launch_halo<64, 32, true, EPI_BF16_DB>(A, B, E, s) : launch_halo<64, 32, false, EPI_BF16_DB>(A, B, E, s);
    return dbl ? launch_halo<64, 16, true, EPI_BF16_DB>(A, B, E, s) : launch_halo<64, 16, false, EPI_BF16_DB>(A, B, E, s);
  }
  if (db && tile == 131) {
    if (wide)
      return dbl ? launch_halo<128, 32, true, EPI_BF16_DB>(A, B, E, s)
                 : launch_halo<128, 32, false, EPI_BF16_DB>(A, B, E, s);
    return dbl ? launch_halo<128, 16, true, EPI_BF16_DB>(A, B, E, s) : launch_halo<128, 16, false, EPI_BF16_DB>(A, B, E, s);
  }
  if (db) return -1;
  if (tile == 130) {
    if (wide) return dbl ? launch_halo<64, 32, true>(A, B, E, s) : launch_halo<64, 32, false>(A, B, E, s);
    return dbl ? launch_halo<64, 16, true>(A, B, E, s) : launch_halo<64, 16, false>(A, B, E, s);
  }
  if (tile == 131) {
    if (wide) return dbl ? launch_halo<128, 32, true>(A, B, E, s) : launch_halo<128, 32, false>(A, B, E, s);
    return dbl ? launch_halo<128, 16, true>(A, B, E, s) : launch_halo<128, 16, false>(A, B, E, s);
  }
  // persistent item walk: one output-channel block
  if (tile == 133) {
    if (A.rows % 8 != 0 || A.rows > 128) return -1;  // whole 16-byte output segments
    return wide ? launch_halo_ps<128, 32>(A, B, E, s) : launch_halo_ps<128, 16>(A, B, E, s);
  }
  return -1;
}
}  // namespace cxg
