// One-wave-per-SIMD bf16 MFMA GEMM with MN-major operands (tile id 120) for gfx950: the conv
// weight-gradient dW[oc][kh][kw][c] += sum over output pixels p of dy[p][oc] * x_col[p][(kh,kw,c)].
//
// Same contract as gemm_glds.hip's MN modes: C[j][i] (+)= alpha * sum_k A(i,k) B(j,k) with the
// K dimension (pixels) outermost in memory: A = the implicit im2col of an NHWC activation
// (MN_GATHER: column i = (kh, kw, c) of group g) or a plain [K][rows] matrix (MN_DIRECT), B = dy
// [pixels][Cout] (MN_DIRECT).  The weight-gradient GEMMs ran at 25-30 % MFMA busy with 4-5 VALU
// per MFMA and a third of the wave cycles parked at barriers on the 8-wave / register kernels
// (profiles/r3_pmc_alexnet_ops.md); this kernel carries gemm_4w.hip's remedies over:
//   * 4 waves, one per SIMD, 128 x 128 tile (2 x 2 waves of 64 x 64), the 4w schedule: k-step-0
//     MFMAs carry the k-step-1 fragment reads, a barrier, the DMAs of K-tile t+2 spread over the
//     MFMAs, a counted vmcnt wait + barrier, the last MFMAs carry the next K-tile's first reads;
//   * operand tiles are 64 k-rows (pixels) x 256 bytes (128 columns), XOR-swizzled at the
//     source exactly as gemm_glds's MN tiles (Op<MN_*> lane layout, frag<MN_*> transposed reads
//     with ds_read_b64_tr_b16), accumulators pinned in AGPRs (inline-asm MFMA);
//   * B (dy) DMAs are address-free: fixed per-lane offsets, the K advance moves the buffer
//     descriptor by 64 pixel rows, the shrinking record count zero-fills the pixels past P;
//   * A gather DMAs: a lane's 8 columns lie in ONE tap of the group (Cg % 8 == 0), so its tap
//     shift is fixed for the whole K loop; the lane's four pixel rows are tracked incrementally (+64 pixels per K-tile: wo, ho, n carries and the NHWC base
//     offset updated with adds), ~16 VALU per DMA, no divisions in the loop;
//   * epilogue: fp32 atomics into dW (split-K over pixel slices), or fp32 slabs (deterministic).
// Reference: src/layer/convolution_layer-inl.hpp:134-155 (the weight-gradient GEMM).
#include "gemm_glds_common.h"

using namespace cxg;

namespace {

__device__ __forceinline__ void lds_dma16m(const char *p, uint32_t n, char *dst, uint32_t voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(make_rsrc(p, n), (lds_void *)dst, 16, voff, 0, 0, 0);
}

template <int N>
__device__ __forceinline__ void wait_lgkm_m() {
  asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(N) : "memory");
}

__device__ __forceinline__ void mfma16m(f32x4 &acc, const bf16x8 &a, const bf16x8 &b) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
}

// MN-major staged tile (64 k-rows x 128 columns, 256-byte rows): the lane's logical 16-byte
// chunk for DMA instruction q = wave + 4 s (k-rows 4q .. 4q+3); identical to Op<MN_*>::init
// with 4 waves: chunk ^ 2 * ((k & 3) | ((k >> 3) & 1) << 2), k = 4q + lane / 16
__device__ __forceinline__ int mn_lchunk(int wave, int lane) {
  return (lane & 15) ^ (2 * ((lane >> 4) | (((wave >> 1) & 1) << 2)));
}

template <int AM, int EPI>
__global__ void __launch_bounds__(256, 1)
gemm_4m(GOperand A, GOperand B, GEpi E, int tiles_i, int tiles_j, int ksplit_tiles, int ktiles_total) {
  constexpr int BM = 128, BN = 128, NW = 4, WM = 64, WN = 64;
  constexpr int MR = WM / 16, NR = WN / 16;
  constexpr int KS = 2;                 // k-steps of 32 per K-tile
  constexpr int NA = 4, NB = 4;         // 1-KiB DMAs per wave per K-tile
  constexpr int NQ = NA + NB;
  constexpr int A_BYTES = BM * 128, STAGE = (BM + BN) * 128;
  constexpr int PER = MR * NR;          // MFMAs per k-step (16)
  constexpr int T = KS * PER;           // per K-tile (32)
  constexpr int NF = MR + NR;           // fragment reads per k-step (each two tr reads)
  constexpr int LA = PER, LC = NF + 6 < PER ? NF + 6 : PER;
  constexpr int DSPAN = T - LA;         // the DMAs ride on [B] + [C]
  constexpr int NQB = [&]() constexpr {
    int n = 0;
    for (int q = 0; q < NQ; ++q) n += (LA + q * DSPAN / NQ) < T - LC;
    return n;
  }();
  static_assert(LA + LC <= T && NF <= LC, "schedule");
  static_assert(NW * 16 * (WM + 4) * 4 <= 2 * STAGE, "epilogue staging fits");
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
  const int lch = mn_lchunk(wave, lane);
  const int krow = lane >> 4;  // + 4 (wave + 4 s): the lane's k-row of DMA s

  // ---- B (dy): fixed per-lane offsets; K-tile t at descriptor base + t * 64 rows
  const uint32_t goB = static_cast<uint32_t>(g * B.gstride) * 2u;
  uint32_t offB[NB];
  {
    const int col = j0 + lch * 8;
#pragma unroll
    for (int s = 0; s < NB; ++s)
      offB[s] = col < B.rows ? goB + static_cast<uint32_t>((4 * (wave + 4 * s) + krow) * B.ld + col) * 2u : OOB;
  }
  const uint32_t rowB = static_cast<uint32_t>(64 * B.ld) * 2u;  // bytes per K-tile

  // ---- A: MN_DIRECT as B, or the im2col gather with per-lane tap and tracked pixel rows
  const uint32_t goA = static_cast<uint32_t>(g * A.gstride) * 2u;
  const int colA = i0 + lch * 8;
  const bool colok = colA < A.rows;
  uint32_t offA[NA];  // MN_DIRECT: fixed offsets
  // MN_GATHER state per DMA row s: NHWC pixel index of the tap-shifted input pixel (pix), its
  // row / column (hi, wi, possibly outside the image), and the pixel limit of the row (lim)
  int pix[NA], phi[NA], pwi[NA], lim[NA];
  uint32_t cofs = 0;  // the lane's channel byte offset (+ group)
  int dwi = 0, dhi = 0, wlim = 0, hlim = 0, wwrap = 0, hwrap = 0, st = 1;
  int k0 = 0, k1 = 0, k2 = 0;  // pixel-index steps: plain / column carry / row carry
  if constexpr (AM == MN_DIRECT) {
#pragma unroll
    for (int s = 0; s < NA; ++s)
      offA[s] = colok ? goA + static_cast<uint32_t>((4 * (wave + 4 * s) + krow) * A.ld + colA) * 2u : OOB;
  } else {
    const int HWo = A.Ho * A.Wo;
    st = A.stride;
    int hoff = 0, woff = 0;
    if (colok) {
      const int q = colA / A.Cg, c = colA - q * A.Cg;
      const int kh = q / A.KW, kw = q - kh * A.KW;
      hoff = kh - A.pad_h;
      woff = kw - A.pad_w;
      cofs = goA + static_cast<uint32_t>(c) * 2u;
    }
    const int dn = 64 / HWo;
    const int dho = (64 - dn * HWo) / A.Wo;
    const int dwo = 64 - dn * HWo - dho * A.Wo;
    dwi = dwo * st;
    dhi = dho * st;
    wlim = A.Wo * st + woff;  // wi >= wlim <=> wo >= Wo
    hlim = A.Ho * st + hoff;
    wwrap = A.Wo * st;
    hwrap = A.Ho * st;
    k0 = dn * A.H * A.W + dhi * A.W + dwi;
    k1 = st * A.W - wwrap;
    k2 = A.H * A.W - hwrap * A.W;
#pragma unroll
    for (int s = 0; s < NA; ++s) {
      const int r = 4 * (wave + 4 * s) + krow;
      const int p = kt_beg * 64 + r;
      const int n = p / HWo, rem = p - n * HWo;
      const int ho = rem / A.Wo, wo = rem - ho * A.Wo;
      phi[s] = ho * st + hoff;
      pwi[s] = wo * st + woff;
      pix[s] = (n * A.H + phi[s]) * A.W + pwi[s];
      lim[s] = colok ? A.kdim - r : -(1 << 30);  // K-tile kt in range for this row: kt * 64 < lim
    }
  }
  // gather offset of DMA s for K-tile kt (tracked state): OOB past P, outside the image or the
  // group's columns (the K-tiles past the slice get a zero-range descriptor instead)
  auto offA_g = [&](int s, int kt) __attribute__((always_inline)) -> uint32_t {
    const bool ok = kt * 64 < lim[s] && static_cast<unsigned>(phi[s]) < static_cast<unsigned>(A.H) &&
                    static_cast<unsigned>(pwi[s]) < static_cast<unsigned>(A.W);
    uint32_t off = ok ? cofs + static_cast<uint32_t>(pix[s] * A.C) * 2u : OOB;
    asm volatile("" : "+v"(off));
    return off;
  };
  auto advance_g = [&]() __attribute__((always_inline)) {  // every tracked pixel row += 64
#pragma unroll
    for (int s = 0; s < NA; ++s) {
      int wi = pwi[s] + dwi, hi = phi[s] + dhi, add = k0;
      if (wi >= wlim) {
        wi -= wwrap;
        hi += st;
        add += k1;
      }
      if (hi >= hlim) {
        hi -= hwrap;
        add += k2;
      }
      pwi[s] = wi;
      phi[s] = hi;
      pix[s] += add;
    }
  };

  auto dmaA = [&](int kt, int stage, int s) __attribute__((always_inline)) {
    char *dst = smem + stage * STAGE + (wave + NW * s) * 1024;
    if constexpr (AM == MN_DIRECT) {
      const bool in = kt < kt_end;
      const uint32_t step = in ? static_cast<uint32_t>(kt) * static_cast<uint32_t>(64 * A.ld) * 2u : 0u;
      lds_dma16m(reinterpret_cast<const char *>(A.ptr) + step, in ? A.nbytes - step : 0u, dst, offA[s]);
    } else {
      lds_dma16m(reinterpret_cast<const char *>(A.ptr), kt < kt_end ? A.nbytes : 0u, dst, offA_g(s, kt));
    }
  };
  auto dmaB = [&](int kt, int stage, int s) __attribute__((always_inline)) {
    const bool in = kt < kt_end;
    const uint32_t step = in ? static_cast<uint32_t>(kt) * rowB : 0u;
    lds_dma16m(reinterpret_cast<const char *>(B.ptr) + step, in ? B.nbytes - step : 0u,
               smem + stage * STAGE + A_BYTES + (wave + NW * s) * 1024, offB[s]);
  };

  f32x4 acc[MR][NR];
#pragma unroll
  for (int m = 0; m < MR; ++m)
#pragma unroll
    for (int n = 0; n < NR; ++n) acc[m][n] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 fa[KS][MR], fb[KS][NR];
  auto read_frag = [&](int set, int f, int stage, int kk) __attribute__((always_inline)) {
    const char *base = smem + stage * STAGE;
    if (f < MR)
      fa[set][f] = frag<MN_DIRECT>(base, wr * WM + f * 16, kk, lane);
    else
      fb[set][f - MR] = frag<MN_DIRECT>(base + A_BYTES, wc * WN + (f - MR) * 16, kk, lane);
  };

  // prologue: K-tiles 0 and 1 in flight (the gather state walks one K-tile per issue)
#pragma unroll
  for (int s = 0; s < NA; ++s) dmaA(kt_beg, 0, s);
#pragma unroll
  for (int s = 0; s < NB; ++s) dmaB(kt_beg, 0, s);
  if constexpr (AM != MN_DIRECT) advance_g();
#pragma unroll
  for (int s = 0; s < NA; ++s) dmaA(kt_beg + 1, 1, s);
#pragma unroll
  for (int s = 0; s < NB; ++s) dmaB(kt_beg + 1, 1, s);
  if constexpr (AM != MN_DIRECT) advance_g();
  wait_vmcnt<NQ>();
  block_barrier();
#pragma unroll
  for (int f = 0; f < NF; ++f) read_frag(0, f, 0, 0);
  __builtin_amdgcn_sched_barrier(0);

  auto ktile = [&](auto stc, int t) __attribute__((always_inline)) {
    constexpr int ST = decltype(stc)::value;
    const int kt2 = kt_beg + t + 2;
    wait_lgkm_m<0>();  // the k-step-0 fragments
    __builtin_amdgcn_sched_barrier(0);
    static_for<T>([&](auto vc) {
      constexpr int v = decltype(vc)::value;
      constexpr int ks = v / PER, u = v % PER;
      if constexpr (v == LA) {
        wait_lgkm_m<0>();  // the k-step-1 reads are in: every wave is done with stage ST
        block_barrier();
      }
      if constexpr (v == T - LC) {
        wait_vmcnt<NQB>();  // this wave's DMAs of K-tile t+1 have landed
        block_barrier();
      }
      if constexpr (v >= LA) {
        static_for<NQ>([&](auto qc) {
          constexpr int q = decltype(qc)::value;
          if constexpr (v == LA + q * DSPAN / NQ) {
            if constexpr (q < NA)
              dmaA(kt2, ST, q);
            else
              dmaB(kt2, ST, q - NA);
            if constexpr (q == NA - 1 && AM != MN_DIRECT) advance_g();
          }
        });
      }
      mfma16m(acc[u / NR][u % NR], fa[ks][u / NR], fb[ks][u % NR]);
      if constexpr (v < LA) {
        if constexpr (v < NF) read_frag(1, v, ST, 32);  // [A]: k-step 1 of this K-tile
      } else if constexpr (v >= T - LC && v < T - LC + NF) {
        read_frag(0, v - (T - LC), ST ^ 1, 0);  // [C]: k-step 0 of K-tile t+1
      }
      __builtin_amdgcn_sched_barrier(0);
    });
  };
  int t = 0;
  for (; t + 1 < nt; t += 2) {
    ktile(std::integral_constant<int, 0>{}, t);
    ktile(std::integral_constant<int, 1>{}, t + 1);
  }
  if (t < nt) ktile(std::integral_constant<int, 0>{}, t);
  asm volatile("s_nop 15\n\ts_nop 15\n\ts_nop 15" ::: "memory");
  wait_vmcnt<0>();
  wait_lgkm_m<0>();
  __syncthreads();  // the epilogue stages through the operand buffers

  // epilogue: per 16-column fragment n of the wave (j), stage 16 j-rows x 64 i-columns, then
  // fp32 atomics (one float per lane: every atomic instruction covers a 64-float row segment)
  // or an fp32 split-K slab (deterministic mode)
  const int Mi = A.rows, Nj = B.rows;
  const int ibase = i0 + wr * WM, jbase = j0 + wc * WN;
  float *ep = reinterpret_cast<float *>(smem) + wave * 16 * (WM + 4);
#pragma unroll
  for (int n = 0; n < NR; ++n) {
#pragma unroll
    for (int m = 0; m < MR; ++m)
      *reinterpret_cast<f32x4 *>(ep + (lane & 15) * (WM + 4) + m * 16 + (lane >> 4) * 4) = acc[m][n];
    wait_lgkm_m<0>();
    if constexpr (EPI == EPI_F32_ATOMIC) {
      float *out = reinterpret_cast<float *>(E.out) + g * E.gstride;
      const int i = ibase + lane;
#pragma unroll 4
      for (int jl = 0; jl < 16; ++jl) {
        const int j = jbase + n * 16 + jl;
        if (j < Nj && i < Mi) atomicAdd(out + static_cast<long>(j) * E.ldc + i, ep[jl * (WM + 4) + lane] * E.alpha);
      }
    } else {
      write_staged<EPI_F32, 16, WM>(ep, E, g, wb.slice, Mi, Nj, ibase, jbase + n * 16, lane);
    }
    wait_lgkm_m<0>();
  }
}

template <int AM, int EPI>
void launch_4m(const GOperand &A, const GOperand &B, const GEpi &E, int groups, int ksplit, hipStream_t s) {
  const int ti = cdiv(A.rows, 128), tj = cdiv(B.rows, 128);
  const int ktiles = cdiv(A.kdim, BK);
  ksplit = ksplit < 1 ? 1 : (ksplit > ktiles ? ktiles : ksplit);
  const int per = cdiv(ktiles, ksplit);
  ksplit = cdiv(ktiles, per);
  CXN_LAUNCH((gemm_4m<AM, EPI>), dim3(ti * tj, ksplit, groups), dim3(256), 0, s, A, B, E, ti, tj, per, ktiles);
}

}  // namespace

namespace cxg {
// 120: 128 x 128, MN-major A (direct, or the weight-gradient im2col gather with Cg % 8 == 0) x
// MN-major B (direct); fp32 atomic or split-K slab epilogue.  -1 when unsupported.
int dispatch_4m(int amode, int bmode, int epi, int tile, const GOperand &A, const GOperand &B, const GEpi &E,
                int groups, int ksplit, hipStream_t s) {
  if (tile != 120 || bmode != MN_DIRECT || (amode != MN_DIRECT && amode != MN_GATHER)) return -1;
  if (A.kdim != B.kdim || (A.ld & 7) || (B.ld & 7)) return -1;
  if (amode == MN_GATHER) {
    if (A.Cg % 8 != 0 || A.C % 8 != 0 || A.KH * A.KW * A.Cg != A.rows || A.Ho * A.Wo <= 0) return -1;
    // tracked pixel rows advance by 64 with at most one carry per level
    if (A.Wo < 1 || A.Ho < 1) return -1;
  }
  if (static_cast<long>(A.nbytes) >= (1L << 31) || static_cast<long>(B.nbytes) >= (1L << 31)) return -1;
#define C4M(AMV, EPV) \
  if (amode == AMV && epi == EPV) { launch_4m<AMV, EPV>(A, B, E, groups, ksplit, s); return 0; }
  C4M(MN_GATHER, EPI_F32_ATOMIC)
  C4M(MN_GATHER, EPI_F32)
  C4M(MN_DIRECT, EPI_F32_ATOMIC)
  C4M(MN_DIRECT, EPI_F32)
#undef C4M
  return -1;
}
}  // namespace cxg
