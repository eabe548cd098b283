// Generic bf16 MFMA GEMM for gfx950 with pluggable operand loaders.
//
// One kernel template serves every GEMM-shaped op of the framework:
//   conv forward      (implicit im2col gather, NHWC)   -- reference K1+K2+K3+K4
//   conv data-grad    (gather over dY, flipped weights) -- reference K7+K8
//   conv weight-grad  (gather, split-K, fp32 atomics)   -- reference K6
//   fully-connected fwd / dgrad / wgrad                  -- reference K9/K10/K12
// (reference: src/layer/convolution_layer-inl.hpp:70-155, src/layer/fullc_layer-inl.hpp:101-130,
//  which do these as im2col + cuBLAS sgemm; here the im2col never exists in memory).
//
// Computes, per group g = blockIdx.z:
//     C[j][i] (+)= alpha * sum_k A(i, k) * B(j, k)          (i contiguous in C)
// A "rows" are i, B "rows" are j.  Each operand is loaded by one of four loaders:
//   DIRECT_K  : elem(row,k) = p[row*ld + k]        (k contiguous)
//   DIRECT_MN : elem(row,k) = p[k*ld + row]        (row contiguous)
//   GATHER_K  : rows = output pixels, k = (kh,kw,c)  -- im2col of an NHWC tensor
//   GATHER_MN : rows = (kh,kw,c),      k = pixels    -- transposed im2col
// K-major operands are staged into LDS as [rows][BK] and read with ds_read_b128;
// MN-major ones as [BK][rows] and read with ds_read_b64_tr_b16 (CDNA4 transpose read).
// Math: v_mfma_f32_16x16x32_bf16, fp32 accumulate, 4 waves (2x2) per 256-thread block,
// LDS double buffer with register staging (issue-early / write-late), one barrier per K step.
// Epilogue is staged through LDS so every global store / atomic is a full contiguous row.
#include <cstdlib>
#include <type_traits>
#include "common.h"

namespace {

enum { DIRECT_K = 0, DIRECT_MN = 1, GATHER_K = 2, GATHER_MN = 3 };
enum { EPI_BF16 = 0, EPI_F32 = 1, EPI_F32_ACC = 2, EPI_F32_ATOMIC = 3 };

constexpr int NT = 256;
constexpr int BK = 64;
constexpr int PADK = 16;  // K-major row pad (elements): conflict-free ds_read_b128 (see notes)
constexpr int PADM = 8;   // MN-major row pad (elements)

struct Operand {
  const bf16_t *ptr;
  long gstride;  // per-group element offset
  int ld;
  int rows;      // valid rows
  int kdim;      // valid k
  int vec_ok;    // 1 when 16-B/8-B vector loads are aligned and legal
  uint32_t nbytes;  // size of the whole buffer (all groups) for the load descriptor
  // gather geometry (GATHER_*): source NHWC tensor [N][H][W][C]
  int H, W, C, Ho, Wo, KH, KW, stride, pad_h, pad_w, dil, Cg;
  FastDiv fd_cg, fd_kw, fd_hw, fd_wo, fd_dil;
};

struct Epilogue {
  void *out;
  long gstride;
  int ldc;
  float alpha;
  const float *bias;  // indexed by i (nullable)
  long bias_gstride;
  int relu;
  int mask_relu;      // bf16 out: keep a value only where the OLD output value is > 0
  long kstride;       // EPI_F32 with split-K: K-slice s writes its own slab at out + s*kstride
};

template <int MODE>
struct KMajorLayout { static constexpr bool kmajor = (MODE == DIRECT_K || MODE == GATHER_K); };

// Per-thread staging registers for one operand tile.
template <int R, int VEC>
struct Stage {
  static constexpr int NV = R * BK / VEC / NT;  // vectors per thread
  typedef typename std::conditional<VEC == 8, uint4, uint2>::type vec_t;
  vec_t v[NV];
};

__device__ __forceinline__ uint4 zero_vec(uint4) { return make_uint4(0, 0, 0, 0); }
__device__ __forceinline__ uint2 zero_vec(uint2) { return make_uint2(0, 0); }

template <typename V>
__device__ __forceinline__ V load_vec(const bf16_t *p) { return *reinterpret_cast<const V *>(p); }

// Buffer loads: 32-bit byte offsets against a wave-uniform resource descriptor; an
// offset past num_records returns zeros, so padding / ragged edges need no branches.
constexpr uint32_t OOB = 0xFFFFFF00u;
typedef __amdgpu_buffer_rsrc_t rsrc_t;
__device__ __forceinline__ rsrc_t make_rsrc(const void *p, uint32_t nbytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), (short)0, static_cast<int>(nbytes), 0x00020000);
}
__device__ __forceinline__ uint4 bload(rsrc_t r, uint32_t off, uint4) {
  return __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
}
__device__ __forceinline__ uint2 bload(rsrc_t r, uint32_t off, uint2) {
  return __builtin_bit_cast(uint2, __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 0));
}

// Scalar fallback (unaligned / ragged edges): gather VEC elements one by one.
template <typename V, int VEC>
__device__ __forceinline__ V load_scalar(const bf16_t *base, long step, int n) {
  bf16_t t[VEC];
#pragma unroll
  for (int e = 0; e < VEC; ++e) t[e] = (e < n) ? base[e * step] : static_cast<bf16_t>(0);
  return *reinterpret_cast<V *>(t);
}

// Load one BK-deep tile of operand `op` starting at k0 into registers.
// Thread->vector assignment: K-major: v = tid + NT*s -> row = v / (BK/VEC), kv = v % (BK/VEC)
//                            MN-major: v = tid + NT*s -> k = v / (R/VEC), rv = v % (R/VEC)
// goff: byte offset of this group's slice within the operand's buffer.
template <int MODE, int R, int VEC>
__device__ __forceinline__ void load_tile(const Operand &op, rsrc_t rs, const bf16_t *gptr, uint32_t goff, int row0,
                                          int k0, Stage<R, VEC> &st, const int *prow) {
  typedef typename Stage<R, VEC>::vec_t V;
  const int tid = threadIdx.x;
  if constexpr (MODE == DIRECT_K) {
    constexpr int VPR = BK / VEC;
    if (op.vec_ok) {
#pragma unroll
      for (int s = 0; s < Stage<R, VEC>::NV; ++s) {
        const int v = tid + NT * s;
        const int row = row0 + v / VPR;
        const int k = k0 + (v % VPR) * VEC;
        const bool ok = row < op.rows && k + VEC <= op.kdim;
        st.v[s] = bload(rs, ok ? goff + static_cast<uint32_t>(row * op.ld + k) * 2u : OOB, V());
      }
    } else {
#pragma unroll
      for (int s = 0; s < Stage<R, VEC>::NV; ++s) {
        const int v = tid + NT * s;
        const int row = row0 + v / VPR;
        const int k = k0 + (v % VPR) * VEC;
        V val = zero_vec(V());
        if (row < op.rows && k < op.kdim) val = load_scalar<V, VEC>(gptr + static_cast<long>(row) * op.ld + k, 1,
                                                                    op.kdim - k);
        st.v[s] = val;
      }
    }
  } else if constexpr (MODE == DIRECT_MN) {
    constexpr int VPK = R / VEC;
    if (op.vec_ok) {
#pragma unroll
      for (int s = 0; s < Stage<R, VEC>::NV; ++s) {
        const int v = tid + NT * s;
        const int k = k0 + v / VPK;
        const int row = row0 + (v % VPK) * VEC;
        const bool ok = row + VEC <= op.rows && k < op.kdim;
        st.v[s] = bload(rs, ok ? goff + static_cast<uint32_t>(k * op.ld + row) * 2u : OOB, V());
      }
    } else {
#pragma unroll
      for (int s = 0; s < Stage<R, VEC>::NV; ++s) {
        const int v = tid + NT * s;
        const int k = k0 + v / VPK;
        const int row = row0 + (v % VPK) * VEC;
        V val = zero_vec(V());
        if (row < op.rows && k < op.kdim) val = load_scalar<V, VEC>(gptr + static_cast<long>(k) * op.ld + row, 1,
                                                                    op.rows - row);
        st.v[s] = val;
      }
    }
  } else if constexpr (MODE == GATHER_K) {
    // rows = output pixels (precomputed in prow: base offset, hi0, wi0 per owned row)
    constexpr int VPR = BK / VEC;
    const int k = k0 + (tid % VPR) * VEC;
    const uint32_t r = fdiv(static_cast<uint32_t>(k), op.fd_cg);
    const int c = k - static_cast<int>(r) * op.Cg;
    const uint32_t kh = fdiv(r, op.fd_kw);
    const int kw = static_cast<int>(r - kh * op.KW);
    const bool kin = k < op.kdim;
    const uint32_t coff = goff + static_cast<uint32_t>(c) * 2u;
#pragma unroll
    for (int s = 0; s < Stage<R, VEC>::NV; ++s) {
      const int base = prow[3 * s + 0];
      int hi = prow[3 * s + 1] + static_cast<int>(kh);
      int wi = prow[3 * s + 2] + kw;
      bool ok = kin && base >= 0;
      if (op.dil > 1) {  // dilated input (strided conv data-grad); uniform branch
        ok = ok && hi >= 0 && wi >= 0 && (hi % op.dil) == 0 && (wi % op.dil) == 0;
        hi /= op.dil;
        wi /= op.dil;
      }
      ok = ok && static_cast<unsigned>(hi) < static_cast<unsigned>(op.H) &&
           static_cast<unsigned>(wi) < static_cast<unsigned>(op.W);
      const uint32_t off = coff + static_cast<uint32_t>(base + (hi * op.W + wi) * op.C) * 2u;
      st.v[s] = bload(rs, ok ? off : OOB, V());
    }
  } else {  // GATHER_MN: rows = (kh, kw, c) filter taps, k = pixels
    constexpr int VPK = R / VEC;
    const int row = row0 + (tid % VPK) * VEC;
    const uint32_t r = fdiv(static_cast<uint32_t>(row), op.fd_cg);
    const int c = row - static_cast<int>(r) * op.Cg;
    const uint32_t kh = fdiv(r, op.fd_kw);
    const int kw = static_cast<int>(r - kh * op.KW);
    const bool rin = row < op.rows;
    const uint32_t coff = goff + static_cast<uint32_t>(c) * 2u;
    const int hoff = static_cast<int>(kh) - op.pad_h, woff = kw - op.pad_w;
    // pixel decomposition once, then advance incrementally by NT/VPK pixels per vector
    constexpr int PSTEP = NT / VPK;
    int p = k0 + tid / VPK;
    uint32_t n = fdiv(static_cast<uint32_t>(p), op.fd_hw);
    const uint32_t rem0 = static_cast<uint32_t>(p) - n * static_cast<uint32_t>(op.Ho * op.Wo);
    uint32_t ho = fdiv(rem0, op.fd_wo);
    uint32_t wo = rem0 - ho * op.Wo;
#pragma unroll
    for (int s = 0; s < Stage<R, VEC>::NV; ++s) {
      if (s > 0) {
        p += PSTEP;
        wo += PSTEP;
        while (wo >= static_cast<uint32_t>(op.Wo)) {
          wo -= op.Wo;
          if (++ho == static_cast<uint32_t>(op.Ho)) {
            ho = 0;
            ++n;
          }
        }
      }
      const int hi = static_cast<int>(ho) * op.stride + hoff;
      const int wi = static_cast<int>(wo) * op.stride + woff;
      const bool ok = rin && p < op.kdim && static_cast<unsigned>(hi) < static_cast<unsigned>(op.H) &&
                      static_cast<unsigned>(wi) < static_cast<unsigned>(op.W);
      const uint32_t off = coff + static_cast<uint32_t>(((static_cast<int>(n) * op.H + hi) * op.W + wi) * op.C) * 2u;
      st.v[s] = bload(rs, ok ? off : OOB, V());
    }
  }
}

// MN-major [BK][R] tiles of 64 or 128 columns are stored without a pad and with the 16-byte
// chunks of k-row k XOR-permuted, so the ds_read_b64_tr_b16 fragment reads (a 32-lane half reads
// k-rows {k0..k0+3, k0+8..k0+11}, 32 contiguous bytes each) hit 8 disjoint 8-bank groups.  The
// padded layout (row stride R+8) put those rows 4 banks apart: 2-way conflicts, ~33% of the
// LDS cycles of the weight-grad kernel (rocprofv3 SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE).
template <int R>
constexpr bool mn_swz() { return R == 128 || R == 64; }
template <int R>
constexpr int mn_stride() { return mn_swz<R>() ? R : R + PADM; }
template <int R>
__device__ __forceinline__ int mn_chunk_xor(int k) {
  if constexpr (R == 128) return 2 * ((k & 3) | (((k >> 3) & 1) << 2));
  else if constexpr (R == 64) return 2 * (((k >> 1) & 1) | (((k >> 3) & 1) << 1));
  else return 0;
}
// element offset of (k, col) in an MN-major tile; col % 4 == 0 (the 8-byte unit is never split)
template <int R>
__device__ __forceinline__ int mn_off(int k, int col) {
  if constexpr (mn_swz<R>()) return k * R + (((col >> 3) ^ mn_chunk_xor<R>(k)) << 3) + (col & 7);
  else return k * (R + PADM) + col;
}

template <int MODE, int R, int VEC>
__device__ __forceinline__ void store_tile(bf16_t *lds, const Stage<R, VEC> &st) {
  const int tid = threadIdx.x;
  typedef typename Stage<R, VEC>::vec_t V;
  if constexpr (KMajorLayout<MODE>::kmajor) {
    constexpr int VPR = BK / VEC;
#pragma unroll
    for (int s = 0; s < Stage<R, VEC>::NV; ++s) {
      const int v = tid + NT * s;
      *reinterpret_cast<V *>(lds + (v / VPR) * (BK + PADK) + (v % VPR) * VEC) = st.v[s];
    }
  } else {
    constexpr int VPK = R / VEC;
#pragma unroll
    for (int s = 0; s < Stage<R, VEC>::NV; ++s) {
      const int v = tid + NT * s;
      *reinterpret_cast<V *>(lds + mn_off<R>(v / VPK, (v % VPK) * VEC)) = st.v[s];
    }
  }
}

// Fragment for v_mfma_f32_16x16x32_bf16: lane l holds rows (l&15), k = 8*(l>>4) + e.
template <int MODE, int R>
__device__ __forceinline__ bf16x8 load_frag(const bf16_t *lds, int row, int kk) {
  const int lane = threadIdx.x & 63;
  if constexpr (KMajorLayout<MODE>::kmajor) {
    return *reinterpret_cast<const bf16x8 *>(lds + (row + (lane & 15)) * (BK + PADK) + kk + 8 * (lane >> 4));
  } else {
    const int i = lane & 15, g = lane >> 4;
    const int k = kk + 8 * g + (i >> 2);
    const bf16_t *p0 = lds + mn_off<R>(k, row + 4 * (i & 3));
    const bf16_t *p1 = lds + mn_off<R>(k + 4, row + 4 * (i & 3));
    s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4 *)(p0));
    s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4 *)(p1));
    typedef short s16x8 __attribute__((ext_vector_type(8)));
    s16x8 r = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8, r);
  }
}

template <int MODE, int R>
constexpr int tile_elems() {
  return KMajorLayout<MODE>::kmajor ? R * (BK + PADK) : BK * mn_stride<R>();
}

template <int BM, int BN, int WAVES_M, int AMODE, int BMODE, int VA, int VB, int EPI, int PF>
__global__ void __launch_bounds__(NT, 2)
gemm_kernel(Operand A, Operand B, Epilogue E, int tiles_i, int tiles_j, int ksplit_tiles, int ktiles_total) {
  constexpr int WAVES_N = 4 / WAVES_M;
  constexpr int WM = BM / WAVES_M, WN = BN / WAVES_N;  // per-wave tile
  static_assert(WM % 16 == 0 && WN % 16 == 0, "wave tile must be a multiple of 16");
  constexpr int MR = WM / 16, NR = WN / 16;
  constexpr int A_ELEMS = tile_elems<AMODE, BM>();
  constexpr int B_ELEMS = tile_elems<BMODE, BN>();
  constexpr int STAGE_BYTES = 2 * (A_ELEMS + B_ELEMS) * 2;
  constexpr int EPI_BYTES = 4 * WN * (WM + 4) * 4;
  constexpr int SMEM = STAGE_BYTES > EPI_BYTES ? STAGE_BYTES : EPI_BYTES;
  __shared__ __attribute__((aligned(16))) char smem[SMEM];
  bf16_t *const As0 = reinterpret_cast<bf16_t *>(smem);
  bf16_t *const Bs0 = As0 + 2 * A_ELEMS;

  const uint32_t nt = static_cast<uint32_t>(tiles_i) * tiles_j;
  const GemmBlock wb = gemm_block(nt);
  const int g = wb.g;
  const uint32_t tile = wb.tile;
  // i-tiles fastest within a j panel: neighbouring blocks share the B (j) panel.
  const int ti = tile % tiles_i, tj = tile / tiles_i;
  const int i0 = ti * BM, j0 = tj * BN;
  const int kt_beg = wb.slice * ksplit_tiles;
  const int kt_end = min(kt_beg + ksplit_tiles, ktiles_total);
  if (kt_beg >= kt_end) return;

  const bf16_t *gA = A.ptr + g * A.gstride;
  const bf16_t *gB = B.ptr + g * B.gstride;
  const rsrc_t rA = make_rsrc(A.ptr, A.nbytes);
  const rsrc_t rB = make_rsrc(B.ptr, B.nbytes);
  const uint32_t goA = static_cast<uint32_t>(g * A.gstride) * 2u;
  const uint32_t goB = static_cast<uint32_t>(g * B.gstride) * 2u;

  // Per-row gather geometry for GATHER_K operands (rows fixed per thread across K).
  constexpr int NVA = Stage<BM, VA>::NV, NVB = Stage<BN, VB>::NV;
  int rowA[3 * (AMODE == GATHER_K ? NVA : 1)];
  int rowB[3 * (BMODE == GATHER_K ? NVB : 1)];
  auto init_rows = [&](const Operand &op, int row0, int *pr, int nv, int vec) {
    const int vpr = BK / vec;
    for (int s = 0; s < nv; ++s) {
      const int p = row0 + (threadIdx.x + NT * s) / vpr;
      if (p < op.rows) {
        const uint32_t n = fdiv(static_cast<uint32_t>(p), op.fd_hw);
        const uint32_t rem = static_cast<uint32_t>(p) - n * static_cast<uint32_t>(op.Ho * op.Wo);
        const uint32_t ho = fdiv(rem, op.fd_wo);
        const uint32_t wo = rem - ho * op.Wo;
        pr[3 * s + 0] = static_cast<int>(n) * op.H * op.W * op.C;  // fits: activations < 2^31 elems
        pr[3 * s + 1] = static_cast<int>(ho) * op.stride - op.pad_h;
        pr[3 * s + 2] = static_cast<int>(wo) * op.stride - op.pad_w;
      } else {
        pr[3 * s + 0] = -1;
        pr[3 * s + 1] = 0;
        pr[3 * s + 2] = 0;
      }
    }
  };
  if constexpr (AMODE == GATHER_K) init_rows(A, i0, rowA, NVA, VA);
  if constexpr (BMODE == GATHER_K) init_rows(B, j0, rowB, NVB, VB);

  const int wave = threadIdx.x >> 6;
  const int wi = wave % WAVES_M, wj = wave / WAVES_M;
  f32x4 acc[MR][NR];
#pragma unroll
  for (int m = 0; m < MR; ++m)
#pragma unroll
    for (int n = 0; n < NR; ++n) acc[m][n] = f32x4{0.f, 0.f, 0.f, 0.f};

  const bf16_t *const as0 = As0, *const bs0 = Bs0;
  auto compute = [&](int cur) {
    const bf16_t *as = as0 + cur * A_ELEMS;
    const bf16_t *bs = bs0 + cur * B_ELEMS;
#pragma unroll
    for (int kk = 0; kk < BK; kk += 32) {
      bf16x8 fa[MR], fb[NR];
#pragma unroll
      for (int m = 0; m < MR; ++m) fa[m] = load_frag<AMODE, BM>(as, wi * WM + m * 16, kk);
#pragma unroll
      for (int n = 0; n < NR; ++n) fb[n] = load_frag<BMODE, BN>(bs, wj * WN + n * 16, kk);
#pragma unroll
      for (int m = 0; m < MR; ++m)
#pragma unroll
        for (int n = 0; n < NR; ++n)
          acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[m], fb[n], acc[m][n], 0, 0, 0);
    }
  };
  // k offset for a tile index; past the slice it is pushed beyond kdim, so the loads
  // become buffer-OOB (no memory traffic) and the loop body stays straight-line.
  constexpr int KOFF_NONE = 1 << 30;
  auto koff = [&](int kt) { return kt < kt_end ? kt * BK : KOFF_NONE; };

  if constexpr (PF == 1) {
    Stage<BM, VA> sa;
    Stage<BN, VB> sb;
    load_tile<AMODE, BM, VA>(A, rA, gA, goA, i0, kt_beg * BK, sa, rowA);
    load_tile<BMODE, BN, VB>(B, rB, gB, goB, j0, kt_beg * BK, sb, rowB);
    store_tile<AMODE, BM, VA>(As0, sa);
    store_tile<BMODE, BN, VB>(Bs0, sb);
    __syncthreads();
    int cur = 0;
    for (int kt = kt_beg; kt < kt_end; ++kt) {
      const bool more = kt + 1 < kt_end;
      if (more) {  // issue next tile's global loads early; they land under this step's MFMAs
        load_tile<AMODE, BM, VA>(A, rA, gA, goA, i0, (kt + 1) * BK, sa, rowA);
        load_tile<BMODE, BN, VB>(B, rB, gB, goB, j0, (kt + 1) * BK, sb, rowB);
      }
      compute(cur);
      if (more) {
        store_tile<AMODE, BM, VA>(As0 + (cur ^ 1) * A_ELEMS, sa);
        store_tile<BMODE, BN, VB>(Bs0 + (cur ^ 1) * B_ELEMS, sb);
      }
      __syncthreads();
      cur ^= 1;
    }
  } else {
    // Two register stages: tile t+2's loads are issued while tile t is computed and
    // tile t+1 (already in registers) waits to be written to the other LDS buffer, so
    // every global load has two K-steps of MFMA work to land under.
    Stage<BM, VA> sa0, sa1;
    Stage<BN, VB> sb0, sb1;
    load_tile<AMODE, BM, VA>(A, rA, gA, goA, i0, koff(kt_beg), sa0, rowA);
    load_tile<BMODE, BN, VB>(B, rB, gB, goB, j0, koff(kt_beg), sb0, rowB);
    load_tile<AMODE, BM, VA>(A, rA, gA, goA, i0, koff(kt_beg + 1), sa1, rowA);
    load_tile<BMODE, BN, VB>(B, rB, gB, goB, j0, koff(kt_beg + 1), sb1, rowB);
    store_tile<AMODE, BM, VA>(As0, sa0);
    store_tile<BMODE, BN, VB>(Bs0, sb0);
    __syncthreads();
    for (int kt = kt_beg; kt < kt_end; kt += 2) {
      load_tile<AMODE, BM, VA>(A, rA, gA, goA, i0, koff(kt + 2), sa0, rowA);
      load_tile<BMODE, BN, VB>(B, rB, gB, goB, j0, koff(kt + 2), sb0, rowB);
      compute(0);
      if (kt + 1 < kt_end) {
        store_tile<AMODE, BM, VA>(As0 + A_ELEMS, sa1);
        store_tile<BMODE, BN, VB>(Bs0 + B_ELEMS, sb1);
      }
      __syncthreads();
      if (kt + 1 >= kt_end) break;
      load_tile<AMODE, BM, VA>(A, rA, gA, goA, i0, koff(kt + 3), sa1, rowA);
      load_tile<BMODE, BN, VB>(B, rB, gB, goB, j0, koff(kt + 3), sb1, rowB);
      compute(1);
      if (kt + 2 < kt_end) {
        store_tile<AMODE, BM, VA>(As0, sa0);
        store_tile<BMODE, BN, VB>(Bs0, sb0);
      }
      __syncthreads();
    }
  }

  // ---- epilogue: stage the wave's fp32 tile in LDS as [j][i], then write full rows
  float *ep = reinterpret_cast<float *>(smem) + wave * WN * (WM + 4);
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int m = 0; m < MR; ++m)
#pragma unroll
    for (int n = 0; n < NR; ++n) {
      const int il = m * 16 + (lane >> 4) * 4;
      const int jl = n * 16 + (lane & 15);
      *reinterpret_cast<f32x4 *>(ep + jl * (WM + 4) + il) = acc[m][n];
    }
  __syncthreads();  // (wave-local region; barrier keeps the compiler's LDS ordering simple)

  const int ibase = i0 + wi * WM;
  const int jbase = j0 + wj * WN;
  const int Mi = A.rows, Nj = B.rows;
  const float *bias = E.bias ? E.bias + g * E.bias_gstride : nullptr;
  if constexpr (EPI == EPI_BF16) {
    constexpr int LPR = WM / 8;        // lanes per row, 8 elements per lane
    constexpr int RPI = 64 / LPR;      // rows per instruction (lanes >= LPR*RPI idle)
    bf16_t *out = reinterpret_cast<bf16_t *>(E.out) + g * E.gstride;
    const int il = (lane % LPR) * 8;
    const bool lane_on = lane < LPR * RPI;
    const int i = ibase + il;
    float bv[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) bv[e] = (bias && i + e < Mi) ? bias[i + e] : 0.f;
    const bool vec_store = ((E.ldc & 7) == 0) && (i + 8 <= Mi);
#pragma unroll 4
    for (int jl = lane / LPR; jl < WN; jl += RPI) {
      const int j = jbase + jl;
      if (j >= Nj || i >= Mi || !lane_on) continue;
      const f32x4 x0 = *reinterpret_cast<const f32x4 *>(ep + jl * (WM + 4) + il);
      const f32x4 x1 = *reinterpret_cast<const f32x4 *>(ep + jl * (WM + 4) + il + 4);
      float f[8] = {x0[0], x0[1], x0[2], x0[3], x1[0], x1[1], x1[2], x1[3]};
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        f[e] = f[e] * E.alpha + bv[e];
        if (E.relu) f[e] = fmaxf(f[e], 0.f);
      }
      bf16_t *dst = out + static_cast<long>(j) * E.ldc + i;
      // mask_relu: the destination holds the forward activation relu(z) of a fused
      // producer->relu pair; the data-grad it is overwritten with is masked by relu'(z).
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
  } else {
    float *out = reinterpret_cast<float *>(E.out) + g * E.gstride;
    if constexpr (EPI == EPI_F32) out += wb.slice * E.kstride;
    constexpr int LPR = WM;            // one fp32 per lane
    constexpr int RPI = 64 / LPR;
    const int il = lane % LPR;
    const int i = ibase + il;
    const bool lane_on = lane < LPR * RPI;
    const float bv = (bias && i < Mi) ? bias[i] : 0.f;
    for (int jl = lane / LPR; jl < WN; jl += RPI) {
      const int j = jbase + jl;
      if (j >= Nj || i >= Mi || !lane_on) continue;
      float v = ep[jl * (WM + 4) + il] * E.alpha + bv;
      float *dst = out + static_cast<long>(j) * E.ldc + i;
      if constexpr (EPI == EPI_F32) {
        *dst = E.relu ? fmaxf(v, 0.f) : v;
      } else if constexpr (EPI == EPI_F32_ACC) {
        *dst += v;
      } else {
        atomicAdd(dst, v);  // global_atomic_add_f32, 256 contiguous bytes per wave-instruction
      }
    }
  }
}

// ------------------------------------------------------------------ host side
struct GemmArgs {
  int amode, bmode, va, vb, epi;
  int tile;    // tile id, see TILES below
  int groups;
  int ksplit;  // number of K splits (>=1)
};

// Global-load prefetch depth of the K loop (1: one tile ahead, 2: two tiles ahead).
// CXXNET_GEMM_PF overrides the default; read once.
int gemm_prefetch_depth() {
  static const int d = [] {
    const char *e = std::getenv("CXXNET_GEMM_PF");
    return (e && e[0] == '1') ? 1 : 2;
  }();
  return d;
}

template <int BM, int BN, int WMs, int AM, int BMo, int VA, int VB, int EPI>
void launch_t(const Operand &A, const Operand &B, const Epilogue &E, int groups, int ksplit, hipStream_t s) {
  const int ti = cdiv(A.rows, BM), tj = cdiv(B.rows, BN);
  const int kdim = A.kdim;
  const int ktiles = cdiv(kdim, BK);
  ksplit = ksplit < 1 ? 1 : (ksplit > ktiles ? ktiles : ksplit);
  const int per = cdiv(ktiles, ksplit);
  ksplit = cdiv(ktiles, per);
  dim3 grid(ti * tj, ksplit, groups);
  if (gemm_prefetch_depth() == 1)
    CXN_LAUNCH((gemm_kernel<BM, BN, WMs, AM, BMo, VA, VB, EPI, 1>), grid, dim3(NT), 0, s, A, B, E, ti, tj,
                       per, ktiles);
  else
    CXN_LAUNCH((gemm_kernel<BM, BN, WMs, AM, BMo, VA, VB, EPI, 2>), grid, dim3(NT), 0, s, A, B, E, ti, tj,
                       per, ktiles);
}

// Tile ids (BM x BN, waves along M x N):
//   0: 128x128 (2x2)   1: 64x64 (2x2)   2: 64x128 (1x4)   3: 32x128 (1x4)
//   4: 96x128 (1x4)    5: 128x64 (2x2)   6: 128x96 (2x2)   7: 128x32 (4x1)
// (6 / 7: weight-grad tiles for 96- / 16..32-output-channel convs -- AlexNet conv1, GoogLeNet's
//  96/192/288-channel and 5x5-reduce layers -- whose j rows padded to 128 / 64 idled MFMA rows)
#define CXN_T0(AM, BMo, VA, VB, EPI) launch_t<128, 128, 2, AM, BMo, VA, VB, EPI>
#define CXN_T1(AM, BMo, VA, VB, EPI) launch_t<64, 64, 2, AM, BMo, VA, VB, EPI>
#define CXN_T2(AM, BMo, VA, VB, EPI) launch_t<64, 128, 1, AM, BMo, VA, VB, EPI>
#define CXN_T3(AM, BMo, VA, VB, EPI) launch_t<32, 128, 1, AM, BMo, VA, VB, EPI>
#define CXN_T4(AM, BMo, VA, VB, EPI) launch_t<96, 128, 1, AM, BMo, VA, VB, EPI>
#define CXN_T5(AM, BMo, VA, VB, EPI) launch_t<128, 64, 2, AM, BMo, VA, VB, EPI>
#define CXN_T6(AM, BMo, VA, VB, EPI) launch_t<128, 96, 2, AM, BMo, VA, VB, EPI>
#define CXN_T7(AM, BMo, VA, VB, EPI) launch_t<128, 32, 4, AM, BMo, VA, VB, EPI>

#define CXN_CASE(AM, BMo, VA, VB, EPI, TID)                                                         \
  if (g.amode == AM && g.bmode == BMo && g.va == VA && g.vb == VB && g.epi == EPI && g.tile == TID) { \
    CXN_T##TID(AM, BMo, VA, VB, EPI)(A, B, E, g.groups, g.ksplit, s);                               \
    return 0;                                                                                       \
  }
#define CXN_CASES_FC(AM, BMo, EPI) \
  CXN_CASE(AM, BMo, 8, 8, EPI, 0) CXN_CASE(AM, BMo, 8, 8, EPI, 1) CXN_CASE(AM, BMo, 8, 8, EPI, 5)

int dispatch(const GemmArgs &g, const Operand &A, const Operand &B, const Epilogue &E, hipStream_t s) {
  // fully-connected: fwd (K,K), dgrad (MN,K), wgrad (MN,MN)
  CXN_CASES_FC(DIRECT_K, DIRECT_K, EPI_BF16)
  CXN_CASES_FC(DIRECT_K, DIRECT_K, EPI_F32)
  CXN_CASES_FC(DIRECT_K, DIRECT_K, EPI_F32_ATOMIC)
  CXN_CASES_FC(DIRECT_MN, DIRECT_K, EPI_BF16)
  CXN_CASES_FC(DIRECT_MN, DIRECT_K, EPI_F32)
  CXN_CASES_FC(DIRECT_MN, DIRECT_K, EPI_F32_ATOMIC)
  CXN_CASES_FC(DIRECT_MN, DIRECT_MN, EPI_F32_ACC)
  CXN_CASES_FC(DIRECT_MN, DIRECT_MN, EPI_F32)
  CXN_CASES_FC(DIRECT_MN, DIRECT_MN, EPI_F32_ATOMIC)
  // convolution forward / data-grad (implicit im2col gather on B)
  CXN_CASE(DIRECT_K, GATHER_K, 8, 8, EPI_BF16, 0)
  CXN_CASE(DIRECT_K, GATHER_K, 8, 8, EPI_BF16, 1)
  CXN_CASE(DIRECT_K, GATHER_K, 8, 8, EPI_BF16, 2)
  CXN_CASE(DIRECT_K, GATHER_K, 8, 8, EPI_BF16, 3)
  CXN_CASE(DIRECT_K, GATHER_K, 8, 8, EPI_BF16, 4)
  CXN_CASE(DIRECT_K, GATHER_K, 4, 4, EPI_BF16, 0)
  CXN_CASE(DIRECT_K, GATHER_K, 4, 4, EPI_BF16, 2)
  CXN_CASE(DIRECT_K, GATHER_K, 4, 4, EPI_BF16, 3)
  CXN_CASE(DIRECT_K, GATHER_K, 4, 4, EPI_BF16, 4)
  // convolution weight-grad (transposed gather on A), split-K fp32 atomics
  CXN_CASE(GATHER_MN, DIRECT_MN, 8, 8, EPI_F32, 0)  // deterministic mode: per-slice fp32 slabs
  CXN_CASE(GATHER_MN, DIRECT_MN, 8, 8, EPI_F32, 5)
  CXN_CASE(GATHER_MN, DIRECT_MN, 4, 8, EPI_F32, 0)
  CXN_CASE(GATHER_MN, DIRECT_MN, 4, 8, EPI_F32, 5)
  CXN_CASE(GATHER_MN, DIRECT_MN, 8, 8, EPI_F32_ATOMIC, 0)
  CXN_CASE(GATHER_MN, DIRECT_MN, 8, 8, EPI_F32_ATOMIC, 5)
  CXN_CASE(GATHER_MN, DIRECT_MN, 4, 8, EPI_F32_ATOMIC, 0)
  CXN_CASE(GATHER_MN, DIRECT_MN, 4, 8, EPI_F32_ATOMIC, 5)
  CXN_CASE(GATHER_MN, DIRECT_MN, 8, 8, EPI_F32, 6)
  CXN_CASE(GATHER_MN, DIRECT_MN, 4, 8, EPI_F32, 6)
  CXN_CASE(GATHER_MN, DIRECT_MN, 8, 8, EPI_F32_ATOMIC, 6)
  CXN_CASE(GATHER_MN, DIRECT_MN, 4, 8, EPI_F32_ATOMIC, 6)
  CXN_CASE(GATHER_MN, DIRECT_MN, 8, 8, EPI_F32, 7)
  CXN_CASE(GATHER_MN, DIRECT_MN, 4, 8, EPI_F32, 7)
  CXN_CASE(GATHER_MN, DIRECT_MN, 8, 8, EPI_F32_ATOMIC, 7)
  CXN_CASE(GATHER_MN, DIRECT_MN, 4, 8, EPI_F32_ATOMIC, 7)
  return -1;
}
#undef CXN_CASE
#undef CXN_CASES_FC

}  // namespace

// Flat C ABI consumed by cxxnet_amd.ops (ctypes).  Returns 0 on success.
struct CxnOperand {
  const void *ptr;
  long gstride;
  long nbytes;
  int ld, rows, kdim;
  int H, W, C, Ho, Wo, KH, KW, stride, pad_h, pad_w, dil, Cg;
};

static Operand to_operand(const CxnOperand &o, int mode, int vec) {
  Operand r{};
  r.ptr = static_cast<const bf16_t *>(o.ptr);
  r.gstride = o.gstride;
  r.ld = o.ld;
  r.rows = o.rows;
  r.kdim = o.kdim;
  r.nbytes = o.nbytes > 0xFFFFFF00L ? 0xFFFFFF00u : static_cast<uint32_t>(o.nbytes);
  r.H = o.H; r.W = o.W; r.C = o.C; r.Ho = o.Ho; r.Wo = o.Wo; r.KH = o.KH; r.KW = o.KW;
  r.stride = o.stride; r.pad_h = o.pad_h; r.pad_w = o.pad_w; r.dil = o.dil < 1 ? 1 : o.dil; r.Cg = o.Cg;
  if (mode == GATHER_K || mode == GATHER_MN) {
    r.fd_cg = make_fastdiv(o.Cg > 0 ? o.Cg : 1);
    r.fd_kw = make_fastdiv(o.KW > 0 ? o.KW : 1);
    r.fd_hw = make_fastdiv(o.Ho * o.Wo > 0 ? o.Ho * o.Wo : 1);
    r.fd_wo = make_fastdiv(o.Wo > 0 ? o.Wo : 1);
    r.vec_ok = 1;
  } else {
    const uintptr_t a = reinterpret_cast<uintptr_t>(o.ptr);
    r.vec_ok = (o.ld % vec == 0) && (a % (vec * 2) == 0) && ((o.gstride % vec) == 0);
  }
  return r;
}

CXN_API int cxn_gemm(const CxnOperand *a, const CxnOperand *b, int amode, int bmode, int va, int vb,
                     void *out, long out_gstride, int ldc, float alpha, const float *bias, long bias_gstride,
                     int relu, int mask_relu, int epi, int tile, int groups, int ksplit, long kstride,
                     void *stream) {
  GemmArgs g{amode, bmode, va, vb, epi, tile, groups < 1 ? 1 : groups, ksplit < 1 ? 1 : ksplit};
  Operand A = to_operand(*a, amode, va), B = to_operand(*b, bmode, vb);
  if (A.kdim != B.kdim) return -2;
  if (A.rows <= 0 || B.rows <= 0 || A.kdim <= 0) return 0;
  Epilogue E{out, out_gstride, ldc, alpha, bias, bias_gstride, relu, mask_relu, kstride};
  hipStream_t s = static_cast<hipStream_t>(stream);
  int rc = dispatch(g, A, B, E, s);
  if (rc != 0) return rc;
  return hipGetLastError() == hipSuccess ? 0 : -3;
}
