// Shared pieces of the LDS-DMA GEMM kernels (gemm_glds.hip, gemm_4w.hip): operand records,
// epilogue record, LDS-DMA loaders, fragment readers and the 8-wave epilogue.
#pragma once
#include <utility>
#include "common.h"

namespace cxg {

constexpr int BK = 64;
constexpr uint32_t OOB = 0x80000000u;  // >= num_records: the load returns zeros
typedef __amdgpu_buffer_rsrc_t rsrc_t;
typedef __attribute__((address_space(3))) void lds_void;

enum { K_DIRECT = 0, K_GATHER = 1, MN_DIRECT = 2, MN_GATHER = 3, K_ROWGATHER = 4 };
// EPI_BF16_DB: the bf16 epilogue that also sums its stored output per column i -- a conv
// data-gradient that writes the gradient of the conv below it (through a fused relu) hands over
// that conv's bias gradient, so that gradient is never re-read.  Each wave writes its column sums
// as one row of a partials workspace (row = j-tile x wave column, no atomics: one fp32 atomic per
// column per wave put ~10^5 adders on each of VGG conv1_1's 64 addresses and ran 3.7x slower),
// and db_partials_reduce adds the rows into dbias.
// EPI_BF16_ADD: EPI_BF16 plus a second bf16 source summed before the store (GEpi.add; its own
// instantiation, so the plain bf16 epilogue carries none of its registers)
enum { EPI_BF16 = 0, EPI_F32 = 1, EPI_F32_ACC = 2, EPI_F32_ATOMIC = 3, EPI_F32_SGD = 4, EPI_BF16_DB = 5, EPI_BF16_ADD = 6 };

struct GOperand {
  const bf16_t *ptr;
  long gstride;     // per-group element offset
  uint32_t nbytes;  // descriptor range (all groups)
  int ld, rows, kdim;
  int H, W, C, Ho, Wo, KW, stride, pad_h, pad_w, Cg;  // gather geometry (NHWC source)
  int KH, rlc;  // row gather: kernel rows, 16-byte chunks per (zero-padded) kernel-row run
  FastDiv fd_cg, fd_kw, fd_hw, fd_wo, fd_rlc;
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
  // EPI_F32_SGD (fc weight-grad fused with the SGD step): the gradient element never goes to
  // memory; w (fp32 master), m (momentum) and the bf16 shadow wb are updated in place, with
  // the fused optimizer's exact arithmetic (optim_kernels.hip step1, algo 0)
  float *sgd_w, *sgd_m;
  bf16_t *sgd_wb;
  float lr, wd, mom, clip;
  float *dbias;  // EPI_BF16_DB: partials workspace [tiles_j * WGN][part_ld] (column g * bias_gstride + i)
  int part_ld;
  long part_elems;     // workspace capacity
  float *dbias_final;  // += the workspace's column sums (db_partials_reduce)
  int group_i;         // tile order (common.h tile_ij); set at launch from cxn_gemm_set_group
  // EPI_F32_SGD: when set, (lr, wd, mom, clip) are read from this device array instead of the
  // fields above -- a recorded / captured step then takes each replay's schedule values
  const float *sgd_hyp;
  // bf16 epilogues of gemm_glds (tiles of its dispatch switch): output columns i >= split_i go
  // to out2 (row stride ldc2) at column i - split_i instead (sibling 1x1 convs sharing one
  // GEMM, NeuralNet._fuse_siblings); out2 == nullptr: one destination.  split_i % 8 == 0.
  void *out2;
  int ldc2, split_i;
  // EPI_BF16_ADD epilogue of the gemm_glds tiles: out = f(acc + add) with add a bf16 matrix laid
  // out like out (same gstride / ldc) -- a data-gradient GEMM summing a second gradient into its
  // node instead of a separate add pass (the split after a sibling group, NeuralNet._fuse_siblings)
  const bf16_t *add;
};

}  // namespace cxg
namespace cxg {
// host-side tile-order setting copied into every GEpi at launch (cxn_gemm_set_group)
extern int g_gemm_group_i;

struct SgdHyp {
  float lr, wd, mom, clip;
};
__device__ __forceinline__ SgdHyp sgd_hyper(const GEpi &E) {
  if (E.sgd_hyp) return {E.sgd_hyp[0], E.sgd_hyp[1], E.sgd_hyp[2], E.sgd_hyp[3]};
  return {E.lr, E.wd, E.mom, E.clip};
}
__device__ __forceinline__ float sgd_step(const SgdHyp &h, float g, float &m, float w) {
  if (h.clip != 0.f) g = (g != g) ? 0.f : fminf(fmaxf(g, -h.clip), h.clip);
  m = fmaf(h.mom, m, -h.lr * fmaf(h.wd, w, g));  // as optim_kernels.hip step1 (SGD)
  return w + m;
}

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

// Lanes of ONE wave hand data to each other through LDS in the epilogues (stage the fp32 tile,
// then read whole rows).  In the per-lane memory model that is a race unless fenced: when some
// lanes sit out the row loop (WM = 48 / 96: 60 of 64 lanes busy) hipcc hoisted the idle lanes'
// next staging stores above the other lanes' reads (96-row tiles: rows 12-15 x 12-15 of every
// 16 x 16 block wrong).  Fence + wave barrier pin the order; emitted only for those tile
// widths so the kernels of the shipped table keep their code.
template <bool ON>
__device__ __forceinline__ void wave_lds_handoff() {
  if constexpr (ON) {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
  }
}

__device__ __forceinline__ void block_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

constexpr bool kmajor(int mode) { return mode == K_DIRECT || mode == K_GATHER || mode == K_ROWGATHER; }

// ---------------------------------------------------------------------------------- operands
// One operand tile: R rows (i or j) x BK k, R*128 bytes, R/32 DMA instructions per wave
// (instruction q = wave + 4s writes LDS bytes [1024q, 1024q + 1024) of the tile).
template <int MODE, int R, int NW>
struct Op {
  static constexpr int NI = R / (8 * NW);
  static_assert(kmajor(MODE) || R == 128, "MN-major tiles are 128 columns wide");
  // K-major: per-instruction row state (byte offset or base/hi/wi); MN-major: column state
  int s0[NI], s1[NI], s2[NI];
  int lchunk;            // this lane's logical 16-byte chunk (fixed for every DMA of the wave)
  uint32_t coff;         // MN: byte offset of the lane's column (+ group), or OOB
  int hoff, woff;        // MN gather: tap offsets of the lane's column

  // K-major: the global row r of DMA instruction s (LDS rows 8 (wave + NW s) + lane/8)
  __device__ __forceinline__ void set_row(const GOperand &op, int s, int r, uint32_t goff) {
    // (values first, stores last: stores to different members in the two branches of the
    // bounds test were merged by hipcc into one store through a selected address, which kept
    // the whole loader in private memory)
    if constexpr (kmajor(MODE)) {
      int v0 = -1, v1 = 0, v2 = 0;
      if constexpr (MODE == K_DIRECT) {
        if (r < op.rows) v0 = static_cast<int>(goff + static_cast<uint32_t>(r * op.ld) * 2u);
      } else if constexpr (MODE == K_ROWGATHER) {
        // byte offset of the pixel's first kernel-row run (pad 0: every run is in bounds)
        if (r < op.rows) {
          const uint32_t n = fdiv(static_cast<uint32_t>(r), op.fd_hw);
          const uint32_t rem = static_cast<uint32_t>(r) - n * static_cast<uint32_t>(op.Ho * op.Wo);
          const uint32_t ho = fdiv(rem, op.fd_wo);
          const uint32_t wo = rem - ho * op.Wo;
          v0 = static_cast<int>(goff) + ((static_cast<int>(n) * op.H + static_cast<int>(ho) * op.stride) * op.W +
                                         static_cast<int>(wo) * op.stride) * op.C * 2;
        }
      } else {
        if (r < op.rows) {
          const uint32_t n = fdiv(static_cast<uint32_t>(r), op.fd_hw);
          const uint32_t rem = static_cast<uint32_t>(r) - n * static_cast<uint32_t>(op.Ho * op.Wo);
          const uint32_t ho = fdiv(rem, op.fd_wo);
          const uint32_t wo = rem - ho * op.Wo;
          v0 = static_cast<int>(n) * op.H * op.W * op.C;
          v1 = static_cast<int>(ho) * op.stride - op.pad_h;
          v2 = static_cast<int>(wo) * op.stride - op.pad_w;
        }
      }
      s0[s] = v0;
      s1[s] = v1;
      s2[s] = v2;
    }
  }

  __device__ __forceinline__ void init(const GOperand &op, int row0, uint32_t goff, int wave, int lane) {
    if constexpr (kmajor(MODE)) {
      // rows 8q + lane/8; chunk ^ ((row >> 1) & 7) with (row >> 1) & 7 == 4(wave&1) + lane/16
      lchunk = (lane & 7) ^ (((wave & 1) << 2) + (lane >> 4));
#pragma unroll
      for (int s = 0; s < NI; ++s) set_row(op, s, row0 + 8 * (wave + NW * s) + (lane >> 3), goff);
    } else {
      // k-rows 4q + lane/16 (256-byte rows of 16 chunks); swizzle 2*((k&3) | ((k>>3)&1) << 2)
      lchunk = (lane & 15) ^ (2 * ((lane >> 4) | (((wave >> 1) & 1) << 2)));
      const int col = row0 + lchunk * 8;  // first of the lane's 8 columns (rows % 8 == 0)
      const bool ok = col < op.rows;
      if constexpr (MODE == MN_DIRECT) {
        coff = ok ? goff + static_cast<uint32_t>(col) * 2u : OOB;
        hoff = woff = 0;
      } else {
        int c = 0, kh = 0, kw = 0;
        if (ok) {
          const uint32_t r = fdiv(static_cast<uint32_t>(col), op.fd_cg);
          c = col - static_cast<int>(r) * op.Cg;
          const uint32_t q = fdiv(r, op.fd_kw);
          kh = static_cast<int>(q);
          kw = static_cast<int>(r - q * op.KW);
        }
        coff = ok ? goff + static_cast<uint32_t>(c) * 2u : OOB;
        hoff = kh - op.pad_h;
        woff = kw - op.pad_w;
      }
    }
  }

  // per K-tile, per lane: K-major -> the lane's k decode; MN-major -> the k-tile base
  struct Prep {
    int k;            // K-major: this lane's k; MN-major: first k of the tile
    int kh, kw;       // K gather
    uint32_t cb;      // K gather: channel byte offset (+ group)
    bool kin;
  };
  __device__ __forceinline__ Prep prep(const GOperand &op, int kt, int kt_end, uint32_t goff) const {
    Prep p;
    if constexpr (kmajor(MODE)) {
      p.k = kt * BK + lchunk * 8;
      p.kin = kt < kt_end && p.k < op.kdim;
      if constexpr (MODE == K_ROWGATHER) {
        // k = (kernel row kh, position j in the row's KW*C-element run padded to rlc chunks)
        const int kc = kt * (BK / 8) + lchunk;
        const int kh = static_cast<int>(fdiv(static_cast<uint32_t>(kc), op.fd_rlc));
        p.kin = p.kin && kh < op.KH;
        p.kh = p.kw = 0;
        p.cb = static_cast<uint32_t>(kh * op.W * op.C + (kc - kh * op.rlc) * 8) * 2u;
      } else if constexpr (MODE == K_GATHER) {
        const uint32_t r = fdiv(static_cast<uint32_t>(p.k), op.fd_cg);
        const int c = p.k - static_cast<int>(r) * op.Cg;
        const uint32_t q = fdiv(r, op.fd_kw);
        p.kh = p.kin ? static_cast<int>(q) : -(1 << 20);  // past the slice: every row OOB
        p.kw = static_cast<int>(r - q * op.KW);
        p.cb = goff + static_cast<uint32_t>(c) * 2u;
      } else {
        p.kh = p.kw = 0;
        p.cb = 0;
      }
    } else {
      p.k = kt * BK;
      p.kin = kt < kt_end;
      p.kh = p.kw = 0;
      p.cb = 0;
    }
    return p;
  }

  template <int S>
  __device__ __forceinline__ uint32_t offset(const GOperand &op, const Prep &p, int wave, int lane) const {
    uint32_t off;
    if constexpr (MODE == K_DIRECT) {
      off = (p.kin && s0[S] >= 0) ? static_cast<uint32_t>(s0[S]) + static_cast<uint32_t>(p.k) * 2u : OOB;
    } else if constexpr (MODE == K_ROWGATHER) {
      off = (p.kin && s0[S] >= 0) ? static_cast<uint32_t>(s0[S]) + p.cb : OOB;
    } else if constexpr (MODE == K_GATHER) {
      const int hi = s1[S] + p.kh, wi = s2[S] + p.kw;
      const bool ok = s0[S] >= 0 && static_cast<unsigned>(hi) < static_cast<unsigned>(op.H) &&
                      static_cast<unsigned>(wi) < static_cast<unsigned>(op.W);
      off = ok ? p.cb + static_cast<uint32_t>(s0[S] + (hi * op.W + wi) * op.C) * 2u : OOB;
    } else {
      const int kp = p.k + 4 * (wave + NW * S) + (lane >> 4);  // this DMA's k (pixel / batch row)
      const bool kin = p.kin && kp < op.kdim && coff != OOB;
      if constexpr (MODE == MN_DIRECT) {
        off = kin ? coff + static_cast<uint32_t>(kp * op.ld) * 2u : OOB;
      } else {
        const uint32_t n = fdiv(static_cast<uint32_t>(kp), op.fd_hw);
        const uint32_t rem = static_cast<uint32_t>(kp) - n * static_cast<uint32_t>(op.Ho * op.Wo);
        const uint32_t ho = fdiv(rem, op.fd_wo);
        const int wo = static_cast<int>(rem - ho * op.Wo);
        const int hi = static_cast<int>(ho) * op.stride + hoff, wi = wo * op.stride + woff;
        const bool ok = kin && static_cast<unsigned>(hi) < static_cast<unsigned>(op.H) &&
                        static_cast<unsigned>(wi) < static_cast<unsigned>(op.W);
        off = ok ? coff + static_cast<uint32_t>((static_cast<int>(n) * op.H + hi) * op.W + wi) * op.C * 2u : OOB;
      }
    }
    asm volatile("" : "+v"(off));  // keep the select: no per-lane branch around the DMA
    return off;
  }
};

// 16x16x32 fragment of rows [base, base+16) at k-step kk (0 or 32) from a staged tile.
template <int MODE>
__device__ __forceinline__ bf16x8 frag(const char *tile, int base, int kk, int lane) {
  if constexpr (kmajor(MODE)) {
    const int row = base + (lane & 15);
    const int ch = ((kk >> 3) + (lane >> 4)) ^ ((lane & 15) >> 1);
    return *reinterpret_cast<const bf16x8 *>(tile + row * 128 + ch * 16);
  } else {
    // ds_read_b64_tr_b16 pair: lane (i, gq) reads k-rows kk + 8gq + i/4 (+4), columns base + 4(i&3)
    const int i = lane & 15, gq = lane >> 4;
    const int f = (i >> 2) | ((gq & 1) << 2);              // swizzle/2 of both k-rows
    const int ch = ((base >> 4) ^ f) * 2 + ((i & 3) >> 1);  // (2*(base/16) + h) ^ 2f
    const char *p0 = tile + (kk + 8 * gq + (i >> 2)) * 256 + ch * 16 + (i & 1) * 8;
    s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4 *)(p0));
    s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4 *)(p0 + 4 * 256));
    typedef short s16x8 __attribute__((ext_vector_type(8)));
    s16x8 r = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8, r);
  }
}

// ======================================================================================
// Segmented 8-wave pipeline (tiles 50-51): the big-tile form for K-major operands
// (conv forward / data-grad, fc forward).
//
// The cdna guide's lesson for this regime: at ~1 block per CU the lever is keeping LDS-DMA
// loads in flight ACROSS barriers, with counted waits, and releasing LDS at a finer grain
// than a whole K-tile.  Here every K-tile (BK = 64) is split into two k-halves and the LDS
// holds four k-half slots (2 K-tiles x 2 halves) of [BM + BN][32] bf16 = 64-byte rows:
//   * one SEGMENT = one k-half of one K-tile: wait for its slot -> barrier -> issue the DMAs
//     of the k-half three segments ahead into the slot the previous segment just released
//     -> read fragments -> MR x NR MFMAs (one 16x16x32 k-step) between s_setprio(1)/(0);
//   * a wave waits with a constant `s_waitcnt vmcnt(2 * NPH)`: two later k-halves stay in
//     flight across every barrier, so a DMA has three segments (~3 x 1000 MFMA cycles per
//     SIMD at 256x256) to land; past the end of the K slice the DMAs are all-OOB dummies so
//     the count never changes;
//   * 8 waves (2 x 4), 2 per SIMD: per wave a (BM/2) x 64 output tile, so a 256 x 256 block
//     reads 24 KiB of fragments per 64 MFMAs per wave (vs 4 KiB per 16 for 64 x 128 tiles);
//   * 64-byte rows, 16 rows per 1-KiB DMA; chunk swizzle `c ^ 2*((row >> 3) & 1)` on the
//     source address keeps both the DMA image lane-linear and every ds_read_b128 lane group
//     of the fragment reads on 16 distinct 16-byte bank slots.
template <int MODE, int R>
struct SegOp {  // one operand's DMAs for a k-half slot: R rows x 32 k, 8 waves
  static constexpr int NI = R / 128;  // 1-KiB DMA instructions per wave per slot
  static_assert(kmajor(MODE) && R % 128 == 0, "segmented kernel: K-major operands, 128-row multiples");
  int s0[NI], s1[NI], s2[NI];
  int lchunk;

  __device__ __forceinline__ void init(const GOperand &op, int row0, uint32_t goff, int wave, int lane) {
    lchunk = (lane & 3) ^ (2 * (lane >> 5));  // rows 16q + lane/4: (row >> 3) & 1 == lane >> 5
#pragma unroll
    for (int s = 0; s < NI; ++s) {
      const int r = row0 + 16 * (wave + 8 * s) + (lane >> 2);
      if constexpr (MODE == K_DIRECT) {
        s0[s] = r < op.rows ? static_cast<int>(goff + static_cast<uint32_t>(r * op.ld) * 2u) : -1;
        s1[s] = s2[s] = 0;
      } else {
        if (r < op.rows) {
          const uint32_t n = fdiv(static_cast<uint32_t>(r), op.fd_hw);
          const uint32_t rem = static_cast<uint32_t>(r) - n * static_cast<uint32_t>(op.Ho * op.Wo);
          const uint32_t ho = fdiv(rem, op.fd_wo);
          const uint32_t wo = rem - ho * op.Wo;
          s0[s] = static_cast<int>(n) * op.H * op.W * op.C;
          s1[s] = static_cast<int>(ho) * op.stride - op.pad_h;
          s2[s] = static_cast<int>(wo) * op.stride - op.pad_w;
        } else {
          s0[s] = -1;
          s1[s] = s2[s] = 0;
        }
      }
    }
  }

  struct Prep {
    int k, kh, kw;
    uint32_t cb;
    bool kin;
  };
  // the lane's 8 k of segment seg (K-tile kt_beg + seg/2, half seg%2)
  __device__ __forceinline__ Prep prep(const GOperand &op, int kt, int half, int kt_end, uint32_t goff) const {
    Prep p;
    p.k = kt * BK + half * 32 + lchunk * 8;
    p.kin = kt < kt_end && p.k < op.kdim;
    if constexpr (MODE == K_GATHER) {
      const uint32_t r = fdiv(static_cast<uint32_t>(p.k), op.fd_cg);
      const int c = p.k - static_cast<int>(r) * op.Cg;
      const uint32_t q = fdiv(r, op.fd_kw);
      p.kh = p.kin ? static_cast<int>(q) : -(1 << 20);
      p.kw = static_cast<int>(r - q * op.KW);
      p.cb = goff + static_cast<uint32_t>(c) * 2u;
    } else {
      p.kh = p.kw = 0;
      p.cb = 0;
    }
    return p;
  }

  template <int S>
  __device__ __forceinline__ uint32_t offset(const GOperand &op, const Prep &p) const {
    uint32_t off;
    if constexpr (MODE == K_DIRECT) {
      off = (p.kin && s0[S] >= 0) ? static_cast<uint32_t>(s0[S]) + static_cast<uint32_t>(p.k) * 2u : OOB;
    } else {
      const int hi = s1[S] + p.kh, wi = s2[S] + p.kw;
      const bool ok = s0[S] >= 0 && static_cast<unsigned>(hi) < static_cast<unsigned>(op.H) &&
                      static_cast<unsigned>(wi) < static_cast<unsigned>(op.W);
      off = ok ? p.cb + static_cast<uint32_t>(s0[S] + (hi * op.W + wi) * op.C) * 2u : OOB;
    }
    asm volatile("" : "+v"(off));
    return off;
  }
};

// 16x16x32 fragment of rows [base, base + 16) of a 64-byte-row slot image
__device__ __forceinline__ bf16x8 seg_frag(const char *tile, int base, int lane) {
  const int row = base + (lane & 15);
  const int ch = (lane >> 4) ^ (2 * ((lane >> 3) & 1));
  return *reinterpret_cast<const bf16x8 *>(tile + row * 64 + ch * 16);
}

// Epilogue of the 8-wave kernels: each wave stages 16 output rows (j) x WM columns (i) of its
// fp32 tile in LDS, then writes contiguous row segments: bf16 (+bias, relu, relu'-mask of the old
// value) or an fp32 split-K slab.
// Write JR staged output rows (j = jrow0 .. jrow0 + JR - 1, WM columns i from ibase; staging row
// pitch WM + 4 floats) of one wave: bf16 (+bias, relu, relu'-mask of the old value) or an fp32
// split-K slab.
// The bias of a lane's 8 output columns (i = ibase + (lane % (WM / 8)) * 8 + e): loaded once per
// epilogue, before its first store -- a load issued after a store waits for it (vmcnt counts
// loads and stores in issue order), so per-row bias loads serialised the epilogue on store latency.
template <int WM>
__device__ __forceinline__ void staged_bias(const GEpi &E, int g, int Mi, int ibase, int lane, float (&bv)[8]) {
  const float *bias = E.bias ? E.bias + g * E.bias_gstride : nullptr;
  const int i = ibase + (lane % (WM / 8)) * 8;
#pragma unroll
  for (int e = 0; e < 8; ++e) bv[e] = (bias && i + e < Mi) ? bias[i + e] : 0.f;
}

template <int EPI, int JR, int WM>
__device__ __forceinline__ void write_staged(const float *ep, const GEpi &E, int g, int slice, int Mi, int Nj,
                                             int ibase, int jrow0, int lane, const float *bv8 = nullptr,
                                             float *bsum = nullptr) {
  // bsum (EPI_BF16, optional): += the stored bf16 values of the lane's 8 columns (a conv
  // data-gradient handing over the lower conv's bias gradient, as EPI_BF16_DB)
  const float *bias = E.bias ? E.bias + g * E.bias_gstride : nullptr;
  if constexpr (EPI == EPI_BF16) {
    bf16_t *out = reinterpret_cast<bf16_t *>(E.out) + g * E.gstride;
    constexpr int LPR = WM / 8;
    constexpr int RPI = 64 / LPR;
    const int il = (lane % LPR) * 8;
    const int i = ibase + il;
    float bv[8];  // bv8: preloaded by the caller (staged_bias)
#pragma unroll
    for (int e = 0; e < 8; ++e) bv[e] = bv8 ? bv8[e] : ((bias && i + e < Mi) ? bias[i + e] : 0.f);
    const bool vec_store = ((E.ldc & 7) == 0) && (i + 8 <= Mi);
    // relu'-mask: every old value of the lane's rows is loaded before the first store.  A load
    // issued after a store waits for it (vmcnt counts loads and stores in issue order), so
    // load / store pairs would serialise the epilogue on store latency.
    constexpr int NIT = (JR + RPI - 1) / RPI;
    uint4 oldv[NIT];
    if (E.mask_relu && vec_store) {
#pragma unroll
      for (int k = 0; k < NIT; ++k) {
        const int jl = lane / LPR + k * RPI;
        if (jl < JR && jrow0 + jl < Nj && i < Mi)
          oldv[k] = *reinterpret_cast<const uint4 *>(out + static_cast<long>(jrow0 + jl) * E.ldc + i);
      }
    }
#pragma unroll
    for (int k = 0; k < NIT; ++k) {
      const int jl = lane / LPR + k * RPI;
      const int j = jrow0 + jl;
      if (jl < JR && j < Nj && i < Mi) {
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
            unpack8(oldv[k], old);
#pragma unroll
            for (int e = 0; e < 8; ++e) f[e] = old[e] > 0.f ? f[e] : 0.f;
          }
          const uint4 packed = pack8(f);
          *reinterpret_cast<uint4 *>(dst) = packed;
          if (bsum) {
            float r[8];
            unpack8(packed, r);
#pragma unroll
            for (int e = 0; e < 8; ++e) bsum[e] += r[e];
          }
        } else {
          for (int e = 0; e < 8 && i + e < Mi; ++e) {
            if (E.mask_relu && !(bf2f(dst[e]) > 0.f)) f[e] = 0.f;
            dst[e] = f2bf(f[e]);
            if (bsum) bsum[e] += bf2f(f2bf(f[e]));
          }
        }
      }
    }
  } else {  // EPI_F32: split-K slab (fc forward)
    float *out = reinterpret_cast<float *>(E.out) + g * E.gstride + slice * E.kstride;
    constexpr int LPR = WM / 4;
    constexpr int RPI = 64 / LPR;
    const int il = (lane % LPR) * 4;
    const int i = ibase + il;
    const bool vec = ((E.ldc & 3) == 0) && (i + 4 <= Mi);
#pragma unroll
    for (int jl = lane / LPR; jl < JR; jl += RPI) {
      const int j = jrow0 + jl;
      if (j < Nj && i < Mi) {
        f32x4 v = *reinterpret_cast<const f32x4 *>(ep + jl * (WM + 4) + il) * E.alpha;
        float *dst = out + static_cast<long>(j) * E.ldc + i;
        if (vec) {
          *reinterpret_cast<f32x4 *>(dst) = v;
        } else {
          for (int e = 0; e < 4 && i + e < Mi; ++e) dst[e] = v[e];
        }
      }
    }
  }
}

template <int EPI, int MR, int NR, int WM>
__device__ __forceinline__ void seg_epilogue(f32x4 (&acc)[MR][NR], char *smem, const GEpi &E, int g, int slice, int Mi,
                                             int Nj, int ibase, int jbase, int wave, int lane) {
  float *ep = reinterpret_cast<float *>(smem) + wave * 16 * (WM + 4);
  float bv[8];  // the lane's 8 bias columns, loaded before the first store (staged_bias)
  if constexpr (EPI == EPI_BF16) staged_bias<WM>(E, g, Mi, ibase, lane, bv);
#pragma unroll
  for (int n = 0; n < NR; ++n) {
#pragma unroll
    for (int m = 0; m < MR; ++m)
      *reinterpret_cast<f32x4 *>(ep + (lane & 15) * (WM + 4) + m * 16 + (lane >> 4) * 4) = acc[m][n];
    __builtin_amdgcn_s_waitcnt(0xc07f);
    if constexpr (EPI == EPI_BF16) {
      bf16_t *out = reinterpret_cast<bf16_t *>(E.out) + g * E.gstride;
      constexpr int LPR = WM / 8;
      constexpr int RPI = 64 / LPR;
      const int il = (lane % LPR) * 8;
      const int i = ibase + il;
      const bool vec_store = ((E.ldc & 7) == 0) && (i + 8 <= Mi);
      // relu'-mask old values all loaded before the fragment's first store (as write_staged)
      constexpr int NIT = (16 + RPI - 1) / RPI;
      uint4 oldv[NIT];
      if (E.mask_relu && vec_store) {
#pragma unroll
        for (int k = 0; k < NIT; ++k) {
          const int jl = lane / LPR + k * RPI;
          if (jl < 16 && jbase + n * 16 + jl < Nj && i < Mi)
            oldv[k] = *reinterpret_cast<const uint4 *>(out + static_cast<long>(jbase + n * 16 + jl) * E.ldc + i);
        }
      }
#pragma unroll
      for (int k = 0; k < NIT; ++k) {
        const int jl = lane / LPR + k * RPI;
        const int j = jbase + n * 16 + jl;
        if (jl < 16 && j < Nj && i < Mi) {
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
              unpack8(oldv[k], old);
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
    } else {  // EPI_F32: split-K slab (fc forward)
      float *out = reinterpret_cast<float *>(E.out) + g * E.gstride + slice * E.kstride;
      constexpr int LPR = WM / 4;
      constexpr int RPI = 64 / LPR;
      const int il = (lane % LPR) * 4;
      const int i = ibase + il;
      const bool vec = ((E.ldc & 3) == 0) && (i + 4 <= Mi);
#pragma unroll
      for (int jl = lane / LPR; jl < 16; jl += RPI) {
        const int j = jbase + n * 16 + jl;
        if (j < Nj && i < Mi) {
          f32x4 v = *reinterpret_cast<const f32x4 *>(ep + jl * (WM + 4) + il) * E.alpha;
          float *dst = out + static_cast<long>(j) * E.ldc + i;
          if (vec) {
            *reinterpret_cast<f32x4 *>(dst) = v;
          } else {
            for (int e = 0; e < 4 && i + e < Mi; ++e) dst[e] = v[e];
          }
        }
      }
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);
  }
}

// the one-wave-per-SIMD address-free tile (gemm_4w.hip): tile 114; -1 when unsupported
int dispatch_4w(int amode, int bmode, int epi, int tile, const GOperand &A, const GOperand &B, const GEpi &E,
                int groups, int ksplit, hipStream_t s);
// direct 3x3 convolution on a resident input halo (conv_halo.hip): tiles 130, 131, 133; -1 when unsupported
int dispatch_halo(int amode, int bmode, int epi, int tile, GOperand A, GOperand B, const GEpi &E, int groups,
                  int ksplit, hipStream_t s);
// direct 3x3 weight-gradient on resident halo / dy tiles (conv_wgrad_halo.hip): tiles 140-142
int dispatch_wgrad_halo(int amode, int bmode, int epi, int tile, const GOperand &A, const GOperand &B, const GEpi &E,
                        int groups, hipStream_t s);

}  // namespace cxg
