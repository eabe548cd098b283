// Shared device helpers of the direct (slot-space / row-run) convolution kernels for gfx950:
// conv_wgrad_direct.hip, conv_rowrun_direct.hip.
#pragma once
#include "gemm_glds_common.h"

namespace cxd {
using namespace cxg;

// One 1-KiB LDS-DMA (16 bytes per lane) as inline asm: hipcc cannot tell the LDS bytes it writes
// from the ones the ds_reads of the current stage touch, and for the builtin it inserts a
// vmcnt(0) before the first ds_read after the DMAs -- the next stage's loads would then be waited
// for at the start of the current stage instead of landing under its MFMAs.  Completion is
// counted by hand (wait_vmcnt + barrier at the end of the stage).  M0 is saved and restored in
// the statement (compiler-reserved).
__device__ __forceinline__ void dma16d(rsrc_t r, uint32_t lds_addr, uint32_t voff) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(voff), "s"(r), "s"(lds_addr) : "memory");
}

template <int N>
__device__ __forceinline__ void wait_lgkm_d() {
  asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(N) : "memory");
}

// accumulators beyond the 256-register AGPR file live in VGPRs (gfx950 MFMAs take either)
template <bool AGPR>
__device__ __forceinline__ void mfma_d(f32x4 &acc, const bf16x8 &a, const bf16x8 &b) {
  if constexpr (AGPR) asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
  else asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+v"(acc) : "v"(a), "v"(b));
}
// bias-gradient MFMA: its B operand (the ones fragment) lives in VGPRs that hipcc may have just
// (re)written with a VALU move; "s_nop 1" covers the VALU-write -> MFMA-operand wait states hipcc
// does not insert for inline asm
__device__ __forceinline__ void mfma_db(f32x4 &acc, const bf16x8 &a, const bf16x8 &b) {
  asm volatile("s_nop 1\n\tv_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+v"(acc) : "v"(a), "v"(b));
}
template <bool AGPR>
__device__ __forceinline__ void pin_d(f32x4 &acc) {
  if constexpr (AGPR) asm volatile("" : "+a"(acc));
  else asm volatile("" : "+v"(acc));
}

// two transposed 8-byte reads (k-rows 8 g4 + q and 8 g4 + 4 + q) -> one 16x16x32 operand fragment
__device__ __forceinline__ bf16x8 frag_d(const char *p0, const char *p1) {
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4 *)(p0));
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4 *)(p1));
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  const s16x8 r = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, r);
}

constexpr int fdiv_floor(int a, int b) { return a >= 0 ? a / b : -((-a + b - 1) / b); }

}  // namespace cxd
