// Shared device helpers for the gfx950 (CDNA4) kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <functional>
#include <vector>

#define CXN_API extern "C" __attribute__((visibility("default")))

typedef unsigned short bf16_t;  // storage type for bf16 tensors
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

__device__ __forceinline__ float bf2f(bf16_t v) { return __uint_as_float(static_cast<uint32_t>(v) << 16); }
__device__ __forceinline__ bf16_t f2bf(float f) {
  __bf16 b = static_cast<__bf16>(f);  // lowers to v_cvt_pk_bf16_f32 (RNE, NaN-preserving)
  return __builtin_bit_cast(bf16_t, b);
}

// 8 x bf16 packed in a uint4 (16 B) -- the unit of every vectorised access.
__device__ __forceinline__ void unpack8(const uint4 &v, float *f) {
  f[0] = __uint_as_float(v.x << 16); f[1] = __uint_as_float(v.x & 0xffff0000u);
  f[2] = __uint_as_float(v.y << 16); f[3] = __uint_as_float(v.y & 0xffff0000u);
  f[4] = __uint_as_float(v.z << 16); f[5] = __uint_as_float(v.z & 0xffff0000u);
  f[6] = __uint_as_float(v.w << 16); f[7] = __uint_as_float(v.w & 0xffff0000u);
}
// Two floats -> one v_cvt_pk_bf16_f32 (the scalar form, f2bf | f2bf << 16, cost two converts
// plus three re-packing ops per pair: the compiler pairs the converts across the wrong operands)
typedef float cxn_f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 cxn_bf16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t pack2(float a, float b) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((cxn_f32x2){a, b}, cxn_bf16x2));
}
__device__ __forceinline__ uint4 pack8(const float *f) {
  return make_uint4(pack2(f[0], f[1]), pack2(f[2], f[3]), pack2(f[4], f[5]), pack2(f[6], f[7]));
}

// Division by a runtime-invariant divisor with a multiply-high (n < 2^31).
struct FastDiv {
  uint32_t d, mul, shift;
};
static inline FastDiv make_fastdiv(uint32_t d) {
  FastDiv f;
  f.d = d;
  uint32_t l = 0;
  while ((1ull << l) < d) ++l;
  f.shift = l;
  f.mul = static_cast<uint32_t>(((1ull << 32) * ((1ull << l) - d)) / d + 1);
  return f;
}
__device__ __forceinline__ uint32_t fdiv(uint32_t n, const FastDiv &f) {
  return (__umulhi(n, f.mul) + n) >> f.shift;
}

// XCD-aware bijective remap of a 1-D block id: consecutive logical tiles land on
// the same XCD (blocks b and b+8 share an XCD under round-robin dispatch), so
// neighbouring tiles share that XCD's L2.  Speed-only; any placement is correct.
__device__ __forceinline__ uint32_t xcd_remap(uint32_t orig, uint32_t nwg) {
  if (nwg < 16) return orig;
  const uint32_t q = nwg / 8, r = nwg % 8, xcd = orig % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
}

// Work item (tile, K slice, group) of a GEMM block on a grid (ntile, ksplit, groups), the whole
// grid remapped as one range so that each XCD runs a contiguous run of work items.  Hardware
// dispatch is x-fastest, so with a split K the ntile blocks of one K slice would otherwise land on
// ntile different XCDs and each fetch the slice's shared operand into its own L2 (VGG conv1_2
// weight-grad: 5 M-tiles per slice, 4.3 GB of HBM reads for 0.8 GB of operands).
struct GemmBlock {
  uint32_t tile;
  int slice, g;
};
__device__ __forceinline__ GemmBlock gemm_block(uint32_t ntile) {
  if (gridDim.y == 1 && gridDim.z == 1) return {xcd_remap(blockIdx.x, ntile), 0, 0};
  const uint32_t ny = gridDim.y, nz = gridDim.z;
  const uint32_t r = xcd_remap(blockIdx.x + ntile * (blockIdx.y + ny * blockIdx.z), ntile * ny * nz);
  const uint32_t rt = r / ntile;
  return {r - rt * ntile, static_cast<int>(rt % ny), static_cast<int>(rt / ny)};
}

// Tile (ti, tj) of a work item.  group_i <= 0 or tiles_i <= group_i: i fastest over all i-tiles
// (neighbouring items share the B panel).  Otherwise i fastest inside groups of group_i i-tiles:
// the ~32 items an XCD runs together then cover a group_i x (32 / group_i) patch of the output,
// re-reading group_i A panels and 32 / group_i B panels from the XCD's L2 instead of 32 A panels
// and one B panel (square / fc GEMMs, where tiles_i is large).  Speed-only.
__device__ __forceinline__ void tile_ij(uint32_t tile, int tiles_i, int tiles_j, int group_i, int &ti, int &tj) {
  if (group_i <= 0 || tiles_i <= group_i) {
    ti = static_cast<int>(tile % static_cast<uint32_t>(tiles_i));
    tj = static_cast<int>(tile / static_cast<uint32_t>(tiles_i));
    return;
  }
  const uint32_t per = static_cast<uint32_t>(group_i) * static_cast<uint32_t>(tiles_j);
  const uint32_t grp = tile / per;
  const int first = static_cast<int>(grp) * group_i;
  const int gm = min(tiles_i - first, group_i);
  const uint32_t r = tile - grp * per;
  ti = first + static_cast<int>(r % static_cast<uint32_t>(gm));
  tj = static_cast<int>(r / static_cast<uint32_t>(gm));
}

static inline int cdiv(long a, long b) { return static_cast<int>((a + b - 1) / b); }

// Deterministic mode (cxn_set_deterministic): reductions that would combine partial sums with
// atomics in a run-dependent order (cross-block channel sums, bias-grad partials) use one
// ordered pass instead, so two identical runs produce bitwise-identical results.
extern int cxn_deterministic;

// ----------------------------------------------------------------------------------------------
// Launch-list recorder (launch_list.hip, cxn_rec_*): the native replay executor.  While a list is
// open on the calling thread, every library launch also stores a closure over its launch shape
// and argument VALUES; cxn_rec_replay re-issues the list on a stream from C++ in one call -- no
// Python per kernel, no graph capture.  Every launch site goes through CXN_LAUNCH.
namespace cxr {
struct LaunchList {
  std::vector<std::function<void(hipStream_t)>> ops;
};
LaunchList *&rec_slot();  // this thread's open list (nullptr: not recording)
}  // namespace cxr

#define CXN_LAUNCH(KER, GRID, BLOCK, SHMEM, STREAM, ...)                                          \
  do {                                                                                           \
    const dim3 cxn_grid_ = dim3(GRID), cxn_block_ = dim3(BLOCK);                                             \
    const size_t cxn_shm_ = static_cast<size_t>(SHMEM);                                          \
    hipLaunchKernelGGL(KER, cxn_grid_, cxn_block_, cxn_shm_, (STREAM), __VA_ARGS__);              \
    if (::cxr::LaunchList *cxn_rec_ = ::cxr::rec_slot())                                         \
      cxn_rec_->ops.emplace_back([=](hipStream_t cxn_s_) {                                       \
        hipLaunchKernelGGL(KER, cxn_grid_, cxn_block_, cxn_shm_, cxn_s_, __VA_ARGS__);            \
      });                                                                                        \
  } while (0)

// Stream-ordered byte fill as a library KERNEL (launch_list.hip cxn_fill_bytes), recorded like a
// launch.  Not hipMemsetAsync: inside a captured HIP graph its memset node zeroed the range on
// the first replay only (later replays left 0x00000106 words; tools/diag_memset_graph.py), which
// let every captured step accumulate gradients on top of the previous one.
hipError_t cxn_fill_bytes(void *p, int v, size_t n, hipStream_t s);
#define CXN_MEMSET(PTR, VAL, BYTES, STREAM) ::cxn_fill_bytes((PTR), (VAL), (BYTES), (STREAM))

// stream-ordered device-to-device copy, recorded like a launch
#define CXN_MEMCPY_D2D(DST, SRC, BYTES, STREAM)                                                  \
  ([&]() -> hipError_t {                                                                         \
    void *cxn_d_ = (DST);                                                                        \
    const void *cxn_s0_ = (SRC);                                                                 \
    const size_t cxn_n_ = (BYTES);                                                               \
    const hipError_t cxn_e_ = hipMemcpyAsync(cxn_d_, cxn_s0_, cxn_n_, hipMemcpyDeviceToDevice, (STREAM)); \
    if (::cxr::LaunchList *cxn_rec_ = ::cxr::rec_slot())                                         \
      cxn_rec_->ops.emplace_back([=](hipStream_t cxn_s_) {                                       \
        (void)hipMemcpyAsync(cxn_d_, cxn_s0_, cxn_n_, hipMemcpyDeviceToDevice, cxn_s_);           \
      });                                                                                        \
    return cxn_e_;                                                                               \
  }())
