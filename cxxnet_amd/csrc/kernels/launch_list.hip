// Native launch-list executor (cxn_rec_*): record the library launches of a step segment once,
// then replay them from C++.
//
// The reference's executor is a C++ loop over layers issuing mshadow kernels
// (src/nnet/neural_net-inl.hpp:107-153); ours decides WHAT to launch in Python (tile tables,
// fusions, zero-copy views), which costs ~10 us of interpreter time per launch.  Every launch
// of this library goes through CXN_LAUNCH (common.h): while a list is open on the calling thread
// the launch also stores a closure over its grid, block, LDS size and argument values.  A
// replay re-issues the closures in order on the given stream -- a few microseconds per kernel,
// with no graph capture, so segments can sit between eager collectives, event waits and host
// work exactly as the eager step does (NetTrainer._record_plans).
//
// Contract for the caller: a recorded segment contains only library launches (no torch kernels),
// and every buffer it touches stays allocated at the same address across replays (node buffers,
// the parameter arena, persistent workspaces; temporaries of the recording run are kept alive
// by the caller's memory pool).  Kernel arguments are frozen: per-step values (dropout seeds,
// the step counter) are read from device memory, as for HIP-graph replay.
#include "common.h"

namespace cxr {
LaunchList *&rec_slot() {
  static thread_local LaunchList *slot = nullptr;
  return slot;
}
}  // namespace cxr

// Open a list on this thread (-1 if one is already open).
CXN_API int cxn_rec_begin() {
  if (cxr::rec_slot() != nullptr) return -1;
  cxr::rec_slot() = new cxr::LaunchList();
  return 0;
}

// Close this thread's list and hand it over (nullptr if none was open).
CXN_API void *cxn_rec_end() {
  cxr::LaunchList *l = cxr::rec_slot();
  cxr::rec_slot() = nullptr;
  return l;
}

CXN_API int cxn_rec_size(void *list) { return list ? static_cast<int>(static_cast<cxr::LaunchList *>(list)->ops.size()) : 0; }

// Re-issue every recorded launch on `stream`; 0, or -3 on a launch error.
CXN_API int cxn_rec_replay(void *list, void *stream) {
  if (!list) return 0;
  hipStream_t s = static_cast<hipStream_t>(stream);
  for (auto &op : static_cast<cxr::LaunchList *>(list)->ops) op(s);
  return hipGetLastError() == hipSuccess ? 0 : -3;
}

// Replay several lists back to back (one call for a run of segments).
CXN_API int cxn_rec_replay_many(void *const *lists, int n, void *stream) {
  hipStream_t s = static_cast<hipStream_t>(stream);
  for (int i = 0; i < n; ++i)
    if (lists[i])
      for (auto &op : static_cast<cxr::LaunchList *>(lists[i])->ops) op(s);
  return hipGetLastError() == hipSuccess ? 0 : -3;
}

CXN_API void cxn_rec_free(void *list) { delete static_cast<cxr::LaunchList *>(list); }

// Device-to-device copy of `bytes` bytes on `stream` (recorded when a list is open).
CXN_API int cxn_copy_d2d(void *dst, const void *src, long bytes, void *stream) {
  if (bytes <= 0) return 0;
  return CXN_MEMCPY_D2D(dst, src, static_cast<size_t>(bytes), static_cast<hipStream_t>(stream)) == hipSuccess ? 0 : -3;
}

namespace {
// 16 bytes per thread where the range is 16-byte aligned, the unaligned head / tail byte-wise
__global__ void fill_bytes_k(unsigned char *p, unsigned v, size_t n) {
  const size_t tid = static_cast<size_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  const size_t stride = static_cast<size_t>(gridDim.x) * blockDim.x;
  const uintptr_t a = reinterpret_cast<uintptr_t>(p);
  const size_t head = ((16 - (a & 15)) & 15) < n ? ((16 - (a & 15)) & 15) : n;
  const size_t nv = (n - head) / 16;
  const unsigned w = v * 0x01010101u;
  uint4 *pv = reinterpret_cast<uint4 *>(p + head);
  for (size_t i = tid; i < nv; i += stride) pv[i] = make_uint4(w, w, w, w);
  const size_t tail0 = head + nv * 16;
  for (size_t i = tid; i < head + (n - tail0); i += stride) {
    const size_t b = i < head ? i : tail0 + (i - head);
    p[b] = static_cast<unsigned char>(v);
  }
}
}  // namespace

hipError_t cxn_fill_bytes(void *p, int v, size_t n, hipStream_t s) {
  if (n == 0) return hipSuccess;
  const size_t nv = n / 16 + 1;
  const unsigned blocks = static_cast<unsigned>(nv / 256 + 1 < 2048 ? nv / 256 + 1 : 2048);
  CXN_LAUNCH(fill_bytes_k, dim3(blocks), dim3(256), 0, s, static_cast<unsigned char *>(p), static_cast<unsigned>(v) & 0xffu, n);
  return hipGetLastError();
}

namespace {
struct ZeroRanges {  // up to 16 disjoint float ranges of one buffer, zeroed by one launch
  long off[16], len[16];
  int n;
};
// blockIdx.y = range; 16 bytes per thread on the 16-byte-aligned body, floats at the edges
__global__ void zero_ranges_k(float *base, ZeroRanges r) {
  const int k = blockIdx.y;
  if (k >= r.n) return;
  float *p = base + r.off[k];
  const long n = r.len[k];
  const long head = min(static_cast<long>((4 - ((reinterpret_cast<uintptr_t>(p) >> 2) & 3)) & 3), n);
  const long nv = (n - head) / 4;
  const long tid = static_cast<long>(blockIdx.x) * blockDim.x + threadIdx.x;
  const long stride = static_cast<long>(gridDim.x) * blockDim.x;
  float4 *pv = reinterpret_cast<float4 *>(p + head);
  for (long i = tid; i < nv; i += stride) pv[i] = make_float4(0.f, 0.f, 0.f, 0.f);
  const long tail0 = head + nv * 4;
  for (long i = tid; i < head + (n - tail0); i += stride) p[i < head ? i : tail0 + (i - head)] = 0.f;
}
}  // namespace

// Zero n float ranges [off[i], off[i] + len[i]) of base in ONE launch (recorded like a launch): the
// accumulated-gradient ranges of the parameter arena at the start of a backward pass.
CXN_API int cxn_zero_ranges(float *base, const long *off, const long *len, int n, void *stream) {
  if (n <= 0) return 0;
  if (n > 16) return -1;
  ZeroRanges r{};
  long mx = 0;
  for (int i = 0; i < n; ++i) {
    if (off[i] < 0 || len[i] < 0) return -2;
    r.off[i] = off[i];
    r.len[i] = len[i];
    mx = len[i] > mx ? len[i] : mx;
  }
  r.n = n;
  const long blocks = (mx / 4 + 255) / 256 + 1;
  CXN_LAUNCH(zero_ranges_k, dim3(static_cast<unsigned>(blocks < 1024 ? blocks : 1024), n), dim3(256), 0,
             static_cast<hipStream_t>(stream), base, r);
  return hipGetLastError() == hipSuccess ? 0 : -3;
}

// Zero `bytes` bytes at dst on `stream` (recorded when a list is open): gradient zeroing at the
// start of a backward pass must be part of the replayed step.
CXN_API int cxn_zero(void *dst, long bytes, void *stream) {
  if (bytes <= 0) return 0;
  return CXN_MEMSET(dst, 0, static_cast<size_t>(bytes), static_cast<hipStream_t>(stream)) == hipSuccess ? 0 : -3;
}
