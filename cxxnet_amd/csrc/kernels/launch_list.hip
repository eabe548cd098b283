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

// Zero `bytes` bytes at dst on `stream` (recorded when a list is open): gradient zeroing at the
// start of a backward pass must be part of the replayed step.
CXN_API int cxn_zero(void *dst, long bytes, void *stream) {
  if (bytes <= 0) return 0;
  return CXN_MEMSET(dst, 0, static_cast<size_t>(bytes), static_cast<hipStream_t>(stream)) == hipSuccess ? 0 : -3;
}
