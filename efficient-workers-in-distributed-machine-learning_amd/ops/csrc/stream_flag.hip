// Device-side hand-offs between two streams of a segmented training step (parallel/engine.py
// SegmentedCapture): a one-thread signal kernel at the end of a compute segment bumps a counter,
// a one-thread wait kernel at the head of the comm-stream graph polls it (and the reverse for the
// apply after the last comm graph).  Every graph replays linear, and the host launches them back
// to back with no event record / stream wait between (a cross-queue event barrier measured
// ~20 us of GPU time per hop at world 1: profiles/ab/segmented_r06.md).
//
// Memory ordering: the producers are whole kernels that completed before the signal kernel
// started (stream order; a kernel's end releases its writes at agent scope), the consumers whole
// kernels that start after the wait kernel ended (their dispatch acquires), so the counter only
// orders kernel boundaries -- relaxed agent-scope atomics, no fences.
//
// Counts, not values: each wait kernel owns a private "seen" word that it alone advances (by
// `need`, the signals per step it waits for), so a graph replayed every step needs no host
// update.  The spin is bounded (a mismatched count reports through `err` instead of hanging).
#include "common.h"
#include "ewdml_ops.h"

namespace {

constexpr uint32_t FLAG_MAX_POLLS = 1u << 24;  // ~3 s of polls

__global__ void k_flag_signal(int* __restrict__ flag) {
  if (threadIdx.x == 0) __hip_atomic_fetch_add(flag, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ void k_flag_wait(const int* __restrict__ flag, int* __restrict__ seen, int need,
                            int* __restrict__ err) {
  if (threadIdx.x != 0) return;
  const int want = *seen + need;
  uint32_t polls = 0;
  while (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - want < 0) {
    if (++polls > FLAG_MAX_POLLS) {
      __hip_atomic_fetch_add(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      break;
    }
    __builtin_amdgcn_s_sleep(8);
  }
  *seen = want;
}

}  // namespace

void ew_flag_signal(uintptr_t flag, uintptr_t stream) {
  hipLaunchKernelGGL(k_flag_signal, dim3(1), dim3(64), 0, (hipStream_t)stream,
                     reinterpret_cast<int*>(flag));
  EW_CHECK_LAUNCH();
}

void ew_flag_wait(uintptr_t flag, uintptr_t seen, int need, uintptr_t err, uintptr_t stream) {
  hipLaunchKernelGGL(k_flag_wait, dim3(1), dim3(64), 0, (hipStream_t)stream,
                     reinterpret_cast<const int*>(flag), reinterpret_cast<int*>(seen), need,
                     reinterpret_cast<int*>(err));
  EW_CHECK_LAUNCH();
}
