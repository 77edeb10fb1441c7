// dg_home.h — the publish step of dg_join_delta_home (device side).
//
// The small join writes its result block straight into `home` (page-locked host memory);
// whichever kernel ends the call (the small join itself, or the tail kernel's last
// workgroup when it copies moved rows) then copies the engine's count block into the
// mapped publish words and, after a system fence, stores the sequence number the host
// polls (api.hip wait_published).  Called by every thread of the workgroup.
#pragma once
#include "dg_launch.h"

namespace dg {

// w: this thread's word of the engine's count block (threads < 16; loaded early by a
// kernel that does not change the block, so the publish waits for no load)
__device__ __forceinline__ void publish_word(u64 w, u64* h_pub, u64 seq) {
  __syncthreads();  // the block's writes are issued
  if (threadIdx.x < 16) h_pub[threadIdx.x] = w;  // d_counts[0..8), ticket words
  __threadfence_system();  // each thread's host writes land before ...
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_store(h_pub + 16, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ __forceinline__ void publish_counts(const u64* d_counts, u64* h_pub, u64 seq) {
  publish_word(d_counts[threadIdx.x & 15], h_pub, seq);
}

}  // namespace dg
