// remap.hip — rewriting a store's value ids after the host relabelled its value table
// (dg_remap_values).
//
// Value ids are order-preserving ranks in Erlang term order (the read
// tie-break of aw_lww_map.ex:211-216) allocated with gaps; when a gap is used up the
// host re-spaces the ids of one region (interning.py / marshal.c: the table values below
// and above the canonical integers).  The map old id -> new id is strictly increasing and
// keeps each id inside its region, so ids outside [old_ids[0], old_ids[n-1]] (canonical
// integers, the other region) pass unchanged, a store stays sorted by
// (key, val, ts, node, cnt) and the rewrite is one streaming
// pass over the val column: 8 B read + 8 B written per row, plus a binary search in
// the (L2-resident) id table.  The table is staged in LDS in 2048-entry slices when
// it is small enough to fit; larger tables are searched in global memory.
#include "dg_launch.h"

namespace dg {

namespace {

constexpr int RB = 256;
constexpr int RLDS = 2048;  // table entries staged in LDS (16 KB)

__device__ __forceinline__ u64 lower_bound_u64(const u64* t, u64 n, u64 x) {
  u64 lo = 0, hi = n;
  while (lo < hi) {
    const u64 mid = (lo + hi) >> 1;
    if (t[mid] < x)
      lo = mid + 1;
    else
      hi = mid;
  }
  return lo;
}

__global__ __launch_bounds__(RB) void remap_values_kernel(u64* val, u64 n, const u64* old_ids,
                                                          const u64* new_ids, u64 n_ids, u32* err) {
  __shared__ u64 s_old[RLDS];
  const bool staged = n_ids <= RLDS;
  if (staged) {
    for (u64 i = threadIdx.x; i < n_ids; i += RB) s_old[i] = old_ids[i];
    __syncthreads();
  }
  for (u64 i = (u64)blockIdx.x * RB + threadIdx.x; i < n; i += (u64)gridDim.x * RB) {
    const u64 v = val[i];
    const u64 j = staged ? lower_bound_u64(s_old, n_ids, v) : lower_bound_u64(old_ids, n_ids, v);
    const bool inside = j < n_ids && (j > 0 || v == (staged ? s_old[0] : old_ids[0]));
    if (!inside) continue;  // outside the relabelled region: unchanged
    if ((staged ? s_old[j] : old_ids[j]) == v)
      val[i] = new_ids[j];
    else
      atomicOr(err, 1u);  // inside the region but not in its table: a stale id
  }
}

}  // namespace

hipError_t launch_remap_values(u64* val, u64 n, const u64* old_ids, const u64* new_ids, u64 n_ids,
                               u32* err, hipStream_t st) {
  if (n == 0) return hipSuccess;
  u64 blocks = (n + RB * 4 - 1) / (RB * 4);
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(remap_values_kernel, dim3((unsigned)blocks), dim3(RB), 0, st, val, n, old_ids,
                     new_ids, n_ids, err);
  return hipGetLastError();
}

}  // namespace dg
