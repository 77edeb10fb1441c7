// dg_tree.h — the term hashes of a Merkle row (dg_term_hashes, include/deltagpu.h),
// shared by the tree kernels (merkle.hip) and the fused small-delta join (small.hip).
#pragma once
#include "dg_launch.h"

namespace dg {

// The value's and the node's terms in a row hash (dg_term_hashes): a canonical integer
// value id [2^58, 2^63) and ids missing from the tables stand for themselves.
__device__ __forceinline__ u64 th_val(const TermH& th, u64 v) {
  if (!th.on || th.nv == 0 || (v >= (1ull << 58) && v < (1ull << 63))) return v;
  u64 lo = 0, hi = th.nv;
  while (lo < hi) {
    const u64 mid = (lo + hi) >> 1;
    if (th.vid[mid] < v)
      lo = mid + 1;
    else
      hi = mid;
  }
  return (lo < th.nv && th.vid[lo] == v) ? th.vh[lo] : v;
}

__device__ __forceinline__ u64 th_node(const TermH& th, u32 n) {
  return (th.on && (u64)n < th.nn) ? th.nh[n] : (u64)n;
}


}  // namespace dg
