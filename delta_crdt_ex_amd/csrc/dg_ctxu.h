// dg_ctxu.h — Dots.union/2 (reference aw_lww_map.ex:39-52) by one workgroup: the join's
// context union (join.hip: its own kernel, or one extra workgroup of the join launch) and
// dg_join_delta's (kdelta.hip: the count kernel's last workgroup).
#pragma once
#include "dg_launch.h"

namespace dg {

namespace {

// ------------------------------------------------------------- context union
// Dots.union/2 (aw_lww_map.ex:39-52) in one 1024-thread workgroup: contexts are
// version vectors of at most a few hundred nodes in practice (one entry per
// replica) or the explicit dot sets of mutation deltas.

struct CtxUnionArgs {
  Ctx a, b;
  u32* out_node;
  u64* out_cnt;
  u64* d_count;
  u32* tmp_node;  // a.n + b.n
  u64* tmp_cnt;   // a.n + b.n
  u32* rank;      // b.n + 1 (after compression)
};

// Chunked exclusive block scan of flags produced by `flag(i)` for i < n; writes the
// running exclusive count to out[i] (and the total to out[n]).  Returns the total.
template <int NT, class F>
__device__ __forceinline__ u32 block_scan_flags(u64 n, F flag, u32* out, u32* s_wave) {
  u32 carry = 0;
  for (u64 base = 0; base < n; base += NT) {
    u64 i = base + threadIdx.x;
    u32 f = i < n ? (flag(i) ? 1u : 0u) : 0u;
    u32 tot;
    u32 ex = block_excl_scan<NT>(f, s_wave, &tot);
    if (i < n) out[i] = carry + ex;
    carry += tot;
    __syncthreads();
  }
  if (threadIdx.x == 0) out[n] = carry;
  __syncthreads();
  return carry;
}

// Compress a dot set (sorted by (node, cnt)) into a VV: the last dot of every node
// run carries the node's max counter (Dots.compress/1, aw_lww_map.ex:13-20).
template <int NT>
__device__ __forceinline__ u64 compress_into(const Ctx c, u32* onode, u64* ocnt, u32* scratch, u32* s_wave) {
  auto tail = [&](u64 i) { return i + 1 == c.n || c.node[i + 1] != c.node[i]; };
  u32 total = block_scan_flags<NT>(c.n, tail, scratch, s_wave);
  for (u64 i = threadIdx.x; i < c.n; i += NT)
    if (tail(i)) {
      onode[scratch[i]] = c.node[i];
      ocnt[scratch[i]] = c.cnt[i];
    }
  __syncthreads();
  return total;
}

// Dots.union/2 by one workgroup of NT threads; `s_wave` holds NT/64 + 1 words of LDS.
template <int NT>
__device__ __forceinline__ void ctx_union_block(const CtxUnionArgs p, u32* s_wave) {
  const int tid = threadIdx.x;
  if (p.a.kind == 1 && p.b.kind == 1) {
    // MapSet.union: sorted set union on (node, cnt)
    const Ctx &X = p.a, &Y = p.b;
    auto lbX = [&](u32 n, u64 c) {
      u64 lo = 0, hi = X.n;
      while (lo < hi) {
        u64 m = (lo + hi) >> 1;
        if (X.node[m] < n || (X.node[m] == n && X.cnt[m] < c))
          lo = m + 1;
        else
          hi = m;
      }
      return lo;
    };
    auto lbY = [&](u32 n, u64 c) {
      u64 lo = 0, hi = Y.n;
      while (lo < hi) {
        u64 m = (lo + hi) >> 1;
        if (Y.node[m] < n || (Y.node[m] == n && Y.cnt[m] < c))
          lo = m + 1;
        else
          hi = m;
      }
      return lo;
    };
    auto ynew = [&](u64 j) {
      u64 q = lbX(Y.node[j], Y.cnt[j]);
      return !(q < X.n && X.node[q] == Y.node[j] && X.cnt[q] == Y.cnt[j]);
    };
    u32 ny = block_scan_flags<NT>(Y.n, ynew, p.rank, s_wave);
    for (u64 i = tid; i < X.n; i += NT) {
      u64 q = lbY(X.node[i], X.cnt[i]);
      u64 o = i + p.rank[q];
      p.out_node[o] = X.node[i];
      p.out_cnt[o] = X.cnt[i];
    }
    for (u64 j = tid; j < Y.n; j += NT)
      if (ynew(j)) {
        u64 o = p.rank[j] + lbX(Y.node[j], Y.cnt[j]);
        p.out_node[o] = Y.node[j];
        p.out_cnt[o] = Y.cnt[j];
      }
    if (tid == 0) *p.d_count = X.n + ny;
    return;
  }
  // At least one VV: fold dot sets into VVs first (union(set, map) = union(map, set)).
  Ctx X = p.a, Y = p.b;
  if (X.kind == 1) {
    u64 n = compress_into<NT>(X, p.tmp_node, p.tmp_cnt, p.rank, s_wave);
    X.node = p.tmp_node;
    X.cnt = p.tmp_cnt;
    X.n = n;
    X.kind = 0;
  }
  if (Y.kind == 1) {
    u64 n = compress_into<NT>(Y, p.tmp_node + p.a.n, p.tmp_cnt + p.a.n, p.rank, s_wave);
    Y.node = p.tmp_node + p.a.n;
    Y.cnt = p.tmp_cnt + p.a.n;
    Y.n = n;
    Y.kind = 0;
  }
  auto lb = [](const Ctx& c, u32 n) {
    u64 lo = 0, hi = c.n;
    while (lo < hi) {
      u64 m = (lo + hi) >> 1;
      if (c.node[m] < n)
        lo = m + 1;
      else
        hi = m;
    }
    return lo;
  };
  auto ynew = [&](u64 j) {
    u64 q = lb(X, Y.node[j]);
    return !(q < X.n && X.node[q] == Y.node[j]);
  };
  u32 ny = block_scan_flags<NT>(Y.n, ynew, p.rank, s_wave);
  for (u64 i = tid; i < X.n; i += NT) {
    u64 q = lb(Y, X.node[i]);
    u64 c = X.cnt[i];
    if (q < Y.n && Y.node[q] == X.node[i] && Y.cnt[q] > c) c = Y.cnt[q];  // Map.update max
    u64 o = i + p.rank[q];
    p.out_node[o] = X.node[i];
    p.out_cnt[o] = c;
  }
  for (u64 j = tid; j < Y.n; j += NT)
    if (ynew(j)) {
      u64 o = p.rank[j] + lb(X, Y.node[j]);
      p.out_node[o] = Y.node[j];
      p.out_cnt[o] = Y.cnt[j];
    }
  if (tid == 0) *p.d_count = X.n + ny;
}


}  // namespace

__host__ __device__ inline CtxUnionArgs make_cu(const Ctx& a, const Ctx& b, u32* out_node, u64* out_cnt, u64* d_count,
                                                 void* tmp) {
  CtxUnionArgs p;
  p.a = a;
  p.b = b;
  p.out_node = out_node;
  p.out_cnt = out_cnt;
  p.d_count = d_count;
  char* t = (char*)tmp;
  p.tmp_cnt = (u64*)t;
  t += (a.n + b.n) * 8;
  p.tmp_node = (u32*)t;
  t += (a.n + b.n) * 4;
  p.rank = (u32*)t;
  return p;
}

}  // namespace dg
