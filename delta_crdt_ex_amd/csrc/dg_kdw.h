// dg_kdw.h — the write step of dg_join_delta's one-wait path (kdelta.hip), as a block
// body: merkle.hip's kd_finish_kernel runs it in the same launch as the tree's chunk
// re-reduction (the two read only what kd_count_kernel wrote, so they overlap instead of
// running back to back).
//
// One workgroup of NT threads covers NT / KD_BLOCK of kd_count_kernel's tiles, one key per
// thread: the key's new rows in tuple order -- in place when no key's row count changed
// (and only for changed keys), else straight to their final places in the spare store --
// the changed keys and their rows, the splice index of the rows that move (splice.hip),
// and (workgroup 0) the union context into the state's.  Every state write is skipped when
// the tree update reported an input error (all or nothing).
#pragma once
#include "dg_device.h"
#include "dg_launch.h"

namespace dg {

namespace {

template <int NT>
__device__ __forceinline__ void kd_write_block(const KdArgs& p, u64 blk) {
  static_assert(NT % KD_BLOCK == 0, "whole count tiles per workgroup");
  constexpr int WPT = KD_BLOCK / WAVE;  // waves per count tile
  __shared__ u64 s_w[4][NT / WAVE];
  const int tid = threadIdx.x, lane = tid & (WAVE - 1), w = tid / WAVE;
  const u64 u = blk * NT + tid;
  const u64 tile = u / KD_BLOCK;
  const u64 guard = p.d_counts[4];
  const bool tree_bad = p.err && (*p.err & MERKLE_INPUT_ERR);
  if (guard) return;  // (uniform) nothing is written: the caller falls back or reports
  const bool moved = p.d_counts[5] != 0;
  if (blk == 0 && !tree_bad) {   // the union context into the state's (Dots.union, :155)
    const u64 nc = p.d_counts[1];  // (and the caller's copy, when it fits)
    const bool co = p.co_node && nc <= p.co_cap;
    for (u64 i = tid; i < nc && i < p.ca_cap; i += NT) {
      const u32 n = p.uc_node[i];
      const u64 c = p.uc_cnt[i];
      p.ca_node[i] = n;
      p.ca_cnt[i] = c;
      if (co) {
        p.co_node[i] = n;
        p.co_cnt[i] = c;
      }
    }
  }
  u64 rn = 0;
  u32 na = 0, nd = 0, ne = 0;
  bool chg = false;
  if (u < p.nk) {
    rn = p.runs[u];
    na = (u32)(rn & 0xFFFF);
    nd = (u32)((rn >> 16) & 0xFFFF);
    ne = (u32)((rn >> 32) & 0xFFFF);
    chg = (rn >> 48) & 1;
  }
  // exclusive in-tile prefixes of (na, ne, chg, chg rows) + the tile's offsets
  const u64 x[4] = {na, ne, chg ? 1u : 0u, chg ? ne : 0u};
  u64 pre[4];
#pragma unroll
  for (int q = 0; q < 4; q++) {
    u64 inc = x[q];
#pragma unroll
    for (int d = 1; d < WAVE; d <<= 1) {
      const u64 y = __shfl_up(inc, d, WAVE);
      if (lane >= d) inc += y;
    }
    if (lane == WAVE - 1) s_w[q][w] = inc;
    pre[q] = inc - x[q];
  }
  // the tiles' offsets: the figures of every earlier tile (kd_count_kernel's per-workgroup
  // sums), added up here by the whole workgroup -- one round of loads -- instead of a scan
  // by the count kernel's last workgroup
  constexpr int TPW = NT / KD_BLOCK;  // count tiles per workgroup
  const u64 t0 = blk * TPW;           // this workgroup's first tile
  __shared__ u64 s_e[4][NT / WAVE], s_own[4][TPW];
  u64 e[4] = {0, 0, 0, 0};
  for (u64 t = tid; t < t0; t += NT) {
    u64 y[4];
#pragma unroll
    for (int q = 0; q < 4; q++) y[q] = p.part[t * KD_NV + q];
#pragma unroll
    for (int q = 0; q < 4; q++) e[q] += y[q];
  }
  if (tid < 4 * TPW && t0 + tid / 4 < p.ntiles) s_own[tid % 4][tid / 4] = p.part[(t0 + tid / 4) * KD_NV + tid % 4];
#pragma unroll
  for (int q = 0; q < 4; q++) {
#pragma unroll
    for (int d = WAVE / 2; d >= 1; d >>= 1) e[q] += __shfl_xor(e[q], d, WAVE);
    if (lane == 0) s_e[q][w] = e[q];
  }
  __syncthreads();
  const int ti = (int)(tile - t0);  // this thread's tile within the workgroup
#pragma unroll
  for (int q = 0; q < 4; q++) {
    u64 below = 0;
    for (int i = 0; i < NT / WAVE; i++) below += s_e[q][i];
    for (int i = 0; i < ti; i++) below += s_own[q][i];
    for (int i = w - w % WPT; i < w; i++) below += s_w[q][i];
    pre[q] += below;
  }
  if (u >= p.nk) return;
  const u64 k = p.keys[u];
  const u64 a_lo = p.a_lo[u], d_lo = p.d_lo[u], am = p.amask[u], dm = p.dmask[u];
  const u64 a_off = pre[0], e_off = pre[1], c_off = pre[2], r_off = pre[3];
  const u64 n_e = p.d_counts[0], n_ak = p.d_counts[6];
  // the splice index (splice.hip): where this key's rows go and where the untouched rows
  // before it move
  const i64 gap = (i64)a_lo - (i64)a_off;
  if (moved) {
    p.end[u] = a_lo + na;
    p.shift[u] = (i64)e_off - (i64)a_off;
    const u64 end_lo = u > 0 ? p.a_lo[u - 1] + (p.runs[u - 1] & 0xFFFF) : 0ull;
    const u64 end_hi = a_lo + na;
    for (u64 t = (end_lo + SPLICE_TILE - 1) / SPLICE_TILE; t <= p.a_tiles && t * SPLICE_TILE < end_hi; t++)
      p.tile_u0[t] = u;
    if (u == p.nk - 1) {
      p.shift[p.nk] = (i64)n_e - (i64)n_ak;
      for (u64 t = (end_hi + SPLICE_TILE - 1) / SPLICE_TILE; t <= p.a_tiles; t++) p.tile_u0[t] = p.nk;
    }
  }
  // the key's new rows in tuple order: the kept state rows and the new delta rows (disjoint)
  const bool wr_state = !tree_bad;  // in place: only when the tree took the update
  const bool wr_rows = chg && p.has_rows && r_off + ne <= p.rows_cap;
  if (!(wr_state || moved) && !wr_rows && !chg) return;
  u32 i = 0, j = 0, o = 0;
  auto next_a = [&]() { while (i < na && !((am >> i) & 1)) i++; };
  auto next_d = [&]() { while (j < nd && !((dm >> j) & 1)) j++; };
  next_a();
  next_d();
  Row ra{}, rb{};
  if (i < na) ra = load_row(p.a, a_lo + i);
  if (j < nd) rb = load_row(p.d, d_lo + j);
  while (i < na || j < nd) {
    bool takeA;
    if (i >= na) {
      takeA = false;
    } else if (j >= nd) {
      takeA = true;
    } else {
      bool lt, eq;
      row_cmp_bf(ra, rb, lt, eq);
      takeA = lt;
    }
    const Row r = takeA ? ra : rb;
    if (moved)
      store_row(p.sp, (u64)((i64)(e_off + o) + gap), r);
    else if (wr_state && chg)  // (unchanged keys keep their rows as they are)
      store_row(p.aw, a_lo + o, r);
    if (wr_rows) store_row(p.rows, r_off + o, r);
    o++;
    if (takeA) {
      i++;
      next_a();
      if (i < na) ra = load_row(p.a, a_lo + i);
    } else {
      j++;
      next_d();
      if (j < nd) rb = load_row(p.d, d_lo + j);
    }
  }
  if (chg && c_off < p.cap) p.changed[c_off] = k;
}

}  // namespace

}  // namespace dg
