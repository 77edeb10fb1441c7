// join.hip — AWLWWMap.join/3 on gfx950 (reference lib/delta_crdt/aw_lww_map.ex:153-209).
//
// Formulation.  Both stores are sorted by the full row tuple (key, val, ts, node,
// cnt).  The joined state is the merge of the two stores filtered per row:
//
//   row of a, also in b  (same key, {v,ts} entry and dot)  -> kept   (s1 ∩ s2)
//   row of a only                                          -> kept iff dot ∉ c_b  (s1 \ c2)
//   row of b only                                          -> kept iff dot ∉ c_a  (s2 \ c1)
//   row of b equal to a row of a                           -> dropped (MapSet dedup)
//
// which is join_dot_sets/4 (:196-209) applied to every {v,ts} entry of every key;
// entries and keys that end up empty simply emit no rows (:177-181).  With an
// explicit `keys` list, rows of keys outside it are carried over right-biased
// (b's rows if b has the key, else a's), as Map.merge(Map.drop(..)) does (:185-188).
//
// Kernel shape (partition pass + one single-pass join launch, HBM-bound):
//   * a tile = 1024 merged positions = 512 threads x 2; tiles are numbered by an
//     atomic ticket so the decoupled look-back only waits on resident tiles;
//   * the tiles' merge-path splits come from a partition pass (one wave per tile
//     boundary, 128-ary search seeded at the uniform-hash estimate: 2 rounds of
//     global loads instead of ~21 dependent ones);
//   * the tile's rows (+1 neighbour on each side) are staged in LDS (SoA, 36 B/row);
//   * each thread merges 4 positions serially from LDS and decides keep/drop;
//   * block scan of keep counts -> block-wide look-back (1024 predecessors per
//     round) -> compacted rows written coalesced.
#include <algorithm>

#include "dg_launch.h"

namespace dg {

namespace {

constexpr int JB = JOIN_BLOCK;
constexpr int JI = JOIN_ITEMS;
constexpr int JT = JOIN_TILE;
constexpr int JS = JT + 4;  // LDS row slots: tile rows + one neighbour on each side per store

#ifdef DG_STAMPS
// Diagnostic build only (DG_STAMPS=1): per-tile phase timestamps (s_memrealtime,
// 100 MHz) written by lane 0 into a buffer no other code reads.
__device__ u64 g_join_stamps[65536 * 8];
#define JSTAMP(tile, k)                                                              \
  do {                                                                               \
    __syncthreads();                                                                 \
    __builtin_amdgcn_sched_barrier(0);                                               \
    if (threadIdx.x == 0 && (tile) < 65536) g_join_stamps[(tile) * 8 + (k)] =        \
        __builtin_amdgcn_s_memrealtime();                                            \
    __builtin_amdgcn_sched_barrier(0);                                               \
  } while (0)
#else
#define JSTAMP(tile, k) \
  do {                  \
  } while (0)
#endif

// ------------------------------------------------------------- context union
// Dots.union/2 (aw_lww_map.ex:39-52) in one 1024-thread workgroup: contexts are
// version vectors of at most a few hundred nodes in practice (one entry per
// replica) or the explicit dot sets of mutation deltas.

constexpr int CB = 1024;  // threads of the standalone context-union kernel

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

__global__ __launch_bounds__(CB) void ctx_union_kernel(CtxUnionArgs p) {
  __shared__ u32 s_wave[CB / WAVE + 1];
  ctx_union_block<CB>(p, s_wave);
}

struct JoinArgs {
  Rows a, b;
  Ctx ca, cb;
  const u64* keys;
  u64 n_keys;
  u64* splits;  // merge-path split (a index) of every tile boundary, from the partition pass
  u64 ntiles;
  RowsOut out;
  Scan scan;        // look-back granules + tile tickets
  u64* d_count;
};

constexpr int SMALL_VV = 8;  // VVs up to this many nodes are probed from LDS

// One staged tile: its rows (+ neighbours) and, after the merge, its compaction list.
struct Buf {
  u64 key[JS];
  u64 val[JS];
  u64 cnt[JS];
  i64 ts[JS];
  u32 node[JS];
  unsigned short comp[JT];
};

// Two tiles live per workgroup: the one being merged and the previous one, whose
// output offset is resolved (look-back) and whose rows are written one iteration later.
struct Lds {
  Buf buf[2];
  unsigned short posinfo[JT];  // merge of the current tile: slot of each position | keep << 15
  u64 vv_cnt[2][SMALL_VV];     // small version vectors (c_a, c_b), staged once
  u32 vv_node[2][SMALL_VV];
  u32 wave[JB / WAVE + 1];
  u64 lb[3 * (JB / WAVE) + 2];
  u64 bcast[8];
};



// Merge-path predicate on diagonal `diag` over global memory: A[i] <= B[diag-1-i].
__device__ __forceinline__ bool mp_pred(const Rows A, const Rows B, u64 diag, u64 i) {
  u64 j = diag - 1 - i;
  u64 ka = A.key[i], kb = B.key[j];
  if (ka != kb) return ka < kb;
  return row_le(load_row(A, i), load_row(B, j));
}

// Dots.member? against a context staged in LDS or read from global memory.

// Merge-path partition: one wave per tile boundary q (diagonal min(q * JT, na + nb))
// finds the boundary's split with a 128-ary search (two samples per lane per round).
// Round 0 samples a +-4160 window around the uniform-hash estimate (key ids are 64-bit
// hashes: the split lies within a few sqrt(d) of d * na / (na + nb)); for any key
// distribution the search stays exact, only slower.  Writes splits[q] = #A rows
// among the first `diag` merged rows (ties go to A).
constexpr int PB = 256;  // threads per partition block = 4 boundaries

__global__ __launch_bounds__(PB) void join2_partition_kernel(Rows A, Rows B, u64 ntiles,
                                                             u64* splits, CtxUnionArgs cu) {
  if (blockIdx.x == gridDim.x - 1) {  // extra workgroup: Dots.union(c1, c2) (aw_lww_map.ex:155)
    __shared__ u32 s_wave[PB / WAVE + 1];
    ctx_union_block<PB>(cu, s_wave);
    return;
  }
  const int lane = threadIdx.x & (WAVE - 1);
  const u64 q = (u64)blockIdx.x * (PB / WAVE) + (threadIdx.x >> 6);
  if (q > ntiles) return;
  const u64 na = A.n, nb = B.n, total = na + nb;
  const u64 d = min(q * (u64)JOIN_TILE, total);
  u64 lo = d > nb ? d - nb : 0, hi = min(d, na);
  const u64 est = total ? (u64)((double)d * (double)na / (double)total) : 0;
  constexpr u64 WIN = 4160;
  constexpr int K = 2 * WAVE;  // samples per round
  for (int round = 0; round < 64 && hi > lo; round++) {
    const u64 span = hi - lo;
    u64 slo = lo, sspan = span;
    if (round == 0 && span > 2 * WIN + K) {
      u64 wlo = est > WIN ? est - WIN : 0, whi = est + WIN;
      wlo = max(wlo, lo);
      whi = min(whi, hi);
      if (whi > wlo + K) {
        slo = wlo;
        sspan = whi - wlo;
      }
    }
    // lane l evaluates samples 2l and 2l+1
    bool f0, f1;
    if (sspan <= (u64)K) {
      const u64 x0 = slo + 2 * lane, x1 = x0 + 1;
      f0 = x0 < slo + sspan && !mp_pred(A, B, d, x0);
      f1 = x1 < slo + sspan && !mp_pred(A, B, d, x1);
    } else {
      const u64 x0 = slo + (sspan * (u64)(2 * lane + 1)) / (K + 1);
      const u64 x1 = slo + (sspan * (u64)(2 * lane + 2)) / (K + 1);
      f0 = !mp_pred(A, B, d, x0);
      f1 = !mp_pred(A, B, d, x1);
    }
    const u64 m0 = __ballot(f0), m1 = __ballot(f1);
    // first false sample index k in [0, K): min over lanes of (2l if f0, 2l+1 if f1)
    int kf = K;
    if (m0 | m1) {
      const int l0 = m0 ? __ffsll((long long)m0) - 1 : 64;
      const int l1 = m1 ? __ffsll((long long)m1) - 1 : 64;
      kf = (l0 <= l1) ? 2 * l0 : 2 * l1 + 1;
    }
    if (sspan <= (u64)K) {
      const u64 ans = (u64)kf < sspan ? slo + kf : slo + sspan;
      lo = hi = ans;  // direct rounds always cover [lo, hi)
    } else if (kf == K) {
      lo = slo + (sspan * (u64)K) / (K + 1) + 1;
    } else {
      const u64 nh = slo + (sspan * (u64)(kf + 1)) / (K + 1);
      if (kf > 0) lo = slo + (sspan * (u64)kf) / (K + 1) + 1;
      hi = nh;
    }
  }
  if (lane == 0) splits[q] = lo;
}

// Version vectors of at most SMALL_VV nodes (one entry per replica: the common case)
// are held in wave-uniform registers and probed with unrolled compares; anything else
// (bigger VVs, explicit dot sets) is binary-searched in global memory (L1/L2-resident).

// A small VV staged in LDS (uniform addresses: every probe is a broadcast read).
struct SmallVV {
  const u32* node;
  const u64* cnt;
  u32 n;
};

// Dots.member?(vv, {dn, dc}): Map.get(vv, dn, 0) >= dc  (aw_lww_map.ex:71-73)
__device__ __forceinline__ bool small_vv_covers(const SmallVV& v, u32 dn, u64 dc) {
  u64 have = 0;
#pragma unroll
  for (int q = 0; q < SMALL_VV; q++)
    if ((u32)q < v.n && v.node[q] == dn) have = v.cnt[q];
  return have >= dc;
}

__device__ __forceinline__ Row lds_row(const Buf& s, int x) {
  Row r;
  r.key = s.key[x];
  r.val = s.val[x];
  r.ts = s.ts[x];
  r.node = s.node[x];
  r.cnt = s.cnt[x];
  return r;
}

// Merge JI consecutive positions of the tile and decide keep/drop for each (the body
// of join_dot_sets/4 per row, see the file header).  Rows are read from LDS whole (all
// five columns in parallel) so every merge step costs one LDS round trip.
template <bool SMALL, bool KEYS>
__device__ __forceinline__ void merge_items(const Ctx ca, const Ctx cb, const SmallVV& va,
                                            const SmallVV& vb, const u64* keys,
                                            const u64 n_keys, const u64 nb, const Buf& s,
                                            int nat, int nbt, u64 a0, u64 b0, u32& keep,
                                            unsigned short (&src)[JI], u64 t_stamp) {
  const int tid = threadIdx.x;
  const int offB = nat + 2;
  const int tt = nat + nbt;
  const int diag = min(tid * JI, tt);
  const int dend = min(diag + JI, tt);
  // Merge-path split of this thread's diagonal: first i with NOT(a[i] <= b[diag-1-i]).
  // (1) key-only binary search for iq = first i with a[i].key > b[diag-1-i].key (two
  //     LDS words per probe); the exact split lies in (iq - r, iq] where r counts the
  //     positions whose keys tie; (2) full-tuple gallop down from iq to find it.
  const int lo0 = diag > nbt ? diag - nbt : 0, hi0 = min(diag, nat);
  int lo = lo0, hi = hi0;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (s.key[1 + mid] <= s.key[offB + 1 + (diag - 1 - mid)])
      lo = mid + 1;
    else
      hi = mid;
  }
  // P(i) = a[i] <= b[diag-1-i] is monotone and P(i) implies key <=, so split <= iq = lo.
  int hiP = lo, loP = lo0, step = 1;
  while (hiP > loP) {  // gallop: find a point where P holds
    const int x = max(hiP - step, loP);
    if (row_le(lds_row(s, 1 + x), lds_row(s, offB + 1 + (diag - 1 - x)))) {
      loP = x + 1;
      break;
    }
    hiP = x;
    step <<= 1;
  }
  lo = loP;
  hi = hiP;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (row_le(lds_row(s, 1 + mid), lds_row(s, offB + 1 + (diag - 1 - mid))))
      lo = mid + 1;
    else
      hi = mid;
  }
  int i = lo, j = diag - lo;
  JSTAMP(t_stamp, 5);
  // ra = a[i], rb = b[j] (possibly the neighbour past the tile), pa = a[i-1]
  Row ra = lds_row(s, 1 + i), rb = lds_row(s, offB + 1 + j), pa = lds_row(s, i);
  keep = 0;
#pragma unroll
  for (int k = 0; k < JI; k++) {
    src[k] = 0;
    if (diag + k < dend) {
      const bool bvalid = (b0 + (u64)j) < nb;  // b[j] exists globally
      const bool takeA = i < nat && (j >= nbt || row_le(ra, rb));
      bool kp;
      if (takeA) {
        const bool joined = !KEYS || keys == nullptr || keyset_has(keys, n_keys, ra.key);
        if (joined) {
          const bool inB = bvalid && row_eq(ra, rb);
          const bool cov = SMALL ? small_vv_covers(vb, ra.node, ra.cnt)
                                 : ctx_covers(cb.node, cb.cnt, cb.n, cb.kind, ra.node, ra.cnt);
          kp = inB || !cov;
        } else {
          // Map.merge(Map.drop(a), Map.drop(b)): a's rows survive iff b lacks the key
          const bool bprev = (b0 + (u64)j) >= 1 && s.key[offB + j] == ra.key;
          const bool bnext = bvalid && rb.key == ra.key;
          kp = !(bprev || bnext);
        }
        src[k] = (unsigned short)(1 + i);
        i++;
        pa = ra;
        if (k + 1 < JI) ra = lds_row(s, 1 + i);
      } else {
        const bool joined = !KEYS || keys == nullptr || keyset_has(keys, n_keys, rb.key);
        if (joined) {
          const bool dupA = (a0 + (u64)i) >= 1 && row_eq(pa, rb);
          const bool cov = SMALL ? small_vv_covers(va, rb.node, rb.cnt)
                                 : ctx_covers(ca.node, ca.cnt, ca.n, ca.kind, rb.node, rb.cnt);
          kp = !dupA && !cov;
        } else {
          kp = true;
        }
        src[k] = (unsigned short)(offB + 1 + j);
        j++;
        if (k + 1 < JI) rb = lds_row(s, offB + 1 + j);
      }
      if (kp) keep |= 1u << k;
    }
  }
}

// Rows of a tile (plus one neighbour on each side of each store) as staged in LDS:
// slot x < nat + 2 is a[a0 - 1 + x], slot x >= nat + 2 is b[b0 - 1 + (x - nat - 2)].
// A thread owns slots tid, tid + JB, ... (SLOTS of them); their rows are prefetched
// into registers one tile ahead so that HBM reads of tile k+1 overlap the merge of k.
constexpr int SLOTS = (JS + JB - 1) / JB;

struct Prefetch {
  u64 key[SLOTS], val[SLOTS], cnt[SLOTS];
  i64 ts[SLOTS];
  u32 node[SLOTS];
};

// Global row index of staging slot x, or -1 if the slot is outside the stores.
__device__ __forceinline__ i64 slot_row(int x, int nat, u64 a0, u64 b0, u64 na, u64 nb,
                                        bool* from_b) {
  if (x < nat + 2) {
    const i64 g = (i64)a0 - 1 + x;
    *from_b = false;
    return (g >= 0 && (u64)g < na) ? g : -1;
  }
  const i64 g = (i64)b0 - 1 + (x - (nat + 2));
  *from_b = true;
  return (g >= 0 && (u64)g < nb) ? g : -1;
}

// FAST: full-state join (no key list) of two version vectors of <= SMALL_VV nodes —
// the anti-entropy shape; everything else takes the general instantiation.
template <bool FAST>
__global__ __launch_bounds__(JB) __attribute__((amdgpu_waves_per_eu(4, 4))) void join2_tiles_kernel(JoinArgs p) {
  __shared__ Lds s;
  const int tid = threadIdx.x;
  const u64 na = p.a.n, nb = p.b.n, total = na + nb, ntiles = p.ntiles;
  const u64 G = gridDim.x;  // persistent tile workers
  if (FAST && tid < SMALL_VV) {
    s.vv_node[0][tid] = (u64)tid < p.ca.n ? p.ca.node[tid] : 0u;
    s.vv_cnt[0][tid] = (u64)tid < p.ca.n ? p.ca.cnt[tid] : 0ull;
    s.vv_node[1][tid] = (u64)tid < p.cb.n ? p.cb.node[tid] : 0u;
    s.vv_cnt[1][tid] = (u64)tid < p.cb.n ? p.cb.cnt[tid] : 0ull;
  }
  const SmallVV va{s.vv_node[0], s.vv_cnt[0], (u32)p.ca.n};
  const SmallVV vb{s.vv_node[1], s.vv_cnt[1], (u32)p.cb.n};
  // Tiles are handed out by an atomic ticket (launch order), so a tile's look-back only
  // ever waits on tiles already held by running workgroups.  Every workgroup takes
  // exactly one ticket >= ntiles (its stop signal): ntiles + G tickets in all, and the
  // taker of the last one resets the counter for the next launch.
  auto take_ticket = [&]() -> u64 {
    const u32 tk = atomicAdd(p.scan.ticket, 1u);
    if ((u64)tk == ntiles + G - 1) atomicExch(p.scan.ticket, 0u);
    return tk;
  };
  if (tid == 0) {
    const u64 t0 = take_ticket();
    s.bcast[0] = t0;
    if (t0 < ntiles) {
      s.bcast[1] = p.splits[t0];
      s.bcast[2] = p.splits[t0 + 1];
      const u64 t1 = take_ticket();
      s.bcast[3] = t1;
      if (t1 < ntiles) {
        s.bcast[4] = p.splits[t1];
        s.bcast[5] = p.splits[t1 + 1];
      }
    }
  }
  __syncthreads();
  u64 t = s.bcast[0];
  if (t >= ntiles) return;
  u64 a0 = s.bcast[1], a1 = s.bcast[2];
  u64 tn = s.bcast[3], a0n = s.bcast[4], a1n = s.bcast[5];

  Prefetch R;
  auto prefetch = [&](u64 tt, u64 x0, u64 x1) {
    const u64 d0 = tt * JT, d1 = min(d0 + (u64)JT, total);
    const int nat = (int)(x1 - x0), nbt = (int)((d1 - x1) - (d0 - x0));
    const u64 y0 = d0 - x0;
#pragma unroll
    for (int k = 0; k < SLOTS; k++) {
      const int x = tid + k * JB;
      bool fb;
      const i64 g = x < nat + nbt + 4 ? slot_row(x, nat, x0, y0, na, nb, &fb) : -1;
      if (g >= 0) {
        const Rows& src = fb ? p.b : p.a;
        R.key[k] = src.key[g];
        R.val[k] = src.val[g];
        R.ts[k] = src.ts[g];
        R.node[k] = src.node[g];
        R.cnt[k] = src.cnt[g];
      }
    }
  };
  prefetch(t, a0, a1);

  // the previous tile, kept in the other buffer until its output offset is known
  bool pending = false;
  u64 tp = 0;
  u32 np = 0;
  int pbuf = 0;

  // resolve the pending tile's prefix (look-back), publish its inclusive prefix and
  // write its compacted rows to the output
  auto flush = [&](int pb) {
    u64 prefix = 0;
    if (tp > 0) prefix = lb_lookback_block<JB, 2>(p.scan.state, tp, p.scan.epoch, p.scan.err, s.lb);
    if (tid == 0) {
      if (tp > 0) lb_publish(p.scan.state, tp, p.scan.epoch, LB_INC, prefix + np);
      if (tp == ntiles - 1) p.d_count[0] = prefix + np;
    }
    const Buf& b = s.buf[pb];
    for (u32 q = tid; q < np; q += JB) {
      const int slot = b.comp[q];
      const u64 o = prefix + q;
      p.out.key[o] = b.key[slot];
      p.out.val[o] = b.val[slot];
      p.out.ts[o] = b.ts[slot];
      p.out.node[o] = b.node[slot];
      p.out.cnt[o] = b.cnt[slot];
    }
  };

  for (int k = 0;; k++) {
    const int cb_ = k & 1;
    Buf& cur = s.buf[cb_];
    const u64 d0 = t * JT, d1 = min(d0 + (u64)JT, total);
    const int nat = (int)(a1 - a0), nbt = (int)((d1 - a1) - (d0 - a0));
    const u64 b0 = d0 - a0;
    JSTAMP(t, 0);
    u64 t2 = 0;  // ticket after next: issued now, consumed after the merge
    if (tid == 0 && tn < ntiles) t2 = take_ticket();
    // ---- commit the prefetched rows of tile t to LDS
#pragma unroll
    for (int q = 0; q < SLOTS; q++) {
      const int x = tid + q * JB;
      bool fb;
      const i64 g = x < nat + nbt + 4 ? slot_row(x, nat, a0, b0, na, nb, &fb) : -1;
      if (g >= 0) {
        cur.key[x] = R.key[q];
        cur.val[x] = R.val[q];
        cur.ts[x] = R.ts[q];
        cur.node[x] = R.node[q];
        cur.cnt[x] = R.cnt[q];
      }
    }
    __syncthreads();
    JSTAMP(t, 2);
    // ---- prefetch the next tile while this one is merged
    if (tn < ntiles) prefetch(tn, a0n, a1n);

    // ---- per-thread merge of JI positions
    u32 keep;
    unsigned short src[JI];
    merge_items<FAST, !FAST>(p.ca, p.cb, va, vb, p.keys, p.n_keys, nb, cur, nat, nbt, a0, b0, keep,
                             src, t);
    JSTAMP(t, 3);

    // ---- compaction list + aggregate of tile t
    u32 tile_total;
    u32 pos = block_excl_scan<JB>(__popc(keep), s.wave, &tile_total);
#pragma unroll
    for (int q = 0; q < JI; q++)
      if (keep & (1u << q)) cur.comp[pos++] = src[q];
    if (tid == 0) {
      lb_publish(p.scan.state, t, p.scan.epoch, t == 0 ? LB_INC : LB_AGG, tile_total);
      if (tn < ntiles) {  // the ticket after next (taken at the top of this iteration)
        s.bcast[3] = t2;
        if (t2 < ntiles) {
          s.bcast[4] = p.splits[t2];
          s.bcast[5] = p.splits[t2 + 1];
        }
      }
    }
    __syncthreads();
    JSTAMP(t, 4);
    // ---- the previous tile: its predecessors' aggregates are out by now
    if (pending) flush(pbuf);
    pending = true;
    tp = t;
    np = tile_total;
    pbuf = cb_;
    JSTAMP(t, 6);
    if (tn >= ntiles) break;
    t = tn;
    a0 = a0n;
    a1 = a1n;
    __syncthreads();  // flushed buffer free; next ticket visible
    tn = s.bcast[3];
    a0n = s.bcast[4];
    a1n = s.bcast[5];
  }
  __syncthreads();
  flush(pbuf);
}

// ---------------------------------------------------------------- two-pass join
// Pass 1: one workgroup per tile (no inter-workgroup dependency at all): stage, merge,
// and write the tile's compacted rows to its own slot of a scratch store + its count.
// Pass 2: each workgroup sums the counts before its tile and moves the slot's rows to
// the output.  (The persistent single-pass kernel above trades the extra pass for a
// decoupled look-back; DG_JOIN_MODE selects between them.)
struct SlotLds {
  Buf buf;
  u32 wave[JB / WAVE + 1];
  u64 vv_cnt[2][SMALL_VV];
  u32 vv_node[2][SMALL_VV];
};

struct SlotArgs {
  Rows a, b;
  Ctx ca, cb;
  const u64* keys;
  u64 n_keys;
  const u64* splits;
  unsigned short* lists;  // tile t's compaction list (staging slots) at lists[t * JT ...]
  u32* counts;            // kept rows per tile
};

template <bool FAST>
__global__ __launch_bounds__(JB) void join2_slot_kernel(SlotArgs p) {
  __shared__ SlotLds s;
  const int tid = threadIdx.x;
  const u64 na = p.a.n, nb = p.b.n, total = na + nb;
  const u64 t = blockIdx.x;
  if (FAST && tid < SMALL_VV) {
    s.vv_node[0][tid] = (u64)tid < p.ca.n ? p.ca.node[tid] : 0u;
    s.vv_cnt[0][tid] = (u64)tid < p.ca.n ? p.ca.cnt[tid] : 0ull;
    s.vv_node[1][tid] = (u64)tid < p.cb.n ? p.cb.node[tid] : 0u;
    s.vv_cnt[1][tid] = (u64)tid < p.cb.n ? p.cb.cnt[tid] : 0ull;
  }
  const SmallVV va{s.vv_node[0], s.vv_cnt[0], (u32)p.ca.n};
  const SmallVV vb{s.vv_node[1], s.vv_cnt[1], (u32)p.cb.n};
  const u64 a0 = p.splits[t], a1 = p.splits[t + 1];
  const u64 d0 = t * JT, d1 = min(d0 + (u64)JT, total);
  const int nat = (int)(a1 - a0), nbt = (int)((d1 - a1) - (d0 - a0));
  const u64 b0 = d0 - a0;
  Buf& cur = s.buf;
  JSTAMP(t, 0);
  // ---- stage a[a0-1 .. a1] and b[b0-1 .. b1] in LDS
  for (int x = tid; x < nat + nbt + 4; x += JB) {
    bool fb;
    const i64 g = slot_row(x, nat, a0, b0, na, nb, &fb);
    if (g >= 0) {
      const Rows& src = fb ? p.b : p.a;
      cur.key[x] = src.key[g];
      cur.val[x] = src.val[g];
      cur.ts[x] = src.ts[g];
      cur.node[x] = src.node[g];
      cur.cnt[x] = src.cnt[g];
    }
  }
  __syncthreads();
  JSTAMP(t, 2);
  u32 keep;
  unsigned short src[JI];
  merge_items<FAST, !FAST>(p.ca, p.cb, va, vb, p.keys, p.n_keys, nb, cur, nat, nbt, a0, b0, keep,
                           src, t);
  JSTAMP(t, 3);
  u32 tile_total;
  u32 pos = block_excl_scan<JB>(__popc(keep), s.wave, &tile_total);
#pragma unroll
  for (int q = 0; q < JI; q++)
    if (keep & (1u << q)) cur.comp[pos++] = src[q];
  if (tid == 0) p.counts[t] = tile_total;
  __syncthreads();
  JSTAMP(t, 4);
  for (u32 q = tid; q < tile_total; q += JB) p.lists[t * JT + q] = cur.comp[q];
#ifdef DG_STAMPS
  JSTAMP(t, 6);
#endif
}

constexpr int CPB = 256;

// Pass 2: tile t's prefix = Σ counts before it (summed by the workgroup itself), then
// every kept row is gathered from a or b through the tile's compaction list (slots of
// the pass-1 staging: slot x < nat + 2 is a[a0 - 1 + x], else b[b0 - 1 + x - nat - 2])
// and written to the output.  The rows were read by pass 1 just before, so the gathers
// mostly hit the Infinity Cache; the list is 2 bytes per kept row.
__global__ __launch_bounds__(CPB) void join2_compact_kernel(Rows a, Rows b, const u64* splits,
                                                            const unsigned short* lists,
                                                            const u32* counts, u64 ntiles,
                                                            RowsOut out, u64* d_count) {
  __shared__ u32 s_wave[CPB / WAVE + 1];
  __shared__ u64 s_pre;
  const u64 tile = blockIdx.x;
  u64 part = 0;
  for (u64 i = threadIdx.x; i < tile; i += CPB) part += counts[i];
#pragma unroll
  for (int d = WAVE / 2; d >= 1; d >>= 1) part += __shfl_xor(part, d, WAVE);
  if ((threadIdx.x & (WAVE - 1)) == 0) s_wave[threadIdx.x / WAVE] = (u32)part;
  __syncthreads();
  if (threadIdx.x == 0) {
    u64 acc = 0;
    for (int w = 0; w < CPB / WAVE; w++) acc += s_wave[w];
    s_pre = acc;
    if (tile == ntiles - 1) d_count[0] = acc + counts[tile];
  }
  __syncthreads();
  const u64 total = a.n + b.n;
  const u64 a0 = splits[tile], a1 = splits[tile + 1];
  const u64 d0 = tile * JT;
  const int nat = (int)(a1 - a0);
  const u64 b0 = d0 - a0;
  const u64 base = s_pre, n = counts[tile];
  (void)total;
  for (u64 q = threadIdx.x; q < n; q += CPB) {
    const int x = lists[tile * JT + q];
    const bool fb = x >= nat + 2;
    const u64 g = fb ? b0 - 1 + (u64)(x - nat - 2) : a0 - 1 + (u64)x;
    const Rows& src = fb ? b : a;
    out.key[base + q] = src.key[g];
    out.val[base + q] = src.val[g];
    out.ts[base + q] = src.ts[g];
    out.node[base + q] = src.node[g];
    out.cnt[base + q] = src.cnt[g];
  }
}

}  // namespace

static CtxUnionArgs make_cu(const Ctx& a, const Ctx& b, u32* out_node, u64* out_cnt,
                            u64* d_count, void* tmp) {
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

hipError_t launch_join2(const Rows& a, const Ctx& ca, const Rows& b, const Ctx& cb,
                        const u64* keys, u64 n_keys, const RowsOut& out, u32* out_ctx_node,
                        u64* out_ctx_cnt, void* ctx_tmp, void* pass_tmp, int mode,
                        const Scan& scan, int workers, u64* d_counts, hipStream_t st) {
  JoinArgs p;
  p.a = a;
  p.b = b;
  p.ca = ca;
  p.cb = cb;
  p.keys = keys;
  p.n_keys = n_keys;
  p.ntiles = join2_tiles(a.n, b.n);
  p.splits = scan.state + p.ntiles;  // look-back granules first, then the splits
  const CtxUnionArgs cu = make_cu(ca, cb, out_ctx_node, out_ctx_cnt, d_counts + 1, ctx_tmp);
  p.out = out;
  p.scan = scan;
  p.d_count = d_counts;
  if (p.ntiles == 0) {
    // no rows: only the context union runs
    hipError_t e = hipMemsetAsync(d_counts, 0, sizeof(u64), st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(ctx_union_kernel, dim3(1), dim3(CB), 0, st, cu);
    return hipGetLastError();
  }
  // 1) merge-path partition (+1 workgroup for the context union), 2) persistent tile
  // workers: merge, decoupled look-back one tile late, direct output writes
  const u64 nb_part = (p.ntiles + 1 + (PB / WAVE) - 1) / (PB / WAVE);
  hipLaunchKernelGGL(join2_partition_kernel, dim3((unsigned)nb_part + 1), dim3(PB), 0, st, a, b,
                     p.ntiles, p.splits, cu);
  const bool fast = keys == nullptr && ca.kind == 0 && cb.kind == 0 && ca.n <= (u64)SMALL_VV &&
                    cb.n <= (u64)SMALL_VV;
  if (mode == JOIN_TWO_PASS) {
    SlotArgs q;
    q.a = a;
    q.b = b;
    q.ca = ca;
    q.cb = cb;
    q.keys = keys;
    q.n_keys = n_keys;
    q.splits = p.splits;
    char* t = (char*)pass_tmp;
    q.counts = (u32*)t;
    t += ((p.ntiles * 4 + 255) / 256) * 256;
    q.lists = (unsigned short*)t;
    if (fast)
      hipLaunchKernelGGL(join2_slot_kernel<true>, dim3((unsigned)p.ntiles), dim3(JB), 0, st, q);
    else
      hipLaunchKernelGGL(join2_slot_kernel<false>, dim3((unsigned)p.ntiles), dim3(JB), 0, st, q);
    hipLaunchKernelGGL(join2_compact_kernel, dim3((unsigned)p.ntiles), dim3(CPB), 0, st, a, b,
                       q.splits, q.lists, q.counts, p.ntiles, out, d_counts);
    return hipGetLastError();
  }
  const u64 g = std::min<u64>(p.ntiles, (u64)(workers > 0 ? workers : 512));
  if (fast)
    hipLaunchKernelGGL(join2_tiles_kernel<true>, dim3((unsigned)g), dim3(JB), 0, st, p);
  else
    hipLaunchKernelGGL(join2_tiles_kernel<false>, dim3((unsigned)g), dim3(JB), 0, st, p);
  return hipGetLastError();
}

hipError_t launch_ctx_union(const Ctx& a, const Ctx& b, u32* out_node, u64* out_cnt,
                            u64* d_count, void* tmp, hipStream_t st) {
  CtxUnionArgs p = make_cu(a, b, out_node, out_cnt, d_count, tmp);
  hipLaunchKernelGGL(ctx_union_kernel, dim3(1), dim3(CB), 0, st, p);
  return hipGetLastError();
}

#ifdef DG_STAMPS
extern "C" int dg_debug_join_stamps(unsigned long long* host, size_t n) {
  if (n > 65536 * 8) n = 65536 * 8;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_join_stamps), n * 8) == hipSuccess ? 0 : -3;
}
#endif

}  // namespace dg
