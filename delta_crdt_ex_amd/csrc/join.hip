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
// Kernel shape (HBM-bound integer merge; no MFMA):
//   1. join2_partition_kernel: one wave per tile boundary finds the merge-path split
//      of diagonal q*JT.  Key ids are 64-bit hashes, so two interpolation probes on
//      the key columns land within a few rows of the split and one 128-wide window
//      round finishes it (~5 cache lines per array instead of a 21-step search); any
//      key distribution stays exact through a 128-ary fallback search.  One extra
//      workgroup computes the context union Dots.union(c1, c2) (:155).
//   2. join2_main_kernel (single pass): one workgroup per tile of JT merged
//      positions, numbered by an atomic ticket (launch order, so the look-back only
//      waits on resident tiles).  Every lane issues all of its row loads before the
//      first LDS write; each thread merges JI positions from LDS and decides
//      keep/drop; a block scan builds the compaction list; the tile publishes its
//      count, resolves its output offset with a block-wide decoupled look-back and
//      writes its kept rows coalesced.  Inputs are read once and outputs written
//      once: 36 B x (N_in + N_out) of HBM traffic plus the partition's probes.
//   (join2_slot_kernel + join2_compact_kernel: the two-pass variant, selected with
//    DG_JOIN_MODE=2, kept for A/B measurement.)
//
// Coverage (Dots.member?, :67-73) of a full-state join of two version vectors goes
// through a direct-indexed LDS table of the VVs' counters for node ids < VT (one
// ds_read per row); larger node ids and explicit dot sets use a binary search.
#include <algorithm>

#include "dg_launch.h"

namespace dg {

namespace {

constexpr int JB = JOIN_BLOCK;
constexpr int JI = JOIN_ITEMS;
constexpr int JT = JOIN_TILE;
constexpr int JS = JT + 5;  // LDS row slots: tile rows + one neighbour on each side per store
                            // (+1: the merge's look-ahead read past the last B slot)
#ifndef DG_JOIN_PIPE
#define DG_JOIN_PIPE 0
#endif
constexpr bool JOIN_PIPE = DG_JOIN_PIPE;  // pass 1: persistent, next tile prefetched in registers
constexpr int VT = 128;     // VV table: node ids below this are looked up directly in LDS

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
  const u64* splits;  // merge-path split (a index) of every tile boundary (partition pass)
  u64 ntiles;
  RowsOut out;
  Scan scan;  // look-back granules + tile tickets
  u64* d_count;
  unsigned short* lists;  // two-pass only: tile t's compaction list at lists[t * JT ...]
  u32* counts;            // two-pass only: kept rows per tile
};

// ------------------------------------------------------------------ partition
// Merge-path predicate on diagonal `diag` over global memory: A[i] <= B[diag-1-i]
// (ties go to A).  Full rows are only loaded when the keys tie.
__device__ __forceinline__ bool mp_pred(const Rows A, const Rows B, u64 diag, u64 i) {
  u64 j = diag - 1 - i;
  u64 ka = A.key[i], kb = B.key[j];
  if (ka != kb) return ka < kb;
  return row_le(load_row(A, i), load_row(B, j));
}

constexpr int PB = 256;      // threads per partition block = 4 boundaries
constexpr int PK = 2 * WAVE;  // samples per search round (two per lane)

// One wave: first i in [lo, hi) with NOT mp_pred(i) (hi if none) by a 128-ary search.
__device__ u64 mp_search(const Rows A, const Rows B, u64 d, u64 lo, u64 hi) {
  const int lane = threadIdx.x & (WAVE - 1);
  for (int round = 0; round < 64 && hi > lo; round++) {
    const u64 span = hi - lo;
    bool f0, f1;  // lane l evaluates samples 2l and 2l+1
    if (span <= (u64)PK) {
      const u64 x0 = lo + 2 * lane, x1 = x0 + 1;
      f0 = x0 < hi && !mp_pred(A, B, d, x0);
      f1 = x1 < hi && !mp_pred(A, B, d, x1);
    } else {
      const u64 x0 = lo + (span * (u64)(2 * lane + 1)) / (PK + 1);
      const u64 x1 = lo + (span * (u64)(2 * lane + 2)) / (PK + 1);
      f0 = !mp_pred(A, B, d, x0);
      f1 = !mp_pred(A, B, d, x1);
    }
    const u64 m0 = __ballot(f0), m1 = __ballot(f1);
    int kf = PK;  // first false sample
    if (m0 | m1) {
      const int l0 = m0 ? __ffsll((long long)m0) - 1 : 64;
      const int l1 = m1 ? __ffsll((long long)m1) - 1 : 64;
      kf = (l0 <= l1) ? 2 * l0 : 2 * l1 + 1;
    }
    if (span <= (u64)PK) {
      return (u64)kf < span ? lo + kf : hi;
    } else if (kf == PK) {
      lo = lo + (span * (u64)PK) / (PK + 1) + 1;
    } else {
      const u64 nh = lo + (span * (u64)(kf + 1)) / (PK + 1);
      if (kf > 0) lo = lo + (span * (u64)kf) / (PK + 1) + 1;
      hi = nh;
    }
  }
  return lo;
}

// Merge-path split of diagonal d (= #A rows among the first d merged rows).
// Interpolation: at a guess i the key gap B.key[d-1-i] - A.key[i] (in units of the
// 2^64 key space) converts to a row shift of gap * na*nb / ((na+nb) * 2^64); two
// such probes (wave-uniform loads) put the guess within a few rows of the split for
// hashed keys, then ONE window of 128 consecutive candidates decides it.  If the
// split is not bracketed by the window, the exact 128-ary search runs instead.
__device__ u64 mp_split(const Rows A, const Rows B, u64 d) {
  const int lane = threadIdx.x & (WAVE - 1);
  const u64 na = A.n, nb = B.n, total = na + nb;
  const u64 lo = d > nb ? d - nb : 0, hi = min(d, na);
  if (hi - lo <= (u64)PK) return mp_search(A, B, d, lo, hi);
  const double scale = (double)na * (double)nb / ((double)total * 18446744073709551616.0);
  u64 i = (u64)((double)d * (double)na / (double)total);
  i = min(max(i, lo), hi - 1);
#pragma unroll
  for (int r = 0; r < 2; r++) {
    const double gap = (double)B.key[d - 1 - i] - (double)A.key[i];
    double s = gap * scale;
    const double lim = (double)(hi - lo);
    s = s > lim ? lim : (s < -lim ? -lim : s);
    const i64 si = (i64)s;
    i64 ni = (i64)i + si;
    ni = ni < (i64)lo ? (i64)lo : (ni > (i64)hi - 1 ? (i64)hi - 1 : ni);
    i = (u64)ni;
  }
  u64 wlo = i > lo + PK / 2 ? i - PK / 2 : lo;
  const u64 whi = min(wlo + (u64)PK, hi);
  wlo = whi - PK > lo ? whi - PK : lo;
  const u64 x0 = wlo + 2 * lane, x1 = x0 + 1;
  const bool f0 = x0 < whi && !mp_pred(A, B, d, x0);
  const bool f1 = x1 < whi && !mp_pred(A, B, d, x1);
  const u64 m0 = __ballot(f0), m1 = __ballot(f1);
  u64 kf = whi - wlo;  // first false candidate in the window (none: whi - wlo)
  if (m0 | m1) {
    const int l0 = m0 ? __ffsll((long long)m0) - 1 : 64;
    const int l1 = m1 ? __ffsll((long long)m1) - 1 : 64;
    kf = (l0 <= l1) ? 2 * l0 : 2 * l1 + 1;
  }
  // bracketed iff the first false is not at the window's low edge (unless that edge is
  // lo) and some candidate is false (unless the window reaches hi)
  const bool ok = (kf > 0 || wlo == lo) && (kf < whi - wlo || whi == hi);
  if (ok) return wlo + kf;
  return mp_search(A, B, d, lo, hi);
}

__global__ __launch_bounds__(PB) void join2_partition_kernel(Rows A, Rows B, u64 ntiles,
                                                             u64* splits, CtxUnionArgs cu) {
  if (blockIdx.x == gridDim.x - 1) {  // extra workgroup: Dots.union(c1, c2) (aw_lww_map.ex:155)
    __shared__ u32 s_wave[PB / WAVE + 1];
    ctx_union_block<PB>(cu, s_wave);
    return;
  }
  const u64 q = (u64)blockIdx.x * (PB / WAVE) + (threadIdx.x >> 6);
  if (q > ntiles) return;
  const u64 d = min(q * (u64)JT, A.n + B.n);
  const u64 s = mp_split(A, B, d);
  if ((threadIdx.x & (WAVE - 1)) == 0) splits[q] = s;
}

// ------------------------------------------------------------------- coverage
// Dots.member?(c, {dn, dc}) (aw_lww_map.ex:67-73).  For a full-state join of two
// version vectors (FAST) the counters of nodes < VT sit in a direct-indexed LDS
// table (Map.get(vv, node, 0) is table[node], absent nodes hold 0); node ids >= VT
// fall back to a binary search of the VV in global memory.
template <bool FAST>
__device__ __forceinline__ bool covers(const u64* tab, const Ctx& c, u32 dn, u64 dc) {
  if (FAST) {
    if (dn < (u32)VT) return tab[dn] >= dc;
    return ctx_covers(c.node, c.cnt, c.n, 0, dn, dc);
  }
  return ctx_covers(c.node, c.cnt, c.n, c.kind, dn, dc);
}

// Map.get(vv, want, 0) by binary search of a VV in global memory.
__device__ __noinline__ u64 vv_get(const u32* node, const u64* cnt, u64 n, u32 want) {
  u64 lo = 0, hi = n;
  while (lo < hi) {
    const u64 m = (lo + hi) >> 1;
    if (node[m] < want)
      lo = m + 1;
    else
      hi = m;
  }
  return (lo < n && node[lo] == want) ? cnt[lo] : 0ull;
}

// Fill the two VV tables (threads of the block; tables zeroed by the caller and a
// barrier in between).
__device__ __forceinline__ void fill_vv_tables(const Ctx& ca, const Ctx& cb, u64* tab_a, u64* tab_b) {
  for (u64 i = threadIdx.x; i < ca.n; i += blockDim.x)
    if (ca.node[i] < (u32)VT) tab_a[ca.node[i]] = ca.cnt[i];
  for (u64 i = threadIdx.x; i < cb.n; i += blockDim.x)
    if (cb.node[i] < (u32)VT) tab_b[cb.node[i]] = cb.cnt[i];
}

// ------------------------------------------------------------------- staging
// One staged tile: its rows (+ one neighbour on each side of each store).
struct Buf {
  u64 key[JS];
  u64 val[JS];
  u64 cnt[JS];
  i64 ts[JS];
  u32 node[JS];
};

// Global row index of staging slot x, or -1 if the slot is outside the stores:
// slot x < nat + 2 is a[a0 - 1 + x], slot x >= nat + 2 is b[b0 - 1 + (x - nat - 2)].
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

constexpr int SLOTS = (JS + JB - 1) / JB;

// Stage the tile's rows in LDS.  Every lane issues the loads of all its slots before
// the first LDS write, so the whole tile is in flight at once (one HBM round trip).
__device__ __forceinline__ void stage_tile(const Rows& A, const Rows& B, int nat, int nbt, u64 a0,
                                           u64 b0, Buf& s) {
  const int tid = threadIdx.x;
  u64 rk[SLOTS], rv[SLOTS], rc[SLOTS];
  i64 rt[SLOTS];
  u32 rn[SLOTS];
  bool ok[SLOTS];
#pragma unroll
  for (int k = 0; k < SLOTS; k++) {
    const int x = tid + k * JB;
    bool fb = false;
    const i64 g = x < nat + nbt + 4 ? slot_row(x, nat, a0, b0, A.n, B.n, &fb) : -1;
    ok[k] = g >= 0;
    if (ok[k]) {
      const Row x = load_row_sel(A, B, fb, (u64)g);
      rk[k] = x.key;
      rv[k] = x.val;
      rt[k] = x.ts;
      rn[k] = x.node;
      rc[k] = x.cnt;
    }
  }
#pragma unroll
  for (int k = 0; k < SLOTS; k++) {
    const int x = tid + k * JB;
    if (ok[k]) {
      s.key[x] = rk[k];
      s.val[x] = rv[k];
      s.ts[x] = rt[k];
      s.node[x] = rn[k];
      s.cnt[x] = rc[k];
    }
  }
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
template <bool FAST>
__device__ __forceinline__ void merge_items(const Ctx& ca, const Ctx& cb, const u64* tab_a,
                                            const u64* tab_b, const u64* keys, const u64 n_keys,
                                            const u64 nb, const Buf& s, int nat, int nbt, u64 a0,
                                            u64 b0, u32& keep, unsigned short (&src)[JI]) {
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
  // ra = a[i], rb = b[j] (possibly the neighbour past the tile), pa = a[i-1]; xa / xb are
  // the rows after them, read one step ahead so no merge step waits on LDS.  (Reads past
  // a side's end land in other slots of the buffer and are never used.)
  Row ra = lds_row(s, 1 + i), rb = lds_row(s, offB + 1 + j), pa = lds_row(s, i);
  Row xa = lds_row(s, 2 + i), xb = lds_row(s, offB + 2 + j);
  keep = 0;
#pragma unroll
  for (int k = 0; k < JI; k++) {
    src[k] = 0;
    if (diag + k < dend) {
      const bool bvalid = (b0 + (u64)j) < nb;  // b[j] exists globally
      const bool takeA = i < nat && (j >= nbt || row_le(ra, rb));
      bool kp;
      if (takeA) {
        const bool joined = FAST || keys == nullptr || keyset_has(keys, n_keys, ra.key);
        if (joined) {
          const bool inB = bvalid && row_eq(ra, rb);
          kp = inB || !covers<FAST>(tab_b, cb, ra.node, ra.cnt);
        } else {
          // Map.merge(Map.drop(a), Map.drop(b)): a's rows survive iff b lacks the key
          const bool bprev = (b0 + (u64)j) >= 1 && s.key[offB + j] == ra.key;
          const bool bnext = bvalid && rb.key == ra.key;
          kp = !(bprev || bnext);
        }
        src[k] = (unsigned short)(1 + i);
        i++;
        pa = ra;
        ra = xa;
        if (k + 1 < JI) xa = lds_row(s, 2 + i);
      } else {
        const bool joined = FAST || keys == nullptr || keyset_has(keys, n_keys, rb.key);
        if (joined) {
          const bool dupA = (a0 + (u64)i) >= 1 && row_eq(pa, rb);
          kp = !dupA && !covers<FAST>(tab_a, ca, rb.node, rb.cnt);
        } else {
          kp = true;
        }
        src[k] = (unsigned short)(offB + 1 + j);
        j++;
        rb = xb;
        if (k + 1 < JI) xb = lds_row(s, offB + 2 + j);
      }
      if (kp) keep |= 1u << k;
    }
  }
}

// LDS of one join workgroup.  The VV tables are only read by the merge and the
// compaction list is only written after it (behind the block scan's barriers), so
// they share storage: the tile stays at 4 workgroups per CU.
struct TileLds {
  Buf buf;
  union {
    u64 tab[2][VT];
    unsigned short comp[JT];
  } u;
  u32 wave[JB / WAVE + 1];
  u64 lb[3 * (JB / WAVE) + 2];
  u64 bcast[4];
};

// Common front half of a tile: stage, merge, block scan -> compaction list in LDS.
// Returns the tile's kept-row count.
template <bool FAST>
__device__ __forceinline__ u32 tile_merge(const JoinArgs& p, TileLds& s, u64 t, u64 a0, u64 a1) {
  const int tid = threadIdx.x;
  const u64 na = p.a.n, nb = p.b.n, total = na + nb;
  const u64 d0 = t * JT, d1 = min(d0 + (u64)JT, total);
  const int nat = (int)(a1 - a0), nbt = (int)((d1 - a1) - (d0 - a0));
  const u64 b0 = d0 - a0;
  if (FAST) fill_vv_tables(p.ca, p.cb, s.u.tab[0], s.u.tab[1]);
  JSTAMP(t, 1);
  stage_tile(p.a, p.b, nat, nbt, a0, b0, s.buf);
  __syncthreads();
  JSTAMP(t, 2);
  u32 keep;
  unsigned short src[JI];
  merge_items<FAST>(p.ca, p.cb, s.u.tab[0], s.u.tab[1], p.keys, p.n_keys, nb, s.buf, nat, nbt, a0,
                    b0, keep, src);
  JSTAMP(t, 3);
  u32 tile_total;
  u32 pos = block_excl_scan<JB>(__popc(keep), s.wave, &tile_total);  // barriers: tables dead
#pragma unroll
  for (int q = 0; q < JI; q++)
    if (keep & (1u << q)) s.u.comp[pos++] = src[q];
  __syncthreads();
  JSTAMP(t, 4);
  return tile_total;
}

// Single-pass join: one workgroup per tile (see the file header).
template <bool FAST>
__global__ __launch_bounds__(JB) void join2_main_kernel(JoinArgs p) {
  __shared__ TileLds s;
  const int tid = threadIdx.x;
  const u64 ntiles = p.ntiles;
  if (FAST)
    for (int x = tid; x < 2 * VT; x += JB) (&s.u.tab[0][0])[x] = 0;
  if (tid == 0) {
    // The ticket numbers tiles in dispatch order; the splits of tile blockIdx.x are
    // loaded speculatively beside it (the ticket almost always equals blockIdx.x).
    const u64 tk = atomicAdd(p.scan.ticket, 1u);
    const u64 g = blockIdx.x;
    u64 s0 = p.splits[g], s1 = p.splits[g + 1];
    if (tk == ntiles - 1) atomicExch(p.scan.ticket, 0u);
    if (tk != g) {
      s0 = p.splits[tk];
      s1 = p.splits[tk + 1];
    }
    s.bcast[0] = tk;
    s.bcast[1] = s0;
    s.bcast[2] = s1;
  }
  __syncthreads();
  const u64 t = s.bcast[0], a0 = s.bcast[1], a1 = s.bcast[2];
  JSTAMP(t, 0);
  const u32 n = tile_merge<FAST>(p, s, t, a0, a1);
  u64 prefix = 0;
  if (t == 0) {
    if (tid == 0) lb_publish(p.scan.state, 0, p.scan.epoch, LB_INC, n);
  } else {
    if (tid == 0) lb_publish(p.scan.state, t, p.scan.epoch, LB_AGG, n);
    prefix = lb_lookback_block<JB, 2>(p.scan.state, t, p.scan.epoch, p.scan.err, s.lb);
    if (tid == 0) lb_publish(p.scan.state, t, p.scan.epoch, LB_INC, prefix + n);
  }
  if (tid == 0 && t == ntiles - 1) p.d_count[0] = prefix + n;
  JSTAMP(t, 5);
  const Buf& b = s.buf;
  for (u32 q = tid; q < n; q += JB) {
    const int slot = s.u.comp[q];
    const u64 o = prefix + q;
    p.out.key[o] = b.key[slot];
    p.out.val[o] = b.val[slot];
    p.out.ts[o] = b.ts[slot];
    p.out.node[o] = b.node[slot];
    p.out.cnt[o] = b.cnt[slot];
  }
  JSTAMP(t, 6);
}

// ---------------------------------------------------------------- two-pass join
// Pass 1 (join2_slot_kernel): persistent workgroups, each merging tiles blockIdx.x,
// blockIdx.x + gridDim.x, ...  While tile t is merged from LDS, the rows of the next
// tile are already in flight into registers (issued right after t was committed to
// LDS), so HBM streams through the merge instead of stalling each tile on its own
// loads.  The VV tables are loaded once per workgroup and kept in registers.  Output
// per tile: its kept-row count and its compaction list (LDS slot numbers, u16).
// Pass 2 (join2_compact_kernel): each workgroup sums the counts before its tile and
// gathers the kept rows from a/b into the output.  No inter-workgroup dependency in
// either pass.
struct Staged {  // one thread's share of a staged tile, in registers
  u64 k[SLOTS], v[SLOTS], c[SLOTS];
  i64 t[SLOTS];
  u32 n[SLOTS];
  bool ok[SLOTS];
};

__device__ __forceinline__ void tile_geom(u64 t, u64 a0, u64 a1, u64 total, int* nat, int* nbt,
                                          u64* b0) {
  const u64 d0 = t * JT, d1 = min(d0 + (u64)JT, total);
  *nat = (int)(a1 - a0);
  *nbt = (int)((d1 - a1) - (d0 - a0));
  *b0 = d0 - a0;
}

__device__ __forceinline__ void issue_tile(const Rows& A, const Rows& B, int nat, int nbt, u64 a0,
                                           u64 b0, Staged& r) {
  const int tid = threadIdx.x;
#pragma unroll
  for (int k = 0; k < SLOTS; k++) {
    const int x = tid + k * JB;
    bool fb = false;
    const i64 g = x < nat + nbt + 4 ? slot_row(x, nat, a0, b0, A.n, B.n, &fb) : -1;
    r.ok[k] = g >= 0;
    if (r.ok[k]) {
      const Row x = load_row_sel(A, B, fb, (u64)g);
      r.k[k] = x.key;
      r.v[k] = x.val;
      r.t[k] = x.ts;
      r.n[k] = x.node;
      r.c[k] = x.cnt;
    }
  }
}

__device__ __forceinline__ void commit_tile(const Staged& r, Buf& s) {
  const int tid = threadIdx.x;
#pragma unroll
  for (int k = 0; k < SLOTS; k++) {
    const int x = tid + k * JB;
    if (r.ok[k]) {
      s.key[x] = r.k[k];
      s.val[x] = r.v[k];
      s.ts[x] = r.t[k];
      s.node[x] = r.n[k];
      s.cnt[x] = r.c[k];
    }
  }
}

template <bool FAST>
__global__ __launch_bounds__(JB) void join2_slot_kernel(JoinArgs p) {
  __shared__ TileLds s;
  const int tid = threadIdx.x;
  const u64 total = p.a.n + p.b.n, ntiles = p.ntiles, G = gridDim.x;
  // this thread's VV-table entries x = tid + q*JB < 2*VT: Map.get(vv, x % VT, 0)
  constexpr int TQ = (2 * VT + JB - 1) / JB;
  u64 tab_entry[TQ];
#pragma unroll
  for (int q = 0; q < TQ; q++) {
    const int x = tid + q * JB;
    tab_entry[q] = 0;
    if (FAST) {
      if (x < VT)
        tab_entry[q] = vv_get(p.ca.node, p.ca.cnt, p.ca.n, (u32)x);
      else if (x < 2 * VT)
        tab_entry[q] = vv_get(p.cb.node, p.cb.cnt, p.cb.n, (u32)(x - VT));
    }
  }
  const Rows& A = p.a;
  const Rows& B = p.b;
  u64 t = blockIdx.x;
  u64 a0 = p.splits[t], a1 = p.splits[t + 1];
  int nat, nbt;
  u64 b0;
  tile_geom(t, a0, a1, total, &nat, &nbt, &b0);
  Staged r;
  issue_tile(A, B, nat, nbt, a0, b0, r);
  while (true) {
    JSTAMP(t, 0);
    JSTAMP(t, 1);
    commit_tile(r, s.buf);
#pragma unroll
    for (int q = 0; q < TQ; q++)
      if (FAST && tid + q * JB < 2 * VT) (&s.u.tab[0][0])[tid + q * JB] = tab_entry[q];
    __syncthreads();
    JSTAMP(t, 2);
    // prefetch the next tile while this one is merged
    const u64 tn = JOIN_PIPE ? t + G : ntiles;
    u64 a0n = 0, a1n = 0, b0n = 0;
    int natn = 0, nbtn = 0;
    if (JOIN_PIPE && tn < ntiles) {
      a0n = p.splits[tn];
      a1n = p.splits[tn + 1];
      tile_geom(tn, a0n, a1n, total, &natn, &nbtn, &b0n);
      issue_tile(A, B, natn, nbtn, a0n, b0n, r);
    }
    u32 keep;
    unsigned short src[JI];
    merge_items<FAST>(p.ca, p.cb, s.u.tab[0], s.u.tab[1], p.keys, p.n_keys, p.b.n, s.buf, nat,
                      nbt, a0, b0, keep, src);
    JSTAMP(t, 3);
    u32 n;
    u32 pos = block_excl_scan<JB>(__popc(keep), s.wave, &n);  // barriers: tables dead
#pragma unroll
    for (int q = 0; q < JI; q++)
      if (keep & (1u << q)) s.u.comp[pos++] = src[q];
    __syncthreads();
    JSTAMP(t, 4);
    JSTAMP(t, 5);
    if (tid == 0) p.counts[t] = n;
    for (u32 q = tid; q < n; q += JB) p.lists[t * JT + q] = s.u.comp[q];
    JSTAMP(t, 6);
    if (tn >= ntiles) break;
    __syncthreads();  // LDS tile and list free for the next commit
    t = tn;
    a0 = a0n;
    a1 = a1n;
    nat = natn;
    nbt = nbtn;
    b0 = b0n;
  }
}

constexpr int CPB = 256;
constexpr int CPU_ = 8;  // counts loaded per thread per batch in the compact prologue

__global__ __launch_bounds__(CPB) void join2_compact_kernel(Rows a, Rows b, const u64* splits,
                                                            const unsigned short* lists,
                                                            const u32* counts, u64 ntiles,
                                                            RowsOut out, u64* d_count) {
  __shared__ u32 s_wave[CPB / WAVE + 1];
  __shared__ u64 s_pre;
  const u64 tile = blockIdx.x;
  // Σ counts[0, tile): every load of a batch is issued before the first add
  u64 part = 0;
  for (u64 base = 0; base < tile; base += (u64)CPB * CPU_) {
    u32 v[CPU_];
#pragma unroll
    for (int k = 0; k < CPU_; k++) {
      const u64 i = base + (u64)k * CPB + threadIdx.x;
      v[k] = i < tile ? counts[i] : 0u;
    }
#pragma unroll
    for (int k = 0; k < CPU_; k++) part += v[k];
  }
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
  const u64 a0 = splits[tile], a1 = splits[tile + 1];
  const u64 d0 = tile * JT;
  const int nat = (int)(a1 - a0);
  const u64 b0 = d0 - a0;
  const u64 base = s_pre, n = counts[tile];
  for (u64 q = threadIdx.x; q < n; q += CPB) {
    const int x = lists[tile * JT + q];
    const bool fb = x >= nat + 2;
    const u64 g = fb ? b0 - 1 + (u64)(x - nat - 2) : a0 - 1 + (u64)x;
    const Row r = load_row_sel(a, b, fb, g);
    out.key[base + q] = r.key;
    out.val[base + q] = r.val;
    out.ts[base + q] = r.ts;
    out.node[base + q] = r.node;
    out.cnt[base + q] = r.cnt;
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
  u64* splits = scan.state + p.ntiles;  // look-back granules first, then the splits
  p.splits = splits;
  const CtxUnionArgs cu = make_cu(ca, cb, out_ctx_node, out_ctx_cnt, d_counts + 1, ctx_tmp);
  p.out = out;
  p.scan = scan;
  p.d_count = d_counts;
  p.lists = nullptr;
  p.counts = nullptr;
  if (p.ntiles == 0) {
    // no rows: only the context union runs
    hipError_t e = hipMemsetAsync(d_counts, 0, sizeof(u64), st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(ctx_union_kernel, dim3(1), dim3(CB), 0, st, cu);
    return hipGetLastError();
  }
  const u64 nb_part = (p.ntiles + 1 + (PB / WAVE) - 1) / (PB / WAVE);
  hipLaunchKernelGGL(join2_partition_kernel, dim3((unsigned)nb_part + 1), dim3(PB), 0, st, a, b,
                     p.ntiles, splits, cu);
  // full-state join of two version vectors: LDS VV table, no key list
  const bool fast = keys == nullptr && ca.kind == 0 && cb.kind == 0;
  if (mode == JOIN_TWO_PASS) {
    char* t = (char*)pass_tmp;
    p.counts = (u32*)t;
    t += ((p.ntiles * 4 + 255) / 256) * 256;
    p.lists = (unsigned short*)t;
    // persistent pass 1: as many workgroups as are resident at once (registers and
    // LDS per tile decide it), unless the caller fixed the count (workers > 0)
    auto kern = fast ? join2_slot_kernel<true> : join2_slot_kernel<false>;
    u64 g = workers > 0 ? (u64)workers : (JOIN_PIPE ? 0 : p.ntiles);
    if (!g) {
      int per_cu = 0, dev = 0, cus = 0;
      if (hipGetDevice(&dev) != hipSuccess ||
          hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
          hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, JB, 0) != hipSuccess ||
          per_cu <= 0 || cus <= 0)
        per_cu = 1, cus = 256;
      g = (u64)per_cu * (u64)cus;
    }
    g = std::min<u64>(p.ntiles, g);
    hipLaunchKernelGGL(kern, dim3((unsigned)g), dim3(JB), 0, st, p);
    hipLaunchKernelGGL(join2_compact_kernel, dim3((unsigned)p.ntiles), dim3(CPB), 0, st, a, b,
                       p.splits, p.lists, p.counts, p.ntiles, out, d_counts);
    return hipGetLastError();
  }
  if (fast)
    hipLaunchKernelGGL(join2_main_kernel<true>, dim3((unsigned)p.ntiles), dim3(JB), 0, st, p);
  else
    hipLaunchKernelGGL(join2_main_kernel<false>, dim3((unsigned)p.ntiles), dim3(JB), 0, st, p);
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
