// small.hip — update_state_with_delta for a SMALL delta in one launch.
//
// CausalCrdt joins every local mutation and every small sync delta into the replica
// (reference causal_crdt.ex:337-342,383-394; aw_lww_map.ex:153-209).  The general
// dg_join_delta (api.hip) takes the keyset's rows out, joins them on the join kernels,
// splices, updates the tree and gathers the changed rows: four steps, each sized by the
// counts of the one before, so four host waits -- ~80 us for a one-key mutation of which
// the device work is a few.  Here ONE workgroup does the whole join of a delta of at most
// SMALL_KEYS keys and SMALL_DELTA rows whose keys' state rows number at most SMALL_TAKEN:
//
//   1. per key, its first state row (an interpolation search: key ids are hashes) and run;
//      the delta, the state's VV and the delta's context staged in LDS (the VVs as tables
//      indexed by node id: interned ids are dense)
//   2. the taken rows staged; every delta key checked to be a keyset key (else the
//      right-biased carry of :185-188 applies: the general path)
//   3. per key (one thread), join_dot_sets over its taken and delta rows (:196-209): a
//      row in both stays, a state row stays iff the delta's context does not cover its
//      dot, a delta row iff the state's does not (Dots.member?, :67-73); the key changed
//      iff a state row went or a delta row came (diff/3, causal_crdt.ex:344-352)
//   4. scans: the edit's offsets, the changed keys', their rows'; Dots.union of the
//      contexts (:39-52; a dot set folds into the VV by per-node max, LDS 64-bit max)
//   5. with a tree: per bucket (keys sorted => a bucket's keys adjacent) the leaf change
//      Σ row_hash(new) - Σ row_hash(old) and the row-count change, checked (65535 rows
//      per bucket, the tree's shard) BEFORE anything is written
//   6. writes: the edit's rows in place when no key's row count changed; else straight to
//      their places in the spare store with the per-key splice index (end, shift) that the
//      tail kernel's copy tiles search (merkle.hip small_tail_kernel: the state's other rows
//      into the spare), or -- a state of more than SMALL_COPY_TILES tiles -- as the edit
//      for the splice kernels after the wait; the union context, the bucket nodes, counts,
//      dirty chunks and chunk-index deltas (the tail kernel re-reduces the dirty chunks:
//      MerkleMap.update_hashes), and the result block.
// Anything outside the limits sets SMALL_FALLBACK before any write: the caller then runs
// the general path on the untouched state.
//
// Roofline: latency, not bandwidth -- a one-key op reads and writes a few hundred bytes;
// what it saves is three host round trips.
#include "dg_hash.h"
#include "dg_home.h"
#include "dg_launch.h"
#include "dg_tree.h"

namespace dg {

namespace {

constexpr int NT = 512;
constexpr u32 SK = SMALL_KEYS, SD = SMALL_DELTA, SC = SMALL_DCTX, SV = SMALL_NODES;
constexpr u32 SA = SMALL_TAKEN, SE = SMALL_EDIT;
static_assert(SK <= (u32)NT, "one thread per key");

struct SmallLds {
  u64 key[SK], alo[SK], leaf[SK];
  u32 na[SK], aoff[SK + 1], ne[SK], eoff[SK + 1], roff[SK], coff[SK];
  u64 dk[SD], dv[SD], dc[SD];
  i64 dt[SD];
  u32 dn[SD];
  u64 ak[SA], av[SA], ac[SA];
  i64 at[SA];
  u32 an[SA];
  u64 tabS[SV], tabU[SV];  // VVs by node id: counter + 1, 0 = absent
  union {
    u64 tabD[SV];  // the delta's VV
    struct {
      u64 c[SC];
      u32 n[SC];
    } dots;        // or its dot set, (node, cnt) ascending
  } cd;
  u64 pb[SK], pv[2][SK];  // the changed buckets (ascending), their nodes per level (two halves)
  int pp[SK + 1];         // their row-count changes' exclusive prefix
  u32 wave[NT / WAVE + 1];
  u32 w4[4 * (NT / WAVE)];
  u32 flags, moved, nctx;
  int dkeys;
};

__device__ __forceinline__ Row lds_a(const SmallLds& s, u32 i) {
  Row r;
  r.key = s.ak[i];
  r.val = s.av[i];
  r.ts = s.at[i];
  r.node = s.an[i];
  r.cnt = s.ac[i];
  return r;
}

__device__ __forceinline__ Row lds_d(const SmallLds& s, u32 i) {
  Row r;
  r.key = s.dk[i];
  r.val = s.dv[i];
  r.ts = s.dt[i];
  r.node = s.dn[i];
  r.cnt = s.dc[i];
  return r;
}

// Key k's first row in a[0, n) (ascending) and its run (at most SA + 1 counted), by the
// lanes of one wave: key ids are uniform hashes, so the first round probes 64 rows around
// the interpolated position (k / 2^64 of the way, 8 standard deviations wide); 64-ary
// rounds narrow [lo, hi] (hi INCLUSIVE: the first row >= k may be hi itself) to at most 64
// candidates (none at 10k rows, one at 10M), which one load per lane settles, run
// included: the window [lo, lo + 63] then holds hi, so a run starting at hi is seen (ADVICE
// r5: narrowing only to hi - lo <= 64 left a run starting at hi = lo + 64 counted as 0).
// Two round trips at 10k rows where a thread's interpolation search takes four or five.
__device__ __forceinline__ void wave_find(const u64* a, u64 n, u64 k, u64& lo_out, u32& run_out) {
  const int lane = threadIdx.x & (WAVE - 1);
  u64 lo = 0, hi = n;  // the first row >= k is in [lo, hi]
  if (n > (u64)WAVE) {
    const i64 g = (i64)__umul64hi(k, n);
    const i64 st = (i64)(8.0 * 0.5 * __builtin_sqrt((double)n) / WAVE) + 1;
    i64 qi = g + ((i64)lane - WAVE / 2) * st;
    qi = qi < 0 ? 0 : (qi > (i64)n - 1 ? (i64)n - 1 : qi);
    const u64 q = (u64)qi;
    const int c = __popcll(__ballot(a[q] < k));  // a prefix of the lanes (q ascending)
    const u64 qlo = __shfl(q, c > 0 ? c - 1 : 0, WAVE), qhi = __shfl(q, c < WAVE ? c : WAVE - 1, WAVE);
    if (c > 0) lo = qlo + 1;
    if (c < WAVE) hi = qhi;
    while (hi - lo >= (u64)WAVE) {  // [lo, hi] has more than WAVE candidates
      const u64 span = hi - lo;
      const u64 p = lo + span * (u64)(lane + 1) / (WAVE + 1);
      const int c2 = __popcll(__ballot(a[p] < k));
      const u64 nlo = c2 ? lo + span * (u64)c2 / (WAVE + 1) + 1 : lo;
      const u64 nhi = c2 < WAVE ? lo + span * (u64)(c2 + 1) / (WAVE + 1) : hi;
      lo = nlo;
      hi = nhi;
    }
  }
  const u64 x = lo + (u64)lane;
  const u64 v = x < n ? a[x] : 0ull;
  const u64 first = lo + (u64)__popcll(__ballot(x < n && v < k));
  const u64 eqm = __ballot(x < n && v == k);
  u32 run = (u32)__popcll(eqm);
  for (u64 e = lo + WAVE; (eqm >> (WAVE - 1)) & 1;) {  // the run goes on past the window
    if (run > SA) break;
    const u64 y = e + (u64)lane;
    const u64 m = __ballot(y < n && a[y] == k);
    run += (u32)__popcll(m);
    if (!((m >> (WAVE - 1)) & 1)) break;
    e += WAVE;
  }
  lo_out = first;
  run_out = run;
}

// Four exclusive block scans with ONE barrier: the wave totals to LDS, every thread adds
// up those of the waves before its own (ex: this thread's offsets, tot: the sums)
__device__ __forceinline__ void block_scan4(const u32 (&v)[4], u32* sw, u32 (&ex)[4], u32 (&tot)[4]) {
  constexpr int NW = NT / WAVE;
  const int lane = threadIdx.x & (WAVE - 1), w = threadIdx.x / WAVE;
  u32 inc[4];
#pragma unroll
  for (int j = 0; j < 4; j++) inc[j] = wave_incl_scan(v[j]);
  if (lane == WAVE - 1)
#pragma unroll
    for (int j = 0; j < 4; j++) sw[j * NW + w] = inc[j];
  __syncthreads();
#pragma unroll
  for (int j = 0; j < 4; j++) {
    u32 below = 0, t = 0;
#pragma unroll
    for (int i = 0; i < NW; i++) {
      const u32 x = sw[j * NW + i];
      below += i < w ? x : 0u;
      t += x;
    }
    ex[j] = below + inc[j] - v[j];
    tot[j] = t;
  }
}

// Map.get(vv, n, 0) >= c for a VV table of counter + 1 (0: absent, which covers cnt 0 as
// the reference's Dots.member? does, aw_lww_map.ex:67-70, and the fused join, join.hip)
__device__ __forceinline__ bool vv_tab_covers(const u64* tab, u32 n, u64 c) {
  return n < SV ? max(tab[n], 1ull) > c : c == 0;
}

// Dots.member?(delta context, dot)
__device__ __forceinline__ bool delta_covers(const SmallLds& s, bool dvv, u32 ncd, u32 n, u64 c) {
  if (dvv) return vv_tab_covers(s.cd.tabD, n, c);
  u32 lo = 0, hi = ncd;
  while (lo < hi) {
    const u32 m = (lo + hi) >> 1;
    if (s.cd.dots.n[m] < n || (s.cd.dots.n[m] == n && s.cd.dots.c[m] < c))
      lo = m + 1;
    else
      hi = m;
  }
  return lo < ncd && s.cd.dots.n[lo] == n && s.cd.dots.c[lo] == c;
}

// first delta row whose key is >= k (or > k with `upper`)
__device__ __forceinline__ u32 delta_bound(const SmallLds& s, u32 nd, u64 k, bool upper) {
  u32 lo = 0, hi = nd;
  while (lo < hi) {
    const u32 m = (lo + hi) >> 1;
    if (s.dk[m] < k || (upper && s.dk[m] == k))
      lo = m + 1;
    else
      hi = m;
  }
  return lo;
}

__device__ __forceinline__ u64 bucket_of_t(const MerkleT& t, u64 key) { return (key << t.sb) >> (64 - t.depth); }

__device__ __forceinline__ u64 row_h(const MerkleT& t, const Row& r) {
  return row_hash(r.key, th_val(t.th, r.val), r.ts, th_node(t.th, r.node), r.cnt);
}

__device__ __forceinline__ void put_row(const RowsOut& o, u64 i, const Row& r) {
  o.key[i] = r.key;
  o.val[i] = r.val;
  o.ts[i] = r.ts;
  o.node[i] = r.node;
  o.cnt[i] = r.cnt;
}

// The per-key merge of step 3: calls emit(row) for every kept row in order; returns
// (kept rows, changed)
template <class F>
__device__ __forceinline__ u32 merge_key(const SmallLds& s, u32 ia, u32 ie, u32 ja, u32 je, bool dvv, u32 ncd,
                                         bool* changed, F emit) {
  u32 ne = 0;
  bool chg = false;
  while (ia < ie || ja < je) {
    int c;  // -1: the state row first, 1: the delta row first, 0: the same row
    if (ia >= ie) {
      c = 1;
    } else if (ja >= je) {
      c = -1;
    } else {
      bool lt, eq;
      row_cmp_bf(lds_a(s, ia), lds_d(s, ja), lt, eq);
      c = eq ? 0 : (lt ? -1 : 1);
    }
    if (c == 0) {  // in both: s1 ∩ s2
      emit(lds_a(s, ia));
      ne++;
      ia++;
      ja++;
    } else if (c < 0) {  // the state's only: kept unless the delta's context covers it
      const Row r = lds_a(s, ia++);
      if (!delta_covers(s, dvv, ncd, r.node, r.cnt)) {
        emit(r);
        ne++;
      } else {
        chg = true;
      }
    } else {  // the delta's only: kept unless the state's VV covers it
      const Row r = lds_d(s, ja++);
      if (!vv_tab_covers(s.tabS, r.node, r.cnt)) {
        emit(r);
        ne++;
        chg = true;
      }
    }
  }
  *changed = chg;
  return ne;
}

// MerkleMap.update_hashes for the changed buckets only: their paths to the root.  The
// changed buckets (head threads with a changed key, in key order = bucket order) are
// compacted to pb / pv; at level l a node's new hash is made by the first entry below it
// (its owner) from its children: a child that changed is its owner's value, one that did
// not is read from the tree -- every such sibling of an entry's path is loaded up front (one
// round trip), so the depth levels cost no memory waits.  At most 64 entries: one wave,
// values in registers, owners found by ballots, no barrier; more: LDS and one barrier per
// level.  Then the chunk index: every chunk after a changed one moves by the row-count
// changes before it (dg_merkle.starts).
#ifdef DG_SMALL_STAMPS
// Diagnostic build only (DG_VARIANT=-DDG_SMALL_STAMPS): thread 0's phase timestamps
// (s_memrealtime, 100 MHz) of the last small join, read with dg_debug_small_stamps
__device__ u64 g_sm_stamps[16];
#define SSTAMP(k)                                                            \
  do {                                                                       \
    if (threadIdx.x == 0) g_sm_stamps[k] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#else
#define SSTAMP(k) \
  do {            \
  } while (0)
#endif
constexpr int TMAXD = 28;  // the deepest tree (api.hip check_merkle)

// the sibling of bucket b's ancestor l levels up (node 0 past the root): every lane
// loads every level unconditionally, so all the loads are in flight together (a load
// under a divergent condition is waited for where the condition ends)
__device__ __forceinline__ u64 sib_at(u32 dep, u64 b, int l) {
  return (u32)l < dep ? ((1ull << (dep - l)) - 1) + ((b >> l) ^ 1ull) : 0ull;
}
__device__ __forceinline__ void tree_paths(const SmallArgs& p, SmallLds& s, bool dirty, u64 v0, int drows,
                                           bool moved, bool one_path, const u64 (&psib)[TMAXD]) {
  const int tid = threadIdx.x;
  const MerkleT& t = p.t;
  const u32 depth = t.depth;
  u64* nodes = t.nodes;
  __syncthreads();  // (s.wave)
  u32 m, dtot;
  const u32 i = block_excl_scan<NT>(dirty ? 1u : 0u, s.wave, &m);
  __syncthreads();
  const u32 pre = block_excl_scan<NT>(dirty ? (u32)drows : 0u, s.wave, &dtot);
  if (dirty) {
    s.pb[i] = bucket_of_t(t, s.key[tid]);
    s.pv[0][i] = v0;
    s.pp[i] = (int)pre;
  }
  if (tid == 0) s.pp[m] = (int)dtot;
  __syncthreads();
  SSTAMP(6);
  if (m == 0) return;  // (uniform)
  auto node_at = [&](u32 level, u64 n) { return nodes + ((1ull << level) - 1) + n; };
  if (one_path) {  // (one key: m == 1) thread 0 up the path, its siblings loaded in step 1
    if (tid == 0) {
      const u64 b = s.pb[0];
      u64 v = s.pv[0][0];
#pragma unroll
      for (int l = 0; l < TMAXD; l++) {
        if ((u32)l < depth) {
          const u64 n = b >> l;
          v = (n & 1) ? node_hash(psib[l], v) : node_hash(v, psib[l]);
          *node_at(depth - l - 1, n >> 1) = v;
        }
      }
    }
  } else if (m <= (u32)WAVE) {
    if (tid < WAVE) {
      const int lane = tid;
      const bool valid = (u32)lane < m;
      const u64 b = valid ? s.pb[lane] : 0ull;
      u64 v = valid ? s.pv[0][lane] : 0ull;
      u64 sib[TMAXD];
#pragma unroll
      for (int l = 0; l < TMAXD; l++) sib[l] = nodes[sib_at(depth, b, l)];
#pragma unroll
      for (int l = 0; l < TMAXD; l++) {
        if ((u32)l < depth) {  // (uniform)
          const u64 n = b >> l;
          const u64 np = __shfl_up(n, 1, WAVE);
          const bool owner = valid && (lane == 0 || np != n);
          const u64 om = __ballot(owner);
          const u64 above = lane < WAVE - 1 ? om & (~0ull << (lane + 1)) : 0ull;
          const u64 below = om & ((1ull << lane) - 1ull);
          const int j = above ? __ffsll((long long)above) - 1 : lane;  // the next owner
          const int k = below ? 63 - __clzll((long long)below) : lane;  // the previous one
          const u64 nj = __shfl(n, j, WAVE), vj = __shfl(v, j, WAVE), nkk = __shfl(n, k, WAVE);
          if (owner) {
            bool make = true;
            u64 par = 0;
            if (!(n & 1))  // a left child: its right sibling changed iff the next owner's node is it
              par = node_hash(v, above && nj == n + 1 ? vj : sib[l]);
            else if (below && nkk == n - 1)  // a right child whose left sibling's owner makes the parent
              make = false;
            else
              par = node_hash(sib[l], v);
            if (make) {
              v = par;
              *node_at(depth - l - 1, n >> 1) = par;
            }
          }
        }
      }
    }
  } else {
    const bool valid = (u32)tid < m;
    const u64 b = valid ? s.pb[tid] : 0ull;
    u64 sib[TMAXD];
#pragma unroll
    for (int l = 0; l < TMAXD; l++) sib[l] = nodes[sib_at(depth, b, l)];
#pragma unroll
    for (int l = 0; l < TMAXD; l++) {
      if ((u32)l < depth) {  // (uniform)
        const int cur = l & 1;
        const u64 n = b >> l;
        if (valid && (tid == 0 || (s.pb[tid - 1] >> l) != n)) {  // the owner of node n
          const u64 v = s.pv[cur][tid];
          bool make = true;
          u64 par = 0;
          if (!(n & 1)) {  // the right sibling's owner, if it changed: the first entry past node n
            u32 lo = (u32)tid + 1, hi = m;
            while (lo < hi) {
              const u32 mid = (lo + hi) >> 1;
              if ((s.pb[mid] >> l) <= n)
                lo = mid + 1;
              else
                hi = mid;
            }
            par = node_hash(v, lo < m && (s.pb[lo] >> l) == n + 1 ? s.pv[cur][lo] : sib[l]);
          } else if (tid > 0 && (s.pb[tid - 1] >> l) == n - 1) {
            make = false;
          } else {
            par = node_hash(sib[l], v);
          }
          if (make) {
            s.pv[cur ^ 1][tid] = par;
            *node_at(depth - l - 1, n >> 1) = par;
          }
        }
        __syncthreads();
      }
    }
  }
  SSTAMP(7);
  if (moved && t.starts) {  // (uniform) chunk x's first row moves by the changes of chunks < x
    const u32 L1 = depth < MERKLE_UPL ? depth : MERKLE_UPL;
    const u64 G = 1ull << (depth - L1);
    const u64 x0 = (s.pb[0] >> L1) + 1;
    constexpr int XB = 8;  // entries per thread and round, their loads issued together
    for (u64 xb = x0 + (u64)tid * XB; xb <= G; xb += (u64)NT * XB) {
      u64 st[XB];
      int add[XB];
#pragma unroll
      for (int q = 0; q < XB; q++) {
        const u64 x = xb + q;
        add[q] = 0;
        st[q] = 0;
        if (x <= G) {
          u32 lo = 0, hi = m;  // the entries of chunks before x
          while (lo < hi) {
            const u32 mid = (lo + hi) >> 1;
            if ((s.pb[mid] >> L1) < x)
              lo = mid + 1;
            else
              hi = mid;
          }
          add[q] = s.pp[lo];
          if (add[q]) st[q] = t.starts[x];
        }
      }
#pragma unroll
      for (int q = 0; q < XB; q++)
        if (add[q]) t.starts[xb + q] = st[q] + (u64)(i64)add[q];
    }
  }
  SSTAMP(8);
}

__global__ __launch_bounds__(NT) void small_delta_kernel(SmallArgs p) {
  SSTAMP(0);
  __shared__ SmallLds s;
  const int tid = threadIdx.x;
  const u32 nk = (u32)p.nk, nd = (u32)p.d.n, ncd = (u32)p.cd.n, ncs = (u32)p.ca.n;
  const bool dvv = p.cd.kind == 0;
  if (tid == 0) {
    s.flags = 0;
    s.moved = 0;
    s.dkeys = 0;
  }
  for (u32 x = tid; x < SV; x += NT) {
    s.tabS[x] = 0;
    s.tabU[x] = 0;
    if (dvv) s.cd.tabD[x] = 0;
  }
  __syncthreads();
  // ---- 1. the keys' state rows; the delta and the contexts staged.  The staging goes to
  //      the threads from the top (each stream at its own offset) and the key searches to
  //      the threads from the bottom, so a one-key op's loads are in flight together
  u32 fl = 0;
  auto from_top = [&](u32 o) { return (u32)((2 * NT - 1 - tid - o) % NT); };
  for (u32 i = from_top(0); i < nd; i += NT) {
    s.dk[i] = p.d.key[i];
    s.dv[i] = p.d.val[i];
    s.dt[i] = p.d.ts[i];
    s.dn[i] = p.d.node[i];
    s.dc[i] = p.d.cnt[i];
  }
  for (u32 i = from_top(NT / 4); i < ncs; i += NT) {
    const u32 n = p.ca.node[i];
    const u64 c = p.ca.cnt[i];
    if (n >= SV || c == ~0ull)
      fl |= SMALL_FALLBACK;
    else
      s.tabS[n] = c + 1;
  }
  for (u32 i = from_top(NT / 2); i < ncd; i += NT) {
    const u32 n = p.cd.node[i];
    const u64 c = p.cd.cnt[i];
    if (n >= SV || c == ~0ull) fl |= SMALL_FALLBACK;
    if (dvv) {
      if (n < SV) s.cd.tabD[n] = c + 1;
    } else {
      s.cd.dots.n[i] = n;
      s.cd.dots.c[i] = c;
    }
  }
  // (has_tree) the key's bucket node and row count, loaded with the search
  u64 t_old = 0;
  u32 t_cnt = 0;
  if ((u32)tid < nk && p.has_tree) {
    const u64 b = bucket_of_t(p.t, p.keys[tid]);
    t_old = p.t.nodes[((1ull << p.t.depth) - 1) + b];
    t_cnt = p.t.counts[b];
  }
  // one key and a tree: its bucket path's siblings too (wave 0; tree_paths' one-path case)
  const bool one_path = nk == 1 && p.has_tree;  // (uniform)
  u64 psib[TMAXD];
  if (one_path && tid < WAVE) {
    const u64 b = bucket_of_t(p.t, p.keys[0]);
#pragma unroll
    for (int l = 0; l < TMAXD; l++) psib[l] = p.t.nodes[sib_at(p.t.depth, b, l)];
  }
  const u64 pubw = p.d_counts[tid & 15];  // the count block (publish_word): unchanged here
  if (nk <= (u32)(NT / WAVE)) {  // (uniform) a few keys: one wave searches each
    const u32 u = (u32)tid / WAVE;
    if (u < nk) {
      const u64 k = p.keys[u];
      u64 lo;
      u32 run;
      wave_find(p.a.key, p.a.n, k, lo, run);
      if ((tid & (WAVE - 1)) == 0) {
        s.key[u] = k;
        s.alo[u] = lo;
        s.na[u] = run;
      }
    }
  } else if ((u32)tid < nk) {
    const u64 k = p.keys[tid];
    const u64 lo = interp_lower_bound(p.a.key, 0, p.a.n, k);
    u64 e = lo;
    while (p.a.n > 0) {  // the key's run, 4 rows per round trip (an empty state: none)
      u64 kk[4];
#pragma unroll
      for (int q = 0; q < 4; q++) {  // (unconditional loads at clamped indices: issued together)
        const u64 v = p.a.key[e + q < p.a.n ? e + q : lo];
        kk[q] = e + q < p.a.n ? v : k + 1;
      }
      u32 c = 0;
#pragma unroll
      for (int q = 0; q < 4; q++) c += (c == (u32)q && kk[q] == k) ? 1u : 0u;
      e += c;
      if (c < 4 || e - lo > SA) break;
    }
    s.key[tid] = k;
    s.alo[tid] = lo;
    s.na[tid] = (u32)(e - lo);
  }
  if (fl) atomicOr(&s.flags, fl);
  __syncthreads();
  SSTAMP(1);
  // ---- 2. the taken rows' offsets, the rows staged; delta keys inside the keyset.  And
  //      Dots.union(state VV, delta context): per node the max, as counter + 1 (a dot set's
  //      entries folded in by LDS atomics behind the scan's barriers)
  for (u32 x = tid; x < SV; x += NT) s.tabU[x] = max(s.tabS[x], dvv ? s.cd.tabD[x] : 0ull);
  u32 tot;
  {
    const u32 v = (u32)tid < nk ? s.na[tid] : 0u;
    const u32 o = block_excl_scan<NT>(v, s.wave, &tot);
    if ((u32)tid < nk) s.aoff[tid] = o;
    if (tid == 0) s.aoff[nk] = tot;
  }
  const u32 n_ak = tot;
  if (n_ak > SA) {  // (uniform)
    if (tid == 0) s.flags |= SMALL_FALLBACK;
  }
  if (!dvv)
    for (u32 i = tid; i < ncd; i += NT)
      if (s.cd.dots.n[i] < SV)
        atomicMax((unsigned long long*)&s.tabU[s.cd.dots.n[i]], (unsigned long long)(s.cd.dots.c[i] + 1));
  __syncthreads();
  if (!(s.flags & SMALL_FALLBACK)) {
    for (u32 q = tid; q < n_ak; q += NT) {
      u32 lo = 0, hi = nk;  // the last key u with aoff[u] <= q
      while (hi - lo > 1) {
        const u32 m = (lo + hi) >> 1;
        if (s.aoff[m] <= q)
          lo = m;
        else
          hi = m;
      }
      const u64 g = s.alo[lo] + (q - s.aoff[lo]);
      s.ak[q] = p.a.key[g];
      s.av[q] = p.a.val[g];
      s.at[q] = p.a.ts[g];
      s.an[q] = p.a.node[g];
      s.ac[q] = p.a.cnt[g];
    }
    for (u32 i = tid; i < nd; i += NT) {
      if (i > 0 && s.dk[i] == s.dk[i - 1]) continue;
      u32 lo = 0, hi = nk;
      while (lo < hi) {
        const u32 m = (lo + hi) >> 1;
        if (s.key[m] < s.dk[i])
          lo = m + 1;
        else
          hi = m;
      }
      if (lo == nk || s.key[lo] != s.dk[i]) atomicOr(&s.flags, SMALL_FALLBACK);
    }
  }
  __syncthreads();
  SSTAMP(2);
  const bool fallback = s.flags & SMALL_FALLBACK;  // (uniform)
  // ---- 3. the join per key: kept rows, changed, distinct-key change
  u32 ne = 0, chg = 0, ja = 0, je = 0;
  if (!fallback && (u32)tid < nk) {
    const u64 k = s.key[tid];
    ja = delta_bound(s, nd, k, false);
    je = delta_bound(s, nd, k, true);
    bool c;
    ne = merge_key(s, s.aoff[tid], s.aoff[tid + 1], ja, je, dvv, ncd, &c, [](const Row&) {});
    chg = c ? 1u : 0u;
    s.ne[tid] = ne;
    if (ne != s.na[tid]) atomicOr(&s.moved, 1u);
    const int dk = (int)(ne > 0) - (int)(s.na[tid] > 0);
    if (dk) atomicAdd(&s.dkeys, dk);
  }
  // ---- 4. offsets: the edit's, the changed keys', their rows', the union context's
  //      entries -- four scans, one barrier
  u32 n_e, n_chg, n_rows, nctx, cpos;
  {
    constexpr u32 PER = SV / NT;  // table entries per thread
    u32 own = 0;
#pragma unroll
    for (u32 q = 0; q < PER; q++) own += s.tabU[tid * PER + q] != 0 ? 1u : 0u;
    const u32 v[4] = {ne, chg, chg ? ne : 0u, own};
    u32 ex[4], tt[4];
    block_scan4(v, s.w4, ex, tt);
    n_e = tt[0];
    n_chg = tt[1];
    n_rows = tt[2];
    nctx = tt[3];
    cpos = ex[3];
    if ((u32)tid < nk) {
      s.eoff[tid] = ex[0];
      s.coff[tid] = ex[1];
      s.roff[tid] = ex[2];
    }
    if (tid == 0) s.eoff[nk] = n_e;
  }
  if (tid == 0 && (n_e > SE || nctx > p.ca_cap)) atomicOr(&s.flags, SMALL_FALLBACK);
  SSTAMP(3);
  // ---- 5. the tree: per bucket the leaf and row-count change, checked before any write
  // (leaf[u]: Σ row_hash of the key's new rows - of its old rows)
  if (!fallback && p.has_tree && (u32)tid < nk && chg) {
    u64 h = 0;
    for (u32 i = s.aoff[tid]; i < s.aoff[tid + 1]; i++) h -= row_h(p.t, lds_a(s, i));
    bool c;
    merge_key(s, s.aoff[tid], s.aoff[tid + 1], ja, je, dvv, ncd, &c,
              [&](const Row& r) { h += row_h(p.t, r); });
    s.leaf[tid] = h;
  }
  __syncthreads();
  if (!fallback && p.has_tree && (u32)tid < nk) {
    const u64 k = s.key[tid];
    const MerkleT& t = p.t;
    const u64 b = bucket_of_t(t, k);
    const bool head = tid == 0 || bucket_of_t(t, s.key[tid - 1]) != b;
    if (chg && t.sb && (k >> (64 - t.sb)) != t.shard) atomicOr(&s.flags, MERKLE_ERR_SHARD);
    if (head) {  // the bucket's keys: this one and the next ones in the same bucket
      i64 drows = 0;
      for (u32 u = tid; u < nk && bucket_of_t(t, s.key[u]) == b; u++) drows += (i64)s.ne[u] - (i64)s.na[u];
      const i64 now = (i64)t_cnt + drows;
      if (now < 0 || now > 0xFFFF) atomicOr(&s.flags, MERKLE_ERR_COUNT);
    }
  }
  __syncthreads();
  const u32 flags = s.flags;
  SSTAMP(4);
  u64* res = p.res;
  // the result block goes straight into `home` (host memory); the header also into `res`
  // (the tail kernel and the splice after the wait read it on the device)
  u64* home = p.home;
  // publish: the engine's count block and the sequence number, after every thread's home
  // writes (dg_home.h); unless the rows moved and the tail kernel copies them (it does)
  const bool moved = s.moved != 0;
  if (flags) {  // (uniform) nothing written: the caller takes the general path or reports
    if (tid < (int)SMALL_HDR) {
      res[tid] = tid ? 0ull : (u64)flags;
      home[tid] = tid ? 0ull : (u64)flags;
    }
    publish_word(pubw, p.h_pub, p.seq);
    return;
  }
  // ---- 6. writes
  u64 t_new = 0;
  int t_drows = 0;
  bool t_dirty = false;  // a head thread whose bucket changed: t_new, its rows' change
  if ((u32)tid < nk) {
    const u32 e0 = s.eoff[tid], r0 = s.roff[tid];
    const u64 a0 = s.alo[tid];
    // the splice's gap shift of this key's edit rows: E's row j goes to j + a_lo - a_off
    const i64 gap = (i64)a0 - (i64)s.aoff[tid];
    u32 j = 0;
    bool c;
    u64* rk = home + SMALL_O_ROWS;
    const RowsOut rr{rk, rk + SE, (i64*)(rk + 2 * SE), (u32*)(rk + 4 * SE), rk + 3 * SE};
    merge_key(s, s.aoff[tid], s.aoff[tid + 1], ja, je, dvv, ncd, &c, [&](const Row& r) {
      if (!moved)
        put_row(p.aw, a0 + j, r);  // in place: every key keeps its row count
      else if (p.splice_here)
        put_row(p.sp, (u64)((i64)(e0 + j) + gap), r);  // straight to its place in the spare
      else
        put_row(p.e, e0 + j, r);  // the edit, for the splice kernels after the wait
      if (chg) put_row(rr, r0 + j, r);  // the changed keys' rows, for the caller
      j++;
    });
    if (moved && p.splice_here) {  // the index the tail kernel's splice tiles search
      p.end[tid] = a0 + s.na[tid];
      p.shift[tid] = (i64)e0 - (i64)s.aoff[tid];
      if (tid == 0) p.shift[nk] = (i64)n_e - (i64)n_ak;
    }
    if (chg) home[SMALL_O_KEYS + s.coff[tid]] = s.key[tid];
    p.a_lo[tid] = a0;
    p.a_off[tid] = s.aoff[tid];
    if (tid == 0) p.a_off[nk] = n_ak;
    if (p.has_tree) {
      const MerkleT& t = p.t;
      const u64 k = s.key[tid], b = bucket_of_t(t, k);
      const bool head = tid == 0 || bucket_of_t(t, s.key[tid - 1]) != b;
      if (head) {  // the bucket's keys: this one and the next ones in the same bucket
        u64 dh = 0;
        i64 drows = 0;
        bool any = false;
        for (u32 u = tid; u < nk && bucket_of_t(t, s.key[u]) == b; u++) {
          drows += (i64)s.ne[u] - (i64)s.na[u];
          const bool cu = (u + 1 < nk ? s.coff[u + 1] : n_chg) != s.coff[u];  // key u changed
          if (cu) {
            dh += s.leaf[u];
            any = true;
          }
        }
        if (any) {  // MerkleMap.put/delete: the bucket's node and row count
          t_dirty = true;
          t_new = t_old + dh;
          t_drows = (int)drows;
          t.nodes[((1ull << t.depth) - 1) + b] = t_new;
          if (drows) t.counts[b] = (uint16_t)((i64)t_cnt + drows);
        }
      }
    }
  }
  // the union context: into the state's and the result block
  {
    constexpr u32 PER = SV / NT;
    u32 o = cpos;
    u64* rc = home + SMALL_O_CTX;
    u32* rn = (u32*)(rc + SV);
#pragma unroll
    for (u32 q = 0; q < PER; q++) {
      const u32 x = tid * PER + q;
      const u64 v = s.tabU[x];
      if (v) {
        p.ca_node[o] = x;
        p.ca_cnt[o] = v - 1;
        rn[o] = x;
        rc[o] = v - 1;
        o++;
      }
    }
  }
  if (tid < (int)SMALL_HDR) {
    const u64 h[SMALL_HDR] = {0, n_chg, n_rows, nctx, n_e, n_ak, moved ? 1u : 0u, (u64)(i64)s.dkeys};
    u64 v = 0;
#pragma unroll
    for (int i = 0; i < (int)SMALL_HDR; i++) v = i == tid ? h[i] : v;
    res[tid] = v;
    home[tid] = v;
  }
  SSTAMP(5);
  if (p.has_tree) tree_paths(p, s, t_dirty, t_new, t_drows, moved, one_path, psib);
  SSTAMP(9);
  if (!(moved && p.splice_here)) publish_word(pubw, p.h_pub, p.seq);
  SSTAMP(10);
}

// ---------------------------------------------------------------- dg_join_delta_home's tail
// (dg_launch.h SmallTailArgs) The moved rows' splice copy behind the small join, and the
// publish by the last workgroup to finish.  A splice tile's rows: thread
// t holds rows 2 (q NT + t) + h of the tile (q, h < 2), each column read as 16-byte pairs;
// the per-key index (<= SMALL_KEYS entries, written by the small join) is staged in LDS
// while the loads are in flight, and row i goes to i + shift[u*] with u* the first key
// whose state rows end after i -- unless i is one of that key's rows (the edit's, placed
// by the small join).
static_assert(SMALL_TILE == 4 * NT, "4 rows per thread");
__device__ __forceinline__ void small_tile_copy(const SmallTailArgs& p, u64 tile) {
  __shared__ u64 s_end[SMALL_KEYS], s_lo[SMALL_KEYS];
  __shared__ i64 s_sh[SMALL_KEYS + 1];
  const u32 tid = threadIdx.x, nk = (u32)p.nk;
  const u64 i0 = tile * SMALL_TILE, i1 = min<u64>(i0 + SMALL_TILE, p.a.n);
  u64 key[4], val[4], cnt[4];
  i64 ts[4];
  u32 nd[4];
#pragma unroll
  for (int q = 0; q < 2; q++) {
    const u64 i = i0 + 2 * ((u64)q * NT + tid);
    if (i + 1 < i1) {  // i0 and i even: an aligned pair
      const ulonglong2 k = *(const ulonglong2*)(p.a.key + i), v = *(const ulonglong2*)(p.a.val + i);
      const longlong2 t2 = *(const longlong2*)(p.a.ts + i);
      const ulonglong2 c = *(const ulonglong2*)(p.a.cnt + i);
      const uint2 n = *(const uint2*)(p.a.node + i);
      key[2 * q] = k.x, key[2 * q + 1] = k.y, val[2 * q] = v.x, val[2 * q + 1] = v.y;
      ts[2 * q] = t2.x, ts[2 * q + 1] = t2.y, cnt[2 * q] = c.x, cnt[2 * q + 1] = c.y;
      nd[2 * q] = n.x, nd[2 * q + 1] = n.y;
    } else if (i < i1) {
      key[2 * q] = p.a.key[i], val[2 * q] = p.a.val[i], ts[2 * q] = p.a.ts[i];
      cnt[2 * q] = p.a.cnt[i], nd[2 * q] = p.a.node[i];
    }
  }
  for (u32 x = tid; x < nk; x += NT) {
    s_end[x] = p.end[x];
    s_lo[x] = p.a_lo[x];
  }
  for (u32 x = tid; x <= nk; x += NT) s_sh[x] = p.shift[x];
  __syncthreads();
#pragma unroll
  for (int r = 0; r < 4; r++) {
    const u64 i = i0 + 2 * ((u64)(r >> 1) * NT + tid) + (r & 1);
    if (i >= i1) continue;
    u32 lo = 0, hi = nk;  // the first key whose rows end after row i
    while (lo < hi) {
      const u32 m = (lo + hi) >> 1;
      if (s_end[m] > i)
        hi = m;
      else
        lo = m + 1;
    }
    if (lo < nk && s_lo[lo] <= i) continue;  // a keyset key's row: the edit replaced it
    const u64 o = (u64)((i64)i + s_sh[lo]);
    p.out.key[o] = key[r];
    p.out.val[o] = val[r];
    p.out.ts[o] = ts[r];
    p.out.node[o] = nd[r];
    p.out.cnt[o] = cnt[r];
  }
}

__global__ __launch_bounds__(NT) void small_tail_kernel(SmallTailArgs p) {
  __shared__ u32 s_all;
  if (blockIdx.x == 0) SSTAMP(12);
  const bool moved = p.res[0] == 0 && p.res[6];  // (uniform) else the small join published
  if (!moved) return;
  small_tile_copy(p, blockIdx.x);
  // every workgroup arrives once its part is done; the last one publishes
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence();
    const u32 n = __hip_atomic_fetch_add(p.arrive_all, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_all = n == gridDim.x - 1;
    if (s_all) __hip_atomic_store(p.arrive_all, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  if (s_all) {
    __threadfence();
    publish_counts(p.d_counts, p.h_pub, p.seq);
  }
}

}  // namespace

#ifdef DG_SMALL_STAMPS
extern "C" int dg_debug_small_stamps(unsigned long long* host, size_t n) {
  if (n > 16) n = 16;
  if (hipDeviceSynchronize() != hipSuccess) return -3;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_sm_stamps), n * 8) == hipSuccess ? 0 : -3;
}
#endif

// Test hook (tests/test_gpu_join_delta.py): wave_find of each query on device arrays, one
// wave per query, on the null stream, synchronous
__global__ __launch_bounds__(256) void wave_find_kernel(const u64* a, u64 n, const u64* q, u64 nq, u64* lo,
                                                         u32* run) {
  const u64 i = (u64)blockIdx.x * (256 / WAVE) + threadIdx.x / WAVE;
  if (i >= nq) return;  // (uniform per wave)
  u64 l;
  u32 r;
  wave_find(a, n, q[i], l, r);
  if ((threadIdx.x & (WAVE - 1)) == 0) {
    lo[i] = l;
    run[i] = r;
  }
}

}  // namespace dg

extern "C" int dg_debug_wave_find(const unsigned long long* a, unsigned long long n, const unsigned long long* q,
                                  unsigned long long nq, unsigned long long* lo, unsigned int* run) {
  if (!nq) return 0;
  hipLaunchKernelGGL(dg::wave_find_kernel, dim3((unsigned)((nq + 3) / 4)), dim3(256), 0, 0, (const dg::u64*)a,
                     (dg::u64)n, (const dg::u64*)q, (dg::u64)nq, (dg::u64*)lo, (dg::u32*)run);
  if (hipGetLastError() != hipSuccess) return -3;
  return hipDeviceSynchronize() == hipSuccess ? 0 : -3;
}

namespace dg {

hipError_t launch_small_delta(const SmallArgs& p, hipStream_t st) {
  hipLaunchKernelGGL(small_delta_kernel, dim3(1), dim3(NT), 0, st, p);
  return hipGetLastError();
}


hipError_t launch_small_tail(const SmallTailArgs& p, hipStream_t st) {
  hipLaunchKernelGGL(small_tail_kernel, dim3((unsigned)(p.tiles ? p.tiles : 1)), dim3(NT), 0, st, p);
  return hipGetLastError();
}

}  // namespace dg
