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
//   6. writes: the edit's rows in place when no key's row count changed (else the caller's
//      guarded splice copy moves the state into its spare buffer, reading the edit and
//      the per-key index from here), the union context, the bucket nodes, counts, dirty
//      chunks and chunk-index deltas (the upsweep launch after this re-reduces the dirty
//      chunks: MerkleMap.update_hashes), and the result block.
// Anything outside the limits sets SMALL_FALLBACK before any write: the caller then runs
// the general path on the untouched state.
//
// Roofline: latency, not bandwidth -- a one-key op reads and writes a few hundred bytes;
// what it saves is three host round trips.
#include "dg_hash.h"
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
  u32 wave[NT / WAVE + 1];
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

// Dots.member?(delta context, dot)
__device__ __forceinline__ bool delta_covers(const SmallLds& s, bool dvv, u32 ncd, u32 n, u64 c) {
  if (dvv) return n < SV && s.cd.tabD[n] > c;
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
      if (!(r.node < SV && s.tabS[r.node] > r.cnt)) {
        emit(r);
        ne++;
        chg = true;
      }
    }
  }
  *changed = chg;
  return ne;
}

__global__ __launch_bounds__(NT) void small_delta_kernel(SmallArgs p) {
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
  // ---- 1. the keys' state rows; the delta and the contexts staged
  u32 fl = 0;
  if ((u32)tid < nk) {
    const u64 k = p.keys[tid];
    const u64 lo = interp_lower_bound(p.a.key, 0, p.a.n, k);
    u64 e = lo;
    while (e < p.a.n && p.a.key[e] == k && e - lo <= SA) e++;
    s.key[tid] = k;
    s.alo[tid] = lo;
    s.na[tid] = (u32)(e - lo);
  }
  for (u32 i = tid; i < nd; i += NT) {
    s.dk[i] = p.d.key[i];
    s.dv[i] = p.d.val[i];
    s.dt[i] = p.d.ts[i];
    s.dn[i] = p.d.node[i];
    s.dc[i] = p.d.cnt[i];
  }
  for (u32 i = tid; i < ncs; i += NT) {
    const u32 n = p.ca.node[i];
    const u64 c = p.ca.cnt[i];
    if (n >= SV || c == ~0ull)
      fl |= SMALL_FALLBACK;
    else
      s.tabS[n] = c + 1;
  }
  for (u32 i = tid; i < ncd; i += NT) {
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
  if (fl) atomicOr(&s.flags, fl);
  __syncthreads();
  // ---- 2. the taken rows' offsets, the rows staged; delta keys inside the keyset
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
  // ---- 4. offsets: the edit's, the changed keys', their rows'
  u32 n_e, n_chg, n_rows;
  {
    const u32 o = block_excl_scan<NT>(ne, s.wave, &n_e);
    if ((u32)tid < nk) s.eoff[tid] = o;
    if (tid == 0) s.eoff[nk] = n_e;
    __syncthreads();
    const u32 oc = block_excl_scan<NT>(chg, s.wave, &n_chg);
    __syncthreads();
    const u32 orr = block_excl_scan<NT>(chg ? ne : 0u, s.wave, &n_rows);
    if ((u32)tid < nk) {
      s.coff[tid] = oc;
      s.roff[tid] = orr;
    }
  }
  if (tid == 0 && n_e > SE) s.flags |= SMALL_FALLBACK;
  // Dots.union(state VV, delta context): per node the max, as counter + 1
  if (!fallback) {
    for (u32 x = tid; x < SV; x += NT) s.tabU[x] = max(s.tabS[x], dvv ? s.cd.tabD[x] : 0ull);
    __syncthreads();
    if (!dvv)
      for (u32 i = tid; i < ncd; i += NT) atomicMax((unsigned long long*)&s.tabU[s.cd.dots.n[i]],
                                                   (unsigned long long)(s.cd.dots.c[i] + 1));
  }
  __syncthreads();
  u32 nctx = 0, cpos = 0;
  {
    constexpr u32 PER = SV / NT;  // table entries per thread
    u32 own = 0;
#pragma unroll
    for (u32 q = 0; q < PER; q++) own += s.tabU[tid * PER + q] != 0 ? 1u : 0u;
    cpos = block_excl_scan<NT>(own, s.wave, &nctx);
  }
  if (tid == 0 && nctx > p.ca_cap) s.flags |= SMALL_FALLBACK;
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
      const i64 now = (i64)t.counts[b] + drows;
      if (now < 0 || now > 0xFFFF) atomicOr(&s.flags, MERKLE_ERR_COUNT);
    }
  }
  __syncthreads();
  const u32 flags = s.flags;
  u64* res = p.res;
  if (flags) {  // (uniform) nothing written: the caller takes the general path or reports
    if (tid == 0) {
      res[0] = flags;
      for (int i = 1; i < (int)SMALL_HDR; i++) res[i] = 0;
    }
    return;
  }
  // ---- 6. writes
  const bool moved = s.moved != 0;
  if ((u32)tid < nk) {
    const u32 e0 = s.eoff[tid], r0 = s.roff[tid];
    const u64 a0 = s.alo[tid];
    u32 j = 0;
    bool c;
    u64* rk = res + SMALL_O_ROWS;
    const RowsOut rr{rk, rk + SE, (i64*)(rk + 2 * SE), (u32*)(rk + 4 * SE), rk + 3 * SE};
    merge_key(s, s.aoff[tid], s.aoff[tid + 1], ja, je, dvv, ncd, &c, [&](const Row& r) {
      put_row(p.e, e0 + j, r);          // the edit (the moved path's splice reads it)
      if (!moved) put_row(p.aw, a0 + j, r);  // in place: every key keeps its row count
      if (chg) put_row(rr, r0 + j, r);   // the changed keys' rows, for the caller
      j++;
    });
    if (chg) res[SMALL_O_KEYS + s.coff[tid]] = s.key[tid];
    p.a_lo[tid] = a0;
    p.a_off[tid] = s.aoff[tid];
    if (tid == 0) p.a_off[nk] = n_ak;
    if (p.has_tree) {
      const MerkleT& t = p.t;
      const u64 k = s.key[tid], b = bucket_of_t(t, k);
      const bool head = tid == 0 || bucket_of_t(t, s.key[tid - 1]) != b;
      if (head) {
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
        if (any) {
          u64* lvl = t.nodes + ((1ull << t.depth) - 1);
          lvl[b] += dh;
          if (drows) t.counts[b] = (uint16_t)((i64)t.counts[b] + drows);
          const u32 L1 = t.depth < MERKLE_UPL ? t.depth : MERKLE_UPL;
          p.dirty[b >> L1] = 1u;
          if (t.starts && drows)
            atomicAdd((unsigned long long*)&p.cdelta[b >> L1], (unsigned long long)drows);
        }
      }
    }
  }
  // the union context: into the state's and the result block
  {
    constexpr u32 PER = SV / NT;
    u32 o = cpos;
    u64* rc = res + SMALL_O_CTX;
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
  if (tid == 0) {
    res[0] = 0;
    res[1] = n_chg;
    res[2] = n_rows;
    res[3] = nctx;
    res[4] = n_e;
    res[5] = n_ak;
    res[6] = moved ? 1 : 0;
    res[7] = (u64)(i64)s.dkeys;
  }
}

// The used part of the result block into `home` (host memory): header, changed keys, their
// rows (each column at its fixed stride), the context -- a few hundred bytes for one key --
// then the engine's counts and the sequence number the host polls (api.hip sync_words).
__global__ __launch_bounds__(256) void small_home_kernel(const u64* res, u64* home, const u64* d_counts,
                                                         u64* h_pub, u64 seq) {
  const u64 n_chg = res[1], n_rows = res[2], nctx = res[3];
  const int tid = threadIdx.x;
  if (tid < (int)SMALL_HDR) home[tid] = res[tid];
  for (u64 i = tid; i < n_chg; i += 256) home[SMALL_O_KEYS + i] = res[SMALL_O_KEYS + i];
  for (int c = 0; c < 4; c++)
    for (u64 i = tid; i < n_rows; i += 256) home[SMALL_O_ROWS + c * SE + i] = res[SMALL_O_ROWS + c * SE + i];
  const u32* rn = (const u32*)(res + SMALL_O_ROWS + 4 * SE);
  u32* hn = (u32*)(home + SMALL_O_ROWS + 4 * SE);
  for (u64 i = tid; i < n_rows; i += 256) hn[i] = rn[i];
  for (u64 i = tid; i < nctx; i += 256) home[SMALL_O_CTX + i] = res[SMALL_O_CTX + i];
  const u32* cn = (const u32*)(res + SMALL_O_CTX + SV);
  u32* hc = (u32*)(home + SMALL_O_CTX + SV);
  for (u64 i = tid; i < nctx; i += 256) hc[i] = cn[i];
  if (tid < 16) h_pub[tid] = d_counts[tid];  // d_counts[0..8) and the ticket words
  __threadfence_system();
  __syncthreads();
  if (tid == 0) __hip_atomic_store(h_pub + 16, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

}  // namespace

hipError_t launch_small_delta(const SmallArgs& p, hipStream_t st) {
  hipLaunchKernelGGL(small_delta_kernel, dim3(1), dim3(NT), 0, st, p);
  return hipGetLastError();
}

hipError_t launch_small_home_publish(const u64* res, u64* home, const u64* d_counts, u64* h_pub, u64 seq,
                                     hipStream_t st) {
  hipLaunchKernelGGL(small_home_kernel, dim3(1), dim3(256), 0, st, res, home, d_counts, h_pub, seq);
  return hipGetLastError();
}

}  // namespace dg
