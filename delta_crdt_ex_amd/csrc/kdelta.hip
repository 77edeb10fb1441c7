// kdelta.hip — update_state_with_delta for a keyed delta of ANY size with one host wait.
//
// CausalCrdt joins every sync delta and every batch of local mutations into the replica
// with its keyset (reference causal_crdt.ex:383-394; aw_lww_map.ex:153-209).  When the
// delta's keys all lie in the keyset, only the keyset's keys change, and each key's new
// rows are join_dot_sets/4 (:196-209) of its state rows and its delta rows -- a handful of
// rows per key.  So instead of a merge-path join of the taken rows (whose launch is sized
// by counts the host must wait for), every keyset key is one thread:
//
//   kd_count_kernel   (one thread per key) its state run (an interpolation search of the
//                     state: key ids are hashes) and delta run, the per-key join: which
//                     state rows stay (s1 ∩ s2 ∪ s1 \ c2) and which delta rows come in
//                     (s2 \ c1) -- kept as two bit masks -- whether the key changed (diff/3,
//                     causal_crdt.ex:344-352) and its Merkle leaf change (Σ row_hash new -
//                     Σ row_hash old), put into the tree right away (segmented wave sums:
//                     one atomic per bucket and chunk); per workgroup the sums of rows, kept
//                     rows, changed keys and their rows, delta rows seen; the last key
//                     workgroup to finish sums them into the totals and the guard word: a
//                     delta row outside the keyset (the right-biased carry of :185-188
//                     applies: the caller runs the full join), a key run over KD_RUN rows,
//                     more changed keys than the caller's capacity.  Workgroup 0 of the
//                     launch computes the context union (Dots.union/2).
//   kd_finish_kernel  (merkle.hip + dg_kdw.h, one launch) one thread per key: its new rows --
//                     in place when no key's row count changed, else straight to their
//                     final places in the spare store -- the changed keys and their rows
//                     (device or page-locked host memory), the splice index of the rows
//                     that move (splice.hip), the union context into the state's; every
//                     state write skipped when the tree update reported an input error (all
//                     or nothing); each workgroup sums the earlier count workgroups'
//                     figures for its offsets.  Beside them, persistent workgroups re-reduce
//                     the dirty chunks of the tree (update_hashes).
//   splice_kernel     (splice.hip, only when rows moved) the untouched rows to the spare
//
// then the count block is published to mapped host memory and the host waits ONCE.
//
// Roofline: each key costs two searches (~6 dependent loads of the state, a few of the
// delta) and reads its few rows twice (the second time from L2); a sync delta of 125k keys
// into a 12.5M-row state reads ~10 MB.  Latency-bound by the search chains, not by bytes.
#include "dg_ctxu.h"
#include "dg_hash.h"
#include "dg_launch.h"
#include "dg_tree.h"

namespace dg {

namespace {

constexpr int KDB = KD_BLOCK;  // keys per workgroup, one per thread
constexpr u32 KVT = 1024;      // VV tables in LDS cover node ids < KVT
static_assert(KD_RUN <= 64, "a key's kept rows are a 64-bit mask per side");

__device__ __forceinline__ u64 rhash(const MerkleT& t, const Row& r) {
  return row_hash(r.key, th_val(t.th, r.val), r.ts, th_node(t.th, r.node), r.cnt);
}

// Map.get(vv, node, 0) >= cnt through the LDS table (node ids < KVT), else a search
__device__ __forceinline__ bool vv_covers(const u64* tab, const Ctx& c, u32 n, u64 cnt) {
  if (n < KVT) return tab[n] >= cnt;
  return ctx_covers(c.node, c.cnt, c.n, 0, n, cnt);
}

// first row of key k in s (lower bound) and its run, at most KD_RUN + 1 counted (4 rows a
// round trip, every load issued together at a clamped index)
__device__ __forceinline__ void key_run(const u64* key, u64 n, u64 k, u64& lo, u32& run) {
  lo = interp_lower_bound(key, 0, n, k);
  u64 e = lo;
  while (e < n) {
    u64 kk[4];
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const u64 v = key[e + q < n ? e + q : lo];
      kk[q] = e + q < n ? v : k + 1;
    }
    u32 c = 0;
#pragma unroll
    for (int q = 0; q < 4; q++) c += (c == (u32)q && kk[q] == k) ? 1u : 0u;
    e += c;
    if (c < 4 || e - lo > KD_RUN) break;
  }
  run = (u32)(e - lo);
}

// agent-scope stores and loads for the hand-off to the last workgroup (written through to
// the point of coherence: the workgroups run on all eight XCDs)
__device__ __forceinline__ void st_ag(u64* p, u64 v) {
  __hip_atomic_store((__attribute__((address_space(1))) u64*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ u64 ld_ag(const u64* p) {
  return __hip_atomic_load((__attribute__((address_space(1))) u64*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// MerkleMap.put/delete of the changed keys (the caller zeroed dirty and cdelta): key u's
// leaf change d and row-count change dr.  The keys are ascending, so a wave's keys of one
// bucket (and of one chunk) are adjacent lanes: segmented sums over the lanes leave ONE
// atomic per bucket and per chunk.  merkle.hip's kd_tree_kernel applies the same with the
// opposite sign to undo it.
template <class T>
__device__ __forceinline__ T seg_sum(T v, u64 seg, int lane) {
#pragma unroll
  for (int d = 1; d < WAVE; d <<= 1) {
    const T y = __shfl_up(v, d, WAVE);
    const u64 sy = __shfl_up(seg, d, WAVE);
    if (lane >= d && sy == seg) v += y;  // (segments are contiguous runs of lanes)
  }
  return v;
}
__device__ __forceinline__ void tree_put(const KdArgs& p, bool valid, u64 x, bool chg, u64 d, int dr) {
  const MerkleT& t = p.t;
  const int lane = threadIdx.x & (WAVE - 1);
  const u32 L1 = t.depth < MERKLE_UPL ? t.depth : MERKLE_UPL;
  bool bad = false, over = false;
  int act = 0;
  const u64 b = valid ? (x << t.sb) >> (64 - t.depth) : ~0ull;
  if (valid && chg && (d != 0 || dr != 0)) {
    if (t.sb && (x >> (64 - t.sb)) != t.shard)
      bad = true;  // (skipped both ways)
    else
      act = 1;
  }
  if (!act) {
    d = 0;
    dr = 0;
  }
  const u64 c = b == ~0ull ? ~0ull : b >> L1;
  const u64 sd = seg_sum<u64>(d, b, lane);
  const int sr = seg_sum<int>(dr, b, lane), sa = seg_sum<int>(act, b, lane);
  const int cr = seg_sum<int>(dr, c, lane), ca = seg_sum<int>(act, c, lane);
  const u64 nb = __shfl_down(b, 1, WAVE), nc = __shfl_down(c, 1, WAVE);
  const bool last = lane == WAVE - 1;
  if (b != ~0ull && (last || nb != b) && sa) {  // the bucket's last lane: its node and row count
    u64* lvl = t.nodes + ((1ull << t.depth) - 1);
    atomicAdd((unsigned long long*)&lvl[b], (unsigned long long)sd);
    if (sr) {  // (its aligned 32-bit word of two u16 counts, as merkle_update_kernel)
      u32* wd = (u32*)t.counts + (b >> 1);
      const u32 sh = 16u * (u32)(b & 1);
      if (sr > 0) {
        const u32 old = atomicAdd(wd, (u32)sr << sh);
        over = ((old >> sh) & 0xFFFFu) + (u32)sr > 0xFFFFu;
      } else {
        atomicSub(wd, (u32)(-sr) << sh);
      }
    }
  }
  if (c != ~0ull && (last || nc != c) && ca) {  // the chunk's last lane: dirty, its row-count change
    p.dirty[c] = 1u;
    if (t.starts && cr) atomicAdd((unsigned long long*)&p.cdelta[c], (unsigned long long)(i64)cr);
  }
  if (__ballot(bad) && lane == 0) atomicOr(p.err, MERKLE_ERR_SHARD);
  if (__ballot(over) && lane == 0) atomicOr(p.err, MERKLE_ERR_COUNT);
}

// ---------------------------------------------------------------- count (+ scan)
// The workgroup's keys are ascending, so their delta rows are one contiguous range: two
// searches find its ends and its keys are staged in LDS (every key's delta run is found
// there, not by a search of the delta in memory).  (Narrowing the state searches to the
// workgroup's range the same way, by 64-ary wave searches, measured slower: 52 against
// 45 us at config 4 -- their 256 scattered lines per bound outweigh what each key saves.)
constexpr u32 KDL = 2048;  // delta keys staged per workgroup (more: searched in memory)
#ifdef DG_STAMPS
// Diagnostic build only (DG_STAMPS=1): per-workgroup timestamps (s_memrealtime, 100 MHz) of
// the count kernel, read back with dg_debug_kd_stamps (tools/kd_stamps.py).  No barriers
// added: thread `th` stamps slot k when it passes that point.
__device__ u64 g_kd_stamps[4096 * 8];
#define KDSTAMP(th, k)                                                        \
  do {                                                                        \
    if (threadIdx.x == (th) && blk < 4096)                                    \
      g_kd_stamps[blk * 8 + (k)] = __builtin_amdgcn_s_memrealtime();          \
  } while (0)
#else
#define KDSTAMP(th, k) \
  do {                 \
  } while (0)
#endif
__global__ __launch_bounds__(KDB) void kd_count_kernel(KdArgs p) {
  __shared__ u64 tabS[KVT], tabD[KVT];
  __shared__ u64 s_dk[KDL];
  __shared__ u64 s_rng[2];
  __shared__ u64 red[KD_NV][KDB / WAVE];
  __shared__ u32 s_last;
  __shared__ u32 s_cw[KDB / WAVE + 1];
  if (blockIdx.x == 0) {
    // Dots.union(state context, delta context) (:155) into the union scratch and
    // d_counts[1], by a workgroup of its own beside the keys' (it needs only the inputs; in
    // the last workgroup's tail it added ~5 us to every call)
    ctx_union_block<KDB>(make_cu(p.ca, p.cd, p.uc_node, p.uc_cnt, p.d_counts + 1, p.cu_tmp), s_cw);
    return;
  }
  const u64 blk = blockIdx.x - 1;  // the keys' workgroups: 1 .. ntiles
  const int tid = threadIdx.x, lane = tid & (WAVE - 1), w = tid / WAVE;
  const u64 u = blk * KDB + tid;
  const u64 u0 = blk * KDB, u1 = min<u64>(u0 + KDB, p.nk);
  const bool dvv = p.cd.kind == 0;
  KDSTAMP(2, 0);
  if (tid < 2) {  // the workgroup's delta range [lo, hi): its keys' rows (two searches)
    const u64 x = tid ? p.keys[u1 - 1] + 1 : p.keys[u0];  // (key + 1: past the last key's run)
    s_rng[tid] = tid && x == 0 ? p.d.n : interp_lower_bound(p.d.key, 0, p.d.n, x);  // (2^64 - 1)
  }
  KDSTAMP(0, 1);
  for (u32 x = tid; x < KVT; x += KDB) {
    tabS[x] = 0;
    tabD[x] = 0;
  }
  __syncthreads();
  for (u64 i = tid; i < p.ca.n; i += KDB)
    if (p.ca.node[i] < KVT) tabS[p.ca.node[i]] = p.ca.cnt[i];
  if (dvv)
    for (u64 i = tid; i < p.cd.n; i += KDB)
      if (p.cd.node[i] < KVT) tabD[p.cd.node[i]] = p.cd.cnt[i];
  const u64 dlo = s_rng[0], dhi = s_rng[1];
  const bool dl = dhi - dlo <= KDL;  // (uniform)
  if (dl)
    for (u64 i = tid; i < dhi - dlo; i += KDB) s_dk[i] = p.d.key[dlo + i];
  u64 v[KD_NV] = {0, 0, 0, 0, 0, 0, 0};
  u64 a_lo = 0, d_lo = 0, am = 0, dm = 0, dh = 0;
  u32 na = 0, nd = 0, ne = 0;
  bool chg = false, big = false;
  u64 k = 0;
  if (u < p.nk) {
    k = p.keys[u];
    key_run(p.a.key, p.a.n, k, a_lo, na);  // the state: an interpolation search
  }
  KDSTAMP(2, 2);
  __syncthreads();  // (the tables, the staged delta keys)
  KDSTAMP(2, 3);
  if (u < p.nk) {
    if (dl) {  // the delta run from LDS
      u32 lo = 0, hi = (u32)(dhi - dlo);
      while (lo < hi) {
        const u32 m = (lo + hi) >> 1;
        if (s_dk[m] < k)
          lo = m + 1;
        else
          hi = m;
      }
      u32 e = lo;
      while (e < (u32)(dhi - dlo) && s_dk[e] == k && e - lo <= KD_RUN) e++;
      d_lo = dlo + lo;
      nd = e - lo;
    } else {
      key_run(p.d.key, p.d.n, k, d_lo, nd);
    }
    big = na > KD_RUN || nd > KD_RUN;
  }
#ifndef DG_KD_EXP
#define DG_KD_EXP 0  // experiment builds only: 1 no row hashes, 2 no per-key join (wrong results)
#endif
  if (u < p.nk && !big && DG_KD_EXP < 2) {
    // join_dot_sets over the key's rows, both sides in tuple order
    u32 i = 0, j = 0;
    Row ra{}, rb{};
    if (na) ra = load_row(p.a, a_lo);
    if (nd) rb = load_row(p.d, d_lo);
    while (i < na || j < nd) {
      int c;  // -1: the state row first, 1: the delta row first, 0: the same row
      if (i >= na) {
        c = 1;
      } else if (j >= nd) {
        c = -1;
      } else {
        bool lt, eq;
        row_cmp_bf(ra, rb, lt, eq);
        c = eq ? 0 : (lt ? -1 : 1);
      }
      if (c <= 0) {
        // the state's row: kept if the delta has it too, or the delta's context does not
        // cover its dot (Dots.member?, :67-73)
        const bool keep = c == 0 || !(dvv ? vv_covers(tabD, p.cd, ra.node, ra.cnt)
                                          : ctx_covers(p.cd.node, p.cd.cnt, p.cd.n, 1, ra.node, ra.cnt));
        if (keep) {
          am |= 1ull << i;
          ne++;
        } else {
          chg = true;
          if (p.has_tree && DG_KD_EXP == 0) dh -= rhash(p.t, ra);
        }
        if (c == 0 && ++j < nd) rb = load_row(p.d, d_lo + j);
        if (++i < na) ra = load_row(p.a, a_lo + i);
      } else {
        // the delta's row only: kept unless the state's context covers it
        if (!vv_covers(tabS, p.ca, rb.node, rb.cnt)) {
          dm |= 1ull << j;
          ne++;
          chg = true;
          if (p.has_tree && DG_KD_EXP == 0) dh += rhash(p.t, rb);
        }
        if (++j < nd) rb = load_row(p.d, d_lo + j);
      }
    }
    p.a_lo[u] = a_lo;
    p.d_lo[u] = d_lo;
    p.amask[u] = am;
    p.dmask[u] = dm;
  }
  KDSTAMP(2, 4);
  if (u < p.nk) {  // (a key over KD_RUN: no change recorded, so the undo skips it too)
    p.runs[u] = big ? 0ull : (na | ((u64)nd << 16) | ((u64)ne << 32) | (chg ? 1ull << 48 : 0ull));
    p.dh[u] = big ? 0ull : dh;
  }
  // the tree's put/delete right away (all or nothing: a guard or an input error found
  // later makes the host undo it, merkle.hip kd_tree_kernel with the opposite sign)
  if (p.has_tree) tree_put(p, u < p.nk && !big, k, chg, dh, (int)ne - (int)na);
  KDSTAMP(2, 5);
  v[0] = na;
  v[1] = ne;
  v[2] = chg ? 1 : 0;
  v[3] = chg ? ne : 0;
  v[4] = nd;
  v[5] = (u64)(i64)((int)(ne > 0) - (int)(na > 0));
  v[6] = (big ? KD_BIG : 0u) | (ne != na ? KD_MOVED : 0u);
#pragma unroll
  for (int q = 0; q < KD_NV; q++) {
    u64 x = v[q];
    if (q < KD_NV - 1) {
#pragma unroll
      for (int d = WAVE / 2; d >= 1; d >>= 1) x += __shfl_xor(x, d, WAVE);
    } else {
      x = __ballot(x & KD_BIG) ? KD_BIG : 0;
      x |= __ballot(v[q] & KD_MOVED) ? KD_MOVED : 0;
    }
    if (lane == 0) red[q][w] = x;
  }
  __syncthreads();
  // the workgroup's figures handed to the last workgroup, which scans them all
  if (tid < KD_NV) {
    u64 s = 0;
#pragma unroll
    for (int x = 0; x < KDB / WAVE; x++) s = tid < KD_NV - 1 ? s + red[tid][x] : (s | red[tid][x]);
    st_ag(p.part + blk * KD_NV + tid, s);
  }
  __syncthreads();
  if (tid == 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    s_last = __hip_atomic_fetch_add(p.arrive, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == p.ntiles - 1;
    if (s_last) __hip_atomic_store(p.arrive, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  KDSTAMP(0, 6);
  if (!s_last) return;
  // ---- the last workgroup: the totals and the guard into the count block: [0] edit rows
  // [2] changed keys [3] their rows [4] guard [5] moved [6] state rows of the keyset [7]
  // distinct-key change (d_counts[1]: the context union's).  (The per-workgroup offsets are
  // summed by the write's workgroups themselves, dg_kdw.h: a scan here was ~3 more round
  // trips on the call's critical path.)
  __shared__ u64 carry[KD_NV];
  {
    u64 x[KD_NV];
#pragma unroll
    for (int q = 0; q < KD_NV; q++) x[q] = 0;
    for (u64 t = tid; t < p.ntiles; t += KDB) {  // (every load of a round issued together)
      u64 y[KD_NV];
#pragma unroll
      for (int q = 0; q < KD_NV; q++) y[q] = ld_ag(p.part + t * KD_NV + q);
#pragma unroll
      for (int q = 0; q < KD_NV; q++) x[q] = q < KD_NV - 1 ? x[q] + y[q] : (x[q] | y[q]);
    }
#pragma unroll
    for (int q = 0; q < KD_NV; q++) {
      if (q < KD_NV - 1) {
#pragma unroll
        for (int d = WAVE / 2; d >= 1; d >>= 1) x[q] += __shfl_xor(x[q], d, WAVE);
      } else {
        x[q] = (__ballot(x[q] & KD_BIG) ? KD_BIG : 0) | (__ballot(x[q] & KD_MOVED) ? KD_MOVED : 0);
      }
      if (lane == 0) red[q][w] = x[q];
    }
    __syncthreads();
    if (tid < KD_NV) {
      u64 c = 0;
#pragma unroll
      for (int i = 0; i < KDB / WAVE; i++) c = tid < KD_NV - 1 ? c + red[tid][i] : (c | red[tid][i]);
      carry[tid] = c;
    }
    __syncthreads();
  }
  if (tid == 0) {
    const u64 n_ak = carry[0], n_e = carry[1], n_chg = carry[2], n_rows = carry[3], n_d = carry[4];
    u64 g = carry[6] & KD_BIG;
    if (n_d != p.d.n) g |= KD_BAD;      // a delta row whose key is outside the keyset
    if (n_chg > p.cap) g |= KD_CAP;     // the caller's changed-key buffer is too small
    p.d_counts[0] = n_e;
    p.d_counts[2] = n_chg;
    p.d_counts[3] = n_rows;
    p.d_counts[4] = g;
    p.d_counts[5] = (carry[6] & KD_MOVED) ? 1 : 0;
    p.d_counts[6] = n_ak;
    p.d_counts[7] = carry[5];
  }
  KDSTAMP(0, 7);
}

}  // namespace

#ifdef DG_STAMPS
extern "C" int dg_debug_kd_stamps(unsigned long long* host, size_t n) {
  if (n > 4096 * 8) n = 4096 * 8;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_kd_stamps), n * 8) == hipSuccess ? 0 : -3;
}
#endif

hipError_t launch_kd_join(const KdArgs& p0, hipStream_t st) {
  KdArgs p = p0;
  p.ntiles = (p.nk + KDB - 1) / KDB;
  if (p.ntiles == 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(kd_count_kernel, dim3((unsigned)(p.ntiles + 1)), dim3(KDB), 0, st, p);  // (+ the union's)
  return hipGetLastError();
}

}  // namespace dg
