// merkle.hip — the MerkleMap role in DeltaCrdt.CausalCrdt sync (reference
// lib/delta_crdt/causal_crdt.ex): MerkleMap.put/delete per changed key (:390-394),
// update_hashes (:94,254), prepare_partial_diff / continue_partial_diff 8 levels per
// message (:96,255) and truncate_diff to max_sync_size (:98,105,206-214).
// merkle_map 0.2.0 is not vendored, so its hash and wire format are "parity unpinned"
// (SURVEY.md §8(c)); the role is reproduced exactly: a key's leaf depends on its raw
// value map (every {v, ts} entry and dot, :392), and two trees differ exactly above
// the keys whose raw value maps differ.
//
// Tree (dg_merkle): the keys whose top `sb` bits equal `shard` (a key-hash shard,
// SURVEY §8(e); sb = 0 covers every key) in 2^depth buckets by the next `depth` bits.
// Key ids are 64-bit hashes, so a bucket is a contiguous row range of the sorted
// store, and the tree keeps NO per-key leaves: the bucket hash is Σ row_hash over the
// bucket's rows (mod 2^64, order-free), a key's leaf Σ row_hash over its rows is
// recomputed from the store where a diff needs it.  Level `depth` holds the buckets,
// parent = node_hash(left, right).  Because node_hash does not depend on position,
// the shard trees of a 2^sb-way split are exactly the level-sb subtrees of the
// unsharded tree (dg_merkle_fold_roots recombines them).
//
// Kernels:
//  * build: one streaming pass over the rows (36 B/row), a wave segmented sum per
//    bucket (plain store for a bucket inside the wave's 64-row chunk, an atomic add
//    for the chunk's first/last run), then ONE fused upsweep launch: every workgroup
//    reduces 2^11 buckets 11 levels in LDS, the last one to finish reduces the rest.
//  * update: one thread per changed key re-hashes the key's rows in the old and the
//    new store and adds the difference to its bucket (put/delete); the upsweep then
//    re-reduces only the 2^11-bucket chunks an update touched (update_hashes).
//  * diff: 256 buckets per workgroup; a workgroup whose level-(depth-8) node matches
//    is skipped, otherwise each differing bucket merges the two stores' rows of the
//    bucket key by key.  count / scan / write passes; keys past `cap` are counted,
//    not written (truncation to max_sync_size).
//  * partial diff: node-form continuations (positions + the sender's hashes at one
//    level) are compared and expanded `levels` levels down; at the bucket level the
//    reply is a leaf-form continuation (the sender's (key, leaf) pairs of the
//    differing buckets), which the peer merges with its own rows into keys.
#include "dg_hash.h"
#include "dg_launch.h"

namespace dg {

namespace {

struct MT {
  u32 depth, sb;
  u64 shard;
  u64* nodes;
};

__device__ __forceinline__ u64 bucket_of(const MT& t, u64 key) {
  return (key << t.sb) >> (64 - t.depth);
}

__device__ __forceinline__ u64 lower_bound_key(const u64* k, u64 n, u64 x) {
  u64 lo = 0, hi = n;
  while (lo < hi) {
    const u64 mid = (lo + hi) >> 1;
    if (k[mid] < x)
      lo = mid + 1;
    else
      hi = mid;
  }
  return lo;
}

// First index of `keys[0, n)` (ascending) at or after bucket b's first key; b may be
// 2^depth (the end of the tree's key range).
__device__ __forceinline__ u64 bucket_start(const MT& t, const u64* keys, u64 n, u64 b) {
  const u32 sh = 64 - t.sb - t.depth;  // >= 20
  if (b >> t.depth) {                  // past the last bucket
    if (t.sb == 0 || t.shard == (1ull << t.sb) - 1) return n;
    return lower_bound_key(keys, n, (t.shard + 1) << (64 - t.sb));
  }
  const u64 base = t.sb ? (t.shard << (64 - t.sb)) : 0ull;
  return lower_bound_key(keys, n, base + (b << sh));
}

__device__ __forceinline__ u64 rh(const Rows& s, u64 i) {
  return row_hash(s.key[i], s.val[i], s.ts[i], s.node[i], s.cnt[i]);
}

// ---------------------------------------------------------------- build
constexpr int BB = 256;  // threads per build workgroup
constexpr int BK = 4;    // 64-row chunks per wave

// Wave-level segmented sum of (bucket, h) over the 64 lanes (lanes ordered by row).
// Returns, in the LAST lane of each run, the run's sum.
__device__ __forceinline__ u64 seg_sum(u64 b, u64 h, int lane) {
#pragma unroll
  for (int d = 1; d < WAVE; d <<= 1) {
    const u64 ob = __shfl_up(b, d, WAVE);
    const u64 oh = __shfl_up(h, d, WAVE);
    if (lane >= d && ob == b) h += oh;
  }
  return h;
}

__global__ __launch_bounds__(BB) void merkle_build_kernel(Rows s, MT t, u64* d_keys, u32* err) {
  const int lane = threadIdx.x & (WAVE - 1);
  const u64 wave = ((u64)blockIdx.x * BB + threadIdx.x) / WAVE;
  u64* lvl = t.nodes + ((1ull << t.depth) - 1);
  u32 heads = 0;
  bool bad = false;
#pragma unroll
  for (int k = 0; k < BK; k++) {
    const u64 base = (wave * BK + k) * WAVE;
    if (base >= s.n) break;
    const u64 i = base + lane;
    const bool valid = i < s.n;
    u64 key = valid ? s.key[i] : ~0ull, h = 0;
    if (valid) {
      h = row_hash(key, s.val[i], s.ts[i], s.node[i], s.cnt[i]);
      if (t.sb && (key >> (64 - t.sb)) != t.shard) bad = true;
    }
    // (every shuffle runs in all lanes: a shuffle from an inactive lane is undefined)
    const u64 up = __shfl_up(key, 1, WAVE);
    const u64 prev_key = lane ? up : (i > 0 && valid ? s.key[i - 1] : ~key);
    heads += (valid && (i == 0 || prev_key != key)) ? 1u : 0u;
    const u64 b = valid ? bucket_of(t, key) : ~0ull;
    const u64 sum = seg_sum(b, h, lane);
    const u64 nb = __shfl_down(b, 1, WAVE);
    const u64 first_b = __shfl(b, 0, WAVE);
    const u64 end_b = __shfl(b, WAVE - 1, WAVE);
    const bool last = valid && (lane == WAVE - 1 || nb != b);  // last lane of its run
    if (last) {
      // a run that touches the chunk's first or last row may share its bucket with the
      // neighbouring chunk: atomic add (the level was zeroed); an inner run owns it
      const bool shared = b == first_b || b == end_b || i + 1 == s.n;
      if (shared)
        atomicAdd((unsigned long long*)&lvl[b], (unsigned long long)sum);
      else
        lvl[b] = sum;
    }
  }
  // distinct keys: wave sum of heads -> one atomic per wave
  u32 c = heads;
#pragma unroll
  for (int d = WAVE / 2; d >= 1; d >>= 1) c += __shfl_xor(c, d, WAVE);
  if (lane == 0 && c) atomicAdd((unsigned long long*)d_keys, (unsigned long long)c);
  if (__ballot(bad) && lane == 0) atomicOr(err, 2u);
}

// ---------------------------------------------------------------- upsweep
constexpr int UPB = 512;   // threads per upsweep workgroup
constexpr int UPL = 11;    // levels reduced per workgroup (2048 nodes in LDS)
constexpr u32 UPW = 1u << UPL;

// Reduce `width` (power of two, <= UPW) nodes of level `hi` starting at node index g0
// (within the level) by log2(width) levels in LDS, writing every produced level.
__device__ void upsweep_chunk(u64* nodes, u32 hi, u64 g0, u32 width, u64* s) {
  const u64* src = nodes + ((1ull << hi) - 1) + g0;
  for (u32 x = threadIdx.x; x < width; x += UPB) s[x] = src[x];
  __syncthreads();
  u32 l = 0;
  for (u32 cnt = width >> 1; cnt >= 1; cnt >>= 1) {
    l++;
    u64* dst = nodes + ((1ull << (hi - l)) - 1) + (g0 >> l);
    u64 v[UPW / UPB / 2 > 0 ? UPW / UPB / 2 : 1];
    int nv = 0;
    for (u32 x = threadIdx.x; x < cnt; x += UPB) v[nv++] = node_hash(s[2 * x], s[2 * x + 1]);
    __syncthreads();
    nv = 0;
    for (u32 x = threadIdx.x; x < cnt; x += UPB) {
      s[x] = v[nv];
      dst[x] = v[nv++];
    }
    __syncthreads();
  }
}

// Workgroup g reduces buckets [g * 2^L1, (g+1) * 2^L1) (L1 = min(UPL, depth)) when its
// chunk is dirty (dirty == nullptr: every chunk); the last workgroup to finish reduces
// the 2^(depth - L1) chunk roots to the root.  ctr is left at 0.
__global__ __launch_bounds__(UPB) void merkle_upsweep_kernel(u64* nodes, u32 depth, u32* dirty,
                                                             u32* ctr) {
  __shared__ u64 s[UPW];
  __shared__ u32 s_last;
  const u32 L1 = depth < (u32)UPL ? depth : (u32)UPL;
  const u64 g = blockIdx.x;
  const bool work = dirty == nullptr || dirty[g] != 0;
  if (work) upsweep_chunk(nodes, depth, g << L1, 1u << L1, s);
  __threadfence();  // every thread's node stores complete before the block signals
  __syncthreads();
  if (threadIdx.x == 0) {
    if (dirty) dirty[g] = 0;
    const u32 done = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    s_last = done == gridDim.x - 1;
  }
  __syncthreads();
  if (!s_last) return;
  __threadfence();
  // the remaining levels: depth - L1 -> 0, UPL levels per round
  u32 hi = depth - L1;
  while (hi > 0) {
    const u32 nlev = hi < (u32)UPL ? hi : (u32)UPL;
    const u64 chunks = 1ull << (hi - nlev);
    for (u64 c = 0; c < chunks; c++) upsweep_chunk(nodes, hi, c << nlev, 1u << nlev, s);
    hi -= nlev;
  }
  if (threadIdx.x == 0) __hip_atomic_store(ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ---------------------------------------------------------------- update
constexpr int UB = 256;

// Σ row_hash of key x's rows in s (0 if absent); *present = x has rows.
__device__ __forceinline__ u64 key_leaf(const Rows& s, u64 x, bool* present) {
  u64 i = lower_bound_key(s.key, s.n, x);
  u64 h = 0;
  *present = i < s.n && s.key[i] == x;
  for (; i < s.n && s.key[i] == x; i++) h += rh(s, i);
  return h;
}

__global__ __launch_bounds__(UB) void merkle_update_kernel(MT t, Rows olds, Rows news, const u64* keys,
                                                           u64 n_keys, u32* dirty, u64* d_keys,
                                                           u32* err) {
  const u64 i = (u64)blockIdx.x * UB + threadIdx.x;
  int dk = 0;
  bool bad = false;
  if (i < n_keys) {
    const u64 x = keys[i];
    bool po, pn;
    const u64 ho = key_leaf(olds, x, &po), hn = key_leaf(news, x, &pn);
    dk = (int)pn - (int)po;
    if (ho != hn || po != pn) {
      if (t.sb && (x >> (64 - t.sb)) != t.shard) {
        bad = true;
      } else {
        const u64 b = bucket_of(t, x);
        u64* lvl = t.nodes + ((1ull << t.depth) - 1);
        atomicAdd((unsigned long long*)&lvl[b], (unsigned long long)(hn - ho));
        const u32 L1 = t.depth < (u32)UPL ? t.depth : (u32)UPL;
        dirty[b >> L1] = 1u;
      }
    }
  }
  int c = dk;
#pragma unroll
  for (int d = WAVE / 2; d >= 1; d >>= 1) c += __shfl_xor(c, d, WAVE);
  if ((threadIdx.x & (WAVE - 1)) == 0 && c)
    atomicAdd((unsigned long long*)d_keys, (unsigned long long)(long long)c);
  if (__ballot(bad) && (threadIdx.x & (WAVE - 1)) == 0) atomicOr(err, 2u);
}

// ---------------------------------------------------------------- key-level merge
// Merge keys[ia, ie) of store A (rows) with B, where B is either a store (rows) or a
// list of (key, leaf) pairs; emit the keys present on one side only or with different
// leaves.  WRITE: store them at out[o..) (only below cap); returns the count.
template <bool B_LEAVES, bool WRITE>
__device__ u32 merge_bucket(const Rows& A, u64 ia, u64 ie, const Rows& B, const u64* bk,
                            const u64* bh, u64 jb, u64 je, u64* out, u64 o, u64 cap) {
  u32 c = 0;
  while (ia < ie || jb < je) {
    const u64 ka = ia < ie ? A.key[ia] : ~0ull;
    const u64 kb = jb < je ? (B_LEAVES ? bk[jb] : B.key[jb]) : ~0ull;
    const bool has_a = ia < ie && (jb >= je || ka <= kb);
    const bool has_b = jb < je && (ia >= ie || kb <= ka);
    const u64 k = has_a ? ka : kb;
    u64 ha = 0, hb = 0;
    if (has_a)
      for (; ia < ie && A.key[ia] == k; ia++) ha += rh(A, ia);
    if (has_b) {
      if (B_LEAVES) {
        hb = bh[jb++];
      } else {
        for (; jb < je && B.key[jb] == k; jb++) hb += rh(B, jb);
      }
    }
    if (!(has_a && has_b) || ha != hb) {
      if (WRITE && o + c < cap) out[o + c] = k;
      c++;
    }
  }
  return c;
}

// ---------------------------------------------------------------- full diff
constexpr int DB = DIFF_BLOCK;

struct DiffArgs {
  MT ta, tb;
  Rows sa, sb;
  u64* out;
  u64 cap;
  u64* cnt;  // differing keys per tile
  u64* off;  // their output offset
  u32* bc;   // differing keys per bucket (the count pass's walk, reused by the write pass)
  u64 ntiles;
  u64* d_count;
};

__device__ __forceinline__ u64 diff_bpt(u32 depth) { return depth >= 8 ? 256ull : (1ull << depth); }

__device__ __forceinline__ u64 diff_bucket_of(const DiffArgs& p, u64 tile, int tid, bool* walk) {
  const u32 depth = p.ta.depth;
  const u32 rl = depth >= 8 ? depth - 8 : 0;  // subtree root level
  const u64 root = ((1ull << rl) - 1) + tile;
  const u64 nbk = 1ull << depth;
  const u64 b = tile * diff_bpt(depth) + tid;
  *walk = false;
  if ((u64)tid < diff_bpt(depth) && p.ta.nodes[root] != p.tb.nodes[root]) {
    const u64 leaf = (nbk - 1) + b;
    *walk = p.ta.nodes[leaf] != p.tb.nodes[leaf];
  }
  return b;
}

template <bool WRITE>
__device__ __forceinline__ u32 diff_walk(const DiffArgs& p, u64 b, u64 o) {
  const u64 ia = bucket_start(p.ta, p.sa.key, p.sa.n, b), ie = bucket_start(p.ta, p.sa.key, p.sa.n, b + 1);
  const u64 jb = bucket_start(p.tb, p.sb.key, p.sb.n, b), je = bucket_start(p.tb, p.sb.key, p.sb.n, b + 1);
  return merge_bucket<false, WRITE>(p.sa, ia, ie, p.sb, nullptr, nullptr, jb, je, p.out, o, p.cap);
}

__global__ __launch_bounds__(DB) void merkle_diff_count_kernel(DiffArgs p) {
  __shared__ u32 s_wave[DB / WAVE + 1];
  bool walk;
  const u64 b = diff_bucket_of(p, blockIdx.x, threadIdx.x, &walk);
  const u32 c = walk ? diff_walk<false>(p, b, 0) : 0u;
  if ((u64)threadIdx.x < diff_bpt(p.ta.depth)) p.bc[b] = c;
  u32 tot;
  block_excl_scan<DB>(c, s_wave, &tot);
  if (threadIdx.x == 0) p.cnt[blockIdx.x] = tot;
}

constexpr int DSB = 1024;
__global__ __launch_bounds__(DSB) void tile_scan_kernel(const u64* cnt, u64* off, u64 ntiles,
                                                        u64* d_count) {
  __shared__ u32 s_wave[DSB / WAVE + 1];
  __shared__ u64 s_carry;
  scan_tile_counts<DSB>(cnt, off, ntiles, d_count, s_wave, &s_carry);
}

__global__ __launch_bounds__(DB) void merkle_diff_write_kernel(DiffArgs p) {
  __shared__ u32 s_wave[DB / WAVE + 1];
  const u64 bpt = diff_bpt(p.ta.depth);
  const u64 b = blockIdx.x * bpt + threadIdx.x;
  const u32 c = (u64)threadIdx.x < bpt ? p.bc[b] : 0u;
  u32 tot;
  const u32 ex = block_excl_scan<DB>(c, s_wave, &tot);
  const u64 o = p.off[blockIdx.x] + ex;
  if (c && o < p.cap) diff_walk<true>(p, b, o);
}

// ---------------------------------------------------------------- partial diff
// Node form: entry i = (pos[i], hash[i]) at level L.  Flag the entries whose own node
// differs; count / scan / compact their positions.
constexpr int PB = 256;

__global__ __launch_bounds__(PB) void cont_count_kernel(MT t, u32 L, const u64* pos, const u64* hash,
                                                        u64 n, u64* cnt) {
  __shared__ u32 s_wave[PB / WAVE + 1];
  const u64 i = (u64)blockIdx.x * PB + threadIdx.x;
  u32 d = 0;
  if (i < n) d = t.nodes[((1ull << L) - 1) + pos[i]] != hash[i] ? 1u : 0u;
  u32 tot;
  block_excl_scan<PB>(d, s_wave, &tot);
  if (threadIdx.x == 0) cnt[blockIdx.x] = tot;
}

__global__ __launch_bounds__(PB) void cont_compact_kernel(MT t, u32 L, const u64* pos, const u64* hash,
                                                          u64 n, const u64* off, u64* dpos) {
  __shared__ u32 s_wave[PB / WAVE + 1];
  const u64 i = (u64)blockIdx.x * PB + threadIdx.x;
  u32 d = 0;
  if (i < n) d = t.nodes[((1ull << L) - 1) + pos[i]] != hash[i] ? 1u : 0u;
  u32 tot;
  const u32 ex = block_excl_scan<PB>(d, s_wave, &tot);
  if (d) dpos[off[blockIdx.x] + ex] = pos[i];
}

// Children at level L + k of the m differing positions: out entry j = child (j & (2^k-1))
// of dpos[j >> k], with this tree's hash.
__global__ __launch_bounds__(PB) void cont_expand_kernel(MT t, u32 L, u32 k, const u64* dpos, u64 m,
                                                         u64* opos, u64* ohash) {
  const u64 j = (u64)blockIdx.x * PB + threadIdx.x;
  if (j >= (m << k)) return;
  const u64 p = (dpos[j >> k] << k) | (j & ((1ull << k) - 1));
  opos[j] = p;
  ohash[j] = t.nodes[((1ull << (L + k)) - 1) + p];
}

// Leaf form, built by the side that found differing buckets: per bucket its distinct
// keys (count pass) and then (key, leaf) pairs at the bucket's offset (write pass).
template <bool WRITE>
__global__ __launch_bounds__(PB) void leaves_kernel(MT t, Rows s, const u64* buckets, u64 nb,
                                                    u64* cnt, const u64* off, u64* ok, u64* oh) {
  __shared__ u32 s_wave[PB / WAVE + 1];
  const u64 i = (u64)blockIdx.x * PB + threadIdx.x;
  u64 r = 0, re = 0;
  u32 c = 0;
  if (i < nb) {
    r = bucket_start(t, s.key, s.n, buckets[i]);
    re = bucket_start(t, s.key, s.n, buckets[i] + 1);
    for (u64 x = r; x < re; x++) c += (x == r || s.key[x] != s.key[x - 1]) ? 1u : 0u;
  }
  u32 tot;
  const u32 ex = block_excl_scan<PB>(c, s_wave, &tot);
  if (!WRITE) {
    if (threadIdx.x == 0) cnt[blockIdx.x] = tot;
    return;
  }
  u64 o = off[blockIdx.x] + ex;
  for (u64 x = r; x < re;) {
    const u64 k = s.key[x];
    u64 h = 0;
    for (; x < re && s.key[x] == k; x++) h += rh(s, x);
    ok[o] = k;
    oh[o++] = h;
  }
}

// Leaf form received: per listed bucket, merge the peer's (key, leaf) pairs with this
// store's rows of the bucket; count / write the differing keys.
template <bool WRITE>
__global__ __launch_bounds__(PB) void leafdiff_kernel(MT t, Rows s, const u64* buckets, u64 nb,
                                                      const u64* pk, const u64* ph, u64 np, u64* cnt,
                                                      const u64* off, u64* out, u64 cap) {
  __shared__ u32 s_wave[PB / WAVE + 1];
  const u64 i = (u64)blockIdx.x * PB + threadIdx.x;
  u64 r = 0, re = 0, j = 0, je = 0;
  u32 c = 0;
  if (i < nb) {
    const u64 b = buckets[i];
    r = bucket_start(t, s.key, s.n, b);
    re = bucket_start(t, s.key, s.n, b + 1);
    j = bucket_start(t, pk, np, b);
    je = bucket_start(t, pk, np, b + 1);
    c = merge_bucket<true, false>(s, r, re, s, pk, ph, j, je, nullptr, 0, 0);
  }
  u32 tot;
  const u32 ex = block_excl_scan<PB>(c, s_wave, &tot);
  if (!WRITE) {
    if (threadIdx.x == 0) cnt[blockIdx.x] = tot;
    return;
  }
  const u64 o = off[blockIdx.x] + ex;
  if (c && o < cap) merge_bucket<true, true>(s, r, re, s, pk, ph, j, je, out, o, cap);
}

__global__ void pairs_before_kernel(MT t, const u64* keys, u64 n, const u64* bucket, u64* out) {
  if (threadIdx.x == 0) out[0] = bucket_start(t, keys, n, bucket[0]);
}

MT mt_of(const MerkleT& m) {
  MT t;
  t.depth = m.depth;
  t.sb = m.sb;
  t.shard = m.shard;
  t.nodes = m.nodes;
  return t;
}

inline unsigned grid_of(u64 n, int b) { return (unsigned)((n + b - 1) / b); }

}  // namespace

hipError_t launch_merkle_build(const Rows& s, const MerkleT& m, u64* d_keys, u32* ctr, u32* err,
                               hipStream_t st) {
  const MT t = mt_of(m);
  const u64 nb = 1ull << t.depth;
  hipError_t e = hipMemsetAsync(t.nodes + (nb - 1), 0, nb * sizeof(u64), st);
  if (e != hipSuccess) return e;
  e = hipMemsetAsync(d_keys, 0, sizeof(u64), st);
  if (e != hipSuccess) return e;
  if (s.n) {
    const u64 rows_per_block = (u64)BB * BK;
    hipLaunchKernelGGL(merkle_build_kernel, dim3(grid_of(s.n, (int)rows_per_block)), dim3(BB), 0, st,
                       s, t, d_keys, err);
  }
  const u32 L1 = t.depth < (u32)UPL ? t.depth : (u32)UPL;
  hipLaunchKernelGGL(merkle_upsweep_kernel, dim3((unsigned)(1ull << (t.depth - L1))), dim3(UPB), 0, st,
                     t.nodes, t.depth, (u32*)nullptr, ctr);
  return hipGetLastError();
}

hipError_t launch_merkle_update(const MerkleT& m, const Rows& olds, const Rows& news, const u64* keys,
                                u64 n_keys, u32* dirty, u64* d_keys, u32* ctr, u32* err,
                                hipStream_t st) {
  const MT t = mt_of(m);
  const u32 L1 = t.depth < (u32)UPL ? t.depth : (u32)UPL;
  const u64 chunks = 1ull << (t.depth - L1);
  if (n_keys)
    hipLaunchKernelGGL(merkle_update_kernel, dim3(grid_of(n_keys, UB)), dim3(UB), 0, st, t, olds, news,
                       keys, n_keys, dirty, d_keys, err);
  hipLaunchKernelGGL(merkle_upsweep_kernel, dim3((unsigned)chunks), dim3(UPB), 0, st, t.nodes, t.depth,
                     dirty, ctr);
  return hipGetLastError();
}

hipError_t launch_merkle_diff(const MerkleT& a, const Rows& sa, const MerkleT& b, const Rows& sb,
                              u64* out_keys, u64 cap, u64* scratch, u64* d_count, hipStream_t st) {
  DiffArgs p;
  p.ta = mt_of(a);
  p.tb = mt_of(b);
  p.sa = sa;
  p.sb = sb;
  p.out = out_keys;
  p.cap = cap;
  p.ntiles = diff_tiles(a.depth);
  p.cnt = scratch;
  p.off = scratch + p.ntiles;
  p.bc = (u32*)(scratch + 2 * p.ntiles);
  p.d_count = d_count;
  hipLaunchKernelGGL(merkle_diff_count_kernel, dim3((unsigned)p.ntiles), dim3(DB), 0, st, p);
  hipLaunchKernelGGL(tile_scan_kernel, dim3(1), dim3(DSB), 0, st, p.cnt, p.off, p.ntiles, d_count);
  hipLaunchKernelGGL(merkle_diff_write_kernel, dim3((unsigned)p.ntiles), dim3(DB), 0, st, p);
  return hipGetLastError();
}

hipError_t launch_cont_compare(const MerkleT& m, u32 L, const u64* pos, const u64* hash, u64 n,
                               u64* scratch, u64* dpos, u64* d_count, hipStream_t st) {
  const MT t = mt_of(m);
  const u64 tiles = (n + PB - 1) / PB;
  if (n == 0) return hipMemsetAsync(d_count, 0, sizeof(u64), st);
  hipLaunchKernelGGL(cont_count_kernel, dim3((unsigned)tiles), dim3(PB), 0, st, t, L, pos, hash, n,
                     scratch);
  hipLaunchKernelGGL(tile_scan_kernel, dim3(1), dim3(DSB), 0, st, scratch, scratch + tiles, tiles,
                     d_count);
  hipLaunchKernelGGL(cont_compact_kernel, dim3((unsigned)tiles), dim3(PB), 0, st, t, L, pos, hash, n,
                     scratch + tiles, dpos);
  return hipGetLastError();
}

hipError_t launch_cont_expand(const MerkleT& m, u32 L, u32 k, const u64* dpos, u64 nd, u64* opos,
                              u64* ohash, hipStream_t st) {
  if (nd == 0) return hipSuccess;
  hipLaunchKernelGGL(cont_expand_kernel, dim3(grid_of(nd << k, PB)), dim3(PB), 0, st, mt_of(m), L, k,
                     dpos, nd, opos, ohash);
  return hipGetLastError();
}

hipError_t launch_leaves_count(const MerkleT& m, const Rows& s, const u64* buckets, u64 nb,
                               u64* scratch, u64* d_count, hipStream_t st) {
  const u64 tiles = (nb + PB - 1) / PB;
  if (nb == 0) return hipMemsetAsync(d_count, 0, sizeof(u64), st);
  hipLaunchKernelGGL(leaves_kernel<false>, dim3((unsigned)tiles), dim3(PB), 0, st, mt_of(m), s, buckets,
                     nb, scratch, (const u64*)nullptr, (u64*)nullptr, (u64*)nullptr);
  hipLaunchKernelGGL(tile_scan_kernel, dim3(1), dim3(DSB), 0, st, scratch, scratch + tiles, tiles,
                     d_count);
  return hipGetLastError();
}

hipError_t launch_leaves_write(const MerkleT& m, const Rows& s, const u64* buckets, u64 nb,
                               const u64* scratch, u64* ok, u64* oh, hipStream_t st) {
  const u64 tiles = (nb + PB - 1) / PB;
  if (nb == 0) return hipSuccess;
  hipLaunchKernelGGL(leaves_kernel<true>, dim3((unsigned)tiles), dim3(PB), 0, st, mt_of(m), s, buckets,
                     nb, (u64*)nullptr, scratch + tiles, ok, oh);
  return hipGetLastError();
}

hipError_t launch_leafdiff(const MerkleT& m, const Rows& s, const u64* buckets, u64 nb, const u64* pk,
                           const u64* ph, u64 np, u64* out, u64 cap, u64* scratch, u64* d_count,
                           hipStream_t st) {
  const u64 tiles = (nb + PB - 1) / PB;
  if (nb == 0) return hipMemsetAsync(d_count, 0, sizeof(u64), st);
  const MT t = mt_of(m);
  hipLaunchKernelGGL(leafdiff_kernel<false>, dim3((unsigned)tiles), dim3(PB), 0, st, t, s, buckets, nb,
                     pk, ph, np, scratch, (const u64*)nullptr, (u64*)nullptr, (u64)0);
  hipLaunchKernelGGL(tile_scan_kernel, dim3(1), dim3(DSB), 0, st, scratch, scratch + tiles, tiles,
                     d_count);
  hipLaunchKernelGGL(leafdiff_kernel<true>, dim3((unsigned)tiles), dim3(PB), 0, st, t, s, buckets, nb,
                     pk, ph, np, (u64*)nullptr, scratch + tiles, out, cap);
  return hipGetLastError();
}

hipError_t launch_pairs_before_bucket(const MerkleT& m, const u64* keys, u64 n, const u64* bucket,
                                     u64* d_count, hipStream_t st) {
  hipLaunchKernelGGL(pairs_before_kernel, dim3(1), dim3(64), 0, st, mt_of(m), keys, n, bucket, d_count);
  return hipGetLastError();
}

}  // namespace dg
