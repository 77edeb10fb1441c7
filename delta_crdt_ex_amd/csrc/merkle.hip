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
//  * build: ONE launch.  A workgroup per chunk of 2^11 buckets streams the chunk's rows
//    (36 B/row; the row range from two wave lower bounds) into LDS bucket sums, reduces
//    the chunk's 11 levels in LDS and writes them; the last workgroup to finish (one
//    arrival counter, write-through hand-off words) reduces the chunk roots to the root.
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

// ---------------------------------------------------------------- lower bounds
// wave_lower_bound of bucket b's first key (b may be 2^depth: the end of the range).
__device__ __forceinline__ u64 wave_bucket_start(const MT& t, const u64* keys, u64 n, u64 b) {
  if (b >> t.depth) {
    if (t.sb == 0 || t.shard == (1ull << t.sb) - 1) return n;
    return wave_lower_bound(keys, n, (t.shard + 1) << (64 - t.sb));
  }
  const u64 base = t.sb ? (t.shard << (64 - t.sb)) : 0ull;
  return wave_lower_bound(keys, n, base + (b << (64 - t.sb - t.depth)));
}

// ---------------------------------------------------------------- build / upsweep
// One workgroup per chunk of 2^L1 buckets (L1 = min(UPL, depth)).  BUILD: the chunk's
// rows (a contiguous range: two wave lower bounds) are hashed into LDS bucket sums
// (LDS atomic adds; no global atomics), UPDATE: the chunk's bucket level is read back
// (merkle_update_kernel has added the changed keys' deltas) -- only where the chunk is
// dirty.  Then L1 levels are reduced in LDS and written.  The last workgroup to finish
// reduces the chunk roots to the root and, for BUILD, sums the per-chunk distinct-key
// counts.  Hand-off (MI355X_MICROARCH.md "Valid forms", hand-off table row 1): ONE lane
// per workgroup stores the chunk's root and key count write-through (sc1), waits for
// them, then adds to ONE arrival counter; the workgroup whose add returns last reads the
// roots and counts with sc1 loads.  No release fence per workgroup: an agent release
// in each of 2048 workgroups cost 75 us of a 219 us build (rocprofv3 A/B).
constexpr int UPB = 512;   // threads per chunk workgroup
constexpr int UPL = MERKLE_UPL;  // levels reduced per workgroup (2048 nodes in LDS)
constexpr u32 UPW = 1u << UPL;

__device__ __forceinline__ void wait_vmem() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

__device__ __forceinline__ void st_sc1(u64* p, u64 v) {
  __hip_atomic_store((__attribute__((address_space(1))) u64*)p, v, __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ u64 ld_sc1(const u64* p) {
  return __hip_atomic_load((__attribute__((address_space(1))) u64*)p, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
}

// s[0, width) holds level `hi` nodes g0 .. g0+width-1; reduce log2(width) levels in LDS
// and write every produced level (s ends with the subtree root in s[0]).
__device__ void lds_upsweep(u64* nodes, u32 hi, u64 g0, u32 width, u64* s) {
  u32 l = 0;
  for (u32 cnt = width >> 1; cnt >= 1; cnt >>= 1) {
    l++;
    u64* dst = nodes + ((1ull << (hi - l)) - 1) + (g0 >> l);
    u64 v[UPW / UPB / 2];
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

// scratch: ctr[0] the arrival counter (zeroed before the launch), then per chunk its
// root and its distinct-key count (u64 each, at hand[0, G) and hand[G, 2G)).
template <bool BUILD>
__global__ __launch_bounds__(UPB) void merkle_chunk_kernel(Rows rows, MT t, const u32* dirty,
                                                           u32* ctr, u64* hand, u64* d_keys,
                                                           u32* err) {
  __shared__ u64 s[UPW];
  __shared__ u64 s_rng[2];
  __shared__ u32 s_red[UPB / WAVE];
  __shared__ u32 s_last;
  const u32 L1 = t.depth < (u32)UPL ? t.depth : (u32)UPL;
  const u32 width = 1u << L1;
  const u64 g = blockIdx.x, g0 = g << L1, G = gridDim.x;
  const int tid = threadIdx.x, lane = tid & (WAVE - 1), w = tid / WAVE;
  u64* lvl = t.nodes + ((1ull << t.depth) - 1);
  u64 chunk_root = 0, chunk_keys = 0;
  if (BUILD) {
    for (u32 x = tid; x < width; x += UPB) s[x] = 0;
    if (w < 2) {
#ifdef MK_INTERP  // timing experiment only: interpolated (inexact) chunk bounds
      const u64 r = (u64)((double)rows.n * (double)(g + w) / (double)gridDim.x);
#else
      const u64 r = wave_bucket_start(t, rows.key, rows.n, g0 + (w ? width : 0));
#endif
      if (lane == 0) s_rng[w] = r;
    }
    __syncthreads();
    const u64 lo = s_rng[0], hi = s_rng[1];
    u32 heads = 0;
    // rows outside the tree's key range (before the first chunk, after the last one)
    bool bad = tid == 0 && ((g == 0 && lo > 0) || (g == G - 1 && hi < rows.n));
    for (u64 i0 = lo; i0 < hi; i0 += 4 * UPB) {
      u64 key[4], h[4];
      bool head[4];
#pragma unroll
      for (int q = 0; q < 4; q++) {  // four rows in flight per thread
        const u64 i = i0 + (u64)q * UPB + tid;
        key[q] = 0;
        h[q] = 0;
        head[q] = false;
        if (i < hi) {
          key[q] = rows.key[i];
          h[q] = row_hash(key[q], rows.val[i], rows.ts[i], rows.node[i], rows.cnt[i]);
          head[q] = i == lo || rows.key[i - 1] != key[q];
        }
      }
#pragma unroll
      for (int q = 0; q < 4; q++) {
        const u64 i = i0 + (u64)q * UPB + tid;
        if (i < hi) {
          if (t.sb && (key[q] >> (64 - t.sb)) != t.shard) bad = true;
          const u64 b = bucket_of(t, key[q]) - g0;
          if (b < width) atomicAdd((unsigned long long*)&s[b], (unsigned long long)h[q]);
          heads += head[q] ? 1u : 0u;
        }
      }
    }
    // distinct keys of the chunk (keys of different chunks differ: a key fixes its bucket)
    u32 c = heads;
#pragma unroll
    for (int d = WAVE / 2; d >= 1; d >>= 1) c += __shfl_xor(c, d, WAVE);
    if (lane == 0) s_red[w] = c;
    if (__ballot(bad) && lane == 0) atomicOr(err, 2u);
    __syncthreads();
    if (tid == 0)
      for (int q = 0; q < UPB / WAVE; q++) chunk_keys += s_red[q];
    for (u32 x = tid; x < width; x += UPB) lvl[g0 + x] = s[x];
#ifndef MK_NO_UPSWEEP  // timing experiment only
    lds_upsweep(t.nodes, t.depth, g0, width, s);
#endif
    chunk_root = s[0];
  } else if (dirty[g]) {
    for (u32 x = tid; x < width; x += UPB) s[x] = lvl[g0 + x];
    __syncthreads();
    lds_upsweep(t.nodes, t.depth, g0, width, s);
    chunk_root = s[0];
  } else if (tid == 0) {  // unchanged: its root as the previous kernels left it
    chunk_root = t.nodes[((1ull << (t.depth - L1)) - 1) + g];
  }
  // ---- hand the chunk root (and key count) to the last workgroup
  if (tid == 0) {
    st_sc1(hand + g, chunk_root);
    if (BUILD) st_sc1(hand + G + g, chunk_keys);
    wait_vmem();
    s_last = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == G - 1;
  }
  __syncthreads();
  if (!s_last) return;
  // ---- the last workgroup: levels depth - L1 .. 0, UPL levels per round; the first
  // round's inputs are the handed-off chunk roots (sc1 loads)
  u32 hl = t.depth - L1;
  bool first = true;
  while (hl > 0) {
    const u32 nlev = hl < (u32)UPL ? hl : (u32)UPL;
    const u64 chunks = 1ull << (hl - nlev);
    const u64* src = t.nodes + ((1ull << hl) - 1);
    wait_vmem();  // this workgroup's own stores of level hl (depth > 2 * UPL) are complete
    __syncthreads();
    for (u64 c = 0; c < chunks; c++) {
      for (u32 x = tid; x < (1u << nlev); x += UPB)
        s[x] = first ? ld_sc1(hand + (c << nlev) + x) : src[(c << nlev) + x];
      __syncthreads();
      lds_upsweep(t.nodes, hl, c << nlev, 1u << nlev, s);
    }
    hl -= nlev;
    first = false;
  }
  if (BUILD) {
    u64 sum = 0;
    for (u64 x = tid; x < G; x += UPB) sum += ld_sc1(hand + G + x);
#pragma unroll
    for (int d = WAVE / 2; d >= 1; d >>= 1) sum += __shfl_xor(sum, d, WAVE);
    __syncthreads();
    if (lane == 0) s[w] = sum;
    __syncthreads();
    if (tid == 0) {
      u64 tot = 0;
      for (int q = 0; q < UPB / WAVE; q++) tot += s[q];
      *d_keys = tot;
    }
  }
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
  // 8 count shards (one word takes ~88 same-address atomics per us): d_keys[0, 8)
  if ((threadIdx.x & (WAVE - 1)) == 0 && c)
    atomicAdd((unsigned long long*)&d_keys[(blockIdx.x * (UB / WAVE) + threadIdx.x / WAVE) & 7],
              (unsigned long long)(long long)c);
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
// Tiles of 256 buckets, one thread per bucket.
//  1. bounds: one wave per tile boundary finds the boundary's first row in both stores
//     (a 64-ary wave lower bound: 4 dependent load rounds at 12.5M rows).
//  2. count: a tile whose level-(depth-8) subtree root matches in both trees is
//     skipped.  Otherwise the tile's key columns are staged in LDS, each thread finds its
//     bucket's rows there, the rows of the DIFFERING buckets are listed and hashed by
//     all threads at once (one round of independent loads instead of a dependent chain
//     per bucket), and each differing bucket merges its keys' leaves from LDS.  The
//     tile's differing keys go to scratch at (A start + B start) of the tile, which is
//     unique and increasing across tiles.
//  3. scan of the per-tile counts; 4. copy: each tile's keys to their output offset,
//     the keys past `cap` counted, not written (truncation to max_sync_size).
// A tile whose rows do not fit the LDS stage (far fewer buckets than keys/3) falls back
// to per-bucket merges over global memory.
constexpr int DB = DIFF_BLOCK;
constexpr u32 DCAP = 1024;  // rows per store staged in LDS
constexpr u32 LCAP = 512;   // rows of a tile's differing buckets hashed through LDS

struct DiffArgs {
  MT ta, tb;
  Rows sa, sb;
  u64* out;
  u64 cap;
  u64* bnd;   // ntiles + 1 boundaries x 2 stores: first row of each tile in A, then in B
  u64* cnt;   // differing keys per tile
  u64* off;   // their output offset
  u64* keys;  // scratch: nA + nB keys
  u64* bsum;  // per DB tiles: the sum of their counts (zeroed before the count kernel)
  u64 ntiles;
  u64* d_count;
};

__device__ __forceinline__ u64 diff_bpt(u32 depth) { return depth >= 8 ? 256ull : (1ull << depth); }

// lower bound of x in keys[0, n) (LDS or global; n small)
__device__ __forceinline__ u32 lb_small(const u64* k, u32 n, u64 x) {
  u32 lo = 0, hi = n;
  while (lo < hi) {
    const u32 mid = (lo + hi) >> 1;
    if (k[mid] < x)
      lo = mid + 1;
    else
      hi = mid;
  }
  return lo;
}

__device__ __forceinline__ u64 bucket_first_key(const MT& t, u64 b) {
  const u64 base = t.sb ? (t.shard << (64 - t.sb)) : 0ull;
  return base + (b << (64 - t.sb - t.depth));
}

__global__ __launch_bounds__(256) void merkle_diff_bounds_kernel(DiffArgs p) {
  const u64 i = ((u64)blockIdx.x * 256 + threadIdx.x) / WAVE;  // one wave per boundary
  const u64 nbnd = p.ntiles + 1;
  if (i >= 2 * nbnd) return;  // uniform per wave
  const bool B = i >= nbnd;
  const u64 t = B ? i - nbnd : i;
  const Rows& r = B ? p.sb : p.sa;
  const u64 x = wave_bucket_start(p.ta, r.key, r.n, t * diff_bpt(p.ta.depth));
  if ((threadIdx.x & (WAVE - 1)) == 0) p.bnd[i] = x;
}

__global__ __launch_bounds__(DB) void merkle_diff_count_kernel(DiffArgs p) {
  __shared__ u64 s_ka[DCAP], s_kb[DCAP];
  __shared__ u64 s_h[LCAP];            // hashes of the listed rows, in list order
  __shared__ uint16_t s_list[LCAP];    // the differing buckets' rows: bit 15 = store B
  __shared__ u32 s_wave[DB / WAVE + 1];
  __shared__ u32 s_bc[DB];             // rows per bucket: A in the low, B in the high half
  const u32 depth = p.ta.depth;
  const u64 tile = blockIdx.x, bpt = diff_bpt(depth), b0 = tile * bpt;
  const int tid = threadIdx.x;
  const u32 rl = depth >= 8 ? depth - 8 : 0;
  const u64 root = ((1ull << rl) - 1) + tile;
  const u64 nbnd = p.ntiles + 1;
  const bool in = (u64)tid < bpt;
  const u64 b = b0 + tid;
  const u64 leaf = ((1ull << depth) - 1) + b;
  // one round of independent loads: the subtree roots, the tile's row bounds, the leaves
  const u64 root_a = p.ta.nodes[root], root_b = p.tb.nodes[root];
  const u64 a0 = p.bnd[tile], a1 = p.bnd[tile + 1], c0 = p.bnd[nbnd + tile], c1 = p.bnd[nbnd + tile + 1];
  const u64 leaf_a = in ? p.ta.nodes[leaf] : 0, leaf_b = in ? p.tb.nodes[leaf] : 0;
  if (root_a == root_b) {  // uniform: the whole tile matches
    if (tid == 0) p.cnt[tile] = 0;
    return;
  }
  const u64 base = a0 + c0;
  const u32 na = (u32)(a1 - a0), nc = (u32)(c1 - c0);
  const bool walk = in && leaf_a != leaf_b;
  const bool last = (u64)tid == bpt - 1;
  const u64 lk = bucket_first_key(p.ta, b), hk = last ? 0 : bucket_first_key(p.ta, b + 1);
  bool lds = a1 - a0 <= DCAP && c1 - c0 <= DCAP;  // uniform
  u32 ia = 0, ie = 0, jb = 0, je = 0, r0 = 0;
  if (lds) {
    {  // every staging load in flight at once (DCAP / DB = 4 per store per thread)
      constexpr int Q = DCAP / DB;
      u64 ka[Q], kb[Q];
#pragma unroll
      for (int q = 0; q < Q; q++) {
        const u32 x = q * DB + tid;
        ka[q] = x < na ? p.sa.key[a0 + x] : 0;
        kb[q] = x < nc ? p.sb.key[c0 + x] : 0;
      }
#pragma unroll
      for (int q = 0; q < Q; q++) {
        const u32 x = q * DB + tid;
        if (x < na) s_ka[x] = ka[q];
        if (x < nc) s_kb[x] = kb[q];
      }
      s_bc[tid] = 0;
      __syncthreads();
      // every bucket's row range from a histogram of the staged keys (LDS atomics) and one
      // scan, instead of four binary searches per differing bucket
      const u64 kbase = p.ta.sb ? (p.ta.shard << (64 - p.ta.sb)) : 0ull;
      const u32 sh = 64 - p.ta.sb - depth;
#pragma unroll
      for (int q = 0; q < Q; q++) {
        const u32 x = q * DB + tid;
        const u64 la = ((ka[q] - kbase) >> sh) - b0, lb = ((kb[q] - kbase) >> sh) - b0;
        if (x < na && la < bpt) atomicAdd(&s_bc[la], 1u);  // (bounds: the tile's buckets)
        if (x < nc && lb < bpt) atomicAdd(&s_bc[lb], 1u << 16);
      }
    }
    __syncthreads();
    {
      const u32 bc = in ? s_bc[tid] : 0u;
      u32 tot_bc;
      const u32 st = block_excl_scan<DB>(bc, s_wave, &tot_bc);  // (counts <= DCAP: no carry)
      ia = st & 0xffffu;
      ie = ia + (bc & 0xffffu);
      jb = st >> 16;
      je = jb + (bc >> 16);
      if (!walk) {  // only the differing buckets' rows are listed and merged
        ie = ia;
        je = jb;
      }
    }
    // list the differing buckets' rows, then hash them all at once
    u32 tot_rows;
    r0 = block_excl_scan<DB>((ie - ia) + (je - jb), s_wave, &tot_rows);
    lds = tot_rows <= LCAP;  // uniform
    if (lds) {
      u32 o = r0;
      for (u32 x = ia; x < ie; x++) s_list[o++] = (uint16_t)x;
      for (u32 x = jb; x < je; x++) s_list[o++] = (uint16_t)(x | 0x8000u);
      __syncthreads();
      for (u32 q = tid; q < tot_rows; q += DB) {
        const u32 e = s_list[q];
        s_h[q] = (e & 0x8000u) ? rh(p.sb, c0 + (e & 0x7FFFu)) : rh(p.sa, a0 + e);
      }
      __syncthreads();
    }
  }
  if (!lds) {  // fallback: per-bucket merges over global memory
    u32 c = 0;
    if (walk) {
      const u64* ka = p.sa.key + a0;
      const u64* kb = p.sb.key + c0;
      ia = (b == b0) ? 0u : lb_small(ka, na, lk);
      ie = last ? na : lb_small(ka, na, hk);
      jb = (b == b0) ? 0u : lb_small(kb, nc, lk);
      je = last ? nc : lb_small(kb, nc, hk);
      c = merge_bucket<false, false>(p.sa, a0 + ia, a0 + ie, p.sb, nullptr, nullptr, c0 + jb, c0 + je,
                                     nullptr, 0, 0);
    }
    u32 tot;
    const u32 ex = block_excl_scan<DB>(c, s_wave, &tot);
    if (c)
      merge_bucket<false, true>(p.sa, a0 + ia, a0 + ie, p.sb, nullptr, nullptr, c0 + jb, c0 + je,
                                p.keys + base, ex, ~0ull);
    if (tid == 0) {
      p.cnt[tile] = tot;
      if (tot) atomicAdd((unsigned long long*)&p.bsum[tile / DB], (unsigned long long)tot);
    }
    return;
  }
  // merge the differing buckets' keys from LDS: count, then write at the scanned offset.
  // This bucket's A rows' hashes sit at s_h[r0 + (x - ia)], its B rows' after them.
  const u32 hb0 = r0 + (ie - ia) - jb;
  u32 c = 0;
  for (int pass = 0; pass < 2; pass++) {
    u32 o = 0;
    if (pass == 1) {
      u32 tot;
      o = block_excl_scan<DB>(c, s_wave, &tot);
      if (tid == 0) {
        p.cnt[tile] = tot;
        if (tot) atomicAdd((unsigned long long*)&p.bsum[tile / DB], (unsigned long long)tot);
      }
    }
    if (walk) {
      u32 i = ia, j = jb, k2 = 0;
      while (i < ie || j < je) {
        const u64 ka = i < ie ? s_ka[i] : ~0ull, kb = j < je ? s_kb[j] : ~0ull;
        const u64 k = ka < kb ? ka : kb;
        u64 ha = 0, hb = 0;
        const bool pa = ka == k, pb = kb == k;
        for (; i < ie && s_ka[i] == k; i++) ha += s_h[r0 + (i - ia)];
        for (; j < je && s_kb[j] == k; j++) hb += s_h[hb0 + j];
        if (!(pa && pb) || ha != hb) {
          if (pass == 1) p.keys[base + o + k2] = k;
          k2++;
        }
      }
      c = k2;
    }
  }
}

constexpr int DSB = 1024;
__global__ __launch_bounds__(DSB) void tile_scan_kernel(const u64* cnt, u64* off, u64 ntiles,
                                                        u64* d_count) {
  __shared__ u32 s_wave[DSB / WAVE + 1];
  __shared__ u64 s_carry;
  scan_tile_counts<DSB>(cnt, off, ntiles, d_count, s_wave, &s_carry);
}

// Scan and copy in one pass, one wave per tile: the tile's output offset is the sum of
// the earlier groups' tile sums (bsum, added by the count kernel: 256 same-word adds per
// group, no scan launch) plus the counts of the earlier tiles of its own group -- at
// most 255 + ntiles / 256 words, loaded by the 64 lanes at once -- then the lanes copy
// the tile's keys from scratch to the output below cap.  The last tile's wave writes
// the total.
__global__ __launch_bounds__(WAVE) void merkle_diff_write_kernel(DiffArgs p) {
  const int lane = threadIdx.x;
  const u64 tile = blockIdx.x, grp = tile / DB;
  const u64 n = p.cnt[tile];
  const bool last = tile + 1 == p.ntiles;
  if (n == 0 && !last) return;  // uniform
  u64 before = 0;
  for (u64 x = lane; x < grp; x += WAVE) before += p.bsum[x];
  for (u64 x = grp * DB + lane; x < tile; x += WAVE) before += p.cnt[x];
#pragma unroll
  for (int d = WAVE / 2; d >= 1; d >>= 1) before += __shfl_xor(before, d, WAVE);
  if (last && lane == 0) *p.d_count = before + n;
  if (n == 0 || before >= p.cap) return;
  const u64 src = p.bnd[tile] + p.bnd[p.ntiles + 1 + tile];
  for (u64 x = lane; x < n && before + x < p.cap; x += WAVE) p.out[before + x] = p.keys[src + x];
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
  const u64 G = merkle_chunks(t.depth);
  // scratch: the arrival counter (zeroed before EVERY launch), then the hand-off words
  hipError_t e = hipMemsetAsync(ctr, 0, 16 * sizeof(u32), st);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(merkle_chunk_kernel<true>, dim3((unsigned)G), dim3(UPB), 0, st, s, t,
                     (const u32*)nullptr, ctr, (u64*)(ctr + 16), d_keys, err);
  return hipGetLastError();
}

hipError_t launch_merkle_update(const MerkleT& m, const Rows& olds, const Rows& news, const u64* keys,
                                u64 n_keys, u32* dirty, u64* d_keys, u32* ctr, u32* err,
                                hipStream_t st) {
  const MT t = mt_of(m);
  const u64 G = merkle_chunks(t.depth);
  hipError_t e = hipMemsetAsync(ctr, 0, 16 * sizeof(u32), st);
  if (e != hipSuccess) return e;
  if (n_keys)
    hipLaunchKernelGGL(merkle_update_kernel, dim3(grid_of(n_keys, UB)), dim3(UB), 0, st, t, olds, news,
                       keys, n_keys, dirty, d_keys, err);
  hipLaunchKernelGGL(merkle_chunk_kernel<false>, dim3((unsigned)G), dim3(UPB), 0, st, news, t, dirty,
                     ctr, (u64*)(ctr + 16), (u64*)nullptr, err);
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
  p.bnd = scratch;
  p.cnt = scratch + 2 * (p.ntiles + 1);
  p.off = p.cnt + p.ntiles;
  p.keys = p.off + p.ntiles;
  p.bsum = p.keys + sa.n + sb.n + 1;
  p.d_count = d_count;
  const u64 waves = 2 * (p.ntiles + 1);
  hipError_t e = hipMemsetAsync(p.bsum, 0, grid_of(p.ntiles, DB) * sizeof(u64), st);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(merkle_diff_bounds_kernel, dim3(grid_of(waves * WAVE, 256)), dim3(256), 0, st, p);
  hipLaunchKernelGGL(merkle_diff_count_kernel, dim3((unsigned)p.ntiles), dim3(DB), 0, st, p);
  hipLaunchKernelGGL(merkle_diff_write_kernel, dim3((unsigned)p.ntiles), dim3(WAVE), 0, st, p);
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
