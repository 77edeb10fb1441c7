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
// Row hashes cover term hashes of the value and node when the tree carries them
// (dg_term_hashes: trees then compare across interning tables and BEAM nodes), the ids
// otherwise.  The tree also keeps each bucket's row count (u16), maintained by build and
// update, read by the diff.
//
// Kernels:
//  * build: ONE launch.  A workgroup per chunk of 2^11 buckets streams the chunk's rows
//    (36 B/row; the row range from two wave lower bounds) into LDS bucket sums, reduces
//    the chunk's 11 levels in LDS and writes them; the last workgroup to finish (one
//    arrival counter, write-through hand-off words) reduces the chunk roots to the root.
//  * update: one thread per changed key re-hashes the key's rows in the old and the
//    new store and adds the difference to its bucket (put/delete); the upsweep then
//    re-reduces only the 2^11-bucket chunks an update touched (update_hashes).
//  * diff: a workgroup per subtree of 4096 buckets; a subtree whose root matches is
//    skipped, otherwise the workgroup descends it in strides of 4 levels (each thread
//    owns 16 buckets and compares their ancestors 4 and 8 levels up, then the buckets
//    only below differing ancestors: two round trips instead of twelve), locates each
//    differing bucket's rows from the trees' per-bucket row counts, hashes just those
//    rows and merges them key by key.  count / write passes; keys past `cap` are
//    counted, not written (max_sync_size truncation).
//  * partial diff: node-form continuations (positions + the sender's hashes at one
//    level) are compared and expanded `levels` levels down; at the bucket level the
//    reply is a leaf-form continuation (the sender's (key, leaf) pairs of the
//    differing buckets), which the peer merges with its own rows into keys.
#include "dg_hash.h"
#include "dg_home.h"
#include "dg_kdw.h"
#include "dg_launch.h"
#include "dg_tree.h"

namespace dg {

namespace {

struct MT {
  u32 depth, sb;
  u64 shard;
  u64* nodes;
  uint16_t* counts;
  TermH th;
  u64* starts;  // optional (nullptr): each chunk's first row, then the end (dg_merkle.starts)
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

__device__ __forceinline__ u64 rh(const Rows& s, u64 i, const TermH& th) {
  return row_hash(s.key[i], th_val(th, s.val[i]), s.ts[i], th_node(th, s.node[i]), s.cnt[i]);
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
#ifndef DG_MERKLE_VEC  // the build's 4-consecutive-rows loop (0: the strided loop, for A/B)
#define DG_MERKLE_VEC 1
#endif
constexpr bool MERKLE_VEC = DG_MERKLE_VEC;
constexpr int UPB = 512;   // threads per chunk workgroup
constexpr int UPL = MERKLE_UPL;  // levels reduced per workgroup (2048 nodes in LDS)
constexpr u32 UPW = 1u << UPL;
constexpr u32 NHL = 1024;  // node hashes staged in LDS by the build (more: read from global)
constexpr u32 ERR_SHARD = MERKLE_ERR_SHARD, ERR_COUNT = MERKLE_ERR_COUNT;  // input-error bits

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

// The same for a full chunk (width == UPW == 4 * UPB) with ONE block barrier instead of
// eleven: a thread takes its 4 leaves from LDS and makes levels 1 and 2 in registers, each
// wave makes the next 6 levels with shuffles (at level 2 + k the lanes that are multiples
// of 2^k combine their node with the one 2^(k-1) lanes up), the 8 wave roots meet in LDS
// and wave 0 makes the last 3 levels.  Writes every level to `nodes` as lds_upsweep does
// and leaves the chunk root in s[0].
static_assert(UPW == 4 * UPB && UPB / WAVE == 8, "4 leaves per thread, 8 waves");
__device__ void chunk_upsweep(u64* nodes, u32 hi, u64 g0, u64* s) {
  const u32 tid = threadIdx.x, lane = tid & (WAVE - 1), w = tid / WAVE;
  auto row = [&](u32 l) { return nodes + ((1ull << (hi - l)) - 1) + (g0 >> l); };
  const u64 l0 = s[4 * tid], l1 = s[4 * tid + 1], l2 = s[4 * tid + 2], l3 = s[4 * tid + 3];
  const u64 p0 = node_hash(l0, l1), p1 = node_hash(l2, l3);
  row(1)[2 * tid] = p0;
  row(1)[2 * tid + 1] = p1;
  u64 v = node_hash(p0, p1);
  row(2)[tid] = v;
#pragma unroll
  for (u32 k = 1; k <= 6; k++) {  // levels 3..8 inside the wave
    const u64 o = __shfl_down(v, 1u << (k - 1), WAVE);
    if ((lane & ((1u << k) - 1)) == 0) {
      v = node_hash(v, o);
      row(2 + k)[tid >> k] = v;
    }
  }
  __syncthreads();  // every wave is done reading s (the leaves)
  if (lane == 0) s[w] = v;  // level-8 node w
  __syncthreads();
  if (w == 0) {
    u64 x = lane < 8 ? s[lane] : 0ull;
#pragma unroll
    for (u32 k = 1; k <= 3; k++) {  // levels 9..11
      const u64 o = __shfl_down(x, 1u << (k - 1), WAVE);
      if (lane < 8 && (lane & ((1u << k) - 1)) == 0) {
        x = node_hash(x, o);
        row(8 + k)[lane >> k] = x;
      }
    }
    if (lane == 0) s[0] = x;
  }
  __syncthreads();
}

// The last workgroup of a chunk launch: levels depth - L1 .. 0, UPL levels per round (the
// first round's inputs are the handed-off chunk roots, sc1 loads), the chunk index moved
// by the chunks' row-count changes (cdelta, when given), and for a build the distinct-key
// count.  s: the caller's UPW-node LDS stage.
template <bool BUILD>
__device__ __forceinline__ void chunk_tail(MT t, u64* hand, u64* d_keys, const i64* cdelta, const u64 G, u64* s) {
  const u32 L1 = t.depth < (u32)UPL ? t.depth : (u32)UPL;
  const int tid = threadIdx.x, lane = tid & (WAVE - 1), w = tid / WAVE;
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
      if ((1u << nlev) == UPW)  // (uniform)
        chunk_upsweep(t.nodes, hl, c << nlev, s);
      else
        lds_upsweep(t.nodes, hl, c << nlev, 1u << nlev, s);
    }
    hl -= nlev;
    first = false;
  }
  if (!BUILD && t.starts && cdelta) {
    // the update moved rows: chunk g's first row shifts by the row-count changes of the
    // chunks before it (an exclusive scan of cdelta, UPB chunks per round; the end by all)
    // (CP consecutive entries per thread, their loads issued together: one round of
    // UPB * CP = 4096 entries covers the 2048 chunks of a depth-22 tree)
    constexpr int CP = 4;
    i64 carry = 0;
    for (u64 c0 = 0; c0 <= G; c0 += (u64)UPB * CP) {
      const u64 x0 = c0 + (u64)tid * CP;
      i64 v[CP], st0[CP];
#pragma unroll
      for (int q = 0; q < CP; q++) {
        const u64 x = x0 + q;
        v[q] = x < G ? cdelta[x] : 0;
        st0[q] = x <= G ? (i64)t.starts[x] : 0;
      }
#pragma unroll
      for (int q = 0; q < CP; q++)  // consumed: zero again for the next update
        if (x0 + q < G && v[q]) ((i64*)cdelta)[x0 + q] = 0;
      i64 own = 0;
#pragma unroll
      for (int q = 0; q < CP; q++) own += v[q];
      i64 incl = own;
#pragma unroll
      for (int d = 1; d < WAVE; d <<= 1) {
        const i64 y = __shfl_up(incl, d, WAVE);
        if (lane >= d) incl += y;
      }
      __syncthreads();
      if (lane == WAVE - 1) s[w] = (u64)incl;
      __syncthreads();
      i64 before = 0, tot = 0;
      for (int q = 0; q < UPB / WAVE; q++) {
        const i64 y = (i64)s[q];
        before += q < w ? y : 0;
        tot += y;
      }
      i64 run = carry + before + incl - own;  // the changes of the chunks before x0
#pragma unroll
      for (int q = 0; q < CP; q++) {
        const u64 x = x0 + q;
        if (x <= G) t.starts[x] = (u64)(st0[q] + run);
        run += v[q];
      }
      carry += tot;
    }
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

// ctr: the arrival counter, zero on entry and left zero (the last workgroup resets it: a
// persistent engine word, no fill launch per build); scratch: per chunk its root and its
// distinct-key count (u64 each, at hand[0, G) and hand[G, 2G)).
// (the body of one workgroup g of G)
template <bool BUILD, bool VEC = false>
__device__ __forceinline__ void chunk_block(Rows rows, MT t, const u32* dirty, u32* ctr, u64* hand,
                                            u64* d_keys, u32* err, const i64* cdelta, const u64 g,
                                            const u64 G) {
  __shared__ u64 s[UPW];
  __shared__ u32 s_c[BUILD ? UPW : 1];  // rows per bucket
  __shared__ u64 s_nh[BUILD ? NHL : 1]; // node term hashes
  __shared__ u64 s_rng[2];
  __shared__ u32 s_red[UPB / WAVE];
  __shared__ u32 s_last;
  const u32 L1 = t.depth < (u32)UPL ? t.depth : (u32)UPL;
  const u32 width = 1u << L1;
  const u64 g0 = g << L1;
  const int tid = threadIdx.x, lane = tid & (WAVE - 1), w = tid / WAVE;
  u64* lvl = t.nodes + ((1ull << t.depth) - 1);
  u64 chunk_root = 0, chunk_keys = 0;
  if (BUILD) {
    for (u32 x = tid; x < width; x += UPB) {
      s[x] = 0;
      s_c[x] = 0;
    }
    const bool nh_lds = t.th.on && t.th.nn <= NHL;  // uniform
    if (nh_lds)
      for (u32 x = tid; x < (u32)t.th.nn; x += UPB) s_nh[x] = t.th.nh[x];
    if (w < 2) {
      const u64 r = wave_bucket_start(t, rows.key, rows.n, g0 + (w ? width : 0));
      if (lane == 0) s_rng[w] = r;
    }
    __syncthreads();
    const u64 lo = s_rng[0], hi = s_rng[1];
    if (t.starts && tid == 0) {  // the chunk index (dg_merkle.starts): its first row, and the end
      t.starts[g] = lo;
      if (g == G - 1) t.starts[G] = hi;
    }
    u32 heads = 0;
    // rows outside the tree's key range (before the first chunk, after the last one)
    bool bad = tid == 0 && ((g == 0 && lo > 0) || (g == G - 1 && hi < rows.n));
    if (VEC) {
      // each thread hashes 4 CONSECUTIVE rows (16-byte loads: 2 per 8-byte column, 1 for
      // the node column), sums the rows of one bucket in registers and adds each run once
      // to LDS: ~1.4 LDS atomics per 4 rows instead of 8, and no two lanes of a wave add to
      // one bucket in the same instruction unless a bucket straddles them
      const u64 a0 = lo & ~3ull;
      const int lane_ = tid & (WAVE - 1);
      for (u64 base = a0; base < hi; base += 4 * UPB) {  // block-uniform trip count
        const u64 gb = base + 4 * (u64)tid;
        const bool any = gb < hi;
        u64 key[4] = {0, 0, 0, 0}, val[4] = {0, 0, 0, 0}, cnt[4] = {0, 0, 0, 0};
        i64 ts[4] = {0, 0, 0, 0};
        u32 nd[4] = {0, 0, 0, 0};
        // the previous row's key for lane 0, loaded by every lane at a clamped index with the
        // rows' own loads (a load under lane 0's branch was waited for on its own: build
        // 0.497 -> 0.510-0.516 of peak, A/B)
        const u64 pkey = rows.key[gb > 0 && gb - 1 < rows.n ? gb - 1 : 0];
        if (any && gb + 3 < rows.n) {
          const ulonglong2 k0 = *(const ulonglong2*)(rows.key + gb), k1 = *(const ulonglong2*)(rows.key + gb + 2);
          const ulonglong2 v0 = *(const ulonglong2*)(rows.val + gb), v1 = *(const ulonglong2*)(rows.val + gb + 2);
          const longlong2 t0 = *(const longlong2*)(rows.ts + gb), t1 = *(const longlong2*)(rows.ts + gb + 2);
          const ulonglong2 c0 = *(const ulonglong2*)(rows.cnt + gb), c1 = *(const ulonglong2*)(rows.cnt + gb + 2);
          const uint4 n4 = *(const uint4*)(rows.node + gb);
          key[0] = k0.x, key[1] = k0.y, key[2] = k1.x, key[3] = k1.y;
          val[0] = v0.x, val[1] = v0.y, val[2] = v1.x, val[3] = v1.y;
          ts[0] = t0.x, ts[1] = t0.y, ts[2] = t1.x, ts[3] = t1.y;
          cnt[0] = c0.x, cnt[1] = c0.y, cnt[2] = c1.x, cnt[3] = c1.y;
          nd[0] = n4.x, nd[1] = n4.y, nd[2] = n4.z, nd[3] = n4.w;
        } else if (any) {  // the store's last rows: no 16-byte load past its end
#pragma unroll
          for (int q = 0; q < 4; q++)
            if (gb + q < rows.n) {
              key[q] = rows.key[gb + q];
              val[q] = rows.val[gb + q];
              ts[q] = rows.ts[gb + q];
              cnt[q] = rows.cnt[gb + q];
              nd[q] = rows.node[gb + q];
            }
        }
        // the row before this thread's first: the previous lane's last key (lane 0: memory)
        u64 prev = __shfl_up(key[3], 1, WAVE);
        if (lane_ == 0) prev = (any && gb > 0) ? pkey : ~key[0];
        u64 run_h = 0;
        u32 run_c = 0;
        u64 run_b = ~0ull;
#pragma unroll
        for (int q = 0; q < 4; q++) {
          const u64 i = gb + (u64)q;
          if (i >= lo && i < hi) {
            const u64 nt = nh_lds ? (nd[q] < (u32)t.th.nn ? s_nh[nd[q]] : (u64)nd[q]) : th_node(t.th, nd[q]);
            const u64 h = row_hash(key[q], th_val(t.th, val[q]), ts[q], nt, cnt[q]);
            const u64 pk = q ? key[q - 1] : prev;
            heads += (i == lo || pk != key[q]) ? 1u : 0u;
            if (t.sb && (key[q] >> (64 - t.sb)) != t.shard) bad = true;
            const u64 b = bucket_of(t, key[q]) - g0;
            if (b != run_b) {
              if (run_b < width) {
                atomicAdd((unsigned long long*)&s[run_b], (unsigned long long)run_h);
                atomicAdd(&s_c[run_b], run_c);
              }
              run_b = b;
              run_h = 0;
              run_c = 0;
            }
            run_h += h;
            run_c++;
          }
        }
        if (run_b < width) {
          atomicAdd((unsigned long long*)&s[run_b], (unsigned long long)run_h);
          atomicAdd(&s_c[run_b], run_c);
        }
      }
    } else {
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
            const u32 nd = rows.node[i];
            const u64 nt = nh_lds ? (nd < (u32)t.th.nn ? s_nh[nd] : (u64)nd) : th_node(t.th, nd);
            h[q] = row_hash(key[q], th_val(t.th, rows.val[i]), rows.ts[i], nt, rows.cnt[i]);
            head[q] = i == lo || rows.key[i - 1] != key[q];
          }
        }
#pragma unroll
        for (int q = 0; q < 4; q++) {
          const u64 i = i0 + (u64)q * UPB + tid;
          if (i < hi) {
            if (t.sb && (key[q] >> (64 - t.sb)) != t.shard) bad = true;
            const u64 b = bucket_of(t, key[q]) - g0;
            if (b < width) {
              atomicAdd((unsigned long long*)&s[b], (unsigned long long)h[q]);
              atomicAdd(&s_c[b], 1u);
            }
            heads += head[q] ? 1u : 0u;
          }
        }
      }
    }
    // distinct keys of the chunk (keys of different chunks differ: a key fixes its bucket)
    u32 c = heads;
#pragma unroll
    for (int d = WAVE / 2; d >= 1; d >>= 1) c += __shfl_xor(c, d, WAVE);
    if (lane == 0) s_red[w] = c;
    if (__ballot(bad) && lane == 0) atomicOr(err, ERR_SHARD);
    __syncthreads();
    if (tid == 0)
      for (int q = 0; q < UPB / WAVE; q++) chunk_keys += s_red[q];
    bool over = false;
    for (u32 x = tid; x < width; x += UPB) {
      lvl[g0 + x] = s[x];
      const u32 c = s_c[x];
      over |= c > 0xFFFFu;
      t.counts[g0 + x] = (uint16_t)(c > 0xFFFFu ? 0xFFFFu : c);
    }
    if (__ballot(over) && lane == 0) atomicOr(err, ERR_COUNT);
    if (width == UPW)  // (uniform)
      chunk_upsweep(t.nodes, t.depth, g0, s);
    else
      lds_upsweep(t.nodes, t.depth, g0, width, s);
    chunk_root = s[0];
  } else if (dirty && dirty[g]) {
    for (u32 x = tid; x < width; x += UPB) s[x] = lvl[g0 + x];
    __syncthreads();
    if (width == UPW)  // (uniform)
      chunk_upsweep(t.nodes, t.depth, g0, s);
    else
      lds_upsweep(t.nodes, t.depth, g0, width, s);
    chunk_root = s[0];
    if (tid == 0) ((u32*)dirty)[g] = 0;  // consumed: the flags are zero again for the next update
  } else if (tid == 0) {  // unchanged: its root as the previous kernels left it
    chunk_root = t.nodes[((1ull << (t.depth - L1)) - 1) + g];
  }
  // ---- hand the chunk root (and key count) to the last workgroup
  if (tid == 0) {
    st_sc1(hand + g, chunk_root);
    if (BUILD) st_sc1(hand + G + g, chunk_keys);
    wait_vmem();
    s_last = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == G - 1;
    if (s_last) __hip_atomic_store(ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // all G arrived
  }
  __syncthreads();
  if (!s_last) return;
  chunk_tail<BUILD>(t, hand, d_keys, cdelta, G, s);
}

template <bool BUILD, bool VEC = false>
__global__ __launch_bounds__(UPB, 4) void merkle_chunk_kernel(Rows rows, MT t, const u32* dirty,
                                                           u32* ctr, u64* hand, u64* d_keys,
                                                           u32* err, const i64* cdelta) {
  chunk_block<BUILD, VEC>(rows, t, dirty, ctr, hand, d_keys, err, cdelta, blockIdx.x, gridDim.x);
}

// The update's re-reduction by NB persistent workgroups, chunks g = cb, cb + NB, ...: a
// workgroup per chunk paid a dirty-flag load, a root load, a write-through hand-off and an
// arrival for every chunk, and 2048 such workgroups took 32 us with nothing dirty (A/B).
// Here a workgroup loads its chunks' flags and old roots in one round trip, re-reduces its
// dirty chunks one after the other (the next chunk's leaves issued before the current
// one's upsweep), hands every root off write-through and arrives once; the last one runs
// chunk_tail.  The leaves are double-buffered in LDS.
#ifndef DG_KDF_EXP
#define DG_KDF_EXP 0  // A/B builds only: 3 = a workgroup per chunk (chunk_block)
#endif
constexpr u32 KCH = 16;  // chunks per workgroup at most (G <= KCH * NB)
__device__ __forceinline__ void kd_chunks(MT t, u32* dirty, u32* ctr, u64* hand, const i64* cdelta, const u64 cb,
                                          const u64 NB, const u64 G) {
  __shared__ u64 s2[2][UPW];
  __shared__ u32 s_fl[KCH];
  __shared__ u64 s_rt[KCH];
  __shared__ u32 s_last;
  const u32 L1 = t.depth < (u32)UPL ? t.depth : (u32)UPL;
  const u32 width = 1u << L1;
  const int tid = threadIdx.x;
  const u64* lvl = t.nodes + ((1ull << t.depth) - 1);
  const u32 nc = (u32)((G - cb + NB - 1) / NB);  // this workgroup's chunks (<= KCH)
  if ((u32)tid < nc) {
    const u64 g = cb + (u64)tid * NB;
    s_fl[tid] = dirty[g];
    s_rt[tid] = t.nodes[((1ull << (t.depth - L1)) - 1) + g];
  }
  __syncthreads();
  // leaves of the i-th dirty chunk from position j on, into buffer b (registers first)
  auto next_dirty = [&](u32 j) {
    while (j < nc && !s_fl[j]) j++;
    return j;
  };
  u32 j = next_dirty(0);
  u64 v[UPW / UPB];
  if (j < nc)
#pragma unroll
    for (u32 q = 0; q < UPW / UPB; q++) {
      const u32 x = tid + q * UPB;
      v[q] = x < width ? lvl[((cb + (u64)j * NB) << L1) + x] : 0ull;
    }
  int b = 0;
  for (u32 i = 0; i < nc; i++) {
    const u64 g = cb + (u64)i * NB;
    if (i != j) {  // clean: its root as the previous kernels left it
      if (tid == 0) st_sc1(hand + g, s_rt[i]);
      continue;
    }
#pragma unroll
    for (u32 q = 0; q < UPW / UPB; q++) s2[b][tid + q * UPB] = v[q];
    __syncthreads();
    j = next_dirty(i + 1);  // the next dirty chunk's leaves in flight during this upsweep
    if (j < nc)
#pragma unroll
      for (u32 q = 0; q < UPW / UPB; q++) {
        const u32 x = tid + q * UPB;
        v[q] = x < width ? lvl[((cb + (u64)j * NB) << L1) + x] : 0ull;
      }
    if (width == UPW)  // (uniform)
      chunk_upsweep(t.nodes, t.depth, g << L1, s2[b]);
    else
      lds_upsweep(t.nodes, t.depth, g << L1, width, s2[b]);
    if (tid == 0) {
      st_sc1(hand + g, s2[b][0]);
      dirty[g] = 0;  // consumed: the flags are zero again for the next update
    }
    b ^= 1;
  }
  if (tid == 0) {
    wait_vmem();
    s_last = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == NB - 1;
    if (s_last) __hip_atomic_store(ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // all NB arrived
  }
  __syncthreads();
  if (!s_last) return;
  chunk_tail<false>(t, hand, nullptr, cdelta, G, s2[0]);
}

// dg_join_delta's write (dg_kdw.h, workgroups [0, nw): dispatched first, they start at once)
// and the dirty chunks' re-reduction (the rest: kd_chunks' persistent workgroups) in ONE
// launch: both read only what kd_count_kernel wrote, so the write's ~15 us run under the
// re-reduction's instead of after it.
#ifndef DG_KDF_WAVES  // waves per SIMD the launch is compiled for: 6 = 73 VGPRs, three
#define DG_KDF_WAVES 6  // workgroups per CU, no spills (8 spills, 4 is two per CU: A/B slower)
#endif
__global__ __launch_bounds__(UPB, DG_KDF_WAVES) void kd_finish_kernel(KdArgs p, u32 nw, MT t, const u32* dirty,
                                                         u32* ctr, u64* hand, const i64* cdelta) {
  if (blockIdx.x < nw) {
    kd_write_block<UPB>(p, blockIdx.x);
    return;
  }
  // no key's row count changed (the count kernel's moved flag): every chunk's row-count
  // change is zero, and the last workgroup skips the chunk index's scan
  const i64* cd = p.d_counts[5] ? cdelta : nullptr;
#if DG_KDF_EXP == 3  // (A/B: a workgroup per chunk)
  chunk_block<false>(Rows{}, t, dirty, ctr, hand, nullptr, nullptr, cd, blockIdx.x - nw, gridDim.x - nw);
#else
  const u32 L1 = t.depth < (u32)UPL ? t.depth : (u32)UPL;
  kd_chunks(t, (u32*)dirty, ctr, hand, cd, blockIdx.x - nw, gridDim.x - nw, 1ull << (t.depth - L1));
#endif
}

// ---------------------------------------------------------------- update
constexpr int UB = 256;


// Σ row_hash of key x's rows in s (0 if absent); *rows = their number.
__device__ __forceinline__ u64 key_leaf(const Rows& s, u64 x, const TermH& th, u32* rows) {
  u64 i = interp_lower_bound(s.key, 0, s.n, x);
  u64 h = 0;
  u32 r = 0;
  for (; i < s.n && s.key[i] == x; i++, r++) h += rh(s, i, th);
  *rows = r;
  return h;
}

__global__ __launch_bounds__(UB) void merkle_update_kernel(MT t, Rows olds, Rows news, const u64* keys,
                                                           u64 n_keys, u32* dirty, u64* d_keys,
                                                           u32* err, i64* cdelta) {
  const u64 i = (u64)blockIdx.x * UB + threadIdx.x;
  int dk = 0;
  bool bad = false, over = false;
  if (i < n_keys) {
    const u64 x = keys[i];
    u32 ro, rn;
    const u64 ho = key_leaf(olds, x, t.th, &ro), hn = key_leaf(news, x, t.th, &rn);
    dk = (int)(rn > 0) - (int)(ro > 0);
    if (ho != hn || ro != rn) {
      if (t.sb && (x >> (64 - t.sb)) != t.shard) {
        bad = true;
      } else {
        const u64 b = bucket_of(t, x);
        u64* lvl = t.nodes + ((1ull << t.depth) - 1);
        atomicAdd((unsigned long long*)&lvl[b], (unsigned long long)(hn - ho));
        if (rn != ro) {  // the bucket's row count, in its aligned 32-bit word (counts stay
                         // in [0, 65535]: no carry or borrow into the neighbour's half)
          u32* wd = (u32*)t.counts + (b >> 1);
          const u32 sh = 16u * (u32)(b & 1);
          if (rn > ro) {
            const u32 old = atomicAdd(wd, (rn - ro) << sh);
            over = ((old >> sh) & 0xFFFFu) + (rn - ro) > 0xFFFFu;
          } else {
            atomicSub(wd, (ro - rn) << sh);
          }
        }
        const u32 L1 = t.depth < (u32)UPL ? t.depth : (u32)UPL;
        dirty[b >> L1] = 1u;
        if (cdelta && rn != ro)  // the chunk's rows changed in number: later chunks' starts move
          atomicAdd((unsigned long long*)&cdelta[b >> L1], (unsigned long long)((i64)rn - (i64)ro));
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
  if (__ballot(bad) && (threadIdx.x & (WAVE - 1)) == 0) atomicOr(err, ERR_SHARD);
  if (__ballot(over) && (threadIdx.x & (WAVE - 1)) == 0) atomicOr(err, ERR_COUNT);
}

// The same put/delete from kdelta.hip's per-key figures: key u changed (runs bit 48) with
// leaf change dh[u] and row-count change ne - na; sign -1 undoes sign +1.  The distinct-key
// change is the count kernel's (d_counts[7]).  The keys are ascending, so a wave's keys of
// one bucket (and of one chunk) are adjacent lanes: segmented sums over the lanes leave ONE
// atomic per bucket and per chunk (a small tree's few buckets took a thousand same-address
// atomics per word from a batch of mutations: 16 us for 1000 keys).
template <class T>
__device__ __forceinline__ T seg_incl(T v, u64 seg, int lane) {
#pragma unroll
  for (int d = 1; d < WAVE; d <<= 1) {
    const T y = __shfl_up(v, d, WAVE);
    const u64 sy = __shfl_up(seg, d, WAVE);
    if (lane >= d && sy == seg) v += y;  // (segments are contiguous runs of lanes)
  }
  return v;
}
__global__ __launch_bounds__(UB) void kd_tree_kernel(MT t, const u64* keys, const u64* runs, const u64* dh,
                                                     u64 nk, const u64* guard, int sign, u32* dirty,
                                                     u32* err, i64* cdelta) {
  if (guard && *guard) return;  // (uniform) the per-key figures are incomplete: nothing to apply
  const u64 i = (u64)blockIdx.x * UB + threadIdx.x;
  const int lane = threadIdx.x & (WAVE - 1);
  const u32 L1 = t.depth < (u32)UPL ? t.depth : (u32)UPL;
  bool bad = false, over = false;
  u64 b = ~0ull, d = 0;
  int dr = 0, act = 0;
  if (i < nk) {
    const u64 rn = runs[i];
    const int na = (int)(rn & 0xFFFF), ne = (int)((rn >> 32) & 0xFFFF);
    const u64 x = keys[i];
    b = bucket_of(t, x);
    if (((rn >> 48) & 1)) {
      const u64 dd = sign > 0 ? dh[i] : (u64)0 - dh[i];
      const int r = sign > 0 ? ne - na : na - ne;
      if (dd != 0 || r != 0) {
        if (t.sb && (x >> (64 - t.sb)) != t.shard) {
          bad = true;  // (skipped both ways)
        } else {
          d = dd;
          dr = r;
          act = 1;
        }
      }
    }
  }
  const u64 c = b == ~0ull ? ~0ull : b >> L1;
  const u64 sd = seg_incl<u64>(d, b, lane);
  const int sr = seg_incl<int>(dr, b, lane), sa = seg_incl<int>(act, b, lane);
  const int cr = seg_incl<int>(dr, c, lane), ca = seg_incl<int>(act, c, lane);
  const u64 nb = __shfl_down(b, 1, WAVE), nc = __shfl_down(c, 1, WAVE);
  const bool last = lane == WAVE - 1;
  if (b != ~0ull && (last || nb != b) && sa) {  // the bucket's last lane: its node and row count
    u64* lvl = t.nodes + ((1ull << t.depth) - 1);
    atomicAdd((unsigned long long*)&lvl[b], (unsigned long long)sd);
    if (sr) {  // the bucket's row count in its aligned 32-bit word (as merkle_update_kernel)
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
    dirty[c] = 1u;
    if (cdelta && cr) atomicAdd((unsigned long long*)&cdelta[c], (unsigned long long)(i64)cr);
  }
  if (__ballot(bad) && lane == 0) atomicOr(err, ERR_SHARD);
  if (__ballot(over) && lane == 0) atomicOr(err, ERR_COUNT);
}

// ---------------------------------------------------------------- key-level merge
// Merge keys[ia, ie) of store A (rows) with B, where B is either a store (rows) or a
// list of (key, leaf) pairs; emit the keys present on one side only or with different
// leaves.  WRITE: store them at out[o..) (only below cap); returns the count.
template <bool B_LEAVES, bool WRITE>
__device__ u32 merge_bucket(const Rows& A, const TermH& tha, u64 ia, u64 ie, const Rows& B,
                            const TermH& thb, const u64* bk, const u64* bh, u64 jb, u64 je,
                            u64* out, u64 o, u64 cap) {
  u32 c = 0;
  while (ia < ie || jb < je) {
    const u64 ka = ia < ie ? A.key[ia] : ~0ull;
    const u64 kb = jb < je ? (B_LEAVES ? bk[jb] : B.key[jb]) : ~0ull;
    const bool has_a = ia < ie && (jb >= je || ka <= kb);
    const bool has_b = jb < je && (ia >= ie || kb <= ka);
    const u64 k = has_a ? ka : kb;
    u64 ha = 0, hb = 0;
    if (has_a)
      for (; ia < ie && A.key[ia] == k; ia++) ha += rh(A, ia, tha);
    if (has_b) {
      if (B_LEAVES) {
        hb = bh[jb++];
      } else {
        for (; jb < je && B.key[jb] == k; jb++) hb += rh(B, jb, thb);
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
// One workgroup per subtree of 2^sub buckets (sub = min(depth, 12)), whose root sits at
// level Ls = depth - sub.
//  1. bounds: two waves of the subtree's workgroup find its first row in both stores
//     (a 64-ary wave lower bound: 4 dependent load rounds at 12.5M rows), beside the
//     descent's first loads (no separate launch).
//  2. count: a subtree whose roots match is skipped.  Otherwise the workgroup descends it
//     in strides of 4 levels.  Each thread owns 16 consecutive buckets: their ancestors
//     4 and 8 levels up (one node each), the subtree's root and the buckets' row counts
//     in both trees (u16) are loaded in one round trip, the 16 bucket nodes (the second
//     round trip) only where both ancestors differ.  (A level-by-level descent through a
//     frontier in LDS read 40 % fewer node bytes at 1 % differing keys but took 12 round
//     trips and 24 barriers: 281 us per config-4 diff.)  A block scan turns the row
//     counts into row ranges.  The
//     differing buckets' rows are listed and hashed by all threads at once (one round of
//     independent loads), and each thread merges its differing buckets' keys from LDS.
//     The subtree's differing keys go to scratch at (A start + B start) of the subtree,
//     unique and increasing across subtrees.  More rows than the LDS stage holds: each
//     thread merges its differing buckets over global memory instead.
//  3. write: each subtree's keys to their output offset, the keys past `cap` counted,
//     not written (truncation to max_sync_size).
constexpr int DB = DIFF_BLOCK;
constexpr u32 XSUB = 1u << DIFF_SUB;  // buckets per subtree (at most)
constexpr u32 OWN = XSUB / DB;        // buckets per thread
#ifndef DG_DIFF_EXP
#define DG_DIFF_EXP 0
#endif
// DG_DIFF_NT (A/B only): the staged rows' columns read with non-temporal loads (1: every
// column, 2: all but the key).  Config-4 round (profiles/r6/ab_diff_take.txt): the count
// kernel 65.7 -> 49.9 us, but the round's next calls read the same rows -- the take B's,
// the keyed join A's -- and lose what the diff's cached loads left in L2 and the
// last-level cache: take_keys 40 -> 54 us, kd_count 52 -> 60 us, the round no faster;
// back to back 50.3 -> 52.0 us.  FETCH unchanged (114 MB).  Kept off.
#ifndef DG_DIFF_NT
#define DG_DIFF_NT 0
#endif
// rows of the differing buckets staged in LDS, differing buckets listed in LDS (the
// subtree's share of a 1 %-differing config-4 shard is ~1000 rows in ~120 buckets at 4096
// buckets, a quarter of that at 1024; a subtree beyond either merges over global memory)
constexpr u32 RCAP = XSUB >= 4096 ? 1664 : 640;
constexpr u32 DCAP = XSUB >= 4096 ? 512 : 160;
constexpr u32 NHD = 128;              // node term hashes staged per tree
#ifndef DG_DIFF_OCC
#define DG_DIFF_OCC 4
#endif
constexpr int DIFF_OCC = DG_DIFF_OCC;  // count workgroups per CU the kernel is compiled for
static_assert(OWN == 16 || OWN == 4, "a thread owns 16 or 4 buckets (32 or 8 bytes of counts per tree)");
constexpr u32 CW = OWN / 2;           // count words (two u16 halves) per thread and tree

struct DiffArgs {
  MT ta, tb;
  Rows sa, sb;
  u64* out;
  u64 cap;
  u64* bnd;   // ntiles + 1 boundaries x 2 stores: first row of each subtree in A, then in B
  u64* cnt;   // differing keys per subtree
  u64* keys;  // scratch: nA + nB keys
  u64* bsum;  // per DB subtrees: the sum of their counts (zero when the count kernel starts)
  u64* bzero;  // the other parity's sums (the previous call's), zeroed by the write kernel
  u64 nzero;   // ... all of its words: a call of another depth may have used more of them
  u64 ntiles;
  u32 sub;
  u64* d_count;
};


// the counts of a thread's 16 buckets (u16) as 8 words of two halves: 32 bytes at
// c + first, one path for every subtree size (the counts array holds at least 16 entries,
// deltagpu.h); mask_counts16 zeroes what the thread does not own, AFTER the round trip's
// other loads are issued (any use of a loaded value -- a second load path for small
// subtrees, a mask -- makes the compiler wait for it right there)
__device__ __forceinline__ void load_counts16(const uint16_t* c, u32 first, u32 w[CW]) {
  if constexpr (OWN == 16) {
    const uint4* v = (const uint4*)(c + first);
    const uint4 x = v[0], y = v[1];
    w[0] = x.x, w[1] = x.y, w[2] = x.z, w[3] = x.w, w[4] = y.x, w[5] = y.y, w[6] = y.z, w[7] = y.w;
  } else {
    const uint2 x = *(const uint2*)(c + first);
    w[0] = x.x, w[1] = x.y;
  }
}
__device__ __forceinline__ void mask_counts16(u32 w[CW], u32 nb, bool owns) {
#pragma unroll
  for (u32 q = 0; q < CW; q++) {  // (nb < OWN: a tree of fewer buckets, thread 0's)
    const u32 keep = (2 * q + 1 < nb ? 0xFFFF0000u : 0u) | (2 * q < nb ? 0xFFFFu : 0u);
    w[q] &= owns ? keep : 0u;
  }
}

__device__ __forceinline__ u32 half16(const u32 w[CW], u32 i) { return (w[i >> 1] >> (16 * (i & 1))) & 0xFFFFu; }

// a buffer descriptor over [base, base + bytes) for a wave-uniform base (the halves go
// through readfirstlane so the compiler can keep the descriptor in SGPRs; gfx950 flags)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t wave_rsrc(const u64* base, u32 bytes) {
  const u32 lo = __builtin_amdgcn_readfirstlane((u32)(uintptr_t)base);
  const u32 hi = __builtin_amdgcn_readfirstlane((u32)((uintptr_t)base >> 32));
  return __builtin_amdgcn_make_buffer_rsrc((void*)(((uintptr_t)hi << 32) | lo), 0, (int)bytes, 0x00020000);
}
// one u64 through a descriptor; an offset past its range reads 0 without an access
__device__ __forceinline__ u64 buf_load_u64(__amdgpu_buffer_rsrc_t r, int off) {
  const auto v = __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 0);
  return ((u64)v[1] << 32) | v[0];
}

#ifdef DG_STAMPS
// Diagnostic build only (DG_STAMPS=1): per-subtree phase timestamps (s_memrealtime) by
// thread 0 of each count workgroup, read back with dg_debug_diff_stamps
// (tools/diff_stamps.py).  Each stamp is behind a barrier, so only shares are meaningful.
__device__ u64 g_df_stamps[4096 * 8];
#define DSTAMP(k)                                                                    \
  do {                                                                               \
    __syncthreads();                                                                 \
    if (threadIdx.x == 0 && tile < 4096)                                             \
      g_df_stamps[tile * 8 + (k)] = __builtin_amdgcn_s_memrealtime();                \
  } while (0)
#else
#define DSTAMP(k) \
  do {            \
  } while (0)
#endif

__global__ __launch_bounds__(DB, DIFF_OCC * DB / 256) void merkle_diff_count_kernel(DiffArgs p) {
  __shared__ u32 s_wave[DB / WAVE + 1];
  __shared__ u32 s_da[DCAP], s_db[DCAP];  // a differing bucket's first row in A / B (from the subtree's)
  __shared__ u32 s_dp[DCAP + 1];          // its first staged row
  __shared__ u32 s_dn[DCAP];              // its rows in A (high half) and B (low half)
  __shared__ u64 s_k[RCAP], s_h[RCAP];    // the staged rows' keys and row hashes
  __shared__ unsigned char s_rl[RCAP];     // bit 7: first row of a store's rows in its bucket;
                                           // at a key run's head, the run's length (< 127)
  __shared__ u64 s_nha[NHD], s_nhb[NHD];  // the trees' node term hashes (<= NHD nodes)
  const u32 depth = p.ta.depth, sub = p.sub, Ls = depth - sub, nb = 1u << sub;
  const u64 tile = blockIdx.x;
  const int tid = threadIdx.x;
  DSTAMP(0);
  const bool nha_lds = p.ta.th.on && p.ta.th.nn <= NHD, nhb_lds = p.tb.th.on && p.tb.th.nn <= NHD;
  const u64 root = ((1ull << Ls) - 1) + tile;
  const u64 nbnd = p.ntiles + 1;
  // ---- descent in strides of 4 levels: thread tid owns buckets [16 tid, 16 tid + 16) of
  //      the subtree, and their common ancestors 4 and 8 levels up (one node each) are
  //      loaded with the subtree's root, the owned buckets' row counts and the node term
  //      hashes in ONE round trip (every load unconditional at a clamped index, the
  //      unused ones selected away: a load under a divergent branch is waited for at the
  //      branch's join, one round trip each); the 16 bucket nodes only below differing
  //      ancestors, in a second one
  const bool owns = (u32)tid * OWN < nb;
  const u64 bucket0 = tile << sub;
  const u64 b0 = bucket0 + (u64)tid * OWN;  // the first owned bucket (tree-wide)
  const u64 b0c = owns ? b0 : bucket0;      // (clamped: the loads stay inside the subtree)
  const u64 ra = p.ta.nodes[root], rb = p.tb.nodes[root];
  const u64 gi = sub >= 8 ? ((1ull << (depth - 8)) - 1) + (b0c >> 8) : root;
  const u64 qi = sub >= 4 ? ((1ull << (depth - 4)) - 1) + (b0c >> 4) : root;
  const u64 ga = p.ta.nodes[gi], gb = p.tb.nodes[gi], qa = p.ta.nodes[qi], qb = p.tb.nodes[qi];
  u32 ca[CW], cb[CW];
  load_counts16(p.ta.counts + bucket0, owns ? (u32)tid * OWN : 0u, ca);
  load_counts16(p.tb.counts + bucket0, owns ? (u32)tid * OWN : 0u, cb);
  const u32 nna = nha_lds ? (u32)p.ta.th.nn : 0u, nnb = nhb_lds ? (u32)p.tb.th.nn : 0u;
  const u64 hna = nna ? p.ta.th.nh[(u32)tid < nna ? (u32)tid : 0u] : 0ull;
  const u64 hnb = nnb ? p.tb.th.nh[(u32)tid < nnb ? (u32)tid : 0u] : 0ull;
  // the subtree's first row in both stores: waves 0 and 1 look it up (the chunk index) or
  // search while the descent's loads are in flight (also for the write kernel, which
  // reads them from p.bnd)
  __shared__ u64 s_bnd[2];
  if (tid < 2 * WAVE) {
    const Rows& r = tid < WAVE ? p.sa : p.sb;
    const u64* st = tid < WAVE ? p.ta.starts : p.tb.starts;  // the trees' chunk index, if kept
    const u32 L1 = depth < (u32)UPL ? depth : (u32)UPL;
#if DG_DIFF_EXP == 1  // diagnostic build only (timing, wrong keys): no bounds search
    const u64 x = r.n * tile / p.ntiles;
#else
    // The chunk index describes the store the tree was built / updated against.  It is
    // trusted only when its end is this store's row count and the start lies inside the
    // store (wave-uniform: every lane reads the same two words); otherwise -- another store
    // handed to the diff, rows changed without a dg_merkle_update, or a shard tree over a
    // store that holds more shards -- the subtree's first row is searched, as without an
    // index, so a stale index never reads past the store or yields wrong keys.
    u64 x = 0;
    bool use_st = st != nullptr && sub >= L1;  // (a subtree smaller than an index chunk: searched)
    if (use_st) {
      x = st[(tile << sub) >> L1];
      use_st = st[1ull << (depth - L1)] == r.n && x <= r.n;
    }
    if (!use_st) x = wave_bucket_start(p.ta, r.key, r.n, tile << sub);
#endif
    if ((tid & (WAVE - 1)) == 0) {
      s_bnd[tid / WAVE] = x;
      p.bnd[(tid < WAVE ? 0 : nbnd) + tile] = x;
    }
  }
  static_assert(NHD <= DB, "one node term hash per thread");
  if ((u32)tid < nna) s_nha[tid] = hna;
  if ((u32)tid < nnb) s_nhb[tid] = hnb;
  if (ra == rb) {  // uniform: the whole subtree matches (the bounds are written anyway)
    if (tid == 0) p.cnt[tile] = 0;
    return;
  }
  DSTAMP(1);
  u32 mine = 0;  // the owned buckets that differ (bit i: bucket 16 tid + i)
  const bool anc = owns && (sub < 8 || ga != gb) && (sub < 4 || qa != qb);
  if (nb >= (u32)(WAVE * OWN)) {
    // the wave's 64 x OWN buckets' nodes, loaded by the wave together: load i of a lane
    // reads node 64 i + lane (owner lane (64 i + lane) / OWN, only under its differing
    // ancestors), so each load instruction reads 512 contiguous bytes instead of one 8-B
    // node from each of 64 lines (a lane's own OWN nodes); every load is issued before any
    // compare, and the ballot of load i hands each of its 64 / OWN owner lanes its OWN bits
    // (buffer loads: a lane that must not load passes an offset past the descriptor's
    // range, which the hardware answers with 0 and no memory access -- a conditional
    // global load would be a branch, and the compiler waits for each load at its join)
    const int lane = tid & (WAVE - 1);
    const u64 amask = __ballot(anc);
    const u64 lv = ((1ull << depth) - 1) + (tile << sub) + (u64)(tid - lane) * OWN;
    const __amdgpu_buffer_rsrc_t na = wave_rsrc(p.ta.nodes + lv, WAVE * OWN * 8);
    const __amdgpu_buffer_rsrc_t nbr = wave_rsrc(p.tb.nodes + lv, WAVE * OWN * 8);
    u64 x[OWN], y[OWN];
    constexpr u32 OPL = WAVE / OWN;  // owner lanes per load
#pragma unroll
    for (u32 i = 0; i < OWN; i++) {
      const bool ld = (amask >> (OPL * i + lane / OWN)) & 1;
      const int off = ld ? (int)((64 * i + lane) * 8) : 0x7ffffff0;
      x[i] = buf_load_u64(na, off);
      y[i] = buf_load_u64(nbr, off);
    }
#pragma unroll
    for (u32 i = 0; i < OWN; i++) {
      const u64 bal = __ballot(x[i] != y[i]);
      if ((u32)lane / OPL == i) mine = (u32)(bal >> (OWN * (lane % OPL))) & ((1u << OWN) - 1);
    }
  } else if (anc) {  // a subtree of fewer than 1024 buckets: a thread loads its own nodes
    const u64 lv = ((1ull << depth) - 1) + b0;
    const u32 m = nb < OWN ? nb : OWN;
#pragma unroll
    for (u32 i0 = 0; i0 < OWN; i0 += 4) {
      u64 x[4], y[4];
#pragma unroll
      for (u32 i = 0; i < 4; i++) {
        x[i] = i0 + i < m ? p.ta.nodes[lv + i0 + i] : 0ull;
        y[i] = i0 + i < m ? p.tb.nodes[lv + i0 + i] : 0ull;
      }
#pragma unroll
      for (u32 i = 0; i < 4; i++) mine |= (x[i] != y[i] ? 1u : 0u) << (i0 + i);
    }
  }
  // ---- the differing buckets as a list (one entry per bucket, in bucket order): its rows'
  //      offsets in both stores (from the subtree's first row) and their place among the
  //      staged rows; then every per-bucket step runs one lane per differing bucket, not
  //      every thread over its 16 owned buckets (which ran each step masked 16 times)
  mask_counts16(ca, nb, owns);
  mask_counts16(cb, nb, owns);
  u32 ta_ = 0, tb_ = 0, rd = 0;
#pragma unroll
  for (u32 i = 0; i < OWN; i++) {
    const u32 x = half16(ca, i), y = half16(cb, i);
    ta_ += x;
    tb_ += y;
    if (mine >> i & 1u) rd += x + y;
  }
  // the four exclusive prefixes (rows in A, rows in B, staged rows, differing buckets) in
  // ONE barrier: four wave scans, the wave totals to LDS, each thread adds up the totals of
  // the waves before its own (4 waves) -- four block scans took 12 barriers
  constexpr int NW = DB / WAVE;
  __shared__ u32 s_w4[4 * NW];
  u32 offa, offb, slot0, d0, ND, R, TA, TB;
  {
    const u32 v[4] = {ta_, tb_, rd, (u32)__popc(mine)};
    u32 inc[4];
    const int lane = tid & (WAVE - 1), w = tid / WAVE;
#pragma unroll
    for (int j = 0; j < 4; j++) inc[j] = wave_incl_scan(v[j]);
    if (lane == WAVE - 1)
#pragma unroll
      for (int j = 0; j < 4; j++) s_w4[j * NW + w] = inc[j];
    __syncthreads();
    u32 below[4], total[4];
#pragma unroll
    for (int j = 0; j < 4; j++) {
      below[j] = total[j] = 0;
#pragma unroll
      for (int i = 0; i < NW; i++) {
        const u32 x = s_w4[j * NW + i];
        below[j] += i < w ? x : 0u;
        total[j] += x;
      }
    }
    offa = below[0] + inc[0] - v[0];
    offb = below[1] + inc[1] - v[1];
    slot0 = below[2] + inc[2] - v[2];
    d0 = below[3] + inc[3] - v[3];
    R = total[2];
    ND = total[3];
    TA = total[0];
    TB = total[1];
  }
  DSTAMP(2);
  const u64 a0 = s_bnd[0], c0 = s_bnd[1];  // (the barrier above came after the searches)
  if (a0 + TA > p.sa.n || c0 + TB > p.sb.n) {
    // (uniform) the trees count more rows here than the stores hold from the subtree's first
    // row: a store the tree does not describe.  No row is read past it and no key written;
    // the marker reaches the total, which the host reports as an input error.
    if (tid == 0) {
      p.cnt[tile] = DIFF_MISMATCH;
      atomicAdd((unsigned long long*)&p.bsum[tile / DB], (unsigned long long)DIFF_MISMATCH);
    }
    return;
  }
  const bool lds = R <= RCAP && ND <= DCAP;  // uniform
  if (lds) {
    u32 d = d0, slot = slot0, ra = offa, rb = offb;
#pragma unroll
    for (u32 i = 0; i < OWN; i++) {
      const u32 x = half16(ca, i), y = half16(cb, i);
      if (mine >> i & 1u) {
        s_da[d] = ra;
        s_db[d] = rb;
        s_dp[d] = slot;
        s_dn[d] = (x << 16) | y;
        d++;
        slot += x + y;
      }
      ra += x;
      rb += y;
    }
    if (tid == 0) s_dp[ND] = R;
    __syncthreads();
    DSTAMP(3);
    // one lane per differing bucket writes, for each of the bucket's staged rows, the row's
    // place in its store into s_k (ROW_B: a row of B, ROW_FIRST: the first of its store's
    // rows in the bucket); the hashing step below reads that one word per row and
    // overwrites it with the row's key.  (Each row used to find its bucket by a binary
    // search of the LDS list: ~9 dependent LDS reads per row before its loads went out.)
    constexpr u64 ROW_B = 1ull << 63, ROW_FIRST = 1ull << 62;
    for (u32 e = tid; e < ND; e += DB) {
      const u32 sp = s_dp[e], xy = s_dn[e], x = xy >> 16, y = xy & 0xFFFFu;
      const u64 fa = a0 + s_da[e], fb = c0 + s_db[e];
      for (u32 r = 0; r < x; r++) s_k[sp + r] = (fa + r) | (r == 0 ? ROW_FIRST : 0ull);
      for (u32 r = 0; r < y; r++) s_k[sp + x + r] = (fb + r) | ROW_B | (r == 0 ? ROW_FIRST : 0ull);
    }
    __syncthreads();
    // hash the staged rows, all at once.  A thread's rows go in batches of RB: every column
    // load of the batch is issued before any row is hashed (one round trip per batch, not
    // one per row), and the node term hashes come from LDS (staged above), not from a
    // dependent global load.  A lane past the staged rows loads row 0 of a non-empty store
    // (its s_k entry may already hold another thread's key): no load sits under a
    // divergent branch, so all of them go out before any wait.
    const bool spare_b = p.sa.n == 0;
    constexpr int RB = 4;
    for (u32 u0 = 0; u0 < (RCAP + DB - 1) / DB; u0 += RB) {
      if (u0 * DB >= R) break;  // uniform
      u64 key[RB], val[RB], cnt[RB];
      i64 ts[RB];
      u32 nd[RB];
      bool fromb[RB];
      bool side0[RB];
#pragma unroll
      for (int j = 0; j < RB; j++) {
        const u32 q = (u0 + j) * DB + tid;
        {
          const u64 e = s_k[min(q, R - 1)];
          const bool in = q < R;
          fromb[j] = in ? (e & ROW_B) != 0 : spare_b;
          side0[j] = (e & ROW_FIRST) != 0;
          const Rows& S = fromb[j] ? p.sb : p.sa;
          const u64 i = in ? e & (ROW_FIRST - 1) : 0ull;
#if DG_DIFF_EXP == 2  // diagnostic build only (timing, wrong keys): no row loads
          key[j] = i;
          val[j] = i ^ 5;
          ts[j] = (i64)i;
          nd[j] = (u32)i & 3;
          cnt[j] = i;
#else
#if DG_DIFF_NT  // (A/B: non-temporal row loads, above)
          key[j] = DG_DIFF_NT == 2 ? S.key[i] : __builtin_nontemporal_load(S.key + i);
          val[j] = __builtin_nontemporal_load(S.val + i);
          ts[j] = __builtin_nontemporal_load(S.ts + i);
          nd[j] = __builtin_nontemporal_load(S.node + i);
          cnt[j] = __builtin_nontemporal_load(S.cnt + i);
#else
          key[j] = S.key[i];
          val[j] = S.val[i];
          ts[j] = S.ts[i];
          nd[j] = S.node[i];
          cnt[j] = S.cnt[i];
#endif
#endif
        }
      }
#pragma unroll
      for (int j = 0; j < RB; j++) {
        const u32 q = (u0 + j) * DB + tid;
        if (q < R) {
          const TermH& th = fromb[j] ? p.tb.th : p.ta.th;
          const u64* snh = fromb[j] ? s_nhb : s_nha;
          const bool lds_ok = fromb[j] ? nhb_lds : nha_lds;
          const u64 nt = lds_ok ? (nd[j] < (u32)th.nn ? snh[nd[j]] : (u64)nd[j]) : th_node(th, nd[j]);
          s_k[q] = key[j];
          s_h[q] = row_hash(key[j], th_val(th, val[j]), ts[j], nt, cnt[j]);
          s_rl[q] = side0[j] ? 0x80 : 0;
        }
      }
    }
    __syncthreads();
    // key runs, one thread per row: at the head of each run of equal keys within one
    // store's rows of a bucket, the run's leaf (its row hashes summed) replaces the head's
    // row hash and the run's length goes to s_rl's low bits (127: longer), so the merge
    // below takes one step per key with all of the step's reads independent.  (Only a
    // head's own thread writes its entries; the others read bit 7 and non-head rows.)
    // Diff 0.169 -> 0.178 of peak back to back, count kernel 68.3 -> 67.4 us in the
    // config-4 round (A/B; the merge used to walk every row with dependent LDS reads).
    for (u32 q = tid; q < R; q += DB) {
      const u64 k = s_k[q];
      if (!(s_rl[q] & 0x80) && s_k[q > 0 ? q - 1 : 0] == k) continue;  // not a head
      u64 sum = s_h[q];
      u32 x = q + 1;
      for (; x < R && !(s_rl[x] & 0x80) && s_k[x] == k; x++) sum += s_h[x];
      s_h[q] = sum;
      s_rl[q] = (unsigned char)((s_rl[q] & 0x80) | min(x - q, 127u));
    }
    __syncthreads();
    DSTAMP(4);
    // merge each differing bucket's keys (one lane per bucket) ONCE: a lane keeps its
    // first KR differing keys in registers, the block scan gives the offsets, and only a
    // lane with more keys than that merges its buckets a second time to write them all
    // (the merge used to run twice for every lane: count, then write)
    constexpr u32 KR = 4;
    u64 kr0 = 0, kr1 = 0, kr2 = 0, kr3 = 0;
    auto merge = [&](bool write, u32 o) {
      u32 k2 = 0;
      // (a lane's buckets are contiguous, so the lanes' outputs in lane order are in
      // bucket order also when there are more differing buckets than lanes)
      const u32 per = (ND + DB - 1) / DB, d1 = min(ND, (tid + 1) * per);
      for (u32 d = tid * per; d < d1; d++) {
        const u32 na = s_dn[d] >> 16;
        u32 ia = s_dp[d], ie = ia + na, jb = ie, je = s_dp[d + 1];
        while (ia < ie || jb < je) {
          // (ia, jb sit on run heads; every read of the step at clamped indices, together)
          const u32 xa = min(ia, R - 1), xb = min(jb, R - 1);
          const u64 ka0 = s_k[xa], kb0 = s_k[xb], ha0 = s_h[xa], hb0 = s_h[xb];
          const u32 la = s_rl[xa] & 127u, lb = s_rl[xb] & 127u;
          const u64 ka = ia < ie ? ka0 : ~0ull, kb = jb < je ? kb0 : ~0ull;
          const u64 k = ka < kb ? ka : kb;
          const bool pa = ia < ie && ka == k, pb = jb < je && kb == k;
          const u64 ha = pa ? ha0 : 0ull, hb = pb ? hb0 : 0ull;
          if (pa) {
            if (la < 127u) ia += la;
            else for (; ia < ie && s_k[ia] == k; ia++) {}
          }
          if (pb) {
            if (lb < 127u) jb += lb;
            else for (; jb < je && s_k[jb] == k; jb++) {}
          }
          if (!(pa && pb) || ha != hb) {
            if (write) {
              p.keys[s_bnd[0] + s_bnd[1] + o + k2] = k;
            } else {
              kr0 = k2 == 0 ? k : kr0;
              kr1 = k2 == 1 ? k : kr1;
              kr2 = k2 == 2 ? k : kr2;
              kr3 = k2 == 3 ? k : kr3;
            }
            k2++;
          }
        }
      }
      return k2;
    };
    const u32 c = merge(false, 0);
    DSTAMP(5);
    u32 t2;
    const u32 o = block_excl_scan<DB>(c, s_wave, &t2);
    if (tid == 0) {
      p.cnt[tile] = t2;
      if (t2) atomicAdd((unsigned long long*)&p.bsum[tile / DB], (unsigned long long)t2);
    }
    if (c > KR) {
      merge(true, o);
    } else {
      // (the subtree's offset re-read from LDS: kept in registers through the kernel, it
      // spilled to scratch, and its reload waited for every store in flight)
      u64* dst = p.keys + (s_bnd[0] + s_bnd[1]) + o;
      if (c > 0) dst[0] = kr0;
      if (c > 1) dst[1] = kr1;
      if (c > 2) dst[2] = kr2;
      if (c > 3) dst[3] = kr3;
    }
    DSTAMP(6);
    return;
  }
  // more differing rows or buckets than the LDS lists hold: each thread merges its owned
  // differing buckets over global memory
  u32 c = 0;
  for (int pass = 0; pass < 2; pass++) {
    u32 o = 0;
    if (pass == 1) {
      u32 t2;
      o = block_excl_scan<DB>(c, s_wave, &t2);
      if (tid == 0) {
        p.cnt[tile] = t2;
        if (t2) atomicAdd((unsigned long long*)&p.bsum[tile / DB], (unsigned long long)t2);
      }
    }
    u32 k2 = 0, ra = offa, rb = offb;
    for (u32 i = 0; i < OWN; i++) {
      // (the counts re-read from memory: indexing the registers by a loop variable here
      // would put them in scratch for the whole kernel)
      const u64 bi = bucket0 + (u64)tid * OWN + i;
      const u32 x = bi - bucket0 < nb ? p.ta.counts[bi] : 0u, y = bi - bucket0 < nb ? p.tb.counts[bi] : 0u;
      if (mine >> i & 1u) {
        if (pass == 0)
          k2 += merge_bucket<false, false>(p.sa, p.ta.th, a0 + ra, a0 + ra + x, p.sb, p.tb.th,
                                           nullptr, nullptr, c0 + rb, c0 + rb + y, nullptr, 0, 0);
        else
          k2 += merge_bucket<false, true>(p.sa, p.ta.th, a0 + ra, a0 + ra + x, p.sb, p.tb.th,
                                          nullptr, nullptr, c0 + rb, c0 + rb + y, p.keys + a0 + c0,
                                          o + k2, ~0ull);
      }
      ra += x;
      rb += y;
    }
    c = k2;
  }
}

#ifdef DG_STAMPS
}  // namespace
extern "C" int dg_debug_diff_stamps(unsigned long long* host, size_t n) {
  if (n > 4096 * 8) n = 4096 * 8;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_df_stamps), n * 8) == hipSuccess ? 0 : -3;
}
namespace {
#endif

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
// the total.  Two round trips: every word the offset and the copy's source need is
// loaded at once (unconditional loads at clamped indices, the unused ones selected away),
// then the keys, all before any store.  (Loads in loops and under branches made it a
// chain of up to nine: count, group sums, the group's counts four times, bounds, keys
// twice.)
__global__ __launch_bounds__(WAVE) void merkle_diff_write_kernel(DiffArgs p) {
  // (subtree `tile`'s keys sit at bnd[tile] + bnd[ntiles + 1 + tile] in scratch)
  const int lane = threadIdx.x;
  const u64 tile = blockIdx.x, grp = tile / DB, g0 = grp * DB;
  if (tile == 0)  // the previous call's group sums: zero for the next call
    for (u64 x = lane; x < p.nzero; x += WAVE) p.bzero[x] = 0;
  const bool last = tile + 1 == p.ntiles;
  constexpr int CQ = DB / WAVE;
  const u64 n = p.cnt[tile];
  const u64 sa = p.bnd[tile], sb = p.bnd[p.ntiles + 1 + tile];
  u64 c[CQ];
#pragma unroll
  for (int q = 0; q < CQ; q++) {
    const u64 x = g0 + (u64)lane + (u64)q * WAVE;
    c[q] = p.cnt[x < tile ? x : tile];
  }
  const u64 b0 = p.bsum[(u64)lane < grp ? (u64)lane : 0ull];
  u64 before = (u64)lane < grp ? b0 : 0ull;
#pragma unroll
  for (int q = 0; q < CQ; q++) before += g0 + (u64)lane + (u64)q * WAVE < tile ? c[q] : 0ull;
  for (u64 x = lane + WAVE; x < grp; x += WAVE) before += p.bsum[x];  // (more than 64 groups)
#pragma unroll
  for (int d = WAVE / 2; d >= 1; d >>= 1) before += __shfl_xor(before, d, WAVE);
  if (last && lane == 0) *p.d_count = before + n;
  // (no keys: an empty subtree, the count kernel's marker, a marker upstream, past cap)
  if (n == 0 || n == DIFF_MISMATCH || before >= DIFF_MISMATCH || before >= p.cap) return;
  const u64 src = sa + sb, m = n < p.cap - before ? n : p.cap - before;
  constexpr int KQ = 4;
  for (u64 x0 = 0; x0 < m; x0 += KQ * WAVE) {
    u64 k[KQ];
#pragma unroll
    for (int q = 0; q < KQ; q++) {
      const u64 x = x0 + (u64)q * WAVE + lane;
      k[q] = p.keys[src + (x < m ? x : m - 1)];
    }
#pragma unroll
    for (int q = 0; q < KQ; q++) {
      const u64 x = x0 + (u64)q * WAVE + lane;
      if (x < m) p.out[before + x] = k[q];
    }
  }
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

// prepare_partial_diff: every node of level L, positions and hashes (host or device)
__global__ __launch_bounds__(PB) void cont_prepare_kernel(MT t, u32 L, u64* opos, u64* ohash) {
  const u64 j = (u64)blockIdx.x * PB + threadIdx.x;
  if (j >> L) return;
  opos[j] = j;
  ohash[j] = t.nodes[((1ull << L) - 1) + j];
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
    for (; x < re && s.key[x] == k; x++) h += rh(s, x, t.th);
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
    c = merge_bucket<true, false>(s, t.th, r, re, s, t.th, pk, ph, j, je, nullptr, 0, 0);
  }
  u32 tot;
  const u32 ex = block_excl_scan<PB>(c, s_wave, &tot);
  if (!WRITE) {
    if (threadIdx.x == 0) cnt[blockIdx.x] = tot;
    return;
  }
  const u64 o = off[blockIdx.x] + ex;
  if (c && o < cap) merge_bucket<true, true>(s, t.th, r, re, s, t.th, pk, ph, j, je, out, o, cap);
}

__global__ void pairs_before_kernel(MT t, const u64* keys, u64 n, const u64* bucket, u64* out) {
  if (threadIdx.x == 0) out[0] = bucket_start(t, keys, n, bucket[0]);
}

// ---------------------------------------------------------------- a small partial-diff hop
// dg_merkle_continue_home: one hop of continue_partial_diff (+ truncate_diff to `max`) for
// a continuation of at most CS_IN entries / CS_B buckets, by ONE workgroup, results written
// straight into the caller's (host) arrays, one host wait -- the general path is three
// to five launches, each waited for.  Same results as dg_merkle_continue followed by
// dg_merkle_truncate(max), except that capacity is asked of the truncated output only.
//   node form, level L < depth : compare, compact the differing positions (input order),
//                                expand by k levels, only the first `max` children made
//   node form, level == depth  : the first `max` differing buckets, their (key, leaf) pairs
//                                from the store (a bucket's rows: an interpolation search
//                                for its first key, the tree's row count for the rest)
//   leaf form                  : per bucket, the store's rows merged with the peer's pairs
//                                (staged in LDS): the differing keys, the first kcap written
// The result header goes to home[0..8) and the sequence number is published (dg_home.h).
constexpr int CSN = 512;  // threads (256 VGPRs: a bucket's 16 rows in registers)
constexpr u32 CS_PER = CS_IN / CSN;
static_assert(CS_IN % CSN == 0, "whole entries per thread");

__device__ __forceinline__ u64 bucket_first_key(const MT& t, u64 b) {
  return (t.sb ? (t.shard << (64 - t.sb)) : 0ull) + (b << (64 - t.sb - t.depth));
}

// the store rows of bucket b: [r, r + counts[b]) (the tree describes the store), clamped
__device__ __forceinline__ void bucket_rows(const MT& t, const Rows& s, u64 b, u64& r, u64& re) {
  r = interp_lower_bound(s.key, 0, s.n, bucket_first_key(t, b));
  re = min<u64>(r + t.counts[b], s.n);
}

// A bucket's (key, leaf) pairs in registers: its rows (at most BR; the tree's row count)
// loaded together -- one round trip after the search, two past BR / 2 rows -- hashed,
// and the runs of equal keys summed (head bit i: row i starts a key, leaf[i] its sum).
// big: more rows than that (the generic loops over global memory).
constexpr int BR = 16;
struct BucketPairs {
  u64 key[BR], leaf[BR];
  u32 head;
  bool big;
  u64 r, re;
};

__device__ __forceinline__ void bucket_pairs(const MT& t, const Rows& s, u64 b, BucketPairs& o) {
  const u32 cnt = t.counts[b];
  const u64 r = interp_lower_bound(s.key, 0, s.n, bucket_first_key(t, b));
  const u64 re = min<u64>(r + cnt, s.n);
  o.r = r;
  o.re = re;
  o.big = re - r > (u64)BR;
  o.head = 0;
  if (o.big || re == r) return;
  const u32 m = (u32)(re - r);
  u64 hs[BR];
#pragma unroll
  for (int half = 0; half < 2; half++) {
    if (half == 1 && m <= (u32)(BR / 2)) {
#pragma unroll
      for (int i = BR / 2; i < BR; i++) {
        o.key[i] = 0;
        hs[i] = 0;
      }
      break;
    }
    u64 k[BR / 2], v[BR / 2], c[BR / 2];
    i64 ts[BR / 2];
    u32 nd[BR / 2];
#pragma unroll
    for (int q = 0; q < BR / 2; q++) {  // every load issued before any is used
      const int i = half * (BR / 2) + q;
      const u64 x = r + (u64)((u32)i < m ? i : m - 1);
      k[q] = s.key[x];
      v[q] = s.val[x];
      ts[q] = s.ts[x];
      nd[q] = s.node[x];
      c[q] = s.cnt[x];
    }
#pragma unroll
    for (int q = 0; q < BR / 2; q++) {
      const int i = half * (BR / 2) + q;
      o.key[i] = k[q];
      hs[i] = row_hash(k[q], th_val(t.th, v[q]), ts[q], th_node(t.th, nd[q]), c[q]);
    }
  }
  u64 acc = 0;
#pragma unroll
  for (int i = BR - 1; i >= 0; i--) {
    const bool valid = (u32)i < m;
    const bool cont = (u32)(i + 1) < m && o.key[i + 1 < BR ? i + 1 : i] == o.key[i];
    acc = valid ? hs[i] + (cont ? acc : 0ull) : 0ull;
    o.leaf[i] = acc;
    if (valid && (i == 0 || o.key[i > 0 ? i - 1 : 0] != o.key[i])) o.head |= 1u << i;
  }
}

// distinct keys of rows [r, re) / their (key, leaf) pairs at out[o..): over global memory
__device__ __forceinline__ u32 distinct_keys(const Rows& s, u64 r, u64 re) {
  u32 c = 0;
  for (u64 x = r; x < re; x++) c += (x == r || s.key[x] != s.key[x - 1]) ? 1u : 0u;
  return c;
}

__device__ __forceinline__ u32 pairs_global(const MT& t, const Rows& s, u64 r, u64 re, u64* opos, u64* ohash,
                                            u64 o) {
  u32 c = 0;
  for (u64 x = r; x < re;) {
    const u64 key = s.key[x];
    u64 lf = 0;
    for (; x < re && s.key[x] == key; x++) lf += rh(s, x, t.th);
    opos[o + c] = key;
    ohash[o + c] = lf;
    c++;
  }
  return c;
}

// merge_bucket with the store side in registers: the keys on one side only or with
// different leaves, ascending (WRITE: out[o..), below cap)
template <bool WRITE>
__device__ __forceinline__ u32 merge_regs(const BucketPairs& bp, const u64* pk, const u64* ph, u64 j, u64 je,
                                          u64* out, u64 o, u64 cap) {
  u32 c = 0;
  auto emit = [&](u64 k) {
    if (WRITE && o + c < cap) out[o + c] = k;
    c++;
  };
#pragma unroll
  for (int i = 0; i < BR; i++) {
    if (!(bp.head >> i & 1u)) continue;
    const u64 k = bp.key[i];
    for (; j < je && pk[j] < k; j++) emit(pk[j]);
    if (j < je && pk[j] == k) {
      if (ph[j] != bp.leaf[i]) emit(k);
      j++;
    } else {
      emit(k);
    }
  }
  for (; j < je; j++) emit(pk[j]);
  return c;
}

__global__ __launch_bounds__(CSN) void cont_small_kernel(ContSmallArgs a, MT t) {
  __shared__ u64 s_dpos[CS_IN];
  __shared__ u64 s_pk[CS_IN], s_ph[CS_IN];  // leaf form in: the peer's pairs; node form: bucket rows
  __shared__ u32 s_wave[CSN / WAVE + 1];
  __shared__ u32 s_bad;
  const int tid = threadIdx.x;
  const u32 depth = t.depth, L = a.level;
  u64 h[CS_HDR] = {0, 0, 0, 0, 0, 0};  // the result header (every thread's copy is the same)
  if (tid == 0) s_bad = 0;
  __syncthreads();
  if (L <= depth) {
    // ---- node form: entries tid*PER .. +PER (consecutive: compaction keeps input order)
    u64 pos[CS_PER];
    u32 d = 0;
    const u64 lim = 1ull << L;
#pragma unroll
    for (u32 q = 0; q < CS_PER; q++) {
      const u64 i = (u64)tid * CS_PER + q;
      const bool ok = i < a.n;
      const u64 ic = ok ? i : 0;  // (n >= 1: the host handles an empty continuation)
      pos[q] = a.ipos[ic];
      const u64 hv = a.ihash[ic];
      if (ok && pos[q] >= lim) atomicOr(&s_bad, 1u);
      const u64 nv = t.nodes[(lim - 1) + (pos[q] < lim ? pos[q] : 0)];
      d |= (ok && pos[q] < lim && nv != hv) ? 1u << q : 0u;
    }
    u32 nd;
    const u32 o = block_excl_scan<CSN>((u32)__popc(d), s_wave, &nd);
    {
      u32 x = o;
#pragma unroll
      for (u32 q = 0; q < CS_PER; q++)
        if (d >> q & 1u) s_dpos[x++] = pos[q];
    }
    __syncthreads();
    if (s_bad) {
      h[0] = CS_BAD;
    } else if (nd == 0) {
      h[0] = CS_OK;  // {:ok, []}
    } else if (L < depth) {
      const u32 k = min(a.levels, depth - L);
      const u64 need = (u64)nd << k, m = min(need, a.max);
      h[3] = L + k;
      if (m > a.ocap) {
        h[0] = CS_CAP;
        h[4] = m;
      } else {
        const u64 mask = (1ull << k) - 1, base = (1ull << (L + k)) - 1;
        for (u64 j = tid; j < m; j += CSN) {
          const u64 p = (s_dpos[j >> k] << k) | (j & mask);
          a.opos[j] = p;
          a.ohash[j] = t.nodes[base + p];
        }
        h[0] = CS_NODE;
        h[1] = m;
      }
    } else {
      // the differing buckets -> leaf form, the first `max` of them: one bucket per thread,
      // its pairs made in registers (the generic loops past CSN buckets)
      const u64 nb = min<u64>(nd, a.max);
      h[3] = depth + 1;
      if (nb <= (u64)CSN) {
        BucketPairs bp;
        bp.big = false;
        bp.head = 0;
        bp.r = bp.re = 0;
        u64 b = 0;
        if ((u64)tid < nb) {
          b = s_dpos[tid];
          bucket_pairs(t, a.s, b, bp);
        }
        const u32 c = bp.big ? distinct_keys(a.s, bp.r, bp.re) : (u32)__popc(bp.head);
        u32 np;
        const u32 po = block_excl_scan<CSN>(c, s_wave, &np);
        if (np > a.ocap || nb > a.ocap_b) {
          h[0] = CS_CAP;
          h[4] = np;
          h[5] = nb;
        } else {
          if ((u64)tid < nb) {
            a.obucket[tid] = b;
            if (bp.big) {
              pairs_global(t, a.s, bp.r, bp.re, a.opos, a.ohash, po);
            } else {
              u64 o2 = po;
#pragma unroll
              for (int i = 0; i < BR; i++)
                if (bp.head >> i & 1u) {
                  a.opos[o2] = bp.key[i];
                  a.ohash[o2++] = bp.leaf[i];
                }
            }
          }
          h[0] = CS_LEAF;
          h[1] = np;
          h[2] = nb;
        }
      } else {
        u32 c = 0;  // this thread's buckets' distinct keys
        u64 r[CS_PER], re[CS_PER];
#pragma unroll
        for (u32 q = 0; q < CS_PER; q++) {
          const u64 u = (u64)tid * CS_PER + q;
          r[q] = re[q] = 0;
          if (u < nb) bucket_rows(t, a.s, s_dpos[u], r[q], re[q]);
          c += distinct_keys(a.s, r[q], re[q]);
        }
        u32 np;
        const u32 po = block_excl_scan<CSN>(c, s_wave, &np);
        if (np > a.ocap || nb > a.ocap_b) {
          h[0] = CS_CAP;
          h[4] = np;
          h[5] = nb;
        } else {
          u64 o2 = po;
#pragma unroll
          for (u32 q = 0; q < CS_PER; q++) {
            const u64 u = (u64)tid * CS_PER + q;
            if (u < nb) a.obucket[u] = s_dpos[u];
            o2 += pairs_global(t, a.s, r[q], re[q], a.opos, a.ohash, o2);
          }
          h[0] = CS_LEAF;
          h[1] = np;
          h[2] = nb;
        }
      }
    }
  } else {
    // ---- leaf form received (<= CS_B = CSN buckets): the peer's pairs staged, then one
    //      bucket per thread, its rows' (key, leaf) pairs in registers merged with them
    static_assert(CS_B <= (u32)CSN, "one bucket per thread");
    for (u64 i = tid; i < a.n; i += CSN) {
      s_pk[i] = a.ipos[i];
      s_ph[i] = a.ihash[i];
    }
    __syncthreads();
    BucketPairs bp;
    bp.big = false;
    bp.head = 0;
    bp.r = bp.re = 0;
    u64 j = 0, je = 0;
    u32 c = 0;
    if ((u64)tid < a.nb) {
      const u64 b = a.ibucket[tid];
      if (b >> depth) {
        atomicOr(&s_bad, 1u);
      } else {
        bucket_pairs(t, a.s, b, bp);
        j = bucket_start(t, s_pk, a.n, b);
        je = bucket_start(t, s_pk, a.n, b + 1);
        c = bp.big ? merge_bucket<true, false>(a.s, t.th, bp.r, bp.re, a.s, t.th, s_pk, s_ph, j, je, nullptr, 0, 0)
                   : merge_regs<false>(bp, s_pk, s_ph, j, je, nullptr, 0, 0);
      }
    }
    u32 tot;
    const u32 ko = block_excl_scan<CSN>(c, s_wave, &tot);
    if (s_bad) {
      h[0] = CS_BAD;
    } else {
      if (c) {
        if (bp.big)
          merge_bucket<true, true>(a.s, t.th, bp.r, bp.re, a.s, t.th, s_pk, s_ph, j, je, a.keys, ko, a.kcap);
        else
          merge_regs<true>(bp, s_pk, s_ph, j, je, a.keys, ko, a.kcap);
      }
      h[0] = CS_OK;
      h[1] = tot;
    }
  }
  if (tid < CS_HDR) {
    u64 v = 0;
#pragma unroll
    for (int i = 0; i < CS_HDR; i++) v = i == tid ? h[i] : v;
    a.home[tid] = v;
  }
  publish_counts(a.d_counts, a.h_pub, a.seq);
}

MT mt_of(const MerkleT& m) {
  MT t;
  t.depth = m.depth;
  t.sb = m.sb;
  t.shard = m.shard;
  t.nodes = m.nodes;
  t.counts = m.counts;
  t.th = m.th;
  t.starts = m.starts;
  return t;
}

inline unsigned grid_of(u64 n, int b) { return (unsigned)((n + b - 1) / b); }

}  // namespace

hipError_t launch_merkle_build(const Rows& s, const MerkleT& m, u64* d_keys, u32* arrive, u64* hand,
                               u32* err, hipStream_t st) {
  const MT t = mt_of(m);
  const u64 G = merkle_chunks(t.depth);
  // 16-byte row loads need 16-byte aligned columns (a view into a packed buffer may not be)
  const bool vec = MERKLE_VEC && !(((uintptr_t)s.key | (uintptr_t)s.val | (uintptr_t)s.ts |
                                    (uintptr_t)s.node | (uintptr_t)s.cnt) & 15);
  if (vec)
    hipLaunchKernelGGL((merkle_chunk_kernel<true, true>), dim3((unsigned)G), dim3(UPB), 0, st, s, t,
                       (const u32*)nullptr, arrive, hand, d_keys, err, (const i64*)nullptr);
  else
    hipLaunchKernelGGL((merkle_chunk_kernel<true, false>), dim3((unsigned)G), dim3(UPB), 0, st, s, t,
                       (const u32*)nullptr, arrive, hand, d_keys, err, (const i64*)nullptr);
  return hipGetLastError();
}

hipError_t launch_merkle_update(const MerkleT& m, const Rows& olds, const Rows& news, const u64* keys,
                                u64 n_keys, u32* dirty, u64* d_keys, u32* arrive, u64* hand, i64* cdelta,
                                u32* err, hipStream_t st) {
  const MT t = mt_of(m);
  const u64 G = merkle_chunks(t.depth);
  i64* cd = t.starts ? cdelta : nullptr;
  if (n_keys)
    hipLaunchKernelGGL(merkle_update_kernel, dim3(grid_of(n_keys, UB)), dim3(UB), 0, st, t, olds, news,
                       keys, n_keys, dirty, d_keys, err, cd);
  hipLaunchKernelGGL(merkle_chunk_kernel<false>, dim3((unsigned)G), dim3(UPB), 0, st, news, t, dirty,
                     arrive, hand, (u64*)nullptr, err, (const i64*)cd);
  return hipGetLastError();
}

hipError_t launch_kd_tree(const MerkleT& m, const u64* keys, const u64* runs, const u64* dh, u64 nk,
                          const u64* guard, int sign, u32* dirty, u32* arrive, u64* hand, i64* cdelta,
                          u32* err, hipStream_t st) {
  const MT t = mt_of(m);
  const u64 G = merkle_chunks(t.depth);
  i64* cd = t.starts ? cdelta : nullptr;
  if (nk)
    hipLaunchKernelGGL(kd_tree_kernel, dim3(grid_of(nk, UB)), dim3(UB), 0, st, t, keys, runs, dh, nk, guard,
                       sign, dirty, err, cd);
  Rows none{};
  hipLaunchKernelGGL(merkle_chunk_kernel<false>, dim3((unsigned)G), dim3(UPB), 0, st, none, t, dirty, arrive,
                     hand, (u64*)nullptr, err, (const i64*)cd);
  return hipGetLastError();
}

hipError_t launch_kd_finish(const KdArgs& p0, const u32* dirty, u32* arrive, u64* hand, const i64* cdelta,
                            hipStream_t st) {
  KdArgs p = p0;
  p.ntiles = (p.nk + KD_BLOCK - 1) / KD_BLOCK;
  const u64 nw = (p.nk + UPB - 1) / UPB;
  const MT t = p.has_tree ? mt_of(p.t) : MT{};
  const u64 G0 = p.has_tree ? merkle_chunks(t.depth) : 0;
#if DG_KDF_EXP == 3
  const u64 G = G0;
#else
  // persistent chunk workgroups: at most 512 (three workgroups per CU beside the write's),
  // at least G / KCH
  const u64 G = G0 ? std::max<u64>(std::min<u64>(G0, 512), (G0 + KCH - 1) / KCH) : 0;
#endif
  if (nw + G == 0) return hipSuccess;
  hipLaunchKernelGGL(kd_finish_kernel, dim3((unsigned)(nw + G)), dim3(UPB), 0, st, p, (u32)nw, t, dirty, arrive,
                     hand, t.starts ? cdelta : (const i64*)nullptr);
  return hipGetLastError();
}

hipError_t launch_cont_prepare(const MerkleT& m, u32 L, u64* opos, u64* ohash, hipStream_t st) {
  hipLaunchKernelGGL(cont_prepare_kernel, dim3(grid_of(1ull << L, PB)), dim3(PB), 0, st, mt_of(m), L, opos, ohash);
  return hipGetLastError();
}

hipError_t launch_cont_small(const ContSmallArgs& a, hipStream_t st) {
  hipLaunchKernelGGL(cont_small_kernel, dim3(1), dim3(CSN), 0, st, a, mt_of(a.t));
  return hipGetLastError();
}

hipError_t launch_merkle_diff(const MerkleT& a, const Rows& sa, const MerkleT& b, const Rows& sb,
                              u64* out_keys, u64 cap, u64* scratch, u64* bsum, u64* bsum_zero, u64 nzero,
                              u64* d_count, hipStream_t st) {
  DiffArgs p;
  p.ta = mt_of(a);
  p.tb = mt_of(b);
  p.sa = sa;
  p.sb = sb;
  p.out = out_keys;
  p.cap = cap;
  p.ntiles = diff_tiles(a.depth);
  p.sub = diff_sub(a.depth);
  p.bnd = scratch;
  p.cnt = scratch + 2 * (p.ntiles + 1);
  p.keys = p.cnt + p.ntiles;
  p.bsum = bsum;  // zero: the write kernel of the call before zeroed it
  p.bzero = bsum_zero;
  p.nzero = nzero;
  p.d_count = d_count;
  // (the subtree bounds are searched inside the count kernel)
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
