// dg_device.h — device-side building blocks shared by the libdeltagpu kernels
// (gfx950 / CDNA4, wave64).
//
//  * Row views over the SoA dot store (include/deltagpu.h) and the full-tuple
//    order (key, val, ts[signed], node, cnt) every store is sorted by.
//  * Causal-context membership: Dots.member?/2 (reference aw_lww_map.ex:67-73).
//  * Wave/block exclusive scans (64-wide shuffles; never 32-wide warp idioms).
//  * The decoupled look-back used for single-pass stream compaction: every tile
//    publishes one 64-bit granule {epoch:20 | flag:2 | value:42} with a relaxed
//    agent-scope atomic store (an `sc1` store) and predecessors poll it with
//    relaxed agent-scope atomic loads.  Data and flag live in the same naturally
//    aligned 8-byte word, so no release/acquire fence is needed (MI355X microarch
//    guide, "Valid forms", R2 granule).  Tiles are numbered by an atomic ticket in
//    launch order, so a tile only waits on tiles that are already resident.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dg {

typedef uint64_t u64;
typedef int64_t i64;
typedef uint32_t u32;

constexpr int WAVE = 64;

struct Rows {
  const u64* key;
  const u64* val;
  const i64* ts;
  const u32* node;
  const u64* cnt;
  u64 n;
};

struct RowsOut {
  u64* key;
  u64* val;
  i64* ts;
  u32* node;
  u64* cnt;
};

struct Ctx {
  const u32* node;
  const u64* cnt;
  u64 n;
  int kind;  // 0 = VV, 1 = explicit dot set
};

struct Row {
  u64 key, val, cnt;
  i64 ts;
  u32 node;
};

__device__ __forceinline__ Row load_row(const Rows& r, u64 i) {
  Row x;
  x.key = r.key[i];
  x.val = r.val[i];
  x.ts = r.ts[i];
  x.node = r.node[i];
  x.cnt = r.cnt[i];
  return x;
}

// A pointer value the optimizer cannot trace back to the memory it was loaded from.
template <class T>
__device__ __forceinline__ T* opaque_ptr(T* p) {
  asm("" : "+s"(p));
  return p;
}

template <class T>
__device__ __forceinline__ T opaque_val(T v) {
  asm("" : "+s"(v));
  return v;
}

// Row g of B if fb else of A.  The per-lane choice is a select between opaque pointer
// VALUES: a select between two loads of struct fields (`fb ? B.key : A.key`) is
// rewritten by the compiler into a load through a selected struct address, which
// spills the kernel's arguments to scratch and turns the row loads into flat loads.
template <class T>
__device__ __forceinline__ T gload(const T* p, u64 g) {  // a global_load, not a flat_load
  return ((const __attribute__((address_space(1))) T*)p)[g];
}

__device__ __forceinline__ Row load_row_sel(const Rows& A, const Rows& B, bool fb, u64 g) {
  // (both opaque values first, then the select: an asm inside each arm of the select
  // makes the compiler branch per column and reload spilled argument SGPRs per branch)
  const u64 *ak = opaque_ptr(A.key), *bk = opaque_ptr(B.key);
  const u64 *av = opaque_ptr(A.val), *bv = opaque_ptr(B.val);
  const i64 *at = opaque_ptr(A.ts), *bt = opaque_ptr(B.ts);
  const u32 *an = opaque_ptr(A.node), *bn = opaque_ptr(B.node);
  const u64 *ac = opaque_ptr(A.cnt), *bc = opaque_ptr(B.cnt);
  Row x;
  x.key = gload(fb ? bk : ak, g);
  x.val = gload(fb ? bv : av, g);
  x.ts = gload(fb ? bt : at, g);
  x.node = gload(fb ? bn : an, g);
  x.cnt = gload(fb ? bc : ac, g);
  return x;
}

// Output row o of a join or fold, with non-temporal stores: the kernels never read their
// output back, and keeping it out of the caches measured 9 % faster on the config-2 join
// (46.5 -> 42.4 us, A/B on one box; non-temporal LOADS of the inputs were slower than
// stores alone).
__device__ __forceinline__ void store_row_nt(const RowsOut& out, u64 o, const Row& x) {
  __builtin_nontemporal_store(x.key, out.key + o);
  __builtin_nontemporal_store(x.val, out.val + o);
  __builtin_nontemporal_store(x.ts, out.ts + o);
  __builtin_nontemporal_store(x.node, out.node + o);
  __builtin_nontemporal_store(x.cnt, out.cnt + o);
}

// The same through the L2 (a row's columns written in pieces by several waves merge there
// before they go to HBM).
__device__ __forceinline__ void store_row(const RowsOut& out, u64 o, const Row& x) {
  out.key[o] = x.key;
  out.val[o] = x.val;
  out.ts[o] = x.ts;
  out.node[o] = x.node;
  out.cnt[o] = x.cnt;
}

// c ? x : y field by field (a conditional on two Row objects selects an ADDRESS and
// copies through it, which keeps both rows in scratch memory).
__device__ __forceinline__ Row row_sel(bool c, const Row& x, const Row& y) {
  Row r;
  r.key = c ? x.key : y.key;
  r.val = c ? x.val : y.val;
  r.ts = c ? x.ts : y.ts;
  r.node = c ? x.node : y.node;
  r.cnt = c ? x.cnt : y.cnt;
  return r;
}

// -1 / 0 / 1 on the full tuple.
__device__ __forceinline__ int row_cmp(const Row& a, const Row& b) {
  if (a.key != b.key) return a.key < b.key ? -1 : 1;
  if (a.val != b.val) return a.val < b.val ? -1 : 1;
  if (a.ts != b.ts) return a.ts < b.ts ? -1 : 1;
  if (a.node != b.node) return a.node < b.node ? -1 : 1;
  if (a.cnt != b.cnt) return a.cnt < b.cnt ? -1 : 1;
  return 0;
}

__device__ __forceinline__ bool row_le(const Row& a, const Row& b) { return row_cmp(a, b) <= 0; }
__device__ __forceinline__ bool row_eq(const Row& a, const Row& b) {
  return (a.key == b.key) & (a.val == b.val) & (a.ts == b.ts) & (a.node == b.node) & (a.cnt == b.cnt);
}

// Branch-free full-tuple comparison for divergent lanes: every field is compared
// unconditionally (ten VALU compares) and the lexicographic result is combined with
// bitwise mask operations, instead of the exec-mask cascade row_cmp's early returns
// compile to.
// (Folded from the last field to the first, so only the two running masks stay live.)
__device__ __forceinline__ void row_cmp_bf(const Row& a, const Row& b, bool& lt, bool& eq) {
  bool l = a.cnt < b.cnt, e = a.cnt == b.cnt;
  l = (a.node < b.node) | ((a.node == b.node) & l);
  e = (a.node == b.node) & e;
  l = (a.ts < b.ts) | ((a.ts == b.ts) & l);
  e = (a.ts == b.ts) & e;
  l = (a.val < b.val) | ((a.val == b.val) & l);
  e = (a.val == b.val) & e;
  lt = (a.key < b.key) | ((a.key == b.key) & l);
  eq = (a.key == b.key) & e;
}

// Dots.member?/2 (aw_lww_map.ex:67-73).  VV: Map.get(vv, node, 0) >= cnt.
// Dot set: exact (node, cnt) membership.  `node`/`cnt` may point at LDS or global
// memory (flat addressing).
__device__ __forceinline__ bool ctx_covers(const u32* node, const u64* cnt, u64 n, int kind,
                                           u32 dn, u64 dc) {
  u64 lo = 0, hi = n;
  if (kind == 0) {
    while (lo < hi) {
      u64 mid = (lo + hi) >> 1;
      if (node[mid] < dn)
        lo = mid + 1;
      else
        hi = mid;
    }
    u64 have = (lo < n && node[lo] == dn) ? cnt[lo] : 0ull;
    return have >= dc;
  }
  while (lo < hi) {
    u64 mid = (lo + hi) >> 1;
    u32 mn = node[mid];
    if (mn < dn || (mn == dn && cnt[mid] < dc))
      lo = mid + 1;
    else
      hi = mid;
  }
  return lo < n && node[lo] == dn && cnt[lo] == dc;
}

// First index of keys[0, n) (ascending) that is >= x, by ONE wave: a 64-ary search
// (every step probes 64 positions, one dependent load round: 12.5M rows in 4 rounds
// instead of a 24-load binary-search chain).  Every lane returns the same value.
__device__ __forceinline__ u64 wave_lower_bound(const u64* k, u64 n, u64 x) {
  const int lane = threadIdx.x & (WAVE - 1);
  u64 lo = 0, hi = n;
  while (hi - lo > WAVE) {
    const u64 span = hi - lo;
    const u64 p = lo + span * (u64)(lane + 1) / (WAVE + 1);
    const u64 m = __ballot(k[p] < x);  // true on a prefix of the lanes
    const int c = __popcll(m);
    const u64 nlo = c ? lo + span * (u64)c / (WAVE + 1) + 1 : lo;
    const u64 nhi = c < WAVE ? lo + span * (u64)(c + 1) / (WAVE + 1) : hi;
    lo = nlo;
    hi = nhi;
  }
  const bool lt = lo + lane < hi && k[lo + lane] < x;
  return lo + (u64)__popcll(__ballot(lt));
}

// First index in [lo, hi) whose key is >= x (hi if none), keys ascending.  Key ids are
// 64-bit hashes, uniform over the store's range, so the answer lies within about
// sqrt(m f (1 - f)) rows of the interpolated position in a bracket of m rows: each round
// probes the two rows 2 such deviations either side of it (two independent loads, one
// round trip) and keeps the sub-bracket that holds x -- about 7000, 170, 30, then <= 16
// rows at 12.5M uniform keys -- and the last <= 16 keys (one or two cache lines) are
// read at once.  About 6 dependent memory rounds instead of a binary search's 24 (a
// one-sided interpolation search stalls on one side: 29-30 probes for 1 key in 10).
// Exact for any key distribution: a round that does not bracket still narrows, and the
// finish is a plain binary search once the round budget is spent.
__device__ __forceinline__ u64 interp_lower_bound(const u64* k, u64 lo, u64 hi, u64 x) {
  if (lo >= hi) return lo;
  u64 kl = k[lo], kh = k[hi - 1];
  if (x <= kl) return lo;
  if (x > kh) return hi;
  u64 a = lo, b = hi - 1;  // k[a] < x <= k[b]: the answer is in (a, b]
#pragma unroll 1
  for (int it = 0; it < 6 && b - a > 16; it++) {
    const double m = (double)(b - a);
    const double f = (double)(x - kl) / (double)(kh - kl);
    const double g = (double)a + f * m;
    const double e = 2.0 * __builtin_sqrt(m * f * (1.0 - f)) + 4.0;
    const double lo_g = g - e, hi_g = g + e;
    const u64 g0 = lo_g <= (double)(a + 1) ? a + 1 : (lo_g >= (double)(b - 1) ? b - 1 : (u64)lo_g);
    const u64 g1 = hi_g <= (double)(a + 1) ? a + 1 : (hi_g >= (double)(b - 1) ? b - 1 : (u64)hi_g);
    const u64 k0 = k[g0], k1 = k[g1];
    if (k0 >= x) {
      b = g0;
      kh = k0;
    } else if (k1 < x) {
      a = g1;
      kl = k1;
    } else {
      a = g0;
      kl = k0;
      b = g1;
      kh = k1;
    }
  }
  if (b - a <= 16) {  // the keys of (a, b): loaded together, counted
    // (every load unconditional at a clamped index: a load under `a + j < b &&` was a
    // branch, and each was waited for before the next went out -- 15 round trips)
    // every load issued before any compare (the empty asm is a compiler barrier for memory
    // operations: without it the scheduler waits for each load before issuing the next)
    u64 v[15];
#pragma unroll
    for (u64 j = 1; j < 16; j++) v[j - 1] = k[a + j < b ? a + j : a];
    asm volatile("" ::: "memory");
    u64 c = 0;
#pragma unroll
    for (u64 j = 1; j < 16; j++) c += ((a + j < b) & (v[j - 1] < x)) ? 1 : 0;
    return a + 1 + c;
  }
  u64 l2 = a + 1, h2 = b;
  while (l2 < h2) {
    const u64 mid = (l2 + h2) >> 1;
    if (k[mid] < x)
      l2 = mid + 1;
    else
      h2 = mid;
  }
  return l2;
}

__device__ __forceinline__ bool keyset_has(const u64* keys, u64 n, u64 k) {
  u64 lo = 0, hi = n;
  while (lo < hi) {
    u64 mid = (lo + hi) >> 1;
    if (keys[mid] < k)
      lo = mid + 1;
    else
      hi = mid;
  }
  return lo < n && keys[lo] == k;
}

// Inclusive scan of a 32-bit value across the 64 lanes of a wave, on the DPP network
// (a few cycles a step) instead of ds_bpermute shuffles (an LDS round trip each): row_shr
// 1/2/4/8 scans each row of 16 lanes, row_bcast:15 carries row 0 into row 1 (and row 2
// into row 3), row_bcast:31 carries rows 0-1 into rows 2-3.  Lanes a step does not write
// add the `old` operand, 0.
__device__ __forceinline__ u32 wave_incl_scan(u32 v) {
  v += (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false);  // row_shr:1
  v += (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false);  // row_shr:2
  v += (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false);  // row_shr:4
  v += (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false);  // row_shr:8
  v += (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false);  // row_bcast:15
  v += (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false);  // row_bcast:31
  return v;
}

// Inclusive max-scan of a 32-bit value across the wave (DPP, as wave_incl_scan).
__device__ __forceinline__ u32 wave_incl_max(u32 v) {
  v = max(v, (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false));
  v = max(v, (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false));
  v = max(v, (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false));
  v = max(v, (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false));
  v = max(v, (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false));
  v = max(v, (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false));
  return v;
}

// The value of the previous lane (lane 0: 0), DPP wave_shr:1.
__device__ __forceinline__ u32 wave_prev(u32 v) {
  return (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x138, 0xf, 0xf, false);
}

// lane l - 1's value, lane 0 gets `first`.  Pass lane 0's own value here rather than
// selecting it after the shift (`lane ? wave_prev(v) : x`): the compiler may move the DPP
// into the `lane != 0` branch of such a select, where lane 0 -- the source of lane 1 --
// is inactive and lane 1 reads the old value (a wrong Merkle bucket count, seen on gfx950).
__device__ __forceinline__ u32 wave_prev_or(u32 v, u32 first) {
  return (u32)__builtin_amdgcn_update_dpp((int)first, (int)v, 0x138, 0xf, 0xf, false);
}

// Sum of a 32-bit value over the wave (every lane gets it).
__device__ __forceinline__ u32 wave_sum_u32(u32 v) {
  return (u32)__builtin_amdgcn_readlane((int)wave_incl_scan(v), WAVE - 1);
}

// Sum over the wave of values below 2^42 (look-back granules): two 21-bit halves, each
// summed on the DPP network (64 x 2^21 fits 32 bits).
__device__ __forceinline__ u64 wave_sum_42(u64 v) {
  return ((u64)wave_sum_u32((u32)(v >> 21)) << 21) + (u64)wave_sum_u32((u32)(v & 0x1FFFFFull));
}

// Exclusive block scan; returns the exclusive prefix of `v` and the block total in
// *total.  `s_wave` must hold BLOCK/64 + 1 words of LDS.
template <int BLOCK>
__device__ __forceinline__ u32 block_excl_scan(u32 v, u32* s_wave, u32* total) {
  constexpr int NW = BLOCK / WAVE;
  const int lane = threadIdx.x & (WAVE - 1);
  const int w = threadIdx.x / WAVE;
  u32 inc = wave_incl_scan(v);
  if (lane == WAVE - 1) s_wave[w] = inc;
  __syncthreads();
  if (threadIdx.x == 0) {
    u32 run = 0;
#pragma unroll
    for (int i = 0; i < NW; i++) {
      u32 t = s_wave[i];
      s_wave[i] = run;
      run += t;
    }
    s_wave[NW] = run;
  }
  __syncthreads();
  *total = s_wave[NW];
  return s_wave[w] + inc - v;
}

// The same scan with ONE barrier: every wave reads all BLOCK/64 wave totals and scans them
// itself on the DPP network (reading its own prefix and the total with readlane), instead
// of one thread prefixing them between two barriers.  Every wave reads every s_wave entry,
// so the next write of s_wave (e.g. the next scan on the same scratch) needs a barrier
// after this call; block_excl_scan above has no such precondition.
template <int BLOCK>
__device__ __forceinline__ u32 block_excl_scan1(u32 v, u32* s_wave, u32* total) {
  constexpr int NW = BLOCK / WAVE;
  static_assert(NW <= WAVE, "one wave total per lane");
  const int lane = threadIdx.x & (WAVE - 1);
  const int w = threadIdx.x / WAVE;
  const u32 inc = wave_incl_scan(v);
  if (lane == WAVE - 1) s_wave[w] = inc;
  __syncthreads();
  const u32 ws = wave_incl_scan(lane < NW ? s_wave[lane] : 0u);
  const u32 below = w > 0 ? (u32)__builtin_amdgcn_readlane((int)ws, w - 1) : 0u;
  *total = (u32)__builtin_amdgcn_readlane((int)ws, NW - 1);
  return below + inc - v;
}

// ---------------------------------------------------------------- tile offsets
// Exclusive offsets of per-tile counts by ONE workgroup of NT threads (the middle pass
// of count / scan / write compactions, used where every tile of a launch is resident
// at once and a decoupled look-back would make each tile poll a whole round of
// predecessors).  cnt values must be < 2^32 / NT.  *total = the sum.
template <int NT>
__device__ __forceinline__ void scan_tile_counts(const u64* cnt, u64* off, u64 ntiles, u64* total,
                                                 u32* s_wave, u64* s_carry) {
  if (threadIdx.x == 0) *s_carry = 0;
  __syncthreads();
  for (u64 c0 = 0; c0 < ntiles; c0 += NT) {
    const u64 t = c0 + threadIdx.x;
    const u32 v = t < ntiles ? (u32)cnt[t] : 0u;
    u32 tot;
    const u32 o = block_excl_scan<NT>(v, s_wave, &tot);
    if (t < ntiles) off[t] = *s_carry + o;
    __syncthreads();
    if (threadIdx.x == 0) *s_carry += tot;
    __syncthreads();
  }
  if (threadIdx.x == 0) *total = *s_carry;
}

// ---------------------------------------------------------------- look-back
constexpr u64 LB_VALUE_MASK = (1ull << 42) - 1;
constexpr u32 LB_AGG = 1, LB_INC = 2;

__device__ __forceinline__ u64 lb_pack(u32 epoch, u32 flag, u64 value) {
  return ((u64)epoch << 44) | ((u64)flag << 42) | (value & LB_VALUE_MASK);
}

__device__ __forceinline__ void lb_publish(u64* state, u64 tile, u32 epoch, u32 flag, u64 value) {
  __hip_atomic_store(state + tile, lb_pack(epoch, flag, value), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}

// Called by ONE full wave of the tile (tile > 0) after it published its aggregate.
// Returns the exclusive prefix of tile `tile` (same value in every lane).  Spins are
// bounded: on timeout *err gets bit 0 set and the partial prefix is returned.
__device__ __forceinline__ u64 lb_lookback(u64* state, u64 tile, u32 epoch, u32* err) {
  const int lane = threadIdx.x & (WAVE - 1);
  u64 prefix = 0;
  i64 base = (i64)tile - 1;
  u32 spins = 0;
  while (true) {
    i64 idx = base - lane;
    u32 flag;
    u64 value;
    if (idx >= 0) {
      u64 w = __hip_atomic_load(state + idx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      bool cur = (u32)(w >> 44) == epoch;
      flag = cur ? (u32)((w >> 42) & 3) : 0u;
      value = w & LB_VALUE_MASK;
    } else {
      flag = LB_INC;
      value = 0;
    }
    u64 inc_mask = __ballot(flag == LB_INC);
    u64 zero_mask = __ballot(flag == 0);
    if (inc_mask) {
      int first = __ffsll((long long)inc_mask) - 1;  // nearest inclusive predecessor
      u64 upto = (first == 63) ? ~0ull : ((2ull << first) - 1);
      if ((zero_mask & upto) == 0) {
        u64 contrib = (lane <= first) ? value : 0;
        contrib = wave_sum_42(contrib);
        return prefix + contrib;
      }
    } else if (zero_mask == 0) {
      u64 contrib = value;
      contrib = wave_sum_42(contrib);
      prefix += contrib;
      base -= WAVE;
      continue;
    }
    if (++spins > (1u << 24)) {
      if (lane == 0) atomicOr(err, 1u);
      return prefix;
    }
    __builtin_amdgcn_s_sleep(1);
  }
}

// Block-wide decoupled look-back: EVERY thread of the NT-thread block calls it after
// the block published its aggregate (tile > 0).  Thread t reads predecessors
// base - (t*Q + q), q < Q, so one round reaches NT*Q tiles back: when all tiles of a
// launch round progress in lockstep (no inclusive prefix published yet), a tile still
// resolves its prefix in one or two round trips instead of tile/64.  `s_lb` is LDS
// scratch of 3 * NT/64 + 2 u64.  Spins are bounded (err bit 0 on timeout).
template <int NT, int Q>
__device__ __forceinline__ u64 lb_lookback_block(u64* state, u64 tile, u32 epoch, u32* err,
                                                 u64* s_lb) {
  constexpr int NW = NT / WAVE;
  const int tid = threadIdx.x, lane = tid & (WAVE - 1), w = tid / WAVE;
  u64 prefix = 0;
  i64 base = (i64)tile - 1;
  u32 spins = 0;
  while (true) {
    u32 fl[Q];
    u64 vl[Q];
#pragma unroll
    for (int q = 0; q < Q; q++) {
      const i64 idx = base - ((i64)tid * Q + q);
      if (idx >= 0) {
        const u64 g = __hip_atomic_load(state + idx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        fl[q] = ((u32)(g >> 44) == epoch) ? (u32)((g >> 42) & 3) : 0u;
        vl[q] = g & LB_VALUE_MASK;
      } else {
        fl[q] = LB_INC;
        vl[q] = 0;
      }
    }
    int qi = Q;
#pragma unroll
    for (int q = Q - 1; q >= 0; q--)
      if (fl[q] == LB_INC) qi = q;
    bool zb = false;
    u64 part = 0;
#pragma unroll
    for (int q = 0; q < Q; q++)
      if (q <= qi) {
        zb |= fl[q] == 0;
        part += vl[q];
      }
    const u64 im = __ballot(qi < Q), bm = __ballot(zb);
    const int first = im ? __ffsll((long long)im) - 1 : WAVE;
    const u64 upto = first >= WAVE - 1 ? ~0ull : ((2ull << first) - 1);
    u64 c = lane <= first ? part : 0;
    c = wave_sum_42(c);
    if (lane == 0) {
      s_lb[w] = c;
      s_lb[NW + w] = im != 0;
      s_lb[2 * NW + w] = (bm & upto) == 0;
    }
    __syncthreads();
    if (tid == 0) {
      u64 acc = 0, st = 2;  // 2: all ready, no inclusive prefix yet -> go further back
      for (int ww = 0; ww < NW; ww++) {
        if (!s_lb[2 * NW + ww]) {
          st = 0;  // a granule before the nearest inclusive prefix is not ready
          break;
        }
        acc += s_lb[ww];
        if (s_lb[NW + ww]) {
          st = 1;
          break;
        }
      }
      s_lb[3 * NW] = st;
      s_lb[3 * NW + 1] = acc;
    }
    __syncthreads();
    const u64 st = s_lb[3 * NW], acc = s_lb[3 * NW + 1];
    __syncthreads();
    if (st == 1) return prefix + acc;
    if (st == 2) {
      prefix += acc;
      base -= (i64)NT * Q;
      continue;
    }
    if (++spins > (1u << 22)) {
      if (tid == 0) atomicOr(err, 1u);
      return prefix;
    }
    __builtin_amdgcn_s_sleep(1);
  }
}

}  // namespace dg
