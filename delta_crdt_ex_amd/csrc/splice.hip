// splice.hip — a sparse keyed join applied to a large device-resident state.
//
// CausalCrdt applies every sync delta as join(state, delta, keys)
// (reference causal_crdt.ex:383-384; aw_lww_map.ex:153-209).  A delta carries the rows of
// a few keys (Map.take(value, keys), causal_crdt.ex:324-335), so the join changes only
// those keys; every other key keeps its rows (the right-biased carry of :185-188 hands A's
// rows through when B lacks the key).  Merging the whole state (dg_join2's stream kernel)
// reads and writes every row through the merge; the splice instead
//   1. takes the state's rows of the keyset out (take_keys_kernel with the per-key index:
//      a_lo[u], the first row >= K[u], and a_off[u], the rows of K[0..u)),
//   2. joins them with the delta on the join kernels (small: the edit E, = the output's
//      rows of every key of K, sorted),
//   3. (this file) computes per key where the untouched rows between two keyset keys move
//      (splice_index_kernel), moves E's rows into their holes (splice_erows_kernel, one
//      thread per key) and the untouched rows to their new positions in one streaming
//      pass (splice_kernel) -- or not at all when no key's row count changed and the
//      output is the state itself (dg_join_delta in place).
// The output is bit-identical to the full keyed join's whenever the delta's keys are a
// subset of the keyset; the caller checks that first (splice_check_kernel) and otherwise
// takes the full join.
//
// Positions.  With PA[u] = a_off[u] (state rows of K[0..u)) and PE[u] = E's rows with key
// < K[u], a state row i outside K whose first keyset key above it is K[u] goes to
// i - PA[u] + PE[u]: the shift of its gap.  E's row j of key K[u] goes to
// j + a_lo[u] - PA[u]: the state rows outside K before K[u] come first.
//
// Roofline: the copy is 36 B read + 36 B written per untouched row, plus E's rows; the
// index is O(|K| log |E|).  Nothing else touches the state.
#include "dg_home.h"
#include "dg_launch.h"

namespace dg {

namespace {

constexpr int SB = 256;            // threads per workgroup
constexpr int SR = 8;              // rows per thread (held in registers: 72 VGPRs)
constexpr int ST = SB * SR;        // rows per tile
constexpr int SLC = 1024;          // keyset entries of a tile staged in LDS

// first index in [0, n) whose value is > x (a nondecreasing), by all lanes of one wave:
// 64-ary rounds (3 at 2^18 entries) instead of a binary search's 18 dependent loads
__device__ __forceinline__ u64 wave_upper(const u64* a, u64 n, u64 x) {
  const int lane = threadIdx.x & (WAVE - 1);
  u64 lo = 0, hi = n;
  while (hi - lo > WAVE) {
    const u64 span = hi - lo;
    const u64 q = lo + span * (u64)(lane + 1) / (WAVE + 1);
    const int c = __popcll(__ballot(a[q] <= x));  // true on a prefix of the lanes
    const u64 nlo = c ? lo + span * (u64)c / (WAVE + 1) + 1 : lo;
    const u64 nhi = c < WAVE ? lo + span * (u64)(c + 1) / (WAVE + 1) : hi;
    lo = nlo;
    hi = nhi;
  }
  const bool le = lo + lane < hi && a[lo + lane] <= x;
  return lo + (u64)__popcll(__ballot(le));
}

__device__ __forceinline__ u64 lower_bound(const u64* a, u64 lo, u64 hi, u64 x) {
  while (lo < hi) {
    const u64 m = (lo + hi) >> 1;
    if (a[m] < x)
      lo = m + 1;
    else
      hi = m;
  }
  return lo;
}

// ---- locate (the take's first half by streaming): one workgroup per LT state rows
// stages the tile's keys in LDS (coalesced, 16 KB) and finds, for every keyset key whose
// first row >= it lies in the tile -- keys in (key[i0 - 1], key[i1 - 1]], the last tile
// also the keys above every row -- that row and the key's rows (a run may continue past
// the tile, read from global memory).
constexpr int LT = 2048;
__global__ __launch_bounds__(SB) void splice_locate_kernel(Rows s, const u64* keys, u64 nk, u64* lo,
                                                           u32* len) {
  __shared__ u64 s_k[LT];
  __shared__ u64 s_b[2];
  const u64 t = blockIdx.x;
  const u64 i0 = t * LT, i1 = min<u64>(i0 + LT, s.n);
  if (threadIdx.x < WAVE) {
    const u64 u = t == 0 ? 0 : wave_upper(keys, nk, s.key[i0 - 1]);
    if (threadIdx.x == 0) s_b[0] = u;
  } else if (threadIdx.x < 2 * WAVE) {
    const u64 u = i1 == s.n ? nk : wave_upper(keys, nk, s.key[i1 - 1]);
    if ((threadIdx.x & (WAVE - 1)) == 0) s_b[1] = u;
  }
  const u32 m = (u32)(i1 - i0);
  for (u32 j = 2 * threadIdx.x; j < m; j += 2 * SB) {  // 16-byte loads (i0 is even)
    if (j + 1 < m) {
      const ulonglong2 v = *(const ulonglong2*)(s.key + i0 + j);
      s_k[j] = v.x;
      s_k[j + 1] = v.y;
    } else {
      s_k[j] = s.key[i0 + j];
    }
  }
  __syncthreads();
  for (u64 u = s_b[0] + threadIdx.x; u < s_b[1]; u += SB) {
    const u64 x = keys[u];
    u32 a = 0, b = m;
    while (a < b) {
      const u32 h = (a + b) >> 1;
      if (s_k[h] < x)
        a = h + 1;
      else
        b = h;
    }
    u32 e = a;
    while (e < m && s_k[e] == x) e++;
    u64 g = i0 + e;
    if (e == m)  // the run may go on into the next tiles
      while (g < s.n && s.key[g] == x) g++;
    lo[u] = i0 + a;
    len[u] = (u32)(g - (i0 + a));
  }
}

__global__ __launch_bounds__(SB) void splice_check_kernel(const u64* bkey, u64 nb, const u64* keys,
                                                          u64 nk, u64* d_bad) {
  const u64 j = (u64)blockIdx.x * SB + threadIdx.x;
  if (j >= nb) return;
  const u64 k = bkey[j];
  if (j > 0 && bkey[j - 1] == k) return;  // one probe per key
  const u64 u = interp_lower_bound(keys, 0, nk, k);
  if (u == nk || keys[u] != k) atomicAdd((unsigned long long*)d_bad, 1ull);
}

// per keyset entry u: end[u], gap[u] and shift[u] (shift[nk]: after the last key), and
// the first entry of every state tile whose first row falls in [end[u-1], end[u]) (so
// the copy's tiles look their entry range up instead of searching for it)
__global__ __launch_bounds__(SB) void splice_index_kernel(SpliceArgs p) {
  if (p.run_if && *p.run_if == 0) return;  // (uniform) nothing moved: not needed
  const u64 u = (u64)blockIdx.x * SB + threadIdx.x;
  if (u > p.nk) return;
  const u64 ne = *p.d_ne;
  const u64 pa = p.a_off[u];
  const u64 pe = u < p.nk ? interp_lower_bound(p.e.key, 0, ne, p.keys[u]) : ne;
  p.shift[u] = (i64)pe - (i64)pa;
  if (pe != pa) atomicOr(p.moved, 1u);
  const u64 end_hi = u < p.nk ? p.a_lo[u] + (p.a_off[u + 1] - pa) : ~0ull;
  const u64 end_lo = u > 0 ? p.a_lo[u - 1] + (pa - p.a_off[u - 1]) : 0ull;
  if (u < p.nk) {
    p.end[u] = end_hi;
    p.gap[u] = (i64)p.a_lo[u] - (i64)pa;
  }
  for (u64 t = (end_lo + ST - 1) / ST; t <= p.a_tiles && t * ST < end_hi; t++) p.tile_u0[t] = u;
}

// A tile's rows, loaded before anything says where they go.  Thread t holds the row
// pairs (2 (q SB + t), +1), q < SR / 2: every column is read with 16-byte loads (8 bytes
// for the node column), a wave covering 1 KB of a column per instruction.  Loads and wide
// stores are non-temporal: the rows stream through once (A/B on one box: 177-180 ->
// 149-151 us per 12.5M-row splice, ~6.0 TB/s, the float4-copy ceiling).
constexpr int SP = SR / 2;  // row pairs per thread
struct TileRows {
  u64 key[SR], val[SR], cnt[SR];
  i64 ts[SR];
  u32 node[SR];
};

__device__ __forceinline__ u64 pair_row(u64 j0, int q, int h) {
  return j0 + 2 * ((u64)q * SB + threadIdx.x) + (u64)h;
}

typedef unsigned long long v2u64 __attribute__((ext_vector_type(2)));
typedef unsigned int v2u32 __attribute__((ext_vector_type(2)));

template <class T>
__device__ __forceinline__ void load2(const T* c, u64 j, u64 j1, T& x0, T& x1) {
  if (j + 1 < j1) {  // j even: an aligned pair
    if constexpr (sizeof(T) == 8) {
      const v2u64 v = __builtin_nontemporal_load((const v2u64*)(c + j));
      x0 = (T)v.x;
      x1 = (T)v.y;
    } else {
      const v2u32 v = __builtin_nontemporal_load((const v2u32*)(c + j));
      x0 = (T)v.x;
      x1 = (T)v.y;
    }
  } else if (j < j1) {
    x0 = c[j];
  }
}

template <class T>
__device__ __forceinline__ void store2(T* c, i64 t0, i64 t1, T x0, T x1) {
  if (t0 >= 0 && t1 == t0 + 1 && !(t0 & 1)) {  // contiguous and aligned: one wide store
    if constexpr (sizeof(T) == 8) {
      __builtin_nontemporal_store(v2u64{(unsigned long long)x0, (unsigned long long)x1}, (v2u64*)(c + t0));
    } else {
      __builtin_nontemporal_store(v2u32{(u32)x0, (u32)x1}, (v2u32*)(c + t0));
    }
  } else {
    if (t0 >= 0) c[t0] = x0;
    if (t1 >= 0) c[t1] = x1;
  }
}

__device__ __forceinline__ void load_tile(const Rows& r, u64 j0, u64 j1, TileRows& x) {
#pragma unroll
  for (int q = 0; q < SP; q++) {
    const u64 j = pair_row(j0, q, 0);
    load2(r.key, j, j1, x.key[2 * q], x.key[2 * q + 1]);
    load2(r.val, j, j1, x.val[2 * q], x.val[2 * q + 1]);
    load2(r.ts, j, j1, x.ts[2 * q], x.ts[2 * q + 1]);
    load2(r.node, j, j1, x.node[2 * q], x.node[2 * q + 1]);
    load2(r.cnt, j, j1, x.cnt[2 * q], x.cnt[2 * q + 1]);
  }
}

__device__ __forceinline__ void store_tile(const RowsOut& o, const TileRows& x, const i64 (&to)[SR]) {
#pragma unroll
  for (int q = 0; q < SP; q++) {
    const i64 t0 = to[2 * q], t1 = to[2 * q + 1];
    store2(o.key, t0, t1, x.key[2 * q], x.key[2 * q + 1]);
    store2(o.val, t0, t1, x.val[2 * q], x.val[2 * q + 1]);
    store2(o.ts, t0, t1, x.ts[2 * q], x.ts[2 * q + 1]);
    store2(o.node, t0, t1, x.node[2 * q], x.node[2 * q + 1]);
    store2(o.cnt, t0, t1, x.cnt[2 * q], x.cnt[2 * q + 1]);
  }
}

// E's rows: one thread per keyset entry u moves its key's rows [PE[u], PE[u + 1]) of E
// (PE = shift + a_off) to j + gap[u] -- no search: the index kernel has placed them.
__global__ __launch_bounds__(SB) void splice_erows_kernel(SpliceArgs p) {
  if (p.run_if && *p.run_if == 0) return;  // (uniform) nothing moved: not needed
  const u64 u = (u64)blockIdx.x * SB + threadIdx.x;
  if (u >= p.nk) return;
  if (p.guard && (*p.guard & MERKLE_INPUT_ERR)) return;  // the tree update failed: no write
  const u64 j0 = (u64)(p.shift[u] + (i64)p.a_off[u]), j1 = (u64)(p.shift[u + 1] + (i64)p.a_off[u + 1]);
  const i64 g = p.gap[u];
  for (u64 j = j0; j < j1; j++) {
    const u64 o = (u64)((i64)j + g);
    p.out.key[o] = p.e.key[j];
    p.out.val[o] = p.e.val[j];
    p.out.ts[o] = p.e.ts[j];
    p.out.node[o] = p.e.node[j];
    p.out.cnt[o] = p.e.cnt[j];
  }
}

// One workgroup per ST state rows: every row outside the keyset to its place.  The
// workgroup issues its rows' loads first: the index entries that place them are staged
// while the loads are in flight.
static_assert(ST == SPLICE_TILE, "dg_launch.h's copy tile");
__global__ __launch_bounds__(SB) void splice_kernel(SpliceArgs p) {
  __shared__ u64 s_end[SLC], s_lo[SLC];
  __shared__ i64 s_shift[SLC];
  __shared__ u32 s_all;
  // (uniform) nothing moved, or the index was not written: no copy
  const bool run = !(p.run_if && *p.run_if == 0) && !(p.kguard && *p.kguard);
  // (a grid-stride loop over the tiles: launch_splice_move's grid is capped, so a launch
  // whose rows did not move exits in a few us whatever the state's size)
  for (u64 t = blockIdx.x; run && t < p.a_tiles; t += gridDim.x) {
  TileRows x;
  i64 to[SR];
  const u64 i0 = t * ST;
  const u64 i1 = min<u64>(i0 + ST, p.a.n);
  // row i's first keyset entry whose state rows end after it: u*(i) = first u with
  // end[u] > i (nk if none); the tile's rows have u* in [u0, u1] (the index kernel's
  // first entries of this tile and the next)
  const u64 u0 = p.tile_u0[t], u1 = p.tile_u0[t + 1];
  load_tile(p.a, i0, i1, x);
  const u64 m = u1 - u0 + 1;
  const bool staged = m <= (u64)SLC;  // block-uniform
  if (staged) {
    for (u64 e = threadIdx.x; e < m; e += SB) {
      const u64 u = u0 + e;
      s_end[e] = u < p.nk ? p.end[u] : ~0ull;
      s_lo[e] = u < p.nk ? p.a_lo[u] : ~0ull;
      s_shift[e] = p.shift[u];
    }
    __syncthreads();
  }
#pragma unroll
  for (int q = 0; q < SR; q++) {
    const u64 i = pair_row(i0, q >> 1, q & 1);
    to[q] = -1;
    if (i >= i1) continue;
    u64 lo = 0, hi = m - 1;  // entry u0 + lo: the first whose end is > i (u1's is)
    if (staged) {
      while (lo < hi) {
        const u64 mid = (lo + hi) >> 1;
        if (s_end[mid] > i)
          hi = mid;
        else
          lo = mid + 1;
      }
      if (s_lo[lo] > i) to[q] = (i64)i + s_shift[lo];  // else: a keyset key's row (E's)
    } else {
      while (lo < hi) {
        const u64 mid = (lo + hi) >> 1;
        if (p.end[u0 + mid] > i)
          hi = mid;
        else
          lo = mid + 1;
      }
      const u64 u = u0 + lo;
      if (u == p.nk || p.a_lo[u] > i) to[q] = (i64)i + p.shift[u];
    }
  }
  store_tile(p.out, x, to);
  __syncthreads();  // (the next tile restages the index)
  }
  if (!p.h_pub) return;
  if (!run) {  // (uniform) no workgroup copies: the first publishes right away
    if (blockIdx.x == 0) publish_counts(p.pub_counts, p.h_pub, p.seq);
    return;
  }
  // every workgroup arrives once its part is done; the last one publishes (dg_home.h)
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
    publish_counts(p.pub_counts, p.h_pub, p.seq);
  }
}

}  // namespace

hipError_t launch_splice_locate(const Rows& s, const u64* keys, u64 n_keys, u64* lo, u32* len,
                                hipStream_t st) {
  const u64 tiles = (s.n + LT - 1) / LT;
  if (tiles == 0 || n_keys == 0) return hipSuccess;
  hipLaunchKernelGGL(splice_locate_kernel, dim3((unsigned)tiles), dim3(SB), 0, st, s, keys, n_keys,
                     lo, len);
  return hipGetLastError();
}

hipError_t launch_splice_check(const u64* bkey, u64 nb, const u64* keys, u64 nk, u64* d_bad,
                               hipStream_t st) {
  if (nb == 0) return hipSuccess;
  hipLaunchKernelGGL(splice_check_kernel, dim3((unsigned)((nb + SB - 1) / SB)), dim3(SB), 0, st,
                     bkey, nb, keys, nk, d_bad);
  return hipGetLastError();
}

u64 splice_tiles(u64 n) { return (n + ST - 1) / ST; }

hipError_t launch_splice_index(SpliceArgs p, hipStream_t st) {
  p.a_tiles = (p.a.n + ST - 1) / ST;
  hipLaunchKernelGGL(splice_index_kernel, dim3((unsigned)((p.nk + 1 + SB - 1) / SB)), dim3(SB), 0,
                     st, p);
  return hipGetLastError();
}

hipError_t launch_splice_move(SpliceArgs p, hipStream_t st) {
  p.a_tiles = (p.a.n + ST - 1) / ST;
  u64 g = p.a_tiles < 512 ? p.a_tiles : 512;  // (a launch whose rows did not move: ~2 us)
  if (p.h_pub && g == 0) g = 1;                // (the publish)
  if (g) hipLaunchKernelGGL(splice_kernel, dim3((unsigned)g), dim3(SB), 0, st, p);
  return hipGetLastError();
}

hipError_t launch_splice_copy(SpliceArgs p, bool e_only, hipStream_t st) {
  p.a_tiles = (p.a.n + ST - 1) / ST;
  hipLaunchKernelGGL(splice_erows_kernel, dim3((unsigned)((p.nk + SB - 1) / SB)), dim3(SB), 0, st, p);
  if (!e_only && p.a_tiles)
    hipLaunchKernelGGL(splice_kernel, dim3((unsigned)p.a_tiles), dim3(SB), 0, st, p);
  return hipGetLastError();
}

// dg_join_delta's set-up and epilogue launches: the tree update's dirty flags, key-count
// shards and input-error word zeroed; the union context copied into the state's (unless
// the guard word reports a failed tree update)
__global__ __launch_bounds__(SB) void splice_finish_kernel(const u32* un, const u64* uc, u64 nc,
                                                           u32* on, u64* oc, u32* dirty, u64 n_dirty,
                                                           u64* counts, u32* err_word,
                                                           const u32* guard) {
  const u64 i = (u64)blockIdx.x * SB + threadIdx.x;
  if (i < nc && !(guard && (*guard & MERKLE_INPUT_ERR))) {
    on[i] = un[i];
    oc[i] = uc[i];
  }
  if (i < n_dirty) dirty[i] = 0;
  if (i < 8 && counts) counts[i] = 0;
  if (i == 0 && err_word) *err_word = 0;
}

hipError_t launch_splice_finish(const u32* un, const u64* uc, u64 nc, u32* on, u64* oc, u32* dirty,
                                u64 n_dirty, u64* counts, u32* err_word, hipStream_t st,
                                const u32* guard) {
  u64 n = nc > n_dirty ? nc : n_dirty;
  n = n > 8 ? n : 8;
  hipLaunchKernelGGL(splice_finish_kernel, dim3((unsigned)((n + SB - 1) / SB)), dim3(SB), 0, st, un,
                     uc, nc, on, oc, dirty, n_dirty, counts, err_word, guard);
  return hipGetLastError();
}

}  // namespace dg
