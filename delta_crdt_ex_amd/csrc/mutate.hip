// mutate.hip — a batch of AWLWWMap.add/4 and remove/3 operations by one node as ONE
// delta.  Reference: aw_lww_map.ex:99-146 builds one delta per op;
// CausalCrdt applies each as join(state, delta, [key]) when the op arrives
// (causal_crdt.ex:337-342).
//
// For an op on key k, state S and version vector C:
//   remove/3: rows {},                      dots = the dots of k's rows in S
//   add/4:    rows {(k, v, ts, i, C[i]+1)}, dots = the dots of k's rows in S ∪ {(i, C[i]+1)}
// (add/4 = join(remove, aw_set_add); aw_set_add's context is the new dot plus the dots of
// an identical {v, ts} entry, which are dots of k too).  Applying the ops in order, a
// later op on k removes what earlier ones wrote, and every add advances C[i] by one.  So
// the batch's delta is, per touched key, the row of its LAST op if that op is an add,
// with context = the dots of the touched keys in S plus the dot of every add of the
// batch -- add number r (in batch order) gets (i, C[i] + 1 + r).  Joining it into S with
// keys = the touched keys equals applying the ops one by one (tests/test_configs.py pins
// this against the term oracle's op-by-op fold).
//
// Ops arrive sorted by key, batch order within a key, with each add's rank among the
// batch's adds.  Passes: count (per tile of ops: touched keys, delta rows, state dots),
// one-workgroup scan, write (keys, rows, the state dots), generate the adds' dots, then
// two stable radix sorts (rocPRIM: by counter, then by node) give the (node, counter)
// order of a dot list.
#include <rocprim/device/device_radix_sort.hpp>

#include "dg_launch.h"

namespace dg {

typedef uint8_t u8;

namespace {

constexpr int MB = 256, MI = 1, MT = MB * MI;  // (one op per thread: its state search is a chain)

struct MutArgs {
  Rows s;
  Ctx c;            // a version vector
  u32 node;
  const u8* kind;   // 1 add, 0 remove
  const u64* key;   // ascending; batch order within a key
  const u64* val;
  const i64* ts;
  const u64* rank;  // add's rank among the batch's adds (batch order)
  u64 m;
  u64 ntiles;
  u64* cnt;         // 3 x ntiles: touched keys, delta rows, state dots per tile
  u64* off;         // 3 x ntiles
  u64* keys_out;
  RowsOut rows_out;
  u32* dnode;       // the delta's dots, unsorted: state dots, then the adds' dots
  u64* dcnt;
  u64* d_counts;    // [0] keys, [1] rows, [2] state dots
  u32* err;         // bit 0: ops not sorted by key
  u32* arrive;      // the count kernel's arrival counter (zero, left zero)
};

__device__ __forceinline__ u64 vv_of(const Ctx& c, u32 node) {
  u64 lo = 0, hi = c.n;
  while (lo < hi) {
    const u64 mid = (lo + hi) >> 1;
    if (c.node[mid] < node)
      lo = mid + 1;
    else
      hi = mid;
  }
  return (lo < c.n && c.node[lo] == node) ? c.cnt[lo] : 0ull;
}

// The touched key opening at op p (if any): its last op and its rows in the state.
struct Group {
  bool head, add;
  u64 key, last, lo, hi;
};

__device__ __forceinline__ Group group_at(const MutArgs& p, u64 i) {
  Group g;
  g.head = false;
  g.add = false;
  g.key = g.last = g.lo = g.hi = 0;
  if (i >= p.m) return g;
  const u64 key = p.key[i];
  if (i > 0) {
    const u64 prev = p.key[i - 1];
    if (prev > key) atomicOr(p.err, 1u);
    if (prev == key) return g;
  }
  g.head = true;
  g.key = key;
  u64 e = i + 1;
  while (e < p.m && p.key[e] == key) e++;
  g.last = e - 1;
  g.add = p.kind[g.last] != 0;
  const u64 lo = interp_lower_bound(p.s.key, 0, p.s.n, key);  // the key's rows in the state
  u64 h = lo;
  while (h < p.s.n && p.s.key[h] == key) h++;
  g.lo = lo;
  g.hi = h;
  return g;
}

__global__ __launch_bounds__(MB) void mutate_count_kernel(MutArgs p) {
  __shared__ u32 s_wave[MB / WAVE + 1];
  const u64 t = blockIdx.x, i0 = t * MT + (u64)threadIdx.x * MI;
  u32 nk = 0, nr = 0, nd = 0;
#pragma unroll
  for (int q = 0; q < MI; q++) {
    const Group g = group_at(p, i0 + q);
    nk += g.head ? 1u : 0u;
    nr += g.add ? 1u : 0u;
    nd += (u32)(g.hi - g.lo);
  }
  u32 tk, tr, td;
  block_excl_scan<MB>(nk, s_wave, &tk);
  block_excl_scan<MB>(nr, s_wave, &tr);
  block_excl_scan<MB>(nd, s_wave, &td);
  // the tile's counts handed to the last tile, which scans them all (no scan launch): stored
  // write-through (agent scope: the tiles run on every XCD), then one arrival
  __shared__ u32 s_last;
  if (threadIdx.x == 0) {
    const u64 v[3] = {tk, tr, td};
    for (int j = 0; j < 3; j++)
      __hip_atomic_store((__attribute__((address_space(1))) u64*)(p.cnt + j * p.ntiles + t), v[j],
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    s_last = __hip_atomic_fetch_add(p.arrive, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
    if (s_last) __hip_atomic_store(p.arrive, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  if (!s_last) return;
  __shared__ u64 s_carry;
  for (int j = 0; j < 3; j++) {  // (the counts read agent-scope: other XCDs wrote them)
    const u64* c = p.cnt + j * p.ntiles;
    if (threadIdx.x == 0) s_carry = 0;
    __syncthreads();
    for (u64 c0 = 0; c0 < p.ntiles; c0 += MB) {
      const u64 x = c0 + threadIdx.x;
      const u32 v = x < p.ntiles ? (u32)__hip_atomic_load((__attribute__((address_space(1))) const u64*)(c + x),
                                                          __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                 : 0u;
      u32 tot;
      const u32 o = block_excl_scan<MB>(v, s_wave, &tot);
      if (x < p.ntiles) p.off[j * p.ntiles + x] = s_carry + o;
      __syncthreads();
      if (threadIdx.x == 0) s_carry += tot;
      __syncthreads();
    }
    if (threadIdx.x == 0) p.d_counts[j] = s_carry;
    __syncthreads();
  }
}

__global__ __launch_bounds__(MB) void mutate_write_kernel(MutArgs p) {
  __shared__ u32 s_wave[MB / WAVE + 1];
  __shared__ u64 s_c0;
  if (threadIdx.x == 0) s_c0 = vv_of(p.c, p.node) + 1;
  const u64 t = blockIdx.x, i0 = t * MT + (u64)threadIdx.x * MI;
  Group g[MI];
  u32 nk = 0, nr = 0, nd = 0;
#pragma unroll
  for (int q = 0; q < MI; q++) {
    g[q] = group_at(p, i0 + q);
    nk += g[q].head ? 1u : 0u;
    nr += g[q].add ? 1u : 0u;
    nd += (u32)(g[q].hi - g[q].lo);
  }
  u32 tk, tr, td;
  u32 pk = block_excl_scan<MB>(nk, s_wave, &tk);
  u32 pr = block_excl_scan<MB>(nr, s_wave, &tr);
  u32 pd = block_excl_scan<MB>(nd, s_wave, &td);
  const u64 ok = p.off[t] + pk, orr = p.off[p.ntiles + t] + pr, od = p.off[2 * p.ntiles + t] + pd;
  const u64 c0 = s_c0;  // (published by the scans' barriers)
  u32 ik = 0, ir = 0;
  u64 id = 0;
#pragma unroll
  for (int q = 0; q < MI; q++) {
    if (!g[q].head) continue;
    p.keys_out[ok + ik++] = g[q].key;
    if (g[q].add) {
      const u64 o = orr + ir++, l = g[q].last;
      p.rows_out.key[o] = g[q].key;
      p.rows_out.val[o] = p.val[l];
      p.rows_out.ts[o] = p.ts[l];
      p.rows_out.node[o] = p.node;
      p.rows_out.cnt[o] = c0 + p.rank[l];
    }
    for (u64 r = g[q].lo; r < g[q].hi; r++, id++) {
      p.dnode[od + id] = p.s.node[r];
      p.dcnt[od + id] = p.s.cnt[r];
    }
  }
}

// the adds' dots after the state dots: (node, C[node] + 1 + r), r < n_adds
__global__ __launch_bounds__(256) void mutate_gen_kernel(MutArgs p, u64 n_adds, u64 at) {
  const u64 c0 = vv_of(p.c, p.node) + 1;
  for (u64 r = (u64)blockIdx.x * 256 + threadIdx.x; r < n_adds; r += (u64)gridDim.x * 256) {
    p.dnode[at + r] = p.node;
    p.dcnt[at + r] = c0 + r;
  }
}

}  // namespace

static MutArgs make_mut(const Rows& s, const Ctx& c, u32 node, const u8* kind, const u64* key,
                        const u64* val, const i64* ts, const u64* rank, u64 m, u64* scratch,
                        u64* d_counts, u32* err, u32* arrive = nullptr) {
  MutArgs p{};
  p.s = s;
  p.c = c;
  p.node = node;
  p.kind = kind;
  p.key = key;
  p.val = val;
  p.ts = ts;
  p.rank = rank;
  p.m = m;
  p.ntiles = mutate_tiles(m);
  p.cnt = scratch;
  p.off = scratch + 3 * p.ntiles;
  p.d_counts = d_counts;
  p.err = err;
  p.arrive = arrive;
  return p;
}

hipError_t launch_mutate_count(const Rows& s, const Ctx& c, u32 node, const u8* kind,
                               const u64* key, const u64* val, const i64* ts, const u64* rank,
                               u64 m, u64* scratch, u64* d_counts, u32* err, u32* arrive,
                               hipStream_t st) {
  MutArgs p = make_mut(s, c, node, kind, key, val, ts, rank, m, scratch, d_counts, err, arrive);
  if (m == 0) return hipMemsetAsync(d_counts, 0, 3 * sizeof(u64), st);
  hipLaunchKernelGGL(mutate_count_kernel, dim3((unsigned)p.ntiles), dim3(MB), 0, st, p);
  return hipGetLastError();
}

hipError_t launch_mutate_write(const Rows& s, const Ctx& c, u32 node, const u8* kind,
                               const u64* key, const u64* val, const i64* ts, const u64* rank,
                               u64 m, u64* scratch, u64* keys_out, const RowsOut& rows_out,
                               u32* dnode, u64* dcnt, u32* err, hipStream_t st) {
  MutArgs p = make_mut(s, c, node, kind, key, val, ts, rank, m, scratch, nullptr, err);
  p.keys_out = keys_out;
  p.rows_out = rows_out;
  p.dnode = dnode;
  p.dcnt = dcnt;
  if (m == 0) return hipSuccess;
  hipLaunchKernelGGL(mutate_write_kernel, dim3((unsigned)p.ntiles), dim3(MB), 0, st, p);
  return hipGetLastError();
}

size_t mutate_sort_tmp_bytes(u64 n) {
  size_t b1 = 0, b2 = 0;
  if (rocprim::radix_sort_pairs(nullptr, b1, (u64*)nullptr, (u64*)nullptr, (u32*)nullptr,
                                (u32*)nullptr, (size_t)n, 0, 64) != hipSuccess ||
      rocprim::radix_sort_pairs(nullptr, b2, (u32*)nullptr, (u32*)nullptr, (u64*)nullptr,
                                (u64*)nullptr, (size_t)n, 0, 32) != hipSuccess)
    return 0;
  return std::max(b1, b2);
}

hipError_t launch_mutate_dots(const Ctx& c, u32 node, u64 n_adds, u64 n_state_dots, u32* dnode,
                              u64* dcnt, u32* tnode, u64* tcnt, void* sort_tmp,
                              size_t sort_tmp_bytes, u32* out_node, u64* out_cnt, hipStream_t st) {
  MutArgs p{};
  p.c = c;
  p.node = node;
  p.dnode = dnode;
  p.dcnt = dcnt;
  const u64 n = n_state_dots + n_adds;
  if (n_state_dots == 0) {  // the adds' dots alone are (node, C + 1 + r) ascending: no sort
    if (n_adds) {
      p.dnode = out_node;
      p.dcnt = out_cnt;
      const u64 g = std::min<u64>((n_adds + 255) / 256, 1024);
      hipLaunchKernelGGL(mutate_gen_kernel, dim3((unsigned)g), dim3(256), 0, st, p, n_adds, (u64)0);
    }
    return hipGetLastError();
  }
  if (n_adds) {
    const u64 g = std::min<u64>((n_adds + 255) / 256, 1024);
    hipLaunchKernelGGL(mutate_gen_kernel, dim3((unsigned)g), dim3(256), 0, st, p, n_adds,
                       n_state_dots);
  }
  if (n == 0) return hipGetLastError();
  // LSD order: by counter, then (stable) by node
  size_t tb = sort_tmp_bytes;
  hipError_t e = rocprim::radix_sort_pairs(sort_tmp, tb, dcnt, tcnt, dnode, tnode, (size_t)n, 0,
                                           64, st);
  if (e != hipSuccess) return e;
  tb = sort_tmp_bytes;
  return rocprim::radix_sort_pairs(sort_tmp, tb, tnode, out_node, tcnt, out_cnt, (size_t)n, 0, 32,
                                   st);
}

}  // namespace dg
