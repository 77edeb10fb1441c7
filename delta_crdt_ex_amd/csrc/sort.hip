// sort.hip — dg_sort_store / dg_sort_context: ordering marshalled rows on the device.
//
// A NIF that walks %AWLWWMap{value: %{key => %{{v, ts} => MapSet}}} (reference
// lib/delta_crdt/aw_lww_map.ex:2-3) emits dots in map iteration order, not in the
// (key, val, ts, node, cnt) order every other entry point needs (include/deltagpu.h).
// This is a hand-written stable LSD radix sort over the whole 36-B tuple:
//
//  * fields least significant first: cnt, node, ts (sign bit flipped: signed order),
//    val, key;  each field's values are gathered once in the current order, then
//    sorted 8 bits at a time together with the u32 row index;
//  * a digit pass whose byte is the same in every row is skipped (one global byte
//    histogram per field decides): counters, dense node ids and nanosecond timestamps
//    of one epoch leave most of their high bytes constant;
//  * each pass: per-tile digit counts (LDS), a per-digit scan across tiles, a global
//    digit base, and a stable scatter.  Stability inside a tile: the tile is walked in
//    rounds of 256 consecutive rows; a row's rank among the round's rows with its digit
//    comes from 8 wave ballots (the rows of equal digit in the wave below it) plus the
//    equal-digit counts of the lower waves (LDS), on top of the running count of the
//    tile's earlier rounds;
//  * finally the five columns are gathered in the sorted order and exact duplicate rows
//    dropped (a store is a set), by a count / scan / write compaction.
// All of it is byte moving, HBM-bound: 12 B read + 12 B written per row per digit pass.
#include "dg_launch.h"

namespace dg {

namespace {

constexpr int RB = 256;            // threads per sort workgroup
constexpr int RI = 16;             // rows per thread per tile
constexpr int RT = RB * RI;        // rows per tile
constexpr int RW = RB / WAVE;

__device__ __forceinline__ u64 field_value(const SortField& f, u64 i) {
  if (f.width == 4) return ((const u32*)f.p)[i];
  const u64 x = ((const u64*)f.p)[i];
  return f.is_signed ? (x ^ (1ull << 63)) : x;
}

// v[i] = field value of row idx[i] (idx == nullptr: row i)
__global__ __launch_bounds__(RB) void gather_field_kernel(SortField f, const u32* idx, u64 n, u64* v) {
  for (u64 i = (u64)blockIdx.x * RB + threadIdx.x; i < n; i += (u64)gridDim.x * RB)
    v[i] = field_value(f, idx ? idx[i] : i);
}

// counts of every byte value of every byte position of v: hist8[byte][256]
__global__ __launch_bounds__(RB) void byte_hist_kernel(const u64* v, u64 n, u32* hist8) {
  __shared__ u32 s[8][256];
  for (int x = threadIdx.x; x < 8 * 256; x += RB) (&s[0][0])[x] = 0;
  __syncthreads();
  for (u64 i = (u64)blockIdx.x * RB + threadIdx.x; i < n; i += (u64)gridDim.x * RB) {
    const u64 x = v[i];
#pragma unroll
    for (int b = 0; b < 8; b++) atomicAdd(&s[b][(x >> (8 * b)) & 255], 1u);
  }
  __syncthreads();
  for (int x = threadIdx.x; x < 8 * 256; x += RB)
    if ((&s[0][0])[x]) atomicAdd(&hist8[x], (&s[0][0])[x]);
}

// per-tile digit counts, digit-major: hist[d * ntiles + tile]
__global__ __launch_bounds__(RB) void tile_hist_kernel(const u64* v, u64 n, u32 shift, u32* hist,
                                                       u64 ntiles) {
  __shared__ u32 s[256];
  s[threadIdx.x] = 0;
  __syncthreads();
  const u64 t0 = (u64)blockIdx.x * RT;
#pragma unroll 4
  for (int k = 0; k < RI; k++) {
    const u64 i = t0 + (u64)k * RB + threadIdx.x;
    if (i < n) atomicAdd(&s[(v[i] >> shift) & 255], 1u);
  }
  __syncthreads();
  hist[(u64)threadIdx.x * ntiles + blockIdx.x] = s[threadIdx.x];
}

// one workgroup per digit: exclusive scan of hist[d][0, ntiles) in place, total[d]
__global__ __launch_bounds__(RB) void digit_scan_kernel(u32* hist, u64 ntiles, u32* total) {
  __shared__ u32 s_wave[RB / WAVE + 1];
  u32* h = hist + (u64)blockIdx.x * ntiles;
  u32 carry = 0;
  for (u64 c0 = 0; c0 < ntiles; c0 += RB) {
    const u64 t = c0 + threadIdx.x;
    const u32 x = t < ntiles ? h[t] : 0u;
    u32 tot;
    const u32 ex = block_excl_scan<RB>(x, s_wave, &tot);
    if (t < ntiles) h[t] = carry + ex;
    carry += tot;
    __syncthreads();
  }
  if (threadIdx.x == 0) total[blockIdx.x] = carry;
}

// stable scatter of (v, idx) by digit: tile rows walked in rounds of RB consecutive rows
__global__ __launch_bounds__(RB) void scatter_kernel(const u64* v, const u32* idx, u64 n, u32 shift,
                                                     const u32* hist, const u32* total, u64 ntiles,
                                                     u64* vo, u32* io) {
  __shared__ u32 s_run[256];       // running output position per digit
  __shared__ u32 s_wcnt[RW][256];  // per-wave digit counts of the current round
  const int tid = threadIdx.x, lane = tid & (WAVE - 1), w = tid / WAVE;
  {
    // digit base = Σ totals of smaller digits (each thread sums its own prefix: 256 words)
    u32 base = 0;
    for (int d = 0; d < tid; d++) base += total[d];
    s_run[tid] = base + hist[(u64)tid * ntiles + blockIdx.x];
  }
  const u64 t0 = (u64)blockIdx.x * RT;
  const u64 lt_mask = (1ull << lane) - 1;
  for (int k = 0; k < RI; k++) {
    const u64 i = t0 + (u64)k * RB + tid;
    const bool valid = i < n;
    const u64 x = valid ? v[i] : 0;
    const u32 r = valid ? (idx ? idx[i] : (u32)i) : 0;  // idx == nullptr: the identity order
    const u32 d = (u32)((x >> shift) & 255);
    // lanes of this wave with the same digit (and valid)
    u64 same = __ballot(valid);
#pragma unroll
    for (int b = 0; b < 8; b++) {
      const u64 m = __ballot((d >> b) & 1);
      same &= ((d >> b) & 1) ? m : ~m;
    }
    const u32 below = (u32)__popcll(same & lt_mask);
    for (int q = tid; q < RW * 256; q += RB) (&s_wcnt[0][0])[q] = 0;
    __syncthreads();
    if (valid && below == 0) s_wcnt[w][d] = (u32)__popcll(same);  // the lowest lane of the group
    __syncthreads();
    if (valid) {
      u32 pos = s_run[d] + below;
      for (int ww = 0; ww < w; ww++) pos += s_wcnt[ww][d];
      vo[pos] = x;
      io[pos] = r;
    }
    __syncthreads();
    // advance the running positions by this round's counts
    {
      u32 add = 0;
#pragma unroll
      for (int ww = 0; ww < RW; ww++) add += s_wcnt[ww][tid];
      s_run[tid] += add;
    }
    __syncthreads();
  }
}

// ---- gather + dedupe
__global__ __launch_bounds__(RB) void gather_rows_kernel(Rows s, const u32* idx, RowsOut o) {
  for (u64 i = (u64)blockIdx.x * RB + threadIdx.x; i < s.n; i += (u64)gridDim.x * RB) {
    const u32 r = idx[i];
    o.key[i] = s.key[r];
    o.val[i] = s.val[r];
    o.ts[i] = s.ts[r];
    o.node[i] = s.node[r];
    o.cnt[i] = s.cnt[r];
  }
}

__device__ __forceinline__ bool keep_row(const Rows& s, u64 i) {
  return i == 0 || !row_eq(load_row(s, i - 1), load_row(s, i));
}

template <bool WRITE>
__global__ __launch_bounds__(RB) void unique_kernel(Rows s, u64* cnt, const u64* off, RowsOut o) {
  __shared__ u32 s_wave[RB / WAVE + 1];
  const u64 t0 = (u64)blockIdx.x * RT;
  u32 c = 0;
  u64 first = t0 + (u64)threadIdx.x * RI;
  for (int k = 0; k < RI; k++) {
    const u64 i = first + k;
    if (i < s.n && keep_row(s, i)) c++;
  }
  u32 tot;
  const u32 ex = block_excl_scan<RB>(c, s_wave, &tot);
  if (!WRITE) {
    if (threadIdx.x == 0) cnt[blockIdx.x] = tot;
    return;
  }
  u64 pos = off[blockIdx.x] + ex;
  for (int k = 0; k < RI; k++) {
    const u64 i = first + k;
    if (i < s.n && keep_row(s, i)) {
      const Row x = load_row(s, i);
      o.key[pos] = x.key;
      o.val[pos] = x.val;
      o.ts[pos] = x.ts;
      o.node[pos] = x.node;
      o.cnt[pos] = x.cnt;
      pos++;
    }
  }
}

constexpr int SSB = 1024;
__global__ __launch_bounds__(SSB) void sort_scan_kernel(const u64* cnt, u64* off, u64 ntiles,
                                                        u64* d_count) {
  __shared__ u32 s_wave[SSB / WAVE + 1];
  __shared__ u64 s_carry;
  scan_tile_counts<SSB>(cnt, off, ntiles, d_count, s_wave, &s_carry);
}

// contexts: (node, cnt) pairs
__global__ __launch_bounds__(RB) void gather_ctx_kernel(const u32* node, const u64* cnt, const u32* idx,
                                                        u64 n, u32* on, u64* oc) {
  for (u64 i = (u64)blockIdx.x * RB + threadIdx.x; i < n; i += (u64)gridDim.x * RB) {
    const u32 r = idx[i];
    on[i] = node[r];
    oc[i] = cnt[r];
  }
}

inline unsigned grid_rows(u64 n) {
  u64 g = (n + RB * 4 - 1) / (RB * 4);
  return (unsigned)(g < 1 ? 1 : (g > 8192 ? 8192 : g));
}

}  // namespace

u64 sort_tiles(u64 n) { return (n + RT - 1) / RT; }

size_t sort_tmp_bytes(u64 n) {
  const u64 nt = sort_tiles(n);
  auto al = [](size_t b) { return (b + 255) / 256 * 256; };
  // 2 x (u64 values + u32 idx) ping-pong, tile histograms, 8x256 byte counts, 256
  // totals, per-tile unique counts and offsets, sorted columns (36 B/row)
  return 2 * al(n * 8) + 2 * al(n * 4) + al(nt * 256 * 4) + al(8 * 256 * 4) + al(256 * 4) +
         2 * al(nt * 8) + al(n * 8) * 4 + al(n * 4) + 1024;
}

hipError_t sort_fields(const SortField* fields, int nf, u64 n, void* tmp, u32** idx_out,
                       u32* h_hist8, hipStream_t st) {
  auto al = [](size_t b) { return (b + 255) / 256 * 256; };
  const u64 nt = sort_tiles(n);
  char* p = (char*)tmp;
  u64* v[2] = {(u64*)p, (u64*)(p + al(n * 8))};
  p += 2 * al(n * 8);
  u32* ix[2] = {(u32*)p, (u32*)(p + al(n * 4))};
  p += 2 * al(n * 4);
  u32* hist = (u32*)p;
  p += al(nt * 256 * 4);
  u32* hist8 = (u32*)p;
  p += al(8 * 256 * 4);
  u32* total = (u32*)p;
  int cur = 0;
  bool have_idx = false;  // before the first pass the order is the identity
  hipError_t e;
  for (int f = 0; f < nf; f++) {
    // the field's values in the current order, and which of its bytes vary
    hipLaunchKernelGGL(gather_field_kernel, dim3(grid_rows(n)), dim3(RB), 0, st, fields[f],
                       have_idx ? (const u32*)ix[cur] : (const u32*)nullptr, n, v[cur]);
    if ((e = hipMemsetAsync(hist8, 0, 8 * 256 * 4, st)) != hipSuccess) return e;
    hipLaunchKernelGGL(byte_hist_kernel, dim3(grid_rows(n)), dim3(RB), 0, st, v[cur], n, hist8);
    if ((e = hipMemcpyAsync(h_hist8, hist8, 8 * 256 * 4, hipMemcpyDeviceToHost, st)) != hipSuccess) return e;
    if ((e = hipStreamSynchronize(st)) != hipSuccess) return e;
    const int bytes = fields[f].width == 4 ? 4 : 8;
    for (int b = 0; b < bytes; b++) {
      bool constant = false;
      for (int d = 0; d < 256; d++) constant |= h_hist8[b * 256 + d] == n;
      if (constant) continue;  // every row has the same digit: the pass is the identity
      const u32 shift = 8 * b;
      hipLaunchKernelGGL(tile_hist_kernel, dim3((unsigned)nt), dim3(RB), 0, st, v[cur], n, shift, hist,
                         nt);
      hipLaunchKernelGGL(digit_scan_kernel, dim3(256), dim3(RB), 0, st, hist, nt, total);
      hipLaunchKernelGGL(scatter_kernel, dim3((unsigned)nt), dim3(RB), 0, st, v[cur],
                         have_idx ? (const u32*)ix[cur] : (const u32*)nullptr, n, shift, hist, total,
                         nt, v[cur ^ 1], ix[cur ^ 1]);
      cur ^= 1;
      have_idx = true;
    }
  }
  *idx_out = have_idx ? ix[cur] : nullptr;
  return hipGetLastError();
}

hipError_t launch_sort_store(const Rows& in, const RowsOut& out, void* tmp, u32* h_hist8,
                             u64* d_count, hipStream_t st) {
  const u64 n = in.n;
  if (n == 0) return hipMemsetAsync(d_count, 0, sizeof(u64), st);
  SortField f[5] = {{in.cnt, 8, 0}, {in.node, 4, 0}, {in.ts, 8, 1}, {in.val, 8, 0}, {in.key, 8, 0}};
  u32* idx = nullptr;
  hipError_t e = sort_fields(f, 5, n, tmp, &idx, h_hist8, st);
  if (e != hipSuccess) return e;
  auto al = [](size_t b) { return (b + 255) / 256 * 256; };
  const u64 nt = sort_tiles(n);
  char* p = (char*)tmp + 2 * al(n * 8) + 2 * al(n * 4) + al(nt * 256 * 4) + al(8 * 256 * 4) + al(256 * 4);
  u64* cnt = (u64*)p;
  p += al(nt * 8);
  u64* off = (u64*)p;
  p += al(nt * 8);
  RowsOut sorted;
  sorted.key = (u64*)p;
  sorted.val = (u64*)(p + al(n * 8));
  sorted.ts = (i64*)(p + 2 * al(n * 8));
  sorted.cnt = (u64*)(p + 3 * al(n * 8));
  sorted.node = (u32*)(p + 4 * al(n * 8));
  Rows s = in;
  if (idx) {
    hipLaunchKernelGGL(gather_rows_kernel, dim3(grid_rows(n)), dim3(RB), 0, st, in, (const u32*)idx,
                       sorted);
    s.key = sorted.key;
    s.val = sorted.val;
    s.ts = sorted.ts;
    s.node = sorted.node;
    s.cnt = sorted.cnt;
  }
  hipLaunchKernelGGL(unique_kernel<false>, dim3((unsigned)nt), dim3(RB), 0, st, s, cnt,
                     (const u64*)nullptr, out);
  hipLaunchKernelGGL(sort_scan_kernel, dim3(1), dim3(SSB), 0, st, cnt, off, nt, d_count);
  hipLaunchKernelGGL(unique_kernel<true>, dim3((unsigned)nt), dim3(RB), 0, st, s, cnt, off, out);
  return hipGetLastError();
}

hipError_t launch_sort_context(int kind, const u32* node, const u64* cnt, u64 n, u32* out_node,
                               u64* out_cnt, void* tmp, u32* h_hist8, hipStream_t st) {
  if (n == 0) return hipSuccess;
  SortField f[2] = {{cnt, 8, 0}, {node, 4, 0}};
  u32* idx = nullptr;
  hipError_t e = kind == 0 ? sort_fields(f + 1, 1, n, tmp, &idx, h_hist8, st)
                           : sort_fields(f, 2, n, tmp, &idx, h_hist8, st);
  if (e != hipSuccess) return e;
  if (idx) {
    hipLaunchKernelGGL(gather_ctx_kernel, dim3(grid_rows(n)), dim3(RB), 0, st, node, cnt,
                       (const u32*)idx, n, out_node, out_cnt);
  } else {
    if ((e = hipMemcpyAsync(out_node, node, n * 4, hipMemcpyDeviceToDevice, st)) != hipSuccess) return e;
    if ((e = hipMemcpyAsync(out_cnt, cnt, n * 8, hipMemcpyDeviceToDevice, st)) != hipSuccess) return e;
  }
  return hipGetLastError();
}

}  // namespace dg
