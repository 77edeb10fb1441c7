// segred.hip — segmented reductions over the key runs of a sorted dot store.
//
//  * read_lww: AWLWWMap.read/1,2 (reference aw_lww_map.ex:211-224).  Per key the
//    value of the entry with the greatest ts; rows inside a key are sorted by
//    ({val, ts}, dot), i.e. the flatmap order the BEAM iterates, so "first maximum
//    in iteration order" (Enum.max_by) == the first row whose ts is strictly
//    greater than every earlier one.
//  * merkle_leaves: per key Σ row_hash (the MerkleMap leaf of the key's raw value
//    map, causal_crdt.ex:392) plus the bucket -> first-leaf offsets the diff uses.
//  * store_check: the sorted+unique precondition.
//
// Shape: one tile = 1024 rows = 256 threads x 4 consecutive rows; a thread owning a
// key head walks the key's run forward (runs are short: one row per dot, <= 32
// entries per key in the reference's reproducible regime); heads are compacted
// with the same single-pass decoupled look-back as the join.
#include "dg_hash.h"
#include "dg_launch.h"

namespace dg {

namespace {

constexpr int SB = SEG_BLOCK;
constexpr int SI = SEG_ITEMS;
constexpr int ST = SEG_TILE;

enum class SegOp { Read, Leaves };

struct SegArgs {
  Rows s;
  const u64* keys;
  u64 n_keys;
  u64* out_a;  // key
  u64* out_b;  // value id / leaf hash
  u64* bucket_off;
  u32 depth;
  Scan scan;
  u64 ntiles;
  u64* d_count;
};

template <SegOp OP>
__global__ __launch_bounds__(SB) void segred_kernel(SegArgs p) {
  __shared__ u64 s_a[ST], s_b[ST], s_row[ST];
  __shared__ u32 s_wave[SB / WAVE + 1];
  __shared__ u64 s_bcast[2];
  const int tid = threadIdx.x;
  const u64 n = p.s.n;
  if (tid == 0) {
    u32 t = atomicAdd(p.scan.ticket, 1u);
    if ((u64)t == p.ntiles - 1) atomicExch(p.scan.ticket, 0u);
    s_bcast[0] = t;
  }
  __syncthreads();
  const u64 tile = s_bcast[0];
  const u64 r0 = tile * ST + (u64)tid * SI;

  u64 oa[SI], ob[SI];
  u32 heads = 0;
  u64 prev_key = (r0 > 0 && r0 - 1 < n) ? p.s.key[r0 - 1] : 0;
#pragma unroll
  for (int k = 0; k < SI; k++) {
    oa[k] = 0;
    ob[k] = 0;
    const u64 i = r0 + k;
    if (i < n) {
      const u64 key = p.s.key[i];
      bool head = (i == 0) || key != prev_key;
      prev_key = key;
      if (head && p.keys != nullptr) head = keyset_has(p.keys, p.n_keys, key);
      if (head) {
        oa[k] = key;
        if (OP == SegOp::Read) {
          i64 best_ts = p.s.ts[i];
          u64 best_val = p.s.val[i];
          for (u64 e = i + 1; e < n && p.s.key[e] == key; e++) {
            i64 t = p.s.ts[e];
            if (t > best_ts) {
              best_ts = t;
              best_val = p.s.val[e];
            }
          }
          ob[k] = best_val;
        } else {
          u64 h = 0;
          for (u64 e = i; e < n && p.s.key[e] == key; e++)
            h += row_hash(key, p.s.val[e], p.s.ts[e], p.s.node[e], p.s.cnt[e]);
          ob[k] = h;
        }
        heads |= 1u << k;
      }
    }
  }
  u32 tile_total;
  u32 pos = block_excl_scan<SB>(__popc(heads), s_wave, &tile_total);
#pragma unroll
  for (int k = 0; k < SI; k++)
    if (heads & (1u << k)) {
      s_a[pos] = oa[k];
      s_b[pos] = ob[k];
      s_row[pos] = r0 + k;
      pos++;
    }

  if (tid < WAVE) {
    u64 prefix = 0;
    if (tile == 0) {
      if (tid == 0) lb_publish(p.scan.state, 0, p.scan.epoch, LB_INC, tile_total);
    } else {
      if (tid == 0) lb_publish(p.scan.state, tile, p.scan.epoch, LB_AGG, tile_total);
      prefix = lb_lookback(p.scan.state, tile, p.scan.epoch, p.scan.err);
      if (tid == 0) lb_publish(p.scan.state, tile, p.scan.epoch, LB_INC, prefix + tile_total);
    }
    if (tid == 0) {
      s_bcast[1] = prefix;
      if (tile == p.ntiles - 1) p.d_count[0] = prefix + tile_total;
    }
  }
  __syncthreads();
  const u64 base = s_bcast[1];
  for (u32 q = tid; q < tile_total; q += SB) {
    const u64 o = base + q;
    p.out_a[o] = s_a[q];
    p.out_b[o] = s_b[q];
    if (OP == SegOp::Leaves) {
      // bucket_off[b] = index of the first leaf whose bucket >= b, for every bucket
      // strictly after the previous key's bucket and up to this key's bucket.
      const u32 sh = 64 - p.depth;
      const u64 row = s_row[q];
      const u64 bk = s_a[q] >> sh;
      const u64 bstart = row == 0 ? 0 : (p.s.key[row - 1] >> sh) + 1;
      for (u64 b = bstart; b <= bk; b++) p.bucket_off[b] = o;
      // after the store's last key: the trailing buckets (and the end sentinel)
      u64 e = row + 1;
      while (e < n && p.s.key[e] == s_a[q]) e++;
      if (e == n) {
        const u64 nbk = 1ull << p.depth;
        for (u64 b = bk + 1; b <= nbk; b++) p.bucket_off[b] = o + 1;
      }
    }
  }
}

__global__ void store_check_kernel(Rows s, u32* bad) {
  for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x + 1; i < s.n;
       i += (u64)gridDim.x * blockDim.x) {
    if (row_cmp(load_row(s, i - 1), load_row(s, i)) >= 0) atomicOr(bad, 1u);
  }
}

__global__ void fill_u64_kernel(u64* p, u64 n, u64 v) {
  for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (u64)gridDim.x * blockDim.x)
    p[i] = v;
}

}  // namespace

hipError_t launch_read_lww(const Rows& s, const u64* keys, u64 n_keys, u64* out_key, u64* out_val,
                           const Scan& scan, u64* d_count, hipStream_t st) {
  SegArgs p{};
  p.s = s;
  p.keys = keys;
  p.n_keys = n_keys;
  p.out_a = out_key;
  p.out_b = out_val;
  p.scan = scan;
  p.ntiles = seg_tiles(s.n);
  p.d_count = d_count;
  if (p.ntiles == 0) return hipMemsetAsync(d_count, 0, sizeof(u64), st);
  hipLaunchKernelGGL(segred_kernel<SegOp::Read>, dim3((unsigned)p.ntiles), dim3(SB), 0, st, p);
  return hipGetLastError();
}

hipError_t launch_merkle_leaves(const Rows& s, u32 depth, u64* leaf_key, u64* leaf_hash,
                                u64* bucket_off, const Scan& scan, u64* d_count, hipStream_t st) {
  SegArgs p{};
  p.s = s;
  p.out_a = leaf_key;
  p.out_b = leaf_hash;
  p.bucket_off = bucket_off;
  p.depth = depth;
  p.scan = scan;
  p.ntiles = seg_tiles(s.n);
  p.d_count = d_count;
  if (p.ntiles == 0) {
    hipLaunchKernelGGL(fill_u64_kernel, dim3(256), dim3(256), 0, st, bucket_off,
                       (1ull << depth) + 1, 0ull);
    return hipMemsetAsync(d_count, 0, sizeof(u64), st);
  }
  hipLaunchKernelGGL(segred_kernel<SegOp::Leaves>, dim3((unsigned)p.ntiles), dim3(SB), 0, st, p);
  return hipGetLastError();
}

hipError_t launch_store_check(const Rows& s, u32* d_bad, hipStream_t st) {
  if (s.n < 2) return hipSuccess;
  u64 blocks = (s.n + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(store_check_kernel, dim3((unsigned)blocks), dim3(256), 0, st, s, d_bad);
  return hipGetLastError();
}

}  // namespace dg
