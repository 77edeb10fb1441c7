// merkle.hip — level-wise Merkle bucket hashing and the parallel tree diff (the
// MerkleMap role in DeltaCrdt.CausalCrdt sync: update_hashes causal_crdt.ex:94,254;
// prepare_partial_diff/continue_partial_diff :96,255).
//
// Tree: 2^depth buckets over the key-id space (bucket = key >> (64 - depth); key
// ids are 64-bit hashes, so buckets are contiguous key ranges of the sorted leaf
// array).  bucket_off[b] (from segred.hip) locates each bucket's leaves.
//
//  * merkle_buckets: bucket hash = Σ leaf hashes of the bucket (thread per bucket).
//  * merkle_upsweep: 1024 nodes of one level per workgroup reduced in LDS up to 10
//    levels per launch (parent = node_hash(left, right)); depth <= 26 needs <= 3.
//  * merkle_diff: a workgroup owns the subtree of 256 buckets below one node of
//    level depth-8; if that node matches in both trees the whole subtree is skipped
//    (no bucket or leaf is read), otherwise each thread compares one bucket and,
//    if it differs, merges the two buckets' leaf runs and emits the keys that are
//    on one side only or whose leaf hash differs.  Output is ascending and
//    compacted with the decoupled look-back (tiles in key order).
#include "dg_hash.h"
#include "dg_launch.h"

namespace dg {

namespace {

__global__ void merkle_buckets_kernel(u32 depth, const u64* leaf_hash, const u64* off, u64* nodes) {
  const u64 nb = 1ull << depth;
  u64* lvl = nodes + (nb - 1);
  for (u64 b = (u64)blockIdx.x * blockDim.x + threadIdx.x; b < nb; b += (u64)gridDim.x * blockDim.x) {
    u64 h = 0;
    for (u64 x = off[b]; x < off[b + 1]; x++) h += leaf_hash[x];
    lvl[b] = h;
  }
}

constexpr int UPB = 512;   // threads per upsweep block
constexpr int UPL = 10;    // levels per launch (1024 nodes in LDS)

// Reduce level `hi` (2^hi nodes) by `nlev` levels.  Block g handles nodes
// [g * 2^nlev, (g+1) * 2^nlev) of level hi.
__global__ __launch_bounds__(UPB) void merkle_upsweep_kernel(u64* nodes, u32 hi, u32 nlev) {
  __shared__ u64 s[1 << UPL];
  const u64 width = 1ull << nlev;
  const u64 g = blockIdx.x;
  const u64* src = nodes + ((1ull << hi) - 1) + g * width;
  for (u64 x = threadIdx.x; x < width; x += UPB) s[x] = src[x];
  __syncthreads();
  for (u32 l = 1; l <= nlev; l++) {
    const u64 cnt = width >> l;
    u64* dst = nodes + ((1ull << (hi - l)) - 1) + g * cnt;
    u64 v[2];
    int nv = 0;
    for (u64 x = threadIdx.x; x < cnt; x += UPB) v[nv++] = node_hash(s[2 * x], s[2 * x + 1]);
    __syncthreads();
    nv = 0;
    for (u64 x = threadIdx.x; x < cnt; x += UPB) {
      s[x] = v[nv];
      dst[x] = v[nv++];
    }
    __syncthreads();
  }
}

constexpr int DB = DIFF_BLOCK;

struct DiffArgs {
  u32 depth;
  const u64 *na, *ka, *ha, *oa;
  const u64 *nb, *kb, *hb, *ob;
  u64* out;
  u64 cap;
  u64* cnt;  // differing keys per tile
  u64* off;  // their output offset
  u32* bc;   // differing keys per bucket (the count pass's walk, reused by the write pass)
  u64 ntiles;
  u64* d_count;
};

// Walk the leaf runs of one bucket in both trees; emit differing keys (or count).
template <bool WRITE>
__device__ __forceinline__ u32 diff_bucket(const DiffArgs& p, u64 b, u64* out, u64 o, u64 cap) {
  u64 i = p.oa[b], ie = p.oa[b + 1], j = p.ob[b], je = p.ob[b + 1];
  u32 c = 0;
  while (i < ie || j < je) {
    u64 k;
    bool d;
    if (j >= je || (i < ie && p.ka[i] < p.kb[j])) {
      k = p.ka[i++];
      d = true;
    } else if (i >= ie || p.kb[j] < p.ka[i]) {
      k = p.kb[j++];
      d = true;
    } else {
      k = p.ka[i];
      d = p.ha[i] != p.hb[j];
      i++;
      j++;
    }
    if (d) {
      if (WRITE && o + c < cap) out[o + c] = k;
      c++;
    }
  }
  return c;
}

// The differing keys in three passes (every tile of a launch is resident at once, so
// a look-back would poll whole rounds of predecessors): per tile of 256 buckets the
// count, one workgroup's offset scan, then the write.  A bucket is walked only where
// its subtree root and its own node differ; the write pass re-reads the count pass's
// per-bucket counts instead of walking every differing bucket a second time.
__device__ __forceinline__ u64 diff_bpt(const DiffArgs& p) {  // buckets per tile
  return p.depth >= 8 ? 256ull : (1ull << p.depth);
}

__device__ __forceinline__ u64 diff_bucket_of(const DiffArgs& p, u64 tile, int tid, bool* walk) {
  const u32 rl = p.depth >= 8 ? p.depth - 8 : 0;  // subtree root level
  const u64 root = ((1ull << rl) - 1) + tile;
  const u64 nbk = 1ull << p.depth;
  const u64 bpt = p.depth >= 8 ? 256ull : nbk;      // buckets per tile
  const u64 b = tile * bpt + tid;
  *walk = false;
  if ((u64)tid < bpt && p.na[root] != p.nb[root]) {
    const u64 leaf = (nbk - 1) + b;
    *walk = p.na[leaf] != p.nb[leaf];
  }
  return b;
}

__global__ __launch_bounds__(DB) void merkle_diff_count_kernel(DiffArgs p) {
  __shared__ u32 s_wave[DB / WAVE + 1];
  bool walk;
  const u64 b = diff_bucket_of(p, blockIdx.x, threadIdx.x, &walk);
  const u32 c = walk ? diff_bucket<false>(p, b, nullptr, 0, 0) : 0u;
  if ((u64)threadIdx.x < diff_bpt(p)) p.bc[b] = c;
  u32 tot;
  block_excl_scan<DB>(c, s_wave, &tot);
  if (threadIdx.x == 0) p.cnt[blockIdx.x] = tot;
}

constexpr int DSB = 1024;
__global__ __launch_bounds__(DSB) void merkle_diff_scan_kernel(DiffArgs p) {
  __shared__ u32 s_wave[DSB / WAVE + 1];
  __shared__ u64 s_carry;
  scan_tile_counts<DSB>(p.cnt, p.off, p.ntiles, p.d_count, s_wave, &s_carry);
}

__global__ __launch_bounds__(DB) void merkle_diff_write_kernel(DiffArgs p) {
  __shared__ u32 s_wave[DB / WAVE + 1];
  const u64 bpt = diff_bpt(p);
  const u64 b = blockIdx.x * bpt + threadIdx.x;
  const u32 c = (u64)threadIdx.x < bpt ? p.bc[b] : 0u;
  u32 tot;
  const u32 ex = block_excl_scan<DB>(c, s_wave, &tot);
  if (c) diff_bucket<true>(p, b, p.out, p.off[blockIdx.x] + ex, p.cap);
}

}  // namespace

hipError_t launch_merkle_levels(u32 depth, const u64* leaf_hash, const u64* bucket_off,
                                u64* nodes, hipStream_t st) {
  const u64 nb = 1ull << depth;
  u64 blocks = (nb + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(merkle_buckets_kernel, dim3((unsigned)blocks), dim3(256), 0, st, depth,
                     leaf_hash, bucket_off, nodes);
  u32 hi = depth;
  while (hi > 0) {
    u32 nlev = hi < (u32)UPL ? hi : (u32)UPL;
    u64 grid = 1ull << (hi - nlev);
    hipLaunchKernelGGL(merkle_upsweep_kernel, dim3((unsigned)grid), dim3(UPB), 0, st, nodes, hi,
                       nlev);
    hi -= nlev;
  }
  return hipGetLastError();
}

hipError_t launch_merkle_diff(u32 depth, const u64* nodes_a, const u64* leaf_key_a,
                              const u64* leaf_hash_a, const u64* off_a, const u64* nodes_b,
                              const u64* leaf_key_b, const u64* leaf_hash_b, const u64* off_b,
                              u64* out_keys, u64 cap, u64* scratch, u64* d_count,
                              hipStream_t st) {
  DiffArgs p;
  p.depth = depth;
  p.na = nodes_a;
  p.ka = leaf_key_a;
  p.ha = leaf_hash_a;
  p.oa = off_a;
  p.nb = nodes_b;
  p.kb = leaf_key_b;
  p.hb = leaf_hash_b;
  p.ob = off_b;
  p.out = out_keys;
  p.cap = cap;
  p.ntiles = diff_tiles(depth);
  p.cnt = scratch;
  p.off = scratch + p.ntiles;
  p.bc = (u32*)(scratch + 2 * p.ntiles);
  p.d_count = d_count;
  hipLaunchKernelGGL(merkle_diff_count_kernel, dim3((unsigned)p.ntiles), dim3(DB), 0, st, p);
  hipLaunchKernelGGL(merkle_diff_scan_kernel, dim3(1), dim3(DSB), 0, st, p);
  hipLaunchKernelGGL(merkle_diff_write_kernel, dim3((unsigned)p.ntiles), dim3(DB), 0, st, p);
  return hipGetLastError();
}

}  // namespace dg
