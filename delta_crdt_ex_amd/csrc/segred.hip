// segred.hip — segmented reductions over the key runs of a sorted dot store.
//
//  * read_lww: AWLWWMap.read/1,2 (reference aw_lww_map.ex:211-224).  Per key the
//    value of the entry with the greatest ts; rows inside a key are sorted by
//    ({val, ts}, dot), i.e. the flatmap order the BEAM iterates, so "first maximum
//    in iteration order" (Enum.max_by) == the first row whose ts is strictly
//    greater than every earlier one.
//  * store_check: the sorted+unique precondition.
//
// Shape: one tile = 1024 rows = 256 threads x 4 consecutive rows; each key run is
// reduced by a segmented scan across lanes and waves (seg_write_kernel), so a key with
// many entries (<= 32 in the reference's reproducible regime, any number here) costs no
// more than as many single-entry keys.  Heads are compacted in three passes -- count per
// tile (key column only), one-workgroup offset scan, write -- not by a decoupled
// look-back: thousands of tiles finishing in lock-step rounds made every tile walk back a
// whole round of predecessors.
#include "dg_launch.h"

namespace dg {

namespace {

constexpr int SB = SEG_BLOCK;
constexpr int SI = SEG_ITEMS;
constexpr int ST = SEG_TILE;

enum class SegOp { Read };

struct SegArgs {
  Rows s;
  const u64* keys;
  u64 n_keys;
  u64* out_a;  // key
  u64* out_b;  // value id
  u64* cnt;    // heads per tile
  u64* off;    // output offset per tile
  u64 ntiles;
  u64* d_count;
};


// Pass 1: key heads per tile (a head opens a key's run; with a key list only listed
// keys count -- read/2, aw_lww_map.ex:218-220).  Coalesced: thread tid looks at rows
// tid, tid + SB, ... of the tile and at the row before each.
template <SegOp OP>
__global__ __launch_bounds__(SB) void seg_count_kernel(SegArgs p) {
  __shared__ u32 s_wave[SB / WAVE + 1];
  const u64 t = blockIdx.x, n = p.s.n;
  u32 c = 0;
  // every key and its predecessor loaded at clamped indices before any is used (a load
  // under `i < n` or behind `i == 0 ||` is a branch, waited for on its own: 11.4 -> 10.2 us
  // at config 5, and 47.5 -> 42.7 us for the write pass's staging, rocprofv3 A/B)
  u64 kc[SI], kp[SI];
#pragma unroll
  for (int k = 0; k < SI; k++) {
    const u64 i = t * ST + (u64)k * SB + threadIdx.x;
    const u64 ic = i < n ? i : n - 1;
    kc[k] = p.s.key[ic];
    kp[k] = p.s.key[ic > 0 ? ic - 1 : 0];
  }
  asm volatile("" ::: "memory");
#pragma unroll
  for (int k = 0; k < SI; k++) {
    const u64 i = t * ST + (u64)k * SB + threadIdx.x;
    if (i < n) {
      bool head = i == 0 || kc[k] != kp[k];
      if (OP == SegOp::Read && head && p.keys != nullptr) head = keyset_has(p.keys, p.n_keys, kc[k]);
      c += head ? 1u : 0u;
    }
  }
  u32 tot;
  block_excl_scan<SB>(c, s_wave, &tot);
  if (threadIdx.x == 0) p.cnt[t] = tot;
}

// Pass 2: exclusive offsets of the tile counts (one workgroup).
constexpr int SSB = 1024;
__global__ __launch_bounds__(SSB) void seg_scan_kernel(SegArgs p) {
  __shared__ u32 s_wave[SSB / WAVE + 1];
  __shared__ u64 s_carry;
  scan_tile_counts<SSB>(p.cnt, p.off, p.ntiles, p.d_count, s_wave, &s_carry);
}

// Pass 3: one output per head at the tile's offset: (key, read value).  The tile's key,
// val and ts are staged in LDS by coalesced loads.  The per-key LWW choice is a
// segmented reduction with the order-aware operator `lww_join` (the later row wins only
// on a strictly greater ts: Enum.max_by's first maximum): each thread reduces its SI
// consecutive rows; the part of a run that crosses thread boundaries is carried by a
// segmented suffix scan across the wave (DPP/shuffle steps) and the block's waves (LDS),
// so no lane walks a long run serially.  The run open at the tile's end continues past
// it: the last wave reduces those rows from global memory, 64 at a time.  Heads are
// compacted in LDS and written coalesced.
struct Lww {  // a partial LWW reduction: the chosen row's ts and value; ok = any row
  i64 ts;
  u64 val;
  bool ok;
};

__device__ __forceinline__ Lww lww_none() { return Lww{0, 0, false}; }

// a covers rows before b's
__device__ __forceinline__ Lww lww_join(const Lww& a, const Lww& b) {
  const bool tb = b.ok & (!a.ok | (b.ts > a.ts));
  return Lww{tb ? b.ts : a.ts, tb ? b.val : a.val, a.ok || b.ok};
}

__device__ __forceinline__ Lww lww_shfl_down(const Lww& x, int d) {
  return Lww{__shfl_down(x.ts, d, WAVE), __shfl_down(x.val, d, WAVE),
             __shfl_down((int)x.ok, d, WAVE) != 0};
}

template <SegOp OP>
__global__ __launch_bounds__(SB) void seg_write_kernel(SegArgs p) {
  constexpr int NW = SB / WAVE;
  __shared__ u64 s_key[ST + 1], s_x[ST], s_y[ST];  // key, val, ts
  __shared__ u32 s_wave[SB / WAVE + 1];
  __shared__ Lww s_agg[NW + 1];  // each wave's suffix from its lane 0; [NW]: past the tile
  __shared__ int s_closed[NW];
  const int tid = threadIdx.x, lane = tid & (WAVE - 1), wv = tid / WAVE;
  const u64 n = p.s.n, tile = blockIdx.x, t0 = tile * ST;
  const u32 nt = (u32)min<u64>(ST, n - t0);
  {  // (all of the tile's loads at clamped indices, issued before any LDS store)
    u64 kk[SI], vx[SI], ty[SI];
#pragma unroll
    for (int k = 0; k < SI; k++) {
      const u32 j = k * SB + tid;
      const u64 i = t0 + (j < nt ? j : nt - 1);
      kk[k] = p.s.key[i];
      vx[k] = p.s.val[i];
      ty[k] = (u64)p.s.ts[i];
    }
    const u64 pk = p.s.key[t0 > 0 ? t0 - 1 : 0];
    asm volatile("" ::: "memory");
#pragma unroll
    for (int k = 0; k < SI; k++) {
      const u32 j = k * SB + tid;
      if (j < nt) {
        s_key[j + 1] = kk[k];
        s_x[j] = vx[k];
        s_y[j] = ty[k];
      }
    }
    if (tid == 0) s_key[0] = t0 > 0 ? pk : ~pk;
  }
  __syncthreads();
  // the run open at the tile's end: its rows past the tile (last wave, 64 per round)
  if (wv == NW - 1) {
    const u64 lastkey = s_key[nt];
    Lww past = lww_none();
    for (u64 g0 = t0 + nt; g0 < n; g0 += WAVE) {
      const u64 g = g0 + lane;
      const bool in = g < n && p.s.key[g] == lastkey;
      Lww x = in ? Lww{p.s.ts[g], p.s.val[g], true} : lww_none();
#pragma unroll
      for (int d = 1; d < WAVE; d <<= 1) x = lww_join(x, lww_shfl_down(x, d));
      past = lww_join(past, Lww{__shfl(x.ts, 0, WAVE), __shfl(x.val, 0, WAVE), __shfl((int)x.ok, 0, WAVE) != 0});
      if (__ballot(in) != ~0ull) break;
    }
    if (lane == 0) s_agg[NW] = past;
  }
  // this thread's rows: heads (segment starts), the keys it outputs, and `lead`, its rows
  // before its first head (the tail of a run that started earlier)
  const u32 j0 = tid * SI;
  u32 hm = 0, om = 0;
  Lww lead = lww_none();
#pragma unroll
  for (int k = 0; k < SI; k++) {
    const u32 j = j0 + k;
    if (j >= nt) break;
    const u64 key = s_key[j + 1];
    if (key != s_key[j]) {
      hm |= 1u << k;
      if (p.keys == nullptr || keyset_has(p.keys, p.n_keys, key)) om |= 1u << k;
    }
    if (!hm) lead = lww_join(lead, Lww{(i64)s_y[j], s_x[j], true});
  }
  // segmented suffix scan of (lead, closed = has a head): S_i = lead_i ⊕ lead_{i+1} ⊕ ...
  // up to and including the first thread with a head
  Lww sv = lead;
  bool sc = hm != 0;
#pragma unroll
  for (int d = 1; d < WAVE; d <<= 1) {
    const Lww y = lww_shfl_down(sv, d);
    const bool yc = __shfl_down((int)sc, d, WAVE) != 0;
    if (!sc && lane + d < WAVE) {
      sv = lww_join(sv, y);
      sc = yc;
    }
  }
  if (lane == 0) {
    s_agg[wv] = sv;
    s_closed[wv] = sc;
  }
  __syncthreads();
  // carry into this thread's last run: S_{i+1}, continued across later waves and past
  // the tile while no head closes it
  Lww c = lww_shfl_down(sv, 1);
  bool cc = __shfl_down((int)sc, 1, WAVE) != 0;
  if (lane == WAVE - 1) {
    c = lww_none();
    cc = false;
  }
  for (int w2 = wv + 1; w2 < NW && !cc; w2++) {
    c = lww_join(c, s_agg[w2]);
    cc = s_closed[w2];
  }
  if (!cc) c = lww_join(c, s_agg[NW]);
  // each head's run: its rows up to the next head, the last one also the carry
  u64 oa[SI], ob[SI];
  Lww acc = c;
#pragma unroll
  for (int k = SI - 1; k >= 0; k--) {
    const u32 j = j0 + k;
    oa[k] = ob[k] = 0;
    if (j >= nt) continue;
    acc = lww_join(Lww{(i64)s_y[j], s_x[j], true}, acc);
    if (hm & (1u << k)) {
      oa[k] = s_key[j + 1];
      ob[k] = acc.val;
      acc = lww_none();
    }
  }
  const u32 heads = om;
  u32 tile_total;
  u32 pos = block_excl_scan<SB>(__popc(heads), s_wave, &tile_total);
  __syncthreads();  // the staged rows are read; their arrays take the compacted heads
#pragma unroll
  for (int k = 0; k < SI; k++)
    if (heads & (1u << k)) {
      s_x[pos] = oa[k];
      s_y[pos] = ob[k];
      pos++;
    }
  __syncthreads();
  const u64 base = p.off[tile];
  for (u32 q = tid; q < tile_total; q += SB) {
    p.out_a[base + q] = s_x[q];
    p.out_b[base + q] = s_y[q];
  }
}

template <SegOp OP>
hipError_t launch_seg(SegArgs& p, hipStream_t st) {
  hipLaunchKernelGGL(seg_count_kernel<OP>, dim3((unsigned)p.ntiles), dim3(SB), 0, st, p);
  hipLaunchKernelGGL(seg_scan_kernel, dim3(1), dim3(SSB), 0, st, p);
  hipLaunchKernelGGL(seg_write_kernel<OP>, dim3((unsigned)p.ntiles), dim3(SB), 0, st, p);
  return hipGetLastError();
}

__global__ void store_check_kernel(Rows s, u32* bad) {
  for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x + 1; i < s.n;
       i += (u64)gridDim.x * blockDim.x) {
    if (row_cmp(load_row(s, i - 1), load_row(s, i)) >= 0) atomicOr(bad, 1u);
  }
}

}  // namespace

hipError_t launch_read_lww(const Rows& s, const u64* keys, u64 n_keys, u64* out_key, u64* out_val,
                           u64* scratch, u64* d_count, hipStream_t st) {
  SegArgs p{};
  p.s = s;
  p.keys = keys;
  p.n_keys = n_keys;
  p.out_a = out_key;
  p.out_b = out_val;
  p.ntiles = seg_tiles(s.n);
  p.cnt = scratch;
  p.off = scratch + p.ntiles;
  p.d_count = d_count;
  if (p.ntiles == 0) return hipMemsetAsync(d_count, 0, sizeof(u64), st);
  return launch_seg<SegOp::Read>(p, st);
}

hipError_t launch_store_check(const Rows& s, u32* d_bad, hipStream_t st) {
  if (s.n < 2) return hipSuccess;
  u64 blocks = (s.n + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(store_check_kernel, dim3((unsigned)blocks), dim3(256), 0, st, s, d_bad);
  return hipGetLastError();
}

}  // namespace dg
