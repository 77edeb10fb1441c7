// take.hip — the value half of a sync delta: Map.take(crdt_state.value, keys)
// (reference causal_crdt.ex:112-123 and :324-335, which send
// {:diff, %{state | dots: diff.dots, value: Map.take(value, keys)}, keys}).  On SoA
// rows: every row of `s` whose key is in the ascending key list, in store order.
//
// One workgroup per tile of TK keys (ticket order): each thread finds the row range of
// its keys by interpolation search (the store is sorted by key ids, which are hashes), a block scan turns the
// range lengths into tile-local offsets, the tile's output offset comes from the
// decoupled look-back, and the workgroup copies the tile's rows with coalesced
// writes (output slot -> its key by a search over the tile-local offsets in LDS).
// Work is O(|keys| log n + rows taken): a 1 % diff of a 12.5M-row shard reads a few
// MB, not the shard.
#include "dg_launch.h"

namespace dg {

namespace {

constexpr int TB = TAKE_TILE, TI = 1, TK = TB * TI;  // one key per thread: the searches run side by side

__global__ __launch_bounds__(TB) void take_keys_kernel(Rows s, const u64* keys, u64 n_keys,
                                                      u64 ntiles, RowsOut out, u64 cap, Scan scan,
                                                      u64* d_count, u64* key_lo, u64* key_off,
                                                      const u32* pre_len) {
  __shared__ u64 s_lo[TK];
  __shared__ u32 s_off[TK + 1];
  __shared__ u32 s_wave[TB / WAVE + 1];
  __shared__ u64 s_b[2];
  constexpr u32 MAPCAP = 4 * TK;  // output rows of a tile mapped to their key in LDS
  __shared__ unsigned short s_map[MAPCAP];
  static_assert(TK <= 65536, "key index in 16 bits");
  if (threadIdx.x == 0) {
    const u32 t = atomicAdd(scan.ticket, 1u);
    if ((u64)t == ntiles - 1) atomicExch(scan.ticket, 0u);
    s_b[0] = t;
  }
  __syncthreads();
  const u64 tile = s_b[0];
  const u64 k0 = tile * TK;
  const u32 nk = (u32)min<u64>(TK, n_keys - k0);
  u64 lo[TI];
  u32 len[TI], sum = 0;
#pragma unroll
  for (int q = 0; q < TI; q++) {
    const u32 i = threadIdx.x * TI + q;
    lo[q] = 0;
    len[q] = 0;
    if (i < nk && pre_len) {  // located already (splice_locate_kernel): key_lo, pre_len
      lo[q] = key_lo[k0 + i];
      len[q] = pre_len[k0 + i];
    } else if (i < nk) {
      const u64 key = keys[k0 + i];
      const u64 a = interp_lower_bound(s.key, 0, s.n, key);  // first row with key >= `key`
      // a key's rows are few: walk them four a round trip, every load issued together at a
      // clamped index (one dependent load per row was two round trips for a one-row key)
      u64 e = a;
      while (e < s.n) {
        u64 kk[4];
#pragma unroll
        for (int j = 0; j < 4; j++) {
          const u64 v = s.key[e + j < s.n ? e + j : a];
          kk[j] = e + j < s.n ? v : ~key;
        }
        u32 c = 0;
#pragma unroll
        for (int j = 0; j < 4; j++) c += (c == (u32)j && kk[j] == key) ? 1u : 0u;
        e += c;
        if (c < 4) break;
      }
      lo[q] = a;
      len[q] = (u32)(e - a);
    }
    sum += len[q];
  }
  u32 total;
  u32 off = block_excl_scan<TB>(sum, s_wave, &total);
#pragma unroll
  for (int q = 0; q < TI; q++) {
    const u32 i = threadIdx.x * TI + q;
    if (i < TK) {
      s_lo[i] = lo[q];
      s_off[i] = off;
    }
    // (each key's output rows point at it: one LDS read per output row below instead of
    // a search of s_off, when the tile's rows fit the map)
    if (total <= MAPCAP)
      for (u32 r = 0; r < len[q]; r++) s_map[off + r] = (unsigned short)i;
    off += len[q];
  }
  if (threadIdx.x == 0) s_off[TK] = total;
  if (threadIdx.x < WAVE) {
    u64 prefix = 0;
    if (tile == 0) {
      if (threadIdx.x == 0) lb_publish(scan.state, 0, scan.epoch, LB_INC, total);
    } else {
      if (threadIdx.x == 0) lb_publish(scan.state, tile, scan.epoch, LB_AGG, total);
      prefix = lb_lookback(scan.state, tile, scan.epoch, scan.err);
      if (threadIdx.x == 0) lb_publish(scan.state, tile, scan.epoch, LB_INC, prefix + total);
    }
    if (threadIdx.x == 0) {
      s_b[1] = prefix;
      if (tile == ntiles - 1) {
        d_count[0] = prefix + total;
        if (key_off) key_off[n_keys] = prefix + total;
      }
    }
  }
  __syncthreads();
  const u64 base = s_b[1];
  if (key_lo) {  // the splice's per-key index (splice.hip): first row and output offset
    for (u32 i = threadIdx.x; i < nk; i += TB) {
      if (!pre_len) key_lo[k0 + i] = s_lo[i];
      key_off[k0 + i] = base + s_off[i];
    }
  }
  const bool mapped = total <= MAPCAP;  // (uniform)
  for (u32 o = threadIdx.x; o < total; o += TB) {
    u32 a = 0, b = TK;  // the key whose range holds o: last i with s_off[i] <= o
    if (mapped) {
      a = s_map[o];
    } else {
      while (b - a > 1) {
        const u32 m = (a + b) >> 1;
        if (s_off[m] <= o)
          a = m;
        else
          b = m;
      }
    }
    const u64 r = s_lo[a] + (o - s_off[a]), g = base + o;
    if (g < cap) {
      out.key[g] = s.key[r];
      out.val[g] = s.val[r];
      out.ts[g] = s.ts[r];
      out.node[g] = s.node[r];
      out.cnt[g] = s.cnt[r];
    }
  }
}

}  // namespace

hipError_t launch_take_keys(const Rows& s, const u64* keys, u64 n_keys, const RowsOut& out,
                            u64 cap, const Scan& scan, u64* d_count, hipStream_t st, u64* key_lo,
                            u64* key_off, const u32* pre_len) {
  const u64 ntiles = take_tiles(n_keys);
  if (ntiles == 0) return hipMemsetAsync(d_count, 0, sizeof(u64), st);
  hipLaunchKernelGGL(take_keys_kernel, dim3((unsigned)ntiles), dim3(TB), 0, st, s, keys, n_keys,
                     ntiles, out, cap, scan, d_count, key_lo, key_off, pre_len);
  return hipGetLastError();
}

}  // namespace dg
