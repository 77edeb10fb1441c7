// join.hip — AWLWWMap.join/3 on gfx950 (reference lib/delta_crdt/aw_lww_map.ex:153-209).
//
// Formulation.  Both stores are sorted by the full row tuple (key, val, ts, node,
// cnt).  The joined state is the merge of the two stores filtered per row:
//
//   row of a, also in b  (same key, {v,ts} entry and dot)  -> kept   (s1 ∩ s2)
//   row of a only                                          -> kept iff dot ∉ c_b  (s1 \ c2)
//   row of b only                                          -> kept iff dot ∉ c_a  (s2 \ c1)
//   row of b equal to a row of a                           -> dropped (MapSet dedup)
//
// which is join_dot_sets/4 (:196-209) applied to every {v,ts} entry of every key;
// entries and keys that end up empty simply emit no rows (:177-181).  With an
// explicit `keys` list, rows of keys outside it are carried over right-biased
// (b's rows if b has the key, else a's), as Map.merge(Map.drop(..)) does (:185-188).
//
// Kernel shape (partition pass + one single-pass join launch, HBM-bound):
//   * a tile = 1024 merged positions = 512 threads x 2; tiles are numbered by an
//     atomic ticket so the decoupled look-back only waits on resident tiles;
//   * the tiles' merge-path splits come from a partition pass (one wave per tile
//     boundary, 128-ary search seeded at the uniform-hash estimate: 2 rounds of
//     global loads instead of ~21 dependent ones);
//   * the tile's rows (+1 neighbour on each side) are staged in LDS (SoA, 36 B/row);
//   * each thread merges 4 positions serially from LDS and decides keep/drop;
//   * block scan of keep counts -> block-wide look-back (1024 predecessors per
//     round) -> compacted rows written coalesced.
#include "dg_launch.h"

namespace dg {

namespace {

constexpr int JB = JOIN_BLOCK;
constexpr int JI = JOIN_ITEMS;
constexpr int JT = JOIN_TILE;
constexpr int JS = JT + 4;  // LDS row slots: tile rows + one neighbour on each side per store
constexpr int CTX_LDS = 64;  // VVs up to 64 nodes are staged in LDS (else read from L2)

#ifdef DG_STAMPS
// Diagnostic build only (DG_STAMPS=1): per-tile phase timestamps (s_memrealtime,
// 100 MHz) written by lane 0 into a buffer no other code reads.
__device__ u64 g_join_stamps[65536 * 8];
#define JSTAMP(tile, k)                                                              \
  do {                                                                               \
    __syncthreads();                                                                 \
    __builtin_amdgcn_sched_barrier(0);                                               \
    if (threadIdx.x == 0 && (tile) < 65536) g_join_stamps[(tile) * 8 + (k)] =        \
        __builtin_amdgcn_s_memrealtime();                                            \
    __builtin_amdgcn_sched_barrier(0);                                               \
  } while (0)
#else
#define JSTAMP(tile, k) \
  do {                  \
  } while (0)
#endif

// ------------------------------------------------------------- context union
// Dots.union/2 (aw_lww_map.ex:39-52) in one 1024-thread workgroup: contexts are
// version vectors of at most a few hundred nodes in practice (one entry per
// replica) or the explicit dot sets of mutation deltas.

constexpr int CB = 1024;  // threads of the standalone context-union kernel

struct CtxUnionArgs {
  Ctx a, b;
  u32* out_node;
  u64* out_cnt;
  u64* d_count;
  u32* tmp_node;  // a.n + b.n
  u64* tmp_cnt;   // a.n + b.n
  u32* rank;      // b.n + 1 (after compression)
};

// Chunked exclusive block scan of flags produced by `flag(i)` for i < n; writes the
// running exclusive count to out[i] (and the total to out[n]).  Returns the total.
template <int NT, class F>
__device__ __forceinline__ u32 block_scan_flags(u64 n, F flag, u32* out, u32* s_wave) {
  u32 carry = 0;
  for (u64 base = 0; base < n; base += NT) {
    u64 i = base + threadIdx.x;
    u32 f = i < n ? (flag(i) ? 1u : 0u) : 0u;
    u32 tot;
    u32 ex = block_excl_scan<NT>(f, s_wave, &tot);
    if (i < n) out[i] = carry + ex;
    carry += tot;
    __syncthreads();
  }
  if (threadIdx.x == 0) out[n] = carry;
  __syncthreads();
  return carry;
}

// Compress a dot set (sorted by (node, cnt)) into a VV: the last dot of every node
// run carries the node's max counter (Dots.compress/1, aw_lww_map.ex:13-20).
template <int NT>
__device__ __forceinline__ u64 compress_into(const Ctx c, u32* onode, u64* ocnt, u32* scratch, u32* s_wave) {
  auto tail = [&](u64 i) { return i + 1 == c.n || c.node[i + 1] != c.node[i]; };
  u32 total = block_scan_flags<NT>(c.n, tail, scratch, s_wave);
  for (u64 i = threadIdx.x; i < c.n; i += NT)
    if (tail(i)) {
      onode[scratch[i]] = c.node[i];
      ocnt[scratch[i]] = c.cnt[i];
    }
  __syncthreads();
  return total;
}

// Dots.union/2 by one workgroup of NT threads; `s_wave` holds NT/64 + 1 words of LDS.
template <int NT>
__device__ __forceinline__ void ctx_union_block(const CtxUnionArgs p, u32* s_wave) {
  const int tid = threadIdx.x;
  if (p.a.kind == 1 && p.b.kind == 1) {
    // MapSet.union: sorted set union on (node, cnt)
    const Ctx &X = p.a, &Y = p.b;
    auto lbX = [&](u32 n, u64 c) {
      u64 lo = 0, hi = X.n;
      while (lo < hi) {
        u64 m = (lo + hi) >> 1;
        if (X.node[m] < n || (X.node[m] == n && X.cnt[m] < c))
          lo = m + 1;
        else
          hi = m;
      }
      return lo;
    };
    auto lbY = [&](u32 n, u64 c) {
      u64 lo = 0, hi = Y.n;
      while (lo < hi) {
        u64 m = (lo + hi) >> 1;
        if (Y.node[m] < n || (Y.node[m] == n && Y.cnt[m] < c))
          lo = m + 1;
        else
          hi = m;
      }
      return lo;
    };
    auto ynew = [&](u64 j) {
      u64 q = lbX(Y.node[j], Y.cnt[j]);
      return !(q < X.n && X.node[q] == Y.node[j] && X.cnt[q] == Y.cnt[j]);
    };
    u32 ny = block_scan_flags<NT>(Y.n, ynew, p.rank, s_wave);
    for (u64 i = tid; i < X.n; i += NT) {
      u64 q = lbY(X.node[i], X.cnt[i]);
      u64 o = i + p.rank[q];
      p.out_node[o] = X.node[i];
      p.out_cnt[o] = X.cnt[i];
    }
    for (u64 j = tid; j < Y.n; j += NT)
      if (ynew(j)) {
        u64 o = p.rank[j] + lbX(Y.node[j], Y.cnt[j]);
        p.out_node[o] = Y.node[j];
        p.out_cnt[o] = Y.cnt[j];
      }
    if (tid == 0) *p.d_count = X.n + ny;
    return;
  }
  // At least one VV: fold dot sets into VVs first (union(set, map) = union(map, set)).
  Ctx X = p.a, Y = p.b;
  if (X.kind == 1) {
    u64 n = compress_into<NT>(X, p.tmp_node, p.tmp_cnt, p.rank, s_wave);
    X.node = p.tmp_node;
    X.cnt = p.tmp_cnt;
    X.n = n;
    X.kind = 0;
  }
  if (Y.kind == 1) {
    u64 n = compress_into<NT>(Y, p.tmp_node + p.a.n, p.tmp_cnt + p.a.n, p.rank, s_wave);
    Y.node = p.tmp_node + p.a.n;
    Y.cnt = p.tmp_cnt + p.a.n;
    Y.n = n;
    Y.kind = 0;
  }
  auto lb = [](const Ctx& c, u32 n) {
    u64 lo = 0, hi = c.n;
    while (lo < hi) {
      u64 m = (lo + hi) >> 1;
      if (c.node[m] < n)
        lo = m + 1;
      else
        hi = m;
    }
    return lo;
  };
  auto ynew = [&](u64 j) {
    u64 q = lb(X, Y.node[j]);
    return !(q < X.n && X.node[q] == Y.node[j]);
  };
  u32 ny = block_scan_flags<NT>(Y.n, ynew, p.rank, s_wave);
  for (u64 i = tid; i < X.n; i += NT) {
    u64 q = lb(Y, X.node[i]);
    u64 c = X.cnt[i];
    if (q < Y.n && Y.node[q] == X.node[i] && Y.cnt[q] > c) c = Y.cnt[q];  // Map.update max
    u64 o = i + p.rank[q];
    p.out_node[o] = X.node[i];
    p.out_cnt[o] = c;
  }
  for (u64 j = tid; j < Y.n; j += NT)
    if (ynew(j)) {
      u64 o = p.rank[j] + lb(X, Y.node[j]);
      p.out_node[o] = Y.node[j];
      p.out_cnt[o] = Y.cnt[j];
    }
  if (tid == 0) *p.d_count = X.n + ny;
}

__global__ __launch_bounds__(CB) void ctx_union_kernel(CtxUnionArgs p) {
  __shared__ u32 s_wave[CB / WAVE + 1];
  ctx_union_block<CB>(p, s_wave);
}

struct JoinArgs {
  Rows a, b;
  Ctx ca, cb;
  const u64* keys;
  u64 n_keys;
  RowsOut out;
  Scan scan;
  u64* splits;  // per-tile merge-path split granules {epoch:20 | a_index:44}
  u64 ntiles;
  u64* d_count;
  CtxUnionArgs cu;  // the context union, run by the grid's extra last workgroup
};

struct Lds {
  u64 key[JS];
  u64 val[JS];
  u64 cnt[JS];
  i64 ts[JS];
  u32 node[JS];
  union {  // the contexts are dead once the merge is done; the compaction list reuses them
    struct {
      u64 ctx_cnt[2][CTX_LDS];
      u32 ctx_node[2][CTX_LDS];
    };
    unsigned short comp[JT];
  };
  u32 wave[JB / WAVE + 1];
  u64 lb[3 * (JB / WAVE) + 2];
  u64 bcast[4];
};

// Full-tuple compare of two LDS slots, key first (the only load for distinct keys).
__device__ __forceinline__ bool slot_le(const Lds& s, int x, int y) {
  u64 kx = s.key[x], ky = s.key[y];
  if (kx != ky) return kx < ky;
  u64 vx = s.val[x], vy = s.val[y];
  if (vx != vy) return vx < vy;
  i64 tx = s.ts[x], ty = s.ts[y];
  if (tx != ty) return tx < ty;
  u32 nx = s.node[x], ny = s.node[y];
  if (nx != ny) return nx < ny;
  return s.cnt[x] <= s.cnt[y];
}

__device__ __forceinline__ bool slot_eq(const Lds& s, int x, int y) {
  return s.key[x] == s.key[y] && s.val[x] == s.val[y] && s.ts[x] == s.ts[y] &&
         s.node[x] == s.node[y] && s.cnt[x] == s.cnt[y];
}

// Merge-path predicate on diagonal `diag` over global memory: A[i] <= B[diag-1-i].
__device__ __forceinline__ bool mp_pred(const Rows A, const Rows B, u64 diag, u64 i) {
  u64 j = diag - 1 - i;
  u64 ka = A.key[i], kb = B.key[j];
  if (ka != kb) return ka < kb;
  return row_le(load_row(A, i), load_row(B, j));
}

// Dots.member? against a context staged in LDS or read from global memory.
template <bool LDS>
__device__ __forceinline__ bool covers(const Lds& s, int which, const Ctx c, u32 dn, u64 dc) {
  if (LDS) return ctx_covers(s.ctx_node[which], s.ctx_cnt[which], c.n, c.kind, dn, dc);
  return ctx_covers(c.node, c.cnt, c.n, c.kind, dn, dc);
}

// Merge-path partition: one wave per tile boundary q (diagonal min(q * JT, na + nb))
// finds the boundary's split with a 128-ary search (two samples per lane per round).
// Round 0 samples a +-4160 window around the uniform-hash estimate (key ids are 64-bit
// hashes: the split lies within a few sqrt(d) of d * na / (na + nb)); for any key
// distribution the search stays exact, only slower.  Writes splits[q] = #A rows
// among the first `diag` merged rows (ties go to A).
constexpr int PB = 256;  // threads per partition block = 4 boundaries

__global__ __launch_bounds__(PB) void join2_partition_kernel(Rows A, Rows B, u64 ntiles,
                                                             u64* splits) {
  const int lane = threadIdx.x & (WAVE - 1);
  const u64 q = (u64)blockIdx.x * (PB / WAVE) + (threadIdx.x >> 6);
  if (q > ntiles) return;
  const u64 na = A.n, nb = B.n, total = na + nb;
  const u64 d = min(q * (u64)JOIN_TILE, total);
  u64 lo = d > nb ? d - nb : 0, hi = min(d, na);
  const u64 est = total ? (u64)((double)d * (double)na / (double)total) : 0;
  constexpr u64 WIN = 4160;
  constexpr int K = 2 * WAVE;  // samples per round
  for (int round = 0; round < 64 && hi > lo; round++) {
    const u64 span = hi - lo;
    u64 slo = lo, sspan = span;
    if (round == 0 && span > 2 * WIN + K) {
      u64 wlo = est > WIN ? est - WIN : 0, whi = est + WIN;
      wlo = max(wlo, lo);
      whi = min(whi, hi);
      if (whi > wlo + K) {
        slo = wlo;
        sspan = whi - wlo;
      }
    }
    // lane l evaluates samples 2l and 2l+1
    bool f0, f1;
    if (sspan <= (u64)K) {
      const u64 x0 = slo + 2 * lane, x1 = x0 + 1;
      f0 = x0 < slo + sspan && !mp_pred(A, B, d, x0);
      f1 = x1 < slo + sspan && !mp_pred(A, B, d, x1);
    } else {
      const u64 x0 = slo + (sspan * (u64)(2 * lane + 1)) / (K + 1);
      const u64 x1 = slo + (sspan * (u64)(2 * lane + 2)) / (K + 1);
      f0 = !mp_pred(A, B, d, x0);
      f1 = !mp_pred(A, B, d, x1);
    }
    const u64 m0 = __ballot(f0), m1 = __ballot(f1);
    // first false sample index k in [0, K): min over lanes of (2l if f0, 2l+1 if f1)
    int kf = K;
    if (m0 | m1) {
      const int l0 = m0 ? __ffsll((long long)m0) - 1 : 64;
      const int l1 = m1 ? __ffsll((long long)m1) - 1 : 64;
      kf = (l0 <= l1) ? 2 * l0 : 2 * l1 + 1;
    }
    if (sspan <= (u64)K) {
      const u64 ans = (u64)kf < sspan ? slo + kf : slo + sspan;
      lo = hi = ans;  // direct rounds always cover [lo, hi)
    } else if (kf == K) {
      lo = slo + (sspan * (u64)K) / (K + 1) + 1;
    } else {
      const u64 nh = slo + (sspan * (u64)(kf + 1)) / (K + 1);
      if (kf > 0) lo = slo + (sspan * (u64)kf) / (K + 1) + 1;
      hi = nh;
    }
  }
  if (lane == 0) splits[q] = lo;
}

template <bool CA_LDS, bool CB_LDS>
__device__ __forceinline__ void merge_items(const Ctx ca, const Ctx cb, const u64* keys,
                                            const u64 n_keys, const u64 nb, const Lds& s,
                                            int nat, int nbt, u64 a0, u64 b0, u32& keep,
                                            unsigned short (&src)[JI]) {
  const int tid = threadIdx.x;
  const int offB = nat + 2;
  const int tt = nat + nbt;
  const int diag = min(tid * JI, tt);
  const int dend = min(diag + JI, tt);
  int lo = diag > nbt ? diag - nbt : 0, hi = min(diag, nat);
  while (lo < hi) {
    int mid = (lo + hi) >> 1;
    if (slot_le(s, 1 + mid, offB + 1 + (diag - 1 - mid)))
      lo = mid + 1;
    else
      hi = mid;
  }
  int i = lo, j = diag - lo;
  keep = 0;
#pragma unroll
  for (int k = 0; k < JI; k++) {
    src[k] = 0;
    if (diag + k < dend) {
      const int sa = 1 + i, sb = offB + 1 + j;
      const bool bvalid = (b0 + (u64)j) < nb;  // b[j] exists (may be the b1 neighbour)
      const bool takeA = i < nat && (j >= nbt || slot_le(s, sa, sb));
      bool kp;
      if (takeA) {
        const u64 key = s.key[sa];
        const bool joined = keys == nullptr || keyset_has(keys, n_keys, key);
        if (joined) {
          const bool inB = bvalid && slot_eq(s, sa, sb);
          kp = inB || !covers<CB_LDS>(s, 1, cb, s.node[sa], s.cnt[sa]);
        } else {
          // Map.merge(Map.drop(a), Map.drop(b)): a's rows survive iff b lacks the key
          const bool bprev = (b0 + (u64)j) >= 1 && s.key[sb - 1] == key;
          const bool bnext = bvalid && s.key[sb] == key;
          kp = !(bprev || bnext);
        }
        src[k] = (unsigned short)sa;
        i++;
      } else {
        const bool joined = keys == nullptr || keyset_has(keys, n_keys, s.key[sb]);
        if (joined) {
          const bool dupA = (a0 + (u64)i) >= 1 && slot_eq(s, sa - 1, sb);  // slot sa-1 = a[i-1]
          kp = !dupA && !covers<CA_LDS>(s, 0, ca, s.node[sb], s.cnt[sb]);
        } else {
          kp = true;
        }
        src[k] = (unsigned short)sb;
        j++;
      }
      if (kp) keep |= 1u << k;
    }
  }
}

__global__ __launch_bounds__(JB, 8) void join2_rows_kernel(JoinArgs p) {
  __shared__ Lds s;
  const int tid = threadIdx.x;
  const u64 na = p.a.n, nb = p.b.n, total = na + nb;
  if (blockIdx.x == p.ntiles) {  // extra workgroup: Dots.union(c1, c2) (aw_lww_map.ex:155)
    ctx_union_block<JB>(p.cu, s.wave);
    return;
  }

  // ---- ticket (tile id in launch order) + context staging
  if (tid == 0) {
    u32 t = atomicAdd(p.scan.ticket, 1u);
    if ((u64)t == p.ntiles - 1) atomicExch(p.scan.ticket, 0u);  // every tile has its ticket
    s.bcast[0] = t;
  }
  const bool ca_lds = p.ca.n <= CTX_LDS, cb_lds = p.cb.n <= CTX_LDS;
  if (ca_lds)
    for (u64 x = tid; x < p.ca.n; x += JB) {
      s.ctx_node[0][x] = p.ca.node[x];
      s.ctx_cnt[0][x] = p.ca.cnt[x];
    }
  if (cb_lds)
    for (u64 x = tid; x < p.cb.n; x += JB) {
      s.ctx_node[1][x] = p.cb.node[x];
      s.ctx_cnt[1][x] = p.cb.cnt[x];
    }
  __syncthreads();
  const u64 tile = s.bcast[0];
  JSTAMP(tile, 0);
  const u64 d0 = tile * JT;
  const u64 d1 = min(d0 + (u64)JT, total);

  // ---- merge-path split from the partition pass
  if (tid == 0) {
    s.bcast[2] = p.splits[tile];
    s.bcast[3] = p.splits[tile + 1];
  }
  __syncthreads();
  JSTAMP(tile, 1);
  const u64 a0 = s.bcast[2], a1 = s.bcast[3];
  const u64 b0 = d0 - a0, b1 = d1 - a1;
  const int nat = (int)(a1 - a0), nbt = (int)(b1 - b0);
  const int offB = nat + 2;

  // ---- stage rows a[a0-1 .. a1] and b[b0-1 .. b1] in LDS
  for (int x = tid; x < nat + 2; x += JB) {
    i64 g = (i64)a0 - 1 + x;
    if (g >= 0 && (u64)g < na) {
      s.key[x] = p.a.key[g];
      s.val[x] = p.a.val[g];
      s.ts[x] = p.a.ts[g];
      s.node[x] = p.a.node[g];
      s.cnt[x] = p.a.cnt[g];
    }
  }
  for (int x = tid; x < nbt + 2; x += JB) {
    i64 g = (i64)b0 - 1 + x;
    if (g >= 0 && (u64)g < nb) {
      s.key[offB + x] = p.b.key[g];
      s.val[offB + x] = p.b.val[g];
      s.ts[offB + x] = p.b.ts[g];
      s.node[offB + x] = p.b.node[g];
      s.cnt[offB + x] = p.b.cnt[g];
    }
  }
  __syncthreads();
  JSTAMP(tile, 2);

  // ---- per-thread merge of JI positions
  u32 keep;
  unsigned short src[JI];
  if (ca_lds && cb_lds)
    merge_items<true, true>(p.ca, p.cb, p.keys, p.n_keys, nb, s, nat, nbt, a0, b0, keep, src);
  else if (ca_lds)
    merge_items<true, false>(p.ca, p.cb, p.keys, p.n_keys, nb, s, nat, nbt, a0, b0, keep, src);
  else if (cb_lds)
    merge_items<false, true>(p.ca, p.cb, p.keys, p.n_keys, nb, s, nat, nbt, a0, b0, keep, src);
  else
    merge_items<false, false>(p.ca, p.cb, p.keys, p.n_keys, nb, s, nat, nbt, a0, b0, keep, src);

  // ---- tile compaction
  JSTAMP(tile, 3);
  u32 tile_total;
  const u32 cnt = __popc(keep);
  u32 pos = block_excl_scan<JB>(cnt, s.wave, &tile_total);
#pragma unroll
  for (int k = 0; k < JI; k++)
    if (keep & (1u << k)) s.comp[pos++] = src[k];

  // ---- decoupled look-back for the tile's output offset
  JSTAMP(tile, 4);
  u64 prefix = 0;
  if (tile == 0) {
    if (tid == 0) lb_publish(p.scan.state, 0, p.scan.epoch, LB_INC, tile_total);
  } else {
    if (tid == 0) lb_publish(p.scan.state, tile, p.scan.epoch, LB_AGG, tile_total);
    prefix = lb_lookback_block<JB, 2>(p.scan.state, tile, p.scan.epoch, p.scan.err, s.lb);
    if (tid == 0) lb_publish(p.scan.state, tile, p.scan.epoch, LB_INC, prefix + tile_total);
  }
  if (tid == 0) {
    s.bcast[1] = prefix;
    if (tile == p.ntiles - 1) p.d_count[0] = prefix + tile_total;
  }
  __syncthreads();
  const u64 base = s.bcast[1];
  JSTAMP(tile, 5);

  // ---- coalesced write of the kept rows
  for (u32 q = tid; q < tile_total; q += JB) {
    const int slot = s.comp[q];
    const u64 o = base + q;
    p.out.key[o] = s.key[slot];
    p.out.val[o] = s.val[slot];
    p.out.ts[o] = s.ts[slot];
    p.out.node[o] = s.node[slot];
    p.out.cnt[o] = s.cnt[slot];
  }
#ifdef DG_STAMPS
  __syncthreads();
  JSTAMP(tile, 6);
#endif
}

}  // namespace

static CtxUnionArgs make_cu(const Ctx& a, const Ctx& b, u32* out_node, u64* out_cnt,
                            u64* d_count, void* tmp) {
  CtxUnionArgs p;
  p.a = a;
  p.b = b;
  p.out_node = out_node;
  p.out_cnt = out_cnt;
  p.d_count = d_count;
  char* t = (char*)tmp;
  p.tmp_cnt = (u64*)t;
  t += (a.n + b.n) * 8;
  p.tmp_node = (u32*)t;
  t += (a.n + b.n) * 4;
  p.rank = (u32*)t;
  return p;
}

hipError_t launch_join2(const Rows& a, const Ctx& ca, const Rows& b, const Ctx& cb,
                        const u64* keys, u64 n_keys, const RowsOut& out, u32* out_ctx_node,
                        u64* out_ctx_cnt, void* ctx_tmp, const Scan& scan, u64* d_counts,
                        hipStream_t st) {
  JoinArgs p;
  p.a = a;
  p.b = b;
  p.ca = ca;
  p.cb = cb;
  p.keys = keys;
  p.n_keys = n_keys;
  p.out = out;
  p.scan = scan;
  p.ntiles = join2_tiles(a.n, b.n);
  p.splits = scan.state + p.ntiles;  // the engine reserves 2 granules per tile + 2
  p.d_count = d_counts;
  p.cu = make_cu(ca, cb, out_ctx_node, out_ctx_cnt, d_counts + 1, ctx_tmp);
  if (p.ntiles == 0) {
    hipError_t e = hipMemsetAsync(d_counts, 0, sizeof(u64), st);
    if (e != hipSuccess) return e;
  }
  if (p.ntiles > 0) {
    const u64 nb_part = (p.ntiles + 1 + (PB / WAVE) - 1) / (PB / WAVE);
    hipLaunchKernelGGL(join2_partition_kernel, dim3((unsigned)nb_part), dim3(PB), 0, st, a, b,
                       p.ntiles, p.splits);
  }
  // one workgroup per tile + one for the context union
  hipLaunchKernelGGL(join2_rows_kernel, dim3((unsigned)p.ntiles + 1), dim3(JB), 0, st, p);
  return hipGetLastError();
}

hipError_t launch_ctx_union(const Ctx& a, const Ctx& b, u32* out_node, u64* out_cnt,
                            u64* d_count, void* tmp, hipStream_t st) {
  CtxUnionArgs p = make_cu(a, b, out_node, out_cnt, d_count, tmp);
  hipLaunchKernelGGL(ctx_union_kernel, dim3(1), dim3(CB), 0, st, p);
  return hipGetLastError();
}

#ifdef DG_STAMPS
extern "C" int dg_debug_join_stamps(unsigned long long* host, size_t n) {
  if (n > 65536 * 8) n = 65536 * 8;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_join_stamps), n * 8) == hipSuccess ? 0 : -3;
}
#endif

}  // namespace dg
