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
// Kernel shape (one launch, single pass, HBM-bound):
//   * a tile = 1024 merged positions = 256 threads x 4; tiles are numbered by an
//     atomic ticket so the decoupled look-back only waits on resident tiles;
//   * the tile's merge-path split (a0, b0)/(a1, b1) is found by a 128-ary
//     cooperative search (two halves of the block search the two diagonals at once,
//     ~3 rounds of global loads for 1M-row inputs instead of ~20 dependent ones);
//   * the tile's rows (+1 neighbour on each side) are staged in LDS (SoA, 36 B/row);
//   * each thread merges 4 positions serially from LDS and decides keep/drop;
//   * block scan of keep counts -> look-back -> compacted rows written coalesced.
#include "dg_launch.h"

namespace dg {

namespace {

constexpr int JB = JOIN_BLOCK;
constexpr int JI = JOIN_ITEMS;
constexpr int JT = JOIN_TILE;
constexpr int JS = JT + 4;  // LDS row slots: tile rows + one neighbour on each side per store
constexpr int CTX_LDS = 256;

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
__device__ u32 block_scan_flags(u64 n, F flag, u32* out, u32* s_wave) {
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
__device__ u64 compress_into(const Ctx& c, u32* onode, u64* ocnt, u32* scratch, u32* s_wave) {
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
__device__ void ctx_union_block(const CtxUnionArgs& p, u32* s_wave) {
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
  u64 ntiles;
  u64* d_count;
  CtxUnionArgs cu;  // the context union, run by the grid's extra last workgroup
};

// Merge-path predicate on diagonal `diag`: A[i] <= B[diag-1-i] (ties go to A).
__device__ __forceinline__ bool mp_pred(const Rows& A, const Rows& B, u64 diag, u64 i) {
  u64 j = diag - 1 - i;
  u64 ka = A.key[i], kb = B.key[j];
  if (ka != kb) return ka < kb;
  return row_le(load_row(A, i), load_row(B, j));
}

struct Lds {
  u64 key[JS];
  u64 val[JS];
  u64 cnt[JS];
  i64 ts[JS];
  u32 node[JS];
  unsigned short comp[JT];
  u32 ctx_node[2][CTX_LDS];
  u64 ctx_cnt[2][CTX_LDS];
  u64 lo[2], hi[2];
  u32 first[2][2];
  u32 wave[JB / WAVE + 1];
  u64 bcast[2];
};

__device__ __forceinline__ Row lds_row(const Lds& s, int slot) {
  Row r;
  r.key = s.key[slot];
  r.val = s.val[slot];
  r.ts = s.ts[slot];
  r.node = s.node[slot];
  r.cnt = s.cnt[slot];
  return r;
}

__global__ __launch_bounds__(JB) void join2_rows_kernel(JoinArgs p) {
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
  const u64 d0 = tile * JT;
  const u64 d1 = min(d0 + (u64)JT, total);

  // ---- cooperative merge-path search for the tile's two diagonals
  const int half = tid / 128, lt = tid & 127;
  const u64 dh = half ? d1 : d0;
  if (lt == 0) {
    s.lo[half] = dh > nb ? dh - nb : 0;
    s.hi[half] = min(dh, na);
  }
  __syncthreads();
  for (int round = 0; round < 64; round++) {
    const u64 lo = s.lo[half], hi = s.hi[half], span = hi - lo;
    bool f = false;
    u64 x = 0;
    if (span > 0) {
      bool valid;
      if (span <= 128) {
        x = lo + lt;
        valid = (u64)lt < span;
      } else {
        x = lo + (span * (u64)(lt + 1)) / 129;
        valid = true;
      }
      f = valid && !mp_pred(p.a, p.b, dh, x);
    }
    u64 m = __ballot(f);
    if ((tid & (WAVE - 1)) == 0) s.first[half][(tid >> 6) & 1] = m ? (u32)(__ffsll((long long)m) - 1) : 64u;
    __syncthreads();
    if (lt == 0 && span > 0) {
      u32 f0 = s.first[half][0], f1 = s.first[half][1];
      u32 kf = f0 < 64 ? f0 : (f1 < 64 ? 64 + f1 : 128);
      if (span <= 128) {
        u64 ans = kf < span ? lo + kf : hi;
        s.lo[half] = ans;
        s.hi[half] = ans;
      } else if (kf == 128) {
        s.lo[half] = lo + (span * 128ull) / 129 + 1;
      } else {
        s.hi[half] = lo + (span * (u64)(kf + 1)) / 129;
        if (kf > 0) s.lo[half] = lo + (span * (u64)kf) / 129 + 1;
      }
    }
    __syncthreads();
    if (s.lo[0] == s.hi[0] && s.lo[1] == s.hi[1]) break;
  }
  const u64 a0 = s.lo[0], a1 = s.lo[1];
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

  const u32* can = ca_lds ? s.ctx_node[0] : p.ca.node;
  const u64* cac = ca_lds ? s.ctx_cnt[0] : p.ca.cnt;
  const u32* cbn = cb_lds ? s.ctx_node[1] : p.cb.node;
  const u64* cbc = cb_lds ? s.ctx_cnt[1] : p.cb.cnt;

  // ---- per-thread merge of JI positions
  const int tt = nat + nbt;
  const int diag = min(tid * JI, tt);
  const int dend = min(diag + JI, tt);
  int lo = diag > nbt ? diag - nbt : 0, hi = min(diag, nat);
  while (lo < hi) {
    int mid = (lo + hi) >> 1;
    if (row_le(lds_row(s, 1 + mid), lds_row(s, offB + 1 + (diag - 1 - mid))))
      lo = mid + 1;
    else
      hi = mid;
  }
  int i = lo, j = diag - lo;
  u32 keep = 0;
  unsigned short src[JI];
#pragma unroll
  for (int k = 0; k < JI; k++) {
    src[k] = 0;
    if (diag + k < dend) {
      const bool bvalid = (b0 + (u64)j) < nb;  // b[j] exists globally (may be the b1 neighbour)
      bool takeA;
      Row ra, rb;
      if (i < nat) ra = lds_row(s, 1 + i);
      if (bvalid) rb = lds_row(s, offB + 1 + j);
      if (i >= nat)
        takeA = false;
      else if (j >= nbt)
        takeA = true;
      else
        takeA = row_le(ra, rb);
      bool kp;
      if (takeA) {
        bool joined = p.keys == nullptr || keyset_has(p.keys, p.n_keys, ra.key);
        if (joined) {
          bool inB = bvalid && row_eq(ra, rb);
          kp = inB || !ctx_covers(cbn, cbc, p.cb.n, p.cb.kind, ra.node, ra.cnt);
        } else {
          // Map.merge(Map.drop(a), Map.drop(b)): a's rows survive iff b lacks the key
          bool bprev = (b0 + (u64)j) >= 1 && s.key[offB + j] == ra.key;
          bool bnext = bvalid && rb.key == ra.key;
          kp = !(bprev || bnext);
        }
        src[k] = (unsigned short)(1 + i);
        i++;
      } else {
        bool joined = p.keys == nullptr || keyset_has(p.keys, p.n_keys, rb.key);
        if (joined) {
          bool dupA = (a0 + (u64)i) >= 1 && row_eq(lds_row(s, i), rb);  // slot i = a[i-1]
          kp = !dupA && !ctx_covers(can, cac, p.ca.n, p.ca.kind, rb.node, rb.cnt);
        } else {
          kp = true;
        }
        src[k] = (unsigned short)(offB + 1 + j);
        j++;
      }
      if (kp) keep |= 1u << k;
    }
  }

  // ---- tile compaction
  u32 tile_total;
  const u32 cnt = __popc(keep);
  u32 pos = block_excl_scan<JB>(cnt, s.wave, &tile_total);
#pragma unroll
  for (int k = 0; k < JI; k++)
    if (keep & (1u << k)) s.comp[pos++] = src[k];

  // ---- decoupled look-back for the tile's output offset
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
      s.bcast[1] = prefix;
      if (tile == p.ntiles - 1) p.d_count[0] = prefix + tile_total;
    }
  }
  __syncthreads();
  const u64 base = s.bcast[1];

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
  p.d_count = d_counts;
  p.cu = make_cu(ca, cb, out_ctx_node, out_ctx_cnt, d_counts + 1, ctx_tmp);
  if (p.ntiles == 0) {
    hipError_t e = hipMemsetAsync(d_counts, 0, sizeof(u64), st);
    if (e != hipSuccess) return e;
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

}  // namespace dg
