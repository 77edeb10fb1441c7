// kfold.hip — CausalCrdt's fold of keyed sync deltas into a state, in ONE pass over
// the state (reference causal_crdt.ex:324-335 builds the deltas, :383-384 applies each
// as join(state, delta_i, keys_i); aw_lww_map.ex:153-209 is the join).
//
// Per key x, the sequential fold S_i = join(S_{i-1}, D_i, K_i) changes x only at the
// deltas that "touch" it (x ∈ K_i, or D_i has rows of x), and it acts on each distinct
// row tuple r of x independently.  With P = "r is in the current state":
//
//   x ∈ K_i:        P ? (r ∈ D_i || dot(r) ∉ c_i)          (s1∩s2 ∪ s1\c2, :196-209)
//                    : (r ∈ D_i && dot(r) ∉ C_{i-1})         (s2\c1)
//   x ∉ K_i, D_i has rows of x:  P = (r ∈ D_i)               (Map.merge(Map.drop..), :185-188)
//   otherwise:      P unchanged
//
// where c_i is delta i's context and C_{i-1} = c_state ⊔ c_1 ⊔ .. ⊔ c_{i-1} the state's
// context before step i (Dots.union, :155).  The output is every candidate tuple (a row
// of the state or of any delta) whose P ends true, in tuple order; the output context
// is C_k.  So the fold needs, per candidate: the bit masks of the deltas touching its
// key (keyset bits K, row bits R), of the deltas holding the identical tuple (M), and
// two VV lookups per touching delta.
//
// Kernels (one stream, no host sync until the end):
//   kfold_prep_kernel   dense VV tables: tabC[i][node] = c_i, tabP[i][node] = C_{i-1}
//                       (node ids < KNT; larger ids in a context -> fallback flag), and
//                       the output context C_k in node order.
//   kfold_fill_kernel   key ids are 64-bit hashes, so the key space is cut into T equal
//                       buckets; for the state and for every delta row run / keyset run,
//                       start[t][run] = its first element of bucket >= t (one coalesced
//                       pass over the keys).
//   kfold_kernel        one workgroup per bucket: loads the state slice and the slices
//                       of all runs into LDS, bitonic-sorts the delta rows + keyset
//                       markers by key, evaluates every candidate as above, ranks the
//                       survivors of each key by tuple, resolves the bucket's output
//                       offset by decoupled look-back and writes the rows.
// A bucket that overflows its LDS capacity (keys far from uniform) sets a flag and the
// caller re-runs the fold step by step (api.hip); nothing falls back to the CPU.
#include "dg_launch.h"

namespace dg {

namespace {

constexpr int KB = KFOLD_BLOCK;
constexpr int CS = KFOLD_CAP_S;  // state rows per bucket
constexpr int CD = KFOLD_CAP_D;  // delta rows per bucket
constexpr int CM = KFOLD_CAP_M;  // keyset markers per bucket
constexpr int CU = CD + CM;
constexpr u32 MARK = 1u << 15;   // utag: (src << 16) | MARK? | pre-sort slot
constexpr u32 SLOT = MARK - 1;
static_assert(CS <= 4 * KB && CU <= 4 * KB, "scan_flags covers 4 items per thread");
static_assert(2 * KFOLD_MAX_K <= KB, "one thread per run");
static_assert(CU <= SLOT + 1, "slot bits");

__device__ __forceinline__ u64 bucket_of(u64 key, u64 T) { return __umul64hi(key, T); }

__device__ __forceinline__ u64 vv_at(const u64* tab, u32 i, u32 node) {
  return node < (u32)KNT ? tab[(u64)i * KNT + node] : 0ull;
}

// P after the touching deltas (bits of K | R, in delta order); see the header.
__device__ __forceinline__ bool present(bool P, u64 K, u64 R, u64 M, u32 node, u64 cnt,
                                        const u64* tabC, const u64* tabP) {
  u64 bits = K | R;
  while (bits) {
    const u32 i = (u32)__builtin_ctzll(bits);
    bits &= bits - 1;
    const bool inD = (M >> i) & 1;
    if ((K >> i) & 1)
      P = P ? (inD || vv_at(tabC, i, node) < cnt) : (inD && vv_at(tabP, i, node) < cnt);
    else
      P = inD;
  }
  return P;
}

// ------------------------------------------------------------------------ prep
__global__ __launch_bounds__(KNT) void kfold_prep_kernel(KFoldArgs p) {
  __shared__ u32 pres[KNT];
  __shared__ u32 wave[KNT / WAVE + 1];
  const u32 n = threadIdx.x;
  const int k = p.k;
  pres[n] = 0;
  __syncthreads();
  // C_0 = the state's context -> tabP row 0; c_i -> tabC row i (tables zeroed by the caller)
  for (u64 e = n; e < p.c0.n; e += KNT) {
    const u32 nd = p.c0.node[e];
    if (nd >= (u32)KNT) {
      atomicOr(p.flag, KF_PREP_FAIL);
      continue;
    }
    p.tabP[nd] = p.c0.cnt[e];
    pres[nd] = 1;
  }
  for (int i = 0; i < k; i++) {
    const Ctx c = p.runs[i].ctx;
    for (u64 e = n; e < c.n; e += KNT) {
      const u32 nd = c.node[e];
      if (nd >= (u32)KNT) {
        atomicOr(p.flag, KF_PREP_FAIL);
        continue;
      }
      p.tabC[(u64)i * KNT + nd] = c.cnt[e];
      pres[nd] = 1;
    }
  }
  __syncthreads();
  // prefix unions: C_i = C_{i-1} ⊔ c_i, per node the max (absent = 0)
  u64 acc = p.tabP[n];
  for (int i = 0; i < k; i++) {
    acc = max(acc, p.tabC[(u64)i * KNT + n]);
    if (i + 1 < k) p.tabP[(u64)(i + 1) * KNT + n] = acc;
  }
  // C_k in node order
  u32 tot;
  const u32 pos = block_excl_scan<KNT>(pres[n], wave, &tot);
  if (pres[n]) {
    p.out_ctx_node[pos] = n;
    p.out_ctx_cnt[pos] = acc;
  }
  if (n == 0) p.d_counts[1] = tot;
}

// ------------------------------------------------------------------------ fill
// start[t][r] for the 2k delta runs (rows of delta r, then keyset r-k) and sstart[t] for
// the state: index of the run's first element whose bucket is >= t, for t in [0, T].
__device__ __forceinline__ const u64* run_keys(const KFoldArgs& p, int r, u64* n) {
  if (r < p.k) {
    *n = p.runs[r].rows.n;
    return p.runs[r].rows.key;
  }
  if (r < 2 * p.k) {
    *n = p.runs[r - p.k].n_keys;
    return p.runs[r - p.k].keys;
  }
  *n = p.s.n;
  return p.s.key;
}

__global__ __launch_bounds__(256) void kfold_fill_kernel(KFoldArgs p) {
  __shared__ u64 flat[2 * KFOLD_MAX_K + 2];
  const int nr = 2 * p.k + 1;  // runs incl. the state
  for (int i = threadIdx.x; i <= nr; i += 256) flat[i] = p.flat[i];
  __syncthreads();
  const u64 total = flat[nr], T = p.T;
  const u32 stride = 2 * p.k;
  for (u64 g = (u64)blockIdx.x * 256 + threadIdx.x; g < total; g += (u64)gridDim.x * 256) {
    int lo = 0, hi = nr;  // flat[lo] <= g < flat[hi]; empty runs are skipped
    while (hi - lo > 1) {
      const int mid = (lo + hi) >> 1;
      if (flat[mid] <= g)
        lo = mid;
      else
        hi = mid;
    }
    const int r = lo;
    const u64 j = g - flat[r];
    u64 n;
    const u64* keys = run_keys(p, r, &n);
    const u64 b = bucket_of(keys[j], T);
    u64 bb = j == 0 ? 0 : bucket_of(keys[j - 1], T) + 1;
    const u64 end = (j == n - 1) ? T : b;
    for (; bb <= end; bb++) {
      const u64 v = bb <= b ? j : n;
      if (r == nr - 1)
        p.sstart[bb] = v;
      else
        p.dstart[bb * stride + r] = (u32)v;
    }
  }
}

// ------------------------------------------------------------------------ main
struct KLds {
  u64 skey[CS], sval[CS], scnt[CS];
  i64 sts[CS];
  u32 snode[CS];
  u64 dkey[CD], dval[CD], dcnt[CD];
  i64 dts[CD];
  u32 dnode[CD];
  u64 ukey[CU];
  u32 utag[CU];
  unsigned short spre[CS + 1], upre[CU + 1], slbu[CS];
  unsigned char ssurv[CS], usurv[CU];
  u32 roff[2 * KFOLD_MAX_K + 1];
  u32 rbeg[2 * KFOLD_MAX_K];
  u32 wave[KB / WAVE + 1];
  u64 bcast[2];
};

__device__ __forceinline__ Row srow(const KLds& s, u32 i) {
  Row r;
  r.key = s.skey[i];
  r.val = s.sval[i];
  r.ts = s.sts[i];
  r.node = s.snode[i];
  r.cnt = s.scnt[i];
  return r;
}

__device__ __forceinline__ Row drow(const KLds& s, u32 d) {
  Row r;
  r.key = s.dkey[d];
  r.val = s.dval[d];
  r.ts = s.dts[d];
  r.node = s.dnode[d];
  r.cnt = s.dcnt[d];
  return r;
}

// first sorted item with key >= x
__device__ __forceinline__ u32 lower_key(const u64* a, u32 n, u64 x) {
  u32 lo = 0, hi = n;
  while (lo < hi) {
    const u32 mid = (lo + hi) >> 1;
    if (a[mid] < x)
      lo = mid + 1;
    else
      hi = mid;
  }
  return lo;
}

// exclusive prefix of n <= 4*KB flags into pre[0..n]
__device__ __forceinline__ void scan_flags(const unsigned char* f, u32 n, unsigned short* pre,
                                           u32* wave) {
  const u32 b = threadIdx.x * 4;
  u32 c[4], sum = 0;
#pragma unroll
  for (int q = 0; q < 4; q++) {
    c[q] = (b + q < n) ? f[b + q] : 0u;
    sum += c[q];
  }
  u32 tot;
  u32 off = block_excl_scan<KB>(sum, wave, &tot);
#pragma unroll
  for (int q = 0; q < 4; q++) {
    if (b + q < n) pre[b + q] = (unsigned short)off;
    off += c[q];
  }
  if (threadIdx.x == 0) pre[n] = (unsigned short)tot;
}

// bitonic sort of n (a power of two) (key, tag) pairs, ascending
__device__ __forceinline__ void sort_items(u64* key, u32* tag, u32 n) {
  for (u32 size = 2; size <= n; size <<= 1)
    for (u32 stride = size >> 1; stride > 0; stride >>= 1) {
      for (u32 idx = threadIdx.x; idx < n / 2; idx += KB) {
        const u32 i = ((idx & ~(stride - 1)) << 1) | (idx & (stride - 1));
        const u32 j = i + stride;
        const u64 ki = key[i], kj = key[j];
        const u32 ti = tag[i], tj = tag[j];
        const bool gt = ki > kj || (ki == kj && ti > tj);
        if (gt == ((i & size) == 0)) {
          key[i] = kj;
          key[j] = ki;
          tag[i] = tj;
          tag[j] = ti;
        }
      }
      __syncthreads();
    }
}

__global__ __launch_bounds__(KB) void kfold_kernel(KFoldArgs p) {
  __shared__ KLds s;
  if (*p.flag & KF_PREP_FAIL) return;  // every workgroup leaves: no ticket is taken
  const int tid = threadIdx.x;
  const int k = p.k, nr = 2 * k;
  if (tid == 0) {
    const u32 t = atomicAdd(p.scan.ticket, 1u);
    if ((u64)t == p.T - 1) atomicExch(p.scan.ticket, 0u);
    s.bcast[0] = t;
  }
  __syncthreads();
  const u64 t = s.bcast[0];
  const u64 s0 = p.sstart[t];
  u32 nS = (u32)min<u64>(p.sstart[t + 1] - s0, 0xffffffffull);
  u32 len = 0;
  bool bad = p.sstart[t + 1] < s0;
  if (tid < nr) {
    const u32 a = p.dstart[t * nr + tid], b = p.dstart[(t + 1) * nr + tid];
    len = b >= a ? min(b - a, (u32)CU + 1) : 0u;  // bounded: the sum cannot wrap
    bad |= b < a;
    s.rbeg[tid] = a;
  }
  bad = __syncthreads_or(bad);
  u32 nU;
  const u32 off = block_excl_scan<KB>(len, s.wave, &nU);
  if (tid < nr) s.roff[tid] = off;
  if (tid == 0) s.roff[nr] = nU;
  __syncthreads();
  u32 nD = s.roff[k];
  if (bad || nS > (u32)CS || nD > (u32)CD || nU - nD > (u32)CM) {
    if (tid == 0) atomicOr(p.flag, KF_OVERFLOW);
    nS = nU = nD = 0;  // publish an empty bucket so the look-back chain stays live
  }

  // ---- stage: state slice, delta rows (slot = pre-sort index), keyset markers
  for (u32 i = tid; i < nS; i += KB) {
    const u64 g = s0 + i;
    s.skey[i] = p.s.key[g];
    s.sval[i] = p.s.val[g];
    s.sts[i] = p.s.ts[g];
    s.snode[i] = p.s.node[g];
    s.scnt[i] = p.s.cnt[g];
  }
  for (u32 q = tid; q < nU; q += KB) {
    int lo = 0, hi = nr;  // roff[lo] <= q < roff[hi]
    while (hi - lo > 1) {
      const int mid = (lo + hi) >> 1;
      if (s.roff[mid] <= q)
        lo = mid;
      else
        hi = mid;
    }
    const u64 j = (u64)s.rbeg[lo] + (q - s.roff[lo]);
    if (lo < k) {
      const Rows& R = p.runs[lo].rows;
      const u64 key = R.key[j];
      s.dkey[q] = key;
      s.dval[q] = R.val[j];
      s.dts[q] = R.ts[j];
      s.dnode[q] = R.node[j];
      s.dcnt[q] = R.cnt[j];
      s.ukey[q] = key;
      s.utag[q] = ((u32)lo << 16) | q;
    } else {
      s.ukey[q] = p.runs[lo - k].keys[j];
      s.utag[q] = ((u32)(lo - k) << 16) | MARK | q;
    }
  }
  u32 np2 = 2;
  while (np2 < nU) np2 <<= 1;
  for (u32 q = nU + tid; q < np2; q += KB) {
    s.ukey[q] = ~0ull;
    s.utag[q] = ~0u;
  }
  __syncthreads();
  if (nU > 1) sort_items(s.ukey, s.utag, np2);

  // ---- evaluate every candidate
  const u64 all = p.allmask;
  for (u32 i = tid; i < nS; i += KB) {
    const u64 x = s.skey[i];
    const u32 lb = lower_key(s.ukey, nU, x);
    s.slbu[i] = (unsigned short)lb;
    u64 K = all, R = 0, M = 0;
    const Row r = srow(s, i);
    for (u32 q = lb; q < nU && s.ukey[q] == x; q++) {
      const u32 tg = s.utag[q], src = tg >> 16;
      if (tg & MARK) {
        K |= 1ull << src;
      } else {
        R |= 1ull << src;
        if (row_eq(drow(s, tg & SLOT), r)) M |= 1ull << src;
      }
    }
    s.ssurv[i] = present(true, K, R, M, r.node, r.cnt, p.tabC, p.tabP);
  }
  for (u32 q = tid; q < nU; q += KB) {
    const u32 tg = s.utag[q];
    bool surv = false;
    if (!(tg & MARK)) {
      const u64 x = s.ukey[q];
      const u32 src = tg >> 16;
      const Row r = drow(s, tg & SLOT);
      u32 gb = q;
      while (gb > 0 && s.ukey[gb - 1] == x) gb--;
      u64 K = all, R = 0, M = 0;
      bool rep = true;  // the first holder of this tuple: the state, else the lowest delta
      for (u32 e = gb; e < nU && s.ukey[e] == x; e++) {
        const u32 te = s.utag[e], se = te >> 16;
        if (te & MARK) {
          K |= 1ull << se;
        } else {
          R |= 1ull << se;
          if (row_eq(drow(s, te & SLOT), r)) {
            M |= 1ull << se;
            if (se < src) rep = false;
          }
        }
      }
      if (rep) {  // a tuple the state holds is evaluated (and emitted) as the state's row
        u32 lo = lower_key(s.skey, nS, x);
        while (lo < nS && s.skey[lo] == x && row_cmp(srow(s, lo), r) < 0) lo++;
        if (lo < nS && row_eq(srow(s, lo), r)) rep = false;
      }
      if (rep) surv = present(false, K, R, M, r.node, r.cnt, p.tabC, p.tabP);
    }
    s.usurv[q] = surv;
  }
  __syncthreads();
  scan_flags(s.ssurv, nS, s.spre, s.wave);
  scan_flags(s.usurv, nU, s.upre, s.wave);
  __syncthreads();

  // ---- output offset of the bucket (decoupled look-back in ticket order)
  const u32 total = (u32)s.spre[nS] + s.upre[nU];
  if (tid < WAVE) {
    u64 prefix = 0;
    if (t == 0) {
      if (tid == 0) lb_publish(p.scan.state, 0, p.scan.epoch, LB_INC, total);
    } else {
      if (tid == 0) lb_publish(p.scan.state, t, p.scan.epoch, LB_AGG, total);
      prefix = lb_lookback(p.scan.state, t, p.scan.epoch, p.scan.err);
      if (tid == 0) lb_publish(p.scan.state, t, p.scan.epoch, LB_INC, prefix + total);
    }
    if (tid == 0) {
      s.bcast[1] = prefix;
      if (t == p.T - 1) p.d_counts[0] = prefix + total;
    }
  }
  __syncthreads();
  const u64 base = s.bcast[1];

  // ---- survivors in tuple order: rank = survivors of smaller keys + of the same key
  //      with a smaller tuple
  for (u32 i = tid; i < nS; i += KB) {
    if (!s.ssurv[i]) continue;
    const Row r = srow(s, i);
    const u32 lb = s.slbu[i];
    u32 less = 0;
    for (u32 q = lb; q < nU && s.ukey[q] == r.key; q++)
      if (s.usurv[q] && row_cmp(drow(s, s.utag[q] & SLOT), r) < 0) less++;
    const u64 o = base + s.spre[i] + s.upre[lb] + less;
    p.out.key[o] = r.key;
    p.out.val[o] = r.val;
    p.out.ts[o] = r.ts;
    p.out.node[o] = r.node;
    p.out.cnt[o] = r.cnt;
  }
  for (u32 q = tid; q < nU; q += KB) {
    if (!s.usurv[q]) continue;
    const Row r = drow(s, s.utag[q] & SLOT);
    u32 gb = q;
    while (gb > 0 && s.ukey[gb - 1] == r.key) gb--;
    u32 less = 0;
    for (u32 e = gb; e < nU && s.ukey[e] == r.key; e++)
      if (s.usurv[e] && row_cmp(drow(s, s.utag[e] & SLOT), r) < 0) less++;
    const u32 ls = lower_key(s.skey, nS, r.key);
    u32 sl = 0;
    for (u32 i = ls; i < nS && s.skey[i] == r.key; i++)
      if (s.ssurv[i] && row_cmp(srow(s, i), r) < 0) sl++;
    const u64 o = base + s.spre[ls] + sl + s.upre[gb] + less;
    p.out.key[o] = r.key;
    p.out.val[o] = r.val;
    p.out.ts[o] = r.ts;
    p.out.node[o] = r.node;
    p.out.cnt[o] = r.cnt;
  }
}

}  // namespace

hipError_t launch_kfold(const KFoldArgs& p, hipStream_t st) {
  hipLaunchKernelGGL(kfold_prep_kernel, dim3(1), dim3(KNT), 0, st, p);
  const u64 total = p.s.n + p.n_run_elems;
  if (total) {
    const u64 g = std::min<u64>((total + 255) / 256, 4096);
    hipLaunchKernelGGL(kfold_fill_kernel, dim3((u32)g), dim3(256), 0, st, p);
  }
  hipLaunchKernelGGL(kfold_kernel, dim3((u32)p.T), dim3(KB), 0, st, p);
  return hipGetLastError();
}

}  // namespace dg
