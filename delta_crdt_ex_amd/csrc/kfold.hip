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
//   kfold_prep          dense VV tables: tabC[i][node] = c_i, tabP[i][node] = C_{i-1}
//                       (node ids < KNT; larger ids in a context -> fallback flag), and
//                       the output context C_k in node order.
//   kfold_fill_kernel   key ids are 64-bit hashes, so the key space is cut into T equal
//                       buckets; for every delta row run / keyset run, start[t][run] = its
//                       first element of bucket >= t (one coalesced pass over the keys);
//                       the same starts for the state by one wave-wide search per bucket
//                       (the state is much longer than the deltas and is not scanned).
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
constexpr int CU = CD + CM;      // items after the keyset fold (delta rows + unfolded entries)
constexpr int CUL = CD + 2 * CM; // items staged: delta rows + keyset entries, before the fold
constexpr u32 MARK = 1u << 15;   // utag: (src << 16) | MARK? | KIN? | pre-sort slot
constexpr u32 KIN = 1u << 14;    // a delta row whose key is in its own delta's keyset
constexpr u32 SLOT = KIN - 1;
static_assert(2 * KFOLD_MAX_K <= KB, "one thread per run");
static_assert(CUL <= SLOT + 1, "slot bits");
static_assert(CD <= KFOLD_BLOCK && CUL <= 2 * KFOLD_BLOCK, "items q and q + KB of a thread: the second is a keyset entry");

__device__ __forceinline__ u64 bucket_of(u64 key, u64 T) { return __umul64hi(key, T); }

__device__ __forceinline__ u64 vv_at(const u64* tab, u32 i, u32 node) {
  return node < (u32)KNT ? tab[(u64)i * KNT + node] : 0ull;
}

// the hash set of the dot-set contexts' dots: key (cnt << 16) | (node << 6) | i
__device__ __forceinline__ u64 dset_key(u32 i, u32 node, u64 cnt) {
  return (cnt << 16) | ((u64)node << 6) | (u64)i;
}
__device__ __forceinline__ u64 dset_slot(u64 key, u64 mask) {
  u64 x = key * 0x9E3779B97F4A7C15ull;
  return (x ^ (x >> 29)) & mask;
}
// c_i covers (node, cnt): a VV entry >= cnt, or the dot in c_i's set (one probe, more
// only on a collision: the table is at most half full)
template <bool DOTS>
__device__ __forceinline__ bool covers(const u64* tabC, const KFoldArgs& p, u32 i, u32 node, u64 cnt,
                                       u64 vv) {
  if (!DOTS || !((p.dotsmask >> i) & 1)) return vv >= cnt;
  if (node >= (u32)KNT || cnt >= KF_CNT_LIMIT) return false;  // never inserted
  const u64 key = dset_key(i, node, cnt);
  for (u64 h = dset_slot(key, p.dset_mask);; h = (h + 1) & p.dset_mask) {
    const u64 x = p.dset[h];
    if (x == key) return true;
    if (x == KF_EMPTY) return false;
  }
}

// P after the touching deltas (bits of K | R, in delta order; see the header), for a
// thread's two candidates (its state row and its item) at once: the
// table reads of both are issued before either is evaluated, so the two candidates cost
// one round trip to the VV tables instead of two.  PB2 touching deltas per candidate per
// round (one round covers almost every candidate).
constexpr int PB2 = 2;
struct Cand {
  bool P;
  u64 K, R, M;
  u32 node;
  u64 cnt;
};
template <bool DOTS>
__device__ __forceinline__ void present2(Cand& a, bool da, Cand& b, bool db, const u64* tabC,
                                         const u64* tabP, const KFoldArgs& p) {
  u64 ba = da ? (a.K | a.R) : 0ull, bb = db ? (b.K | b.R) : 0ull;
  while (ba | bb) {
    u32 ia[PB2], ib[PB2];
    u64 ca[PB2], qa[PB2], cb[PB2], qb[PB2];
    int na = 0, nb = 0;
#pragma unroll
    for (int j = 0; j < PB2; j++) {
      ia[j] = ba ? (u32)__builtin_ctzll(ba) : 0u;
      na += ba ? 1 : 0;
      ba &= ba - 1;
      ib[j] = bb ? (u32)__builtin_ctzll(bb) : 0u;
      nb += bb ? 1 : 0;
      bb &= bb - 1;
    }
#pragma unroll
    for (int j = 0; j < PB2; j++) {
      ca[j] = j < na ? vv_at(tabC, ia[j], a.node) : 0ull;
      qa[j] = j < na ? vv_at(tabP, ia[j], a.node) : 0ull;
      cb[j] = j < nb ? vv_at(tabC, ib[j], b.node) : 0ull;
      qb[j] = j < nb ? vv_at(tabP, ib[j], b.node) : 0ull;
    }
#pragma unroll
    for (int j = 0; j < PB2; j++) {
      if (j < na) {
        const u32 i = ia[j];
        const bool inD = (a.M >> i) & 1;
        a.P = ((a.K >> i) & 1) ? (a.P ? (inD || !covers<DOTS>(tabC, p, i, a.node, a.cnt, ca[j]))
                                      : (inD && qa[j] < a.cnt))
                               : inD;
      }
      if (j < nb) {
        const u32 i = ib[j];
        const bool inD = (b.M >> i) & 1;
        b.P = ((b.K >> i) & 1) ? (b.P ? (inD || !covers<DOTS>(tabC, p, i, b.node, b.cnt, cb[j]))
                                      : (inD && qb[j] < b.cnt))
                               : inD;
      }
    }
  }
}

// ------------------------------------------------------------------------ prep
// One workgroup of KNT threads (workgroup 0 of the fill launch, so that this single-block
// latency chain runs beside the fill instead of before it).
__device__ __forceinline__ void kfold_prep(const KFoldArgs& p) {
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
  for (int i = n / WAVE; i < k; i += KNT / WAVE) {  // one wave per delta context
    const Ctx c = p.runs[i].ctx;
    const bool dots = (p.dotsmask >> i) & 1;  // a dot set: its per-node max (several lanes
                                              // may meet one node: atomicMax)
    for (u64 e = n % WAVE; e < c.n; e += WAVE) {
      const u32 nd = c.node[e];
      const u64 cn = c.cnt[e];
      if (nd >= (u32)KNT || (dots && cn >= KF_CNT_LIMIT)) {
        atomicOr(p.flag, KF_PREP_FAIL);
        continue;
      }
      if (dots)
        atomicMax((unsigned long long*)&p.tabC[(u64)i * KNT + nd], (unsigned long long)cn);
      else
        p.tabC[(u64)i * KNT + nd] = cn;
      pres[nd] = 1;
    }
  }
  __syncthreads();
  // prefix unions: C_i = C_{i-1} ⊔ c_i, per node the max (absent = 0); loads batched
  // ahead of the stores they would otherwise be ordered behind
  u64 acc = p.tabP[n];
  for (int i0 = 0; i0 < k; i0 += 8) {
    u64 c[8];
#pragma unroll
    for (int q = 0; q < 8; q++) c[q] = p.tabC[(u64)(i0 + q < k ? i0 + q : i0) * KNT + n];
    asm volatile("" ::: "memory");  // (all eight issued before any is used)
#pragma unroll
    for (int q = 0; q < 8; q++) c[q] = i0 + q < k ? c[q] : 0ull;
#pragma unroll
    for (int q = 0; q < 8; q++) {
      acc = max(acc, c[q]);
      if (i0 + q + 1 < k) p.tabP[(u64)(i0 + q + 1) * KNT + n] = acc;
    }
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

// sstart[t] for t in [0, T]: the state's first row whose bucket is >= t, one wave per t
// (a 64-ary search: 4 dependent load rounds at 10M rows) instead of a pass over all of the
// state's keys (80 MB at config 3).  Every wave's first rounds read the same keys, so
// they are L2 hits; a probe span around the proportional position n t / T (two rounds)
// measured slower, 57.9 vs 51.4 us for the fill: its 64 lines per wave are all distinct.
__device__ __forceinline__ void state_start(const KFoldArgs& p, u64 t) {
  const int lane = threadIdx.x & (WAVE - 1);
  const u64* k = p.s.key;
  const u64 T = p.T;
  u64 lo = 0, hi = p.s.n;
  while (hi - lo > WAVE) {
    const u64 span = hi - lo;
    const u64 q = lo + span * (u64)(lane + 1) / (WAVE + 1);
    const u64 m = __ballot(bucket_of(k[q], T) < t);  // true on a prefix of the lanes
    const int c = __popcll(m);
    const u64 nlo = c ? lo + span * (u64)c / (WAVE + 1) + 1 : lo;
    const u64 nhi = c < WAVE ? lo + span * (u64)(c + 1) / (WAVE + 1) : hi;
    lo = nlo;
    hi = nhi;
  }
  const bool lt = lo + lane < hi && bucket_of(k[lo + lane], T) < t;
  const u64 r = lo + (u64)__popcll(__ballot(lt));
  if (lane == 0) p.sstart[t] = r;
}

// One launch of KNT-thread workgroups: workgroup 0 builds the VV tables (kfold_prep);
// workgroups [1, 1 + fill_blocks) walk the delta runs; the workgroups past them search the
// state's starts, one bucket per wave.
//
// The delta walk writes the (T+1) x 2k start table, bucket-major: the entry of (bucket,
// run) is one u32 of the 512-B row the bucket's workgroup reads in one go.  Every run is
// cut into the same number P of equal slices (P = fill_p, a multiple of 8), and slice i of
// EVERY run goes to a workgroup of XCD i mod 8 (workgroups are dealt to the XCDs
// round-robin by index).  Keys are uniform hashes, so slice i of every run covers about
// the same bucket range: a row of the table is written, 4 bytes at a time, by the 2k runs
// all from one XCD, and the pieces merge in that XCD's L2 before they go to HBM (6.5 MB
// written for config 3's 6.5 MB table; chunks dealt to any XCD wrote 64 MB: every piece a
// partial line of its own).  Within a slice each thread issues its elements' loads before
// any store; the previous key comes from the neighbour lane by DPP.
constexpr int FILL_BLOCK = KNT;
constexpr int FILL_PER = 2;  // elements per thread per round (slices are <= 2048 long)
constexpr int FILL_WAVES = FILL_BLOCK / WAVE;
constexpr u32 FILL_XCD = 8;
__host__ __device__ __forceinline__ u32 fill_blocks(u32 fill_p, int k) {
  const u64 items = (u64)fill_p * 2 * (u64)k;  // (run, slice) pairs
  const u64 g = items < 2048 ? items : 2048;
  return (u32)((g + FILL_XCD - 1) / FILL_XCD * FILL_XCD);
}

__global__ __launch_bounds__(FILL_BLOCK) void kfold_fill_kernel(KFoldArgs p) {
  if (blockIdx.x == 0) {
    kfold_prep(p);
    return;
  }
  const u32 g = fill_blocks(p.fill_p, p.k);
  const u32 blk = blockIdx.x - 1;
  if (blk >= g) {  // block-uniform
    const u64 t = (u64)(blk - g) * FILL_WAVES + threadIdx.x / WAVE;  // wave-uniform
    if (t <= p.T) state_start(p, t);
    return;
  }
  const int nr = 2 * p.k;  // the delta runs
  const u64 T = p.T, stride = 2 * (u64)p.k;
  const u32 P = p.fill_p, per_x = P / FILL_XCD;
  const u32 x = blockIdx.x % FILL_XCD;        // this workgroup's XCD
  const u32 w = blk / FILL_XCD, nw = g / FILL_XCD;  // its index among the XCD's workgroups
  const int lane = threadIdx.x & (WAVE - 1);
  for (u64 m = w; m < (u64)nr * per_x; m += nw) {
    const int r = (int)(m / per_x);
    const u64 i = (m % per_x) * FILL_XCD + x;  // slice i of run r
    u64 n;
    const u64* keys = run_keys(p, r, &n);
    const u64 j0 = n * i / P, jend = n * (i + 1) / P;
    for (u64 jb = j0; jb < jend; jb += (u64)FILL_PER * FILL_BLOCK) {
      u64 kc[FILL_PER], kp[FILL_PER];
      // (every load unconditional at a clamped index and issued before any use -- the empty
      // asm keeps the compiler from waiting for each before issuing the next)
#pragma unroll
      for (int u = 0; u < FILL_PER; u++) {
        const u64 j = jb + (u64)u * FILL_BLOCK + threadIdx.x;
        const u64 jc = j < jend ? j : j0;
        kc[u] = keys[jc];
        kp[u] = keys[jc > 0 ? jc - 1 : 0];  // (lane 0's previous key; lanes > 0: DPP)
      }
      asm volatile("" ::: "memory");
#pragma unroll
      for (int u = 0; u < FILL_PER; u++) {
        const u64 j = jb + (u64)u * FILL_BLOCK + threadIdx.x;
        kc[u] = j < jend ? kc[u] : 0;
        kp[u] = (lane == 0 && j > 0 && j < jend) ? kp[u] : 0;
      }
#pragma unroll
      for (int u = 0; u < FILL_PER; u++) {
        const u64 j = jb + (u64)u * FILL_BLOCK + threadIdx.x;
        const u32 b = (u32)bucket_of(kc[u], T);  // every lane, for the DPP shift
        const u32 pb = wave_prev_or(b, (u32)bucket_of(kp[u], T));  // lane 0: its loaded key's
        if (j < jend) {
          u64 bb = j == 0 ? 0 : (u64)pb + 1;
          const u64 end = (j == n - 1) ? T : b;
          for (; bb <= end; bb++) p.dstart[bb * stride + r] = (u32)(bb <= b ? j : n);
        }
      }
    }
  }
}

// ------------------------------------------------------------------------ dot sets
// Every dot of the dot-set contexts into the hash set (one thread per dot; the context of
// dot j by a search of the k + 1 prefix sums).  Linear probing with atomicCAS; a dot is
// inserted once (a MapSet holds it once; a duplicate would find itself).
constexpr int DSB = 256;
__global__ __launch_bounds__(DSB) void kfold_dset_kernel(KFoldArgs p) {
  const u64 j = (u64)blockIdx.x * DSB + threadIdx.x;
  const u64 total = p.cflat[p.k];
  if (j >= total) return;
  int lo = 0, hi = p.k;  // cflat[lo] <= j < cflat[lo + 1]
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (p.cflat[mid] <= j)
      lo = mid;
    else
      hi = mid;
  }
  while (p.cflat[lo + 1] <= j) lo++;  // empty contexts between
  const Ctx c = p.runs[lo].ctx;
  const u64 e = j - p.cflat[lo];
  const u32 nd = c.node[e];
  const u64 cn = c.cnt[e];
  if (nd >= (u32)KNT || cn >= KF_CNT_LIMIT) return;  // the prep flags it: stepwise
  const u64 key = dset_key((u32)lo, nd, cn);
  for (u64 h = dset_slot(key, p.dset_mask);; h = (h + 1) & p.dset_mask) {
    const u64 old = atomicCAS((unsigned long long*)&p.dset[h], (unsigned long long)KF_EMPTY,
                              (unsigned long long)key);
    if (old == KF_EMPTY || old == key) return;
  }
}

// ------------------------------------------------------------------------ main
#ifdef DG_STAMPS
// Diagnostic build only (DG_STAMPS=1): per-bucket phase timestamps (s_memrealtime) by
// lane 0, read back with dg_debug_kfold_stamps (tools/kfold_stamps.py).
__device__ u64 g_kf_stamps[65536 * 16];
#define KSTAMP(tile, k)                                                              \
  do {                                                                               \
    __syncthreads();                                                                 \
    if (threadIdx.x == 0 && (tile) < 65536)                                          \
      g_kf_stamps[(tile) * 16 + (k)] = __builtin_amdgcn_s_memrealtime();             \
  } while (0)
#else
#define KSTAMP(tile, k) \
  do {                  \
  } while (0)
#endif

#ifndef DG_KFOLD_NSUB
#define DG_KFOLD_NSUB 1024  // (512: 904 us vs 878 us per config-3 fold; 768: 897 us)
#endif
constexpr int NSUB = DG_KFOLD_NSUB;  // sub-buckets of a bucket's key range (LDS counting sort)
constexpr int PER = 2;     // items per thread in the block scans
static_assert(CS <= PER * KB && CU <= PER * KB && NSUB <= PER * KB, "scan coverage");

struct KLds {
  u64 skey[CS], sval[CS], scnt[CS];
  i64 sts[CS];
  u32 snode[CS];
  u64 dkey[CD], dval[CD], dcnt[CD];  // delta rows by slot (= pre-sort item index)
  i64 dts[CD];
  u32 dnode[CD];
  u64 ukey[CU];                       // items: delta rows [0, nD), keyset markers [nD, nU)
  u32 utag[CU];                       // (src << 16) | MARK? | slot; (key, tag) order once sorted
  union {
    struct {
      unsigned short ustart[NSUB + 1];  // sub-bucket b: items [ustart[b], ustart[b+1])
      unsigned short sfirst[NSUB + 1];  //               state rows [sfirst[b], sfirst[b+1])
      unsigned short slbu[CS];          // state row -> first sorted item with key >= its key
      unsigned char ssurv[CS], usurv[CU];  // usurv by sorted position
    } e;
    u64 mkey[CUL - CD];               // while staging: the keyset entries' keys, before the
                                      // ones with rows of the key fold into those rows
  } y;
  union {
    u32 ucnt[NSUB];                   // counting-sort histogram / fill counters
    struct {
      unsigned short spre[CS + 1], upre[CU + 1];  // exclusive survivor prefixes
    } pre;
    struct {                          // while staging: the runs' column pointers
      RowsOut d[KFOLD_MAX_K];         //   delta rows (read only)
      const u64* keys[KFOLD_MAX_K];   //   keysets
    } run;
  } x;
  u32 roff[2 * KFOLD_MAX_K + 1];
  u32 rbeg[2 * KFOLD_MAX_K];
  u32 wave[KB / WAVE + 1];
  u64 lb[3 * (KB / WAVE) + 2];
  u64 bcast[1];
};

static_assert(sizeof(KLds) <= 80 * 1024, "two buckets per CU (160 KB of LDS)");

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

// Delta row d / state row i equal to r, whose key is already known to be equal: the
// other columns read one at a time, stopping at the first that differs (usually the value).
// The key-mask walks compare this way (and skip an item's compare with itself): 707 ->
// 691 us per config-3 fold (rocprofv3 A/B); the rank walks' order compares read lazily
// measured 695 us, and stay eager.
__device__ __forceinline__ bool drow_eq_k(const KLds& s, u32 d, const Row& r) {
  return s.dval[d] == r.val && s.dts[d] == r.ts && s.dnode[d] == r.node && s.dcnt[d] == r.cnt;
}
__device__ __forceinline__ bool srow_eq_k(const KLds& s, u32 i, const Row& r) {
  return s.sval[i] == r.val && s.sts[i] == r.ts && s.snode[i] == r.node && s.scnt[i] == r.cnt;
}

// sub-bucket of a key of bucket t: the next log2(NSUB) bits of its position in key space
__device__ __forceinline__ u32 sub_of(u64 key, u64 T, u64 t) {
  return (u32)(__umul64hi(key, T * NSUB) - t * NSUB);
}

// exclusive prefix of n <= PER*KB values into pre[0..n] (pre[n] = total)
// CURSOR: in[i] is also overwritten with pre[i] (each thread rewrites what it read)
template <bool CURSOR = false, class V>
__device__ __forceinline__ void scan_excl(V* in, u32 n, unsigned short* pre, u32* wave) {
  const u32 b = threadIdx.x * PER;
  u32 c[PER], sum = 0;
#pragma unroll
  for (int q = 0; q < PER; q++) {
    c[q] = (b + q < n) ? (u32)in[b + q] : 0u;
    sum += c[q];
  }
  u32 tot;
  u32 off = block_excl_scan<KB>(sum, wave, &tot);
#pragma unroll
  for (int q = 0; q < PER; q++) {
    if (b + q < n) {
      pre[b + q] = (unsigned short)off;
      if (CURSOR) in[b + q] = (V)off;
    }
    off += c[q];
  }
  if (threadIdx.x == 0) pre[n] = (unsigned short)tot;
}

// two 1024-thread buckets per CU: 8 waves per SIMD, so at most 64 VGPRs.  DOTS: some delta
// contexts are dot sets (their coverage through the hash set)
template <bool DOTS>
__global__ __launch_bounds__(KB) __attribute__((amdgpu_waves_per_eu(2 * KB / 256, 8))) void kfold_kernel(KFoldArgs p) {
  __shared__ KLds s;
  if (*p.flag & KF_PREP_FAIL) return;  // every workgroup leaves: no ticket is taken
  const int tid = threadIdx.x;
  const int k = p.k, nr = 2 * k;
  const u64 T = p.T;
  if (tid == 0) {  // (the ticket: buckets in workgroup order measured the same, 692-697 us)
    const u32 t = atomicAdd(p.scan.ticket, 1u);
    if ((u64)t == T - 1) atomicExch(p.scan.ticket, 0u);
    s.bcast[0] = t;
  }
  __syncthreads();
  const u64 t = s.bcast[0];
  KSTAMP(t, 0);
  if (tid < k) {  // the runs' column pointers (bucket-independent) for the staging below
    const Rows& R = p.runs[tid].rows;
    s.x.run.d[tid] = RowsOut{(u64*)R.key, (u64*)R.val, (i64*)R.ts, (u32*)R.node, (u64*)R.cnt};
  } else if (tid < nr) {
    s.x.run.keys[tid - k] = p.runs[tid - k].keys;
  }
  const u64 s0 = p.sstart[t];
  u32 nS = (u32)min<u64>(p.sstart[t + 1] - s0, 0xffffffffull);
  u32 len = 0;
  bool bad = p.sstart[t + 1] < s0;
  if (tid < nr) {
    const u32 a = p.dstart[t * nr + tid], b = p.dstart[(t + 1) * nr + tid];
    len = b >= a ? min(b - a, (u32)CUL + 1) : 0u;  // bounded: the sum cannot wrap
    bad |= b < a;
    s.rbeg[tid] = a;
  }
  bad = __syncthreads_or(bad);
#ifdef DG_KFOLD_NO_STATE  // experiment build only: the delta-only half of the bucket work
  nS = 0;                 // (what pass 1 of a two-pass fold would cost)
#endif
  // the state row's loads go out now (they need only s0 and nS): they fly during the run
  // offsets' scan and the item loads, so staging costs one round trip, not two
  static_assert(CS <= KB && CU <= KB, "one state row and one item per thread");
  const bool hs = !bad && nS <= (u32)CS && (u32)tid < nS;
  Row sr{};
  if (hs) sr = load_row(p.s, s0 + tid);
  u32 nU;
  const u32 off = block_excl_scan<KB>(len, s.wave, &nU);
  if (tid < nr) s.roff[tid] = off;
  if (tid == 0) s.roff[nr] = nU;
  KSTAMP(t, 12);
  __syncthreads();
  u32 nD = s.roff[k];
  if (bad || nS > (u32)CS || nD > (u32)CD || nU > (u32)CUL || nU - nD > (u32)(CUL - CD)) {
    if (tid == 0) atomicOr(p.flag, KF_OVERFLOW);
    nS = nU = nD = 0;  // publish an empty bucket so the look-back chain stays live
  }

  // ---- stage: state slice, delta rows (slot = pre-sort index) and the keyset entries'
  //      keys (y.mkey, by index - nD); a thread stages items q and q + KB (the second,
  //      past every delta row, is a keyset entry); the loads are issued before any row is
  //      written to LDS
  const u32 q = tid;  // this thread's items: q, and q2 = q + KB
  const u32 q2 = tid + KB;
  Row ir{};
  u32 itag = 0;
  u64 key2 = 0;
  u32 tag2 = 0;
  auto run_of = [&](u32 x) {  // roff[lo] <= x < roff[lo + 1]
    int lo = 0, hi = nr;
    while (hi - lo > 1) {
      const int mid = (lo + hi) >> 1;
      if (s.roff[mid] <= x)
        lo = mid;
      else
        hi = mid;
    }
    return lo;
  };
  if (q < nU) {
    const int lo = run_of(q);
    const u64 j = (u64)s.rbeg[lo] + (q - s.roff[lo]);
    if (lo < k) {
      const RowsOut& R = s.x.run.d[lo];
      ir = Row{R.key[j], R.val[j], R.cnt[j], R.ts[j], R.node[j]};
      itag = ((u32)lo << 16) | q;
    } else {
      ir.key = s.x.run.keys[lo - k][j];
      itag = ((u32)(lo - k) << 16) | MARK | q;
    }
  }
  if (q2 < nU) {
    const int lo = run_of(q2);
    key2 = s.x.run.keys[lo - k][(u64)s.rbeg[lo] + (q2 - s.roff[lo])];
    tag2 = ((u32)(lo - k) << 16) | MARK | q2;
  }
  if (hs && (u32)tid < nS) {
    s.skey[tid] = sr.key;
    s.sval[tid] = sr.val;
    s.sts[tid] = sr.ts;
    s.snode[tid] = sr.node;
    s.scnt[tid] = sr.cnt;
  }
  if (q < nU) {
    if (!(itag & MARK)) {
      s.ukey[q] = ir.key;
      s.dkey[q] = ir.key;
      s.dval[q] = ir.val;
      s.dts[q] = ir.ts;
      s.dnode[q] = ir.node;
      s.dcnt[q] = ir.cnt;
    } else {
      s.y.mkey[q - nD] = ir.key;
    }
  }
  if (q2 < nU) s.y.mkey[q2 - nD] = key2;
  KSTAMP(t, 1);
  __syncthreads();  // (the run pointers in s.x are dead: the histogram takes it)

  // ---- a keyset entry of a delta that also has rows of the key is folded into those
  //      rows (KIN on their tags) and dropped from the items: a sync delta's keyset is
  //      mostly its row keys (Map.take(value, keys)), so the sort and every walk below
  //      see about half the items.  Rows search their delta's keyset slice (y.mkey),
  //      entries their delta's row slice (dkey; both sorted).
  auto in_slice = [&](const u64* col, u32 lo, u32 hi, u64 x) {
    u32 a = lo, b = hi;
    while (a < b) {
      const u32 m = (a + b) >> 1;
      if (col[m] < x)
        a = m + 1;
      else
        b = m;
    }
    return a < hi && col[a] == x;
  };
  bool keep = false, keep2 = false;
  if (q < nU) {
    const u32 src = itag >> 16;
    if (itag & MARK) {
      keep = !in_slice(s.dkey, s.roff[src], s.roff[src + 1], ir.key);
    } else if (in_slice(s.y.mkey, s.roff[k + src] - nD, s.roff[k + src + 1] - nD, ir.key)) {
      itag |= KIN;
    }
  }
  if (q2 < nU) {
    const u32 src = tag2 >> 16;
    keep2 = !in_slice(s.dkey, s.roff[src], s.roff[src + 1], key2);
  }
  for (u32 b = tid; b < NSUB; b += KB) s.x.ucnt[b] = 0;  // (the scan's barriers order it)
  u32 n_keep;
  // (the scan's barriers come after every search: the entries may move after it)
  const u32 kpos = block_excl_scan<KB>((keep ? 1u : 0u) + (keep2 ? 1u : 0u), s.wave, &n_keep);
  if (nD + n_keep > (u32)CU) {  // more unfolded keyset entries than item slots (uniform)
    if (tid == 0) atomicOr(p.flag, KF_OVERFLOW);
    nS = nD = n_keep = 0;
    keep = keep2 = false;
  }
  // the remaining items in place, each counted in its sub-bucket (the counting sort's
  // histogram, from the registers)
  if (q < nD) {
    s.utag[q] = itag;
    atomicAdd(&s.x.ucnt[sub_of(ir.key, T, t)], 1u);
  } else if (keep) {
    const u32 nq = nD + kpos;
    s.ukey[nq] = ir.key;
    s.utag[nq] = (itag & ~SLOT) | nq;
    atomicAdd(&s.x.ucnt[sub_of(ir.key, T, t)], 1u);
  }
  if (keep2) {
    const u32 nq = nD + kpos + (keep ? 1u : 0u);
    s.ukey[nq] = key2;
    s.utag[nq] = (tag2 & ~SLOT) | nq;
    atomicAdd(&s.x.ucnt[sub_of(key2, T, t)], 1u);
  }
  nU = nD + n_keep;

  // ---- counting sort of the items by sub-bucket, then (key, tag) within one
  for (u32 i = tid; i < nS; i += KB) {  // state rows: first row of every sub-bucket
    const u32 sb = sub_of(s.skey[i], T, t);
    u32 b = i == 0 ? 0 : sub_of(s.skey[i - 1], T, t) + 1;
    for (; b <= sb; b++) s.y.e.sfirst[b] = (unsigned short)i;
    if (i == nS - 1)
      for (b = sb + 1; b <= (u32)NSUB; b++) s.y.e.sfirst[b] = (unsigned short)nS;
  }
  if (nS == 0)
    for (u32 b = tid; b <= (u32)NSUB; b += KB) s.y.e.sfirst[b] = 0;
  KSTAMP(t, 13);
  __syncthreads();
  // sub-bucket starts; the counts become the scatter's cursors (each thread rewrites the
  // entries it read)
  scan_excl<true>(s.x.ucnt, NSUB, s.y.e.ustart, s.wave);
  KSTAMP(t, 9);
  __syncthreads();
  unsigned short* bin = s.y.e.slbu;  // items grouped by sub-bucket (slbu is free until evaluation)
  for (u32 q = tid; q < nU; q += KB) {
    const u32 sb = sub_of(s.ukey[q], T, t);
    bin[atomicAdd(&s.x.ucnt[sb], 1u)] = (unsigned short)q;
  }
  KSTAMP(t, 10);
  __syncthreads();
  // rank by (key, tag) within the (small) sub-bucket, then every item moves itself to
  // its sorted position (the items of a thread are read before the barrier, written
  // after it), so later phases index ukey/utag directly
  u64 mk[(CU + KB - 1) / KB];
  u32 mt[(CU + KB - 1) / KB], mp[(CU + KB - 1) / KB];
#pragma unroll
  for (int j = 0; j < (CU + KB - 1) / KB; j++) {
    const u32 q = tid + j * KB;
    mp[j] = ~0u;
    if (q >= nU) continue;
    const u64 kq = s.ukey[q];
    const u32 tq = s.utag[q], sb = sub_of(kq, T, t), lo = s.y.e.ustart[sb], hi = s.y.e.ustart[sb + 1];
    u32 rank = 0;
    for (u32 e = lo; e < hi; e++) {
      const u32 w = bin[e];
      const u64 kw = s.ukey[w];
      rank += (kw < kq || (kw == kq && s.utag[w] < tq)) ? 1u : 0u;
    }
    mk[j] = kq;
    mt[j] = tq;
    mp[j] = lo + rank;
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < (CU + KB - 1) / KB; j++)
    if (mp[j] != ~0u) {
      s.ukey[mp[j]] = mk[j];
      s.utag[mp[j]] = mt[j];
    }
  KSTAMP(t, 2);
  __syncthreads();

  // ---- evaluate every candidate (a key's items and state rows share its sub-bucket)
  // (one state row and one item per thread; both candidates' VV-table reads go out
  // together in present2)
  const u64 all = p.allmask;
  Cand cs{true, all, 0, 0, 0, 0}, cu{false, all, 0, 0, 0, 0};
  const bool ds = (u32)tid < nS;
  bool du = false;
  if (ds) {
    const u32 i = tid;
    const Row r = srow(s, i);
    const u32 sb = sub_of(r.key, T, t);
    u32 e = s.y.e.ustart[sb];
    const u32 qe = s.y.e.ustart[sb + 1];
    while (e < qe && s.ukey[e] < r.key) e++;
    s.y.e.slbu[i] = (unsigned short)e;
    for (; e < qe && s.ukey[e] == r.key; e++) {
      const u32 tg = s.utag[e], src = tg >> 16;
      if (tg & (MARK | KIN)) cs.K |= 1ull << src;
      if (!(tg & MARK)) {
        cs.R |= 1ull << src;
        if (drow_eq_k(s, tg & SLOT, r)) cs.M |= 1ull << src;
      }
    }
    cs.node = r.node;
    cs.cnt = r.cnt;
  }
  if ((u32)tid < nU && !(s.utag[tid] & MARK)) {
    const u32 tg = s.utag[tid], src = tg >> 16;
    const Row r = drow(s, tg & SLOT);
    const u32 sb = sub_of(r.key, T, t);
    bool first = true;  // the first holder of this tuple: the state, else the lowest delta
    // (the items are sorted by (key, tag) and this one sits at position tid: its key's
    // group starts at most a few items before it)
    u32 e = tid;
    while (e > 0 && s.ukey[e - 1] == r.key) e--;
    for (; e < nU && s.ukey[e] == r.key; e++) {
      const u32 te = s.utag[e], se = te >> 16;
      if (te & (MARK | KIN)) cu.K |= 1ull << se;
      if (!(te & MARK)) {
        cu.R |= 1ull << se;
        if (e == (u32)tid || drow_eq_k(s, te & SLOT, r)) {  // (the item itself: no reads)
          cu.M |= 1ull << se;
          if (se < src) first = false;
        }
      }
    }
    // a tuple the state holds is evaluated (and emitted) as the state's row (the state
    // rows of the sub-bucket are sorted: compare full rows only under the same key)
    u32 i = s.y.e.sfirst[sb];
    const u32 ie = s.y.e.sfirst[sb + 1];
    while (i < ie && s.skey[i] < r.key) i++;
    for (; first && i < ie && s.skey[i] == r.key; i++)
      if (srow_eq_k(s, i, r)) first = false;
    du = first;
    cu.node = r.node;
    cu.cnt = r.cnt;
  }
  KSTAMP(t, 7);
  present2<DOTS>(cs, ds, cu, du, p.tabC, p.tabP, p);
  const bool ss_ = ds && cs.P, us_ = (u32)tid < nU && du && cu.P;
  if (ds) s.y.e.ssurv[tid] = ss_;
  if ((u32)tid < nU) s.y.e.usurv[tid] = us_;
  KSTAMP(t, 3);
  // the survivors' exclusive prefixes, state rows (low half) and items (high half) in ONE
  // block scan of the thread's own flags (one state row and one item per thread); entry n
  // holds the total (the threads past nS / nU write it too)
  {
    u32 tot2;
    const u32 pre2 = block_excl_scan<KB>((ss_ ? 1u : 0u) | (us_ ? 1u << 16 : 0u), s.wave, &tot2);
    s.x.pre.spre[tid] = (unsigned short)(pre2 & 0xFFFFu);
    s.x.pre.upre[tid] = (unsigned short)(pre2 >> 16);
    if (tid == 0) {
      s.x.pre.spre[nS] = (unsigned short)(tot2 & 0xFFFFu);
      s.x.pre.upre[nU] = (unsigned short)(tot2 >> 16);
    }
  }
  __syncthreads();
  KSTAMP(t, 4);

  // ---- the bucket's survivor count goes out first (decoupled look-back in ticket
  //      order), then every survivor's position inside the bucket is ranked while the
  //      predecessors publish theirs, and only then is the bucket's offset looked up
  const u32 total = (u32)s.x.pre.spre[nS] + s.x.pre.upre[nU];
  if (tid == 0) lb_publish(p.scan.state, t, p.scan.epoch, t == 0 ? LB_INC : LB_AGG, total);

  // survivors in tuple order: rank = survivors of smaller keys + of the same key with a
  // smaller tuple
  constexpr int RS = (CS + KB - 1) / KB, RU = (CU + KB - 1) / KB;
  u32 so[RS], uo[RU];  // in-bucket output position, ~0u: not a survivor of this thread
  const unsigned short* spre = s.x.pre.spre;
  const unsigned short* upre = s.x.pre.upre;
#pragma unroll
  for (int j = 0; j < RS; j++) {
    const u32 i = tid + j * KB;
    so[j] = ~0u;
    if (i >= nS || !s.y.e.ssurv[i]) continue;
    const Row r = srow(s, i);
    const u32 lb = s.y.e.slbu[i];
    u32 less = 0;
    for (u32 q = lb; q < nU && s.ukey[q] == r.key; q++)
      if (s.y.e.usurv[q] && row_cmp(drow(s, s.utag[q] & SLOT), r) < 0) less++;
    so[j] = spre[i] + upre[lb] + less;
  }
#pragma unroll
  for (int j = 0; j < RU; j++) {
    const u32 q = tid + j * KB;
    uo[j] = ~0u;
    if (q >= nU || !s.y.e.usurv[q]) continue;
    const Row r = drow(s, s.utag[q] & SLOT);
    const u32 sb = sub_of(r.key, T, t);
    u32 gb = q;  // the first item of its key: a few positions back at most
    while (gb > 0 && s.ukey[gb - 1] == r.key) gb--;
    u32 less = 0;
    for (u32 e = gb; e < nU && s.ukey[e] == r.key; e++)
      if (s.y.e.usurv[e] && row_cmp(drow(s, s.utag[e] & SLOT), r) < 0) less++;
    u32 ls = s.y.e.sfirst[sb];
    const u32 le = s.y.e.sfirst[sb + 1];
    while (ls < le && s.skey[ls] < r.key) ls++;
    u32 sl = 0;
    for (u32 i = ls; i < le && s.skey[i] == r.key; i++)
      if (s.y.e.ssurv[i] && row_cmp(srow(s, i), r) < 0) sl++;
    uo[j] = spre[ls] + sl + upre[gb] + less;
  }
  KSTAMP(t, 5);

  // ---- the bucket's output offset (block-wide: one round trip reaches a whole launch
  //      round of predecessors), then the rows
  u64 base = 0;
  if (t > 0) {
    base = lb_lookback_block<KB, 1>(p.scan.state, t, p.scan.epoch, p.scan.err, s.lb);
    if (tid == 0) lb_publish(p.scan.state, t, p.scan.epoch, LB_INC, base + total);
  }
  if (tid == 0 && t == T - 1) p.d_counts[0] = base + total;
// plain stores, not non-temporal: a bucket's state rows and items interleave in the
// output, so every line is written in pieces by several waves, and the pieces must merge
// in the L2 (non-temporal: 783 MB written per config-3 fold; plain: 376 MB = the output)
#pragma unroll
  for (int j = 0; j < RS; j++)
    if (so[j] != ~0u) store_row(p.out, base + so[j], srow(s, tid + j * KB));
#pragma unroll
  for (int j = 0; j < RU; j++)
    if (uo[j] != ~0u) store_row(p.out, base + uo[j], drow(s, s.utag[tid + j * KB] & SLOT));
  KSTAMP(t, 6);
}

}  // namespace

#ifdef DG_STAMPS
extern "C" int dg_debug_kfold_stamps(unsigned long long* host, size_t n) {
  if (n > 65536 * 16) n = 65536 * 16;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_kf_stamps), n * 8) == hipSuccess ? 0 : -3;
}
#endif

hipError_t launch_kfold(const KFoldArgs& p, hipStream_t st) {
  if (p.dotsmask) {  // the host set p.dset to KF_EMPTY and passes the contexts' total in dset_n
    const u64 n = p.dset_n;
    if (n) hipLaunchKernelGGL(kfold_dset_kernel, dim3((u32)((n + DSB - 1) / DSB)), dim3(DSB), 0, st, p);
  }
  // prep + delta fill + the state's starts
  const u64 g = 1 + fill_blocks(p.fill_p, p.k) + (p.T + FILL_WAVES) / FILL_WAVES;
  hipLaunchKernelGGL(kfold_fill_kernel, dim3((u32)g), dim3(FILL_BLOCK), 0, st, p);
  if (p.dotsmask)
    hipLaunchKernelGGL(kfold_kernel<true>, dim3((u32)p.T), dim3(KB), 0, st, p);
  else
    hipLaunchKernelGGL(kfold_kernel<false>, dim3((u32)p.T), dim3(KB), 0, st, p);
  return hipGetLastError();
}

}  // namespace dg
