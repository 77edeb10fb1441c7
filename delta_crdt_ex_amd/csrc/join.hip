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
// Kernel shape (HBM-bound integer merge; no MFMA):
//   1. join2_partition_kernel: one wave per tile boundary finds the merge-path split
//      of diagonal q*jt (jt = JT, or less: balance_tiles).  Key ids are 64-bit hashes,
//      so the key gap at the proportional split (one probe) lands within a few rows of
//      the split and one 64-wide window
//      round finishes it (~5 cache lines per array instead of a 21-step search); any
//      key distribution stays exact through a 128-ary fallback search.  One extra
//      workgroup (the grid's first) computes the context union Dots.union(c1, c2) (:155).
//   2. join2_stream_kernel (single pass, the default): a persistent grid of G
//      resident workgroups (occupancy API) walks the tiles statically, t = w + k*G,
//      so tiles k*G .. k*G+G-1 form "stripe" k.  Per iteration a workgroup commits
//      the tile it prefetched into registers to one of two LDS buffers, issues the
//      loads of its next tile, merges JI positions per thread from LDS (keep/drop),
//      block-scans the keep flags into a u16 compaction list and publishes the
//      tile's count as an {epoch, count} granule in a per-stripe array.  The tile is
//      written out one iteration LATER: by then every workgroup has published its
//      count for that stripe, so each workgroup sums the G counts of the stripe
//      itself (a 1-4 KB coalesced read) instead of chaining look-backs, and the
//      output offset is a running sum over stripes.  Inputs are read once, outputs
//      written once: 36 B x (N_in + N_out) of HBM traffic plus the partition's probes.
//   (join2_slot_kernel + join2_compact_kernel: the two-pass variant, selected with
//    DG_JOIN_MODE=2, kept for A/B measurement.)
//
// Coverage (Dots.member?, :67-73) of a full-state join of two version vectors goes
// through a direct-indexed LDS table of the VVs' counters for node ids < VT (one
// ds_read per row); larger node ids and explicit dot sets use a binary search.
#include <algorithm>
#include <mutex>

#include "dg_ctxu.h"
#include "dg_launch.h"

namespace dg {

namespace {

constexpr int JB = JOIN_BLOCK;
constexpr int JI = JOIN_ITEMS;
constexpr int JT = JOIN_TILE;
static_assert(JT % 2 == 0, "even tiles (balance_tiles keeps them even)");
constexpr int JS = JT + 5;  // LDS row slots: tile rows + one neighbour on each side per store
                            // (+1: the merge's look-ahead read past the last B slot)
constexpr int VT = 64;      // VV table: node ids below this are looked up directly in LDS

#ifdef DG_STAMPS
// Diagnostic build only (DG_STAMPS=1): per-tile phase timestamps (s_memrealtime,
// 100 MHz) written by lane 0 into a buffer no other code reads.
__device__ u64 g_join_stamps[65536 * 16];
#define JSTAMP(tile, k)                                                              \
  do {                                                                               \
    __syncthreads();                                                                 \
    __builtin_amdgcn_sched_barrier(0);                                               \
    if (threadIdx.x == 0 && (tile) < 65536) g_join_stamps[(tile) * 16 + (k)] =       \
        __builtin_amdgcn_s_memrealtime();                                            \
    __builtin_amdgcn_sched_barrier(0);                                               \
  } while (0)
#else
#define JSTAMP(tile, k) \
  do {                  \
  } while (0)
#endif

// ------------------------------------------------------------- context union
// (Dots.union/2, aw_lww_map.ex:39-52: dg_ctxu.h; here its standalone one-workgroup kernel)
constexpr int CB = 1024;  // threads of the standalone context-union kernel

__global__ __launch_bounds__(CB) void ctx_union_kernel(CtxUnionArgs p) {
  __shared__ u32 s_wave[CB / WAVE + 1];
  ctx_union_block<CB>(p, s_wave);
}

// Scratch of dg_join2_changes (join2_changes_tmp_bytes): per tile JT event keys, then
// per-tile arrays: output offset, event count, differing-event count, first-event repeat
// flag, first and last event.
struct ChgLayout {
  u64* ev;
  u64* off;
  u32* cnt;
  u32* wu;
  u64* fk;
  u64* lk;
};

static __host__ ChgLayout chg_layout(void* tmp, u64 ntiles) {
  ChgLayout l;
  char* c = (char*)tmp;
  l.ev = (u64*)c;
  c += ntiles * (u64)JT * 8;
  l.off = (u64*)c;
  c += ntiles * 8;
  l.cnt = (u32*)c;
  c += ntiles * 4;
  l.wu = (u32*)c;
  c += ntiles * 4;
  c += ntiles * 4;  // (spare)
  c = (char*)(((uintptr_t)c + 7) & ~(uintptr_t)7);
  l.fk = (u64*)c;
  c += ntiles * 8;
  l.lk = (u64*)c;
  return l;
}

struct JoinArgs {
  Rows a, b;
  Ctx ca, cb;
  const u64* keys;
  u64 n_keys;
  const u64* splits;  // merge-path split (a index) of every tile boundary (partition pass)
  u64* ksplits;       // keyed joins: first index of `keys` >= the key at every tile boundary
  u64 ntiles;
  u64 jt;     // merged positions per tile, <= JT (launch_join2 spreads the tiles evenly
              // over the grid's stripes)
  RowsOut out;
  Scan scan;  // look-back granules + tile tickets
  u64* d_count;
  unsigned short* lists;  // two-pass only: tile t's compaction list at lists[t * JT ...]
  u32* counts;            // two-pass only: kept rows per tile
  u64* chg_tmp;           // CHG: JT change-event keys per tile
  u32* chg_cnt;           // CHG: events per tile
  u32* chg_wu;            // CHG: events after the tile's first that differ from their predecessor
  u64* chg_fk;            // CHG: the tile's first and last event (tiles with events)
  u64* chg_lk;
  int fused;              // stream kernel: splits searched in-kernel (no partition launch);
                          // the grid's last workgroup computes the context union
  CtxUnionArgs cu;
};

// ------------------------------------------------------------------ partition
// Merge-path predicate on diagonal `diag` over global memory: A[i] <= B[diag-1-i]
// (ties go to A).  Full rows are only loaded when the keys tie.
__device__ __forceinline__ bool mp_pred(const Rows A, const Rows B, u64 diag, u64 i) {
  u64 j = diag - 1 - i;
  u64 ka = A.key[i], kb = B.key[j];
  if (ka != kb) return ka < kb;
  return row_le(load_row(A, i), load_row(B, j));
}

constexpr int PB = 256;      // threads per partition block = 4 boundaries
constexpr int PK = 2 * WAVE;  // samples per search round (two per lane)

// One wave: first i in [lo, hi) with NOT mp_pred(i) (hi if none) by a 128-ary search.
__device__ u64 mp_search(const Rows A, const Rows B, u64 d, u64 lo, u64 hi) {
  const int lane = threadIdx.x & (WAVE - 1);
  for (int round = 0; round < 64 && hi > lo; round++) {
    const u64 span = hi - lo;
    bool f0, f1;  // lane l evaluates samples 2l and 2l+1
    if (span <= (u64)PK) {
      const u64 x0 = lo + 2 * lane, x1 = x0 + 1;
      f0 = x0 < hi && !mp_pred(A, B, d, x0);
      f1 = x1 < hi && !mp_pred(A, B, d, x1);
    } else {
      const u64 x0 = lo + (span * (u64)(2 * lane + 1)) / (PK + 1);
      const u64 x1 = lo + (span * (u64)(2 * lane + 2)) / (PK + 1);
      f0 = !mp_pred(A, B, d, x0);
      f1 = !mp_pred(A, B, d, x1);
    }
    const u64 m0 = __ballot(f0), m1 = __ballot(f1);
    int kf = PK;  // first false sample
    if (m0 | m1) {
      const int l0 = m0 ? __ffsll((long long)m0) - 1 : 64;
      const int l1 = m1 ? __ffsll((long long)m1) - 1 : 64;
      kf = (l0 <= l1) ? 2 * l0 : 2 * l1 + 1;
    }
    if (span <= (u64)PK) {
      return (u64)kf < span ? lo + kf : hi;
    } else if (kf == PK) {
      lo = lo + (span * (u64)PK) / (PK + 1) + 1;
    } else {
      const u64 nh = lo + (span * (u64)(kf + 1)) / (PK + 1);
      if (kf > 0) lo = lo + (span * (u64)kf) / (PK + 1) + 1;
      hi = nh;
    }
  }
  return lo;
}

// Merge-path split of diagonal d (= #A rows among the first d merged rows).
// A window of 64 consecutive candidates is decided in ONE round trip (one per lane,
// a ballot), first around the proportional guess d * na / (na + nb): replicas that share
// most keys (config 2) split there exactly.  If the window does not bracket the split,
// the key gap B.key[d-1-c] - A.key[c] at the window's middle c (in units of the 2^64
// key space; the rows were just loaded, so this is a cache hit) converts to a row shift
// of gap * na*nb / ((na+nb) * 2^64), which lands within a few rows for hashed keys, and
// the next window is decided there.  Three windows without a bracket fall back to the
// exact 128-ary search for any key distribution.
__device__ u64 mp_split(const Rows A, const Rows B, u64 d) {
  const int lane = threadIdx.x & (WAVE - 1);
  const u64 na = A.n, nb = B.n, total = na + nb;
  const u64 lo = d > nb ? d - nb : 0, hi = min(d, na);
  if (hi - lo <= (u64)PK) return mp_search(A, B, d, lo, hi);
  const double scale = (double)na * (double)nb / ((double)total * 18446744073709551616.0);
  u64 i = (u64)((double)d * (double)na / (double)total);
  i = min(max(i, lo), hi - 1);
  {  // the key gap at the proportional guess first (one scalar round trip): replicas that
     // differ (config 5: the guess is a median 342 rows off, 90 % of the boundaries needed
     // a second window) now bracket in the first.  Partition at config 5: 26.2 -> 20.4 us
    const double gap = (double)B.key[d - 1 - i] - (double)A.key[i];
    const double lim = (double)(hi - lo);
    double sft = gap * scale;
    sft = sft > lim ? lim : (sft < -lim ? -lim : sft);
    i64 ni = (i64)i + (i64)sft;
    ni = ni < (i64)lo ? (i64)lo : (ni > (i64)hi - 1 ? (i64)hi - 1 : ni);
    i = (u64)ni;
  }
  for (int r = 0; r < 3; r++) {
    // one candidate per lane: the gap-shifted guess is a median 11 rows off at config 5,
    // so 64-wide windows bracket as well as 128-wide ones and read half the keys
    // (partition 19.0 -> 16.9 us per config-5 join, rocprofv3 A/B)
    constexpr u64 PW = WAVE;
    u64 wlo = i > lo + PW / 2 ? i - PW / 2 : lo;
    const u64 whi = min(wlo + PW, hi);
    wlo = whi - PW > lo ? whi - PW : lo;
    const u64 x0 = wlo + lane;
    const u64 m0 = __ballot(x0 < whi && !mp_pred(A, B, d, x0));
    const u64 kf = m0 ? (u64)(__ffsll((long long)m0) - 1) : whi - wlo;
    // bracketed iff the first false is not at the window's low edge (unless that edge is
    // lo) and some candidate is false (unless the window reaches hi)
    if ((kf > 0 || wlo == lo) && (kf < whi - wlo || whi == hi)) return wlo + kf;
    const u64 c = (wlo + whi) / 2;
    const double gap = (double)B.key[d - 1 - c] - (double)A.key[c];
    double sft = gap * scale;
    const double lim = (double)(hi - lo);
    sft = sft > lim ? lim : (sft < -lim ? -lim : sft);
    i64 ni = (i64)c + (i64)sft;
    ni = ni < (i64)lo ? (i64)lo : (ni > (i64)hi - 1 ? (i64)hi - 1 : ni);
    i = (u64)ni;
  }
  return mp_search(A, B, d, lo, hi);
}

// The proportional split of diagonal d, d * na / (na + nb) clamped to the diagonal's
// range: exact for replicas that hold the same keys (config 2).
__device__ __forceinline__ u64 split_guess(u64 na, u64 nb, u64 d) {
  const u64 lo = d > nb ? d - nb : 0, hi = min(d, na);
  const u64 i = (u64)((double)d * (double)na / (double)(na + nb));
  return min(max(i, lo), hi);
}

// Whether g is diagonal d's split: A[g-1] <= B[d-g] and not A[g] <= B[d-1-g] (full tuples;
// at the diagonal's ends one side is vacuous).  Uniform indices: scalar loads.
__device__ __forceinline__ bool guess_exact(const Rows& A, const Rows& B, u64 d, u64 g) {
  const u64 lo = d > B.n ? d - B.n : 0, hi = min(d, A.n);
  bool ok = true;
  if (g > lo) ok = row_le(load_row(A, g - 1), load_row(B, d - g));
  if (g < hi) ok = ok && !row_le(load_row(A, g), load_row(B, d - 1 - g));
  return ok;
}

// Keyed joins: the first index of keys[0, n_keys) >= the key at merged position d (split
// s), by the calling wave.  Tile t's keys lie in [key(t*jt), key((t+1)*jt)], so the
// keyset entries they can match are [ksplit(t), ksplit(t+1)] (keys are unique).
__device__ __forceinline__ u64 key_split(const Rows& A, const Rows& B, const u64* keys, u64 n_keys,
                                         u64 d, u64 s) {
  const u64 ib = d - s;
  const bool va = s < A.n, vb = ib < B.n;
  if (!va && !vb) return n_keys;
  const u64 ka = va ? A.key[s] : ~0ull, kb = vb ? B.key[ib] : ~0ull;
  return wave_lower_bound(keys, n_keys, min(ka, kb));
}

__global__ __launch_bounds__(PB) void join2_partition_kernel(Rows A, Rows B, u64 ntiles, u64 jt,
                                                             u64* splits, CtxUnionArgs cu,
                                                             const u64* keys, u64 n_keys,
                                                             u64* ksplits) {
  // the extra workgroup computes Dots.union(c1, c2) (aw_lww_map.ex:155); it is the FIRST
  // of the grid so its latency chain runs beside the searches instead of after the last
  // of them has been dispatched (config 5: partition 20.4 -> 18.1 us, A/B)
  if (blockIdx.x == 0) {
    __shared__ u32 s_wave[PB / WAVE + 1];
    ctx_union_block<PB>(cu, s_wave);
    return;
  }
  const u64 q = (u64)(blockIdx.x - 1) * (PB / WAVE) + (threadIdx.x >> 6);
  if (q > ntiles) return;
  const u64 d = min(q * jt, A.n + B.n);
  const u64 s = mp_split(A, B, d);
  if ((threadIdx.x & (WAVE - 1)) == 0) splits[q] = s;
  if (keys) {
    const u64 kq = key_split(A, B, keys, n_keys, d, s);
    if ((threadIdx.x & (WAVE - 1)) == 0) ksplits[q] = kq;
  }
}

// ------------------------------------------------------------------- coverage
// Dots.member?(c, {dn, dc}) (aw_lww_map.ex:67-73).  For a full-state join of two
// version vectors (FAST) the counters of nodes < VT sit in a direct-indexed LDS
// table (Map.get(vv, node, 0) is table[node], absent nodes hold 0); node ids >= VT
// fall back to a binary search of the VV in global memory.
template <bool FAST>
__device__ __forceinline__ bool covers(const u64* tab, const Ctx& c, u32 dn, u64 dc) {
  if (FAST) {
    if (dn < (u32)VT) return tab[dn] >= dc;
    return ctx_covers(c.node, c.cnt, c.n, 0, dn, dc);
  }
  return ctx_covers(c.node, c.cnt, c.n, c.kind, dn, dc);
}

// The keyset entries a tile's keys can match (keyed joins): keys[kl, kl + km), staged in
// LDS (lds) when km <= KS -- a sync delta's few keys per tile -- else searched in global
// memory (lds == nullptr).  Membership replaces a binary search of the whole keyset per
// merged row.
constexpr int KS = 64;
struct KeySlice {
  const u64* lds;
  const u64* keys;  // keys + kl
  u64 km;
};

__device__ __forceinline__ bool key_in(const KeySlice& ks, u64 x) {
  if (ks.lds) {  // (uniform per tile) branch-free binary lifting over the staged slice
    const int km = (int)ks.km;
    int pos = 0;  // entries < x
#pragma unroll
    for (int step = KS; step >= 1; step >>= 1) {
      const int m = pos + step;
      const bool c = (m <= km) & (ks.lds[min(m, KS) - 1] < x);
      pos = c ? m : pos;
    }
    return (pos < km) & (ks.lds[min(pos, KS - 1)] == x);
  }
  return keyset_has(ks.keys, ks.km, x);
}

// VV tables: tab_a[node] / tab_b[node] = the VV's counter for node ids < VT (coalesced
// loads; the tables must have been zeroed behind a barrier).
// Returns whether this thread met a node id >= VT (a VV entry outside the tables).
__device__ __forceinline__ bool fill_vv_tables(const Ctx& ca, const Ctx& cb, u64* tab_a, u64* tab_b) {
  bool far = false;
  for (u64 i = threadIdx.x; i < ca.n; i += JB) {
    const u32 nd = ca.node[i];
    if (nd < (u32)VT) tab_a[nd] = ca.cnt[i];
    far |= nd >= (u32)VT;
  }
  for (u64 i = threadIdx.x; i < cb.n; i += JB) {
    const u32 nd = cb.node[i];
    if (nd < (u32)VT) tab_b[nd] = cb.cnt[i];
    far |= nd >= (u32)VT;
  }
  return far;
}

// ------------------------------------------------------------------- staging
// One staged tile: its rows (+ one neighbour on each side of each store), as 16-byte
// {key, val} and {ts, cnt} pairs plus the node column: a whole row is 3 LDS accesses
// (2 x ds_read_b128 + ds_read_b32) instead of 5, and the key-only search reads the
// low half of kv.
struct Buf {
  alignas(16) u64 kv[JS][2];
  alignas(16) u64 tc[JS][2];
  u32 node[JS];
};

__device__ __forceinline__ u64 buf_key(const Buf& s, int x) { return s.kv[x][0]; }

__device__ __forceinline__ void buf_put(Buf& s, int x, u64 key, u64 val, i64 ts, u32 node, u64 cnt) {
  typedef u64 v2u64 __attribute__((ext_vector_type(2)));
  *(v2u64*)s.kv[x] = v2u64{key, val};
  *(v2u64*)s.tc[x] = v2u64{(u64)ts, cnt};
  s.node[x] = node;
}

// Global row index of staging slot x, or -1 if the slot is outside the stores:
// slot x < nat + 2 is a[a0 - 1 + x], slot x >= nat + 2 is b[b0 - 1 + (x - nat - 2)].
__device__ __forceinline__ i64 slot_row(int x, int nat, u64 a0, u64 b0, u64 na, u64 nb,
                                        bool* from_b) {
  if (x < nat + 2) {
    const i64 g = (i64)a0 - 1 + x;
    *from_b = false;
    return (g >= 0 && (u64)g < na) ? g : -1;
  }
  const i64 g = (i64)b0 - 1 + (x - (nat + 2));
  *from_b = true;
  return (g >= 0 && (u64)g < nb) ? g : -1;
}

constexpr int SLOTS = (JS + JB - 1) / JB;

__device__ __forceinline__ Row lds_row(const Buf& s, int x) {
  typedef u64 v2u64 __attribute__((ext_vector_type(2)));
  const v2u64 kv = *(const v2u64*)s.kv[x];
  const v2u64 tc = *(const v2u64*)s.tc[x];
  Row r;
  r.key = kv.x;
  r.val = kv.y;
  r.ts = (i64)tc.x;
  r.cnt = tc.y;
  r.node = s.node[x];
  return r;
}

// Highest power of two <= JT: the first step of the binary-lifting search.
constexpr int search_top(int n) { return n <= 1 ? 1 : 2 * search_top(n / 2); }
constexpr int STOP = search_top(JT);

// Merge JI consecutive positions of the tile and decide keep/drop for each (the body
// of join_dot_sets/4 per row, see the file header).  Branch-free where it matters:
// the key search runs a fixed number of binary-lifting steps and each merge step
// selects between the a and b candidates instead of branching (divergent branches
// cost exec-mask SALU work on every path).
// CHG: also set bit k of `ev` when item k changes its key's rows (diff/3 of
// causal_crdt.ex:343-351 over `keys`): a dropped a row or a newly kept b row.
// FAST: both contexts are version vectors (LDS counter tables); KEYED: a `keys` list.
template <bool FAST, bool KEYED, bool CHG = false, bool NOFB = false>
__device__ __forceinline__ void merge_items(const Ctx& ca, const Ctx& cb, const u64* tab_a,
                                            const u64* tab_b, const KeySlice& ks,
                                            const u64 nb, const Buf& s, int nat, int nbt, u64 a0,
                                            u64 b0, u32& keep, unsigned short (&src)[JI],
                                            u32* ev = nullptr) {
  const int tid = threadIdx.x;
  const int offB = nat + 2;
  const int tt = nat + nbt;
  const int diag = min(tid * JI, tt);
  const int dend = min(diag + JI, tt);
  // Merge-path split of this thread's diagonal: first i with NOT(a[i] <= b[diag-1-i]).
  // (1) key-only: iq = first i in [lo0, hi0] with a[i].key > b[diag-1-i].key, by binary
  //     lifting (lo grows while a[m-1].key <= b[diag-m].key); slot of a[x] is 1 + x,
  //     of b[y] is offB + 1 + y.
  const int lo0 = diag > nbt ? diag - nbt : 0, hi0 = min(diag, nat);
  int lo = lo0;
#pragma unroll
  for (int step = STOP; step >= 1; step >>= 1) {
    // (both reads unconditional at a clamped index, combined bitwise: no exec-mask branch)
    const int m = lo + step;
    const int mc = min(m, hi0);
    const bool c = (m <= hi0) & (buf_key(s, mc) <= buf_key(s, offB + 1 + diag - mc));
    lo = c ? m : lo;
  }
  // (2) P(i) implies key <=, so the split is <= iq; step down while the full tuples of
  //     a[i-1] and b[diag-i] (equal keys) say a > b.  Runs of tied keys are short, and
  //     distinct keys (the common case) settle on the key columns alone.
  int i = lo;
  while (i > lo0 && buf_key(s, i) == buf_key(s, offB + 1 + diag - i)) {
    bool lt, eq;
    row_cmp_bf(lds_row(s, i), lds_row(s, offB + 1 + diag - i), lt, eq);
    if (lt | eq) break;
    i--;
  }
  int j = diag - i;
  // ra = a[i], rb = b[j] (possibly the neighbour past the tile); xa / xb are the rows
  // after them, read one step ahead so no merge step waits on LDS.  (Reads past a side's
  // end land in other slots of the buffer and are never used.)  dup: the current b row
  // equals the last a row merged before it -- ties go to a, so an a row and its equal b
  // row are adjacent and the b row is the MapSet duplicate.
  // (dup reads the last a row's key first and the whole row only under an equal key: the
  // merge is bound by its LDS reads, and in a join of replicas that hold the same keys the
  // row before a thread's first b row has another key -- config 2 36.9-37.1 against
  // 38.1-38.9 us per join, config 5 343-346 against 341 us, A/B)
  Row ra = lds_row(s, 1 + i), rb = lds_row(s, offB + 1 + j);
  bool dup = false;
  if (((a0 + (u64)i) >= 1) && buf_key(s, i) == rb.key) dup = row_eq(lds_row(s, i), rb);
  Row xa = lds_row(s, 2 + i), xb = lds_row(s, offB + 2 + j);
  keep = 0;
  if (CHG) *ev = 0;
#pragma unroll
  for (int k = 0; k < JI; k++) {
    const bool valid = diag + k < dend;
    const bool bvalid = (b0 + (u64)j) < nb;  // b[j] exists globally
    bool lt, eq;
    row_cmp_bf(ra, rb, lt, eq);
    const bool takeA = (i < nat) & ((j >= nbt) | lt | eq);
    const bool inB = bvalid & eq;
    bool kp;
    // the key is joined (in `keys`), not carried right-biased
    const bool jn = KEYED ? key_in(ks, takeA ? ra.key : rb.key) : true;
    if (FAST) {
      // Dots.member?(c_other, dot of the taken row): one LDS table read
      const u32 dn = takeA ? ra.node : rb.node;
      const u64 dc = takeA ? ra.cnt : rb.cnt;
      // (the other side's VV by field VALUES: a select between the two Ctx structs
      // would make them addressable and spill them to scratch)
      bool cov;
      if (dn < (u32)VT) {
        cov = (takeA ? tab_b : tab_a)[dn] >= dc;
      } else if (NOFB) {
        cov = dc == 0;  // no VV has an entry >= VT: Map.get(vv, dn, 0) = 0
      } else {
        const u32* vn = takeA ? opaque_ptr(cb.node) : opaque_ptr(ca.node);
        const u64* vc = takeA ? opaque_ptr(cb.cnt) : opaque_ptr(ca.cnt);
        const u64 vnn = takeA ? opaque_val(cb.n) : opaque_val(ca.n);
        cov = ctx_covers(vn, vc, vnn, 0, dn, dc);
      }
      if (KEYED) {
        // Map.merge(Map.drop(a), Map.drop(b)) for keys outside `keys`: a's rows survive
        // iff b lacks the key, b's rows always
        const bool bprev = ((b0 + (u64)j) >= 1) & (buf_key(s, offB + j) == ra.key);
        const bool bnext = bvalid & (rb.key == ra.key);
        kp = takeA ? (jn ? (inB | !cov) : !(bprev | bnext)) : (!jn | (!dup & !cov));
      } else {
        kp = takeA ? (inB || !cov) : (!dup && !cov);
      }
    } else if (takeA) {
      if (jn) {
        kp = inB || !covers<FAST>(tab_b, cb, ra.node, ra.cnt);
      } else {
        // Map.merge(Map.drop(a), Map.drop(b)): a's rows survive iff b lacks the key
        const bool bprev = (b0 + (u64)j) >= 1 && buf_key(s, offB + j) == ra.key;
        const bool bnext = bvalid && rb.key == ra.key;
        kp = !(bprev || bnext);
      }
    } else {
      if (jn)
        kp = !dup && !covers<FAST>(tab_a, ca, rb.node, rb.cnt);
      else
        kp = true;
    }
    src[k] = valid ? (unsigned short)(takeA ? 1 + i : offB + 1 + j) : (unsigned short)0;
    if (valid && kp) keep |= 1u << k;
    if (CHG && valid && jn && (takeA ? !kp : kp)) *ev |= 1u << k;
    // advance the taken side; the next row after it is read one step ahead
    // (b rows are unique and larger than every a row merged so far, so a taken b row
    // clears dup; a taken a row passes its inB on to the b row it tied with)
    dup = takeA ? inB : false;
    i += takeA ? 1 : 0;
    j += takeA ? 0 : 1;
    ra = row_sel(takeA, xa, ra);
    rb = row_sel(takeA, rb, xb);
    if (k + 1 < JI) {
      const Row nx = lds_row(s, takeA ? 2 + i : offB + 2 + j);
      xa = row_sel(takeA, nx, xa);
      xb = row_sel(takeA, xb, nx);
    }
  }
}

// LDS of one join workgroup.  The VV tables are only read by the merge and the
// compaction list is only written after it (behind the block scan's barriers), so
// they share storage: the tile stays at 4 workgroups per CU.
struct TileLds {
  Buf buf;
  union {
    u64 tab[2][VT];
    unsigned short comp[JT];
  } u;
  u32 wave[JB / WAVE + 1];
  u64 lb[3 * (JB / WAVE) + 2];
  u64 bcast[4];
};

// Register staging of a tile: every lane issues the loads of all its slots (issue_tile)
// long before it writes them to LDS (commit_tile), so a whole tile streams in while the
// previous one is merged.
struct Staged {  // one thread's share of a staged tile, in registers
  u64 k[SLOTS], v[SLOTS], c[SLOTS];
  i64 t[SLOTS];
  u32 n[SLOTS];
  bool ok[SLOTS];
};

__device__ __forceinline__ void tile_geom(u64 t, u64 jt, u64 a0, u64 a1, u64 total, int* nat,
                                          int* nbt, u64* b0) {
  const u64 d0 = t * jt, d1 = min(d0 + jt, total);
  *nat = (int)(a1 - a0);
  *nbt = (int)((d1 - a1) - (d0 - a0));
  *b0 = d0 - a0;
}

__device__ __forceinline__ void issue_tile(const Rows& A, const Rows& B, int nat, int nbt, u64 a0,
                                           u64 b0, Staged& r) {
  const int tid = threadIdx.x;
#pragma unroll
  for (int k = 0; k < SLOTS; k++) {
    const int x = tid + k * JB;
    bool fb = false;
    const i64 g = x < nat + nbt + 4 ? slot_row(x, nat, a0, b0, A.n, B.n, &fb) : -1;
    r.ok[k] = g >= 0;
    if (r.ok[k]) {
      const Row x = load_row_sel(A, B, fb, (u64)g);
      r.k[k] = x.key;
      r.v[k] = x.val;
      r.t[k] = x.ts;
      r.n[k] = x.node;
      r.c[k] = x.cnt;
    }
  }
}

__device__ __forceinline__ void commit_tile(const Staged& r, Buf& s) {
  const int tid = threadIdx.x;
#pragma unroll
  for (int k = 0; k < SLOTS; k++) {
    const int x = tid + k * JB;
    if (r.ok[k]) buf_put(s, x, r.k[k], r.v[k], r.t[k], r.n[k], r.c[k]);
  }
}

// ------------------------------------------------------------- single-pass join
// join2_stream_kernel: persistent workgroups (the whole grid is co-resident: it is
// sized from the occupancy query); workgroup w merges tiles w, w + G, w + 2G, ...
// so iteration k of every workgroup together covers the stripe of tiles [kG, (k+1)G).
// Two LDS tile buffers alternate.  Iteration k of workgroup w (tile t = w + kG):
//   1. commit tile t's rows (prefetched into registers) to buffer k%2;
//   2. issue the loads of tile t + G into registers, and the loads of stripe k-1's
//      G tile counts (they stream during the merge);
//   3. merge tile t, block-scan its keep bits: count n_t and compaction list;
//      publish n_t (an epoch-tagged 32-bit granule, written once);
//   4. offsets of stripe k-1, computed redundantly by every workgroup from its G
//      counts: tile (w + (k-1)G) starts at base_{k-1} + Σ_{w' < w} n, and
//      base_k = base_{k-1} + Σ_{all w'} n;
//   5. write tile t - G's kept rows (still in buffer (k-1)%2), coalesced, at that
//      offset.
// No look-back chain and no ticket: a stripe's counts were all published one merge
// earlier, so step 4 rarely waits; its cost is one G-word read per iteration, issued
// before the merge.  Spins stay bounded (scan.err bit 0 on timeout).
constexpr int FUSE_IT = 4;  // fused: tiles per workgroup whose splits the kernel searches itself
// (stripe_sums' partials are double-buffered by iteration parity, which drops the barrier
// a single buffer needs before its writes: measured neutral, config 5 356-360 vs 358-360 us
// and config 2 34.5-35.4 vs 34.6-34.7 us, rocprofv3 on one box; kept, one barrier fewer)

template <bool KEYED>
struct StreamLds {
  Buf buf[2];
  unsigned short comp[2][JT];
  u64 tab[2][VT];
  u64 kslice[2][KEYED ? KS : 1];    // keyed: the tile's keyset slice (<= KS entries)
  u64 kspl[KEYED ? 2 * FUSE_IT : 1];  // keyed + fused: keyset splits of this workgroup's tiles
  u32 wave[JB / WAVE + 1];
  u64 red[2][2 * (JB / WAVE)];  // stripe_sums' wave partials, double-buffered by iteration parity
  u64 spl[2 * FUSE_IT];  // fused: splits of this workgroup's tiles (start, end per tile)
  u64 chk[JB / WAVE];    // CHG: each wave's last change event, and 1 + its lane (0: none)
  int chf[JB / WAVE];
};

constexpr u32 CNT_BITS = 12;  // count field of a tile-count granule (JT < 4096)
static_assert(JT < (1 << CNT_BITS), "tile count must fit the granule's count field");
constexpr int CQ = (1024 + JB - 1) / JB;  // stripe counts per thread (grid <= CQ * JB)
static_assert((u64)CQ * JB + 1 <= JOIN_MAX_GRID, "start flags cover every join grid");

__device__ __forceinline__ void publish_count(u32* cs, u64 t, u32 epoch, u32 n) {
  __hip_atomic_store(cs + t, (epoch << CNT_BITS) | n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Stripe counts of tiles [base_t, base_t + G) ∩ [0, ntiles), CQ per thread: issued
// early (stripe_load), consumed after the merge (stripe_sums), which re-polls the ones
// not yet published and returns (Σ over workgroups w' < w, Σ over all).
struct StripeCounts {
  u32 v[CQ];
  bool ready;
};

__device__ __forceinline__ void stripe_load(const u32* cs, u64 base_t, u64 G, u64 ntiles, u32 epoch,
                                            StripeCounts& c) {
  c.ready = true;
#pragma unroll
  for (int q = 0; q < CQ; q++) {
    const u64 x = (u64)threadIdx.x + (u64)q * JB;  // workgroup index within the stripe
    c.v[q] = epoch << CNT_BITS;                     // absent tiles count 0
    if (x < G && base_t + x < ntiles)
      c.v[q] = __hip_atomic_load(cs + base_t + x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// Waiting is safe only while the whole grid is resident.  Polls that go on for long
// check the start flags of the workgroups waited on: one that has started stays
// resident until it finishes, so the wait ends; one that has not (another stream's or
// process's kernels hold the CUs) makes the waiter raise the abort flag after
// ABORT_POLLS, and the grid runs on without waiting (err bit 2; the caller re-runs the
// join on the two-pass kernels).  Each workgroup stores its start flag once: no
// contended counter at launch.
constexpr u32 ABORT_POLLS = 1u << 13;

// The check's own arguments are read from the kernel-argument segment where they are
// used (volatile: not hoisted), so they hold no registers across the tile loop.
template <class T>
__device__ __forceinline__ T cold(const T* field) {
  return *(const volatile T*)field;
}

__device__ __forceinline__ const Scan* cold_scan() {
  return &((const JoinArgs*)__builtin_amdgcn_kernarg_segment_ptr())->scan;
}

// Whether this thread stops waiting: the grid has aborted, or (after ABORT_POLLS) a
// workgroup whose count it still lacks has not started.
__device__ __forceinline__ bool grid_check(u32 epoch, u32 spins, u64 need, const StripeCounts& c) {
  const Scan* sc = cold_scan();
  u32* abort = cold(&sc->abort);
  if (__hip_atomic_load(abort, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == epoch) return true;
  if (spins <= ABORT_POLLS) return false;
  const u32* started = cold(&sc->started);
  bool absent = false;
#pragma unroll
  for (int q = 0; q < CQ; q++) {
    const u64 x = (u64)threadIdx.x + (u64)q * JB;
    if (x < need && (c.v[q] >> CNT_BITS) != epoch &&
        __hip_atomic_load(started + x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != epoch)
      absent = true;
  }
  if (!absent) return false;
  __hip_atomic_store(abort, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  atomicOr(cold(&sc->err), 2u);
  return true;
}

// After an abort the counts not yet published read as 0, so the rest of the grid runs
// through its tiles without waiting and writes stay inside the output (whose rows the
// caller discards).
__device__ __forceinline__ void stripe_sums(const u32* cs, u32 epoch, u32* err, u64 base_t,
                                            u64 G, u64 w, bool need_all, StripeCounts& c,
                                            u64* s_red, u64* below, u64* all) {
  const int tid = threadIdx.x;
  // counts this workgroup needs: all of the stripe's (for the next stripe's base), or
  // only those of the workgroups below it (its last tile: no next stripe)
  const u64 need = need_all ? G : w;
  for (u32 spins = 0;; spins++) {  // (rare) wait for counts not yet published
    bool ready = true;
#pragma unroll
    for (int q = 0; q < CQ; q++)
      ready &= (u64)tid + (u64)q * JB >= need || (c.v[q] >> CNT_BITS) == epoch;
    if (ready) break;
    if ((spins & 63) == 63 && grid_check(epoch, spins, need, c)) {
#pragma unroll
      for (int q = 0; q < CQ; q++)
        if ((c.v[q] >> CNT_BITS) != epoch) c.v[q] = epoch << CNT_BITS;
      break;
    }
    if (spins > (1u << 24)) {  // unreachable on a co-resident grid
      atomicOr(err, 1u);
      break;
    }
    __builtin_amdgcn_s_sleep(2);
#pragma unroll
    for (int q = 0; q < CQ; q++) {
      const u64 x = (u64)tid + (u64)q * JB;
      if (x < need && (c.v[q] >> CNT_BITS) != epoch)
        c.v[q] = __hip_atomic_load(cs + base_t + x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  u64 lo = 0, tot = 0;
#pragma unroll
  for (int q = 0; q < CQ; q++) {
    const u64 x = (u64)tid + (u64)q * JB;
    const u64 n = c.v[q] & ((1u << CNT_BITS) - 1);
    tot += n;
    lo += x < w ? n : 0;
  }
  // (a wave's sums of <= 2 x 64 twelve-bit counts fit 32 bits: DPP reductions)
  lo = wave_sum_u32((u32)lo);
  tot = wave_sum_u32((u32)tot);
  constexpr int NW = JB / WAVE;
  // (no barrier before the writes: the caller alternates two s_red buffers by iteration
  // parity, and the previous reader of this buffer finished two iterations ago, behind the
  // iterations' own barriers)
  if ((tid & (WAVE - 1)) == 0) {
    s_red[tid / WAVE] = lo;
    s_red[NW + tid / WAVE] = tot;
  }
  __syncthreads();
  lo = 0;
  tot = 0;
#pragma unroll
  for (int i = 0; i < NW; i++) {
    lo += s_red[i];
    tot += s_red[NW + i];
  }
  *below = lo;
  *all = tot;
}

template <bool KEYED>
__device__ __forceinline__ void write_tile(const JoinArgs& p, const StreamLds<KEYED>& s, int bi,
                                           u64 o0, u32 n) {
  const Buf& b = s.buf[bi];
  for (u32 q = threadIdx.x; q < n; q += JB) {
    const Row x = lds_row(b, s.comp[bi][q]);
    store_row_nt(p.out, o0 + q, x);
  }
}

template <bool FAST, bool KEYED, bool CHG, bool LATE>
__global__ __launch_bounds__(JB) __attribute__((amdgpu_waves_per_eu(4, 8))) void join2_stream_kernel(JoinArgs p) {
  __shared__ StreamLds<KEYED> s;
  const int tid = threadIdx.x;
  const u64 total = p.a.n + p.b.n, ntiles = p.ntiles, w = blockIdx.x;
  const u64 G = gridDim.x - (LATE ? 1 : 0);  // tile workgroups
  u32* cs = p.scan.counts;  // tile-count granules
  const u32 epoch = p.scan.epoch;
  const Rows& A = p.a;
  const Rows& B = p.b;
  if (tid == 0)  // residency check (stripe_sums)
    __hip_atomic_store(cold(&cold_scan()->started) + w, epoch, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  if (w < G) JSTAMP(w, 0);  // (stamps build: slot 0 of a workgroup's first tile = its entry)
  Staged r;
  u64 ga0 = 0, ga1 = 0;  // fused: the first tile's speculative splits
  if (LATE) {
    if (w == G) {  // Dots.union(c1, c2) (aw_lww_map.ex:155), beside the tiles
      ctx_union_block<JB>(p.cu, s.wave);
      return;
    }
    // The first tile's loads go out at the proportional splits d * na / (na + nb) BEFORE
    // the exact search: replicas that hold the same keys (config 2) split exactly there,
    // so the tile streams in during the search (checked below; re-issued otherwise).
    {
      ga0 = split_guess(A.n, B.n, w * p.jt);
      ga1 = split_guess(A.n, B.n, min((w + 1) * p.jt, total));
      int gnat, gnbt;
      u64 gb0;
      tile_geom(w, p.jt, ga0, ga1, total, &gnat, &gnbt, &gb0);
      issue_tile(A, B, gnat, gnbt, ga0, gb0, r);
    }
    // merge-path splits of this workgroup's (<= FUSE_IT) tiles: boundary q (tile q / 2,
    // side q % 2) by wave q mod the block's waves
    for (int q = tid / WAVE; q < 2 * FUSE_IT; q += JB / WAVE) {  // (wave-uniform)
      const u64 tk = w + (u64)(q >> 1) * G;
      if (tk >= ntiles) break;
      const u64 d = min((tk + (q & 1)) * p.jt, total);
      // the proportional split is checked first with scalar loads (a counter the tile
      // loads in flight do not hold up); the search runs only where it is not exact
      const u64 g = split_guess(A.n, B.n, d);
      const u64 sp = guess_exact(A, B, d, g) ? g : mp_split(A, B, d);
      if ((tid & (WAVE - 1)) == 0) s.spl[q] = sp;
      if (KEYED) {
        const u64 kq = key_split(A, B, p.keys, p.n_keys, d, sp);
        if ((tid & (WAVE - 1)) == 0) s.kspl[q] = kq;
      }
    }
  }
  if (FAST)
    for (int x = tid; x < 2 * VT; x += JB) (&s.tab[0][0])[x] = 0;
  if (LATE) __syncthreads();
  if (w < G) JSTAMP(w, 8);  // (stamps build: splits searched)
  // split of boundary `side` (0 start, 1 end) of the tile of iteration k.  The fused
  // launch is exactly the LATE kernel, so the choice between the LDS copy and the
  // partition's array is made at compile time: a run-time flag let the compiler merge the
  // two reads into one flat load, whose wait (vmcnt 0) drained the previous tile's output
  // stores on every iteration (A/B: config 5 0.375-0.379 vs 0.381-0.388 ms per join, config 2
  // 33-35 vs 34-36 us)
  auto split = [&](u64 tile, int k, int side) -> u64 {
    if (LATE) return s.spl[2 * k + side];
    return p.splits[tile + side];
  };
  // keyed: the keyset slice [kl, kl + km) of the tile of iteration k; its entries are
  // staged with the tile's rows (one per lane) when km <= KS
  auto kslice = [&](u64 tile, int k, u64* kl) -> u64 {
    u64 lo, hi;
    if (LATE) {
      lo = s.kspl[2 * k];
      hi = s.kspl[2 * k + 1];
    } else {
      lo = p.ksplits[tile];
      hi = p.ksplits[tile + 1];
    }
    *kl = lo;
    return min(hi + 1, p.n_keys) - lo;
  };
  u64 t = w;
  u64 a0 = split(t, 0, 0), a1 = split(t, 0, 1);
  int nat, nbt;
  u64 b0;
  tile_geom(t, p.jt, a0, a1, total, &nat, &nbt, &b0);
  if (!LATE || a0 != ga0 || a1 != ga1) issue_tile(A, B, nat, nbt, a0, b0, r);  // (uniform)
  u64 kl = 0, km = 0, kk = 0;
  if (KEYED) {
    km = kslice(t, 0, &kl);
    if (km <= (u64)KS && (u64)tid < km) kk = p.keys[kl + tid];
  }
  __syncthreads();  // zeroed tables visible
  if (w < G) JSTAMP(w, 9);  // (stamps build: first tile's loads issued)
  bool vv_far = false;
  if (FAST) {
    vv_far = fill_vv_tables(p.ca, p.cb, s.tab[0], s.tab[1]);  // once per workgroup
    if (LATE) vv_far = __syncthreads_or(vv_far);
  }
  u64 base = 0;  // output offset of the first tile of the current stripe
  u32 np = 0;    // kept rows of this workgroup's tile of the previous stripe
  for (int k = 0;; k++) {
    const int bi = k & 1;
    if (k > 0) JSTAMP(t, 0);
    JSTAMP(t, 1);
    commit_tile(r, s.buf[bi]);
    if (KEYED && km <= (u64)KS && (u64)tid < km) s.kslice[bi][tid] = kk;
    __syncthreads();
    JSTAMP(t, 2);
    const u64 tn = t + G;
    u64 a0n = 0, a1n = 0, b0n = 0, kln = 0, kmn = 0;
    int natn = 0, nbtn = 0;
    // the next tile's loads: issued before the merge, so they land while it runs.  (Until
    // round 6 the fused kernel issued them after its merge, measured faster then, 39 vs 42 us;
    // since the fused merge has no flat loads left (NOFB below) the early issue wins there
    // too: config 2 34.1-35.2 against 36.1-37.2 us per join, A/B on one box, three rounds.)
    auto issue_next = [&]() {
      a0n = split(tn, k + 1, 0);
      a1n = split(tn, k + 1, 1);
      tile_geom(tn, p.jt, a0n, a1n, total, &natn, &nbtn, &b0n);
      issue_tile(A, B, natn, nbtn, a0n, b0n, r);
      if (KEYED) {
        kmn = kslice(tn, k + 1, &kln);
        if (kmn <= (u64)KS && (u64)tid < kmn) kk = p.keys[kln + tid];
      }
    };
    if (tn < ntiles) issue_next();
    StripeCounts sc;  // stripe k-1's counts, in flight during the merge
    if (k > 0) stripe_load(cs, t - G - w, G, ntiles, epoch, sc);
    JSTAMP(t, 7);
    u32 keep, ev = 0;
    unsigned short src[JI];
    const KeySlice ks{KEYED && km <= (u64)KS ? s.kslice[bi] : nullptr, p.keys + kl, km};
    // (fused joins whose VVs have no entry beyond the LDS tables -- every real replica set:
    // the merge without the global-memory coverage search, whose flat loads made each of
    // the merge's LDS waits also wait for the stripe counts in flight; config 2 35.7-37.5
    // against 36.3-39.6 us per join over three A/B sessions.  The partitioned kernel keeps
    // one merge: its copy without the search measured slower, 375-377 vs 340-367 us)
    if (LATE && FAST && !vv_far)
      merge_items<FAST, KEYED, CHG, true>(p.ca, p.cb, s.tab[0], s.tab[1], ks, B.n, s.buf[bi], nat,
                                          nbt, a0, b0, keep, src, &ev);
    else
      merge_items<FAST, KEYED, CHG>(p.ca, p.cb, s.tab[0], s.tab[1], ks, B.n, s.buf[bi], nat, nbt, a0,
                                    b0, keep, src, &ev);
    JSTAMP(t, 3);
    u32 n;
    u32 pos = block_excl_scan1<JB>(__popc(keep), s.wave, &n);  // (barriers before s.wave's next use)
#pragma unroll
    for (int q = 0; q < JI; q++)
      if (keep & (1u << q)) s.comp[bi][pos++] = src[q];
    if (tid == 0) publish_count(cs, t, epoch, n);
    __syncthreads();
    if (CHG) {  // the tile's change events (keys, ascending, repeats allowed) -> chg_tmp,
                // with the per-tile figures the changed-key kernels need (chg_sum/write)
      const Buf& cb = s.buf[bi];
      const int ne = __popc(ev);
      u64 fkey = 0, lkey = 0;
      u32 diff = 0;  // own events after this thread's first that differ from their predecessor
      bool seen = false;
#pragma unroll
      for (int q = 0; q < JI; q++)
        if (ev & (1u << q)) {
          const u64 k = buf_key(cb, src[q]);
          if (seen && k != lkey) diff++;
          if (!seen) fkey = k;
          lkey = k;
          seen = true;
        }
      // the event before this thread's first: a max-scan of (lane + 1, last event) over
      // the wave's lanes with events, then the nearest earlier wave with events
      // (DPP max-scan of the lane tags, then one shuffle for the key of the lane found)
      const int lane = tid & (WAVE - 1), wv = tid / WAVE;
      const u32 mi = wave_incl_max(ne ? (u32)lane + 1 : 0u);  // last lane <= this with events, + 1
      const u32 mx = wave_prev(mi);                            // ... < this lane
      const u64 pk = __shfl(lkey, mx > 0 ? (int)mx - 1 : 0, WAVE);
      const u32 ml = (u32)__builtin_amdgcn_readlane((int)mi, WAVE - 1);  // the wave's last
      const u64 wk = __shfl(lkey, ml > 0 ? (int)ml - 1 : 0, WAVE);
      if (lane == WAVE - 1) {
        s.chf[wv] = (int)ml;
        s.chk[wv] = wk;
      }
      int pm = (int)mx;
      u64 pkey = pk;
      __syncthreads();
      if (pm == 0)
        for (int w2 = wv - 1; w2 >= 0; w2--)
          if (s.chf[w2] > 0) {
            pm = 1;
            pkey = s.chk[w2];
            break;
          }
      if (ne && pm > 0 && fkey != pkey) diff++;
      // one scan for both: events (low 16 bits) and differing events (high 16 bits)
      u32 tot2;
      const u32 sc2 = block_excl_scan1<JB>((diff << 16) | (u32)ne, s.wave, &tot2);
      const u32 n2 = tot2 & 0xffffu, p0 = sc2 & 0xffffu;
      u64* dst = p.chg_tmp + t * (u64)JT;
      u32 p2 = p0;
#pragma unroll
      for (int q = 0; q < JI; q++)
        if (ev & (1u << q)) dst[p2++] = buf_key(cb, src[q]);
      if (tid == 0) {
        p.chg_cnt[t] = n2;
        p.chg_wu[t] = tot2 >> 16;
      }
      if (ne && p0 == 0) p.chg_fk[t] = fkey;
      if (ne && p2 == n2) p.chg_lk[t] = lkey;
    }
    JSTAMP(t, 4);
    if (k > 0) {  // stripe k-1: this workgroup's tile t - G
      u64 below, all;
      stripe_sums(cs, epoch, p.scan.err, t - G - w, G, w, true, sc, s.red[k & 1], &below, &all);
      JSTAMP(t, 5);
      write_tile(p, s, bi ^ 1, base + below, np);
      base += all;
    }
    JSTAMP(t, 6);
    np = n;
    if (tn >= ntiles) {
      u64 below, all;
      StripeCounts last;
      stripe_load(cs, t - w, G, ntiles, epoch, last);
      stripe_sums(cs, epoch, p.scan.err, t - w, G, w, false, last, s.red[(k + 1) & 1], &below, &all);
      write_tile(p, s, bi, base + below, np);
      if (tid == 0 && t == ntiles - 1) p.d_count[0] = base + below + np;
      break;
    }
    t = tn;
    a0 = a0n;
    a1 = a1n;
    nat = natn;
    nbt = nbtn;
    b0 = b0n;
    kl = kln;
    km = kmn;
    __syncthreads();  // buffer bi^1 written out: free for the next commit
  }
}

// ---------------------------------------------------------------- changed keys
// The keys whose rows the join changed (CausalCrdt's diff/3 after every join,
// causal_crdt.ex:343-351, over `keys`), ascending and unique, from the stream
// kernel's per-tile change events (ascending; a key repeats when several of its rows
// changed, possibly across tiles).  An event is kept where it differs from the event
// before it: inside its tile, or -- for a tile's first event -- the last event of the
// nearest non-empty earlier tile.  Every input is complete when these kernels run (the
// stream kernel wrote them), so nothing waits on another workgroup:
//   join2_stream_kernel<_, _, CHG>  per tile: its events, their count, the events that
//                     differ from their in-tile predecessor, the first and last event
//   chg_sum_kernel    per chunk of CCH tiles: the chunk's summary (below)
//   chg_write_kernel  per CWT tiles: its offset from the chunk summaries before it and the
//                     tiles of its own chunk before it, then one wave per tile writes the
//                     tile's kept events
// A summary of a run of tiles: the unique events the run would hold on its own, whether
// it has events, its first and last event.  Summaries combine associatively (the right
// run's first event repeats the left run's last one, or not), so any prefix is a
// reduction of a few of them.
constexpr int CCH = WAVE;  // tiles per chunk summary (one wave's)
constexpr int CB2 = 256;   // threads of the changed-key kernels
constexpr int CWT = CB2 / WAVE;  // tiles per chg_write_kernel workgroup: one per wave
constexpr int CEV = (JT + WAVE - 1) / WAVE;  // events per lane of one tile

struct ChgSum {
  u64 u;    // unique events of the run on its own
  u64 has;  // the run has events
  u64 fk, lk;
};

__device__ __forceinline__ ChgSum chg_combine(const ChgSum& L, const ChgSum& R) {
  if (!L.has) return ChgSum{L.u + R.u, R.has, R.fk, R.lk};
  if (!R.has) return L;
  return ChgSum{L.u + R.u - (R.fk == L.lk ? 1ull : 0ull), 1ull, L.fk, R.lk};
}

struct ChgArgs {
  const u64* ev;   // JT events per tile
  const u32* cnt;  // events per tile
  const u32* wu;   // events after the first that differ from their predecessor
  const u64* fk;   // the tile's first and last event (written when it has any)
  const u64* lk;
  ChgSum* chunk;   // per chunk of CCH tiles
  u64 ntiles;
  u64* out;
  u64 cap;
  u64* d_count;
};

__device__ __forceinline__ ChgSum chg_tile(const ChgArgs& p, u64 t) {
  const u32 n = p.cnt[t];
  if (n == 0) return ChgSum{0, 0, 0, 0};
  return ChgSum{(u64)p.wu[t] + 1, 1, p.fk[t], p.lk[t]};
}

// Ordered reduction of one summary per thread (thread order = tile order) over the block:
// shuffles down within each wave (lane 0 ends with its wave's run), then the waves in
// order.  Every thread returns the block's summary.
__device__ __forceinline__ ChgSum shfl_down_sum(const ChgSum& x, int d) {
  return ChgSum{__shfl_down(x.u, d, WAVE), __shfl_down(x.has, d, WAVE), __shfl_down(x.fk, d, WAVE),
                __shfl_down(x.lk, d, WAVE)};
}

__device__ ChgSum chg_block_reduce(ChgSum x, ChgSum* s_red) {
  const int lane = threadIdx.x & (WAVE - 1), wv = threadIdx.x / WAVE;
#pragma unroll
  for (int d = 1; d < WAVE; d <<= 1) {
    const ChgSum y = shfl_down_sum(x, d);
    if (lane + d < WAVE) x = chg_combine(x, y);
  }
  if (lane == 0) s_red[wv] = x;
  __syncthreads();
  if (threadIdx.x == 0) {
    ChgSum r = s_red[0];
    for (int i = 1; i < CB2 / WAVE; i++) r = chg_combine(r, s_red[i]);
    s_red[CB2 / WAVE] = r;
  }
  __syncthreads();
  const ChgSum r = s_red[CB2 / WAVE];
  __syncthreads();
  return r;
}

// Summary of [t0, t1) (t1 - t0 <= WAVE) by one wave: one tile per lane, every lane
// returns it.
__device__ __forceinline__ ChgSum chg_wave_range(const ChgArgs& p, u64 t0, u64 t1) {
  const int lane = threadIdx.x & (WAVE - 1);
  const u64 t = t0 + lane;
  ChgSum x = t < t1 ? chg_tile(p, t) : ChgSum{0, 0, 0, 0};
#pragma unroll
  for (int d = 1; d < WAVE; d <<= 1) {
    const ChgSum y = shfl_down_sum(x, d);
    if (lane + d < WAVE) x = chg_combine(x, y);
  }
  return ChgSum{__shfl(x.u, 0, WAVE), __shfl(x.has, 0, WAVE), __shfl(x.fk, 0, WAVE),
                __shfl(x.lk, 0, WAVE)};  // lane 0's run, to every lane
}

// one wave per chunk of CCH tiles
__global__ __launch_bounds__(CB2) void chg_sum_kernel(ChgArgs p, u64 nchunk) {
  const u64 c = (u64)blockIdx.x * (CB2 / WAVE) + threadIdx.x / WAVE;
  if (c >= nchunk) return;  // (uniform per wave)
  const ChgSum r = chg_wave_range(p, c * CCH, min(c * CCH + CCH, p.ntiles));
  if ((threadIdx.x & (WAVE - 1)) == 0) p.chunk[c] = r;
}

__global__ __launch_bounds__(CB2) void chg_write_kernel(ChgArgs p) {
  __shared__ ChgSum s_red[CB2 / WAVE + 1];
  __shared__ ChgSum s_tile[CWT];
  __shared__ u64 s_off[CWT];
  __shared__ u32 s_dup[CWT];
  const int tid = threadIdx.x, lane = tid & (WAVE - 1), wv = tid / WAVE;
  const u64 t0 = (u64)blockIdx.x * CWT, chunk = t0 / CCH;
  // the prefix [0, t0): the chunk summaries before this chunk (CB2 at a time), then this
  // chunk's tiles before t0 (at most CCH - CWT of them)
  ChgSum acc{0, 0, 0, 0};
  for (u64 c0 = 0; c0 < chunk; c0 += CB2) {
    const ChgSum x = c0 + tid < chunk ? p.chunk[c0 + tid] : ChgSum{0, 0, 0, 0};
    acc = chg_combine(acc, chg_block_reduce(x, s_red));
  }
  // (wave 0: this chunk's tiles before t0; the block reduce's barriers above retired s_red)
  if (wv == 0) {
    const ChgSum in = chg_wave_range(p, chunk * CCH, t0);
    if (lane == 0) s_red[0] = chg_combine(acc, in);
  }
  if (tid < CWT) s_tile[tid] = t0 + tid < p.ntiles ? chg_tile(p, t0 + tid) : ChgSum{0, 0, 0, 0};
  __syncthreads();
  if (tid == 0) {  // this workgroup's tiles: offsets and first-event repeats, in order
    ChgSum run = s_red[0];
    for (int i = 0; i < CWT; i++) {
      const ChgSum x = s_tile[i];
      const bool dup = x.has && run.has && x.fk == run.lk;
      s_dup[i] = dup ? 1u : 0u;
      s_off[i] = run.u;
      run = chg_combine(run, x);
    }
    if (t0 + CWT >= p.ntiles) p.d_count[0] = run.u;  // the last workgroup: the total
  }
  __syncthreads();
  // one wave per tile: the tile's kept events at its offset (below cap)
  {
    const int i = wv;
    const u64 t = t0 + i;
    if (t >= p.ntiles) return;
    const u32 n = p.cnt[t];
    const u64* ev = p.ev + t * (u64)JT;
    u64 o = s_off[i];
    const bool dup0 = s_dup[i] != 0;
    for (u32 e0 = 0; e0 < n; e0 += WAVE) {
      const u32 e = e0 + lane;
      const u64 k = e < n ? ev[e] : 0;
      const bool keep = e < n && (e > 0 ? ev[e - 1] != k : !dup0);
      const u64 m = __ballot(keep);
      const u64 pos = o + __popcll(m & ((1ull << lane) - 1));
      if (keep && pos < p.cap) p.out[pos] = k;
      o += __popcll(m);
    }
  }
}

// ---------------------------------------------------------------- two-pass join
// Pass 1 (join2_slot_kernel): persistent workgroups, each merging tiles blockIdx.x,
// blockIdx.x + gridDim.x, ...  While tile t is merged from LDS, the rows of the next
// tile are already in flight into registers (issued right after t was committed to
// LDS), so HBM streams through the merge instead of stalling each tile on its own
// loads.  The VV tables are loaded once per workgroup and kept in registers.  Output
// per tile: its kept-row count and its compaction list (LDS slot numbers, u16).
// Pass 2 (join2_compact_kernel): each workgroup sums the counts before its tile and
// gathers the kept rows from a/b into the output.  No inter-workgroup dependency in
// either pass.
template <bool FAST, bool KEYED>
__global__ __launch_bounds__(JB) void join2_slot_kernel(JoinArgs p) {
  __shared__ TileLds s;
  const int tid = threadIdx.x;
  const u64 total = p.a.n + p.b.n;
  if (FAST)
    for (int x = tid; x < 2 * VT; x += JB) (&s.u.tab[0][0])[x] = 0;
  const u64 t = blockIdx.x;
  const u64 a0 = p.splits[t], a1 = p.splits[t + 1];
  int nat, nbt;
  u64 b0;
  tile_geom(t, p.jt, a0, a1, total, &nat, &nbt, &b0);
  Staged r;
  issue_tile(p.a, p.b, nat, nbt, a0, b0, r);
  __syncthreads();  // zeroed tables visible
  if (FAST) fill_vv_tables(p.ca, p.cb, s.u.tab[0], s.u.tab[1]);
  JSTAMP(t, 0);
  JSTAMP(t, 1);
  commit_tile(r, s.buf);
  __syncthreads();
  JSTAMP(t, 2);
  u32 keep;
  unsigned short src[JI];
  const KeySlice ks{nullptr, p.keys, p.n_keys};
  merge_items<FAST, KEYED>(p.ca, p.cb, s.u.tab[0], s.u.tab[1], ks, p.b.n, s.buf, nat, nbt, a0, b0,
                           keep, src);
  JSTAMP(t, 3);
  u32 n;
  u32 pos = block_excl_scan<JB>(__popc(keep), s.wave, &n);  // barriers: tables dead
#pragma unroll
  for (int q = 0; q < JI; q++)
    if (keep & (1u << q)) s.u.comp[pos++] = src[q];
  __syncthreads();
  JSTAMP(t, 4);
  JSTAMP(t, 5);
  if (tid == 0) p.counts[t] = n;
  for (u32 q = tid; q < n; q += JB) p.lists[t * JT + q] = s.u.comp[q];
  JSTAMP(t, 6);
}

constexpr int CPB = 256;
constexpr int CPU_ = 8;  // counts loaded per thread per batch in the compact prologue

__global__ __launch_bounds__(CPB) void join2_compact_kernel(Rows a, Rows b, const u64* splits,
                                                            const unsigned short* lists,
                                                            const u32* counts, u64 ntiles,
                                                            RowsOut out, u64* d_count) {
  __shared__ u32 s_wave[CPB / WAVE + 1];
  __shared__ u64 s_pre;
  const u64 tile = blockIdx.x;
  // Σ counts[0, tile): every load of a batch is issued before the first add
  u64 part = 0;
  for (u64 base = 0; base < tile; base += (u64)CPB * CPU_) {
    u32 v[CPU_];
#pragma unroll
    for (int k = 0; k < CPU_; k++) {
      const u64 i = base + (u64)k * CPB + threadIdx.x;
      v[k] = i < tile ? counts[i] : 0u;
    }
#pragma unroll
    for (int k = 0; k < CPU_; k++) part += v[k];
  }
#pragma unroll
  for (int d = WAVE / 2; d >= 1; d >>= 1) part += __shfl_xor(part, d, WAVE);
  if ((threadIdx.x & (WAVE - 1)) == 0) s_wave[threadIdx.x / WAVE] = (u32)part;
  __syncthreads();
  if (threadIdx.x == 0) {
    u64 acc = 0;
    for (int w = 0; w < CPB / WAVE; w++) acc += s_wave[w];
    s_pre = acc;
    if (tile == ntiles - 1) d_count[0] = acc + counts[tile];
  }
  __syncthreads();
  const u64 base = s_pre, n = counts[tile];
  const u64 a0 = splits[tile], a1 = splits[tile + 1];
  const u64 d0 = tile * JT;
  const int nat = (int)(a1 - a0);
  const u64 b0 = d0 - a0;
  for (u64 q = threadIdx.x; q < n; q += CPB) {
    const int x = lists[tile * JT + q];
    const bool fb = x >= nat + 2;
    const u64 g = fb ? b0 - 1 + (u64)(x - nat - 2) : a0 - 1 + (u64)x;
    const Row r = load_row_sel(a, b, fb, g);
    store_row_nt(out, base + q, r);
  }
}

}  // namespace

// Workgroups of kernel `k` (JB threads) resident at once on the current device: the
// grid of a persistent kernel whose workgroups wait on each other.
// Workgroups of kernel k resident on the current device at once.  Cached per (kernel,
// device): the occupancy query costs microseconds of host time on every launch otherwise.
static u64 resident_grid(const void* k) {
  struct Entry {
    const void* k;
    int dev;
    u64 n;
  };
  static Entry cache[32];
  static int used = 0;
  static std::mutex mu;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 256;
  {
    std::lock_guard<std::mutex> g(mu);
    for (int i = 0; i < used; i++)
      if (cache[i].k == k && cache[i].dev == dev) return cache[i].n;
  }
  int per_cu = 0, cus = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k, JB, 0) != hipSuccess || per_cu <= 0 ||
      cus <= 0)
    return 256;
  const u64 n = (u64)per_cu * (u64)cus;
  std::lock_guard<std::mutex> g(mu);
  if (used < 32) cache[used++] = {k, dev, n};
  return n;
}

// Launch of the persistent stream kernel.  Its workgroups wait on each other's tile
// counts, so the whole grid must be resident at once even while other kernels (another
// engine's join on another stream) compete for the CUs: a cooperative launch, which the
// runtime only dispatches as one co-resident grid (DG_JOIN_COOP=1; default: a plain
// launch).
static hipError_t launch_stream(void (*kern)(JoinArgs), u64 grid, JoinArgs& p, hipStream_t st) {
  static const bool coop = [] {
    const char* v = getenv("DG_JOIN_COOP");
    return v && v[0] == '1';
  }();
  if (!coop) {
    hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(JB), 0, st, p);
    return hipGetLastError();
  }
  void* args[] = {&p};
  return hipLaunchCooperativeKernel((const void*)kern, dim3((unsigned)grid), dim3(JB), args, 0, st);
}


// A stream grid of G workgroups runs ceil(ntiles / G) stripes, the last one partly
// idle (config 2: 1969 tiles of 1016 positions on 512 workgroups, the fourth stripe 433
// tiles).  The tiles are re-cut to jt = ceil(total / (stripes x G)) <= JT positions, so
// every stripe is full and each of them carries less: ntiles grows by less than G
// (join2_tiles_cap sizes the scratch).  Fused joins only (at most FUSE_IT stripes, so a
// part-idle last stripe is a large share): config 2 34.3-35.0 against 36.4-38.6 us per
// join (A/B, one box).  The long partitioned joins keep JT (config 5 measured 368-370
// against 340-344 us re-cut, one stripe in 44 being part idle), and so do the
// changed-keys joins, whose event scratch is laid out by join2_tiles.
static void balance_tiles(JoinArgs& p, u64 G) {
  const u64 total = p.a.n + p.b.n;
  if (G == 0 || p.ntiles <= G) return;
  const u64 k = (p.ntiles + G - 1) / G;
  // (even, as JT is: two replicas of the same keys merge in pairs, so an even diagonal is
  // split exactly by the proportional guess the fused kernel checks first -- odd tiles
  // sent half the boundaries to the search: 42.4 against 35.1 us at config 2)
  const u64 jt = std::min<u64>(((total + k * G - 1) / (k * G) + 1) & ~1ull, JT);
  p.jt = jt;
  p.ntiles = (total + jt - 1) / jt;
}

hipError_t launch_join2(const Rows& a, const Ctx& ca, const Rows& b, const Ctx& cb,
                        const u64* keys, u64 n_keys, const RowsOut& out, u32* out_ctx_node,
                        u64* out_ctx_cnt, void* ctx_tmp, void* pass_tmp, int mode,
                        const Scan& scan, int workers, u64* d_counts, hipStream_t st,
                        void* chg_tmp) {
  JoinArgs p;
  p.a = a;
  p.b = b;
  p.ca = ca;
  p.cb = cb;
  p.keys = keys;
  p.n_keys = n_keys;
  p.ntiles = join2_tiles(a.n, b.n);
  p.jt = JT;
  // scan.state: look-back granules first, then the splits, then the keyset splits (keyed
  // joins); set again when the tiles are re-cut (balance below)
  auto place_splits = [&]() {
    p.splits = scan.state + p.ntiles;
    p.ksplits = scan.state + 2 * p.ntiles + 1;
  };
  place_splits();
  const CtxUnionArgs cu = make_cu(ca, cb, out_ctx_node, out_ctx_cnt, d_counts + 1, ctx_tmp);
  p.out = out;
  p.scan = scan;
  p.d_count = d_counts;
  p.lists = nullptr;
  p.counts = nullptr;
  p.chg_tmp = chg_tmp ? (u64*)chg_tmp : nullptr;
  p.chg_cnt = p.chg_wu = nullptr;
  p.chg_fk = p.chg_lk = nullptr;
  if (chg_tmp) {
    const ChgLayout l = chg_layout(chg_tmp, p.ntiles);
    p.chg_cnt = l.cnt;
    p.chg_wu = l.wu;
    p.chg_fk = l.fk;
    p.chg_lk = l.lk;
  }
  if (p.ntiles == 0) {
    // no rows: only the context union runs
    hipError_t e = hipMemsetAsync(d_counts, 0, sizeof(u64), st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(ctx_union_kernel, dim3(1), dim3(CB), 0, st, cu);
    return hipGetLastError();
  }
  // two version vectors: LDS VV tables; a key list: per-tile keyset slices
  const bool fast = ca.kind == 0 && cb.kind == 0;
  const bool keyed = keys != nullptr;
  p.fused = 0;
  p.cu = cu;
  void (*const kerns[2][2][2][2])(JoinArgs) = {
      {{{join2_stream_kernel<false, false, false, false>, join2_stream_kernel<false, false, false, true>},
        {join2_stream_kernel<false, false, true, false>, join2_stream_kernel<false, false, true, true>}},
       {{join2_stream_kernel<false, true, false, false>, join2_stream_kernel<false, true, false, true>},
        {join2_stream_kernel<false, true, true, false>, join2_stream_kernel<false, true, true, true>}}},
      {{{join2_stream_kernel<true, false, false, false>, join2_stream_kernel<true, false, false, true>},
        {join2_stream_kernel<true, false, true, false>, join2_stream_kernel<true, false, true, true>}},
       {{join2_stream_kernel<true, true, false, false>, join2_stream_kernel<true, true, false, true>},
        {join2_stream_kernel<true, true, true, false>, join2_stream_kernel<true, true, true, true>}}}};
  auto kern = kerns[fast][keyed][chg_tmp != nullptr][0];
  auto kern_late = kerns[fast][keyed][chg_tmp != nullptr][1];  // the fused launch
  const bool stream = mode != JOIN_TWO_PASS || chg_tmp;
  u64 g = 0;
  if (stream) {
    g = workers > 0 ? (u64)workers : resident_grid((const void*)kern);
    g = std::min<u64>(std::min<u64>(p.ntiles, g), (u64)CQ * JB);  // stripe counts: CQ per thread
    // small joins (<= FUSE_IT tiles per workgroup): the splits are searched inside the
    // stream kernel and the context union runs in one extra co-resident workgroup, so
    // the partition launch (~5 us of mostly fixed cost) disappears
    static const bool no_fuse = [] {
      const char* v = getenv("DG_JOIN_FUSE");
      return v && v[0] == '0';
    }();
    const u64 gr = workers > 0 ? g + 1 : resident_grid((const void*)kern_late);
    const u64 gt = std::min<u64>(std::min<u64>(p.ntiles, gr - 1), (u64)CQ * JB);
    if (!no_fuse && gr >= 2 && p.ntiles <= (u64)FUSE_IT * gt) {
      if (!chg_tmp) balance_tiles(p, gt);
      place_splits();
      p.fused = 1;
      return launch_stream(kern_late, gt + 1, p, st);
    }
  }
  const u64 nb_part = (p.ntiles + 1 + (PB / WAVE) - 1) / (PB / WAVE);
  hipLaunchKernelGGL(join2_partition_kernel, dim3((unsigned)nb_part + 1), dim3(PB), 0, st, a, b,
                     p.ntiles, p.jt, scan.state + p.ntiles, cu, keys, n_keys, p.ksplits);
  if (!stream) {
    char* t = (char*)pass_tmp;
    p.counts = (u32*)t;
    t += ((p.ntiles * 4 + 255) / 256) * 256;
    p.lists = (unsigned short*)t;
    auto kern = fast ? (keyed ? join2_slot_kernel<true, true> : join2_slot_kernel<true, false>)
                     : (keyed ? join2_slot_kernel<false, true> : join2_slot_kernel<false, false>);
    hipLaunchKernelGGL(kern, dim3((unsigned)p.ntiles), dim3(JB), 0, st, p);
    hipLaunchKernelGGL(join2_compact_kernel, dim3((unsigned)p.ntiles), dim3(CPB), 0, st, a, b,
                       p.splits, p.lists, p.counts, p.ntiles, out, d_counts);
    return hipGetLastError();
  }
  return launch_stream(kern, g, p, st);
}

hipError_t launch_join2_changes(u64 na, u64 nb, void* chg_tmp, u64* out, u64 cap, u64* d_count,
                                hipStream_t st) {
  const u64 ntiles = join2_tiles(na, nb);
  if (ntiles == 0) return hipMemsetAsync(d_count, 0, sizeof(u64), st);
  const ChgLayout l = chg_layout(chg_tmp, ntiles);
  ChgArgs p;
  p.ev = l.ev;
  p.cnt = l.cnt;
  p.wu = l.wu;
  p.fk = l.fk;
  p.lk = l.lk;
  p.chunk = (ChgSum*)l.off;  // (ntiles / CCH + 1) x 32 B <= the ntiles x 8 B + slack region
  p.ntiles = ntiles;
  p.out = out;
  p.cap = cap;
  p.d_count = d_count;
  const u64 nchunk = (ntiles + CCH - 1) / CCH;
  if (nchunk > 1) {  // (the last chunk's summary is never read)
    const u64 nc = nchunk - 1;
    hipLaunchKernelGGL(chg_sum_kernel, dim3((unsigned)((nc + CB2 / WAVE - 1) / (CB2 / WAVE))),
                       dim3(CB2), 0, st, p, nc);
  }
  hipLaunchKernelGGL(chg_write_kernel, dim3((unsigned)((ntiles + CWT - 1) / CWT)), dim3(CB2), 0,
                     st, p);
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
  if (n > 65536 * 16) n = 65536 * 16;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_join_stamps), n * 8) == hipSuccess ? 0 : -3;
}
#endif

}  // namespace dg
