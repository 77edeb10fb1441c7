// dg_launch.h — host-side launchers exported by each kernel translation unit to the
// C-ABI layer (api.hip).  Plain structs only; no torch types anywhere in libdeltagpu.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dg_device.h"

namespace dg {

// Per-launch scratch for single-pass compaction kernels (decoupled look-back).
struct Scan {
  u64* state;   // one granule per tile (device)
  u32* ticket;  // tile ticket counter, left at 0 by every launch (device)
  u32* err;     // error bits (device): 1 = look-back timeout
  u32 epoch;    // granules of other epochs are ignored
  u32* counts;  // per-tile count granules {epoch:20 | count:12} of the single-pass join
                // (written only by that kernel, zeroed when allocated)
  // residency check of the persistent join grid: workgroup w stores the epoch to
  // started[w] (JOIN_MAX_GRID entries, device) at its start.  A workgroup that waits long
  // on the count of one that has not started sets *abort = epoch; the grid then runs on
  // without waiting and the caller re-runs the join on the two-pass kernels.
  u32* started;
  u32* abort;
};

constexpr u64 JOIN_MAX_GRID = 2048;  // >= every single-pass join grid (join.hip checks)

// ---- join.hip
#ifndef DG_JOIN_BLOCK
#define DG_JOIN_BLOCK 512
#endif
#ifndef DG_JOIN_ITEMS
#define DG_JOIN_ITEMS 2
#endif
constexpr int JOIN_BLOCK = DG_JOIN_BLOCK;  // threads per join tile (one wave per SIMD)
constexpr int JOIN_ITEMS = DG_JOIN_ITEMS;  // merged positions per thread
// merged positions per tile: JOIN_BLOCK * JOIN_ITEMS less 8, so the staged rows (tile +
// 2 neighbours per store + 1 look-ahead) fit JOIN_ITEMS register slots per thread
constexpr int JOIN_TILE = JOIN_BLOCK * JOIN_ITEMS - 8;

inline u64 join2_tiles(u64 na, u64 nb) { return (na + nb + JOIN_TILE - 1) / JOIN_TILE; }
// tiles of a join after launch_join2 re-cuts them to fill its grid's stripes (fewer than
// one more per workgroup): what the split and tile-count scratch is sized for
inline u64 join2_tiles_cap(u64 na, u64 nb) { return join2_tiles(na, nb) + JOIN_MAX_GRID; }
// join/3: a merge-path partition pass (its extra workgroup computes the context union,
// d_counts[1] = its size), then one workgroup per tile that merges it, resolves its
// output offset by decoupled look-back and writes its kept rows (d_counts[0] = output
// rows).  Uses scan.state[0, 2 * ntiles + 2).  JOIN_TWO_PASS replaces the look-back by
// a count/compact pass pair (pass_tmp: join2_pass_tmp_bytes) whose first pass runs
// `workers` persistent workgroups.
enum { JOIN_SINGLE_PASS = 0, JOIN_TWO_PASS = 1 };
hipError_t launch_join2(const Rows& a, const Ctx& ca, const Rows& b, const Ctx& cb,
                        const u64* keys, u64 n_keys, const RowsOut& out, u32* out_ctx_node,
                        u64* out_ctx_cnt, void* ctx_tmp, void* pass_tmp, int mode,
                        const Scan& scan, int workers, u64* d_counts, hipStream_t st,
                        void* chg_tmp = nullptr);
// Changed keys (dg_join2_changes): with chg_tmp (join2_changes_tmp_bytes) the join
// records per-tile change events (always the single-pass kernel); launch_join2_changes
// then drops repeats and compacts them into out[0, cap) (*d_count = changed keys).
// chg_tmp: JOIN_TILE u64 events + u64 offset + 3 u32 + first/last event (2 u64) per tile.
inline size_t join2_changes_tmp_bytes(u64 na, u64 nb) {
  const u64 t = join2_tiles(na, nb);
  return t * ((u64)JOIN_TILE * 8 + 8 + 12 + 16) + 8 + 256;
}
hipError_t launch_join2_changes(u64 na, u64 nb, void* chg_tmp, u64* out, u64 cap, u64* d_count,
                                hipStream_t st);
inline size_t join2_pass_tmp_bytes(u64 na, u64 nb) {
  const u64 t = join2_tiles(na, nb);
  return ((t * 4 + 255) / 256) * 256 + t * (u64)JOIN_TILE * 2 + 256;  // counts + slot lists
}
// Dots.union/2 of two contexts; out kind: DOTS iff both DOTS.  Writes |out| to *d_count.
// tmp: (a.n + b.n) u32 + (a.n + b.n) u64 + (a.n + b.n + 1) u32 of device scratch.
hipError_t launch_ctx_union(const Ctx& a, const Ctx& b, u32* out_node, u64* out_cnt,
                            u64* d_count, void* tmp, hipStream_t st);
inline size_t ctx_union_tmp_bytes(u64 na, u64 nb) {
  return (size_t)(na + nb) * 4 + (size_t)(na + nb) * 8 + (size_t)(na + nb + 1) * 4 + 64;
}

// ---- kfold.hip (dg_apply_deltas in one pass; see the file header)
#ifndef DG_KFOLD_BLOCK  // 1024 threads at <= 64 VGPRs: 2 buckets x 16 waves per CU
#define DG_KFOLD_BLOCK 1024  // (config 3: 2.08-2.33 vs 2.25-2.48 ms per call at 512, A/B)
#endif
#ifndef DG_KFOLD_SCALE  // bucket capacities and means are 1024 / 512 / 512 (640 / 320 / 320) >> this
#define DG_KFOLD_SCALE 0
#endif
constexpr int KFOLD_BLOCK = DG_KFOLD_BLOCK;
constexpr int KFOLD_CAP_S = 1024 >> DG_KFOLD_SCALE;  // LDS capacity per key bucket: state rows,
constexpr int KFOLD_CAP_D = 512 >> DG_KFOLD_SCALE;   //   delta rows,
constexpr int KFOLD_CAP_M = 512 >> DG_KFOLD_SCALE;   //   keyset entries
constexpr int KFOLD_MAX_K = 64;    // deltas per pass (delta masks are u64)
constexpr int KNT = 1024;          // VV tables cover node ids < KNT
constexpr u32 KF_PREP_FAIL = 1, KF_OVERFLOW = 2;
constexpr u64 KFOLD_FILL_SLICE = 2048;  // the fill cuts every delta run into slices of at most this
// mean fill per bucket the host sizes T for, each >= 5.5 sigma below its LDS capacity:
// state rows (cap 1024), delta rows (their payload slots: cap 512), keyset entries as
// staged (cap 1024: a thread stages two items) and all staged items (delta rows + keyset
// entries, cap 1536).  After the keyset fold (entries with rows of the key fold into
// them) at most 1024 items remain; a bucket over that re-runs the pass with 8x the
// buckets.  Config 3: 12.7k buckets (the delta rows bind), 14.7k when every keyset entry
// took an item slot of its own.
constexpr u64 KFOLD_MEAN_S = 800 >> DG_KFOLD_SCALE, KFOLD_MEAN_D = 400 >> DG_KFOLD_SCALE,
              KFOLD_MEAN_M = 800 >> DG_KFOLD_SCALE, KFOLD_MEAN_U = 1200 >> DG_KFOLD_SCALE;
struct KRun {  // delta i: its rows, keyset (keys == nullptr: every key) and context
  Rows rows;
  const u64* keys;
  u64 n_keys;
  Ctx ctx;
};
struct KFoldArgs {
  Rows s;              // the state
  Ctx c0;              // its context (a VV)
  const KRun* runs;    // k deltas (device array)
  int k;
  u64 allmask;         // bit i: delta i joins every key (keys_i == NULL)
  u64 T;               // key buckets
  u32 fill_p;          // slices per delta run in the fill: a multiple of 8 (kfold.hip)
  u64* sstart;         // T+1
  u32* dstart;         // (T+1) x 2k
  u64* tabC;           // k x KNT: c_i
  u64* tabP;           // k x KNT: the state's context before delta i
  RowsOut out;
  u32* out_ctx_node;
  u64* out_ctx_cnt;
  Scan scan;
  u64* d_counts;       // [0] output rows, [1] output context entries
  u32* flag;           // KF_* bits: the caller must re-run the fold step by step
  // dot-set contexts (MapSet deltas of add/remove, aw_lww_map.ex:124-146): bit i of
  // dotsmask = c_i is a dot set; its dots go to an open-addressing hash set of
  // (i, node, counter) keys (kfold_dset_kernel), so "c_i covers the dot" stays one
  // probe -- tabC[i] then holds c_i's per-node max, which is what Dots.union folds into
  // the VV prefix unions (aw_lww_map.ex:45-52)
  u64 dotsmask;
  u64* dset;           // dset_mask + 1 entries, KF_EMPTY when unused
  u64 dset_mask;
  const u64* cflat;    // k + 1: prefix sums of the dot-set contexts' sizes (VV: 0)
  u64 dset_n;          // their total (host copy of cflat[k])
};
constexpr u64 KF_EMPTY = ~0ull;
constexpr u64 KF_CNT_LIMIT = (1ull << 48) - 1;  // dot-set counters below this pack into a key
hipError_t launch_kfold(const KFoldArgs& p, hipStream_t st);

// ---- take.hip (sync-delta values: Map.take(value, keys))
#ifndef DG_TAKE_TILE
#define DG_TAKE_TILE 256  // 489 workgroups for 125k keys: 42.8 vs 50.0 us at 1024, 51 at 128 (A/B)
#endif
constexpr int TAKE_TILE = DG_TAKE_TILE;  // keys per take workgroup, one per thread
inline u64 take_tiles(u64 n_keys) { return (n_keys + TAKE_TILE - 1) / TAKE_TILE; }
// rows of s whose key is in keys (ascending) into out[0, cap); *d_count = their number.
// Uses look-back granules [0, take_tiles(n_keys)).  key_lo / key_off (optional, n_keys and
// n_keys + 1 entries): per key its first row in s (the first row >= the key) and the
// output offset of its rows (key_off[n_keys] = *d_count).
// pre_len (optional, with key_lo): the keys' rows located already (launch_splice_locate:
// key_lo[u] and pre_len[u] are inputs), so the kernel only scans and copies.
hipError_t launch_take_keys(const Rows& s, const u64* keys, u64 n_keys, const RowsOut& out,
                            u64 cap, const Scan& scan, u64* d_count, hipStream_t st,
                            u64* key_lo = nullptr, u64* key_off = nullptr,
                            const u32* pre_len = nullptr);

// ---- splice.hip (a sparse keyed join applied to a large state without merging it)
// The keyed join of a small delta into a large state, as a splice: the state's rows of the
// keyset K are taken out (launch_take_keys with the per-key index), joined with the delta
// (the join kernels on the small inputs: the edit E), and the output is the state with
// each key's rows replaced by E's, its untouched rows moved by a streaming copy.
struct SpliceArgs {
  Rows a;              // the state
  const u64* keys;     // K, ascending unique
  u64 nk;
  const u64* a_lo;     // nk: first row of A >= K[u]                        (take)
  const u64* a_off;    // nk + 1: rows of A with keys K[0..u)                (take)
  u64* end;            // nk: a_lo[u] + rows of K[u] in A                     (index)
  i64* shift;          // nk + 1: out - in of the A rows after K[u-1], before K[u] (index)
  i64* gap;            // nk: A rows outside K before K[u]                    (index)
  u64* tile_u0;        // a_tiles + 1: first u with end[u] > the tile's first row (index)
  u32* moved;          // (index) set when some shift is nonzero: rows outside K move
  Rows e;              // the edit (e.n: an upper bound; the count is *d_ne)
  const u64* d_ne;
  RowsOut out;
  u64 a_tiles, e_tiles;
  // (optional) an input-error word: when it has a MERKLE_INPUT_ERR bit set, E's rows are
  // not written (dg_join_delta's in-place copy runs after the tree update it depends on)
  const u32* guard;
  // (optional) the index and copy kernels run only when *run_if != 0 (the fused small
  // join enqueues the moved-rows copy before the host knows whether rows moved)
  const u64* run_if;
  // (optional) the copy kernels run only when *kguard == 0 (dg_join_delta's one-wait path:
  // its guard word says the index was not written)
  const u64* kguard;
  // (optional, launch_splice_move) the publish of the count block by the last workgroup
  u64* h_pub;
  const u64* pub_counts;
  u64 seq;
  u32* arrive_all;
};
// For every key of keys (ascending, n_keys): lo[u] = the first row of s whose key is >=
// keys[u] and len[u] = its rows, found by streaming s's key column in tiles (each tile's
// keys searched in the tile staged in LDS) instead of one search per key: cheaper than
// the searches once more than about 1 key in 150 rows is looked up.
hipError_t launch_splice_locate(const Rows& s, const u64* keys, u64 n_keys, u64* lo, u32* len,
                                hipStream_t st);
// every row of b whose key starts a run and is not in keys: *d_bad += 1
hipError_t launch_splice_check(const u64* bkey, u64 nb, const u64* keys, u64 nk, u64* d_bad,
                               hipStream_t st);
// the per-key index (end, shift, gap, tile_u0; *moved |= some shift != 0), then the copy:
// every state row outside K to its place and E's rows into the holes; e_only: E's rows
// alone (in place: out is the state itself and no shift is nonzero)
hipError_t launch_splice_index(SpliceArgs p, hipStream_t st);
hipError_t launch_splice_copy(SpliceArgs p, bool e_only, hipStream_t st);
// on[0, nc) = un, oc[0, nc) = uc (skipped when `guard` is non-null and holds a
// MERKLE_INPUT_ERR bit); dirty[0, n_dirty) = 0; counts[0, 8) = 0 (if non-null);
// *err_word = 0 (if non-null): one launch instead of two copies and three fills
hipError_t launch_splice_finish(const u32* un, const u64* uc, u64 nc, u32* on, u64* oc, u32* dirty,
                                u64 n_dirty, u64* counts, u32* err_word, hipStream_t st,
                                const u32* guard = nullptr);
u64 splice_tiles(u64 n);  // state tiles of the copy (tile_u0 holds one more entry)
constexpr u64 SPLICE_TILE = 2048;  // state rows per copy tile (splice.hip ST)
// the copy of the untouched rows alone (splice_kernel; E's rows placed by the caller); with
// p.h_pub the last workgroup publishes the count block (dg_home.h) when every one is done
hipError_t launch_splice_move(SpliceArgs p, hipStream_t st);

// ---- mutate.hip (a batch of add/remove ops as one delta; see the file header)
inline u64 mutate_tiles(u64 m) { return (m + 255) / 256; }  // (mutate.hip MT)
// count + scan (its last tile): d_counts[0..2] = touched keys, delta rows, state dots;
// scratch: 6 * mutate_tiles(m) u64; err bit 0: ops not sorted by key; arrive: a counter,
// zero on entry and left zero.
hipError_t launch_mutate_count(const Rows& s, const Ctx& c, u32 node, const uint8_t* kind,
                               const u64* key, const u64* val, const i64* ts, const u64* rank,
                               u64 m, u64* scratch, u64* d_counts, u32* err, u32* arrive,
                               hipStream_t st);
// keys_out, rows_out and the state dots into dnode/dcnt[0, n_state_dots)
hipError_t launch_mutate_write(const Rows& s, const Ctx& c, u32 node, const uint8_t* kind,
                               const u64* key, const u64* val, const i64* ts, const u64* rank,
                               u64 m, u64* scratch, u64* keys_out, const RowsOut& rows_out,
                               u32* dnode, u64* dcnt, u32* err, hipStream_t st);
size_t mutate_sort_tmp_bytes(u64 n);
// the adds' dots after the state dots, then the (node, counter) sort through t* into out_*
hipError_t launch_mutate_dots(const Ctx& c, u32 node, u64 n_adds, u64 n_state_dots, u32* dnode,
                              u64* dcnt, u32* tnode, u64* tcnt, void* sort_tmp,
                              size_t sort_tmp_bytes, u32* out_node, u64* out_cnt, hipStream_t st);

// ---- segred.hip (segmented reductions over key runs)
constexpr int SEG_BLOCK = 256;
constexpr int SEG_ITEMS = 4;
constexpr int SEG_TILE = SEG_BLOCK * SEG_ITEMS;
inline u64 seg_tiles(u64 n) { return (n + SEG_TILE - 1) / SEG_TILE; }
// scratch: 2 * seg_tiles(n) u64 (per-tile counts and offsets).
hipError_t launch_read_lww(const Rows& s, const u64* keys, u64 n_keys, u64* out_key, u64* out_val,
                           u64* scratch, u64* d_count, hipStream_t st);
// Sortedness check: sets *d_bad to nonzero if rows are not strictly ascending.
hipError_t launch_store_check(const Rows& s, u32* d_bad, hipStream_t st);

// ---- sort.hip (rows and contexts marshalled in map order -> the sorted forms)
struct SortField {  // one column of the sort tuple
  const void* p;
  int width;      // 4 (u32) or 8 (u64 / i64)
  int is_signed;  // i64: order by the sign-flipped bits
};
u64 sort_tiles(u64 n);
size_t sort_tmp_bytes(u64 n);
// rows sorted by (key, val, ts, node, cnt), exact duplicates dropped; *d_count = rows out.
// h_hist8: 8 KB of pinned host memory (a digit pass whose byte is constant is skipped,
// decided per field on the host: synchronizes once per field).
hipError_t launch_sort_store(const Rows& in, const RowsOut& out, void* tmp, u32* h_hist8,
                             u64* d_count, hipStream_t st);
// context entries sorted by node (kind 0, a VV) or (node, cnt) (kind 1, a dot set)
hipError_t launch_sort_context(int kind, const u32* node, const u64* cnt, u64 n, u32* out_node,
                               u64* out_cnt, void* tmp, u32* h_hist8, hipStream_t st);

// ---- remap.hip (value ids after a host relabel)
// val[i] <- new_ids[j] where old_ids[j] == val[i] (old_ids ascending); err bit 0 if a
// value is not in old_ids.
hipError_t launch_remap_values(u64* val, u64 n, const u64* old_ids, const u64* new_ids, u64 n_ids,
                               u32* err, hipStream_t st);

// ---- merkle.hip (see the file header)
// term hashes of a tree's rows (dg_term_hashes; on = 0: the ids themselves)
struct TermH {
  const u64* nh;   // node_hash[node id]
  u64 nn;
  const u64* vid;  // ascending non-canonical value ids
  const u64* vh;   // their hashes
  u64 nv;
  u32 on;
};
struct MerkleT {
  u32 depth, sb;  // buckets 2^depth; the tree covers keys whose top sb bits == shard
  u64 shard;
  u64* nodes;     // heap, 2^(depth+1) - 1
  uint16_t* counts;  // rows per bucket, 2^depth
  TermH th;
  u64* starts;    // optional: first row of each 2^MERKLE_UPL-bucket chunk (+ the end)
};
constexpr u32 MERKLE_UPL = 11;  // levels reduced per upsweep workgroup
// input-error bits a build / update leaves in its error word: a key outside the tree's
// shard (2), a bucket over 65535 rows (4)
constexpr u32 MERKLE_ERR_SHARD = 2u, MERKLE_ERR_COUNT = 4u;
constexpr u32 MERKLE_INPUT_ERR = MERKLE_ERR_SHARD | MERKLE_ERR_COUNT;
inline u64 merkle_chunks(u32 depth) { return 1ull << (depth - (depth < MERKLE_UPL ? depth : MERKLE_UPL)); }
// scratch words of a build / update: a u64 chunk root and a u64 key count per chunk (the
// in-launch hand-off), in u32 units
inline u64 merkle_ctr_words(u32 depth) { return 4 * merkle_chunks(depth); }
// an update's per-chunk row-count changes (i64, zero on entry): how the chunk starts move
// one fused launch: rows hashed into LDS bucket sums per chunk, levels reduced, the last
// chunk reduces to the root; *d_keys = distinct keys; arrive: a persistent counter, zero
// on entry and left zero; hand: merkle_ctr_words(depth) u32 of scratch; err bit 1: a row
// outside the tree's shard.
hipError_t launch_merkle_build(const Rows& s, const MerkleT& t, u64* d_keys, u32* arrive, u64* hand,
                               u32* err, hipStream_t st);
// put/delete of the changed keys + update_hashes; dirty: merkle_chunks(depth) u32, zero
// on entry; d_keys[0, 8) (zero on entry) sum to the change in distinct keys.  The update
// adds (new leaf - old leaf) and (new rows - old rows) per key, so the same launch with
// olds and news exchanged undoes it bit for bit (keys outside the shard are skipped both
// ways; counts wrap mod 2^32 and unwrap).
hipError_t launch_merkle_update(const MerkleT& t, const Rows& olds, const Rows& news, const u64* keys,
                                u64 n_keys, u32* dirty, u64* d_keys, u32* arrive, u64* hand, i64* cdelta,
                                u32* err, hipStream_t st);
// the same from kdelta.hip's per-key figures (runs, dh; skipped when guard && *guard);
// sign -1 undoes what kdelta.hip's count kernel applied, bit for bit, then the dirty chunks
// are re-reduced
hipError_t launch_kd_tree(const MerkleT& t, const u64* keys, const u64* runs, const u64* dh, u64 nk,
                          const u64* guard, int sign, u32* dirty, u32* arrive, u64* hand, i64* cdelta,
                          u32* err, hipStream_t st);
// ---- kdelta.hip: dg_join_delta of a keyed delta of any size, one host wait (see the file header)
constexpr int KD_BLOCK = 256;  // keys per workgroup
constexpr u32 KD_RUN = 64;     // rows per key and side the per-key join takes (more: KD_BIG)
constexpr int KD_NV = 7;       // per-workgroup figures: rows, kept rows, changed keys, their rows,
                               // delta rows, distinct-key change, flags
// guard bits (d_counts[4]): the delta has a row outside the keyset (the full join applies);
// a key run over KD_RUN rows (the splice applies); more changed keys than `cap`
constexpr u64 KD_BAD = 1, KD_BIG = 2, KD_CAP = 4;
constexpr u64 KD_MOVED = 8;    // (flags only) a key's row count changed
struct KdArgs {
  Rows a;              // the state (read)
  RowsOut aw;          // the same columns (the in-place write)
  Ctx ca;              // its context (a VV)
  u32* ca_node;        // ... written with the union (uc, d_counts[1] entries)
  u64* ca_cnt;
  u64 ca_cap;
  u32* uc_node;        // the union context (the count kernel's last workgroup computes it)
  u64* uc_cnt;
  void* cu_tmp;        // its scratch (ctx_union_tmp_bytes)
  Rows d;              // the delta, sorted
  Ctx cd;              // its context, sorted
  const u64* keys;     // the keyset, ascending unique
  u64 nk;
  // per key (nk): first state row, first delta row, runs (na | nd << 16 | ne << 32 | chg << 48),
  // kept-row masks, leaf change
  u64 *a_lo, *d_lo, *runs, *amask, *dmask, *dh;
  u64* part;           // per count workgroup its KD_NV figures (the write sums the earlier ones)
  u64 ntiles;
  u64* changed;        // changed keys (cap), device or mapped host memory
  u64 cap;
  RowsOut rows;        // their rows (rows_cap), when has_rows
  u64 rows_cap;
  int has_rows;
  u32* co_node;        // (optional) a copy of the joined context (co_cap entries)
  u64* co_cnt;
  u64 co_cap;
  RowsOut sp;          // the spare store: the output when rows move
  u64* end;            // the splice index (nk, nk + 1, a_tiles + 1)
  i64* shift;
  u64* tile_u0;
  u64 a_tiles;
  MerkleT t;           // the tree (has_tree): put/delete by the count kernel
  int has_tree;
  u32* dirty;          // the tree update's dirty chunk flags and chunk row-count changes: zero
  i64* cdelta;         //   on entry, left zero (the re-reduction consumes them)
  u64* d_counts;       // the count block (the count kernel's last workgroup)
  u32* arrive;         // the count kernel's arrival counter (zero, left zero)
  u32* err;            // the tree update's input-error word, zero on entry (state writes
                       //   skipped when set; the host zeroes it after reporting)
};
// kd_count_kernel (its last workgroup scans)
hipError_t launch_kd_join(const KdArgs& p, hipStream_t st);
// kd_finish_kernel (merkle.hip): the write (dg_kdw.h) and, with a tree, its dirty chunks' re-reduction in one launch
hipError_t launch_kd_finish(const KdArgs& p, const u32* dirty, u32* arrive, u64* hand, const i64* cdelta,
                            hipStream_t st);

// ---- small.hip: dg_join_delta of a small delta, one launch (see the file header)
constexpr u32 SMALL_KEYS = 512, SMALL_DELTA = 512, SMALL_DCTX = 1024, SMALL_NODES = 2048;
constexpr u32 SMALL_TAKEN = 1024, SMALL_EDIT = 1536;
struct SmallArgs {
  Rows a;              // the state (read)
  RowsOut aw;          // the same columns (the in-place write)
  Ctx ca;              // the state's context (a VV)
  u32* ca_node;        // ... written with the union
  u64* ca_cnt;
  u64 ca_cap;
  Rows d;              // the delta, sorted
  Ctx cd;              // its context, sorted
  const u64* keys;     // ascending unique
  u64 nk;
  RowsOut e;           // scratch: the edit (SMALL_EDIT rows), the splice layout
  u64* a_lo;           // scratch: nk, the keys' first state rows
  u64* a_off;          // scratch: nk + 1, their offsets among the taken rows
  MerkleT t;           // the tree (has_tree): nodes, counts and chunk index updated here
  int has_tree;
  u64* res;            // the result block's header (device)
  u64* home;           // the whole result block (host memory the device writes)
  const u64* d_counts; // the engine's count block ...
  u64* h_pub;          // ... published here with `seq` (dg_home.h) unless the tail kernel does
  u64 seq;
  // the moved-rows splice done by the tail kernel (splice_here): the edit's rows go
  // straight to their places in `sp` and the per-key index (end, shift) is written here
  int splice_here;
  RowsOut sp;          // the spare store (the rows moved: the output)
  u64* end;            // scratch: nk, each key's state rows' end
  i64* shift;          // scratch: nk + 1, the shift of the gap before each key (and after all)
};
// result block words: header [0] flags [1] changed keys [2] their rows [3] context entries
// [4] edit rows [5] taken rows [6] moved [7] distinct-key change; then the changed keys
// (SMALL_KEYS), their rows as key | val | ts | cnt (SMALL_EDIT each) and node (u32,
// SMALL_EDIT / 2 words), the context's cnt (SMALL_NODES) and node (u32, SMALL_NODES / 2)
constexpr u64 SMALL_HDR = 8;
constexpr u64 SMALL_O_KEYS = SMALL_HDR, SMALL_O_ROWS = SMALL_O_KEYS + SMALL_KEYS;
constexpr u64 SMALL_O_CTX = SMALL_O_ROWS + 4 * (u64)SMALL_EDIT + SMALL_EDIT / 2;
constexpr u64 SMALL_WORDS = SMALL_O_CTX + SMALL_NODES + SMALL_NODES / 2;

constexpr u32 SMALL_FALLBACK = 1u;  // flags: nothing written, the general path runs
hipError_t launch_small_delta(const SmallArgs& p, hipStream_t st);
// small.hip: the moved rows' splice copy behind the small join, one launch: blocks
// [0, tiles) copy the state's rows outside the keyset into the spare store (when the join
// moved rows: res[6], res[0] == 0; the small join placed the edit's rows), and the last
// workgroup to arrive publishes `seq` (dg_home.h) -- the small join does when no row moved.
struct SmallTailArgs {
  Rows a;              // the state (read)
  RowsOut out;         // the spare store
  const u64* end;      // per key (nk): its state rows' end
  const u64* a_lo;     // per key: its first state row
  const i64* shift;    // nk + 1
  u64 nk, tiles;       // keys; splice tiles (SMALL_TILE rows each)
  const u64* res;      // the small join's result header
  const u64* d_counts;
  u64* h_pub;
  u64 seq;
  u32* arrive_all;     // every block's arrival counter (zero, left zero)
};
constexpr u64 SMALL_TILE = 2048;  // rows per splice tile of the tail kernel
hipError_t launch_small_tail(const SmallTailArgs& p, hipStream_t st);
constexpr int DIFF_BLOCK = 256;
#ifndef DG_DIFF_SUB
#define DG_DIFF_SUB 12
#endif
constexpr u32 DIFF_SUB = DG_DIFF_SUB;  // levels a diff workgroup descends: subtrees of 2^DIFF_SUB buckets
inline u32 diff_sub(u32 depth) { return depth < DIFF_SUB ? depth : DIFF_SUB; }
inline u64 diff_tiles(u32 depth) { return 1ull << (depth - diff_sub(depth)); }
// subtree boundaries in both stores, per-subtree counts, then the differing keys staged
// per subtree (at most one per row of either store), then the group sums
inline u64 diff_groups(u32 depth) { return (diff_tiles(depth) + DIFF_BLOCK - 1) / DIFF_BLOCK; }  // of DIFF_BLOCK subtrees
inline u64 diff_scratch_words(u32 depth, u64 na, u64 nb) {
  return 2 * (diff_tiles(depth) + 1) + diff_tiles(depth) + na + nb + 1;
}
// a subtree whose tree row counts overrun a store adds this to the total (no keys): at most
// 2^18 subtrees (depth 30) keep the sum of markers below 2^63, and no total of real keys
// reaches it (deltagpu.h DG_DIFF_MISMATCH)
constexpr u64 DIFF_MISMATCH = 1ull << 44;
// differing keys, ascending; the first min(total, cap) written; *d_count = total.
hipError_t launch_merkle_diff(const MerkleT& a, const Rows& sa, const MerkleT& b, const Rows& sb,
                              u64* out_keys, u64 cap, u64* scratch, u64* bsum, u64* bsum_zero, u64 nzero,
                              u64* d_count, hipStream_t st);
// dg_merkle_continue_home's one-workgroup hop (merkle.hip cont_small_kernel): limits,
// result kinds (home[0]) and arguments
constexpr u32 CS_IN = 4096, CS_B = 512;  // entries / pairs in, buckets in (leaf form)
constexpr u64 CS_OK = 0, CS_NODE = 1, CS_LEAF = 2, CS_CAP = 3, CS_BAD = 4;
constexpr int CS_HDR = 6;
struct ContSmallArgs {
  MerkleT t;
  Rows s;
  u32 level, levels;
  u64 max;                      // truncate_diff: node entries / leaf buckets kept
  const u64 *ipos, *ihash, *ibucket;
  u64 n, nb;                    // entries (pairs), buckets in
  u64 *opos, *ohash, *obucket;  // the next continuation (host or device)
  u64 ocap, ocap_b;
  u64* keys;                    // {:ok, keys}: the first kcap
  u64 kcap;
  u64* home;                    // result header: kind, n | total, n_buckets, level, needed n, needed buckets
  const u64* d_counts;
  u64* h_pub;
  u64 seq;
};
hipError_t launch_cont_small(const ContSmallArgs& a, hipStream_t st);
// prepare_partial_diff: level L's positions and node hashes (2^L entries)
hipError_t launch_cont_prepare(const MerkleT& t, u32 L, u64* opos, u64* ohash, hipStream_t st);
// partial diff.  scratch: 2 * ceil(n / 256) u64.
inline u64 cont_tiles(u64 n) { return (n + 255) / 256; }
hipError_t launch_cont_compare(const MerkleT& t, u32 L, const u64* pos, const u64* hash, u64 n,
                               u64* scratch, u64* dpos, u64* d_count, hipStream_t st);
hipError_t launch_cont_expand(const MerkleT& t, u32 L, u32 k, const u64* dpos, u64 nd, u64* opos,
                              u64* ohash, hipStream_t st);
hipError_t launch_leaves_count(const MerkleT& t, const Rows& s, const u64* buckets, u64 nb,
                               u64* scratch, u64* d_count, hipStream_t st);
hipError_t launch_leaves_write(const MerkleT& t, const Rows& s, const u64* buckets, u64 nb,
                               const u64* scratch, u64* ok, u64* oh, hipStream_t st);
// d_count[0] = the number of keys[0, n) (ascending) before bucket[0]'s first key
hipError_t launch_pairs_before_bucket(const MerkleT& t, const u64* keys, u64 n, const u64* bucket,
                                     u64* d_count, hipStream_t st);
hipError_t launch_leafdiff(const MerkleT& t, const Rows& s, const u64* buckets, u64 nb, const u64* pk,
                           const u64* ph, u64 np, u64* out, u64 cap, u64* scratch, u64* d_count,
                           hipStream_t st);

}  // namespace dg
