/*
 * deltagpu.h — C-ABI of libdeltagpu, the MI355X-native batched delta-join and
 * anti-entropy engine for DeltaCrdt.AWLWWMap (reference: burmajam/delta_crdt_ex 0.5.10).
 *
 * This header is the drop-in boundary.  Each entry point names the reference
 * function it replaces (path:line relative to the reference repository).  A
 * caller (the Erlang NIF sketched in INTEGRATION.md, or the Python host mirror in
 * delta_crdt_ex_amd/aw_lww_map.py via ctypes) marshals `%AWLWWMap{}` terms into
 * the SoA dot rows below and back.
 *
 * Data model.  A state `%AWLWWMap{dots: c, value: %{key =>
 * %{{v, ts} => MapSet[{node, counter}]}}}` is flattened to one ROW per dot:
 *
 *     key  u64   interned key id (a 64-bit hash of the key; exact interning on the host)
 *     val  u64   order-preserving id of the value (Erlang term order), see H2
 *     ts   i64   System.monotonic_time(:nanosecond) of the add (signed)
 *     node u32   interned node id of the dot
 *     cnt  u64   dot counter
 *
 * Rows are stored column-wise (SoA, device memory), sorted ascending by the tuple
 * (key, val, ts [signed], node, cnt) and free of duplicates.  Every entry point
 * that consumes a store assumes this; `dg_store_check` verifies it.
 *
 * A causal context is either a version vector (DG_CTX_VV: node[i] ascending and
 * unique, cnt[i] = max counter, as produced by `Dots.compress/1`) or an explicit
 * dot set (DG_CTX_DOTS: (node, cnt) ascending and unique, a `MapSet` of dots).
 *
 * Conventions: every function returns DG_OK (0) or a negative DG_E_* code and sets
 * a thread-local message readable with dg_last_error().  Input pointers are
 * caller-owned device pointers (a context's arrays may also be host pointers where
 * noted).  Output stores/contexts are caller-allocated with `cap` set; on return
 * `n` holds the produced count; DG_E_CAPACITY if `cap` is too small (nothing
 * else is touched).  One dg_engine owns one HIP stream; engines are independent
 * and may be used from different threads; a single engine is not re-entrant.
 */
#ifndef DELTAGPU_H
#define DELTAGPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DG_ABI_VERSION 4

enum dg_status {
  DG_OK = 0,
  DG_E_INVAL = -1,     /* bad argument (null pointer, mixed context kinds where forbidden, ...) */
  DG_E_CAPACITY = -2,  /* output capacity too small */
  DG_E_DEVICE = -3,    /* HIP runtime error */
  DG_E_NOMEM = -4,     /* device allocation failed */
  DG_E_ORDER = -5,     /* input store/context not sorted+unique (dg_store_check) */
  DG_E_CLAUSE = -6     /* the reference would raise FunctionClauseError / RuntimeError */
};

enum dg_context_kind { DG_CTX_VV = 0, DG_CTX_DOTS = 1 };

typedef struct dg_store {
  uint64_t* key;
  uint64_t* val;
  int64_t* ts;
  uint32_t* node;
  uint64_t* cnt;
  uint64_t n;   /* rows present */
  uint64_t cap; /* rows allocated (outputs only) */
} dg_store;

typedef struct dg_context {
  int32_t kind; /* enum dg_context_kind */
  int32_t reserved;
  uint32_t* node;
  uint64_t* cnt;
  uint64_t n;
  uint64_t cap;
} dg_context;

/* Term hashes for the Merkle rows: with them a tree covers the TERMS of each row, not the
 * ids one host's interning tables gave them, so two replicas' trees compare on any BEAM
 * node (the reference hashes the raw value map, causal_crdt.ex:390-394, and diffs against
 * neighbours on other nodes, causal_crdt_test.exs:68-78).  In a row's hash
 *   the node id n becomes node_hash[n]                         (n < n_nodes)
 *   the value id v becomes val_hash[j] where val_id[j] == v    (v outside [2^58, 2^63))
 * -- a canonical integer value's id (v + 2^62 for integers in [-2^62 + 2^58, 2^62)) is the
 * same on every host and hashes as itself; key ids are term hashes already.  The Python
 * mirror (interning.py Universe.term_tables) and the NIF (c_src/marshal.c dgm_node_hashes,
 * dgm_value_hashes) produce these tables; ids missing from them hash as themselves. */
typedef struct dg_term_hashes {
  const uint64_t* node_hash; /* device: the hash of node id i, n_nodes entries */
  uint64_t n_nodes;
  const uint64_t* val_id;    /* device, ascending: the non-canonical value ids */
  const uint64_t* val_hash;  /* device: their term hashes */
  uint64_t n_vals;
} dg_term_hashes;

/* Merkle index over a store (the MerkleMap role, causal_crdt.ex:21,94,96,254,255,390-394).
 * The tree covers the keys whose top `shard_bits` bits equal `shard` (a key-hash shard,
 * SURVEY.md §8(e); shard_bits = 0: every key) in 2^depth buckets by the next `depth`
 * bits: bucket(key) = (key << shard_bits) >> (64 - depth).
 *   bucket hash = Σ row_hash over the bucket's rows (mod 2^64; a key's leaf is the sum
 *                 over its own rows: its raw value map, causal_crdt.ex:392)
 *   parent      = node_hash(left, right)                       (dg_hash.h)
 * `nodes` is a heap in level order: level l (root l = 0) occupies [2^l - 1, 2^(l+1) - 1);
 * level `depth` holds the buckets.  `counts` holds each bucket's row count (at most 65535
 * rows per bucket; DG_E_CAPACITY beyond): the diff finds a differing bucket's rows from
 * them instead of reading every key.  The tree keeps no per-key leaves: a diff recomputes
 * them from the store the tree indexes, so the diff entry points take the stores too.
 * The 2^b shard trees (shard_bits = b, depth d - b) are exactly the level-b subtrees of
 * the unsharded depth-d tree; dg_merkle_fold_roots recombines their roots. */
typedef struct dg_merkle {
  uint32_t depth;      /* 1..28; shard_bits + depth <= 44 */
  uint32_t shard_bits; /* 0..16 */
  uint64_t shard;      /* < 2^shard_bits */
  uint64_t* nodes;     /* 2^(depth+1) - 1 entries (caller-allocated, device) */
  uint64_t n_keys;     /* distinct keys indexed (set by build / update) */
  uint16_t* counts;    /* max(2^depth, 16) entries, 16-B aligned (caller-allocated, device;
                          set by build / update) */
  const dg_term_hashes* terms; /* host pointer (its arrays: device); NULL: hash the ids */
  uint64_t* starts;    /* optional (NULL: none): dg_merkle_chunks(depth) + 1 entries (device),
                          the first row of every 2^11-bucket chunk in the indexed store and,
                          last, the end of the tree's rows; set by build, kept by update (they
                          move with the rows).  The diff reads a subtree's rows from it instead
                          of searching the store's keys. */
} dg_merkle;

/* The number of 2^11-bucket chunks of a depth-`depth` tree (1 up to depth 11): `starts`
 * holds one more entry.  Host only. */
uint64_t dg_merkle_chunks(uint32_t depth);

/* A partial-diff continuation (the `continuation` of CausalCrdt's %Diff{},
 * causal_crdt.ex:29,96,255): either NODE form -- the sender's hashes of the nodes
 * pos[0, n) of tree level `level` -- or LEAF form (level == depth + 1) -- the sender's
 * (key, leaf hash) pairs pos/hash[0, n) of the buckets bucket[0, n_buckets), all
 * ascending.  Device arrays, caller-allocated with capacities. */
typedef struct dg_merkle_cont {
  uint32_t level;
  uint32_t reserved;
  uint64_t* pos;       /* node positions (node form) or keys (leaf form) */
  uint64_t* hash;
  uint64_t n, cap;
  uint64_t* bucket;    /* leaf form: the differing buckets the pairs cover */
  uint64_t n_buckets, cap_buckets;
} dg_merkle_cont;

typedef struct dg_engine dg_engine;

/* ---- lifecycle ------------------------------------------------------------ */
/* Synchronous calls (every entry point without _async) return when their work is done:
 * the calling thread polls a word in host-mapped memory for up to 20 ms (a CPU core
 * stays busy, as on a BEAM dirty scheduler), then waits on the stream instead. */
int dg_abi_version(void);
const char* dg_last_error(void);
/* The sha256 prefix (16 hex digits) of the sources this library was built from
 * (the .hip and .h files of csrc/ and this header, delta_crdt_ex_amd/build.py): the host side
 * refuses a library whose digest differs from its tree's, so a stale build is never the
 * one tested or measured. */
const char* dg_build_digest(void);
/* `hip_stream` NULL: the engine creates its own stream; otherwise it launches on the
 * given hipStream_t (e.g. torch.cuda.current_stream().cuda_stream) and never
 * destroys it. */
int dg_engine_create(int device, void* hip_stream, dg_engine** out);
int dg_engine_destroy(dg_engine* e);
void* dg_engine_stream(dg_engine* e);
/* Waits for the engine stream.  The single-pass join is a persistent grid; when it
 * cannot become resident (other kernels hold the CUs) it aborts, and dg_engine_sync then
 * replays the asynchronous calls made since the last sync (joins on the two-pass
 * kernels), so their outputs are correct when it returns DG_OK.  Their arguments (and
 * dg_merkle objects) must stay valid until then.  Every synchronous call first settles
 * the asynchronous calls made before it, as dg_engine_sync does (an error of theirs is
 * then that call's error).  At most 4096 asynchronous calls are logged: the next one
 * settles the log first. */
int dg_engine_sync(dg_engine* e);

/* ---- device buffers (for callers without a device runtime of their own: the NIF) -- */
/* Allocate / free a store's device columns (s->cap = cap, s->n = 0). */
int dg_store_alloc(dg_engine* e, uint64_t cap, dg_store* s);
int dg_store_free(dg_engine* e, dg_store* s);
/* Host columns -> device columns (dev->cap >= host->n; dev->n = host->n), and back
 * (host->cap >= dev->n; host->n = dev->n).  Synchronous. */
int dg_store_upload(dg_engine* e, const dg_store* host, dg_store* dev);
int dg_store_download(dg_engine* e, const dg_store* dev, dg_store* host);
/* The same for contexts (kind copied). */
int dg_context_alloc(dg_engine* e, uint64_t cap, dg_context* c);
int dg_context_free(dg_engine* e, dg_context* c);
int dg_context_upload(dg_engine* e, const dg_context* host, dg_context* dev);
int dg_context_download(dg_engine* e, const dg_context* dev, dg_context* host);
/* Raw device memory (key lists, Merkle nodes, continuations) and copies
 * (dg_copy_to_device also copies device to device: its source may be device memory). */
int dg_buffer_alloc(dg_engine* e, uint64_t bytes, void** p);
int dg_buffer_free(dg_engine* e, void* p);
int dg_copy_to_device(dg_engine* e, void* dst, const void* src, uint64_t bytes);
int dg_copy_to_host(dg_engine* e, void* dst, const void* src, uint64_t bytes);
/* A copy in any direction ENQUEUED on the engine stream (no wait): it is ordered with the
 * engine's kernels, so a synchronous call after it sees its data, and its destination is
 * complete once any later synchronous call (or dg_engine_sync) returns.  Not replayed by
 * dg_engine_sync.  The NIF packs a delta message into pinned memory and ships it with one
 * such copy, and brings several result ranges home with one wait (c_src/replica.c). */
int dg_copy_async(dg_engine* e, void* dst, const void* src, uint64_t bytes);
/* Page-locked host memory (what dg_copy_async needs to overlap and what makes small copies
 * cheap), mapped into the device's address space: an entry point's device OUTPUT pointers
 * may point into it, and the kernels then write the result straight to the host (small
 * outputs: no copy, no second wait).  dg_host_free waits for the engine stream first. */
int dg_host_alloc(dg_engine* e, uint64_t bytes, void** p);
int dg_host_free(dg_engine* e, void* p);

/* Verify the sorted+unique precondition of a store (DG_E_ORDER if violated). */
int dg_store_check(dg_engine* e, const dg_store* s);

/* ---- the join (hot path) --------------------------------------------------- */
/* AWLWWMap.join/3 (lib/delta_crdt/aw_lww_map.ex:153-158) with join_or_maps/4
 * (:161-193) and join_dot_sets/4 (:196-209):
 *   per (key, {v, ts}) entry:  s1 ∩ s2  ∪  s1 \ c2  ∪  s2 \ c1      (Dots.difference :54-65,
 *                                                                     Dots.member? :67-73)
 *   empty entries and keys dropped (:177-181); out_ctx = Dots.union(c1, c2) (:39-52).
 * `keys` (device, ascending unique, n_keys entries) is the reference's `keys`
 * argument; NULL means "every key of a and b" (a full-state join).  Keys of a or b
 * outside `keys` are not joined but carried over right-biased, as
 * Map.merge(Map.drop(d1, keys), Map.drop(d2, keys)) does (:185-188).
 * out->cap must be >= a->n + b->n; out_ctx->cap >= ca->n + cb->n.  Synchronous. */
int dg_join2(dg_engine* e, const dg_store* a, const dg_context* ca, const dg_store* b,
             const dg_context* cb, const uint64_t* keys, uint64_t n_keys, dg_store* out,
             dg_context* out_ctx);

/* Same, asynchronous on the engine stream: the output row count is written to
 * d_counts[0] and the output context size to d_counts[1] (device memory); out->n
 * and out_ctx->n are NOT updated and out_ctx->kind is set on the host. */
int dg_join2_async(dg_engine* e, const dg_store* a, const dg_context* ca, const dg_store* b,
                   const dg_context* cb, const uint64_t* keys, uint64_t n_keys,
                   dg_store* out, dg_context* out_ctx, uint64_t* d_counts);

/* join/3 (as dg_join2) plus the changed-key diff CausalCrdt computes after every join
 * (update_state_with_delta/3 -> diff/3, causal_crdt.ex:343-351,383-393): the keys of
 * `keys` (every key when NULL) whose rows in `out` differ from their rows in `a` --
 * removed keys, new keys and keys whose entries or dots changed -- ascending and
 * unique, into changed[0, cap), *n_changed = their number (DG_E_CAPACITY if > cap).
 * The caller's on_diffs / MerkleMap work (:386-404) reads these keys (dg_read_lww
 * with them as `keys` on `a` and `out`).  Recorded inside the join's merge; always the
 * single-pass join kernel.  Synchronous. */
int dg_join2_changes(dg_engine* e, const dg_store* a, const dg_context* ca, const dg_store* b,
                     const dg_context* cb, const uint64_t* keys, uint64_t n_keys, dg_store* out,
                     dg_context* out_ctx, uint64_t* changed, uint64_t cap, uint64_t* n_changed);

/* CausalCrdt.update_state_with_delta (causal_crdt.ex:383-404) on a device-resident
 * state: state = AWLWWMap.join(state, delta, keys) (aw_lww_map.ex:153-209), the keys whose
 * value changed (diff/3, :343-351) into changed[0, cap) ascending, and the state's
 * MerkleMap `tree` (NULL: none) updated for them (MerkleMap.put/delete + update_hashes,
 * :390-394).  state_ctx becomes the union (cap >= state_ctx->n + delta_ctx->n).
 * The join is applied IN PLACE when every key of the keyset keeps its number of rows (the
 * rows outside the keyset do not move: only the keyset's rows are rewritten); otherwise
 * the joined state is written to `spare` (cap >= state->n + delta->n) and the two
 * dg_store structs are exchanged, *swapped = 1 -- on return *state always describes the
 * joined state and *spare a free buffer.  A delta with a key outside `keys` (not a sync
 * delta) takes the full join, also through `spare`; as in the reference, the tree then
 * follows the changed keys of the keyset only (diff/3 runs over `keys`).  Synchronous. */
int dg_join_delta(dg_engine* e, dg_store* state, dg_context* state_ctx, const dg_store* delta,
                  const dg_context* delta_ctx, const uint64_t* keys, uint64_t n_keys,
                  dg_store* spare, dg_merkle* tree, uint64_t* changed, uint64_t cap,
                  uint64_t* n_changed, int* swapped);

/* dg_join_delta plus the rows of the changed keys in the joined state -- what the caller
 * hands to on_diffs and its reply (the changed keys' new value maps, causal_crdt.ex:344-352,
 * the NIF's join_delta) -- into rows[0, rows->cap), rows->n = their number, in store
 * order.  On the in-place and moved paths they are taken from the join's own edit of the
 * keyset (small and cache-resident) instead of by a search of the whole state, as a
 * dg_take_keys call after dg_join_delta would.  More rows than rows->cap is not an
 * error (the join is complete): rows->n > rows->cap on return says the rows were not
 * written; take them with dg_take_keys.  The same holds for any failure of that gather,
 * which runs after the join is committed: an error return always means the state, its
 * context and tree are unchanged.  Synchronous. */
int dg_join_delta_rows(dg_engine* e, dg_store* state, dg_context* state_ctx, const dg_store* delta,
                       const dg_context* delta_ctx, const uint64_t* keys, uint64_t n_keys,
                       dg_store* spare, dg_merkle* tree, uint64_t* changed, uint64_t cap,
                       uint64_t* n_changed, int* swapped, dg_store* rows);

/* dg_join_delta_rows plus a copy of the joined context into ctx_out (ctx_out->n set; more
 * than ctx_out->cap entries: not written).  `changed`, `rows` and ctx_out may be host memory
 * from dg_host_alloc: a delta whose keys all lie in the keyset (a sync delta, a batch of
 * mutations) is then joined, its tree updated and its results written there by the kernels,
 * with ONE host wait (the NIF's join_delta and mutate_batch). */
int dg_join_delta_out(dg_engine* e, dg_store* state, dg_context* state_ctx, const dg_store* delta,
                      const dg_context* delta_ctx, const uint64_t* keys, uint64_t n_keys,
                      dg_store* spare, dg_merkle* tree, uint64_t* changed, uint64_t cap,
                      uint64_t* n_changed, int* swapped, dg_store* rows, dg_context* ctx_out);

/* dg_join_delta_rows for a SMALL delta in ONE launch chain with ONE host wait (the general
 * path waits after each of its four steps): the keyed join, the changed keys, the MerkleMap
 * put/delete + update_hashes, and the results written straight into `home`, host memory
 * from dg_host_alloc of DG_HOME_WORDS words:
 *   home[0] flags (0: done; DG_HOME_FALLBACK: nothing was done -- call dg_join_delta_rows)
 *   home[1] changed keys   home[2] their rows   home[3] the state's context entries
 *   home[DG_HOME_KEYS ...]  the changed keys, ascending
 *   home[DG_HOME_ROWS ...]  their rows in store order: key | val | ts | cnt columns at stride
 *                           DG_HOME_STRIDE, then node (uint32) at DG_HOME_ROWS + 4 stride
 *   home[DG_HOME_CTX ...]   the new context: cnt (DG_HOME_NODES), then node (uint32)
 * Small: keys <= 512, delta rows <= 512, delta context <= 1024 entries, a VV state context
 * of <= 2048 entries, node ids < 2048, at most 1024 state rows under the keys, every
 * delta key in `keys` (the sync and mutation shape) -- else DG_HOME_FALLBACK with the
 * state, its context and the tree untouched.  Rows move (a key's row count changed) ->
 * the joined state is in `spare` and the structs are exchanged (*swapped = 1), as
 * dg_join_delta.  The delta, its context and `keys` may be device memory or host memory
 * from dg_host_alloc (the kernel reads them over PCIe: no copy launch for a one-key op);
 * they must stay unchanged until the call returns.  Synchronous. */
#define DG_HOME_FALLBACK 1
#define DG_HOME_KEYS 8
#define DG_HOME_STRIDE 1536
#define DG_HOME_ROWS (DG_HOME_KEYS + 512)
#define DG_HOME_NODES 2048
#define DG_HOME_CTX (DG_HOME_ROWS + 4 * DG_HOME_STRIDE + DG_HOME_STRIDE / 2)
#define DG_HOME_WORDS (DG_HOME_CTX + DG_HOME_NODES + DG_HOME_NODES / 2)
int dg_join_delta_home(dg_engine* e, dg_store* state, dg_context* state_ctx, const dg_store* delta,
                       const dg_context* delta_ctx, const uint64_t* keys, uint64_t n_keys,
                       dg_store* spare, dg_merkle* tree, uint64_t* home, int* swapped);

/* Fold of join/3 over k stores (how CausalCrdt applies k deltas in a row,
 * causal_crdt.ex:86-89,383-384): out = join(...join(join(s0, s1), s2)..., s_{k-1})
 * over all keys.  A row survives iff for every input i it is present in s_i or its
 * dot is not covered by c_i.  out->cap >= Σ n_i. */
int dg_joink(dg_engine* e, int k, const dg_store* stores, const dg_context* ctxs, dg_store* out,
             dg_context* out_ctx);

/* A batch of deltas applied to a state as CausalCrdt applies delta messages, one
 * join/3 per delta with that delta's own `keys` (causal_crdt.ex:86-89,383-384, and
 * the sync shape {%{dots: VV, value: Map.take(value, keys)}, keys} of :324-335):
 *   out = join(...join(join(state, deltas[0], keys[0]), deltas[1], keys[1])...,
 *              deltas[k-1], keys[k-1]).
 * keys[i] (device, ascending unique, n_keys[i] entries) or keys == NULL / keys[i] ==
 * NULL for a full-state join of that delta.  out->cap >= state->n + Σ deltas[i].n,
 * out_ctx->cap >= ctx->n + Σ dctxs[i].n.  Synchronous.
 * Runs as ONE pass over the state per 64 deltas when the state's context is a VV, every
 * context names node ids < 1024 only, dot-set contexts (mutation deltas) have counters
 * below 2^48 - 1, and the key ids are spread like hashes (the interned form); otherwise,
 * and always with DG_APPLY_MODE=fold in the environment at engine creation, as k
 * dg_join2 steps through engine scratch.  Both give the same rows. */
int dg_apply_deltas(dg_engine* e, const dg_store* state, const dg_context* ctx, int k,
                    const dg_store* deltas, const dg_context* dctxs,
                    const uint64_t* const* keys, const uint64_t* n_keys, dg_store* out,
                    dg_context* out_ctx);

/* ---- sync deltas ----------------------------------------------------------- */
/* The value half of a sync delta, Map.take(state.value, keys) (causal_crdt.ex:112-123,
 * 324-335: {:diff, %{state | dots: diff.dots, value: Map.take(value, keys)}, keys}):
 * the rows of `s` whose key is in `keys` (device, ascending unique), in store order,
 * into out[0, out->cap); out->n = their number (DG_E_CAPACITY if > out->cap).  The
 * delta's context is the caller's VV snapshot (diff.dots); with it and `keys` the
 * result goes straight into dg_join2 / dg_apply_deltas on the receiving side.
 * Synchronous. */
int dg_take_keys(dg_engine* e, const dg_store* s, const uint64_t* keys, uint64_t n_keys,
                 dg_store* out);

/* ---- batched mutations ----------------------------------------------------- */
/* A batch of AWLWWMap.add/4 and remove/3 operations by node `node` as ONE delta
 * (aw_lww_map.ex:99-146; CausalCrdt applies each op's delta with keys = [key] as the op
 * arrives, causal_crdt.ex:337-342).  The m ops (device arrays) are sorted by key,
 * ascending, in batch order within a key (DG_E_ORDER otherwise): kind[i] 1 = add
 * (value val[i] at ts[i]), 0 = remove; add_rank[i] = the number of adds before op i in
 * batch order; n_adds = the batch's adds.  Outputs:
 *   delta      one row per touched key whose last op is an add, with dot
 *              {node, C[node] + 1 + add_rank} (C = ctx, a version vector);
 *   delta_dots the delta's context as a sorted dot list: the dots of the touched keys'
 *              rows in `state` plus the dot of every add;
 *   keys_out   the touched keys, ascending, *n_keys_out of them (cap keys_cap).
 * dg_join2(state, ctx, delta, delta_dots, keys_out, ...) then equals applying the ops
 * one by one.  Capacities: delta->cap >= touched keys, delta_dots->cap >= touched
 * keys' rows + n_adds (DG_E_CAPACITY names the sizes).  Synchronous. */
int dg_mutate_batch(dg_engine* e, const dg_store* state, const dg_context* ctx, uint32_t node,
                    uint64_t m, const uint8_t* kind, const uint64_t* key, const uint64_t* val,
                    const int64_t* ts, const uint64_t* add_rank, uint64_t n_adds, dg_store* delta,
                    dg_context* delta_dots, uint64_t* keys_out, uint64_t keys_cap,
                    uint64_t* n_keys_out);

/* The same, asynchronous: the host values (delta->n, delta_dots->n, *n_keys_out) are set on
 * return (one wait, for the counts), the outputs' device writes are enqueued on the engine
 * stream -- later calls of this engine (dg_join_delta_rows with the delta) read them in
 * order; any other reader calls dg_engine_sync first.  What the NIF's mutate_batch uses. */
int dg_mutate_batch_async(dg_engine* e, const dg_store* state, const dg_context* ctx, uint32_t node,
                          uint64_t m, const uint8_t* kind, const uint64_t* key, const uint64_t* val,
                          const int64_t* ts, const uint64_t* add_rank, uint64_t n_adds, dg_store* delta,
                          dg_context* delta_dots, uint64_t* keys_out, uint64_t keys_cap,
                          uint64_t* n_keys_out);

/* ---- causal-context algebra ----------------------------------------------- */
/* Dots.union/2 (aw_lww_map.ex:39-52): VV ⊔ VV = per-node max; VV ⊔ DOTS folds the
 * dots into the VV; DOTS ⊔ DOTS = set union. */
int dg_context_union(dg_engine* e, const dg_context* a, const dg_context* b, dg_context* out);
/* Dots.compress/1 + compress_dots/1 (aw_lww_map.ex:13-20,115-117).  DG_E_CLAUSE if
 * `dots` is already a VV (the reference raises FunctionClauseError there). */
int dg_compress_dots(dg_engine* e, const dg_context* dots, dg_context* out_vv);

/* ---- read (LWW) ------------------------------------------------------------ */
/* AWLWWMap.read/1,2 (aw_lww_map.ex:211-224): per key, the value of the entry with
 * the greatest ts; a tie goes to the smallest {val, ts} (the first entry in flatmap
 * order).  `keys` NULL: every key; otherwise only those keys
 * (Map.take).  Output ascending by key. */
int dg_read_lww(dg_engine* e, const dg_store* s, const uint64_t* keys, uint64_t n_keys,
                uint64_t* out_key, uint64_t* out_val, uint64_t cap, uint64_t* n_out);

/* ---- marshalling ------------------------------------------------------------ */
/* Order rows produced by walking %AWLWWMap{value: %{key => %{{v, ts} => MapSet}}}
 * (aw_lww_map.ex:2-3) in map iteration order: `out` = the rows of `in` sorted by
 * (key, val, ts [signed], node, cnt) with exact duplicates dropped -- the precondition
 * of every other entry point.  A hand-written LSD radix sort on the device (csrc/
 * sort.hip).  in and out: device columns, out->cap >= in->n, distinct from in.
 * Synchronous. */
int dg_sort_store(dg_engine* e, const dg_store* in, dg_store* out);
/* The same for a context: a VV by node (kind DG_CTX_VV), a dot set by (node, cnt)
 * (DG_CTX_DOTS).  Entries are assumed distinct (a map / MapSet).  out->cap >= in->n. */
int dg_sort_context(dg_engine* e, const dg_context* in, dg_context* out);

/* ---- interning maintenance -------------------------------------------------- */
/* Value ids are order-preserving ranks in Erlang term order with gaps (the read
 * tie-break, aw_lww_map.ex:211-216).  When the host's value table runs out of room
 * between two neighbours it re-spaces the ids of that region (a strictly increasing
 * map inside the region); this rewrites s->val in place: val = new_ids[j] where
 * old_ids[j] == val; values outside [old_ids[0], old_ids[n_ids-1]] (canonical integers,
 * the other region) are left as they are.  old_ids / new_ids: device arrays of n_ids
 * entries, both ascending.  The store stays sorted.  DG_E_INVAL if a row's value lies
 * inside that range but is not in old_ids (a stale id).  Synchronous. */
int dg_remap_values(dg_engine* e, dg_store* s, const uint64_t* old_ids, const uint64_t* new_ids,
                    uint64_t n_ids);

/* ---- Merkle anti-entropy (MerkleMap role) --------------------------------- */
/* Build the tree of `s` (MerkleMap.new + put of every key, causal_crdt.ex:21,390-394):
 * t->depth, shard_bits, shard, nodes, counts and terms set by the caller; sets t->n_keys.
 * DG_E_INVAL if a row's key is outside the tree's shard, DG_E_CAPACITY if a bucket holds
 * more than 65535 rows (use a deeper tree).  Synchronous. */
int dg_merkle_build(dg_engine* e, const dg_store* s, dg_merkle* t);
/* Same, asynchronous on the engine stream: the distinct-key count goes to d_n_keys[0]
 * (device); t->n_keys is not updated and a key outside the shard is not reported. */
int dg_merkle_build_async(dg_engine* e, const dg_store* s, dg_merkle* t, uint64_t* d_n_keys);

/* MerkleMap.put/delete of the keys a join changed plus update_hashes
 * (update_state_with_delta, causal_crdt.ex:383-394; update_hashes :94,254): `t` indexes
 * `old_s`; afterwards it indexes `new_s`, bit-identical (nodes and counts) to
 * dg_merkle_build(new_s), having
 * re-hashed only `keys` (device, ascending unique: every key whose rows differ between
 * the stores, e.g. dg_join2_changes's output; extra keys are harmless) and the 2^11-bucket
 * chunks they touch.  Synchronous. */
int dg_merkle_update(dg_engine* e, dg_merkle* t, const dg_store* old_s, const dg_store* new_s,
                     const uint64_t* keys, uint64_t n_keys);

/* The keys whose raw value maps differ between two indexed stores (present in one only,
 * or with different rows), ascending -- the key list MerkleMap.continue_partial_diff ends
 * with (causal_crdt.ex:96,104-105), here with both trees at hand.  The trees are descended
 * from the roots of their 4096-bucket subtrees through the differing nodes only, and only
 * the rows of differing buckets are read (located by the trees' row counts).  The first
 * min(total, cap) keys are written to out_keys, *n_out = that number and *n_total = the
 * total: a total above cap is the reference's truncate(keys, max_sync_size)
 * (Enum.take, causal_crdt.ex:105,206-210), not an error.  Trees: same depth and shard.
 * Each store must be the one its tree was built / updated against: where a tree counts
 * more rows than its store holds, nothing is read past the store and DG_E_INVAL is
 * returned (the async form's total is then >= DG_DIFF_MISMATCH). */
#define DG_DIFF_MISMATCH (1ull << 44)
int dg_merkle_diff(dg_engine* e, const dg_merkle* a, const dg_store* sa, const dg_merkle* b,
                   const dg_store* sb, uint64_t* out_keys, uint64_t cap, uint64_t* n_out,
                   uint64_t* n_total);

/* Same, asynchronous on the engine stream (the loop a replica's anti-entropy timer runs,
 * or several shard diffs in flight): the total goes to d_total[0] (device) and the first
 * min(total, cap) keys to out_keys once the stream reaches them.  Pending asynchronous
 * joins are settled first, as by every call that reads a store. */
int dg_merkle_diff_async(dg_engine* e, const dg_merkle* a, const dg_store* sa, const dg_merkle* b,
                         const dg_store* sb, uint64_t* out_keys, uint64_t cap, uint64_t* d_total);

/* MerkleMap.prepare_partial_diff(mm, levels) (causal_crdt.ex:255): a node-form
 * continuation of the tree's level min(levels, depth), every node of it.  `out`'s arrays
 * may be device memory or host memory from dg_host_alloc.  Synchronous. */
int dg_merkle_prepare(dg_engine* e, const dg_merkle* t, uint32_t levels, dg_merkle_cont* out);

/* MerkleMap.continue_partial_diff(cont, mm, levels) (causal_crdt.ex:96) on the receiving
 * replica's tree `t` over its store `s`:
 *   node form, level < depth : the entries whose node differs, expanded `levels` levels
 *                              down (at most to the buckets) -> *status = 1 (:continue),
 *                              `out` holds this tree's hashes of those nodes;
 *   node form, level == depth: the differing buckets -> *status = 1, `out` in leaf form
 *                              (this store's (key, leaf) pairs of those buckets);
 *   leaf form                : the keys of the listed buckets whose leaves differ from
 *                              this store's -> *status = 0 (:ok), keys as dg_merkle_diff
 *                              (first min(total, cap) in keys, *n_keys, *n_total).
 * No differing entry -> *status = 0 with *n_keys = *n_total = 0 ({:ok, []}).  DG_E_CAPACITY
 * if `out` is too small (out->n / out->n_buckets then hold the sizes needed). */
int dg_merkle_continue(dg_engine* e, const dg_merkle* t, const dg_store* s, const dg_merkle_cont* in,
                       uint32_t levels, dg_merkle_cont* out, uint64_t* keys, uint64_t cap,
                       uint64_t* n_keys, uint64_t* n_total, int* status);

/* One hop of dg_merkle_continue + dg_merkle_truncate(`max`) in ONE launch with ONE host
 * wait, for a continuation of at most DG_CONT_HOME_ENTRIES entries (node form) or pairs and
 * DG_CONT_HOME_BUCKETS buckets (leaf form): what a replica does per anti-entropy message.
 * `in`, `out` and `keys` may be device memory or host memory from dg_host_alloc (the kernel
 * reads and writes them over PCIe).  Results as the two calls give them, except that the
 * capacity asked of `out` is the truncated output's (node form: min(children, max)
 * entries; leaf form: the first min(buckets, max) buckets and their pairs).  A larger
 * continuation: *status = DG_CONT_DECLINED and nothing done (use dg_merkle_continue).
 * DG_E_INVAL for a position or bucket outside the tree (the general path does not check). */
#define DG_CONT_DECLINED 2
#define DG_CONT_HOME_ENTRIES 4096
#define DG_CONT_HOME_BUCKETS 512
int dg_merkle_continue_home(dg_engine* e, const dg_merkle* t, const dg_store* s, const dg_merkle_cont* in,
                            uint32_t levels, uint64_t max, dg_merkle_cont* out, uint64_t* keys, uint64_t cap,
                            uint64_t* n_keys, uint64_t* n_total, int* status);

/* MerkleMap.truncate_diff(cont, max) (causal_crdt.ex:98,212-214): keep the first `max`
 * entries of a node-form continuation, or the pairs of the first `max` buckets of a
 * leaf-form one (`t`: the tree that produced it; a leaf form needs one device
 * lower-bound to count the pairs it keeps). */
int dg_merkle_truncate(dg_engine* e, const dg_merkle* t, dg_merkle_cont* cont, uint64_t max);

/* The root of the unsharded tree from the 2^shard_bits shard roots (shard order), as the
 * RCCL all-gather of per-GPU roots needs it.  Host only. */
int dg_merkle_fold_roots(const uint64_t* roots, uint32_t shard_bits, uint64_t* root);

#ifdef __cplusplus
}
#endif
#endif /* DELTAGPU_H */
