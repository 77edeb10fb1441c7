/*
 * replica.h — the device-resident replica state behind the Erlang NIF
 * (c_src/deltagpu_nif.c), term-independent: what a GPU-attached %AWLWWMap{} holds on the
 * device and the calls CausalCrdt makes on it (reference lib/delta_crdt/causal_crdt.ex,
 * lib/delta_crdt/aw_lww_map.ex).  The NIF is a term layer over this file; the Python
 * mirror of the NIF (delta_crdt_ex_amd/nif.py) binds the SAME functions over ctypes, and
 * c_src/bench_mutate.c times them, so the code the tests and the bench run is the code a
 * BEAM node would run.
 *
 * Value semantics over one in-place device state.  The reference's states are immutable
 * terms: diffs_to_callback reads the OLD state after the join produced the new one
 * (causal_crdt.ex:361-365), and diff/3 compares old and new (:344-351).  The device state
 * is updated in place, so every state carries a VERSION: dgr_state_load returns version
 * 1, every call that changes the rows or the context (dgr_join_delta, dgr_mutate_batch)
 * takes the caller's version and returns the next one, and every call refuses a version
 * that is not the state's current one with DGR_E_STALE -- the caller's struct is then an
 * older value whose terms are authoritative (the Elixir side reads or joins those on the
 * CPU).  A call that fails after it may have touched the device (any
 * error of dgr_join_delta / dgr_mutate_batch) also moves the version on: the caller
 * detaches, and no struct can read a half-known state.
 *
 * Memory: every buffer a call needs is owned by the engine or the state and grown on
 * demand (the packed delta message in page-locked memory, the return block, the read
 * output, the continuation buffers), so a warm call allocates nothing.  Results are host
 * views into engine-owned page-locked buffers, valid until the next call on the engine.
 *
 * Threading: one call at a time per engine (the NIF holds the engine mutex).
 */
#ifndef DG_REPLICA_H
#define DG_REPLICA_H

#include <stddef.h>
#include <stdint.h>

#include "../include/deltagpu.h"

#ifdef __cplusplus
extern "C" {
#endif

#define DGR_E_STALE (-16) /* the caller's version is not the state's (an older struct) */

typedef struct dgr_engine dgr_engine;
typedef struct dgr_state dgr_state;

int dgr_engine_open(int device, dgr_engine** out);
/* Frees the engine's buffers and the dg_engine; every state must be freed before. */
int dgr_engine_close(dgr_engine* g);
dg_engine* dgr_dg(dgr_engine* g);
/* The live states of the engine (a relabel rewrites them all). */
uint64_t dgr_live_states(const dgr_engine* g);

/* The interning universe's term-hash tables (host arrays: dgm_node_hashes /
 * dgm_value_hashes, or the Python Universe.term_tables), uploaded when their sizes
 * changed or a relabel made them stale; every tree of the engine hashes rows through
 * them (dg_term_hashes, include/deltagpu.h). */
int dgr_refresh_terms(dgr_engine* g, const uint64_t* node_hash, uint64_t n_nodes,
                      const uint64_t* val_id, const uint64_t* val_hash, uint64_t n_vals);
/* A value relabel of the universe (marshal.h dgm_last_relabel): rewrites the val column of
 * every live state (dg_remap_values; ids move monotonically, stores stay sorted) and marks
 * the term tables stale.  Versions do not change: the terms the rows stand for do not. */
int dgr_remap(dgr_engine* g, const uint64_t* old_ids, const uint64_t* new_ids, uint64_t n);

/* A replica's state marshalled by a map walk (rows in any order, a context in any order:
 * a %{node => max} VV or a MapSet of dots) -> a device-resident state, version 1. */
int dgr_state_load(dgr_engine* g, const dg_store* rows, const dg_context* ctx, dgr_state** out);
int dgr_state_free(dgr_state* s);
uint64_t dgr_state_version(const dgr_state* s);
uint64_t dgr_state_rows(const dgr_state* s);
int dgr_state_has_tree(const dgr_state* s);

/* The result of a join on the state: the keys whose raw value maps changed (diff/3,
 * causal_crdt.ex:344-352), ascending by key id; their rows in the joined state (store
 * order: key, {value, ts}, dot -- the walk the NIF turns into value maps); the state's new
 * context.  Host views, valid until the next call on the engine. */
typedef struct dgr_changed {
  uint64_t version;
  uint64_t n_changed;
  const uint64_t* keys;
  dg_store rows;
  dg_context ctx;
} dgr_changed;

/* update_state_with_delta's join/3 (causal_crdt.ex:383-394; aw_lww_map.ex:153-209) of the
 * state with a delta (host rows and context in any order: the NIF's map walk) over `keys`
 * (host key ids, any order, duplicates allowed), in place on the device (dg_join_delta_rows),
 * with the tree's put/delete of the changed keys when a tree is built.  The delta, its
 * context and the keyset go down as ONE packed copy; the changed keys, their rows and the
 * new context come home with one wait. */
int dgr_join_delta(dgr_state* s, uint64_t version, const dg_store* delta, const dg_context* delta_ctx,
                   const uint64_t* keys, uint64_t n_keys, dgr_changed* out);

/* A batch of mutations by node `node` (m ops in the order they were made: kind 1 = add of
 * val[i] at ts[i], 0 = remove; keys host ids) as ONE delta built on the device
 * (dg_mutate_batch, aw_lww_map.ex:99-146) applied as dgr_join_delta applies one with the
 * touched keys.  The state's context must be a VV (CausalCrdt's, causal_crdt.ex:72). */
int dgr_mutate_batch(dgr_state* s, uint64_t version, uint32_t node, uint64_t m, const uint8_t* kind,
                     const uint64_t* key, const uint64_t* val, const int64_t* ts, dgr_changed* out);

/* read/1 (all != 0) or read/2 of `keys` (host ids, any order) (aw_lww_map.ex:211-224):
 * the winning value id per key, ascending by key id.  Host views. */
int dgr_read(dgr_state* s, uint64_t version, int all, const uint64_t* keys, uint64_t n_keys,
             const uint64_t** out_key, const uint64_t** out_val, uint64_t* n_out);

/* Map.take(value, keys) (causal_crdt.ex:118,331): the rows of those keys (host view). */
int dgr_take(dgr_state* s, uint64_t version, const uint64_t* keys, uint64_t n_keys, dg_store* out);

/* MerkleMap.new + put of every key (causal_crdt.ex:21): the state's tree, rows hashed
 * through the engine's term tables (refresh them first).  Rebuilding replaces it. */
int dgr_merkle_build(dgr_state* s, uint64_t version, uint32_t depth);

/* prepare_partial_diff(mm, levels) (:255) and continue_partial_diff + truncate (:96-105,
 * 206-214) with continuations as bytes: u32 level | u64 n | u64 n_buckets | pos[n] |
 * hash[n] | bucket[n_buckets] (little-endian).  continue: *status 1 -> *out_bin is the
 * next continuation (truncated to max_sync entries); 0 -> the first max_sync differing
 * keys in *keys (UINT64_MAX: :infinite).  Host views. */
int dgr_merkle_prepare(dgr_state* s, uint64_t version, uint32_t levels, const uint8_t** bin,
                       uint64_t* len);
int dgr_merkle_continue(dgr_state* s, uint64_t version, const uint8_t* bin, uint64_t len,
                        uint32_t levels, uint64_t max_sync, int* status, const uint8_t** out_bin,
                        uint64_t* out_len, const uint64_t** keys, uint64_t* n_keys);

#ifdef __cplusplus
}
#endif
#endif /* DG_REPLICA_H */
