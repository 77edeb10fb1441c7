/*
 * marshal.h — the term-independent half of the Erlang NIF (c_src/deltagpu_nif.c) that
 * binds DeltaCrdt.AWLWWMap (reference lib/delta_crdt/aw_lww_map.ex) to libdeltagpu
 * (include/deltagpu.h).  Everything here is plain C over opaque term handles, so it
 * builds and is unit-tested without erl_nif.h (c_src/test_marshal.c); the NIF supplies
 * the term operations (enif_compare with the exact map-key tie-break, a stable hash of
 * the external term format, enif_make_copy into a process-independent env).
 *
 *   dgm_universe   the interning tables of one engine (all replicas of one BEAM node):
 *                    key   -> u64 id   (the caller's stable 64-bit hash; collisions are
 *                                       detected exactly and reported)
 *                    value -> u64 id   ORDER-PRESERVING in Erlang term order, the read
 *                                       tie-break of aw_lww_map.ex:211-216:
 *                                       gapped ranks, re-spaced when a gap is used up;
 *                                       the caller then rewrites its device stores with
 *                                       dg_remap_values(old ids, new ids)
 *                    node  -> u32 id   dense, in first-seen order (real node ids are
 *                                       :rand.uniform(1_000_000_000), causal_crdt.ex:65)
 *   dgm_rows       growable host SoA rows + context, filled by a map walk in any order
 *                  (dg_sort_store orders them on the device)
 *   dgm_walk_rows  the unmarshal order: key runs -> {value, ts} entries -> dots.
 */
#ifndef DG_MARSHAL_H
#define DG_MARSHAL_H

#include <stddef.h>
#include <stdint.h>

#include "../include/deltagpu.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct dgm_term_ops {
  /* exact Erlang term order: < 0, 0 (only for =:= terms), > 0 */
  int (*cmp)(const void* a, const void* b, void* ud);
  /* a stable 64-bit hash (the key id of a key term) */
  uint64_t (*hash)(const void* t, void* ud);
  /* a retained copy of the term (owned by the universe) and its release */
  void* (*keep)(const void* t, void* ud);
  void (*drop)(void* t, void* ud);
  void* ud;
} dgm_term_ops;

typedef struct dgm_universe dgm_universe;

dgm_universe* dgm_universe_new(const dgm_term_ops* ops);
void dgm_universe_free(dgm_universe* u);

/* 0 = ok, DG_E_INVAL on a 64-bit key-id collision between two distinct terms */
int dgm_key(dgm_universe* u, const void* term, uint64_t* id);
const void* dgm_key_term(const dgm_universe* u, uint64_t id); /* NULL if unknown */

/* *relabeled = 1 when this insert re-spaced every value id: dgm_last_relabel then
 * hands out the (old, new) id arrays, both ascending, for dg_remap_values. */
int dgm_value(dgm_universe* u, const void* term, uint64_t* id, int* relabeled);
const void* dgm_value_term(const dgm_universe* u, uint64_t id); /* NULL if unknown */
void dgm_last_relabel(const dgm_universe* u, const uint64_t** old_ids, const uint64_t** new_ids,
                      uint64_t* n);
uint64_t dgm_value_count(const dgm_universe* u);

int dgm_node(dgm_universe* u, const void* term, uint32_t* id);
const void* dgm_node_term(const dgm_universe* u, uint32_t id); /* NULL if unknown */
uint32_t dgm_node_count(const dgm_universe* u);

/* host rows and a context, grown on demand (the columns of a dg_store / dg_context) */
typedef struct dgm_rows {
  dg_store s;
  dg_context c;
} dgm_rows;

int dgm_rows_init(dgm_rows* r, uint64_t cap_rows, uint64_t cap_ctx);
void dgm_rows_free(dgm_rows* r);
void dgm_rows_clear(dgm_rows* r);
int dgm_rows_push(dgm_rows* r, uint64_t key, uint64_t val, int64_t ts, uint32_t node, uint64_t cnt);
int dgm_ctx_push(dgm_rows* r, uint32_t node, uint64_t cnt);

/* Walk SORTED rows: key() once per key run, entry() once per {val, ts} entry of it,
 * dot() once per row.  A callback returning nonzero stops the walk with that value. */
typedef struct dgm_walk {
  int (*key)(void* ud, uint64_t key, uint64_t n_entries);
  int (*entry)(void* ud, uint64_t val, int64_t ts, uint64_t n_dots);
  int (*dot)(void* ud, uint32_t node, uint64_t cnt);
} dgm_walk;

int dgm_walk_rows(const dg_store* rows, const dgm_walk* w, void* ud);

/* The stable 64-bit hash the NIF uses for key ids: xxh64-style over bytes (the
 * external term format of the key). */
uint64_t dgm_hash_bytes(const void* p, size_t n, uint64_t seed);

#ifdef __cplusplus
}
#endif
#endif /* DG_MARSHAL_H */
