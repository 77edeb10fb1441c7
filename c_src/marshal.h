/*
 * marshal.h — the term-independent half of the Erlang NIF (c_src/deltagpu_nif.c) that
 * binds DeltaCrdt.AWLWWMap (reference lib/delta_crdt/aw_lww_map.ex) to libdeltagpu
 * (include/deltagpu.h).  Everything here is plain C over opaque term handles, so it
 * builds and is unit-tested without erl_nif.h (c_src/test_marshal.c); the NIF supplies
 * the term operations (enif_compare with the exact map-key tie-break, a stable hash of
 * the external term format, enif_make_copy into a process-independent env).
 *
 *   dgm_universe   the interning tables of one engine (all replicas of one BEAM node):
 *                    key   -> u64 id   integers 0 <= k < 2^64: splitmix64(k); any other term:
 *                                       xxh64 of its canonical encoding (collisions are
 *                                       detected exactly and reported)
 *                    value -> u64 id   ORDER-PRESERVING in map-key order, the read tie-break
 *                                       of aw_lww_map.ex:211-216: integers in
 *                                       [DGM_CANON_LO, 2^62) have the closed-form id v + 2^62
 *                                       (the same on every node); other terms gapped ranks in
 *                                       two regions around them, re-spaced when a gap is used
 *                                       up (the caller then rewrites its device stores with
 *                                       dg_remap_values(old ids, new ids))
 *                    node  -> u32 id   dense, in first-seen order (real node ids are
 *                                       :rand.uniform(1_000_000_000), causal_crdt.ex:65)
 *                  plus the term hashes of nodes and table values (dg_term_hashes): Merkle
 *                  trees built with them compare across universes and BEAM nodes
 *   dgm_buf        the canonical encoding of a term, built by the caller's term walk with
 *                  dgm_enc_* (the Python mirror's interning.canon writes the same bytes)
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

/* ------------------------------------------------------------ canonical encoding */
/* A tag byte and a little-endian u32 length, then (delta_crdt_ex_amd/interning.py canon):
 *   a <utf8 text>   atom          i <sign 0|1><magnitude, little-endian, minimal>  integer
 *   f <f64 LE>      float (no length field)                 b <bytes>     binary
 *   t <n> elements  tuple         l <n> elements  proper list
 *   m <n> pairs     map, (key, value) pairs in map-key order of the keys */
typedef struct dgm_buf {
  unsigned char* p;
  size_t n, cap;
} dgm_buf;

void dgm_buf_free(dgm_buf* b);
int dgm_enc_atom(dgm_buf* b, const char* utf8, size_t n);
int dgm_enc_int(dgm_buf* b, int negative, const unsigned char* mag_le, size_t n);
int dgm_enc_i64(dgm_buf* b, int64_t v);
int dgm_enc_u64(dgm_buf* b, uint64_t v);
int dgm_enc_float(dgm_buf* b, double v);
int dgm_enc_binary(dgm_buf* b, const void* p, size_t n);
int dgm_enc_tuple(dgm_buf* b, uint32_t arity); /* then the elements */
int dgm_enc_list(dgm_buf* b, uint32_t len);    /* then the elements */
int dgm_enc_map(dgm_buf* b, uint32_t size);    /* then key, value, ... in key order */

/* Seeds of the term hashes: xxh64(canonical encoding, seed). */
#define DGM_NODE_SEED 0x6E6F6465ull
#define DGM_VAL_SEED 0x76616C75ull
/* The canonical integer values [DGM_CANON_LO, DGM_CANON_HI) and their ids v + 2^62. */
#define DGM_CANON_LO (-(INT64_C(1) << 62) + (INT64_C(1) << 58))
#define DGM_CANON_HI (INT64_C(1) << 62)

/* The key id of an encoded term (integer 0 <= k < 2^64: splitmix64(k), else xxh64 seed 0). */
uint64_t dgm_key_id(const unsigned char* enc, size_t n);
/* 1 and *v = the integer when `id` is a canonical value id (closed form), else 0. */
int dgm_value_is_canonical(uint64_t id, int64_t* v);

typedef struct dgm_term_ops {
  /* exact map-key order (integers before floats, recursively): < 0, 0 (=:= terms), > 0 */
  int (*cmp)(const void* a, const void* b, void* ud);
  /* append the term's canonical encoding to buf (DG_OK, or an error: an unsupported term) */
  int (*encode)(const void* t, dgm_buf* buf, void* ud);
  /* optional: the key id instead of dgm_key_id (tests force collisions with it) */
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

/* *relabeled = 1 when this insert re-spaced the value ids of its region: dgm_last_relabel
 * then hands out the (old, new) id arrays, both ascending, for dg_remap_values. */
int dgm_value(dgm_universe* u, const void* term, uint64_t* id, int* relabeled);
/* The term of a table value id; NULL if unknown and for canonical integer ids (the caller
 * makes those from dgm_value_is_canonical). */
const void* dgm_value_term(const dgm_universe* u, uint64_t id);
void dgm_last_relabel(const dgm_universe* u, const uint64_t** old_ids, const uint64_t** new_ids,
                      uint64_t* n);
uint64_t dgm_value_count(const dgm_universe* u);

int dgm_node(dgm_universe* u, const void* term, uint32_t* id);
const void* dgm_node_term(const dgm_universe* u, uint32_t id); /* NULL if unknown */
uint32_t dgm_node_count(const dgm_universe* u);

/* The term-hash tables of dg_term_hashes (include/deltagpu.h), host arrays owned by the
 * universe (valid until its next insert): node_hash[dense node id], and the table value
 * ids (ascending) with their hashes.  Upload them and point a dg_term_hashes at the copies. */
void dgm_node_hashes(const dgm_universe* u, const uint64_t** hash, uint32_t* n);
void dgm_value_hashes(const dgm_universe* u, const uint64_t** ids, const uint64_t** hash,
                      uint64_t* n);

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

/* xxh64 of bytes (the term hash of a canonical encoding). */
uint64_t dgm_hash_bytes(const void* p, size_t n, uint64_t seed);

#ifdef __cplusplus
}
#endif
#endif /* DG_MARSHAL_H */
