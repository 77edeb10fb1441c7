/*
 * deltagpu_nif.c — the Erlang NIF that binds DeltaCrdt.AWLWWMap (reference
 * lib/delta_crdt/aw_lww_map.ex) and the MerkleMap role of DeltaCrdt.CausalCrdt
 * (lib/delta_crdt/causal_crdt.ex) to libdeltagpu (include/deltagpu.h).  Built by the
 * Elixir project against its OTP's erl_nif.h; this image has no
 * Erlang/OTP, so this file is not compiled here.  The term-independent half
 * (c_src/marshal.c: interning tables, host rows, unmarshal order) is, and is tested
 * from C with the same C-ABI calls this file makes (c_src/test_marshal.c).
 *
 * Resources
 *   engine   a dgr_engine (c_src/replica.h: one dg_engine, one HIP stream, engine-owned
 *            buffers) + the interning universe of this BEAM node + a mutex: every NIF
 *            below takes it (an engine is not re-entrant, and several CausalCrdt
 *            processes call in from several dirty schedulers).
 *   state    a DEVICE-RESIDENT replica state (a dgr_state: rows, context, spare buffer,
 *            tree) at a VERSION.  The Elixir struct keeps `dots` and `value` as real terms
 *            -- CausalCrdt reads them directly (causal_crdt.ex:118,259,331,346) -- and
 *            carries {state, version, pending} beside them; the device answers only the
 *            struct whose version it holds.
 *
 * This file is the term layer only: everything on the device is c_src/replica.c, which
 * the Python mirror of this NIF (delta_crdt_ex_amd/nif.py) and c_src/bench_mutate.c call
 * too.
 *
 * NIFs (dirty-CPU scheduled but resolve_keys; errors are {:error, :stale} for an older
 * struct and {:error, {code, message}} otherwise -- the Elixir side then uses the terms):
 *   engine_open(device)                                -> {:ok, engine}
 *   state_load(engine, dots, value)                    -> {:ok, state, version}
 *   join_delta(state, version, dots, value, keys)      -> {:ok, version', new_dots, changed}
 *        join/3 (aw_lww_map.ex:153-158) of the resident state with a delta
 *        %{dots: dots, value: value} over `keys`, in place on the device
 *        (dg_join_delta_rows); changed = [{key, value_map | nil}] for the keys whose raw
 *        value maps changed (causal_crdt.ex:344-352); the Merkle tree, if built, gets
 *        put/delete + update_hashes of them (:390-394).
 *   mutate_batch(state, version, node, ops)            -> {:ok, version', new_dots, changed}
 *        a batch of {:add, key, value, ts} / {:remove, key} ops by `node` as ONE delta
 *        (dg_mutate_batch, aw_lww_map.ex:99-146) applied like join_delta with the
 *        touched keys (the queued mutations of a GPU-attached replica)
 *   read(state, version, keys | :all)                  -> {:ok, %{key => value}}  (:211-224)
 *   take(state, version, keys)                         -> {:ok, value map}  (Map.take, :118,331)
 *   merkle_build(state, version, depth)                -> :ok
 *   merkle_prepare(state, version, levels)             -> {:continue, cont}     (:255)
 *   merkle_continue(state, version, cont, levels, max) -> {:continue, cont} | {:ok, keys}
 *        (:96-105; `max` is max_sync_size or :infinite, :98,105,206-214; a key this node
 *        never interned comes back as {:"$dg_key", id})
 *   resolve_keys(engine, keys)                         -> keys (placeholders -> terms)
 *   (a continuation is an opaque binary)
 */
#include <erl_nif.h>
#include <stdlib.h>
#include <string.h>

#include "../include/deltagpu.h"
#include "marshal.h"
#include "replica.h"

/* ------------------------------------------------------------ term operations */
/* Exact map-key order (the order a flatmap's {value, ts} keys are sorted in, which decides
 * read/1's tie-break, aw_lww_map.ex:211-216): the standard term order
 * number < atom < reference < fun < port < pid < tuple < map < list < bitstring, except
 * that numbers compare as map keys do -- every integer before every float ("in maps key
 * order integers types are considered less than floats types") -- recursively inside
 * tuples, lists and maps.  Leaves of one class other than numbers compare by enif_compare
 * (exact and arithmetic order agree there). */
static int term_rank(ErlNifEnv* env, ERL_NIF_TERM t) {
  switch (enif_term_type(env, t)) {
    case ERL_NIF_TERM_TYPE_INTEGER:
    case ERL_NIF_TERM_TYPE_FLOAT: return 0;
    case ERL_NIF_TERM_TYPE_ATOM: return 1;
    case ERL_NIF_TERM_TYPE_REFERENCE: return 2;
    case ERL_NIF_TERM_TYPE_FUN: return 3;
    case ERL_NIF_TERM_TYPE_PORT: return 4;
    case ERL_NIF_TERM_TYPE_PID: return 5;
    case ERL_NIF_TERM_TYPE_TUPLE: return 6;
    case ERL_NIF_TERM_TYPE_MAP: return 7;
    case ERL_NIF_TERM_TYPE_LIST: return 8;
    default: return 9; /* bitstring */
  }
}

static int sgn(int x) { return x < 0 ? -1 : x > 0; }
static int exact_cmp(ErlNifEnv* env, ERL_NIF_TERM a, ERL_NIF_TERM b);

/* a map's keys in map-key order (insertion sort: value maps are small) */
static ERL_NIF_TERM* sorted_keys(ErlNifEnv* env, ERL_NIF_TERM m, size_t n) {
  ERL_NIF_TERM* k = (ERL_NIF_TERM*)enif_alloc((n ? n : 1) * sizeof *k);
  ErlNifMapIterator it;
  ERL_NIF_TERM key, val;
  size_t i = 0;
  enif_map_iterator_create(env, m, &it, ERL_NIF_MAP_ITERATOR_FIRST);
  for (; i < n && enif_map_iterator_get_pair(env, &it, &key, &val); enif_map_iterator_next(env, &it)) {
    size_t j = i++;
    for (; j > 0 && exact_cmp(env, k[j - 1], key) > 0; j--) k[j] = k[j - 1];
    k[j] = key;
  }
  enif_map_iterator_destroy(env, &it);
  return k;
}

static int exact_cmp(ErlNifEnv* env, ERL_NIF_TERM a, ERL_NIF_TERM b) {
  const int ra = term_rank(env, a), rb = term_rank(env, b);
  if (ra != rb) return ra < rb ? -1 : 1;
  switch (ra) {
    case 0: {
      const int ia = enif_term_type(env, a) == ERL_NIF_TERM_TYPE_INTEGER;
      const int ib = enif_term_type(env, b) == ERL_NIF_TERM_TYPE_INTEGER;
      if (ia != ib) return ia ? -1 : 1;
      return sgn(enif_compare(a, b));
    }
    case 6: {
      int na, nb;
      const ERL_NIF_TERM *ea, *eb;
      enif_get_tuple(env, a, &na, &ea);
      enif_get_tuple(env, b, &nb, &eb);
      if (na != nb) return na < nb ? -1 : 1;
      for (int i = 0; i < na; i++) {
        const int x = exact_cmp(env, ea[i], eb[i]);
        if (x) return x;
      }
      return 0;
    }
    case 7: { /* size, then keys in key order, then values in key order */
      size_t na, nb;
      enif_get_map_size(env, a, &na);
      enif_get_map_size(env, b, &nb);
      if (na != nb) return na < nb ? -1 : 1;
      ERL_NIF_TERM *ka = sorted_keys(env, a, na), *kb = sorted_keys(env, b, nb);
      int x = 0;
      for (size_t i = 0; !x && i < na; i++) x = exact_cmp(env, ka[i], kb[i]);
      for (size_t i = 0; !x && i < na; i++) {
        ERL_NIF_TERM va, vb;
        enif_get_map_value(env, a, ka[i], &va);
        enif_get_map_value(env, b, kb[i], &vb);
        x = exact_cmp(env, va, vb);
      }
      enif_free(ka);
      enif_free(kb);
      return x;
    }
    case 8: /* element-wise, [] first; an improper tail compares as a term */
      for (;;) {
        const int ea = enif_is_empty_list(env, a), eb = enif_is_empty_list(env, b);
        if (ea || eb) return (ea && eb) ? 0 : (ea ? -1 : 1);
        ERL_NIF_TERM ha, ta, hb, tb;
        if (!enif_get_list_cell(env, a, &ha, &ta) || !enif_get_list_cell(env, b, &hb, &tb))
          return exact_cmp(env, a, b); /* a tail that is not a list: of another class */
        const int x = exact_cmp(env, ha, hb);
        if (x) return x;
        a = ta;
        b = tb;
      }
    default:
      return sgn(enif_compare(a, b));
  }
}

typedef struct {
  ErlNifEnv* env; /* the universe's own env: retained terms live here */
} term_ud;

typedef struct {
  ERL_NIF_TERM t;
} boxed;

static int op_cmp(const void* a, const void* b, void* ud) {
  term_ud* u = (term_ud*)ud;
  return exact_cmp(u->env, ((const boxed*)a)->t, ((const boxed*)b)->t);
}

/* The canonical encoding of a term (marshal.h; the Python mirror's interning.canon):
 * key ids, and the node / value term hashes of Merkle rows, are xxh64 of it, so they are
 * the same on every node.  Big integers come from the external term format's digits. */
static int encode_term(ErlNifEnv* env, ERL_NIF_TERM t, dgm_buf* b) {
  switch (enif_term_type(env, t)) {
    case ERL_NIF_TERM_TYPE_INTEGER: {
      ErlNifSInt64 i;
      ErlNifUInt64 u;
      if (enif_get_int64(env, t, &i)) return dgm_enc_i64(b, i);
      if (enif_get_uint64(env, t, &u)) return dgm_enc_u64(b, u);
      ErlNifBinary e; /* SMALL_BIG_EXT 110: n, sign, n digits LE; LARGE_BIG_EXT 111: u32 n */
      if (!enif_term_to_binary(env, t, &e)) return DG_E_NOMEM;
      int rc = DG_E_INVAL;
      if (e.size > 3 && e.data[1] == 110)
        rc = dgm_enc_int(b, e.data[3], e.data + 4, e.data[2]);
      else if (e.size > 6 && e.data[1] == 111)
        rc = dgm_enc_int(b, e.data[6], e.data + 7,
                         ((size_t)e.data[2] << 24) | ((size_t)e.data[3] << 16) | ((size_t)e.data[4] << 8) | e.data[5]);
      enif_release_binary(&e);
      return rc;
    }
    case ERL_NIF_TERM_TYPE_FLOAT: {
      double d;
      enif_get_double(env, t, &d);
      return dgm_enc_float(b, d);
    }
    case ERL_NIF_TERM_TYPE_ATOM: {
      unsigned len;
      if (!enif_get_atom_length(env, t, &len, ERL_NIF_UTF8)) return DG_E_INVAL;
      char* s = (char*)enif_alloc(len + 1);
      enif_get_atom(env, t, s, len + 1, ERL_NIF_UTF8);
      const int rc = dgm_enc_atom(b, s, len);
      enif_free(s);
      return rc;
    }
    case ERL_NIF_TERM_TYPE_BITSTRING: {
      ErlNifBinary bin;
      if (!enif_inspect_binary(env, t, &bin)) return DG_E_INVAL; /* not byte-aligned */
      return dgm_enc_binary(b, bin.data, bin.size);
    }
    case ERL_NIF_TERM_TYPE_TUPLE: {
      int n;
      const ERL_NIF_TERM* e;
      enif_get_tuple(env, t, &n, &e);
      int rc = dgm_enc_tuple(b, (uint32_t)n);
      for (int i = 0; !rc && i < n; i++) rc = encode_term(env, e[i], b);
      return rc;
    }
    case ERL_NIF_TERM_TYPE_LIST: {
      unsigned n;
      if (!enif_get_list_length(env, t, &n)) return DG_E_INVAL; /* improper: unsupported */
      int rc = dgm_enc_list(b, n);
      ERL_NIF_TERM h;
      while (!rc && enif_get_list_cell(env, t, &h, &t)) rc = encode_term(env, h, b);
      return rc;
    }
    case ERL_NIF_TERM_TYPE_MAP: {
      size_t n;
      enif_get_map_size(env, t, &n);
      ERL_NIF_TERM* k = sorted_keys(env, t, n);
      int rc = dgm_enc_map(b, (uint32_t)n);
      for (size_t i = 0; !rc && i < n; i++) {
        ERL_NIF_TERM v;
        enif_get_map_value(env, t, k[i], &v);
        rc = encode_term(env, k[i], b);
        if (!rc) rc = encode_term(env, v, b);
      }
      enif_free(k);
      return rc;
    }
    default: /* pids, ports, references, funs: node-local terms, not interned */
      return DG_E_INVAL;
  }
}

static int op_encode(const void* p, dgm_buf* b, void* ud) {
  term_ud* u = (term_ud*)ud;
  return encode_term(u->env, ((const boxed*)p)->t, b);
}

static void* op_keep(const void* p, void* ud) {
  term_ud* u = (term_ud*)ud;
  boxed* c = (boxed*)enif_alloc(sizeof *c);
  c->t = enif_make_copy(u->env, ((const boxed*)p)->t);
  return c;
}

static void op_drop(void* p, void* ud) {
  (void)ud;
  enif_free(p);
}

/* ------------------------------------------------------------ resources */
typedef struct {
  dgr_engine* r;   /* the device half: states, buffers, term tables (c_src/replica.h) */
  dgm_universe* u; /* the interning tables of this BEAM node */
  term_ud tu;
  ErlNifMutex* lock;
} engine_res;

typedef struct {
  engine_res* eng;
  dgr_state* s; /* the device-resident state; its version is in every struct that holds it */
} state_res;

static ErlNifResourceType* ENGINE_RT;
static ErlNifResourceType* STATE_RT;
static ERL_NIF_TERM A_OK, A_ERROR, A_NIL, A_ALL, A_CONTINUE, A_MAP, A_STRUCT, A_MAPSET, A_STALE,
    A_INFINITE, A_DGKEY;

static void engine_dtor(ErlNifEnv* env, void* obj) {
  (void)env;
  engine_res* r = (engine_res*)obj;
  if (r->r) dgr_engine_close(r->r); /* every state resource holds the engine: none is left */
  if (r->u) dgm_universe_free(r->u);
  if (r->tu.env) enif_free_env(r->tu.env);
  if (r->lock) enif_mutex_destroy(r->lock);
}

static void state_dtor(ErlNifEnv* env, void* obj) {
  (void)env;
  state_res* s = (state_res*)obj;
  engine_res* g = s->eng;
  enif_mutex_lock(g->lock);
  dgr_state_free(s->s);
  enif_mutex_unlock(g->lock);
  enif_release_resource(g);
}

/* {:error, :stale} for an older struct (its terms are authoritative: the Elixir side reads
 * or joins those on the CPU), {:error, {code, message}} otherwise */
static ERL_NIF_TERM error_term(ErlNifEnv* env, int rc) {
  if (rc == DGR_E_STALE) return enif_make_tuple2(env, A_ERROR, A_STALE);
  return enif_make_tuple2(env, A_ERROR,
                          enif_make_tuple2(env, enif_make_int(env, rc),
                                           enif_make_string(env, dg_last_error(), ERL_NIF_LATIN1)));
}

#define TRY(x)                          \
  do {                                  \
    int rc_ = (x);                      \
    if (rc_ != DG_OK) { rc = rc_; goto out; } \
  } while (0)

/* ------------------------------------------------------------ marshal */
/* The universe's term-hash tables to the device (when they grew or a relabel changed the
 * value ids); every tree of the engine hashes rows through them. */
static int refresh_terms(engine_res* g) {
  const uint64_t *nh, *vid, *vh;
  uint32_t nn;
  uint64_t nv;
  dgm_node_hashes(g->u, &nh, &nn);
  dgm_value_hashes(g->u, &vid, &vh, &nv);
  return dgr_refresh_terms(g->r, nh, nn, vid, vh, nv);
}

/* After any dgm_value that relabelled: every live state's val column rewritten
 * (dgr_remap).  Trees hash terms, so they stay valid; versions do not move. */
static int remap_live(engine_res* g) {
  const uint64_t *old_ids, *new_ids;
  uint64_t n;
  dgm_last_relabel(g->u, &old_ids, &new_ids, &n);
  return dgr_remap(g->r, old_ids, new_ids, n);
}

static int intern_value(ErlNifEnv* env, engine_res* g, ERL_NIF_TERM v, uint64_t* id) {
  boxed b = {v};
  (void)env;
  int relabeled = 0;
  int rc = dgm_value(g->u, &b, id, &relabeled);
  if (!rc && relabeled) rc = remap_live(g);
  return rc;
}

/* a MapSet's members: %MapSet{map: %{member => []}} (Elixir 1.7+) */
static int mapset_map(ErlNifEnv* env, ERL_NIF_TERM set, ERL_NIF_TERM* map) {
  return enif_get_map_value(env, set, A_MAP, map);
}

/* walk %{key => %{{v, ts} => MapSet[{node, counter}]}} in map order into host rows */
static int marshal_value(ErlNifEnv* env, engine_res* g, ERL_NIF_TERM value, dgm_rows* out) {
  ErlNifMapIterator ki, ei, di;
  ERL_NIF_TERM key, entries, vt, dots, dmap, dot, unused;
  /* pass 1: intern every value first (a relabel re-spaces ids already handed out) */
  if (!enif_map_iterator_create(env, value, &ki, ERL_NIF_MAP_ITERATOR_FIRST)) return DG_E_INVAL;
  for (; enif_map_iterator_get_pair(env, &ki, &key, &entries); enif_map_iterator_next(env, &ki)) {
    if (!enif_map_iterator_create(env, entries, &ei, ERL_NIF_MAP_ITERATOR_FIRST)) return DG_E_INVAL;
    for (; enif_map_iterator_get_pair(env, &ei, &vt, &dots); enif_map_iterator_next(env, &ei)) {
      int ar;
      const ERL_NIF_TERM* e;
      uint64_t id;
      if (!enif_get_tuple(env, vt, &ar, &e) || ar != 2 || intern_value(env, g, e[0], &id)) {
        enif_map_iterator_destroy(env, &ei);
        enif_map_iterator_destroy(env, &ki);
        return DG_E_INVAL;
      }
    }
    enif_map_iterator_destroy(env, &ei);
  }
  enif_map_iterator_destroy(env, &ki);
  /* pass 2: the rows */
  enif_map_iterator_create(env, value, &ki, ERL_NIF_MAP_ITERATOR_FIRST);
  for (; enif_map_iterator_get_pair(env, &ki, &key, &entries); enif_map_iterator_next(env, &ki)) {
    boxed bk = {key};
    uint64_t kid;
    if (dgm_key(g->u, &bk, &kid)) goto bad_k;
    enif_map_iterator_create(env, entries, &ei, ERL_NIF_MAP_ITERATOR_FIRST);
    for (; enif_map_iterator_get_pair(env, &ei, &vt, &dots); enif_map_iterator_next(env, &ei)) {
      int ar;
      const ERL_NIF_TERM* e;
      ErlNifSInt64 ts;
      uint64_t vid;
      int rl = 0;
      boxed bv;
      enif_get_tuple(env, vt, &ar, &e);
      bv.t = e[0];
      if (dgm_value(g->u, &bv, &vid, &rl) || rl || !enif_get_int64(env, e[1], &ts) ||
          !mapset_map(env, dots, &dmap) ||
          !enif_map_iterator_create(env, dmap, &di, ERL_NIF_MAP_ITERATOR_FIRST))
        goto bad_e;
      for (; enif_map_iterator_get_pair(env, &di, &dot, &unused); enif_map_iterator_next(env, &di)) {
        const ERL_NIF_TERM* d;
        ErlNifUInt64 cnt;
        uint32_t nid;
        boxed bn;
        if (!enif_get_tuple(env, dot, &ar, &d) || ar != 2 || !enif_get_uint64(env, d[1], &cnt)) goto bad_d;
        bn.t = d[0];
        if (dgm_node(g->u, &bn, &nid) || dgm_rows_push(out, kid, vid, ts, nid, cnt)) goto bad_d;
      }
      enif_map_iterator_destroy(env, &di);
    }
    enif_map_iterator_destroy(env, &ei);
  }
  enif_map_iterator_destroy(env, &ki);
  return DG_OK;
bad_d:
  enif_map_iterator_destroy(env, &di);
bad_e:
  enif_map_iterator_destroy(env, &ei);
bad_k:
  enif_map_iterator_destroy(env, &ki);
  return DG_E_INVAL;
}

/* a context: a MapSet of dots (DG_CTX_DOTS) or a %{node => max} VV (DG_CTX_VV) */
static int marshal_dots(ErlNifEnv* env, engine_res* g, ERL_NIF_TERM dots, dgm_rows* out) {
  ERL_NIF_TERM m, k, v, st;
  const int is_set = enif_get_map_value(env, dots, A_STRUCT, &st) && enif_is_identical(st, A_MAPSET);
  out->c.kind = is_set ? DG_CTX_DOTS : DG_CTX_VV;
  if (is_set) {
    if (!mapset_map(env, dots, &m)) return DG_E_INVAL;
  } else {
    m = dots;
  }
  ErlNifMapIterator it;
  if (!enif_map_iterator_create(env, m, &it, ERL_NIF_MAP_ITERATOR_FIRST)) return DG_E_INVAL;
  for (; enif_map_iterator_get_pair(env, &it, &k, &v); enif_map_iterator_next(env, &it)) {
    ERL_NIF_TERM node = k, cnt_t = v;
    int ar;
    const ERL_NIF_TERM* d;
    if (is_set) {
      if (!enif_get_tuple(env, k, &ar, &d) || ar != 2) goto bad;
      node = d[0];
      cnt_t = d[1];
    }
    ErlNifUInt64 cnt;
    uint32_t nid;
    boxed bn = {node};
    if (!enif_get_uint64(env, cnt_t, &cnt) || dgm_node(g->u, &bn, &nid) || dgm_ctx_push(out, nid, cnt))
      goto bad;
  }
  enif_map_iterator_destroy(env, &it);
  return DG_OK;
bad:
  enif_map_iterator_destroy(env, &it);
  return DG_E_INVAL;
}

/* {:"$dg_key", id}: a differing key this node never interned (only the peer holds it),
 * named by its id -- merkle_continue's {:ok, keys} holds such placeholders, every NIF
 * that takes keys accepts them as the id, and resolve_keys turns them back into terms on
 * a node that knows the key (the originator's get_diff, causal_crdt.ex:112-123). */
static int placeholder_id(ErlNifEnv* env, ERL_NIF_TERM t, uint64_t* id) {
  int ar;
  const ERL_NIF_TERM* e;
  ErlNifUInt64 x;
  if (!enif_get_tuple(env, t, &ar, &e) || ar != 2 || !enif_is_identical(e[0], A_DGKEY) ||
      !enif_get_uint64(env, e[1], &x))
    return 0;
  *id = x;
  return 1;
}

/* a key list -> host key ids (any order; the replica layer sorts them) */
static int marshal_keys(ErlNifEnv* env, engine_res* g, ERL_NIF_TERM keys, uint64_t** ids, uint64_t* n_keys) {
  unsigned len;
  *ids = NULL;
  *n_keys = 0;
  if (!enif_get_list_length(env, keys, &len)) return DG_E_INVAL;
  *ids = (uint64_t*)enif_alloc((len ? len : 1) * sizeof **ids);
  if (!*ids) return DG_E_NOMEM;
  ERL_NIF_TERM h, t = keys;
  unsigned n = 0;
  while (enif_get_list_cell(env, t, &h, &t)) {
    if (placeholder_id(env, h, &(*ids)[n])) {
      n++;
      continue;
    }
    boxed b = {h};
    if (dgm_key(g->u, &b, &(*ids)[n++])) return DG_E_INVAL;
  }
  *n_keys = n;
  return DG_OK;
}

/* the key's term, or {:"$dg_key", id} when this node never interned it */
static ERL_NIF_TERM key_term(ErlNifEnv* env, engine_res* g, uint64_t id) {
  const boxed* b = (const boxed*)dgm_key_term(g->u, id);
  if (b) return enif_make_copy(env, b->t);
  return enif_make_tuple2(env, A_DGKEY, enif_make_uint64(env, id));
}

/* ------------------------------------------------------------ unmarshal */
typedef struct {
  ErlNifEnv* env;
  engine_res* g;
  ERL_NIF_TERM out;     /* %{key => %{{v, ts} => MapSet}} being built */
  ERL_NIF_TERM entries; /* the current key's map */
  ERL_NIF_TERM dots;    /* the current entry's MapSet map */
  ERL_NIF_TERM key, vt;
  int open_key, open_entry;
} unm;

static ERL_NIF_TERM make_mapset(ErlNifEnv* env, ERL_NIF_TERM map) {
  ERL_NIF_TERM ks[3] = {A_STRUCT, A_MAP, enif_make_atom(env, "version")};
  ERL_NIF_TERM vs[3] = {A_MAPSET, map, enif_make_int(env, 2)};
  ERL_NIF_TERM s;
  enif_make_map_from_arrays(env, ks, vs, 3, &s);
  return s;
}

static void close_entry(unm* u) {
  if (u->open_entry) {
    enif_make_map_put(u->env, u->entries, u->vt, make_mapset(u->env, u->dots), &u->entries);
    u->open_entry = 0;
  }
}
static void close_key(unm* u) {
  close_entry(u);
  if (u->open_key) {
    enif_make_map_put(u->env, u->out, u->key, u->entries, &u->out);
    u->open_key = 0;
  }
}
static int u_key(void* ud, uint64_t key, uint64_t n) {
  (void)n;
  unm* u = (unm*)ud;
  close_key(u);
  const boxed* b = (const boxed*)dgm_key_term(u->g->u, key);
  if (!b) return DG_E_INVAL;
  u->key = enif_make_copy(u->env, b->t);
  u->entries = enif_make_new_map(u->env);
  u->open_key = 1;
  return 0;
}
/* the term of a value id: a canonical integer from its closed form, else the table's */
static int value_term(ErlNifEnv* env, engine_res* g, uint64_t id, ERL_NIF_TERM* out) {
  int64_t v;
  if (dgm_value_is_canonical(id, &v)) {
    *out = enif_make_int64(env, v);
    return DG_OK;
  }
  const boxed* b = (const boxed*)dgm_value_term(g->u, id);
  if (!b) return DG_E_INVAL;
  *out = enif_make_copy(env, b->t);
  return DG_OK;
}

static int u_entry(void* ud, uint64_t val, int64_t ts, uint64_t n) {
  (void)n;
  unm* u = (unm*)ud;
  close_entry(u);
  ERL_NIF_TERM vt;
  if (value_term(u->env, u->g, val, &vt)) return DG_E_INVAL;
  u->vt = enif_make_tuple2(u->env, vt, enif_make_int64(u->env, ts));
  u->dots = enif_make_new_map(u->env);
  u->open_entry = 1;
  return 0;
}
static int u_dot(void* ud, uint32_t node, uint64_t cnt) {
  unm* u = (unm*)ud;
  const boxed* b = (const boxed*)dgm_node_term(u->g->u, node);
  if (!b) return DG_E_INVAL;
  ERL_NIF_TERM d = enif_make_tuple2(u->env, enif_make_copy(u->env, b->t), enif_make_uint64(u->env, cnt));
  enif_make_map_put(u->env, u->dots, d, enif_make_list(u->env, 0), &u->dots);
  return 0;
}

/* host rows -> %{key => value map} */
static int unmarshal_host_rows(ErlNifEnv* env, engine_res* g, const dg_store* h, ERL_NIF_TERM* out) {
  unm u;
  memset(&u, 0, sizeof u);
  u.env = env;
  u.g = g;
  u.out = enif_make_new_map(env);
  dgm_walk w = {u_key, u_entry, u_dot};
  const int rc = dgm_walk_rows(h, &w, &u);
  close_key(&u);
  *out = u.out;
  return rc;
}

/* a host context -> a %{node => max} VV or a MapSet of dots */
static int unmarshal_dots(ErlNifEnv* env, engine_res* g, const dg_context* c, ERL_NIF_TERM* out) {
  ERL_NIF_TERM m = enif_make_new_map(env);
  for (uint64_t i = 0; i < c->n; i++) {
    const boxed* b = (const boxed*)dgm_node_term(g->u, c->node[i]);
    if (!b) return DG_E_INVAL;
    ERL_NIF_TERM n = enif_make_copy(env, b->t), k = enif_make_uint64(env, c->cnt[i]);
    if (c->kind == DG_CTX_VV)
      enif_make_map_put(env, m, n, k, &m);
    else
      enif_make_map_put(env, m, enif_make_tuple2(env, n, k), enif_make_list(env, 0), &m);
  }
  *out = c->kind == DG_CTX_VV ? m : make_mapset(env, m);
  return DG_OK;
}

/* ------------------------------------------------------------ NIFs */
static ERL_NIF_TERM engine_open(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  (void)argc;
  int dev;
  if (!enif_get_int(env, argv[0], &dev)) return enif_make_badarg(env);
  engine_res* g = (engine_res*)enif_alloc_resource(ENGINE_RT, sizeof *g);
  memset(g, 0, sizeof *g);
  g->lock = enif_mutex_create("deltagpu_engine");
  g->tu.env = enif_alloc_env();
  dgm_term_ops ops = {op_cmp, op_encode, NULL, op_keep, op_drop, &g->tu};
  g->u = dgm_universe_new(&ops);
  const int rc = dgr_engine_open(dev, &g->r);
  ERL_NIF_TERM r = rc ? error_term(env, rc) : enif_make_tuple2(env, A_OK, enif_make_resource(env, g));
  enif_release_resource(g);
  return r;
}

static int get_state(ErlNifEnv* env, ERL_NIF_TERM t, ERL_NIF_TERM v, state_res** s, uint64_t* version) {
  ErlNifUInt64 x;
  if (!enif_get_resource(env, t, STATE_RT, (void**)s) || !enif_get_uint64(env, v, &x)) return 0;
  *version = x;
  return 1;
}

/* state_load(engine, dots, value) -> {:ok, state, version} */
static ERL_NIF_TERM state_load(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  (void)argc;
  engine_res* g;
  if (!enif_get_resource(env, argv[0], ENGINE_RT, (void**)&g)) return enif_make_badarg(env);
  enif_mutex_lock(g->lock);
  dgm_rows h;
  dgr_state* ds = NULL;
  int rc = dgm_rows_init(&h, 1024, 64);
  ERL_NIF_TERM r;
  if (!rc) rc = marshal_dots(env, g, argv[1], &h);
  if (!rc) rc = marshal_value(env, g, argv[2], &h);
  if (!rc) rc = dgr_state_load(g->r, &h.s, &h.c, &ds);
  dgm_rows_free(&h);
  if (rc) {
    r = error_term(env, rc);
  } else {
    state_res* s = (state_res*)enif_alloc_resource(STATE_RT, sizeof *s);
    enif_keep_resource(g);
    s->eng = g;
    s->s = ds;
    r = enif_make_tuple3(env, A_OK, enif_make_resource(env, s), enif_make_uint64(env, dgr_state_version(ds)));
    enif_release_resource(s);
  }
  enif_mutex_unlock(g->lock);
  return r;
}

/* {:ok, version, new_dots, [{key, value_map | nil}]} from a join's result: the changed
 * keys' rows (in key order) walked into value maps, the context into its term */
static int changed_result(ErlNifEnv* env, engine_res* g, const dgr_changed* c, ERL_NIF_TERM* r) {
  ERL_NIF_TERM values, dots, changed = enif_make_list(env, 0);
  int rc = unmarshal_host_rows(env, g, &c->rows, &values);
  if (!rc) rc = unmarshal_dots(env, g, &c->ctx, &dots);
  if (rc) return rc;
  for (uint64_t i = c->n_changed; i-- > 0;) {
    const boxed* b = (const boxed*)dgm_key_term(g->u, c->keys[i]);
    if (!b) return DG_E_INVAL;
    ERL_NIF_TERM k = enif_make_copy(env, b->t), v;
    if (!enif_get_map_value(env, values, k, &v)) v = A_NIL; /* the key's entries all went */
    changed = enif_make_list_cell(env, enif_make_tuple2(env, k, v), changed);
  }
  *r = enif_make_tuple4(env, A_OK, enif_make_uint64(env, c->version), dots, changed);
  return DG_OK;
}

/* join_delta(state, version, dots, value, keys) -> {:ok, version', new_dots, changed}
 * join/3 (aw_lww_map.ex:153-158) of the resident state with the delta %{dots, value} over
 * `keys`, in place on the device; `changed` = the keys whose raw value maps changed
 * (causal_crdt.ex:344-352) with their new maps; the tree (if built) gets their put/delete. */
static ERL_NIF_TERM join_delta(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  (void)argc;
  state_res* s;
  uint64_t version;
  if (!get_state(env, argv[0], argv[1], &s, &version)) return enif_make_badarg(env);
  engine_res* g = s->eng;
  enif_mutex_lock(g->lock);
  int rc = DG_OK;
  dgm_rows h;
  uint64_t *keys = NULL, n_keys = 0;
  dgr_changed c;
  ERL_NIF_TERM r = A_NIL;
  TRY(dgm_rows_init(&h, 256, 16));
  TRY(marshal_dots(env, g, argv[2], &h));
  TRY(marshal_value(env, g, argv[3], &h));
  TRY(marshal_keys(env, g, argv[4], &keys, &n_keys));
  if (dgr_state_has_tree(s->s)) TRY(refresh_terms(g));
  TRY(dgr_join_delta(s->s, version, &h.s, &h.c, keys, n_keys, &c));
  TRY(changed_result(env, g, &c, &r));
out:
  if (rc) r = error_term(env, rc);
  dgm_rows_free(&h);
  if (keys) enif_free(keys);
  enif_mutex_unlock(g->lock);
  return r;
}

/* mutate_batch(state, version, node, ops) -> {:ok, version', new_dots, changed}: a batch of
 * mutations by `node` -- ops = [{:add, key, value, ts} | {:remove, key}] in the order they
 * were made (the queued mutations of a GPU-attached replica, causal_crdt.ex:196-198,
 * 337-342) -- as ONE delta built on the device (dg_mutate_batch: per touched key the last
 * op's row if it is an add, context = the touched keys' dots plus every add's dot,
 * aw_lww_map.ex:99-146), applied like join_delta with the touched keys. */
static ERL_NIF_TERM mutate_batch_nif(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  (void)argc;
  state_res* s;
  uint64_t version;
  unsigned m;
  if (!get_state(env, argv[0], argv[1], &s, &version) || !enif_get_list_length(env, argv[3], &m))
    return enif_make_badarg(env);
  engine_res* g = s->eng;
  enif_mutex_lock(g->lock);
  int rc = DG_OK;
  uint32_t node = 0;
  dgr_changed c;
  ERL_NIF_TERM r = A_NIL, head, tail = argv[3];
  uint8_t* kind = (uint8_t*)enif_alloc(m ? m : 1);
  uint64_t* key = (uint64_t*)enif_alloc((m ? m : 1) * 8);
  uint64_t* val = (uint64_t*)enif_alloc((m ? m : 1) * 8);
  int64_t* ts = (int64_t*)enif_alloc((m ? m : 1) * 8);
  if (!kind || !key || !val || !ts) {
    rc = DG_E_NOMEM;
    goto out;
  }
  {
    boxed bn = {argv[2]};
    TRY(dgm_node(g->u, &bn, &node));
  }
  /* pass 1: every value interned (a relabel re-spaces ids already handed out) */
  for (unsigned i = 0; i < m; i++) {
    int ar;
    const ERL_NIF_TERM* e;
    if (!enif_get_list_cell(env, tail, &head, &tail) || !enif_get_tuple(env, head, &ar, &e) ||
        (ar != 2 && ar != 4)) {
      rc = DG_E_INVAL;
      goto out;
    }
    kind[i] = ar == 4;
    val[i] = 0;
    ts[i] = 0;
    if (ar == 4) {
      ErlNifSInt64 t;
      if (!enif_get_int64(env, e[3], &t)) {
        rc = DG_E_INVAL;
        goto out;
      }
      ts[i] = t;
      TRY(intern_value(env, g, e[2], &val[i]));
    }
  }
  /* pass 2: keys, and the value ids as they stand after any relabel */
  tail = argv[3];
  for (unsigned i = 0; i < m; i++) {
    int ar;
    const ERL_NIF_TERM* e;
    enif_get_list_cell(env, tail, &head, &tail);
    enif_get_tuple(env, head, &ar, &e);
    boxed bk = {e[1]};
    TRY(dgm_key(g->u, &bk, &key[i]));
    if (ar == 4) {
      boxed bv = {e[2]};
      int relabeled = 0;
      TRY(dgm_value(g->u, &bv, &val[i], &relabeled));
      if (relabeled) TRY(remap_live(g));
    }
  }
  if (dgr_state_has_tree(s->s)) TRY(refresh_terms(g));
  TRY(dgr_mutate_batch(s->s, version, node, m, kind, key, val, ts, &c));
  TRY(changed_result(env, g, &c, &r));
out:
  if (rc) r = error_term(env, rc);
  if (kind) enif_free(kind);
  if (key) enif_free(key);
  if (val) enif_free(val);
  if (ts) enif_free(ts);
  enif_mutex_unlock(g->lock);
  return r;
}

/* read(state, version, keys | :all) -> {:ok, %{key => value}}  (read/1,2, :211-224) */
static ERL_NIF_TERM read_nif(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  (void)argc;
  state_res* s;
  uint64_t version;
  if (!get_state(env, argv[0], argv[1], &s, &version)) return enif_make_badarg(env);
  engine_res* g = s->eng;
  enif_mutex_lock(g->lock);
  int rc = DG_OK;
  uint64_t *keys = NULL, n_keys = 0, n = 0;
  const uint64_t *hk = NULL, *hv = NULL;
  ERL_NIF_TERM r, m = enif_make_new_map(env);
  const int all = enif_is_identical(argv[2], A_ALL);
  if (!all) TRY(marshal_keys(env, g, argv[2], &keys, &n_keys));
  TRY(dgr_read(s->s, version, all, keys, n_keys, &hk, &hv, &n));
  for (uint64_t i = 0; i < n; i++) {
    const boxed* k = (const boxed*)dgm_key_term(g->u, hk[i]);
    ERL_NIF_TERM v;
    TRY(value_term(env, g, hv[i], &v));
    enif_make_map_put(env, m, enif_make_copy(env, k->t), v, &m);
  }
out:
  r = rc ? error_term(env, rc) : enif_make_tuple2(env, A_OK, m);
  if (keys) enif_free(keys);
  enif_mutex_unlock(g->lock);
  return r;
}

/* take(state, version, keys) -> {:ok, value map of those keys}  (Map.take, :118,331) */
static ERL_NIF_TERM take_nif(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  (void)argc;
  state_res* s;
  uint64_t version;
  if (!get_state(env, argv[0], argv[1], &s, &version)) return enif_make_badarg(env);
  engine_res* g = s->eng;
  enif_mutex_lock(g->lock);
  int rc = DG_OK;
  uint64_t *keys = NULL, n_keys = 0;
  dg_store taken;
  ERL_NIF_TERM r, values = A_NIL;
  TRY(marshal_keys(env, g, argv[2], &keys, &n_keys));
  TRY(dgr_take(s->s, version, keys, n_keys, &taken));
  TRY(unmarshal_host_rows(env, g, &taken, &values));
out:
  r = rc ? error_term(env, rc) : enif_make_tuple2(env, A_OK, values);
  if (keys) enif_free(keys);
  enif_mutex_unlock(g->lock);
  return r;
}

/* merkle_build(state, version, depth) -> :ok  (MerkleMap.new + put of every key, :21) */
static ERL_NIF_TERM merkle_build_nif(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  (void)argc;
  state_res* s;
  uint64_t version;
  unsigned depth;
  if (!get_state(env, argv[0], argv[1], &s, &version) || !enif_get_uint(env, argv[2], &depth))
    return enif_make_badarg(env);
  engine_res* g = s->eng;
  enif_mutex_lock(g->lock);
  int rc = refresh_terms(g);
  if (!rc) rc = dgr_merkle_build(s->s, version, depth);
  ERL_NIF_TERM r = rc ? error_term(env, rc) : A_OK;
  enif_mutex_unlock(g->lock);
  return r;
}

static ERL_NIF_TERM bytes_term(ErlNifEnv* env, const uint8_t* p, uint64_t n) {
  ERL_NIF_TERM t;
  unsigned char* d = enif_make_new_binary(env, n, &t);
  memcpy(d, p, n);
  return t;
}

/* merkle_prepare(state, version, levels) -> {:continue, cont}  (:255) */
static ERL_NIF_TERM merkle_prepare_nif(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  (void)argc;
  state_res* s;
  uint64_t version;
  unsigned levels;
  if (!get_state(env, argv[0], argv[1], &s, &version) || !enif_get_uint(env, argv[2], &levels))
    return enif_make_badarg(env);
  engine_res* g = s->eng;
  enif_mutex_lock(g->lock);
  const uint8_t* bin = NULL;
  uint64_t len = 0;
  const int rc = dgr_merkle_prepare(s->s, version, levels, &bin, &len);
  ERL_NIF_TERM r = rc ? error_term(env, rc) : enif_make_tuple2(env, A_CONTINUE, bytes_term(env, bin, len));
  enif_mutex_unlock(g->lock);
  return r;
}

/* merkle_continue(state, version, cont, levels, max_sync_size | :infinite)
 *   -> {:continue, cont} | {:ok, keys}  (continue_partial_diff + truncate, :96-105,206-214) */
static ERL_NIF_TERM merkle_continue_nif(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  (void)argc;
  state_res* s;
  uint64_t version;
  ErlNifBinary in;
  unsigned levels;
  ErlNifUInt64 max_sync = UINT64_MAX;
  if (!get_state(env, argv[0], argv[1], &s, &version) || !enif_inspect_binary(env, argv[2], &in) ||
      !enif_get_uint(env, argv[3], &levels) ||
      (!enif_is_identical(argv[4], A_INFINITE) && !enif_get_uint64(env, argv[4], &max_sync)))
    return enif_make_badarg(env);
  engine_res* g = s->eng;
  enif_mutex_lock(g->lock);
  int rc = DG_OK, status = 0;
  const uint8_t* bin = NULL;
  const uint64_t* keys = NULL;
  uint64_t len = 0, n_keys = 0;
  ERL_NIF_TERM r = A_NIL;
  TRY(refresh_terms(g));
  TRY(dgr_merkle_continue(s->s, version, in.data, in.size, levels, max_sync, &status, &bin, &len, &keys,
                          &n_keys));
  if (status == 1) {
    r = enif_make_tuple2(env, A_CONTINUE, bytes_term(env, bin, len));
  } else {
    ERL_NIF_TERM l = enif_make_list(env, 0);
    for (uint64_t i = n_keys; i-- > 0;) l = enif_make_list_cell(env, key_term(env, g, keys[i]), l);
    r = enif_make_tuple2(env, A_OK, l);
  }
out:
  if (rc) r = error_term(env, rc);
  enif_mutex_unlock(g->lock);
  return r;
}

/* resolve_keys(engine, keys) -> keys: placeholders of keys this node knows -> their terms
 * (the others stay placeholders) */
static ERL_NIF_TERM resolve_keys_nif(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  (void)argc;
  engine_res* g;
  unsigned len;
  if (!enif_get_resource(env, argv[0], ENGINE_RT, (void**)&g) || !enif_get_list_length(env, argv[1], &len))
    return enif_make_badarg(env);
  enif_mutex_lock(g->lock);
  ERL_NIF_TERM* v = (ERL_NIF_TERM*)enif_alloc((len ? len : 1) * sizeof *v);
  ERL_NIF_TERM h, t = argv[1], r;
  unsigned n = 0;
  while (enif_get_list_cell(env, t, &h, &t)) {
    uint64_t id;
    v[n++] = placeholder_id(env, h, &id) ? key_term(env, g, id) : h;
  }
  r = enif_make_list_from_array(env, v, n);
  enif_free(v);
  enif_mutex_unlock(g->lock);
  return r;
}

/* ------------------------------------------------------------ load */
static int load(ErlNifEnv* env, void** priv, ERL_NIF_TERM info) {
  (void)priv;
  (void)info;
  ENGINE_RT = enif_open_resource_type(env, NULL, "deltagpu_engine", engine_dtor, ERL_NIF_RT_CREATE, NULL);
  STATE_RT = enif_open_resource_type(env, NULL, "deltagpu_state", state_dtor, ERL_NIF_RT_CREATE, NULL);
  A_OK = enif_make_atom(env, "ok");
  A_ERROR = enif_make_atom(env, "error");
  A_NIL = enif_make_atom(env, "nil");
  A_ALL = enif_make_atom(env, "all");
  A_CONTINUE = enif_make_atom(env, "continue");
  A_MAP = enif_make_atom(env, "map");
  A_STRUCT = enif_make_atom(env, "__struct__");
  A_MAPSET = enif_make_atom(env, "Elixir.MapSet");
  A_STALE = enif_make_atom(env, "stale");
  A_INFINITE = enif_make_atom(env, "infinite");
  A_DGKEY = enif_make_atom(env, "$dg_key");
  return (ENGINE_RT && STATE_RT) ? 0 : 1;  /* a failed load -> the Elixir code path */
}

static ErlNifFunc funcs[] = {
    {"engine_open", 1, engine_open, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"state_load", 3, state_load, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"join_delta", 5, join_delta, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"mutate_batch", 4, mutate_batch_nif, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"read", 3, read_nif, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"take", 3, take_nif, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"merkle_build", 3, merkle_build_nif, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"merkle_prepare", 3, merkle_prepare_nif, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"merkle_continue", 5, merkle_continue_nif, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"resolve_keys", 2, resolve_keys_nif, 0},
};

ERL_NIF_INIT(Elixir.DeltaCrdt.GPU, funcs, load, NULL, NULL, NULL)
