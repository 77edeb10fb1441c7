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
 *   engine   one dg_engine (one HIP stream) + the interning universe of this BEAM node
 *            + a mutex: every NIF below takes it (a dg_engine is not re-entrant, and
 *            several CausalCrdt processes call in from several dirty schedulers).
 *   state    a DEVICE-RESIDENT replica state: rows, context and, once built, its Merkle
 *            tree.  The Elixir struct keeps `dots` and `value` as real terms -- CausalCrdt
 *            reads them directly (causal_crdt.ex:118,259,331,346) -- and carries the
 *            state resource beside them, so a join ships only the delta to the device
 *            and brings back only the keys it changed.
 *
 * NIFs (all dirty-CPU scheduled; errors are {:error, reason}, the Elixir side then
 * runs the reference code instead):
 *   engine_open(device)                       -> {:ok, engine}
 *   state_load(engine, dots, value)           -> {:ok, state}          (marshal once)
 *   join_delta(state, dots, value, keys)      -> {:ok, new_dots, changed}
 *        join/3 (aw_lww_map.ex:153-158) of the resident state with a delta
 *        %{dots: dots, value: value} over `keys`, in place on the device
 *        (dg_join_delta: in place when every joined key keeps its row count);
 *        changed = [{key, value_map | nil}] for the keys whose raw
 *        value maps changed (causal_crdt.ex:344-352), so the caller updates its term
 *        map with Map.merge/Map.drop of those keys only; the Merkle tree, if built,
 *        gets put/delete + update_hashes of them (dg_merkle_update, :390-394).
 *   mutate_batch(state, node, ops)            -> {:ok, new_dots, changed}
 *        a batch of {:add, key, value, ts} / {:remove, key} ops by `node` as ONE delta
 *        (dg_mutate_batch, aw_lww_map.ex:99-146) applied like join_delta with the
 *        touched keys (the queued mutate_async calls of a GPU-attached replica)
 *   read(state, keys | :all)                  -> %{key => value}       (read/1,2, :211-224)
 *   take(state, keys)                         -> value map of those keys (Map.take, :118,331)
 *   merkle_build(state, depth)                -> :ok
 *   merkle_prepare(state, levels)             -> {:continue, cont}     (:255)
 *   merkle_continue(state, cont, levels, max) -> {:continue, cont} | {:ok, keys}  (:96-105)
 *   (a continuation is an opaque binary; `max` is max_sync_size, :98,105,206-214)
 */
#include <erl_nif.h>
#include <stdlib.h>
#include <string.h>

#include "../include/deltagpu.h"
#include "marshal.h"

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
typedef struct state_res state_res;

typedef struct {
  dg_engine* e;
  dgm_universe* u;
  term_ud tu;
  ErlNifMutex* lock;
  state_res* live; /* every state of this engine (a relabel rewrites them all) */
  /* the universe's term-hash tables on the device, for the trees (dg_term_hashes) */
  dg_term_hashes th;
  uint64_t *d_nh, *d_vid, *d_vh;
  uint64_t th_nodes, th_vals; /* the table sizes uploaded; a relabel clears th_vals */
} engine_res;

/* A delta's device buffers, kept per state and grown on demand: a local mutation (a
 * one-key delta, causal_crdt.ex:337-342) then allocates nothing -- a hipMalloc / hipFree
 * pair per call cost more than the join itself (c_src/bench_mutate.c). */
typedef struct {
  dg_store raw, rows;       /* as marshalled (map-walk order), and sorted */
  dg_context rawc, ctx;
  uint64_t* keys;           /* the keyset */
  uint64_t keys_cap;
  /* the return block: dg_join_delta's changed keys [0, back_cap), then their rows
   * (dg_take_keys) as key | val | ts | cnt | node columns at stride back_cap -- brought
   * home with ONE copy */
  uint64_t* back;
  uint64_t back_cap;
  uint64_t* h_back;         /* its host copy (enif_alloc) */
} delta_buf;

struct state_res {
  engine_res* eng;
  dg_store rows;
  dg_store spare; /* dg_join_delta's second buffer (allocated on first need, kept) */
  dg_context ctx;
  dg_merkle tree;
  int has_tree;
  delta_buf d;
  state_res *prev, *next;
};

static ErlNifResourceType* ENGINE_RT;
static ErlNifResourceType* STATE_RT;
static ERL_NIF_TERM A_OK, A_ERROR, A_NIL, A_ALL, A_CONTINUE, A_MAP, A_STRUCT, A_MAPSET;

static void engine_dtor(ErlNifEnv* env, void* obj) {
  (void)env;
  engine_res* r = (engine_res*)obj;
  if (r->e) {
    dg_buffer_free(r->e, r->d_nh);
    dg_buffer_free(r->e, r->d_vid);
    dg_buffer_free(r->e, r->d_vh);
  }
  if (r->u) dgm_universe_free(r->u);
  if (r->tu.env) enif_free_env(r->tu.env);
  if (r->e) dg_engine_destroy(r->e);
  if (r->lock) enif_mutex_destroy(r->lock);
}

static void state_dtor(ErlNifEnv* env, void* obj) {
  (void)env;
  state_res* s = (state_res*)obj;
  engine_res* g = s->eng;
  enif_mutex_lock(g->lock);
  if (s->prev) s->prev->next = s->next; else g->live = s->next;
  if (s->next) s->next->prev = s->prev;
  dg_store_free(g->e, &s->rows);
  dg_store_free(g->e, &s->spare);
  dg_context_free(g->e, &s->ctx);
  dg_store_free(g->e, &s->d.raw);
  dg_store_free(g->e, &s->d.rows);
  dg_context_free(g->e, &s->d.rawc);
  dg_context_free(g->e, &s->d.ctx);
  dg_buffer_free(g->e, s->d.keys);
  dg_buffer_free(g->e, s->d.back);
  if (s->d.h_back) enif_free(s->d.h_back);
  if (s->has_tree) {
    dg_buffer_free(g->e, s->tree.nodes);
    dg_buffer_free(g->e, s->tree.counts);
    dg_buffer_free(g->e, s->tree.starts);
  }
  enif_mutex_unlock(g->lock);
  enif_release_resource(g);
}

static ERL_NIF_TERM error_term(ErlNifEnv* env, int rc) {
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
/* The universe's term-hash tables on the device (re-uploaded when they grew or a relabel
 * changed the value ids); every tree points at g->th. */
static int refresh_terms(engine_res* g) {
  const uint64_t *nh, *vid, *vh;
  uint32_t nn;
  uint64_t nv;
  dgm_node_hashes(g->u, &nh, &nn);
  dgm_value_hashes(g->u, &vid, &vh, &nv);
  int rc = DG_OK;
  if (nn != g->th_nodes) {
    dg_buffer_free(g->e, g->d_nh);
    g->d_nh = NULL;
    if (!(rc = dg_buffer_alloc(g->e, (nn ? nn : 1) * 8, (void**)&g->d_nh)))
      rc = dg_copy_to_device(g->e, g->d_nh, nh, (uint64_t)nn * 8);
    g->th_nodes = rc ? 0 : nn;
  }
  if (!rc && nv != g->th_vals) {
    dg_buffer_free(g->e, g->d_vid);
    dg_buffer_free(g->e, g->d_vh);
    g->d_vid = g->d_vh = NULL;
    if (!(rc = dg_buffer_alloc(g->e, (nv ? nv : 1) * 8, (void**)&g->d_vid)) &&
        !(rc = dg_buffer_alloc(g->e, (nv ? nv : 1) * 8, (void**)&g->d_vh)) &&
        !(rc = dg_copy_to_device(g->e, g->d_vid, vid, nv * 8)))
      rc = dg_copy_to_device(g->e, g->d_vh, vh, nv * 8);
    g->th_vals = rc ? UINT64_MAX : nv;
  }
  g->th.node_hash = g->d_nh;
  g->th.n_nodes = g->th_nodes;
  g->th.val_id = g->d_vid;
  g->th.val_hash = g->d_vh;
  g->th.n_vals = g->th_vals == UINT64_MAX ? 0 : g->th_vals;
  return rc;
}

/* After any dgm_value that relabelled: rewrite every live state's val column.  Trees hash
 * terms, so they stay valid; the value table is re-uploaded with the new ids. */
static int remap_live(engine_res* g) {
  const uint64_t *old_ids, *new_ids;
  uint64_t n;
  dgm_last_relabel(g->u, &old_ids, &new_ids, &n);
  void *dold = NULL, *dnew = NULL;
  int rc = dg_buffer_alloc(g->e, n * 8, &dold);
  if (!rc) rc = dg_buffer_alloc(g->e, n * 8, &dnew);
  if (!rc) rc = dg_copy_to_device(g->e, dold, old_ids, n * 8);
  if (!rc) rc = dg_copy_to_device(g->e, dnew, new_ids, n * 8);
  for (state_res* s = g->live; !rc && s; s = s->next)
    rc = dg_remap_values(g->e, &s->rows, (const uint64_t*)dold, (const uint64_t*)dnew, n);
  dg_buffer_free(g->e, dold);
  dg_buffer_free(g->e, dnew);
  g->th_vals = UINT64_MAX - 1; /* stale: the next refresh_terms re-uploads the value table */
  return rc;
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

/* host rows -> sorted device store + context (dg_sort_store / dg_sort_context) */
static int upload_sorted(engine_res* g, const dgm_rows* h, dg_store* rows, dg_context* ctx) {
  dg_store raw;
  dg_context rawc;
  int rc = dg_store_alloc(g->e, h->s.n, &raw);
  if (rc) return rc;
  if (!(rc = dg_store_alloc(g->e, h->s.n, rows)) && !(rc = dg_store_upload(g->e, &h->s, &raw)))
    rc = dg_sort_store(g->e, &raw, rows);
  dg_store_free(g->e, &raw);
  if (rc) return rc;
  if ((rc = dg_context_alloc(g->e, h->c.n, &rawc))) return rc;
  if (!(rc = dg_context_alloc(g->e, h->c.n, ctx)) && !(rc = dg_context_upload(g->e, &h->c, &rawc)))
    rc = dg_sort_context(g->e, &rawc, ctx);
  dg_context_free(g->e, &rawc);
  return rc;
}

/* grow a kept device store / context / buffer to at least n entries (doubling) */
static int grow_store(engine_res* g, dg_store* s, uint64_t n) {
  if (s->key && s->cap >= n) return DG_OK;
  const uint64_t want = n > 2 * s->cap ? n : 2 * s->cap + 16;
  dg_store_free(g->e, s);
  memset(s, 0, sizeof *s);
  return dg_store_alloc(g->e, want, s);
}
static int grow_ctx(engine_res* g, dg_context* c, uint64_t n) {
  if (c->node && c->cap >= n) return DG_OK;
  dg_context_free(g->e, c);
  memset(c, 0, sizeof *c);
  return dg_context_alloc(g->e, n + 16, c);
}
static int grow_buf(engine_res* g, uint64_t** p, uint64_t* cap, uint64_t n) {
  if (*p && *cap >= n) return DG_OK;
  dg_buffer_free(g->e, *p);
  *p = NULL;
  *cap = 0;
  const uint64_t c = n + 16;
  int rc = dg_buffer_alloc(g->e, c * 8, (void**)p);
  if (!rc) *cap = c;
  return rc;
}

/* the return block for n changed keys and up to `rows` of their rows (6 x cap words) */
static int grow_back(engine_res* g, delta_buf* d, uint64_t n) {
  if (d->back && d->back_cap >= n) return DG_OK;
  dg_buffer_free(g->e, d->back);
  if (d->h_back) enif_free(d->h_back);
  d->back = NULL;
  d->h_back = NULL;
  const uint64_t c = n + 64;
  d->back_cap = 0;
  int rc = dg_buffer_alloc(g->e, 6 * c * 8, (void**)&d->back);
  if (rc) return rc;
  d->h_back = (uint64_t*)enif_alloc(6 * c * 8);
  if (!d->h_back) return DG_E_NOMEM;
  d->back_cap = c;
  return DG_OK;
}

/* rows already in (key, val, ts, node, cnt) order without duplicates, a context in
 * (node, cnt) order: a delta built by add/remove (one key, its dots) usually is */
static int rows_sorted(const dg_store* s) {
  for (uint64_t i = 1; i < s->n; i++) {
    const uint64_t a[5] = {s->key[i - 1], s->val[i - 1], (uint64_t)s->ts[i - 1] ^ (1ull << 63),
                           s->node[i - 1], s->cnt[i - 1]};
    const uint64_t b[5] = {s->key[i], s->val[i], (uint64_t)s->ts[i] ^ (1ull << 63), s->node[i],
                           s->cnt[i]};
    int c = 0;
    for (int f = 0; f < 5 && !c; f++) c = a[f] < b[f] ? -1 : a[f] > b[f];
    if (c >= 0) return 0;
  }
  return 1;
}
static int ctx_sorted(const dg_context* c) {
  for (uint64_t i = 1; i < c->n; i++) {
    if (c->node[i - 1] > c->node[i]) return 0;
    if (c->node[i - 1] == c->node[i] && (c->kind == DG_CTX_VV || c->cnt[i - 1] >= c->cnt[i])) return 0;
  }
  return 1;
}

/* host rows -> the state's kept delta buffers, sorted on the device only when the map
 * walk did not already produce the order */
static int upload_delta(engine_res* g, const dgm_rows* h, delta_buf* d) {
  int rc;
  if ((rc = grow_store(g, &d->rows, h->s.n ? h->s.n : 1))) return rc;
  if (rows_sorted(&h->s)) {
    if ((rc = dg_store_upload(g->e, &h->s, &d->rows))) return rc;
  } else {
    if ((rc = grow_store(g, &d->raw, h->s.n))) return rc;
    if ((rc = dg_store_upload(g->e, &h->s, &d->raw))) return rc;
    if ((rc = dg_sort_store(g->e, &d->raw, &d->rows))) return rc;
  }
  if ((rc = grow_ctx(g, &d->ctx, h->c.n ? h->c.n : 1))) return rc;
  if (ctx_sorted(&h->c)) {
    rc = dg_context_upload(g->e, &h->c, &d->ctx);
  } else {
    if ((rc = grow_ctx(g, &d->rawc, h->c.n))) return rc;
    if ((rc = dg_context_upload(g->e, &h->c, &d->rawc))) return rc;
    rc = dg_sort_context(g->e, &d->rawc, &d->ctx);
  }
  d->ctx.kind = h->c.kind;
  return rc;
}

/* a key list -> its ids, ascending unique, on the device */
static int grow_buf(engine_res* g, uint64_t** p, uint64_t* cap, uint64_t n);

/* keep: *d_keys is a kept buffer of *keep_cap entries, grown as needed (else allocated) */
static int marshal_keys(ErlNifEnv* env, engine_res* g, ERL_NIF_TERM keys, uint64_t** d_keys,
                        uint64_t* n_keys, int keep, uint64_t* keep_cap) {
  unsigned len;
  if (!enif_get_list_length(env, keys, &len)) return DG_E_INVAL;
  uint64_t* ids = (uint64_t*)enif_alloc((len ? len : 1) * sizeof *ids);
  ERL_NIF_TERM h, t = keys;
  unsigned n = 0;
  while (enif_get_list_cell(env, t, &h, &t)) {
    boxed b = {h};
    if (dgm_key(g->u, &b, &ids[n++])) {
      enif_free(ids);
      return DG_E_INVAL;
    }
  }
  /* sort + unique (small: the delta's keys) */
  for (unsigned i = 1; i < n; i++)
    for (unsigned j = i; j > 0 && ids[j - 1] > ids[j]; j--) {
      uint64_t x = ids[j];
      ids[j] = ids[j - 1];
      ids[j - 1] = x;
    }
  unsigned m = 0;
  for (unsigned i = 0; i < n; i++)
    if (!m || ids[m - 1] != ids[i]) ids[m++] = ids[i];
  int rc = keep ? grow_buf(g, d_keys, keep_cap, m ? m : 1)
                : dg_buffer_alloc(g->e, (m ? m : 1) * 8, (void**)d_keys);
  if (!rc) rc = dg_copy_to_device(g->e, *d_keys, ids, m * 8);
  *n_keys = m;
  enif_free(ids);
  return rc;
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

/* device rows -> %{key => value map} (host copy of just those rows) */
static int unmarshal_rows(ErlNifEnv* env, engine_res* g, const dg_store* dev, ERL_NIF_TERM* out) {
  dgm_rows h;
  int rc = dgm_rows_init(&h, dev->n, 1);
  if (rc) return rc;
  if (!(rc = dg_store_download(g->e, dev, &h.s))) rc = unmarshal_host_rows(env, g, &h.s, out);
  dgm_rows_free(&h);
  return rc;
}

static int unmarshal_dots(ErlNifEnv* env, engine_res* g, const dg_context* dev, ERL_NIF_TERM* out) {
  dgm_rows h;
  int rc = dgm_rows_init(&h, 1, dev->n);
  if (rc) return rc;
  if (!(rc = dg_context_download(g->e, dev, &h.c))) {
    ERL_NIF_TERM m = enif_make_new_map(env);
    for (uint64_t i = 0; i < h.c.n; i++) {
      const boxed* b = (const boxed*)dgm_node_term(g->u, h.c.node[i]);
      ERL_NIF_TERM n = enif_make_copy(env, b->t), c = enif_make_uint64(env, h.c.cnt[i]);
      if (dev->kind == DG_CTX_VV)
        enif_make_map_put(env, m, n, c, &m);
      else
        enif_make_map_put(env, m, enif_make_tuple2(env, n, c), enif_make_list(env, 0), &m);
    }
    *out = dev->kind == DG_CTX_VV ? m : make_mapset(env, m);
  }
  dgm_rows_free(&h);
  return rc;
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
  const int rc = dg_engine_create(dev, NULL, &g->e);
  ERL_NIF_TERM r = rc ? error_term(env, rc) : enif_make_tuple2(env, A_OK, enif_make_resource(env, g));
  enif_release_resource(g);
  return r;
}

static state_res* new_state(engine_res* g) {
  state_res* s = (state_res*)enif_alloc_resource(STATE_RT, sizeof *s);
  memset(s, 0, sizeof *s);
  enif_keep_resource(g);
  s->eng = g;
  s->next = g->live;
  if (g->live) g->live->prev = s;
  g->live = s;
  return s;
}

static ERL_NIF_TERM state_load(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  (void)argc;
  engine_res* g;
  if (!enif_get_resource(env, argv[0], ENGINE_RT, (void**)&g)) return enif_make_badarg(env);
  enif_mutex_lock(g->lock);
  state_res* s = new_state(g);
  dgm_rows h;
  int rc = dgm_rows_init(&h, 1024, 64);
  ERL_NIF_TERM r;
  if (!rc) rc = marshal_dots(env, g, argv[1], &h);
  if (!rc) rc = marshal_value(env, g, argv[2], &h);
  if (!rc) rc = upload_sorted(g, &h, &s->rows, &s->ctx);
  dgm_rows_free(&h);
  r = rc ? error_term(env, rc) : enif_make_tuple2(env, A_OK, enif_make_resource(env, s));
  enif_mutex_unlock(g->lock);
  enif_release_resource(s);
  return r;
}

/* The rows half of the return block: key | val | ts | cnt | node columns at stride
 * back_cap after the changed keys. */
static dg_store back_rows(delta_buf* d) {
  const uint64_t S = d->back_cap;
  uint64_t* b = d->back + S;
  dg_store tk = {b, b + S, (int64_t*)(b + 2 * S), (uint32_t*)(b + 4 * S), b + 3 * S, 0, S};
  return tk;
}

/* The keys a dg_join_delta_rows changed (in d->back[0, n_changed)) as
 * [{key, value_map | nil}] and the state's new context: their rows, which the join wrote
 * into the return block (`taken` = their number; UINT64_MAX: not written, more than the
 * block's stride holds -> grown and taken from the state), the block copied home ONCE. */
static int changed_result(ErlNifEnv* env, engine_res* g, state_res* s, uint64_t n_changed,
                          uint64_t taken, ERL_NIF_TERM* new_dots, ERL_NIF_TERM* changed_terms) {
  delta_buf* d = &s->d;
  ERL_NIF_TERM values = enif_make_new_map(env);
  int rc = DG_OK;
  for (int attempt = 0;; attempt++) {
    const uint64_t S = d->back_cap;
    dg_store tk = back_rows(d);
    if (attempt == 0 && taken != UINT64_MAX) {
      tk.n = taken;
      rc = DG_OK;
    } else {
      rc = dg_take_keys(g->e, &s->rows, d->back, n_changed, &tk);
    }
    if (rc == DG_E_CAPACITY && attempt == 0) {
      /* grow, keeping the changed keys: they pass through the host */
      uint64_t* keep = (uint64_t*)enif_alloc((n_changed ? n_changed : 1) * 8);
      if (!keep) return DG_E_NOMEM;
      rc = dg_copy_to_host(g->e, keep, d->back, n_changed * 8);
      if (!rc) rc = grow_back(g, d, tk.n > n_changed ? tk.n : n_changed);
      if (!rc) rc = dg_copy_to_device(g->e, d->back, keep, n_changed * 8);
      enif_free(keep);
      if (rc) return rc;
      continue;
    }
    if (rc) return rc;
    if ((rc = dg_copy_to_host(g->e, d->h_back, d->back, 6 * S * 8))) return rc;
    uint64_t* hb = d->h_back + S;
    dg_store hs = {hb, hb + S, (int64_t*)(hb + 2 * S), (uint32_t*)(hb + 4 * S), hb + 3 * S, tk.n, S};
    if ((rc = unmarshal_host_rows(env, g, &hs, &values))) return rc;
    break;
  }
  if ((rc = unmarshal_dots(env, g, &s->ctx, new_dots))) return rc;
  for (uint64_t i = n_changed; i-- > 0;) {
    const boxed* b = (const boxed*)dgm_key_term(g->u, d->h_back[i]);
    ERL_NIF_TERM k = enif_make_copy(env, b->t), v;
    if (!enif_get_map_value(env, values, k, &v)) v = A_NIL;
    *changed_terms = enif_make_list_cell(env, enif_make_tuple2(env, k, v), *changed_terms);
  }
  return DG_OK;
}

/* The spare buffer and the context's room for a union with `dn` more entries, grown. */
static int room_for(engine_res* g, state_res* s, uint64_t rows, uint64_t dn) {
  int rc = DG_OK;
  if (s->spare.cap < s->rows.n + rows) {
    dg_store_free(g->e, &s->spare);
    if ((rc = dg_store_alloc(g->e, 2 * (s->rows.n + rows), &s->spare))) return rc;
  }
  if (s->ctx.cap < s->ctx.n + dn) {
    dg_context nctx;
    memset(&nctx, 0, sizeof nctx);
    if ((rc = dg_context_alloc(g->e, 2 * (s->ctx.n + dn), &nctx))) return rc;
    rc = dg_copy_to_device(g->e, nctx.node, s->ctx.node, s->ctx.n * 4); /* device to device */
    if (!rc) rc = dg_copy_to_device(g->e, nctx.cnt, s->ctx.cnt, s->ctx.n * 8);
    if (rc) {
      dg_context_free(g->e, &nctx);
      return rc;
    }
    nctx.n = s->ctx.n;
    nctx.kind = s->ctx.kind;
    dg_context_free(g->e, &s->ctx);
    s->ctx = nctx;
  }
  return rc;
}

static ERL_NIF_TERM join_delta(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  (void)argc;
  state_res* s;
  if (!enif_get_resource(env, argv[0], STATE_RT, (void**)&s)) return enif_make_badarg(env);
  engine_res* g = s->eng;
  enif_mutex_lock(g->lock);
  int rc = DG_OK;
  dgm_rows h;
  delta_buf* d = &s->d;
  uint64_t n_keys = 0, n_changed = 0;
  int swapped = 0;
  ERL_NIF_TERM r, new_dots = A_NIL, changed_terms = enif_make_list(env, 0);
  TRY(dgm_rows_init(&h, 256, 16));
  TRY(marshal_dots(env, g, argv[1], &h));
  TRY(marshal_value(env, g, argv[2], &h));
  /* the delta into the state's kept buffers (no allocation once they are big enough) */
  TRY(upload_delta(g, &h, d));
  TRY(marshal_keys(env, g, argv[3], &d->keys, &n_keys, 1, &d->keys_cap));
  TRY(room_for(g, s, d->rows.n, d->ctx.n));
  TRY(grow_back(g, d, n_keys ? n_keys : 1));
  if (s->has_tree) TRY(refresh_terms(g));
  /* update_state_with_delta: the join (in place, or through the spare buffer: the structs
   * come back exchanged), the changed keys, the MerkleMap put/delete of them -- all or
   * nothing: on an error the state, its context and tree are as they were */
  {
    dg_store tk = back_rows(d);
    TRY(dg_join_delta_rows(g->e, &s->rows, &s->ctx, &d->rows, &d->ctx, d->keys, n_keys, &s->spare,
                           s->has_tree ? &s->tree : NULL, d->back, d->back_cap, &n_changed,
                           &swapped, &tk));
    TRY(changed_result(env, g, s, n_changed, tk.n <= tk.cap ? tk.n : UINT64_MAX, &new_dots,
                       &changed_terms));
  }
out:
  r = rc ? error_term(env, rc) : enif_make_tuple3(env, A_OK, new_dots, changed_terms);
  dgm_rows_free(&h);
  enif_mutex_unlock(g->lock);
  return r;
}

/* mutate_batch(state, node, ops): a batch of mutations by replica `node` -- ops =
 * [{:add, key, value, ts} | {:remove, key}] in the order they were made (the queued
 * mutate_async calls of one CausalCrdt, causal_crdt.ex:196-198,337-342) -- applied to
 * the resident state as ONE delta: dg_mutate_batch builds it on the device exactly as
 * the ops' add/remove deltas would compose (aw_lww_map.ex:99-146: per touched key the last
 * op's row if it is an add, context = the touched keys' dots plus every add's dot), then
 * dg_join_delta applies it with the touched keys.  -> {:ok, new_dots, changed} as
 * join_delta.  A one-key mutate costs ~0.1-0.2 ms on the device and a few us on the BEAM
 * (bench.py `mutate`), so the Elixir side applies single ops with join_cpu and ships them
 * here in batches. */
typedef struct {
  uint64_t key, val, rank;
  int64_t ts;
  uint32_t idx;
  uint8_t kind;
} mop;

static int mop_cmp(const void* a, const void* b) {  /* by key, then batch order: stable */
  const mop *x = (const mop*)a, *y = (const mop*)b;
  if (x->key != y->key) return x->key < y->key ? -1 : 1;
  return x->idx < y->idx ? -1 : x->idx > y->idx;
}

static ERL_NIF_TERM mutate_batch_nif(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  (void)argc;
  state_res* s;
  unsigned m;
  if (!enif_get_resource(env, argv[0], STATE_RT, (void**)&s) || !enif_get_list_length(env, argv[2], &m))
    return enif_make_badarg(env);
  engine_res* g = s->eng;
  enif_mutex_lock(g->lock);
  int rc = DG_OK, swapped = 0;
  delta_buf* d = &s->d;
  uint64_t n_keys = 0, n_changed = 0, n_adds = 0;
  uint32_t node = 0;
  ERL_NIF_TERM r, new_dots = A_NIL, changed_terms = enif_make_list(env, 0), head, tail = argv[2];
  mop* ops = (mop*)enif_alloc((m ? m : 1) * sizeof *ops);
  uint64_t* h = NULL;
  uint64_t* dev = NULL;
  if (!ops) {
    rc = DG_E_NOMEM;
    goto out;
  }
  {
    boxed bn = {argv[1]};
    TRY(dgm_node(g->u, &bn, &node));
  }
  /* intern every op (values first: a relabel re-spaces ids already handed out) */
  for (unsigned i = 0; i < m; i++) {
    int ar;
    const ERL_NIF_TERM* e;
    if (!enif_get_list_cell(env, tail, &head, &tail) || !enif_get_tuple(env, head, &ar, &e) || ar < 2) {
      rc = DG_E_INVAL;
      goto out;
    }
    ops[i].idx = i;
    ops[i].kind = ar == 4;
    ops[i].val = 0;
    ops[i].ts = 0;
    if (ar == 4) {
      ErlNifSInt64 ts;
      if (!enif_get_int64(env, e[3], &ts)) {
        rc = DG_E_INVAL;
        goto out;
      }
      ops[i].ts = ts;
      TRY(intern_value(env, g, e[2], &ops[i].val));
    } else if (ar != 2) {
      rc = DG_E_INVAL;
      goto out;
    }
  }
  tail = argv[2];
  for (unsigned i = 0; i < m; i++) {
    int ar;
    const ERL_NIF_TERM* e;
    enif_get_list_cell(env, tail, &head, &tail);
    enif_get_tuple(env, head, &ar, &e);
    boxed bk = {e[1]};
    TRY(dgm_key(g->u, &bk, &ops[i].key));
    if (ar == 4) {  /* a later relabel may have moved this value's id: take it again */
      boxed bv = {e[2]};
      int relabeled = 0;
      TRY(dgm_value(g->u, &bv, &ops[i].val, &relabeled));
      if (relabeled) TRY(remap_live(g));
      ops[i].rank = n_adds++;
    }
  }
  qsort(ops, m, sizeof *ops, mop_cmp);
  /* kind | key | val | ts | add_rank, one upload (the u8 kinds packed at the end) */
  {
    const uint64_t words = 4 * (uint64_t)m + (m + 7) / 8 + 1;
    h = (uint64_t*)enif_alloc(words * 8);
    if (!h) {
      rc = DG_E_NOMEM;
      goto out;
    }
    uint8_t* kinds = (uint8_t*)(h + 4 * (uint64_t)m);
    for (unsigned i = 0; i < m; i++) {
      h[i] = ops[i].key;
      h[m + i] = ops[i].val;
      h[2 * (uint64_t)m + i] = (uint64_t)ops[i].ts;
      h[3 * (uint64_t)m + i] = ops[i].rank;
      kinds[i] = ops[i].kind;
    }
    TRY(dg_buffer_alloc(g->e, words * 8, (void**)&dev));
    TRY(dg_copy_to_device(g->e, dev, h, words * 8));
  }
  /* the delta in the state's kept buffers: one row per touched key, a dot list of at most
   * the touched keys' rows + the adds (retried with the exact sizes when short) */
  TRY(grow_store(g, &d->rows, m ? m : 1));
  TRY(grow_buf(g, &d->keys, &d->keys_cap, m ? m : 1));
  for (int attempt = 0;; attempt++) {
    TRY(grow_ctx(g, &d->ctx, attempt ? s->rows.n + n_adds + 1 : 8 * (uint64_t)m + n_adds + 1));
    rc = dg_mutate_batch(g->e, &s->rows, &s->ctx, node, m, (const uint8_t*)(dev + 4 * (uint64_t)m), dev,
                         dev + m, (const int64_t*)(dev + 2 * (uint64_t)m), dev + 3 * (uint64_t)m, n_adds,
                         &d->rows, &d->ctx, d->keys, d->keys_cap, &n_keys);
    if (rc == DG_E_CAPACITY && attempt == 0) continue;
    TRY(rc);
    break;
  }
  TRY(room_for(g, s, d->rows.n, d->ctx.n));
  TRY(grow_back(g, d, n_keys ? n_keys : 1));
  if (s->has_tree) TRY(refresh_terms(g));
  {
    dg_store tk = back_rows(d);
    TRY(dg_join_delta_rows(g->e, &s->rows, &s->ctx, &d->rows, &d->ctx, d->keys, n_keys, &s->spare,
                           s->has_tree ? &s->tree : NULL, d->back, d->back_cap, &n_changed,
                           &swapped, &tk));
    TRY(changed_result(env, g, s, n_changed, tk.n <= tk.cap ? tk.n : UINT64_MAX, &new_dots,
                       &changed_terms));
  }
out:
  r = rc ? error_term(env, rc) : enif_make_tuple3(env, A_OK, new_dots, changed_terms);
  if (ops) enif_free(ops);
  if (h) enif_free(h);
  dg_buffer_free(g->e, dev);
  enif_mutex_unlock(g->lock);
  return r;
}

static ERL_NIF_TERM read_nif(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  (void)argc;
  state_res* s;
  if (!enif_get_resource(env, argv[0], STATE_RT, (void**)&s)) return enif_make_badarg(env);
  engine_res* g = s->eng;
  enif_mutex_lock(g->lock);
  int rc = DG_OK;
  uint64_t *d_keys = NULL, n_keys = 0, *dk = NULL, *dv = NULL, n_out = 0;
  uint64_t *hk = NULL, *hv = NULL;
  ERL_NIF_TERM r, m = enif_make_new_map(env);
  const int all = enif_is_identical(argv[1], A_ALL);
  if (!all) TRY(marshal_keys(env, g, argv[1], &d_keys, &n_keys, 0, NULL));
  const uint64_t cap = s->rows.n ? s->rows.n : 1;
  TRY(dg_buffer_alloc(g->e, cap * 8, (void**)&dk));
  TRY(dg_buffer_alloc(g->e, cap * 8, (void**)&dv));
  TRY(dg_read_lww(g->e, &s->rows, all ? NULL : d_keys, n_keys, dk, dv, cap, &n_out));
  hk = (uint64_t*)enif_alloc((n_out ? n_out : 1) * 8);
  hv = (uint64_t*)enif_alloc((n_out ? n_out : 1) * 8);
  TRY(dg_copy_to_host(g->e, hk, dk, n_out * 8));
  TRY(dg_copy_to_host(g->e, hv, dv, n_out * 8));
  for (uint64_t i = 0; i < n_out; i++) {
    const boxed* k = (const boxed*)dgm_key_term(g->u, hk[i]);
    ERL_NIF_TERM v;
    TRY(value_term(env, g, hv[i], &v));
    enif_make_map_put(env, m, enif_make_copy(env, k->t), v, &m);
  }
out:
  r = rc ? error_term(env, rc) : m;
  if (hk) enif_free(hk);
  if (hv) enif_free(hv);
  dg_buffer_free(g->e, d_keys);
  dg_buffer_free(g->e, dk);
  dg_buffer_free(g->e, dv);
  enif_mutex_unlock(g->lock);
  return r;
}

static ERL_NIF_TERM take_nif(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  (void)argc;
  state_res* s;
  if (!enif_get_resource(env, argv[0], STATE_RT, (void**)&s)) return enif_make_badarg(env);
  engine_res* g = s->eng;
  enif_mutex_lock(g->lock);
  int rc = DG_OK;
  uint64_t* d_keys = NULL;
  uint64_t n_keys = 0;
  dg_store taken;
  memset(&taken, 0, sizeof taken);
  ERL_NIF_TERM r, values = enif_make_new_map(env);
  TRY(marshal_keys(env, g, argv[1], &d_keys, &n_keys, 0, NULL));
  TRY(dg_store_alloc(g->e, s->rows.n, &taken));
  TRY(dg_take_keys(g->e, &s->rows, d_keys, n_keys, &taken));
  TRY(unmarshal_rows(env, g, &taken, &values));
out:
  r = rc ? error_term(env, rc) : values;
  dg_store_free(g->e, &taken);
  dg_buffer_free(g->e, d_keys);
  enif_mutex_unlock(g->lock);
  return r;
}

static ERL_NIF_TERM merkle_build_nif(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  (void)argc;
  state_res* s;
  unsigned depth;
  if (!enif_get_resource(env, argv[0], STATE_RT, (void**)&s) || !enif_get_uint(env, argv[1], &depth))
    return enif_make_badarg(env);
  engine_res* g = s->eng;
  enif_mutex_lock(g->lock);
  int rc = DG_OK;
  if (s->has_tree) {
    dg_buffer_free(g->e, s->tree.nodes);
    dg_buffer_free(g->e, s->tree.counts);
  }
  memset(&s->tree, 0, sizeof s->tree);
  s->has_tree = 0;
  s->tree.depth = depth;
  TRY(refresh_terms(g));
  s->tree.terms = &g->th; /* rows hashed through their terms: comparable across nodes */
  TRY(dg_buffer_alloc(g->e, ((2ull << depth) - 1) * 8, (void**)&s->tree.nodes));
  TRY(dg_buffer_alloc(g->e, ((1ull << depth) > 16 ? (1ull << depth) : 16) * 2, (void**)&s->tree.counts));
  TRY(dg_buffer_alloc(g->e, (dg_merkle_chunks(depth) + 1) * 8, (void**)&s->tree.starts));
  s->has_tree = 1;
  TRY(dg_merkle_build(g->e, &s->rows, &s->tree));
out:;
  ERL_NIF_TERM r = rc ? error_term(env, rc) : A_OK;
  enif_mutex_unlock(g->lock);
  return r;
}

/* continuation <-> binary: u32 level | u64 n | u64 n_buckets | pos[n] | hash[n] | bucket[nb] */
static int cont_to_binary(ErlNifEnv* env, engine_res* g, const dg_merkle_cont* c, ERL_NIF_TERM* out) {
  const size_t bytes = 4 + 16 + c->n * 16 + c->n_buckets * 8;
  ErlNifBinary b;
  if (!enif_alloc_binary(bytes, &b)) return DG_E_NOMEM;
  unsigned char* p = b.data;
  memcpy(p, &c->level, 4);
  memcpy(p + 4, &c->n, 8);
  memcpy(p + 12, &c->n_buckets, 8);
  int rc = dg_copy_to_host(g->e, p + 20, c->pos, c->n * 8);
  if (!rc) rc = dg_copy_to_host(g->e, p + 20 + c->n * 8, c->hash, c->n * 8);
  if (!rc && c->n_buckets) rc = dg_copy_to_host(g->e, p + 20 + c->n * 16, c->bucket, c->n_buckets * 8);
  if (rc) {
    enif_release_binary(&b);
    return rc;
  }
  *out = enif_make_binary(env, &b);
  return DG_OK;
}

static int cont_alloc(engine_res* g, uint64_t cap, uint64_t cap_b, dg_merkle_cont* c) {
  memset(c, 0, sizeof *c);
  int rc = dg_buffer_alloc(g->e, (cap ? cap : 1) * 8, (void**)&c->pos);
  if (!rc) rc = dg_buffer_alloc(g->e, (cap ? cap : 1) * 8, (void**)&c->hash);
  if (!rc) rc = dg_buffer_alloc(g->e, (cap_b ? cap_b : 1) * 8, (void**)&c->bucket);
  c->cap = cap;
  c->cap_buckets = cap_b;
  return rc;
}

static void cont_free(engine_res* g, dg_merkle_cont* c) {
  dg_buffer_free(g->e, c->pos);
  dg_buffer_free(g->e, c->hash);
  dg_buffer_free(g->e, c->bucket);
}

static ERL_NIF_TERM merkle_prepare_nif(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  (void)argc;
  state_res* s;
  unsigned levels;
  if (!enif_get_resource(env, argv[0], STATE_RT, (void**)&s) || !enif_get_uint(env, argv[1], &levels) ||
      !s->has_tree)
    return enif_make_badarg(env);
  engine_res* g = s->eng;
  enif_mutex_lock(g->lock);
  int rc = DG_OK;
  dg_merkle_cont c;
  ERL_NIF_TERM bin = A_NIL, r;
  const unsigned L = levels < s->tree.depth ? levels : s->tree.depth;
  TRY(cont_alloc(g, 1ull << L, 1, &c));
  TRY(dg_merkle_prepare(g->e, &s->tree, levels, &c));
  TRY(cont_to_binary(env, g, &c, &bin));
out:
  r = rc ? error_term(env, rc) : enif_make_tuple2(env, A_CONTINUE, bin);
  cont_free(g, &c);
  enif_mutex_unlock(g->lock);
  return r;
}

static ERL_NIF_TERM merkle_continue_nif(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  (void)argc;
  state_res* s;
  ErlNifBinary in;
  unsigned levels;
  ErlNifUInt64 max_sync;
  if (!enif_get_resource(env, argv[0], STATE_RT, (void**)&s) || !enif_inspect_binary(env, argv[1], &in) ||
      !enif_get_uint(env, argv[2], &levels) || !enif_get_uint64(env, argv[3], &max_sync) ||
      !s->has_tree || in.size < 20)
    return enif_make_badarg(env);
  engine_res* g = s->eng;
  enif_mutex_lock(g->lock);
  int rc = DG_OK, status = 0;
  dg_merkle_cont ci, co;
  memset(&co, 0, sizeof co);
  uint64_t *keys = NULL, n_keys = 0, n_total = 0;
  ERL_NIF_TERM r, res = A_NIL;
  uint32_t level;
  uint64_t n, nb;
  memcpy(&level, in.data, 4);
  memcpy(&n, in.data + 4, 8);
  memcpy(&nb, in.data + 12, 8);
  TRY(refresh_terms(g));
  TRY(cont_alloc(g, n, nb, &ci));
  ci.level = level;
  ci.n = n;
  ci.n_buckets = nb;
  TRY(dg_copy_to_device(g->e, ci.pos, in.data + 20, n * 8));
  TRY(dg_copy_to_device(g->e, ci.hash, in.data + 20 + n * 8, n * 8));
  if (nb) TRY(dg_copy_to_device(g->e, ci.bucket, in.data + 20 + n * 16, nb * 8));
  const uint64_t cap_keys = max_sync ? max_sync : 1;
  TRY(dg_buffer_alloc(g->e, cap_keys * 8, (void**)&keys));
  /* the output: grown to the sizes a DG_E_CAPACITY reports */
  uint64_t cap = 4 * (n ? n : 1), cap_b = n ? n : 1;
  for (int attempt = 0; attempt < 3; attempt++) {
    TRY(cont_alloc(g, cap, cap_b, &co));
    rc = dg_merkle_continue(g->e, &s->tree, &s->rows, &ci, levels, &co, keys, cap_keys, &n_keys,
                            &n_total, &status);
    if (rc != DG_E_CAPACITY) break;
    cap = co.n > cap ? co.n : cap;
    cap_b = co.n_buckets > cap_b ? co.n_buckets : cap_b;
    cont_free(g, &co);
    memset(&co, 0, sizeof co);
  }
  if (rc) goto out;
  if (status == 1) {
    TRY(dg_merkle_truncate(g->e, &s->tree, &co, max_sync));  /* truncate_diff, :98 */
    TRY(cont_to_binary(env, g, &co, &res));
    res = enif_make_tuple2(env, A_CONTINUE, res);
  } else {
    /* {:ok, keys}: the first max_sync_size differing keys (Enum.take, :105) */
    uint64_t* hk = (uint64_t*)enif_alloc((n_keys ? n_keys : 1) * 8);
    rc = dg_copy_to_host(g->e, hk, keys, n_keys * 8);
    ERL_NIF_TERM l = enif_make_list(env, 0);
    for (uint64_t i = n_keys; !rc && i-- > 0;) {
      const boxed* b = (const boxed*)dgm_key_term(g->u, hk[i]);
      l = enif_make_list_cell(env, enif_make_copy(env, b->t), l);
    }
    enif_free(hk);
    res = enif_make_tuple2(env, A_OK, l);
  }
out:
  r = rc ? error_term(env, rc) : res;
  cont_free(g, &ci);
  cont_free(g, &co);
  dg_buffer_free(g->e, keys);
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
  return (ENGINE_RT && STATE_RT) ? 0 : 1;  /* a failed load -> the Elixir code path */
}

static ErlNifFunc funcs[] = {
    {"engine_open", 1, engine_open, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"state_load", 3, state_load, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"join_delta", 4, join_delta, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"mutate_batch", 3, mutate_batch_nif, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"read", 2, read_nif, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"take", 2, take_nif, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"merkle_build", 2, merkle_build_nif, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"merkle_prepare", 2, merkle_prepare_nif, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"merkle_continue", 4, merkle_continue_nif, ERL_NIF_DIRTY_JOB_CPU_BOUND},
};

ERL_NIF_INIT(Elixir.DeltaCrdt.GPU, funcs, load, NULL, NULL, NULL)
