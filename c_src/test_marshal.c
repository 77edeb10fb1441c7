/*
 * test_marshal.c — the NIF's term-independent half (marshal.c) and the C-ABI path a NIF
 * drives, from C:
 *
 *   1. value ids follow Erlang term order across thousands of inserts and relabels;
 *      node ids are dense; a 64-bit key-id collision is refused;
 *   2. (with a GPU) two replicas marshalled in map-walk order (unsorted rows and
 *      contexts) are uploaded, ordered by dg_sort_store / dg_sort_context, joined
 *      (dg_join2) and read (dg_read_lww): bit-exact against the C oracle
 *      (oracle/deltaref.c ref_join2 / ref_read_lww on host-sorted rows), and the read
 *      winners are the reference's (aw_lww_map.ex:211-216: greatest ts, a tie to the
 *      smallest {value, ts} in term order) by TERM comparison;
 *   3. (with a GPU) a relabel rewrites a device store with dg_remap_values.
 *
 * Test terms stand in for BEAM terms: integers, floats, atoms and binaries in map-key
 * order: integers < floats < atoms < binaries.
 * Exit status 0 = pass.  Without a device part 1 runs and the rest prints SKIP, unless
 * DG_REQUIRE_GPU=1.
 */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "marshal.h"

/* the C oracle (oracle/_build/libdeltaref.so) */
int ref_join2(const dg_store* a, const dg_context* ca, const dg_store* b, const dg_context* cb,
              const uint64_t* keys, uint64_t n_keys, dg_store* out, dg_context* out_ctx);
int ref_read_lww(const dg_store* s, const uint64_t* keys, uint64_t n_keys, uint64_t* out_key,
                 uint64_t* out_val, uint64_t cap, uint64_t* n_out);

#define CHECK(c)                                                            \
  do {                                                                      \
    if (!(c)) {                                                             \
      fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #c);          \
      exit(1);                                                              \
    }                                                                       \
  } while (0)
#define DG(x)                                                               \
  do {                                                                      \
    int rc_ = (x);                                                          \
    if (rc_ != DG_OK) {                                                     \
      fprintf(stderr, "FAIL %s:%d: %s -> %d (%s)\n", __FILE__, __LINE__, #x, rc_, \
              dg_last_error());                                             \
      exit(1);                                                              \
    }                                                                       \
  } while (0)

/* ------------------------------------------------------------ test terms */
enum { T_INT = 0, T_FLOAT = 1, T_ATOM = 2, T_BIN = 3 };
typedef struct {
  int kind;
  int64_t i;
  double f;
  char s[16];
} tterm;

static int cls(const tterm* t) { return t->kind <= T_FLOAT ? 0 : t->kind == T_ATOM ? 1 : 10; }

static int tcmp(const void* pa, const void* pb, void* ud) {
  (void)ud;
  const tterm *a = (const tterm*)pa, *b = (const tterm*)pb;
  if (cls(a) != cls(b)) return cls(a) < cls(b) ? -1 : 1;
  if (cls(a) == 0) { /* map-key order: every integer before every float */
    if (a->kind != b->kind) return a->kind == T_INT ? -1 : 1;
    if (a->kind == T_INT) return a->i < b->i ? -1 : a->i > b->i;
    return a->f < b->f ? -1 : a->f > b->f;
  }
  return strcmp(a->s, b->s) < 0 ? -1 : strcmp(a->s, b->s) > 0 ? 1 : 0;
}

static int tenc(const void* p, dgm_buf* b, void* ud) {
  (void)ud;
  const tterm* t = (const tterm*)p;
  switch (t->kind) {
    case T_INT: return dgm_enc_i64(b, t->i);
    case T_FLOAT: return dgm_enc_float(b, t->f);
    case T_ATOM: return dgm_enc_atom(b, t->s, strlen(t->s));
    default: return dgm_enc_binary(b, t->s, strlen(t->s));
  }
}

static void* tkeep(const void* t, void* ud) {
  (void)ud;
  tterm* c = (tterm*)malloc(sizeof *c);
  memcpy(c, t, sizeof *c);
  return c;
}
static void tdrop(void* t, void* ud) {
  (void)ud;
  free(t);
}

static tterm ti(int64_t i) {
  tterm t;
  memset(&t, 0, sizeof t);
  t.kind = T_INT;
  t.i = i;
  return t;
}
static tterm tf(double f) {
  tterm t;
  memset(&t, 0, sizeof t);
  t.kind = T_FLOAT;
  t.f = f;
  return t;
}
/* the term of a value id: a canonical integer from its closed form, else the table's */
static const tterm* value_term(const dgm_universe* u, uint64_t id, tterm* scratch) {
  int64_t v;
  if (dgm_value_is_canonical(id, &v)) {
    memset(scratch, 0, sizeof *scratch);
    scratch->kind = T_INT;
    scratch->i = v;
    return scratch;
  }
  return (const tterm*)dgm_value_term(u, id);
}

static tterm ts_(int kind, const char* s) {
  tterm t;
  memset(&t, 0, sizeof t);
  t.kind = kind;
  snprintf(t.s, sizeof t.s, "%s", s);
  return t;
}

static uint64_t rng_state = 0x1234567;
static uint64_t rnd(void) {
  rng_state += 0x9E3779B97F4A7C15ull;
  uint64_t z = rng_state;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

static tterm random_value(void) {
  static const char* words[] = {"a", "b", "ab", "zz", "x", "nil", "ok", "q"};
  switch (rnd() % 4) {
    case 0: return ti((int64_t)(rnd() % 21) - 10);
    case 1: return tf((double)(rnd() % 41) / 4.0 - 5.0);
    case 2: return ts_(T_ATOM, words[rnd() % 8]);
    default: return ts_(T_BIN, words[rnd() % 8]);
  }
}

static dgm_term_ops ops(void) {
  dgm_term_ops o;
  o.cmp = tcmp;
  o.encode = tenc;
  o.hash = NULL;
  o.keep = tkeep;
  o.drop = tdrop;
  o.ud = NULL;
  return o;
}

/* ------------------------------------------------------------ part 1 */
static uint64_t const_hash(const void* p, void* ud) {
  (void)p;
  (void)ud;
  return 42;
}

static void test_universe(void) {
  dgm_term_ops o = ops();
  dgm_universe* u = dgm_universe_new(&o);
  CHECK(u);
  enum { N = 4000 };
  static uint64_t ids[N];
  static tterm vals[N];
  int relabels = 0;
  for (int i = 0; i < N; i++) {
    vals[i] = random_value();
    int rl;
    CHECK(dgm_value(u, &vals[i], &ids[i], &rl) == DG_OK);
    relabels += rl;
  }
  /* squeeze floats into one gap until the universe re-spaces its ids */
  tterm lo = tf(1.0);
  double hi = 1.25;
  uint64_t id_lo;
  int rl;
  CHECK(dgm_value(u, &lo, &id_lo, &rl) == DG_OK);
  for (int i = 0; i < 80; i++) {
    hi = (1.0 + hi) / 2;
    tterm t = tf(hi);
    uint64_t id;
    CHECK(dgm_value(u, &t, &id, &rl) == DG_OK);
    if (rl) {
      const uint64_t *old_ids, *new_ids;
      uint64_t n;
      dgm_last_relabel(u, &old_ids, &new_ids, &n);
      CHECK(n > 0);
      for (uint64_t k = 1; k < n; k++) CHECK(old_ids[k - 1] < old_ids[k] && new_ids[k - 1] < new_ids[k]);
    }
    relabels += rl;
  }
  CHECK(relabels >= 1);
  /* every value keeps its term; ids compare as the terms do (equal terms share ids) */
  for (int i = 0; i < N; i++) {
    uint64_t id;
    CHECK(dgm_value(u, &vals[i], &id, &rl) == DG_OK && !rl);
    tterm sc;
    const tterm* back = value_term(u, id, &sc);
    CHECK(back && tcmp(back, &vals[i], NULL) == 0);
  }
  for (int j = 0; j < 200000; j++) {
    const int a = (int)(rnd() % N), b = (int)(rnd() % N);
    uint64_t ia, ib;
    dgm_value(u, &vals[a], &ia, &rl);
    dgm_value(u, &vals[b], &ib, &rl);
    const int c = tcmp(&vals[a], &vals[b], NULL);
    CHECK((ia < ib) == (c < 0) && (ia == ib) == (c == 0));
  }
  /* nodes: dense, first-seen order */
  uint32_t n0, n1, n2;
  tterm na = ti(999999937), nb = ts_(T_ATOM, "node"), nc = ti(5);
  CHECK(dgm_node(u, &na, &n0) == DG_OK && dgm_node(u, &nb, &n1) == DG_OK &&
        dgm_node(u, &nc, &n2) == DG_OK);
  CHECK(n0 == 0 && n1 == 1 && n2 == 2);
  CHECK(dgm_node(u, &na, &n2) == DG_OK && n2 == 0);
  CHECK(tcmp(dgm_node_term(u, 1), &nb, NULL) == 0);
  dgm_universe_free(u);

  /* canonical integers have closed-form ids; others land in the two regions around them */
  {
    dgm_term_ops o2 = ops();
    dgm_universe* w = dgm_universe_new(&o2);
    tterm a = ti(7), bneg = ti(INT64_MIN), bpos = ti(INT64_C(1) << 62), f = tf(-1e300);
    uint64_t ia, in, ip, ifl;
    int64_t back;
    CHECK(dgm_value(w, &a, &ia, &rl) == DG_OK && ia == 7 + (1ull << 62));
    CHECK(dgm_value_is_canonical(ia, &back) && back == 7 && !dgm_value_term(w, ia));
    CHECK(dgm_value(w, &bneg, &in, &rl) == DG_OK && in > 0 && in < (1ull << 58));
    CHECK(dgm_value(w, &bpos, &ip, &rl) == DG_OK && ip >= (1ull << 63));
    CHECK(dgm_value(w, &f, &ifl, &rl) == DG_OK && ifl > ip);  /* every float after every int */
    const uint64_t *vids, *vh;
    uint64_t nv;
    dgm_value_hashes(w, &vids, &vh, &nv);
    CHECK(nv == 3 && vids[0] == in && vids[1] == ip && vids[2] == ifl);
    dgm_universe_free(w);
  }
  /* a key-id collision is refused: every key hashes alike here */
  dgm_term_ops c = ops();
  c.encode = NULL;
  CHECK(dgm_universe_new(&c) == NULL);
  c.encode = tenc;
  c.hash = const_hash;
  dgm_universe* v = dgm_universe_new(&c);
  uint64_t k1, k2;
  tterm x = ti(1), y = ti(2);
  CHECK(dgm_key(v, &x, &k1) == DG_OK && k1 == 42);
  CHECK(dgm_key(v, &x, &k2) == DG_OK && k2 == 42);
  CHECK(dgm_key(v, &y, &k2) == DG_E_INVAL);
  CHECK(tcmp(dgm_key_term(v, 42), &x, NULL) == 0);
  dgm_universe_free(v);
  printf("universe ok (%d relabels)\n", relabels);
}

/* ------------------------------------------------------------ part 2 */
typedef struct {
  tterm key, val, node;
  int64_t ts;
  uint64_t cnt;
} trow;

typedef struct {
  trow* r;
  int n;
  tterm vv_node[8];
  uint64_t vv_cnt[8];
  int nvv;
} trep;

/* two replicas of one key space: shared base rows, then each adds its own rows with
 * ts ties; contexts are VVs covering each replica's own dots */
static void make_replicas(trep* a, trep* b, int n_keys) {
  tterm nodes[4];
  for (int i = 0; i < 4; i++) nodes[i] = ti(1 + (int64_t)(rnd() % 1000000000));
  trep* reps[2] = {a, b};
  uint64_t counters[4] = {0, 0, 0, 0};
  for (int r = 0; r < 2; r++) {
    reps[r]->r = (trow*)calloc((size_t)n_keys * 6, sizeof(trow));
    reps[r]->n = 0;
  }
  for (int k = 0; k < n_keys; k++) {
    tterm key = (k % 3 == 0) ? ts_(T_BIN, "") : ti(k);
    if (k % 3 == 0) snprintf(key.s, sizeof key.s, "k%d", k);
    /* base entry written by node 0, in both replicas unless one removed it */
    const uint64_t c0 = ++counters[0];
    trow base = {key, random_value(), nodes[0], (int64_t)(rnd() % 4), c0};
    for (int r = 0; r < 2; r++)
      if (rnd() % 5) reps[r]->r[reps[r]->n++] = base;
    for (int r = 0; r < 2; r++) {
      const int extra = (int)(rnd() % 3);
      for (int e = 0; e < extra; e++) {
        const int nd = (rnd() % 4 == 0) ? 3 : 1 + r;  /* the replica's own node, or node 3 */
        trow x = {key, random_value(), nodes[nd], (int64_t)(rnd() % 4), ++counters[nd]};
        reps[r]->r[reps[r]->n++] = x;
      }
    }
  }
  for (int r = 0; r < 2; r++) {
    reps[r]->nvv = 4;
    for (int i = 0; i < 4; i++) {
      reps[r]->vv_node[i] = nodes[i];
      reps[r]->vv_cnt[i] = counters[i] - (rnd() % 2);  /* not always covering (H5) */
    }
    /* a map walk emits rows in no particular order */
    for (int i = reps[r]->n - 1; i > 0; i--) {
      const int j = (int)(rnd() % (uint64_t)(i + 1));
      trow t = reps[r]->r[i];
      reps[r]->r[i] = reps[r]->r[j];
      reps[r]->r[j] = t;
    }
  }
}

static void marshal(dgm_universe* u, const trep* t, dgm_rows* out) {
  int rl;
  uint64_t id;
  for (int i = 0; i < t->n; i++) CHECK(dgm_value(u, &t->r[i].val, &id, &rl) == DG_OK);
  dgm_rows_clear(out);
  for (int i = 0; i < t->n; i++) {
    uint64_t k, v;
    uint32_t nd;
    CHECK(dgm_key(u, &t->r[i].key, &k) == DG_OK);
    CHECK(dgm_value(u, &t->r[i].val, &v, &rl) == DG_OK && !rl);
    CHECK(dgm_node(u, &t->r[i].node, &nd) == DG_OK);
    CHECK(dgm_rows_push(out, k, v, t->r[i].ts, nd, t->r[i].cnt) == DG_OK);
  }
  for (int i = t->nvv - 1; i >= 0; i--) { /* map order, not node order */
    uint32_t nd;
    CHECK(dgm_node(u, &t->vv_node[i], &nd) == DG_OK);
    CHECK(dgm_ctx_push(out, nd, t->vv_cnt[i]) == DG_OK);
  }
  out->c.kind = DG_CTX_VV;
}

/* host sort of marshalled rows / contexts (what dg_sort_store must reproduce) */
static const dg_store* g_s;
static int row_cmp_idx(const void* pa, const void* pb) {
  const uint64_t i = *(const uint64_t*)pa, j = *(const uint64_t*)pb;
  const dg_store* s = g_s;
#define C3(f) if (s->f[i] != s->f[j]) return s->f[i] < s->f[j] ? -1 : 1;
  C3(key) C3(val) C3(ts) C3(node) C3(cnt)
#undef C3
  return 0;
}

static void host_sorted(const dgm_rows* r, dgm_rows* out) {
  uint64_t n = r->s.n;
  uint64_t* idx = (uint64_t*)malloc((n ? n : 1) * sizeof *idx);
  for (uint64_t i = 0; i < n; i++) idx[i] = i;
  g_s = &r->s;
  qsort(idx, n, sizeof *idx, row_cmp_idx);
  dgm_rows_clear(out);
  for (uint64_t i = 0; i < n; i++) {
    const uint64_t x = idx[i];
    if (i && row_cmp_idx(&idx[i - 1], &idx[i]) == 0) continue;
    dgm_rows_push(out, r->s.key[x], r->s.val[x], r->s.ts[x], r->s.node[x], r->s.cnt[x]);
  }
  /* VV by node */
  for (uint64_t i = 0; i < r->c.n; i++) dgm_ctx_push(out, r->c.node[i], r->c.cnt[i]);
  for (uint64_t i = 1; i < out->c.n; i++)
    for (uint64_t j = i; j > 0 && out->c.node[j - 1] > out->c.node[j]; j--) {
      uint32_t tn = out->c.node[j];
      out->c.node[j] = out->c.node[j - 1];
      out->c.node[j - 1] = tn;
      uint64_t tc = out->c.cnt[j];
      out->c.cnt[j] = out->c.cnt[j - 1];
      out->c.cnt[j - 1] = tc;
    }
  out->c.kind = DG_CTX_VV;
  free(idx);
}

/* read/1 by TERM comparison over sorted rows: per key the greatest ts, a tie to the
 * smallest value term (aw_lww_map.ex:211-216) */
typedef struct {
  const dgm_universe* u;
  uint64_t* keys;
  uint64_t* vals;
  uint64_t n;
  uint64_t cur_key;
  int have;
  int64_t best_ts;
  uint64_t best_val;
  tterm s1, s2;
} readst;

static void flush(readst* r) {
  if (r->have) {
    r->keys[r->n] = r->cur_key;
    r->vals[r->n++] = r->best_val;
  }
}
static int w_key(void* ud, uint64_t key, uint64_t n_entries) {
  (void)n_entries;
  readst* r = (readst*)ud;
  flush(r);
  r->cur_key = key;
  r->have = 0;
  return 0;
}
static int w_entry(void* ud, uint64_t val, int64_t ts, uint64_t n_dots) {
  (void)n_dots;
  readst* r = (readst*)ud;
  if (!r->have || ts > r->best_ts ||
      (ts == r->best_ts &&
       tcmp(value_term(r->u, val, &r->s1), value_term(r->u, r->best_val, &r->s2), NULL) < 0)) {
    r->best_ts = ts;
    r->best_val = val;
    r->have = 1;
  }
  return 0;
}

static int device_present(dg_engine** e) {
  if (dg_engine_create(0, NULL, e) != DG_OK) {
    *e = NULL;
    return 0;
  }
  return 1;
}

static void test_gpu_path(dg_engine* e) {
  dgm_term_ops o = ops();
  dgm_universe* u = dgm_universe_new(&o);
  trep ta, tb;
  make_replicas(&ta, &tb, 3000);
  dgm_rows ra, rb, sa, sb;
  dgm_rows_init(&ra, 1024, 16);
  dgm_rows_init(&rb, 1024, 16);
  dgm_rows_init(&sa, 1024, 16);
  dgm_rows_init(&sb, 1024, 16);
  marshal(u, &ta, &ra);
  marshal(u, &tb, &rb);
  host_sorted(&ra, &sa);
  host_sorted(&rb, &sb);

  /* the oracle on host-sorted rows */
  const uint64_t cap = sa.s.n + sb.s.n;
  dgm_rows want;
  dgm_rows_init(&want, cap, sa.c.n + sb.c.n);
  DG(ref_join2(&sa.s, &sa.c, &sb.s, &sb.c, NULL, 0, &want.s, &want.c));

  /* the device: upload the map-order rows, sort, join, read */
  dg_store da, db, xa, xb, dj, hj;
  dg_context dca, dcb, xca, xcb, dcj;
  DG(dg_store_alloc(e, ra.s.n, &da));
  DG(dg_store_alloc(e, rb.s.n, &db));
  DG(dg_store_alloc(e, ra.s.n, &xa));
  DG(dg_store_alloc(e, rb.s.n, &xb));
  DG(dg_store_alloc(e, cap, &dj));
  DG(dg_context_alloc(e, ra.c.n, &dca));
  DG(dg_context_alloc(e, rb.c.n, &dcb));
  DG(dg_context_alloc(e, ra.c.n, &xca));
  DG(dg_context_alloc(e, rb.c.n, &xcb));
  DG(dg_context_alloc(e, ra.c.n + rb.c.n, &dcj));
  DG(dg_store_upload(e, &ra.s, &da));
  DG(dg_store_upload(e, &rb.s, &db));
  DG(dg_context_upload(e, &ra.c, &dca));
  DG(dg_context_upload(e, &rb.c, &dcb));
  DG(dg_sort_store(e, &da, &xa));
  DG(dg_sort_store(e, &db, &xb));
  DG(dg_sort_context(e, &dca, &xca));
  DG(dg_sort_context(e, &dcb, &xcb));
  CHECK(xa.n == sa.s.n && xb.n == sb.s.n);
  DG(dg_store_check(e, &xa));
  DG(dg_join2(e, &xa, &xca, &xb, &xcb, NULL, 0, &dj, &dcj));
  dgm_rows got;
  dgm_rows_init(&got, cap, ra.c.n + rb.c.n);
  hj = got.s;
  DG(dg_store_download(e, &dj, &hj));
  got.s.n = hj.n;
  CHECK(got.s.n == want.s.n);
  CHECK(!memcmp(got.s.key, want.s.key, want.s.n * 8) && !memcmp(got.s.val, want.s.val, want.s.n * 8) &&
        !memcmp(got.s.ts, want.s.ts, want.s.n * 8) && !memcmp(got.s.node, want.s.node, want.s.n * 4) &&
        !memcmp(got.s.cnt, want.s.cnt, want.s.n * 8));
  dg_context hc = got.c;
  DG(dg_context_download(e, &dcj, &hc));
  CHECK(hc.n == want.c.n && !memcmp(hc.node, want.c.node, hc.n * 4) &&
        !memcmp(hc.cnt, want.c.cnt, hc.n * 8));

  /* read/1 on the device == the oracle == the TERM-order tie-break */
  uint64_t *dk, *dv, n_read = 0;
  DG(dg_buffer_alloc(e, cap * 8, (void**)&dk));
  DG(dg_buffer_alloc(e, cap * 8, (void**)&dv));
  DG(dg_read_lww(e, &dj, NULL, 0, dk, dv, cap, &n_read));
  uint64_t* gk = (uint64_t*)malloc(cap * 8);
  uint64_t* gv = (uint64_t*)malloc(cap * 8);
  DG(dg_copy_to_host(e, gk, dk, n_read * 8));
  DG(dg_copy_to_host(e, gv, dv, n_read * 8));
  uint64_t* wk = (uint64_t*)malloc(cap * 8);
  uint64_t* wv = (uint64_t*)malloc(cap * 8);
  uint64_t n_want = 0;
  DG(ref_read_lww(&want.s, NULL, 0, wk, wv, cap, &n_want));
  CHECK(n_read == n_want && !memcmp(gk, wk, n_read * 8) && !memcmp(gv, wv, n_read * 8));
  readst rs;
  memset(&rs, 0, sizeof rs);
  rs.u = u;
  rs.keys = (uint64_t*)malloc(cap * 8);
  rs.vals = (uint64_t*)malloc(cap * 8);
  dgm_walk w = {w_key, w_entry, NULL};
  CHECK(dgm_walk_rows(&want.s, &w, &rs) == 0);
  flush(&rs);
  CHECK(rs.n == n_read && !memcmp(rs.keys, gk, n_read * 8) && !memcmp(rs.vals, gv, n_read * 8));
  printf("gpu marshal/sort/join/read ok: %llu + %llu rows -> %llu, %llu keys read\n",
         (unsigned long long)ra.s.n, (unsigned long long)rb.s.n, (unsigned long long)want.s.n,
         (unsigned long long)n_read);

  /* part 3: a relabel rewrites the device store (dg_remap_values) */
  int relabeled = 0;
  double hi = 2.0;
  tterm lo = tf(1.75);
  uint64_t id;
  int rl;
  CHECK(dgm_value(u, &lo, &id, &rl) == DG_OK);
  for (int i = 0; i < 100 && !relabeled; i++) {
    hi = (1.75 + hi) / 2;
    tterm t = tf(hi);
    CHECK(dgm_value(u, &t, &id, &relabeled) == DG_OK);
  }
  CHECK(relabeled);
  const uint64_t *old_ids, *new_ids;
  uint64_t nr;
  dgm_last_relabel(u, &old_ids, &new_ids, &nr);
  uint64_t *dold, *dnew;
  DG(dg_buffer_alloc(e, nr * 8, (void**)&dold));
  DG(dg_buffer_alloc(e, nr * 8, (void**)&dnew));
  DG(dg_copy_to_device(e, dold, old_ids, nr * 8));
  DG(dg_copy_to_device(e, dnew, new_ids, nr * 8));
  DG(dg_remap_values(e, &dj, dold, dnew, nr));
  DG(dg_store_download(e, &dj, &hj));
  for (uint64_t i = 0; i < hj.n; i++) {
    /* the same term as before the relabel, under its new id; ids outside the relabelled
     * region (canonical integers, the other region) unchanged */
    if (nr == 0 || want.s.val[i] < old_ids[0] || want.s.val[i] > old_ids[nr - 1]) {
      CHECK(hj.val[i] == want.s.val[i]);
      continue;
    }
    uint64_t lo_i = 0, hi_i = nr;
    while (lo_i < hi_i) {
      uint64_t mid = (lo_i + hi_i) / 2;
      if (old_ids[mid] < want.s.val[i]) lo_i = mid + 1; else hi_i = mid;
    }
    CHECK(lo_i < nr && new_ids[lo_i] == hj.val[i]);
  }
  DG(dg_store_check(e, &dj));
  printf("gpu relabel remap ok (%llu value ids re-spaced)\n", (unsigned long long)nr);

  dg_buffer_free(e, dk);
  dg_buffer_free(e, dv);
  dg_buffer_free(e, dold);
  dg_buffer_free(e, dnew);
  dg_store_free(e, &da);
  dg_store_free(e, &db);
  dg_store_free(e, &xa);
  dg_store_free(e, &xb);
  dg_store_free(e, &dj);
  dg_context_free(e, &dca);
  dg_context_free(e, &dcb);
  dg_context_free(e, &xca);
  dg_context_free(e, &xcb);
  dg_context_free(e, &dcj);
  free(gk);
  free(gv);
  free(wk);
  free(wv);
  free(rs.keys);
  free(rs.vals);
  dgm_rows_free(&ra);
  dgm_rows_free(&rb);
  dgm_rows_free(&sa);
  dgm_rows_free(&sb);
  dgm_rows_free(&want);
  dgm_rows_free(&got);
  free(ta.r);
  free(tb.r);
  dgm_universe_free(u);
}

int main(void) {
  test_universe();
  dg_engine* e = NULL;
  if (!device_present(&e)) {
    const char* req = getenv("DG_REQUIRE_GPU");
    if (req && req[0] == '1') {
      fprintf(stderr, "FAIL: no device (%s)\n", dg_last_error());
      return 1;
    }
    printf("SKIP gpu part: %s\n", dg_last_error());
    return 0;
  }
  test_gpu_path(e);
  dg_engine_destroy(e);
  printf("all ok\n");
  return 0;
}
