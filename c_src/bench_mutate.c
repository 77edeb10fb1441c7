/*
 * bench_mutate.c — per-operation latency of a local mutation applied to a device-resident
 * replica state through the C-ABI, the shape of the reference's own benchmark
 * (bench/basic_operations.exs:25-41): a replica set up with `n` adds of key x -> x
 * (1..n, one mutate each, so node 0's counter ends at n), then
 *   read    DeltaCrdt.read(crdt)                  read/1 of every key (dg_read_lww + D2H)
 *   add     mutate(crdt, :add, ["key4", "value"])  a new key              (rows move)
 *   update  mutate(crdt, :add, [10, 12])           key 10: one row -> one (in place)
 *   remove  mutate(crdt, :remove, [10])            key 10's row removed   (rows move)
 * with the reference's before_each (add [10, 10], remove ["key4"]) before every op.
 *
 * A mutation is handle_operation (causal_crdt.ex:337-342): AWLWWMap.add/remove builds a
 * one-key delta with a MapSet context (aw_lww_map.ex:99-146) from the replica's terms,
 * and update_state_with_delta (:383-404) joins it with keys = [key].  The delta is built
 * on the host here, as the Elixir side builds it from its own `value` map (INTEGRATION.md
 * §3), and each op goes through c_src/replica.c's dgr_join_delta -- the function the NIF's
 * join_delta calls -- so one op costs what the NIF pays below the term layer: the delta
 * packed into one page-locked message, the versioned in-place join (dg_join_delta_rows:
 * the keyed join, the changed keys, the MerkleMap put/delete), and the changed keys'
 * rows and the new context home with one wait.  `read` is dgr_read (the NIF's read/1),
 * with its engine-owned output buffers.
 * Also `batch`: the reference's trace workload (1000 x mutate(:add, ["key#{x}", "value"]),
 * :9-23) as ONE host-built delta through dgr_join_delta, and the same through
 * dgr_mutate_batch (the delta built on the device: the NIF's mutate_batch) -- how
 * mutate_async batches amortize.
 *
 * Built twice from this file: bench_mutate (the GPU path, links libdeltagpu) and, with
 * -DDG_REF, bench_mutate_ref (the CPU restatement's keyed join per op, oracle/deltaref.c
 * ref_join2 on host rows -- bench.py's cpu_baseline leg only).  Prints one JSON line.
 *     bench_mutate N_KEYS [REPS [ops]]   ("ops": the single-op sections only)
 */
#define _POSIX_C_SOURCE 200809L
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#ifndef DG_REF
#include <dlfcn.h>
#endif

#include "marshal.h"
#ifndef DG_REF
#include "replica.h"
#endif

#ifdef DG_REF
int ref_join2(const dg_store* a, const dg_context* ca, const dg_store* b, const dg_context* cb,
              const uint64_t* keys, uint64_t n_keys, dg_store* out, dg_context* out_ctx);
int ref_read_lww(const dg_store* s, const uint64_t* keys, uint64_t n_keys, uint64_t* out_key,
                 uint64_t* out_val, uint64_t cap, uint64_t* n_out);
int ref_store_diff(const dg_store* a, const dg_store* b, uint64_t* out, uint64_t cap, uint64_t* n);
#endif

#define DG(x)                                                                          \
  do {                                                                                 \
    int rc_ = (x);                                                                     \
    if (rc_ != DG_OK) {                                                                \
      fprintf(stderr, "FAIL %s:%d: %s -> %d (%s)\n", __FILE__, __LINE__, #x, rc_,        \
              dg_last_error());                                                        \
      exit(1);                                                                         \
    }                                                                                  \
  } while (0)

static double now_us(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec * 1e6 + t.tv_nsec * 1e-3;
}

static int cmp_d(const void* a, const void* b) {
  const double x = *(const double*)a, y = *(const double*)b;
  return x < y ? -1 : x > y;
}

static double median(double* v, int n) {
  qsort(v, (size_t)n, sizeof *v, cmp_d);
  return n ? v[n / 2] : 0.0;
}

static uint64_t key_int(int64_t k) {
  dgm_buf b = {0};
  dgm_enc_i64(&b, k);
  const uint64_t id = dgm_key_id(b.p, b.n);
  dgm_buf_free(&b);
  return id;
}

static uint64_t key_bin(const char* s) {
  dgm_buf b = {0};
  dgm_enc_binary(&b, s, strlen(s));
  const uint64_t id = dgm_key_id(b.p, b.n);
  dgm_buf_free(&b);
  return id;
}

static uint64_t val_int(int64_t v) { return (uint64_t)v + (UINT64_C(1) << 62); }
static const uint64_t VAL_VALUE = (UINT64_C(1) << 63) + 4096;  /* "value": a table id */

/* ---------------------------------------------------------------- host rows */
typedef struct {
  uint64_t *key, *val, *cnt;
  int64_t* ts;
  uint32_t* node;
  uint64_t n, cap;
} hrows;

static void hrows_init(hrows* r, uint64_t cap) {
  r->key = calloc(cap, 8);
  r->val = calloc(cap, 8);
  r->cnt = calloc(cap, 8);
  r->ts = calloc(cap, 8);
  r->node = calloc(cap, 4);
  r->n = 0;
  r->cap = cap;
}

static dg_store hview(hrows* r) {
  dg_store s = {r->key, r->val, r->ts, r->node, r->cnt, r->n, r->cap};
  return s;
}

/* the replica after `n` adds of x -> x: rows sorted by (key id, ...), dot (0, x) */
typedef struct {
  uint64_t key;
  uint64_t x;
} kx;

static int cmp_kx(const void* a, const void* b) {
  const uint64_t x = ((const kx*)a)->key, y = ((const kx*)b)->key;
  return x < y ? -1 : x > y;
}

static void setup_rows(hrows* r, int64_t n) {
  kx* v = malloc((size_t)n * sizeof *v);
  for (int64_t x = 1; x <= n; x++) {
    v[x - 1].key = key_int(x);
    v[x - 1].x = (uint64_t)x;
  }
  qsort(v, (size_t)n, sizeof *v, cmp_kx);
  for (int64_t i = 0; i < n; i++) {
    r->key[i] = v[i].key;
    r->val[i] = val_int((int64_t)v[i].x);
    r->ts[i] = (int64_t)v[i].x;
    r->node[i] = 0;
    r->cnt[i] = v[i].x;
  }
  r->n = (uint64_t)n;
  free(v);
}

static int cmp_u64(const void* a, const void* b) {
  const uint64_t x = *(const uint64_t*)a, y = *(const uint64_t*)b;
  return x < y ? -1 : x > y;
}

/* ---------------------------------------------------------------- one-key deltas */
/* A delta as the reference's add/remove builds it (aw_lww_map.ex:99-146): the key's old
 * dots plus (add) the fresh dot {0, c + 1} as a MapSet context, and (add) one row. */
typedef struct {
  uint64_t key, val, cnt;
  int64_t ts;
  int has_row;
  uint32_t dnode[2];
  uint64_t dcnt[2];
  int nd;
} delta1;

typedef struct {
  uint64_t c;        /* node 0's counter (its VV entry) */
  int64_t clock;     /* the add timestamps */
  uint64_t dot10;    /* key 10's current dot counter (0: absent) */
  uint64_t dot_k4;   /* "key4"'s */
} replica;

static delta1 mk_add(replica* R, uint64_t key, uint64_t val, uint64_t* cur) {
  delta1 d;
  memset(&d, 0, sizeof d);
  d.key = key;
  d.val = val;
  d.ts = ++R->clock;
  d.cnt = ++R->c;
  d.has_row = 1;
  if (*cur) { /* the old dot, then the new one (both node 0: ascending counters) */
    d.dnode[d.nd] = 0;
    d.dcnt[d.nd++] = *cur;
  }
  d.dnode[d.nd] = 0;
  d.dcnt[d.nd++] = d.cnt;
  *cur = d.cnt;
  return d;
}

static delta1 mk_remove(uint64_t key, uint64_t* cur) {
  delta1 d;
  memset(&d, 0, sizeof d);
  d.key = key;
  if (*cur) {
    d.dnode[d.nd] = 0;
    d.dcnt[d.nd++] = *cur;
  }
  *cur = 0;
  return d;
}

enum { OP_READ = 0, OP_ADD, OP_UPDATE, OP_REMOVE, N_OPS };
static const char* OP_NAMES[N_OPS] = {"read", "add", "update", "remove"};

#ifndef DG_REF
/* ================================================================ the GPU path */
/* Everything goes through c_src/replica.c, the code the NIF runs (deltagpu_nif.c's
 * join_delta / mutate_batch / read): the delta packed into ONE page-locked message, the
 * versioned in-place join with the MerkleMap update, the changed keys, their rows and the
 * new context home with one wait, engine-owned buffers (no allocation per call). */
typedef struct {
  dgr_engine* g;
  dgr_state* s;
  uint64_t version;
} gpu;

static void gpu_upload(gpu* g, hrows* r) {
  DG(dgr_engine_open(0, &g->g));
  dg_store hs = hview(r);
  uint32_t n0 = 0;
  uint64_t c0 = r->n;
  dg_context hc = {DG_CTX_VV, 0, &n0, &c0, 1, 1};
  DG(dgr_state_load(g->g, &hs, &hc, &g->s));
  g->version = dgr_state_version(g->s);
  /* the MerkleMap: ~3 keys per bucket (the bench's config-4 rule); rows hashed by id */
  uint32_t depth = 8;
  while (depth < 28 && (UINT64_C(3) << depth) < r->n) depth++;
  DG(dgr_refresh_terms(g->g, NULL, 0, NULL, NULL, 0));
  DG(dgr_merkle_build(g->s, g->version, depth));
}

/* one delta as the NIF's join_delta applies it (host rows and dot list in, the changed
 * keys' rows and the context out) */
static void gpu_apply(gpu* g, const uint64_t* key, const uint64_t* val, const int64_t* ts,
                      const uint64_t* cnt, uint64_t n_rows, const uint32_t* dnode,
                      const uint64_t* dcnt, uint64_t nd, const uint64_t* keys, uint64_t nk,
                      double* t) {
  static uint32_t* node = NULL;
  static uint64_t node_cap = 0;
  if (node_cap < n_rows + 1) {
    free(node);
    node_cap = 2 * n_rows + 16;
    node = calloc(node_cap, 4);  /* every row of these deltas is node 0's */
  }
  dg_store ds = {(uint64_t*)key, (uint64_t*)val, (int64_t*)ts, node, (uint64_t*)cnt, n_rows, n_rows};
  dg_context dc = {DG_CTX_DOTS, 0, (uint32_t*)dnode, (uint64_t*)dcnt, nd, nd};
  dgr_changed c;
  const double t0 = now_us();
  DG(dgr_join_delta(g->s, g->version, &ds, &dc, keys, nk, &c));
  g->version = c.version;
  t[0] = 0;
  t[1] = now_us() - t0;
  t[2] = 0;
}

/* a batch of m adds by node 0 built ON THE DEVICE (the NIF's mutate_batch) */
static void gpu_mutate_batch(gpu* g, const uint64_t* key, const uint64_t* val, const int64_t* ts,
                             uint64_t m) {
  static uint8_t* kinds = NULL;
  if (!kinds) kinds = malloc(1 << 16);
  memset(kinds, 1, m);
  dgr_changed c;
  DG(dgr_mutate_batch(g->s, g->version, 0, m, kinds, key, val, ts, &c));
  g->version = c.version;
}

static void gpu_read(gpu* g) {
  const uint64_t *k, *v;
  uint64_t n = 0;
  DG(dgr_read(g->s, g->version, 1, NULL, 0, &k, &v, &n));
}
#else
/* ================================================================ the CPU restatement */
typedef struct {
  hrows st, out;
  uint32_t vv_node;
  uint64_t vv_cnt;
  uint64_t *rk, *rv, *diff;
} cpu;

static void cpu_apply(cpu* c, const uint64_t* key, const uint64_t* val, const int64_t* ts,
                      const uint64_t* cnt, uint64_t n_rows, const uint32_t* dnode,
                      const uint64_t* dcnt, uint64_t nd, const uint64_t* keys, uint64_t nk,
                      double* t) {
  const double t0 = now_us();
  uint32_t* node = calloc(n_rows ? n_rows : 1, 4);
  dg_store ds = {(uint64_t*)key, (uint64_t*)val, (int64_t*)ts, node, (uint64_t*)cnt, n_rows, n_rows};
  dg_context dc = {DG_CTX_DOTS, 0, (uint32_t*)dnode, (uint64_t*)dcnt, nd, nd};
  dg_store sa = hview(&c->st);
  dg_context ca = {DG_CTX_VV, 0, &c->vv_node, &c->vv_cnt, 1, 1};
  uint32_t* on = malloc((nd + 2) * 4);
  uint64_t* oc = malloc((nd + 2) * 8);
  dg_context octx = {DG_CTX_VV, 0, on, oc, 0, nd + 2};
  if (c->out.cap < c->st.n + n_rows) exit(2);
  dg_store so = hview(&c->out);
  if (ref_join2(&sa, &ca, &ds, &dc, keys, nk, &so, &octx) != 0) exit(3);
  /* diff/3's changed keys: the join's rows against the state's (causal_crdt.ex:344-352) */
  uint64_t n_diff = 0;
  if (ref_store_diff(&sa, &so, c->diff, c->st.n + so.n + 1, &n_diff) != 0) exit(4);
  c->out.n = so.n;
  hrows tmp = c->st;
  c->st = c->out;
  c->out = tmp;
  c->vv_cnt = oc[0];
  free(node);
  free(on);
  free(oc);
  const double t1 = now_us();
  t[0] = 0;
  t[1] = t1 - t0;
  t[2] = 0;
}
#endif

int main(int argc, char** argv) {
  const int64_t n = argc > 1 ? atoll(argv[1]) : 1000;
  const int reps = argc > 2 ? atoi(argv[2]) : 200;
  const int ops_only = argc > 3 && !strcmp(argv[3], "ops");  /* no batch sections (profiling) */
  hrows r;
  hrows_init(&r, (uint64_t)n + 16384);
  setup_rows(&r, n);
  replica R = {(uint64_t)n, n, 10, 0};
  const uint64_t K10 = key_int(10), K4 = key_bin("key4");
#ifndef DG_REF
  gpu g;
  memset(&g, 0, sizeof g);
  gpu_upload(&g, &r);
#define APPLY(...) gpu_apply(&g, __VA_ARGS__)
#else
  cpu c;
  memset(&c, 0, sizeof c);
  c.st = r;
  hrows_init(&c.out, (uint64_t)n + 16384);
  c.vv_node = 0;
  c.vv_cnt = (uint64_t)n;
  c.rk = calloc((size_t)n + 16384, 8);
  c.rv = calloc((size_t)n + 16384, 8);
  c.diff = calloc(2 * ((size_t)n + 16384), 8);
#define APPLY(...) cpu_apply(&c, __VA_ARGS__)
#endif
  double* ts[N_OPS][3];
  for (int o = 0; o < N_OPS; o++)
    for (int p = 0; p < 3; p++) ts[o][p] = calloc((size_t)reps, sizeof(double));
  double* tot[N_OPS];
  for (int o = 0; o < N_OPS; o++) tot[o] = calloc((size_t)reps, sizeof(double));

#define RUN_DELTA(dd, out3)                                                                \
  do {                                                                                     \
    const delta1 d_ = (dd);                                                                \
    APPLY(&d_.key, &d_.val, &d_.ts, &d_.cnt, (uint64_t)d_.has_row, d_.dnode, d_.dcnt,       \
          (uint64_t)d_.nd, &d_.key, 1, (out3));                                            \
  } while (0)

  double scratch[3];
#ifndef DG_REF
  /* a DG_SMALL_STAMPS library build (tools/small_stamps.sh): the small join's phase stamps
   * after every timed op, their medians printed per op (diagnostic; perturbs the timing) */
  typedef int (*stamps_fn)(unsigned long long*, size_t);
  stamps_fn stamps = (stamps_fn)dlsym(dlopen(NULL, RTLD_NOW), "dg_debug_small_stamps");
  double* sph[N_OPS][16];
  for (int o = 0; o < N_OPS; o++)
    for (int k = 0; k < 16; k++) sph[o][k] = calloc((size_t)reps, sizeof(double));
#endif
  for (int it = -5; it < reps; it++) {
    for (int o = 0; o < N_OPS; o++) {
      /* before_each: add [10, 10], remove ["key4"] */
      RUN_DELTA(mk_add(&R, K10, val_int(10), &R.dot10), scratch);
      RUN_DELTA(mk_remove(K4, &R.dot_k4), scratch);
      double t3[3] = {0, 0, 0};
      const double t0 = now_us();
      if (o == OP_READ) {
#ifndef DG_REF
        gpu_read(&g);
#else
        uint64_t nr = 0;
        dg_store sa = hview(&c.st);
        if (ref_read_lww(&sa, NULL, 0, c.rk, c.rv, c.st.n + 1, &nr) != 0) exit(5);
#endif
      } else if (o == OP_ADD) {
        RUN_DELTA(mk_add(&R, K4, VAL_VALUE, &R.dot_k4), t3);
      } else if (o == OP_UPDATE) {
        RUN_DELTA(mk_add(&R, K10, val_int(12), &R.dot10), t3);
      } else {
        RUN_DELTA(mk_remove(K10, &R.dot10), t3);
      }
      const double el = now_us() - t0;
      if (it >= 0) {
        tot[o][it] = el;
        for (int p = 0; p < 3; p++) ts[o][p][it] = t3[p];
#ifndef DG_REF
        if (stamps && o != OP_READ) {
          unsigned long long st[16];
          memset(st, 0, sizeof st);
          stamps(st, 16);
          for (int k = 1; k < 16; k++) /* phase k: from the previous nonzero stamp, us */
            sph[o][k][it] = (st[k] && st[0] && st[k] >= st[0]) ? (double)(st[k] - st[0]) * 0.01 : -1.0;
        }
#endif
      }
    }
  }
  /* the trace workload as one batched delta: 1000 adds of new keys "key<x>" */
  const int nb = 1000;
  uint64_t* bk = malloc(nb * 8);
  uint64_t *bv = malloc(nb * 8), *bc = malloc(nb * 8), *bd = malloc(nb * 8);
  int64_t* bt = malloc(nb * 8);
  uint32_t* bn = calloc(nb, 4);
  double bt_us[16];
  int n_batch = 0;
  for (int rep = 0; rep < (ops_only ? 0 : 6); rep++) {
    for (int i = 0; i < nb; i++) {
      char s[32];
      snprintf(s, sizeof s, "key%d_%d", i, rep);
      bk[i] = key_bin(s);
    }
    /* sorted keys; every add's fresh dot {0, c + 1 + i} (new keys: no old dots) */
    qsort(bk, nb, 8, cmp_u64);
    for (int i = 0; i < nb; i++) {
      bv[i] = VAL_VALUE;
      bt[i] = ++R.clock;
      bc[i] = R.c + 1 + (uint64_t)i;
      bd[i] = bc[i];
    }
    R.c += nb;
    double t3[3];
    const double t0 = now_us();
    APPLY(bk, bv, bt, bc, nb, bn, bd, nb, bk, nb, t3);
    const double el = now_us() - t0;
    if (rep) bt_us[n_batch++] = el;
  }
  double dmb[16];
  int n_dmb = 0;
#ifndef DG_REF
  /* the same workload with the delta built on the device (the NIF's mutate_batch) */
  for (int rep = 0; rep < (ops_only ? 0 : 6); rep++) {
    for (int i = 0; i < nb; i++) {
      char s[32];
      snprintf(s, sizeof s, "mkey%d_%d", i, rep);
      bk[i] = key_bin(s);
    }
    qsort(bk, nb, 8, cmp_u64);
    for (int i = 0; i < nb; i++) {
      bv[i] = VAL_VALUE;
      bt[i] = ++R.clock;
    }
    R.c += nb;
    const double t0 = now_us();
    gpu_mutate_batch(&g, bk, bv, bt, nb);
    const double el = now_us() - t0;
    if (rep) dmb[n_dmb++] = el;
  }
#endif
  printf("{\"n_keys\": %lld, \"reps\": %d, \"path\": \"%s\", \"us\": {", (long long)n, reps,
#ifndef DG_REF
         "gpu (c_src/replica.c: the NIF's calls)"
#else
         "cpu_restatement"
#endif
  );
  for (int o = 0; o < N_OPS; o++) {
    printf("%s\"%s\": %.2f", o ? ", " : "", OP_NAMES[o], median(tot[o], reps));
  }
  const double bmed = median(bt_us, n_batch);
  printf("}, \"batch_1000_adds_us\": %.2f, \"batch_us_per_op\": %.3f", bmed, bmed / nb);
  if (n_dmb) {
    const double m2 = median(dmb, n_dmb);
    printf(", \"mutate_batch_1000_adds_us\": %.2f, \"mutate_batch_us_per_op\": %.3f", m2, m2 / nb);
  }
  printf("}\n");
#ifndef DG_REF
  if (stamps)
    for (int o = 1; o < N_OPS; o++) {
      printf("stamps %-6s (us from kernel start):", OP_NAMES[o]);
      for (int k = 1; k < 16; k++) {
        const double m = median(sph[o][k], reps);
        if (m >= 0) printf(" %d:%.2f", k, m);
      }
      printf("\n");
    }
  dgr_state_free(g.s);
  dgr_engine_close(g.g);
#endif
  return 0;
}
