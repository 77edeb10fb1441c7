/*
 * replica.c — the NIF's device-resident replica state (replica.h): versions, the packed
 * delta message, the return block, engine-owned buffers.  Plain C over libdeltagpu's
 * C-ABI (include/deltagpu.h); no term in sight.
 */
#define _POSIX_C_SOURCE 200809L
#include "replica.h"

#include <stdlib.h>
#include <string.h>

struct dgr_state {
  dgr_engine* g;
  dg_store rows;
  dg_store spare; /* dg_join_delta's second buffer (allocated on first need, kept) */
  dg_context ctx;
  dg_merkle tree;
  int has_tree;
  uint64_t version;
  dgr_state *prev, *next;
};

struct dgr_engine {
  dg_engine* e;
  dgr_state* live;
  uint64_t n_live;
  /* the universe's term hashes on the device; every tree points at th */
  dg_term_hashes th;
  uint64_t *d_nh, *d_vid, *d_vh;
  uint64_t nh_cap, vid_cap, vh_cap;
  uint64_t th_nodes, th_vals;
  int th_stale;
  /* the packed message (a delta, a key list, ops, a continuation): page-locked host
   * words and their device copy */
  uint64_t *h_msg, *d_msg;
  uint64_t msg_cap;
  /* a delta sorted on the device when the map walk did not give the order */
  dg_store drows;
  dg_context dctx;
  /* dg_mutate_batch's delta, its dot list and touched keys */
  dg_store mrows;
  dg_context mctx;
  uint64_t* mkeys;
  uint64_t mkeys_cap;
  /* the return block (words): changed keys [0, S) | key | val | ts | cnt [S, 5S) |
   * node u32 [5S, 6S) | context cnt [6S, 6S + C) | context node u32 [6S + C, 6S + 2C) */
  uint64_t *d_back, *h_back;
  uint64_t back_s, back_c;
  /* dg_join_delta_home's result block (page-locked, DG_HOME_WORDS) */
  uint64_t* h_home;
  /* read output: keys [0, cap) | values [cap, 2 cap) */
  uint64_t *d_rd, *h_rd;
  uint64_t rd_cap, h_rd_cap;
  /* take output */
  dg_store tk;
  uint64_t* h_tk;
  uint64_t h_tk_cap;
  /* continuations: the output (device), the keys, and the bytes handed back */
  dg_merkle_cont co;
  uint64_t *d_ckeys, *h_ckeys, *h_cstage;
  uint64_t ckeys_cap, h_ckeys_cap, h_cstage_cap;
  uint8_t* h_bin;
  uint64_t bin_cap;
};

#define TRY(x)                     \
  do {                             \
    const int rc_ = (x);           \
    if (rc_ != DG_OK) return rc_;  \
  } while (0)

static uint64_t umax(uint64_t a, uint64_t b) { return a > b ? a : b; }
static uint64_t umin(uint64_t a, uint64_t b) { return a < b ? a : b; }
static uint64_t even(uint64_t w) { return (w + 1) & ~UINT64_C(1); } /* 16-B aligned offsets */

/* ------------------------------------------------------------ buffers */
static int grow_dev(dgr_engine* g, uint64_t** p, uint64_t* cap, uint64_t words) {
  if (*p && *cap >= words) return DG_OK;
  const uint64_t want = umax(words, 2 * *cap) + 16;
  TRY(dg_buffer_free(g->e, *p));
  *p = NULL;
  *cap = 0;
  TRY(dg_buffer_alloc(g->e, want * 8, (void**)p));
  *cap = want;
  return DG_OK;
}

static int grow_host(dgr_engine* g, uint64_t** p, uint64_t* cap, uint64_t words) {
  if (*p && *cap >= words) return DG_OK;
  const uint64_t want = umax(words, 2 * *cap) + 16;
  TRY(dg_host_free(g->e, *p));
  *p = NULL;
  *cap = 0;
  TRY(dg_host_alloc(g->e, want * 8, (void**)p));
  *cap = want;
  return DG_OK;
}

/* the message buffers (host and device, the same capacity) */
static int grow_msg(dgr_engine* g, uint64_t words) {
  if (g->h_msg && g->msg_cap >= words) return DG_OK;
  const uint64_t want = umax(words, 2 * g->msg_cap) + 64;
  TRY(dg_host_free(g->e, g->h_msg));
  TRY(dg_buffer_free(g->e, g->d_msg));
  g->h_msg = g->d_msg = NULL;
  g->msg_cap = 0;
  TRY(dg_host_alloc(g->e, want * 8, (void**)&g->h_msg));
  TRY(dg_buffer_alloc(g->e, want * 8, (void**)&g->d_msg));
  g->msg_cap = want;
  return DG_OK;
}

static int grow_store(dgr_engine* g, dg_store* s, uint64_t n) {
  if (s->key && s->cap >= n) return DG_OK;
  const uint64_t want = umax(n, 2 * s->cap) + 16;
  TRY(dg_store_free(g->e, s));
  return dg_store_alloc(g->e, want, s);
}

static int grow_ctx(dgr_engine* g, dg_context* c, uint64_t n) {
  if (c->node && c->cap >= n) return DG_OK;
  const int32_t kind = c->kind;
  TRY(dg_context_free(g->e, c));
  TRY(dg_context_alloc(g->e, umax(n, 2 * c->cap) + 16, c));
  c->kind = kind;
  return DG_OK;
}

static int grow_cont(dgr_engine* g, dg_merkle_cont* c, uint64_t cap, uint64_t cap_b) {
  if (!c->pos || c->cap < cap) {
    TRY(dg_buffer_free(g->e, c->pos));
    TRY(dg_buffer_free(g->e, c->hash));
    c->pos = c->hash = NULL;
    c->cap = 0;
    const uint64_t want = umax(cap, 16);
    TRY(dg_buffer_alloc(g->e, want * 8, (void**)&c->pos));
    TRY(dg_buffer_alloc(g->e, want * 8, (void**)&c->hash));
    c->cap = want;
  }
  if (!c->bucket || c->cap_buckets < cap_b) {
    TRY(dg_buffer_free(g->e, c->bucket));
    c->bucket = NULL;
    c->cap_buckets = 0;
    const uint64_t want = umax(cap_b, 16);
    TRY(dg_buffer_alloc(g->e, want * 8, (void**)&c->bucket));
    c->cap_buckets = want;
  }
  return DG_OK;
}

/* The return block for S changed keys / rows and a context of C entries (contents not
 * kept). */
static int grow_back(dgr_engine* g, uint64_t S, uint64_t C) {
  if (g->d_back && g->back_s >= S && g->back_c >= C) return DG_OK;
  S = umax(umax(S, g->back_s), 64);
  C = umax(umax(C, g->back_c), 64);
  TRY(dg_buffer_free(g->e, g->d_back));
  TRY(dg_host_free(g->e, g->h_back));
  g->d_back = g->h_back = NULL;
  g->back_s = g->back_c = 0;
  TRY(dg_buffer_alloc(g->e, (6 * S + 2 * C) * 8, (void**)&g->d_back));
  TRY(dg_host_alloc(g->e, (6 * S + 2 * C) * 8, (void**)&g->h_back));
  g->back_s = S;
  g->back_c = C;
  return DG_OK;
}

static dg_store back_rows(uint64_t* b, uint64_t S) {
  dg_store r = {b + S, b + 2 * S, (int64_t*)(b + 3 * S), (uint32_t*)(b + 5 * S), b + 4 * S, 0, S};
  return r;
}

/* ------------------------------------------------------------ host packing */
static int cmp_u64(const void* a, const void* b) {
  const uint64_t x = *(const uint64_t*)a, y = *(const uint64_t*)b;
  return x < y ? -1 : x > y;
}

/* keys -> ascending unique at dst; returns their number */
static uint64_t sort_unique(const uint64_t* keys, uint64_t n, uint64_t* dst) {
  if (n) memcpy(dst, keys, n * 8);
  qsort(dst, n, 8, cmp_u64);
  uint64_t m = 0;
  for (uint64_t i = 0; i < n; i++)
    if (!m || dst[m - 1] != dst[i]) dst[m++] = dst[i];
  return m;
}

static int rows_sorted(const dg_store* s) {
  for (uint64_t i = 1; i < s->n; i++) {
    const uint64_t a[5] = {s->key[i - 1], s->val[i - 1], (uint64_t)s->ts[i - 1] ^ (UINT64_C(1) << 63),
                           s->node[i - 1], s->cnt[i - 1]};
    const uint64_t b[5] = {s->key[i], s->val[i], (uint64_t)s->ts[i] ^ (UINT64_C(1) << 63), s->node[i],
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

/* the host (page-locked, mapped) side of a device view into the message buffer: the small
 * join reads a small delta straight from there, with no copy launch */
static void* on_host(const dgr_engine* g, const void* d) {
  return (char*)g->h_msg + ((const char*)d - (const char*)g->d_msg);
}

static dg_store host_rows(const dgr_engine* g, const dg_store* d) {
  dg_store v = {(uint64_t*)on_host(g, d->key), (uint64_t*)on_host(g, d->val), (int64_t*)on_host(g, d->ts),
                (uint32_t*)on_host(g, d->node), (uint64_t*)on_host(g, d->cnt), d->n, d->cap};
  return v;
}

static dg_context host_ctx(const dgr_engine* g, const dg_context* d) {
  dg_context v = {d->kind, 0, (uint32_t*)on_host(g, d->node), (uint64_t*)on_host(g, d->cnt), d->n, d->cap};
  return v;
}

static uint64_t rows_words(uint64_t n) { return 4 * even(n) + even((n + 1) / 2); }
static uint64_t ctx_words(uint64_t n) { return even(n) + even((n + 1) / 2); }

/* host rows into msg at word o; *dev = the device view of the same place */
static uint64_t pack_rows(dgr_engine* g, uint64_t o, const dg_store* r, dg_store* dev) {
  const uint64_t n = r->n, w = even(n);
  uint64_t* h = g->h_msg + o;
  uint64_t* d = g->d_msg + o;
  if (n) {
    memcpy(h, r->key, n * 8);
    memcpy(h + w, r->val, n * 8);
    memcpy(h + 2 * w, r->ts, n * 8);
    memcpy(h + 3 * w, r->cnt, n * 8);
    memcpy(h + 4 * w, r->node, n * 4);
  }
  dg_store v = {d, d + w, (int64_t*)(d + 2 * w), (uint32_t*)(d + 4 * w), d + 3 * w, n, n};
  *dev = v;
  return o + rows_words(n);
}

static uint64_t pack_ctx(dgr_engine* g, uint64_t o, const dg_context* c, dg_context* dev) {
  const uint64_t n = c->n, w = even(n);
  uint64_t* h = g->h_msg + o;
  uint64_t* d = g->d_msg + o;
  if (n) {
    memcpy(h, c->cnt, n * 8);
    memcpy(h + w, c->node, n * 4);
  }
  dg_context v = {c->kind, 0, (uint32_t*)(d + w), d, n, n};
  *dev = v;
  return o + ctx_words(n);
}

/* ------------------------------------------------------------ engine */
int dgr_engine_open(int device, dgr_engine** out) {
  if (!out) return DG_E_INVAL;
  *out = NULL;
  dgr_engine* g = (dgr_engine*)calloc(1, sizeof *g);
  if (!g) return DG_E_NOMEM;
  const int rc = dg_engine_create(device, NULL, &g->e);
  if (rc) {
    free(g);
    return rc;
  }
  g->th_stale = 1;
  g->mctx.kind = DG_CTX_DOTS;
  *out = g;
  return DG_OK;
}

int dgr_engine_close(dgr_engine* g) {
  if (!g) return DG_OK;
  if (g->live) return DG_E_INVAL; /* states first */
  dg_engine* e = g->e;
  dg_buffer_free(e, g->d_nh);
  dg_buffer_free(e, g->d_vid);
  dg_buffer_free(e, g->d_vh);
  dg_host_free(e, g->h_msg);
  dg_buffer_free(e, g->d_msg);
  dg_store_free(e, &g->drows);
  dg_context_free(e, &g->dctx);
  dg_store_free(e, &g->mrows);
  dg_context_free(e, &g->mctx);
  dg_buffer_free(e, g->mkeys);
  dg_buffer_free(e, g->d_back);
  dg_host_free(e, g->h_back);
  dg_host_free(e, g->h_home);
  dg_buffer_free(e, g->d_rd);
  dg_host_free(e, g->h_rd);
  dg_store_free(e, &g->tk);
  dg_host_free(e, g->h_tk);
  dg_buffer_free(e, g->co.pos);
  dg_buffer_free(e, g->co.hash);
  dg_buffer_free(e, g->co.bucket);
  dg_buffer_free(e, g->d_ckeys);
  dg_host_free(e, g->h_ckeys);
  dg_host_free(e, g->h_cstage);
  free(g->h_bin);
  const int rc = dg_engine_destroy(e);
  free(g);
  return rc;
}

dg_engine* dgr_dg(dgr_engine* g) { return g ? g->e : NULL; }
uint64_t dgr_live_states(const dgr_engine* g) { return g ? g->n_live : 0; }

int dgr_refresh_terms(dgr_engine* g, const uint64_t* node_hash, uint64_t n_nodes, const uint64_t* val_id,
                      const uint64_t* val_hash, uint64_t n_vals) {
  if (!g || (n_nodes && !node_hash) || (n_vals && (!val_id || !val_hash))) return DG_E_INVAL;
  if (g->th_stale || n_nodes != g->th_nodes) {
    g->th_nodes = 0;
    TRY(grow_dev(g, &g->d_nh, &g->nh_cap, n_nodes));
    TRY(dg_copy_to_device(g->e, g->d_nh, node_hash, n_nodes * 8));
    g->th_nodes = n_nodes;
  }
  if (g->th_stale || n_vals != g->th_vals) {
    g->th_vals = 0;
    TRY(grow_dev(g, &g->d_vid, &g->vid_cap, n_vals));
    TRY(grow_dev(g, &g->d_vh, &g->vh_cap, n_vals));
    TRY(dg_copy_to_device(g->e, g->d_vid, val_id, n_vals * 8));
    TRY(dg_copy_to_device(g->e, g->d_vh, val_hash, n_vals * 8));
    g->th_vals = n_vals;
  }
  g->th_stale = 0;
  g->th.node_hash = g->d_nh;
  g->th.n_nodes = g->th_nodes;
  g->th.val_id = g->d_vid;
  g->th.val_hash = g->d_vh;
  g->th.n_vals = g->th_vals;
  return DG_OK;
}

int dgr_remap(dgr_engine* g, const uint64_t* old_ids, const uint64_t* new_ids, uint64_t n) {
  if (!g || (n && (!old_ids || !new_ids))) return DG_E_INVAL;
  g->th_stale = 1; /* the value table's ids moved: re-upload before the next tree call */
  if (!n) return DG_OK;
  TRY(grow_msg(g, 2 * n));
  memcpy(g->h_msg, old_ids, n * 8);
  memcpy(g->h_msg + n, new_ids, n * 8);
  TRY(dg_copy_async(g->e, g->d_msg, g->h_msg, 2 * n * 8));
  for (dgr_state* s = g->live; s; s = s->next)
    TRY(dg_remap_values(g->e, &s->rows, g->d_msg, g->d_msg + n, n));
  return DG_OK;
}

/* ------------------------------------------------------------ states */
static void link_state(dgr_engine* g, dgr_state* s) {
  s->next = g->live;
  if (g->live) g->live->prev = s;
  g->live = s;
  g->n_live++;
}

static void free_tree(dgr_state* s) {
  dg_engine* e = s->g->e;
  if (s->has_tree || s->tree.nodes) {
    dg_buffer_free(e, s->tree.nodes);
    dg_buffer_free(e, s->tree.counts);
    dg_buffer_free(e, s->tree.starts);
  }
  memset(&s->tree, 0, sizeof s->tree);
  s->has_tree = 0;
}

int dgr_state_free(dgr_state* s) {
  if (!s) return DG_OK;
  dgr_engine* g = s->g;
  if (s->prev) s->prev->next = s->next; else g->live = s->next;
  if (s->next) s->next->prev = s->prev;
  g->n_live--;
  dg_store_free(g->e, &s->rows);
  dg_store_free(g->e, &s->spare);
  dg_context_free(g->e, &s->ctx);
  free_tree(s);
  free(s);
  return DG_OK;
}

int dgr_state_load(dgr_engine* g, const dg_store* rows, const dg_context* ctx, dgr_state** out) {
  if (!g || !rows || !ctx || !out) return DG_E_INVAL;
  *out = NULL;
  dgr_state* s = (dgr_state*)calloc(1, sizeof *s);
  if (!s) return DG_E_NOMEM;
  s->g = g;
  link_state(g, s);
  int rc = dg_store_alloc(g->e, umax(rows->n, 1), &s->rows);
  if (!rc) rc = dg_context_alloc(g->e, umax(2 * ctx->n, 16), &s->ctx);
  if (!rc) rc = grow_msg(g, rows_words(rows->n) + ctx_words(ctx->n));
  dg_store rv;
  dg_context cv;
  if (!rc) {
    const uint64_t o = pack_rows(g, 0, rows, &rv);
    const uint64_t w = pack_ctx(g, o, ctx, &cv);
    rc = dg_copy_async(g->e, g->d_msg, g->h_msg, w * 8);
  }
  /* the map walk's order -> the store's (the radix sort also drops exact duplicates) */
  if (!rc && rows->n) rc = dg_sort_store(g->e, &rv, &s->rows);
  if (!rc && ctx->n) rc = dg_sort_context(g->e, &cv, &s->ctx);
  s->ctx.kind = ctx->kind;
  if (!rc && !ctx->n) s->ctx.n = 0;
  if (rc) {
    dgr_state_free(s);
    return rc;
  }
  s->version = 1;
  *out = s;
  return DG_OK;
}

uint64_t dgr_state_version(const dgr_state* s) { return s ? s->version : 0; }
uint64_t dgr_state_rows(const dgr_state* s) { return s ? s->rows.n : 0; }
int dgr_state_has_tree(const dgr_state* s) { return s ? s->has_tree : 0; }

static int check_version(const dgr_state* s, uint64_t version) {
  return version == s->version ? DG_OK : DGR_E_STALE;
}

/* the spare buffer and the context's room for a union with `dn` more entries, grown */
static int room_for(dgr_state* s, uint64_t rows, uint64_t dn) {
  dgr_engine* g = s->g;
  if (s->spare.cap < s->rows.n + rows) {
    TRY(dg_store_free(g->e, &s->spare));
    TRY(dg_store_alloc(g->e, 2 * (s->rows.n + rows) + 16, &s->spare));
  }
  if (s->ctx.cap < s->ctx.n + dn) {
    dg_context nctx;
    memset(&nctx, 0, sizeof nctx);
    TRY(dg_context_alloc(g->e, 2 * (s->ctx.n + dn) + 16, &nctx));
    int rc = dg_copy_async(g->e, nctx.node, s->ctx.node, s->ctx.n * 4);
    if (!rc) rc = dg_copy_async(g->e, nctx.cnt, s->ctx.cnt, s->ctx.n * 8);
    if (rc) {
      dg_context_free(g->e, &nctx);
      return rc;
    }
    nctx.n = s->ctx.n;
    nctx.kind = s->ctx.kind;
    TRY(dg_context_free(g->e, &s->ctx)); /* (waits for the copies) */
    s->ctx = nctx;
  }
  return DG_OK;
}

/* A small delta (a local mutation, a small sync delta): dg_join_delta_home does the whole
 * update_state_with_delta in one launch chain and writes the result into page-locked
 * memory with ONE wait.  *done = 0: not small after all (nothing happened). */
static int small_fits(const dgr_state* s, const dg_store* drows, const dg_context* dctx, uint64_t n_keys) {
  return n_keys <= 512 && drows->n <= 512 && dctx->n <= 1024 && s->ctx.kind == DG_CTX_VV;
}

static int apply_small(dgr_state* s, const dg_store* drows, const dg_context* dctx, const uint64_t* dkeys,
                       uint64_t n_keys, dgr_changed* out, int* done) {
  dgr_engine* g = s->g;
  *done = 0;
  if (!small_fits(s, drows, dctx, n_keys)) return DG_OK;
  if (!g->h_home) TRY(dg_host_alloc(g->e, DG_HOME_WORDS * 8, (void**)&g->h_home));
  int swapped = 0;
  const int rc = dg_join_delta_home(g->e, &s->rows, &s->ctx, drows, dctx, dkeys, n_keys, &s->spare,
                                    s->has_tree ? &s->tree : NULL, g->h_home, &swapped);
  if (rc) {
    s->version++;
    return rc;
  }
  const uint64_t* h = g->h_home;
  if (h[0] & DG_HOME_FALLBACK) return DG_OK;
  s->version++;
  *done = 1;
  uint64_t* r = g->h_home + DG_HOME_ROWS;
  const uint64_t S = DG_HOME_STRIDE;
  out->version = s->version;
  out->n_changed = h[1];
  out->keys = h + DG_HOME_KEYS;
  dg_store rows = {r, r + S, (int64_t*)(r + 2 * S), (uint32_t*)(r + 4 * S), r + 3 * S, h[2], S};
  out->rows = rows;
  dg_context c = {DG_CTX_VV, 0, (uint32_t*)(g->h_home + DG_HOME_CTX + DG_HOME_NODES),
                  g->h_home + DG_HOME_CTX, h[3], DG_HOME_NODES};
  out->ctx = c;
  return DG_OK;
}

/* The join of a delta on the device (rows and context sorted, keys ascending unique) into
 * the state, and the result brought home with one wait.  try_small: the small join first. */
static int apply_delta(dgr_state* s, const dg_store* drows, const dg_context* dctx, const uint64_t* dkeys,
                       uint64_t n_keys, dgr_changed* out, int try_small) {
  dgr_engine* g = s->g;
  TRY(room_for(s, drows->n, dctx->n));
  if (try_small) {
    int done = 0;
    TRY(apply_small(s, drows, dctx, dkeys, n_keys, out, &done));
    if (done) return DG_OK;
  }
  /* the changed keys, their rows and the joined context straight into the page-locked
   * block (dg_join_delta_out: the kernels write it, one wait); rows of the changed keys
   * past the block (a key with several entries) are taken afterwards */
  uint64_t S = umax(2 * n_keys + 64, 1);
  TRY(grow_back(g, S, s->ctx.n + dctx->n));
  S = g->back_s;
  uint64_t C = g->back_c;
  uint64_t* hb = g->h_back;
  dg_store tk = back_rows(hb, S);
  dg_context co = {DG_CTX_VV, 0, (uint32_t*)(hb + 6 * S + C), hb + 6 * S, 0, C};
  uint64_t n_changed = 0;
  int swapped = 0;
  const int rc = dg_join_delta_out(g->e, &s->rows, &s->ctx, drows, dctx, dkeys, n_keys, &s->spare,
                                   s->has_tree ? &s->tree : NULL, hb, S, &n_changed, &swapped, &tk, &co);
  s->version++; /* applied, or failed: either way no older struct reads the device again */
  TRY(rc);
  if (tk.n > tk.cap || co.n > co.cap) {
    /* park the changed keys, grow the block, take the rows from the joined state and copy
     * the context (the kernels write the page-locked block directly) */
    TRY(grow_msg(g, n_changed + 1));
    memcpy(g->h_msg, hb, n_changed * 8);
    TRY(grow_back(g, umax(tk.n, n_changed), s->ctx.n));
    S = g->back_s;
    C = g->back_c;
    hb = g->h_back;
    memcpy(hb, g->h_msg, n_changed * 8);
    TRY(dg_copy_async(g->e, g->d_msg, g->h_msg, n_changed * 8));
    tk = back_rows(hb, S);
    TRY(dg_take_keys(g->e, &s->rows, g->d_msg, n_changed, &tk));
    TRY(dg_copy_async(g->e, hb + 6 * S, s->ctx.cnt, s->ctx.n * 8));
    TRY(dg_copy_async(g->e, hb + 6 * S + C, s->ctx.node, s->ctx.n * 4));
    TRY(dg_engine_sync(g->e));
    co.n = s->ctx.n;
    co.kind = s->ctx.kind;
  }
  out->version = s->version;
  out->n_changed = n_changed;
  out->keys = hb;
  out->rows = back_rows(hb, S);
  out->rows.n = tk.n;
  dg_context c = {co.kind, 0, (uint32_t*)(hb + 6 * S + C), hb + 6 * S, co.n, C};
  out->ctx = c;
  return DG_OK;
}

int dgr_join_delta(dgr_state* s, uint64_t version, const dg_store* delta, const dg_context* delta_ctx,
                   const uint64_t* keys, uint64_t n_keys, dgr_changed* out) {
  if (!s || !delta || !delta_ctx || !out || (n_keys && !keys)) return DG_E_INVAL;
  TRY(check_version(s, version));
  dgr_engine* g = s->g;
  /* ONE message: rows | context | keyset (sorted, unique) */
  TRY(grow_msg(g, rows_words(delta->n) + ctx_words(delta_ctx->n) + n_keys + 2));
  dg_store rv;
  dg_context cv;
  uint64_t o = pack_rows(g, 0, delta, &rv);
  o = pack_ctx(g, o, delta_ctx, &cv);
  const uint64_t nk = sort_unique(keys, n_keys, g->h_msg + o);
  const uint64_t* dk = g->d_msg + o;
  if (rows_sorted(delta) && ctx_sorted(delta_ctx) && small_fits(s, delta, delta_ctx, nk)) {
    /* a mutation or a small sync delta: the small join reads the message where the host
     * packed it (mapped memory) -- no copy launch; declined, the general path copies it */
    const dg_store hr = host_rows(g, &rv);
    const dg_context hc = host_ctx(g, &cv);
    TRY(room_for(s, delta->n, delta_ctx->n));
    int done = 0;
    TRY(apply_small(s, &hr, &hc, g->h_msg + o, nk, out, &done));
    if (done) return DG_OK;
    TRY(dg_copy_async(g->e, g->d_msg, g->h_msg, (o + nk) * 8));
    return apply_delta(s, &rv, &cv, dk, nk, out, 0);
  }
  TRY(dg_copy_async(g->e, g->d_msg, g->h_msg, (o + nk) * 8));
  const dg_store* dr = &rv;
  const dg_context* dc = &cv;
  if (!rows_sorted(delta)) { /* a map walk of more than 32 keys: HAMT order */
    TRY(grow_store(g, &g->drows, delta->n));
    TRY(dg_sort_store(g->e, &rv, &g->drows));
    dr = &g->drows;
  }
  if (!ctx_sorted(delta_ctx)) {
    TRY(grow_ctx(g, &g->dctx, delta_ctx->n));
    TRY(dg_sort_context(g->e, &cv, &g->dctx));
    dc = &g->dctx;
  }
  return apply_delta(s, dr, dc, dk, nk, out, 1);
}

typedef struct {
  uint64_t key;
  uint64_t idx;
} kidx;

static int cmp_kidx(const void* a, const void* b) { /* by key, then batch order: stable */
  const kidx *x = (const kidx*)a, *y = (const kidx*)b;
  if (x->key != y->key) return x->key < y->key ? -1 : 1;
  return x->idx < y->idx ? -1 : x->idx > y->idx;
}

int dgr_mutate_batch(dgr_state* s, uint64_t version, uint32_t node, uint64_t m, const uint8_t* kind,
                     const uint64_t* key, const uint64_t* val, const int64_t* ts, dgr_changed* out) {
  if (!s || !out || (m && (!kind || !key || !val || !ts))) return DG_E_INVAL;
  TRY(check_version(s, version));
  dgr_engine* g = s->g;
  /* kind | key | val | ts | add_rank, sorted by key (batch order within a key), one copy */
  kidx* ord = (kidx*)malloc((m ? m : 1) * sizeof *ord);
  if (!ord) return DG_E_NOMEM;
  for (uint64_t i = 0; i < m; i++) {
    ord[i].key = key[i];
    ord[i].idx = i;
  }
  qsort(ord, m, sizeof *ord, cmp_kidx);
  int rc = grow_msg(g, 4 * m + (m + 7) / 8 + 2);
  if (rc) {
    free(ord);
    return rc;
  }
  uint64_t* h = g->h_msg;
  uint8_t* hk = (uint8_t*)(h + 4 * m);
  uint64_t n_adds = 0;
  uint64_t* rank = (uint64_t*)malloc((m ? m : 1) * 8);
  if (!rank) {
    free(ord);
    return DG_E_NOMEM;
  }
  for (uint64_t i = 0; i < m; i++) { /* the adds before each op, in batch order */
    rank[i] = n_adds;
    n_adds += kind[i] != 0;
  }
  for (uint64_t j = 0; j < m; j++) {
    const uint64_t i = ord[j].idx;
    h[j] = key[i];
    h[m + j] = kind[i] ? val[i] : 0;
    h[2 * m + j] = kind[i] ? (uint64_t)ts[i] : 0;
    h[3 * m + j] = rank[i];
    hk[j] = kind[i] != 0;
  }
  free(ord);
  free(rank);
  const uint64_t words = 4 * m + (m + 7) / 8;
  TRY(dg_copy_async(g->e, g->d_msg, h, words * 8));
  const uint64_t* d = g->d_msg;
  TRY(grow_store(g, &g->mrows, umax(m, 1)));
  TRY(grow_dev(g, &g->mkeys, &g->mkeys_cap, umax(m, 1)));
  uint64_t n_keys = 0;
  for (int attempt = 0;; attempt++) {
    TRY(grow_ctx(g, &g->mctx, attempt ? s->rows.n + n_adds + 1 : 8 * m + n_adds + 1));
    g->mctx.kind = DG_CTX_DOTS;
    g->mrows.n = 0;
    rc = dg_mutate_batch_async(g->e, &s->rows, &s->ctx, node, m, (const uint8_t*)(d + 4 * m), d, d + m,
                         (const int64_t*)(d + 2 * m), d + 3 * m, n_adds, &g->mrows, &g->mctx, g->mkeys,
                         g->mkeys_cap, &n_keys);
    if (rc == DG_E_CAPACITY && attempt == 0) continue;
    TRY(rc);
    break;
  }
  return apply_delta(s, &g->mrows, &g->mctx, g->mkeys, n_keys, out, 1);
}

int dgr_read(dgr_state* s, uint64_t version, int all, const uint64_t* keys, uint64_t n_keys,
             const uint64_t** out_key, const uint64_t** out_val, uint64_t* n_out) {
  if (!s || !out_key || !out_val || !n_out || (!all && n_keys && !keys)) return DG_E_INVAL;
  TRY(check_version(s, version));
  dgr_engine* g = s->g;
  *n_out = 0;
  uint64_t nk = 0;
  if (!all) {
    TRY(grow_msg(g, n_keys + 1));
    nk = sort_unique(keys, n_keys, g->h_msg);
    TRY(dg_copy_async(g->e, g->d_msg, g->h_msg, nk * 8));
  }
  const uint64_t cap = umax(all ? s->rows.n : umin(nk, s->rows.n), 1);
  TRY(grow_dev(g, &g->d_rd, &g->rd_cap, 2 * cap));
  TRY(grow_host(g, &g->h_rd, &g->h_rd_cap, g->rd_cap));
  const uint64_t half = g->rd_cap / 2;
  *out_key = g->h_rd;
  *out_val = g->h_rd + half;
  if (s->rows.n == 0 || (!all && nk == 0)) return DG_OK;
  uint64_t n = 0;
  if (half <= 65536) {
    /* a small read: the kernels write the page-locked output directly (it is mapped into
     * the device's address space), so the read's own wait is the only one */
    TRY(dg_read_lww(g->e, &s->rows, all ? NULL : g->d_msg, nk, g->h_rd, g->h_rd + half, half, &n));
  } else {
    TRY(dg_read_lww(g->e, &s->rows, all ? NULL : g->d_msg, nk, g->d_rd, g->d_rd + half, half, &n));
    TRY(dg_copy_async(g->e, g->h_rd, g->d_rd, n * 8));
    TRY(dg_copy_async(g->e, g->h_rd + half, g->d_rd + half, n * 8));
    TRY(dg_engine_sync(g->e));
  }
  *n_out = n;
  return DG_OK;
}

int dgr_take(dgr_state* s, uint64_t version, const uint64_t* keys, uint64_t n_keys, dg_store* out) {
  if (!s || !out || (n_keys && !keys)) return DG_E_INVAL;
  TRY(check_version(s, version));
  dgr_engine* g = s->g;
  TRY(grow_msg(g, n_keys + 1));
  const uint64_t nk = sort_unique(keys, n_keys, g->h_msg);
  TRY(dg_copy_async(g->e, g->d_msg, g->h_msg, nk * 8));
  uint64_t cap = umin(s->rows.n, 4 * nk + 64);
  for (int attempt = 0;; attempt++) {
    TRY(grow_store(g, &g->tk, umax(cap, 1)));
    g->tk.n = 0;
    const int rc = dg_take_keys(g->e, &s->rows, g->d_msg, nk, &g->tk);
    if (rc == DG_E_CAPACITY && attempt == 0) {
      cap = g->tk.n;
      continue;
    }
    TRY(rc);
    break;
  }
  const uint64_t n = g->tk.n, w = even(n);
  TRY(grow_host(g, &g->h_tk, &g->h_tk_cap, rows_words(n) + 2));
  uint64_t* h = g->h_tk;
  dg_store hv = {h, h + w, (int64_t*)(h + 2 * w), (uint32_t*)(h + 4 * w), h + 3 * w, 0, umax(n, 1)};
  TRY(dg_store_download(g->e, &g->tk, &hv));
  *out = hv;
  return DG_OK;
}

int dgr_merkle_build(dgr_state* s, uint64_t version, uint32_t depth) {
  if (!s || depth < 1 || depth > 28) return DG_E_INVAL;
  TRY(check_version(s, version));
  dgr_engine* g = s->g;
  free_tree(s);
  dg_merkle* t = &s->tree;
  t->depth = depth;
  t->terms = &g->th; /* rows hashed through their terms: comparable across BEAM nodes */
  int rc = dg_buffer_alloc(g->e, ((UINT64_C(2) << depth) - 1) * 8, (void**)&t->nodes);
  if (!rc) rc = dg_buffer_alloc(g->e, umax(UINT64_C(1) << depth, 16) * 2, (void**)&t->counts);
  if (!rc) rc = dg_buffer_alloc(g->e, (dg_merkle_chunks(depth) + 1) * 8, (void**)&t->starts);
  if (!rc) rc = dg_merkle_build(g->e, &s->rows, t);
  if (rc) {
    free_tree(s);
    return rc;
  }
  s->has_tree = 1;
  return DG_OK;
}

/* a device continuation -> bytes (u32 level | u64 n | u64 n_buckets | pos | hash | bucket) */
#define CONT_SMALL_OUT 65536 /* entries of an outgoing continuation / keys kept in host memory */

/* a continuation in host memory (the kernel wrote it there) framed as the message */
static int frame_cont(dgr_engine* g, const dg_merkle_cont* co, const uint8_t** bin, uint64_t* len) {
  const uint64_t bytes = 20 + 8 * (2 * co->n + co->n_buckets);
  if (g->bin_cap < bytes) {
    uint8_t* p = (uint8_t*)realloc(g->h_bin, bytes);
    if (!p) return DG_E_NOMEM;
    g->h_bin = p;
    g->bin_cap = bytes;
  }
  memcpy(g->h_bin, &co->level, 4);
  memcpy(g->h_bin + 4, &co->n, 8);
  memcpy(g->h_bin + 12, &co->n_buckets, 8);
  memcpy(g->h_bin + 20, co->pos, 8 * co->n);
  memcpy(g->h_bin + 20 + 8 * co->n, co->hash, 8 * co->n);
  if (co->n_buckets) memcpy(g->h_bin + 20 + 16 * co->n, co->bucket, 8 * co->n_buckets);
  *bin = g->h_bin;
  *len = bytes;
  return DG_OK;
}

static int cont_to_bytes(dgr_engine* g, const dg_merkle_cont* c, const uint8_t** bin, uint64_t* len) {
  const uint64_t words = 2 * c->n + c->n_buckets;
  const uint64_t bytes = 20 + 8 * words;
  /* staged 8-byte aligned in page-locked memory (one wait), then framed */
  TRY(grow_host(g, &g->h_cstage, &g->h_cstage_cap, umax(words, 1)));
  TRY(dg_copy_async(g->e, g->h_cstage, c->pos, c->n * 8));
  TRY(dg_copy_async(g->e, g->h_cstage + c->n, c->hash, c->n * 8));
  TRY(dg_copy_async(g->e, g->h_cstage + 2 * c->n, c->bucket, c->n_buckets * 8));
  TRY(dg_engine_sync(g->e));
  if (g->bin_cap < bytes) {
    uint8_t* p = (uint8_t*)realloc(g->h_bin, bytes);
    if (!p) return DG_E_NOMEM;
    g->h_bin = p;
    g->bin_cap = bytes;
  }
  memcpy(g->h_bin, &c->level, 4);
  memcpy(g->h_bin + 4, &c->n, 8);
  memcpy(g->h_bin + 12, &c->n_buckets, 8);
  memcpy(g->h_bin + 20, g->h_cstage, 8 * words);
  *bin = g->h_bin;
  *len = bytes;
  return DG_OK;
}

int dgr_merkle_prepare(dgr_state* s, uint64_t version, uint32_t levels, const uint8_t** bin, uint64_t* len) {
  if (!s || !bin || !len || !s->has_tree) return DG_E_INVAL;
  TRY(check_version(s, version));
  dgr_engine* g = s->g;
  const uint32_t L = levels < s->tree.depth ? levels : s->tree.depth;
  const uint64_t n = UINT64_C(1) << L;
  if (n <= CONT_SMALL_OUT) { /* written by the kernel into page-locked memory: framed here */
    TRY(grow_host(g, &g->h_cstage, &g->h_cstage_cap, 2 * n));
    dg_merkle_cont co;
    memset(&co, 0, sizeof co);
    co.pos = g->h_cstage;
    co.hash = g->h_cstage + n;
    co.cap = n;
    TRY(dg_merkle_prepare(g->e, &s->tree, levels, &co));
    return frame_cont(g, &co, bin, len);
  }
  TRY(grow_cont(g, &g->co, n, 1));
  g->co.n = g->co.n_buckets = 0;
  TRY(dg_merkle_prepare(g->e, &s->tree, levels, &g->co));
  return cont_to_bytes(g, &g->co, bin, len);
}

/* One hop through dg_merkle_continue_home: the incoming continuation read where it was
 * unpacked (mapped memory), the next one (truncated to max_sync) or the keys written by
 * the kernel into page-locked memory, one launch and one wait.  *done = 0: over its
 * limits (nothing happened; the general path runs). */
static int continue_small(dgr_state* s, uint32_t level, uint64_t n, uint64_t nb, uint32_t levels,
                          uint64_t max_sync, int* status, const uint8_t** out_bin, uint64_t* out_len,
                          const uint64_t** keys, uint64_t* n_keys, int* done) {
  dgr_engine* g = s->g;
  *done = 0;
  static int general = -1; /* DGR_CONT_GENERAL=1: always the general calls (A/B) */
  if (general < 0) general = getenv("DGR_CONT_GENERAL") != NULL;
  const uint32_t depth = s->tree.depth;
  if (general || n > DG_CONT_HOME_ENTRIES || nb > DG_CONT_HOME_BUCKETS || level > depth + 1) return DG_OK;
  dg_merkle_cont ci;
  memset(&ci, 0, sizeof ci);
  ci.level = level;
  ci.pos = g->h_msg;
  ci.hash = g->h_msg + n;
  ci.bucket = g->h_msg + 2 * n;
  ci.n = ci.cap = n;
  ci.n_buckets = ci.cap_buckets = nb;
  uint64_t C, CB = umax(umin(n, max_sync), 1);
  if (level < depth) {
    const uint32_t k = levels < depth - level ? levels : depth - level;
    C = umin(n << k, max_sync);
  } else {
    C = umax(4 * umin(n, max_sync), 64);
  }
  C = umax(C, 1);
  const uint64_t kcap = umax(umin(umin(max_sync, s->rows.n + n + 1), CONT_SMALL_OUT), 1);
  TRY(grow_host(g, &g->h_ckeys, &g->h_ckeys_cap, kcap));
  uint64_t nk = 0, ntot = 0;
  dg_merkle_cont co;
  for (int attempt = 0;; attempt++) {
    if (C > CONT_SMALL_OUT) return DG_OK;
    TRY(grow_host(g, &g->h_cstage, &g->h_cstage_cap, 2 * C + CB));
    memset(&co, 0, sizeof co);
    co.pos = g->h_cstage;
    co.hash = g->h_cstage + C;
    co.bucket = g->h_cstage + 2 * C;
    co.cap = C;
    co.cap_buckets = CB;
    const int rc = dg_merkle_continue_home(g->e, &s->tree, &s->rows, &ci, levels, max_sync, &co, g->h_ckeys,
                                           kcap, &nk, &ntot, status);
    if (rc == DG_E_CAPACITY && attempt == 0) {
      C = umax(co.n, C);
      CB = umax(co.n_buckets, CB);
      continue;
    }
    TRY(rc);
    break;
  }
  if (*status == DG_CONT_DECLINED) return DG_OK;
  if (*status == 0) {
    if (ntot > nk && nk < max_sync) return DG_OK; /* more keys than kept here: the general path */
    *keys = g->h_ckeys;
    *n_keys = nk;
    *done = 1;
    return DG_OK;
  }
  TRY(frame_cont(g, &co, out_bin, out_len));
  *done = 1;
  return DG_OK;
}

int dgr_merkle_continue(dgr_state* s, uint64_t version, const uint8_t* bin, uint64_t len, uint32_t levels,
                        uint64_t max_sync, int* status, const uint8_t** out_bin, uint64_t* out_len,
                        const uint64_t** keys, uint64_t* n_keys) {
  if (!s || !bin || !status || !out_bin || !out_len || !keys || !n_keys || !s->has_tree || len < 20)
    return DG_E_INVAL;
  TRY(check_version(s, version));
  dgr_engine* g = s->g;
  uint32_t level;
  uint64_t n, nb;
  memcpy(&level, bin, 4);
  memcpy(&n, bin + 4, 8);
  memcpy(&nb, bin + 12, 8);
  if (n > (len - 20) / 16 || len != 20 + 16 * n + 8 * nb) return DG_E_INVAL;
  *status = 0;
  *n_keys = 0;
  *out_bin = NULL;
  *out_len = 0;
  /* the incoming continuation as ONE copy: pos | hash | bucket in the message buffer */
  TRY(grow_msg(g, 2 * n + nb + 1));
  if (2 * n + nb) memcpy(g->h_msg, bin + 20, (2 * n + nb) * 8);
  int done = 0;
  TRY(continue_small(s, level, n, nb, levels, max_sync, status, out_bin, out_len, keys, n_keys, &done));
  if (done) return DG_OK;
  *status = 0;
  TRY(dg_copy_async(g->e, g->d_msg, g->h_msg, (2 * n + nb) * 8));
  dg_merkle_cont ci;
  memset(&ci, 0, sizeof ci);
  ci.level = level;
  ci.pos = g->d_msg;
  ci.hash = g->d_msg + n;
  ci.bucket = g->d_msg + 2 * n;
  ci.n = ci.cap = n;
  ci.n_buckets = ci.cap_buckets = nb;
  /* keys: max_sync of them (UINT64_MAX, :infinite -- at most every key of both sides) */
  const uint64_t cap_keys = umax(umin(max_sync, s->rows.n + n + 1), 1);
  TRY(grow_dev(g, &g->d_ckeys, &g->ckeys_cap, cap_keys));
  uint64_t cap = 4 * umax(n, 1), cap_b = umax(n, 1), nk = 0, ntot = 0;
  int rc = DG_OK;
  for (int attempt = 0; attempt < 3; attempt++) {
    TRY(grow_cont(g, &g->co, cap, cap_b));
    g->co.n = g->co.n_buckets = 0;
    rc = dg_merkle_continue(g->e, &s->tree, &s->rows, &ci, levels, &g->co, g->d_ckeys, cap_keys, &nk, &ntot,
                            status);
    if (rc != DG_E_CAPACITY) break;
    cap = umax(g->co.n, cap);
    cap_b = umax(g->co.n_buckets, cap_b);
  }
  TRY(rc);
  if (*status == 1) {
    if (max_sync != UINT64_MAX) TRY(dg_merkle_truncate(g->e, &s->tree, &g->co, max_sync)); /* :98 */
    return cont_to_bytes(g, &g->co, out_bin, out_len);
  }
  /* {:ok, keys}: the first max_sync_size differing keys (Enum.take, :105) */
  TRY(grow_host(g, &g->h_ckeys, &g->h_ckeys_cap, umax(nk, 1)));
  TRY(dg_copy_async(g->e, g->h_ckeys, g->d_ckeys, nk * 8));
  TRY(dg_engine_sync(g->e));
  *keys = g->h_ckeys;
  *n_keys = nk;
  return DG_OK;
}
