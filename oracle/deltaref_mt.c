/* deltaref_mt.c — the C restatement's join/3 on all host cores.  TEST / BASELINE
 * INFRASTRUCTURE ONLY: bench.py's cpu_baseline times it beside the single-thread
 * restatement ("at all host cores (OpenMP over key shards)").
 *
 * join/3 is per key (aw_lww_map.ex:161-193), so the two stores are cut into P shards at
 * key boundaries (every row of a key falls in one shard), each shard is joined by
 * ref_join2_rows (deltaref.c) into its own region of `scratch`, and the shard outputs
 * are copied contiguously into `out`.  The context union (:155) is computed once. */
#include <omp.h>
#include <string.h>

#include "../include/deltagpu.h"

int ref_join2_rows(const dg_store* a, const dg_context* ca, const dg_store* b,
                   const dg_context* cb, const uint64_t* keys, uint64_t n_keys, dg_store* out);
int ref_context_union(const dg_context* a, const dg_context* b, dg_context* out);

#define MAX_SHARDS 1024

static uint64_t lower_key(const uint64_t* k, uint64_t n, uint64_t x) {
  uint64_t lo = 0, hi = n;
  while (lo < hi) {
    uint64_t mid = (lo + hi) >> 1;
    if (k[mid] < x)
      lo = mid + 1;
    else
      hi = mid;
  }
  return lo;
}

static dg_store slice(const dg_store* s, uint64_t lo, uint64_t hi) {
  dg_store r = *s;
  r.key = s->key + lo;
  r.val = s->val + lo;
  r.ts = s->ts + lo;
  r.node = s->node + lo;
  r.cnt = s->cnt + lo;
  r.n = hi - lo;
  r.cap = hi - lo;
  return r;
}

/* scratch: a store with cap >= a->n + b->n (reused across calls by the caller). */
int ref_join2_mt(const dg_store* a, const dg_context* ca, const dg_store* b,
                 const dg_context* cb, const uint64_t* keys, uint64_t n_keys, dg_store* out,
                 dg_context* out_ctx, dg_store* scratch, int threads) {
  if (out->cap < a->n + b->n || scratch->cap < a->n + b->n) return DG_E_CAPACITY;
  if (out_ctx->cap < ca->n + cb->n) return DG_E_CAPACITY;
  if (threads < 1) threads = omp_get_max_threads();
  int P = threads * 4;
  if (P > MAX_SHARDS) P = MAX_SHARDS;
  const dg_store* big = a->n >= b->n ? a : b;
  uint64_t alo[MAX_SHARDS + 1], blo[MAX_SHARDS + 1], cnt[MAX_SHARDS], off[MAX_SHARDS + 1];
  alo[0] = blo[0] = 0;
  for (int p = 1; p < P; p++) {
    const uint64_t x = big->n ? big->key[(uint64_t)p * big->n / P] : 0;
    alo[p] = lower_key(a->key, a->n, x);
    blo[p] = lower_key(b->key, b->n, x);
    if (alo[p] < alo[p - 1]) alo[p] = alo[p - 1];
    if (blo[p] < blo[p - 1]) blo[p] = blo[p - 1];
  }
  alo[P] = a->n;
  blo[P] = b->n;
  int rc = DG_OK;
#pragma omp parallel for num_threads(threads) schedule(dynamic, 1)
  for (int p = 0; p < P; p++) {
    dg_store sa = slice(a, alo[p], alo[p + 1]), sb = slice(b, blo[p], blo[p + 1]);
    dg_store so = slice(scratch, alo[p] + blo[p], alo[p + 1] + blo[p + 1]);
    so.n = 0;
    int r = ref_join2_rows(&sa, ca, &sb, cb, keys, n_keys, &so);
    cnt[p] = so.n;
    if (r != DG_OK) {
#pragma omp atomic write
      rc = r;
    }
  }
  if (rc != DG_OK) return rc;
  off[0] = 0;
  for (int p = 0; p < P; p++) off[p + 1] = off[p] + cnt[p];
#pragma omp parallel for num_threads(threads) schedule(static)
  for (int p = 0; p < P; p++) {
    const uint64_t s = alo[p] + blo[p], d = off[p], n = cnt[p];
    memcpy(out->key + d, scratch->key + s, n * 8);
    memcpy(out->val + d, scratch->val + s, n * 8);
    memcpy(out->ts + d, scratch->ts + s, n * 8);
    memcpy(out->node + d, scratch->node + s, n * 4);
    memcpy(out->cnt + d, scratch->cnt + s, n * 8);
  }
  out->n = off[P];
  return ref_context_union(ca, cb, out_ctx);
}
