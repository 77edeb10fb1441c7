/*
 * deltaref.c — C restatement of DeltaCrdt.AWLWWMap over SoA dot rows: the CPU ORACLE.
 *
 * TEST INFRASTRUCTURE ONLY.  Built into oracle/_build/libdeltaref.so by
 * oracle/Makefile.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg load it, and only as the checker / the timed CPU baseline
 * ("port").  The product (libdeltagpu) never links or calls it.
 *
 * It follows lib/delta_crdt/aw_lww_map.ex structurally (not the GPU's merge-path
 * formulation): an outer loop over keys (join_or_maps/4, :161-193), an inner loop
 * over {value, ts} entries (the nested join_or_maps), and per entry the dot-set
 * join s1∩s2 ∪ s1\c2 ∪ s2\c1 (join_dot_sets/4, :196-209) with Dots.member?/2
 * (:67-73).  It uses the public structs of include/deltagpu.h with HOST pointers.
 *
 * Pinning: tests/test_c_oracle.py checks it against the term-level restatement
 * (oracle/awlww_term.py), which tests/test_oracle_reference_tests.py pins to the
 * reference's own unit tests and properties; tests/golden/ holds fixtures of both.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/deltagpu.h"

#define REF_E(code) return (code)

/* ------------------------------------------------------------------ helpers */

static int row_cmp(const dg_store* s, uint64_t i, const dg_store* t, uint64_t j) {
  if (s->key[i] != t->key[j]) return s->key[i] < t->key[j] ? -1 : 1;
  if (s->val[i] != t->val[j]) return s->val[i] < t->val[j] ? -1 : 1;
  if (s->ts[i] != t->ts[j]) return s->ts[i] < t->ts[j] ? -1 : 1;
  if (s->node[i] != t->node[j]) return s->node[i] < t->node[j] ? -1 : 1;
  if (s->cnt[i] != t->cnt[j]) return s->cnt[i] < t->cnt[j] ? -1 : 1;
  return 0;
}

static int entry_cmp(const dg_store* s, uint64_t i, const dg_store* t, uint64_t j) {
  if (s->val[i] != t->val[j]) return s->val[i] < t->val[j] ? -1 : 1;
  if (s->ts[i] != t->ts[j]) return s->ts[i] < t->ts[j] ? -1 : 1;
  return 0;
}

static int dot_cmp(uint32_t n1, uint64_t c1, uint32_t n2, uint64_t c2) {
  if (n1 != n2) return n1 < n2 ? -1 : 1;
  if (c1 != c2) return c1 < c2 ? -1 : 1;
  return 0;
}

/* Dots.member?/2 (aw_lww_map.ex:67-73):
 *   MapSet: MapSet.member?(dots, dot)        VV: Map.get(dots, i, 0) >= x */
static int ctx_member(const dg_context* c, uint32_t node, uint64_t cnt) {
  uint64_t lo = 0, hi = c->n;
  while (lo < hi) {
    uint64_t mid = (lo + hi) / 2;
    int cmp = c->kind == DG_CTX_VV ? (c->node[mid] < node ? -1 : (c->node[mid] > node ? 1 : 0))
                                   : dot_cmp(c->node[mid], c->cnt[mid], node, cnt);
    if (cmp < 0)
      lo = mid + 1;
    else
      hi = mid;
  }
  if (c->kind == DG_CTX_VV) {
    uint64_t have = (lo < c->n && c->node[lo] == node) ? c->cnt[lo] : 0;
    return have >= cnt;
  }
  return lo < c->n && c->node[lo] == node && c->cnt[lo] == cnt;
}

static int keyset_member(const uint64_t* keys, uint64_t n, uint64_t k) {
  uint64_t lo = 0, hi = n;
  while (lo < hi) {
    uint64_t mid = (lo + hi) / 2;
    if (keys[mid] < k)
      lo = mid + 1;
    else
      hi = mid;
  }
  return lo < n && keys[lo] == k;
}

static void emit(dg_store* out, const dg_store* s, uint64_t i) {
  uint64_t o = out->n++;
  out->key[o] = s->key[i];
  out->val[o] = s->val[i];
  out->ts[o] = s->ts[i];
  out->node[o] = s->node[i];
  out->cnt[o] = s->cnt[i];
}

/* ------------------------------------------------------ Dots.union / compress */

/* Dots.union/2 (aw_lww_map.ex:39-52). */
int ref_context_union(const dg_context* a, const dg_context* b, dg_context* out) {
  if (out->cap < a->n + b->n) REF_E(DG_E_CAPACITY);
  if (a->kind == DG_CTX_DOTS && b->kind == DG_CTX_DOTS) {
    /* MapSet.union */
    uint64_t i = 0, j = 0, o = 0;
    while (i < a->n || j < b->n) {
      int c = i >= a->n ? 1 : j >= b->n ? -1 : dot_cmp(a->node[i], a->cnt[i], b->node[j], b->cnt[j]);
      if (c <= 0) {
        out->node[o] = a->node[i];
        out->cnt[o++] = a->cnt[i];
        i++;
        if (c == 0) j++;
      } else {
        out->node[o] = b->node[j];
        out->cnt[o++] = b->cnt[j];
        j++;
      }
    }
    out->kind = DG_CTX_DOTS;
    out->n = o;
    return DG_OK;
  }
  /* union(set, map) = union(map, set); then Enum.reduce(dots2, dots1, Map.update max).
   * A dot set is sorted by (node, cnt), so each node's run ends with its max. */
  const dg_context* m = a->kind == DG_CTX_VV ? a : b;
  const dg_context* o2 = a->kind == DG_CTX_VV ? b : a;
  uint64_t i = 0, j = 0, o = 0;
  while (i < m->n || j < o2->n) {
    uint32_t node;
    uint64_t best = 0;
    int have = 0;
    if (j >= o2->n || (i < m->n && m->node[i] <= o2->node[j]))
      node = m->node[i];
    else
      node = o2->node[j];
    while (i < m->n && m->node[i] == node) {
      if (!have || m->cnt[i] > best) best = m->cnt[i];
      have = 1;
      i++;
    }
    while (j < o2->n && o2->node[j] == node) {
      if (!have || o2->cnt[j] > best) best = o2->cnt[j];
      have = 1;
      j++;
    }
    out->node[o] = node;
    out->cnt[o++] = best;
  }
  out->kind = DG_CTX_VV;
  out->n = o;
  return DG_OK;
}

/* Dots.compress/1 (aw_lww_map.ex:13-20) as used by compress_dots/1 (:115-117). */
int ref_compress_dots(const dg_context* dots, dg_context* out) {
  if (dots->kind != DG_CTX_DOTS) REF_E(DG_E_CLAUSE);
  if (out->cap < dots->n) REF_E(DG_E_CAPACITY);
  uint64_t o = 0;
  for (uint64_t i = 0; i < dots->n; i++) {
    if (o > 0 && out->node[o - 1] == dots->node[i]) {
      if (dots->cnt[i] > out->cnt[o - 1]) out->cnt[o - 1] = dots->cnt[i];
    } else {
      out->node[o] = dots->node[i];
      out->cnt[o++] = dots->cnt[i];
    }
  }
  out->kind = DG_CTX_VV;
  out->n = o;
  return DG_OK;
}

/* ------------------------------------------------------------------- join/3 */

/* join_dot_sets/4 (aw_lww_map.ex:196-209) for one {v, ts} entry: a[p:pe) are s1,
 * b[q:qe) are s2 (both sorted by dot).  Emits s1∩s2 ∪ s1\c2 ∪ s2\c1 in dot order. */
static void join_dot_sets(const dg_store* a, uint64_t p, uint64_t pe, const dg_context* c1,
                          const dg_store* b, uint64_t q, uint64_t qe, const dg_context* c2,
                          dg_store* out) {
  while (p < pe || q < qe) {
    int c = p >= pe ? 1
          : q >= qe ? -1
                    : dot_cmp(a->node[p], a->cnt[p], b->node[q], b->cnt[q]);
    if (c == 0) { /* MapSet.intersection(s1, s2) */
      emit(out, a, p);
      p++;
      q++;
    } else if (c < 0) { /* Dots.difference(s1, c2) */
      if (!ctx_member(c2, a->node[p], a->cnt[p])) emit(out, a, p);
      p++;
    } else { /* Dots.difference(s2, c1) */
      if (!ctx_member(c1, b->node[q], b->cnt[q])) emit(out, b, q);
      q++;
    }
  }
}

/* join_or_maps/4 over the rows (aw_lww_map.ex:161-193); out->n = rows written. */
int ref_join2_rows(const dg_store* a, const dg_context* ca, const dg_store* b,
                   const dg_context* cb, const uint64_t* keys, uint64_t n_keys, dg_store* out) {
  if (out->cap < a->n + b->n) REF_E(DG_E_CAPACITY);
  out->n = 0;
  uint64_t i = 0, j = 0;
  while (i < a->n || j < b->n) {
    uint64_t key;
    if (j >= b->n || (i < a->n && a->key[i] <= b->key[j]))
      key = a->key[i];
    else
      key = b->key[j];
    uint64_t ie = i, je = j;
    while (ie < a->n && a->key[ie] == key) ie++;
    while (je < b->n && b->key[je] == key) je++;
    int joined = keys == NULL || keyset_member(keys, n_keys, key);
    if (!joined) {
      /* Map.merge(Map.drop(d1.value, keys), Map.drop(d2.value, keys)) :185-188 */
      if (je > j)
        for (uint64_t q = j; q < je; q++) emit(out, b, q);
      else
        for (uint64_t p = i; p < ie; p++) emit(out, a, p);
    } else {
      /* nested join_or_maps over the union of the key's {v, ts} entries (:167-173) */
      uint64_t p = i, q = j;
      while (p < ie || q < je) {
        int c = p >= ie ? 1 : q >= je ? -1 : entry_cmp(a, p, b, q);
        uint64_t pe = p, qe = q;
        if (c <= 0)
          while (pe < ie && entry_cmp(a, pe, a, p) == 0) pe++;
        if (c >= 0)
          while (qe < je && entry_cmp(b, qe, b, q) == 0) qe++;
        /* Map.get(delta.value, entry, %{}) — a side without the entry joins as ∅ */
        join_dot_sets(a, p, pe, ca, b, q, qe, cb, out);
        p = pe;
        q = qe;
      }
      /* keys/entries whose joined set is empty emitted no rows (:177-181) */
    }
    i = ie;
    j = je;
  }
  return DG_OK;
}

/* join/3 (aw_lww_map.ex:153-158) = Dots.union of contexts + join_or_maps/4. */
int ref_join2(const dg_store* a, const dg_context* ca, const dg_store* b, const dg_context* cb,
              const uint64_t* keys, uint64_t n_keys, dg_store* out, dg_context* out_ctx) {
  if (out->cap < a->n + b->n) REF_E(DG_E_CAPACITY);
  if (out_ctx->cap < ca->n + cb->n) REF_E(DG_E_CAPACITY);
  int rc = ref_join2_rows(a, ca, b, cb, keys, n_keys, out);
  if (rc != DG_OK) return rc;
  return ref_context_union(ca, cb, out_ctx);
}

/* The k-way join as CausalCrdt performs it: a left fold of join/3 over all keys. */
int ref_joink(int k, const dg_store* stores, const dg_context* ctxs, dg_store* out,
              dg_context* out_ctx) {
  if (k <= 0) REF_E(DG_E_INVAL);
  uint64_t total = 0, total_ctx = 0;
  for (int s = 0; s < k; s++) {
    total += stores[s].n;
    total_ctx += ctxs[s].n;
  }
  if (out->cap < total || out_ctx->cap < total_ctx) REF_E(DG_E_CAPACITY);
  dg_store acc[2];
  dg_context acc_ctx[2];
  for (int t = 0; t < 2; t++) {
    acc[t].key = malloc(total * 8 + 8);
    acc[t].val = malloc(total * 8 + 8);
    acc[t].ts = malloc(total * 8 + 8);
    acc[t].node = malloc(total * 4 + 4);
    acc[t].cnt = malloc(total * 8 + 8);
    acc[t].cap = total;
    acc[t].n = 0;
    acc_ctx[t].node = malloc(total_ctx * 4 + 4);
    acc_ctx[t].cnt = malloc(total_ctx * 8 + 8);
    acc_ctx[t].cap = total_ctx;
    acc_ctx[t].n = 0;
  }
  /* acc0 = stores[0] */
  memcpy(acc[0].key, stores[0].key, stores[0].n * 8);
  memcpy(acc[0].val, stores[0].val, stores[0].n * 8);
  memcpy(acc[0].ts, stores[0].ts, stores[0].n * 8);
  memcpy(acc[0].node, stores[0].node, stores[0].n * 4);
  memcpy(acc[0].cnt, stores[0].cnt, stores[0].n * 8);
  acc[0].n = stores[0].n;
  memcpy(acc_ctx[0].node, ctxs[0].node, ctxs[0].n * 4);
  memcpy(acc_ctx[0].cnt, ctxs[0].cnt, ctxs[0].n * 8);
  acc_ctx[0].n = ctxs[0].n;
  acc_ctx[0].kind = ctxs[0].kind;
  int cur = 0, rc = DG_OK;
  for (int s = 1; s < k && rc == DG_OK; s++) {
    rc = ref_join2(&acc[cur], &acc_ctx[cur], &stores[s], &ctxs[s], NULL, 0, &acc[1 - cur],
                   &acc_ctx[1 - cur]);
    cur = 1 - cur;
  }
  if (rc == DG_OK) {
    memcpy(out->key, acc[cur].key, acc[cur].n * 8);
    memcpy(out->val, acc[cur].val, acc[cur].n * 8);
    memcpy(out->ts, acc[cur].ts, acc[cur].n * 8);
    memcpy(out->node, acc[cur].node, acc[cur].n * 4);
    memcpy(out->cnt, acc[cur].cnt, acc[cur].n * 8);
    out->n = acc[cur].n;
    memcpy(out_ctx->node, acc_ctx[cur].node, acc_ctx[cur].n * 4);
    memcpy(out_ctx->cnt, acc_ctx[cur].cnt, acc_ctx[cur].n * 8);
    out_ctx->n = acc_ctx[cur].n;
    out_ctx->kind = acc_ctx[cur].kind;
  }
  for (int t = 0; t < 2; t++) {
    free(acc[t].key);
    free(acc[t].val);
    free(acc[t].ts);
    free(acc[t].node);
    free(acc[t].cnt);
    free(acc_ctx[t].node);
    free(acc_ctx[t].cnt);
  }
  return rc;
}

/* ------------------------------------------------------------------- read/1,2 */

/* read/1 (aw_lww_map.ex:211-216): per key Enum.max_by(entries, ts) — the first
 * maximum in flatmap (= {v, ts} term) order wins; read/2 (:218-220) = Map.take. */
int ref_read_lww(const dg_store* s, const uint64_t* keys, uint64_t n_keys, uint64_t* out_key,
                 uint64_t* out_val, uint64_t cap, uint64_t* n_out) {
  uint64_t o = 0;
  uint64_t i = 0;
  while (i < s->n) {
    uint64_t key = s->key[i];
    uint64_t best_val = s->val[i];
    int64_t best_ts = s->ts[i];
    uint64_t e = i + 1;
    while (e < s->n && s->key[e] == key) {
      if (s->ts[e] > best_ts) {
        best_ts = s->ts[e];
        best_val = s->val[e];
      }
      e++;
    }
    if (keys == NULL || keyset_member(keys, n_keys, key)) {
      if (o >= cap) REF_E(DG_E_CAPACITY);
      out_key[o] = key;
      out_val[o] = best_val;
      o++;
    }
    i = e;
  }
  *n_out = o;
  return DG_OK;
}

/* ------------------------------------------------------------------- Merkle */

static inline uint64_t mix64(uint64_t x) {
  x ^= x >> 30;
  x *= 0xbf58476d1ce4e5b9ULL;
  x ^= x >> 27;
  x *= 0x94d049bb133111ebULL;
  x ^= x >> 31;
  return x;
}

uint64_t ref_row_hash(uint64_t key, uint64_t val, int64_t ts, uint64_t node, uint64_t cnt) {
  uint64_t h = mix64(key ^ 0x9E3779B97F4A7C15ULL);
  h = mix64(h ^ val);
  h = mix64(h ^ (uint64_t)ts);
  h = mix64(h ^ node);
  return mix64(h ^ cnt);
}

/* The term in a row hash of a value id / node id (include/deltagpu.h dg_term_hashes; the
 * arrays here are HOST arrays): th == NULL, a canonical integer value id [2^58, 2^63) and
 * ids absent from the tables stand for themselves. */
uint64_t ref_term_val(const dg_term_hashes* th, uint64_t v) {
  if (!th || !th->val_id || !th->val_hash || (v >= (1ULL << 58) && v < (1ULL << 63))) return v;
  uint64_t lo = 0, hi = th->n_vals;
  while (lo < hi) {
    uint64_t mid = (lo + hi) / 2;
    if (th->val_id[mid] < v) lo = mid + 1; else hi = mid;
  }
  return (lo < th->n_vals && th->val_id[lo] == v) ? th->val_hash[lo] : v;
}

uint64_t ref_term_node(const dg_term_hashes* th, uint32_t n) {
  return (th && th->node_hash && n < th->n_nodes) ? th->node_hash[n] : (uint64_t)n;
}

uint64_t ref_node_hash(uint64_t left, uint64_t right) {
  return mix64(left ^ mix64(right ^ 0xD6E8FEB86659FD93ULL));
}

/* The MerkleMap role (csrc/merkle.hip, include/deltagpu.h dg_merkle): the tree over the
 * keys whose top `sb` bits equal `shard`, 2^depth buckets by the next depth bits;
 * bucket = Σ row hashes of its rows (a key's leaf = Σ over its rows, the raw per-key
 * value map, causal_crdt.ex:392), parents = ref_node_hash(children).  `nodes` holds
 * 2^(depth+1) - 1 entries in level order, `counts` (may be NULL) each bucket's rows.
 * th: term hashes (host arrays) or NULL.  DG_E_INVAL for a key outside the shard,
 * DG_E_CAPACITY for a bucket over 65535 rows. */
int ref_merkle_build(const dg_store* s, uint32_t depth, uint32_t sb, uint64_t shard,
                     const dg_term_hashes* th, uint64_t* nodes, uint16_t* counts, uint64_t* n_keys) {
  if (depth < 1 || depth > 28 || sb > 16 || depth + sb > 44) REF_E(DG_E_INVAL);
  uint64_t nb = 1ULL << depth;
  uint64_t base = nb - 1;
  memset(nodes, 0, (2 * nb - 1) * 8);
  uint32_t* c32 = (uint32_t*)calloc(nb, sizeof *c32);
  if (!c32) REF_E(DG_E_NOMEM);
  uint64_t keys = 0;
  for (uint64_t i = 0; i < s->n; i++) {
    uint64_t key = s->key[i];
    if (sb && (key >> (64 - sb)) != shard) {
      free(c32);
      REF_E(DG_E_INVAL);
    }
    if (i == 0 || s->key[i - 1] != key) keys++;
    const uint64_t b = (key << sb) >> (64 - depth);
    nodes[base + b] += ref_row_hash(key, ref_term_val(th, s->val[i]), s->ts[i],
                                    ref_term_node(th, s->node[i]), s->cnt[i]);
    c32[b]++;
  }
  for (uint64_t b = 0; b < nb; b++) {
    if (c32[b] > 0xFFFF) {
      free(c32);
      REF_E(DG_E_CAPACITY);
    }
    if (counts) counts[b] = (uint16_t)c32[b];
  }
  free(c32);
  for (int l = (int)depth - 1; l >= 0; l--) {
    uint64_t first = (1ULL << l) - 1;
    for (uint64_t x = 0; x < (1ULL << l); x++) {
      uint64_t idx = first + x;
      nodes[idx] = ref_node_hash(nodes[2 * idx + 1], nodes[2 * idx + 2]);
    }
  }
  if (n_keys) *n_keys = keys;
  return DG_OK;
}

/* Exact semantic diff (no hashing): keys whose row sets differ. */
int ref_store_diff(const dg_store* a, const dg_store* b, uint64_t* out, uint64_t cap,
                   uint64_t* n_out) {
  uint64_t i = 0, j = 0, o = 0;
  while (i < a->n || j < b->n) {
    uint64_t key;
    if (j >= b->n || (i < a->n && a->key[i] <= b->key[j]))
      key = a->key[i];
    else
      key = b->key[j];
    uint64_t ie = i, je = j;
    while (ie < a->n && a->key[ie] == key) ie++;
    while (je < b->n && b->key[je] == key) je++;
    int differ = (ie - i) != (je - j);
    for (uint64_t x = 0; !differ && x < ie - i; x++) differ = row_cmp(a, i + x, b, j + x) != 0;
    if (differ) {
      if (o >= cap) REF_E(DG_E_CAPACITY);
      out[o++] = key;
    }
    i = ie;
    j = je;
  }
  *n_out = o;
  return DG_OK;
}

/* Sorted+unique precondition of a store. */
int ref_store_check(const dg_store* s) {
  for (uint64_t i = 1; i < s->n; i++)
    if (row_cmp(s, i - 1, s, i) >= 0) REF_E(DG_E_ORDER);
  return DG_OK;
}
