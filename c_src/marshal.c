/* marshal.c — see marshal.h.  Plain C99; no Erlang or HIP headers. */
#include "marshal.h"

#include <stdlib.h>
#include <string.h>

#define ID_STRIDE (1ull << 32) /* id step past either end of a region's values */

/* ------------------------------------------------------------ a u64 -> slot map */
typedef struct {
  uint64_t* h;   /* hash (0 = empty slot; stored hashes are forced nonzero) */
  uint32_t* v;   /* payload index */
  uint64_t cap;  /* power of two */
  uint64_t n;
} hmap;

static uint64_t nz(uint64_t h) { return h ? h : 0x9E3779B97F4A7C15ull; }

static int hmap_grow(hmap* m) {
  uint64_t cap = m->cap ? m->cap * 2 : 64;
  uint64_t* h = (uint64_t*)calloc(cap, sizeof *h);
  uint32_t* v = (uint32_t*)calloc(cap, sizeof *v);
  if (!h || !v) {
    free(h);
    free(v);
    return DG_E_NOMEM;
  }
  for (uint64_t i = 0; i < m->cap; i++)
    if (m->h[i]) {
      uint64_t j = m->h[i] & (cap - 1);
      while (h[j]) j = (j + 1) & (cap - 1);
      h[j] = m->h[i];
      v[j] = m->v[i];
    }
  free(m->h);
  free(m->v);
  m->h = h;
  m->v = v;
  m->cap = cap;
  return DG_OK;
}

/* visit the slots of hash h: *slot = first slot with this hash at or after *slot */
static int hmap_next(const hmap* m, uint64_t h, uint64_t* slot) {
  if (!m->cap) return 0;
  for (uint64_t j = *slot;; j = (j + 1) & (m->cap - 1)) {
    if (!m->h[j]) return 0;
    if (m->h[j] == h) {
      *slot = j;
      return 1;
    }
  }
}

static int hmap_put(hmap* m, uint64_t h, uint32_t v) {
  if ((m->n + 1) * 2 > m->cap) {
    int rc = hmap_grow(m);
    if (rc) return rc;
  }
  uint64_t j = h & (m->cap - 1);
  while (m->h[j]) j = (j + 1) & (m->cap - 1);
  m->h[j] = h;
  m->v[j] = v;
  m->n++;
  return DG_OK;
}

/* ------------------------------------------------------------ canonical encoding */
void dgm_buf_free(dgm_buf* b) {
  free(b->p);
  memset(b, 0, sizeof *b);
}

static int buf_put(dgm_buf* b, const void* p, size_t n) {
  if (b->n + n > b->cap) {
    size_t c = b->cap ? b->cap : 64;
    while (c < b->n + n) c *= 2;
    unsigned char* q = (unsigned char*)realloc(b->p, c);
    if (!q) return DG_E_NOMEM;
    b->p = q;
    b->cap = c;
  }
  if (n) memcpy(b->p + b->n, p, n);
  b->n += n;
  return DG_OK;
}

static int buf_head(dgm_buf* b, char tag, uint32_t len) {
  unsigned char h[5] = {(unsigned char)tag, (unsigned char)len, (unsigned char)(len >> 8),
                        (unsigned char)(len >> 16), (unsigned char)(len >> 24)};
  return buf_put(b, h, 5);
}

int dgm_enc_atom(dgm_buf* b, const char* utf8, size_t n) {
  int rc = buf_head(b, 'a', (uint32_t)n);
  return rc ? rc : buf_put(b, utf8, n);
}

int dgm_enc_int(dgm_buf* b, int negative, const unsigned char* mag_le, size_t n) {
  while (n && mag_le[n - 1] == 0) n--; /* minimal magnitude (zero: none) */
  const unsigned char sign = (negative && n) ? 1 : 0;
  int rc = buf_head(b, 'i', (uint32_t)(n + 1));
  if (!rc) rc = buf_put(b, &sign, 1);
  return rc ? rc : buf_put(b, mag_le, n);
}

int dgm_enc_u64(dgm_buf* b, uint64_t v) {
  unsigned char m[8];
  for (int i = 0; i < 8; i++) m[i] = (unsigned char)(v >> (8 * i));
  return dgm_enc_int(b, 0, m, 8);
}

int dgm_enc_i64(dgm_buf* b, int64_t v) {
  const uint64_t mag = v < 0 ? (uint64_t)0 - (uint64_t)v : (uint64_t)v;
  unsigned char m[8];
  for (int i = 0; i < 8; i++) m[i] = (unsigned char)(mag >> (8 * i));
  return dgm_enc_int(b, v < 0, m, 8);
}

int dgm_enc_float(dgm_buf* b, double v) {
  uint64_t x;
  memcpy(&x, &v, 8);
  unsigned char m[9] = {'f'};
  for (int i = 0; i < 8; i++) m[1 + i] = (unsigned char)(x >> (8 * i));
  return buf_put(b, m, 9);
}

int dgm_enc_binary(dgm_buf* b, const void* p, size_t n) {
  int rc = buf_head(b, 'b', (uint32_t)n);
  return rc ? rc : buf_put(b, p, n);
}

int dgm_enc_tuple(dgm_buf* b, uint32_t arity) { return buf_head(b, 't', arity); }
int dgm_enc_list(dgm_buf* b, uint32_t len) { return buf_head(b, 'l', len); }
int dgm_enc_map(dgm_buf* b, uint32_t size) { return buf_head(b, 'm', size); }

static uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

/* An encoded integer that fits: 1, with *neg and *mag (magnitude < 2^64). */
static int enc_small_int(const unsigned char* e, size_t n, int* neg, uint64_t* mag) {
  if (n < 6 || e[0] != 'i') return 0;
  const uint32_t len = (uint32_t)e[1] | (uint32_t)e[2] << 8 | (uint32_t)e[3] << 16 | (uint32_t)e[4] << 24;
  if (len < 1 || len > 9 || 5 + (size_t)len != n) return 0;
  *neg = e[5];
  uint64_t m = 0;
  for (uint32_t i = 0; i + 1 < len; i++) m |= (uint64_t)e[6 + i] << (8 * i);
  *mag = m;
  return 1;
}

uint64_t dgm_key_id(const unsigned char* enc, size_t n) {
  int neg;
  uint64_t m;
  if (enc_small_int(enc, n, &neg, &m) && !neg) return splitmix64(m);
  return dgm_hash_bytes(enc, n, 0);
}

/* canonical integer value of an encoding: 1 and *v */
static int enc_canonical(const unsigned char* e, size_t n, int64_t* v) {
  int neg;
  uint64_t m;
  if (!enc_small_int(e, n, &neg, &m)) return 0;
  if (!neg) {
    if (m >= (uint64_t)DGM_CANON_HI) return 0;
    *v = (int64_t)m;
    return 1;
  }
  if (m > (uint64_t)0 - (uint64_t)DGM_CANON_LO) return 0;
  *v = (int64_t)((uint64_t)0 - m);
  return 1;
}

int dgm_value_is_canonical(uint64_t id, int64_t* v) {
  if (id < (1ull << 58) || id >= (1ull << 63)) return 0;
  if (v) *v = (int64_t)(id - (1ull << 62));
  return 1;
}

/* ------------------------------------------------------------ the universe */
struct dgm_universe {
  dgm_term_ops ops;
  dgm_buf enc; /* scratch: the encoding of the term at hand */
  /* keys: id and term, found by the key id */
  hmap kmap;
  uint64_t* kid;
  void** kterm;
  uint64_t nk, capk;
  /* table values (every value but the canonical integers): ascending ids, their terms in
   * the same (map-key) order, their term hashes */
  uint64_t* vid;
  void** vterm;
  uint64_t* vhash;
  uint64_t nv, capv;
  uint64_t* rl_old; /* the last relabel */
  uint64_t* rl_new;
  uint64_t nrl;
  /* nodes: dense; found by their term hash */
  hmap nmap;
  void** nterm;
  uint64_t* nhash;
  uint32_t nn, capn;
};

dgm_universe* dgm_universe_new(const dgm_term_ops* ops) {
  if (!ops || !ops->cmp || !ops->encode || !ops->keep || !ops->drop) return NULL;
  dgm_universe* u = (dgm_universe*)calloc(1, sizeof *u);
  if (u) u->ops = *ops;
  return u;
}

void dgm_universe_free(dgm_universe* u) {
  if (!u) return;
  for (uint64_t i = 0; i < u->nk; i++) u->ops.drop(u->kterm[i], u->ops.ud);
  for (uint64_t i = 0; i < u->nv; i++) u->ops.drop(u->vterm[i], u->ops.ud);
  for (uint32_t i = 0; i < u->nn; i++) u->ops.drop(u->nterm[i], u->ops.ud);
  dgm_buf_free(&u->enc);
  free(u->kmap.h);
  free(u->kmap.v);
  free(u->kid);
  free(u->kterm);
  free(u->vid);
  free(u->vterm);
  free(u->vhash);
  free(u->rl_old);
  free(u->rl_new);
  free(u->nmap.h);
  free(u->nmap.v);
  free(u->nterm);
  free(u->nhash);
  free(u);
}

static int grow(void** p, uint64_t* cap, uint64_t need, size_t elem) {
  if (need <= *cap) return DG_OK;
  uint64_t c = *cap ? *cap : 16;
  while (c < need) c *= 2;
  void* q = realloc(*p, c * elem);
  if (!q) return DG_E_NOMEM;
  *p = q;
  *cap = c;
  return DG_OK;
}

/* the canonical encoding of `term` into u->enc */
static int encode(dgm_universe* u, const void* term) {
  u->enc.n = 0;
  return u->ops.encode(term, &u->enc, u->ops.ud);
}

int dgm_key(dgm_universe* u, const void* term, uint64_t* id) {
  uint64_t h;
  if (u->ops.hash) {
    h = u->ops.hash(term, u->ops.ud);
  } else {
    int rc = encode(u, term);
    if (rc) return rc;
    h = dgm_key_id(u->enc.p, u->enc.n);
  }
  const uint64_t hk = nz(h);
  uint64_t slot = u->kmap.cap ? (hk & (u->kmap.cap - 1)) : 0;
  while (hmap_next(&u->kmap, hk, &slot)) {
    const uint32_t i = u->kmap.v[slot];
    if (u->ops.cmp(u->kterm[i], term, u->ops.ud) == 0) {
      *id = u->kid[i];
      return DG_OK;
    }
    /* the same 64-bit id for a different term: an exact collision */
    return DG_E_INVAL;
  }
  int rc;
  if ((rc = grow((void**)&u->kid, &u->capk, u->nk + 1, sizeof *u->kid))) return rc;
  {
    uint64_t capt = u->capk;
    void* q = realloc(u->kterm, capt * sizeof *u->kterm);
    if (!q) return DG_E_NOMEM;
    u->kterm = (void**)q;
  }
  if ((rc = hmap_put(&u->kmap, hk, (uint32_t)u->nk))) return rc;
  u->kid[u->nk] = h;
  u->kterm[u->nk] = u->ops.keep(term, u->ops.ud);
  u->nk++;
  *id = h;
  return DG_OK;
}

const void* dgm_key_term(const dgm_universe* u, uint64_t id) {
  const uint64_t hk = nz(id);
  uint64_t slot = u->kmap.cap ? (hk & (u->kmap.cap - 1)) : 0;
  while (hmap_next(&u->kmap, hk, &slot)) {
    const uint32_t i = u->kmap.v[slot];
    if (u->kid[i] == id) return u->kterm[i];
    slot = (slot + 1) & (u->kmap.cap - 1);
  }
  return NULL;
}

/* first index whose term is >= t (term order); *eq = that term equals t */
static uint64_t value_lb(const dgm_universe* u, const void* t, int* eq) {
  uint64_t lo = 0, hi = u->nv;
  *eq = 0;
  while (lo < hi) {
    const uint64_t mid = (lo + hi) / 2;
    const int c = u->ops.cmp(u->vterm[mid], t, u->ops.ud);
    if (c < 0) {
      lo = mid + 1;
    } else {
      if (c == 0) *eq = 1;
      hi = mid;
    }
  }
  if (*eq && !(lo < u->nv && u->ops.cmp(u->vterm[lo], t, u->ops.ud) == 0)) *eq = 0;
  return lo;
}

/* The two table regions (exclusive bounds) around the canonical ids [2^58, 2^63): integers
 * below DGM_CANON_LO in (0, 2^58), everything above the canonical integers in
 * (2^63 - 1, 2^64) -- in map-key order numbers precede every other class and integers
 * precede floats, so each region holds a contiguous part of the order. */
#define LOW_LO 0ull
#define LOW_HI (1ull << 58)
#define HIGH_LO ((1ull << 63) - 1)

static int in_region(uint64_t id, int low) { return low ? id < LOW_HI : id > HIGH_LO; }

/* an id strictly between the neighbours of insertion point p inside the region, the same
 * choice as the Python Universe (interning.py): the midpoint, or a fixed stride past
 * either end; 0 if the gap is used up */
static uint64_t gap_id(const dgm_universe* u, uint64_t p, int low) {
  const int has_lo = p > 0 && in_region(u->vid[p - 1], low);
  const int has_hi = p < u->nv && in_region(u->vid[p], low);
  /* bounds as (a, b] with b - a = the gap's width, computed without overflow */
  const uint64_t a = has_lo ? u->vid[p - 1] : (low ? LOW_LO : HIGH_LO);
  const uint64_t width = has_hi ? u->vid[p] - a : (low ? LOW_HI : 0ull) - a; /* 2^64 - a wraps */
  if (width < 2) return 0;
  const uint64_t half = width / 2;
  if (!has_lo && !has_hi) return a + half;
  if (!has_hi) return a + (half < ID_STRIDE ? half : ID_STRIDE);
  if (!has_lo) return a + width - (half < ID_STRIDE ? half : ID_STRIDE);
  return a + half;
}

/* re-space the region's value ids evenly (order kept), leaving room for `extra` more */
static int relabel(dgm_universe* u, uint64_t extra, int low) {
  free(u->rl_old);
  free(u->rl_new);
  uint64_t i0 = 0, m = 0;
  while (i0 < u->nv && !in_region(u->vid[i0], low)) i0++;
  while (i0 + m < u->nv && in_region(u->vid[i0 + m], low)) m++;
  u->nrl = m;
  u->rl_old = (uint64_t*)malloc((m ? m : 1) * sizeof(uint64_t));
  u->rl_new = (uint64_t*)malloc((m ? m : 1) * sizeof(uint64_t));
  if (!u->rl_old || !u->rl_new) return DG_E_NOMEM;
  /* step = width / (m + extra + 1); HIGH's width 2^64 - HIGH_LO = 2^63 + 1 */
  const uint64_t d = m + extra + 1;
  const uint64_t base = low ? LOW_LO : HIGH_LO;
  const uint64_t step = low ? LOW_HI / d : ((1ull << 63) / d + ((1ull << 63) % d + 1) / d);
  for (uint64_t j = 0; j < m; j++) {
    u->rl_old[j] = u->vid[i0 + j];
    u->vid[i0 + j] = base + (j + 1) * step;
    u->rl_new[j] = u->vid[i0 + j];
  }
  return DG_OK;
}

int dgm_value(dgm_universe* u, const void* term, uint64_t* id, int* relabeled) {
  if (relabeled) *relabeled = 0;
  int rc = encode(u, term);
  if (rc) return rc;
  int64_t cv;
  if (enc_canonical(u->enc.p, u->enc.n, &cv)) {
    *id = (uint64_t)cv + (1ull << 62);
    return DG_OK;
  }
  /* a negative integer that is not canonical lies below DGM_CANON_LO: the low region */
  const int low = u->enc.p[0] == 'i' && u->enc.p[5] == 1;
  int eq;
  const uint64_t p = value_lb(u, term, &eq);
  if (eq) {
    *id = u->vid[p];
    return DG_OK;
  }
  const uint64_t vh = dgm_hash_bytes(u->enc.p, u->enc.n, DGM_VAL_SEED);
  uint64_t nid = gap_id(u, p, low);
  if (nid == 0) {
    rc = relabel(u, 1, low);
    if (rc) return rc;
    if (relabeled) *relabeled = 1;
    nid = gap_id(u, p, low);
    if (nid == 0) return DG_E_CAPACITY; /* the region is full */
  }
  uint64_t capv = u->capv;
  if ((rc = grow((void**)&u->vid, &u->capv, u->nv + 1, sizeof *u->vid))) return rc;
  if (u->capv != capv || !u->vterm || !u->vhash) {
    void* q = realloc(u->vterm, u->capv * sizeof *u->vterm);
    if (!q) return DG_E_NOMEM;
    u->vterm = (void**)q;
    q = realloc(u->vhash, u->capv * sizeof *u->vhash);
    if (!q) return DG_E_NOMEM;
    u->vhash = (uint64_t*)q;
  }
  memmove(u->vid + p + 1, u->vid + p, (u->nv - p) * sizeof *u->vid);
  memmove(u->vterm + p + 1, u->vterm + p, (u->nv - p) * sizeof *u->vterm);
  memmove(u->vhash + p + 1, u->vhash + p, (u->nv - p) * sizeof *u->vhash);
  u->vid[p] = nid;
  u->vterm[p] = u->ops.keep(term, u->ops.ud);
  u->vhash[p] = vh;
  u->nv++;
  *id = nid;
  return DG_OK;
}

const void* dgm_value_term(const dgm_universe* u, uint64_t id) {
  uint64_t lo = 0, hi = u->nv;
  while (lo < hi) {
    const uint64_t mid = (lo + hi) / 2;
    if (u->vid[mid] < id)
      lo = mid + 1;
    else
      hi = mid;
  }
  return (lo < u->nv && u->vid[lo] == id) ? u->vterm[lo] : NULL;
}

void dgm_last_relabel(const dgm_universe* u, const uint64_t** old_ids, const uint64_t** new_ids,
                      uint64_t* n) {
  *old_ids = u->rl_old;
  *new_ids = u->rl_new;
  *n = u->nrl;
}

uint64_t dgm_value_count(const dgm_universe* u) { return u->nv; }

int dgm_node(dgm_universe* u, const void* term, uint32_t* id) {
  int rc = encode(u, term);
  if (rc) return rc;
  const uint64_t h = dgm_hash_bytes(u->enc.p, u->enc.n, DGM_NODE_SEED);
  const uint64_t hk = nz(h);
  uint64_t slot = u->nmap.cap ? (hk & (u->nmap.cap - 1)) : 0;
  while (hmap_next(&u->nmap, hk, &slot)) {
    const uint32_t i = u->nmap.v[slot];
    if (u->ops.cmp(u->nterm[i], term, u->ops.ud) == 0) {
      *id = i;
      return DG_OK;
    }
    slot = (slot + 1) & (u->nmap.cap - 1);
  }
  if (u->nn == UINT32_MAX) return DG_E_CAPACITY;
  if (u->nn >= u->capn) {
    uint32_t c = u->capn ? u->capn * 2 : 16;
    void* q = realloc(u->nterm, (size_t)c * sizeof *u->nterm);
    if (!q) return DG_E_NOMEM;
    u->nterm = (void**)q;
    q = realloc(u->nhash, (size_t)c * sizeof *u->nhash);
    if (!q) return DG_E_NOMEM;
    u->nhash = (uint64_t*)q;
    u->capn = c;
  }
  rc = hmap_put(&u->nmap, hk, u->nn);
  if (rc) return rc;
  u->nterm[u->nn] = u->ops.keep(term, u->ops.ud);
  u->nhash[u->nn] = h;
  *id = u->nn++;
  return DG_OK;
}

const void* dgm_node_term(const dgm_universe* u, uint32_t id) {
  return id < u->nn ? u->nterm[id] : NULL;
}

uint32_t dgm_node_count(const dgm_universe* u) { return u->nn; }

void dgm_node_hashes(const dgm_universe* u, const uint64_t** hash, uint32_t* n) {
  *hash = u->nhash;
  *n = u->nn;
}

void dgm_value_hashes(const dgm_universe* u, const uint64_t** ids, const uint64_t** hash,
                      uint64_t* n) {
  *ids = u->vid;
  *hash = u->vhash;
  *n = u->nv;
}

/* ------------------------------------------------------------ host rows */
int dgm_rows_init(dgm_rows* r, uint64_t cap_rows, uint64_t cap_ctx) {
  memset(r, 0, sizeof *r);
  if (cap_rows < 16) cap_rows = 16;
  if (cap_ctx < 16) cap_ctx = 16;
  r->s.key = (uint64_t*)malloc(cap_rows * 8);
  r->s.val = (uint64_t*)malloc(cap_rows * 8);
  r->s.ts = (int64_t*)malloc(cap_rows * 8);
  r->s.node = (uint32_t*)malloc(cap_rows * 4);
  r->s.cnt = (uint64_t*)malloc(cap_rows * 8);
  r->c.node = (uint32_t*)malloc(cap_ctx * 4);
  r->c.cnt = (uint64_t*)malloc(cap_ctx * 8);
  r->s.cap = cap_rows;
  r->c.cap = cap_ctx;
  if (!r->s.key || !r->s.val || !r->s.ts || !r->s.node || !r->s.cnt || !r->c.node || !r->c.cnt) {
    dgm_rows_free(r);
    return DG_E_NOMEM;
  }
  return DG_OK;
}

void dgm_rows_free(dgm_rows* r) {
  free(r->s.key);
  free(r->s.val);
  free(r->s.ts);
  free(r->s.node);
  free(r->s.cnt);
  free(r->c.node);
  free(r->c.cnt);
  memset(r, 0, sizeof *r);
}

void dgm_rows_clear(dgm_rows* r) {
  r->s.n = 0;
  r->c.n = 0;
}

#define REGROW(p, T, cap) \
  do {                    \
    void* q_ = realloc((p), (cap) * sizeof(T)); \
    if (!q_) return DG_E_NOMEM; \
    (p) = (T*)q_;         \
  } while (0)

int dgm_rows_push(dgm_rows* r, uint64_t key, uint64_t val, int64_t ts, uint32_t node, uint64_t cnt) {
  if (r->s.n == r->s.cap) {
    const uint64_t c = r->s.cap * 2;
    REGROW(r->s.key, uint64_t, c);
    REGROW(r->s.val, uint64_t, c);
    REGROW(r->s.ts, int64_t, c);
    REGROW(r->s.node, uint32_t, c);
    REGROW(r->s.cnt, uint64_t, c);
    r->s.cap = c;
  }
  const uint64_t i = r->s.n++;
  r->s.key[i] = key;
  r->s.val[i] = val;
  r->s.ts[i] = ts;
  r->s.node[i] = node;
  r->s.cnt[i] = cnt;
  return DG_OK;
}

int dgm_ctx_push(dgm_rows* r, uint32_t node, uint64_t cnt) {
  if (r->c.n == r->c.cap) {
    const uint64_t c = r->c.cap * 2;
    REGROW(r->c.node, uint32_t, c);
    REGROW(r->c.cnt, uint64_t, c);
    r->c.cap = c;
  }
  r->c.node[r->c.n] = node;
  r->c.cnt[r->c.n++] = cnt;
  return DG_OK;
}

/* ------------------------------------------------------------ unmarshal order */
int dgm_walk_rows(const dg_store* s, const dgm_walk* w, void* ud) {
  uint64_t i = 0;
  while (i < s->n) {
    const uint64_t k = s->key[i];
    uint64_t ke = i, entries = 0;
    while (ke < s->n && s->key[ke] == k) {
      const uint64_t v = s->val[ke];
      const int64_t t = s->ts[ke];
      while (ke < s->n && s->key[ke] == k && s->val[ke] == v && s->ts[ke] == t) ke++;
      entries++;
    }
    int rc = w->key ? w->key(ud, k, entries) : 0;
    if (rc) return rc;
    while (i < ke) {
      const uint64_t v = s->val[i];
      const int64_t t = s->ts[i];
      uint64_t ee = i;
      while (ee < ke && s->val[ee] == v && s->ts[ee] == t) ee++;
      rc = w->entry ? w->entry(ud, v, t, ee - i) : 0;
      if (rc) return rc;
      for (; i < ee; i++) {
        rc = w->dot ? w->dot(ud, s->node[i], s->cnt[i]) : 0;
        if (rc) return rc;
      }
    }
  }
  return 0;
}

/* ------------------------------------------------------------ key hash */
static uint64_t rotl(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }

uint64_t dgm_hash_bytes(const void* p, size_t n, uint64_t seed) {
  /* xxh64 */
  const uint64_t P1 = 11400714785074694791ull, P2 = 14029467366897019727ull,
                 P3 = 1609587929392839161ull, P4 = 9650029242287828579ull,
                 P5 = 2870177450012600261ull;
  const unsigned char* b = (const unsigned char*)p;
  const unsigned char* end = b + n;
  uint64_t h;
  if (n >= 32) {
    uint64_t v1 = seed + P1 + P2, v2 = seed + P2, v3 = seed, v4 = seed - P1;
    const unsigned char* lim = end - 32;
    do {
      uint64_t x[4];
      memcpy(x, b, 32);
      v1 = rotl(v1 + x[0] * P2, 31) * P1;
      v2 = rotl(v2 + x[1] * P2, 31) * P1;
      v3 = rotl(v3 + x[2] * P2, 31) * P1;
      v4 = rotl(v4 + x[3] * P2, 31) * P1;
      b += 32;
    } while (b <= lim);
    h = rotl(v1, 1) + rotl(v2, 7) + rotl(v3, 12) + rotl(v4, 18);
    uint64_t vs[4] = {v1, v2, v3, v4};
    for (int i = 0; i < 4; i++) {
      h ^= rotl(vs[i] * P2, 31) * P1;
      h = h * P1 + P4;
    }
  } else {
    h = seed + P5;
  }
  h += (uint64_t)n;
  while (b + 8 <= end) {
    uint64_t x;
    memcpy(&x, b, 8);
    h ^= rotl(x * P2, 31) * P1;
    h = rotl(h, 27) * P1 + P4;
    b += 8;
  }
  if (b + 4 <= end) {
    uint32_t x;
    memcpy(&x, b, 4);
    h ^= (uint64_t)x * P1;
    h = rotl(h, 23) * P2 + P3;
    b += 4;
  }
  while (b < end) {
    h ^= (*b++) * P5;
    h = rotl(h, 11) * P1;
  }
  h ^= h >> 33;
  h *= P2;
  h ^= h >> 29;
  h *= P3;
  h ^= h >> 32;
  return h;
}
