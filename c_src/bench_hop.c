/*
 * bench_hop.c — per-message cost of CausalCrdt's anti-entropy exchange as the NIF runs it
 * (c_src/replica.c, the calls deltagpu_nif.c makes): two replicas of `n` keys differing
 * on `frac` of them, Merkle trees of depth `depth`, then
 *   A: prepare_partial_diff(mm, 8)                         (causal_crdt.ex:255)
 *   B: continue_partial_diff(cont, mm, 8), truncated       (:96-98)
 *   A: continue ..., B: continue ... until {:ok, keys}     (:104-105)
 * each message as the bytes the NIF hands to the BEAM and gets back (copied between the
 * calls, as a send would), max_sync_size 200 (delta_crdt.ex:32).  Wall time per hop,
 * median over reps.  Prints one JSON line.
 *     bench_hop N_KEYS DEPTH [REPS [FRAC_PERMILLE [MAX_SYNC]]]
 */
#define _POSIX_C_SOURCE 200809L
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "replica.h"

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

static int cmp_u64(const void* a, const void* b) {
  const uint64_t x = *(const uint64_t*)a, y = *(const uint64_t*)b;
  return x < y ? -1 : x > y;
}

static uint64_t mix(uint64_t x) {
  x += 0x9E3779B97F4A7C15ULL;
  x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ULL;
  x = (x ^ (x >> 27)) * 0x94d049bb133111ebULL;
  return x ^ (x >> 31);
}

#define MAX_HOPS 16

int main(int argc, char** argv) {
  const uint64_t n = argc > 1 ? strtoull(argv[1], NULL, 10) : 1000000;
  const uint32_t depth = argc > 2 ? (uint32_t)atoi(argv[2]) : 18;
  const int reps = argc > 3 ? atoi(argv[3]) : 20;
  const uint64_t permille = argc > 4 ? strtoull(argv[4], NULL, 10) : 10;
  const uint64_t max_sync = argc > 5 ? strtoull(argv[5], NULL, 10) : 200;
  const uint32_t levels = 8;
  /* one row per key: key = a hash, val = i, ts = i, node 0, cnt = i + 1; B's values
   * differ on `permille` / 1000 of the keys (the rows stay in key order) */
  uint64_t* key = malloc(n * 8);
  for (uint64_t i = 0; i < n; i++) key[i] = mix(i);
  qsort(key, n, 8, cmp_u64);
  uint64_t *val = malloc(n * 8), *cnt = malloc(n * 8), *valb = malloc(n * 8);
  int64_t* ts = malloc(n * 8);
  uint32_t* node = calloc(n, 4);
  for (uint64_t i = 0; i < n; i++) {
    val[i] = i;
    ts[i] = (int64_t)i;
    cnt[i] = i + 1;
    valb[i] = (mix(i ^ 0x5555) % 1000) < permille ? i + (UINT64_C(1) << 40) : i;
  }
  dgr_engine* g;
  DG(dgr_engine_open(0, &g));
  DG(dgr_refresh_terms(g, NULL, 0, NULL, NULL, 0));
  uint32_t n0 = 0;
  uint64_t c0 = n;
  dg_context vv = {DG_CTX_VV, 0, &n0, &c0, 1, 1};
  dg_store ra = {key, val, ts, node, cnt, n, n}, rb = {key, valb, ts, node, cnt, n, n};
  dgr_state *A, *B;
  DG(dgr_state_load(g, &ra, &vv, &A));
  DG(dgr_state_load(g, &rb, &vv, &B));
  DG(dgr_merkle_build(A, dgr_state_version(A), depth));
  DG(dgr_merkle_build(B, dgr_state_version(B), depth));
  double* t[MAX_HOPS];
  for (int h = 0; h < MAX_HOPS; h++) t[h] = calloc((size_t)reps, sizeof(double));
  uint64_t bytes[MAX_HOPS] = {0}, keys_out = 0;
  int hops = 0;
  uint8_t* msg = malloc(1);
  uint64_t msg_cap = 1;
  for (int it = -3; it < reps; it++) {
    const uint8_t* out;
    uint64_t len;
    double t0 = now_us();
    DG(dgr_merkle_prepare(A, dgr_state_version(A), levels, &out, &len));
    double el = now_us() - t0;
    int h = 0;
    if (it >= 0) t[h][it] = el;
    bytes[h] = len;
    for (;;) {
      if (msg_cap < len) {
        msg = realloc(msg, len);
        msg_cap = len;
      }
      memcpy(msg, out, len); /* the message crosses to the other replica */
      const uint64_t mlen = len;
      dgr_state* S = (h % 2 == 0) ? B : A;
      int status;
      const uint64_t* k;
      uint64_t nk;
      t0 = now_us();
      DG(dgr_merkle_continue(S, dgr_state_version(S), msg, mlen, levels, max_sync, &status, &out, &len, &k, &nk));
      el = now_us() - t0;
      h++;
      if (h >= MAX_HOPS) {
        fprintf(stderr, "too many hops\n");
        return 1;
      }
      if (it >= 0) t[h][it] = el;
      if (status == 0) {
        bytes[h] = 8 * nk;
        keys_out = nk;
        break;
      }
      bytes[h] = len;
    }
    hops = h + 1;
  }
  printf("{\"n_keys\": %llu, \"depth\": %u, \"levels\": %u, \"max_sync_size\": %llu, \"differing_permille\": %llu, "
         "\"reps\": %d, \"path\": \"c_src/replica.c (the NIF's calls)\", \"keys\": %llu, \"hops\": [",
         (unsigned long long)n, depth, levels, (unsigned long long)max_sync, (unsigned long long)permille, reps,
         (unsigned long long)keys_out);
  double total = 0;
  for (int h = 0; h < hops; h++) {
    qsort(t[h], (size_t)reps, sizeof(double), cmp_d);
    const double m = t[h][reps / 2];
    total += m;
    printf("%s{\"call\": \"%s\", \"us\": %.2f, \"bytes\": %llu}", h ? ", " : "",
           h == 0 ? "prepare" : (h == hops - 1 ? "continue -> ok" : "continue"), m, (unsigned long long)bytes[h]);
  }
  printf("], \"total_us\": %.2f}\n", total);
  dgr_state_free(A);
  dgr_state_free(B);
  dgr_engine_close(g);
  return 0;
}
