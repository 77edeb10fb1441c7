// dg_hash.h — the Merkle hash functions (host and device).
//
// MerkleMap 0.2.0 (the reference's dependency, mix.lock:13) is not vendored, so its
// hash and wire format cannot be reproduced ("parity unpinned").
// What is reproduced is its role: a key's leaf depends on the key's raw value map
// (every {v, ts} entry and dot, causal_crdt.ex:392), and two replicas' trees differ
// exactly above the keys whose raw value maps differ.
//
//   row_hash  = mix(mix(mix(mix(mix(key ^ G) ^ val) ^ ts) ^ node) ^ cnt)
//               (val / node: the ids, or their term hashes -- dg_term_hashes)
//   leaf(k)   = Σ row_hash over k's rows                  (mod 2^64, order-free)
//   bucket(b) = Σ leaf(k) over keys with k >> (64-depth) == b
//   parent    = mix(left ^ mix(right ^ H))
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define DG_HD __host__ __device__ inline
#else
#define DG_HD static inline
#endif

namespace dg {

DG_HD uint64_t mix64(uint64_t x) {
  x ^= x >> 30;
  x *= 0xbf58476d1ce4e5b9ULL;
  x ^= x >> 27;
  x *= 0x94d049bb133111ebULL;
  x ^= x >> 31;
  return x;
}

DG_HD uint64_t row_hash(uint64_t key, uint64_t val, int64_t ts, uint64_t node, uint64_t cnt) {
  uint64_t h = mix64(key ^ 0x9E3779B97F4A7C15ULL);
  h = mix64(h ^ val);
  h = mix64(h ^ (uint64_t)ts);
  h = mix64(h ^ node);
  return mix64(h ^ cnt);
}

DG_HD uint64_t node_hash(uint64_t left, uint64_t right) {
  return mix64(left ^ mix64(right ^ 0xD6E8FEB86659FD93ULL));
}

}  // namespace dg
