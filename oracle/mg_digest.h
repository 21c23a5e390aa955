/* mg_digest.h — TEST INFRASTRUCTURE ONLY (oracle/).
 *
 * Order-independent digests of a directed edge multiset and of a superReadID
 * vector, so that a 10^8-row result can be pinned by a few numbers instead of
 * a multi-GB dump.  The same formulas are implemented, independently, by the
 * product (mg_rows_digest / mg_super_digest in include/mg_overlap.h, computed
 * on the device) and by tests/digest.py (numpy); the three must agree.
 *
 *   mix64(x)  = the murmur3-style finaliser below (bijective)
 *   row (u, v, orient, offset):
 *     h = mix64(((u << 32) | v) ^ mix64(((orient << 16) | offset) + 0x9E3779B97F4A7C15))
 *   rows digest  = { n, sum h, xor h, sum mix64(h ^ 0xD6E8FEB86659FD93) }   (mod 2^64)
 *   super digest = { contained reads, sum g, xor g, sum mix64(g ^ 0xD6E8...) }
 *                  with g = mix64((id << 32) | superReadID) over ids with superReadID != 0
 */
#ifndef MG_DIGEST_H_
#define MG_DIGEST_H_
#include <stdint.h>

typedef struct mgo_digest {
  uint64_t n, sum, xr, sum2;
} mgo_digest;

static inline uint64_t mgo_mix64(uint64_t x) {
  x ^= x >> 31;
  x *= 0x7fb5d329728ea185ULL;
  x ^= x >> 27;
  x *= 0x81dadef4bc2dd44dULL;
  x ^= x >> 33;
  return x;
}

static inline void mgo_digest_add(mgo_digest* d, uint64_t h) {
  d->n += 1;
  d->sum += h;
  d->xr ^= h;
  d->sum2 += mgo_mix64(h ^ 0xD6E8FEB86659FD93ULL);
}

static inline uint64_t mgo_row_hash(uint64_t u, uint64_t v, uint64_t orient, uint64_t offset) {
  return mgo_mix64(((u << 32) | v) ^ mgo_mix64(((orient << 16) | offset) + 0x9E3779B97F4A7C15ULL));
}

static inline uint64_t mgo_super_hash(uint64_t id, uint64_t super_id) { return mgo_mix64((id << 32) | super_id); }

#endif /* MG_DIGEST_H_ */
