/* mg_oracle.c — TEST INFRASTRUCTURE ONLY (oracle/).  See mg_oracle.h.
 *
 * Plain-C, single-threaded restatement of the reference algorithm.  Every
 * function cites the reference file:line it restates (paths relative to
 * /root/reference/MetaGenomics).  Parity is pinned by tests/golden/ fixtures
 * produced by the reference itself (oracle/_ref/ref_harness).
 */
#define _POSIX_C_SOURCE 199309L
#include "mg_oracle.h"
#include "mg_digest.h"

#include <ctype.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

typedef struct {
  char* fwd;  /* canonical forward string  (Read::read,        Read.h:35) */
  char* rev;  /* its reverse complement    (Read::readReverse, Read.h:36) */
  uint32_t len;
  uint32_t freq;
} oread;

struct mgo_dataset {
  oread* reads; /* sorted unique reads; ID = index + 1 */
  uint64_t n_unique, n_reads, cap;
  uint64_t shortest, longest; /* Dataset.h:35-36 */
  /* exact-key hash table (HashTable.h:18-24) */
  uint64_t h;
  int64_t* slots;
  uint64_t slot_mask;
  struct bucket {
    const char* key;
    uint64_t* items; /* id | o << 62, insertion order (HashTable.cpp:165,188) */
    uint32_t n, cap;
  } * buckets;
  uint64_t n_buckets, bucket_cap;
};

static double now_s(void) {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec + 1e-9 * ts.tv_nsec;
}

/* Dataset::reverseComplement (Dataset.cpp:463-475): XOR trick on ASCII. */
static void revcomp(const char* s, uint32_t n, char* out) {
  for (uint32_t i = 0; i < n; i++) {
    char c = s[i];
    out[n - i - 1] = (c & 0x02) ? (char)(c ^ 0x04) : (char)(c ^ 0x15);
  }
  out[n] = 0;
}

/* Dataset::testRead (Dataset.cpp:398-413). */
static int test_read(const char* s, uint32_t n) {
  uint64_t cnt[4] = {0, 0, 0, 0};
  for (uint32_t i = 0; i < n; i++) {
    char c = s[i];
    if (c != 'A' && c != 'C' && c != 'G' && c != 'T') return 0;
    cnt[(c >> 1) & 3]++;
  }
  uint64_t threshold = (uint64_t)(n * .8);
  if (cnt[0] >= threshold || cnt[1] >= threshold || cnt[2] >= threshold || cnt[3] >= threshold) return 0;
  return 1;
}

/* Body of the read loop in Dataset::readDataset (Dataset.cpp:158-181):
 * upper-case, keep if len > minOverlap && testRead, store min(s, rc(s)). */
static void add_read(mgo_dataset* ds, const char* s, uint64_t n, uint64_t min_overlap) {
  if (!(n > min_overlap)) return;
  char* up = (char*)malloc(n + 1);
  for (uint64_t i = 0; i < n; i++) up[i] = (char)toupper((unsigned char)s[i]);
  up[n] = 0;
  if (!test_read(up, (uint32_t)n)) {
    free(up);
    return;
  }
  char* rc = (char*)malloc(n + 1);
  revcomp(up, (uint32_t)n, rc);
  if (ds->n_reads == ds->cap) {
    ds->cap = ds->cap ? 2 * ds->cap : 1024;
    ds->reads = (oread*)realloc(ds->reads, ds->cap * sizeof(oread));
  }
  oread* r = &ds->reads[ds->n_reads++];
  r->len = (uint32_t)n;
  r->freq = 1;
  if (memcmp(up, rc, n) < 0) { /* line1.compare(rc) < 0  (Dataset.cpp:164) */
    r->fwd = up;
    r->rev = rc;
  } else {
    r->fwd = rc;
    r->rev = up;
  }
  if (n > ds->longest) ds->longest = n;
  if (n < ds->shortest) ds->shortest = n;
}

/* compareReads (Dataset.cpp:16-19): std::string operator<. */
static int cmp_reads(const void* a, const void* b) {
  const oread* x = (const oread*)a;
  const oread* y = (const oread*)b;
  uint32_t m = x->len < y->len ? x->len : y->len;
  int c = memcmp(x->fwd, y->fwd, m);
  if (c) return c;
  return (x->len > y->len) - (x->len < y->len);
}

/* sortReads + removeDupicateReads (Dataset.cpp:197-202,316-345). */
static void finish_dataset(mgo_dataset* ds) {
  if (ds->n_reads) qsort(ds->reads, ds->n_reads, sizeof(oread), cmp_reads);
  uint64_t j = 0;
  for (uint64_t i = 0; i < ds->n_reads; i++) {
    if (i == 0) continue;
    oread* a = &ds->reads[j];
    oread* b = &ds->reads[i];
    if (a->len != b->len || memcmp(a->fwd, b->fwd, a->len)) {
      j++;
      oread t = ds->reads[j];
      ds->reads[j] = ds->reads[i];
      ds->reads[i] = t;
    } else {
      a->freq++;
    }
  }
  ds->n_unique = ds->n_reads ? j + 1 : 0;
  for (uint64_t i = ds->n_unique; i < ds->n_reads; i++) {
    free(ds->reads[i].fwd);
    free(ds->reads[i].rev);
  }
}

static mgo_dataset* new_dataset(void) {
  mgo_dataset* ds = (mgo_dataset*)calloc(1, sizeof(mgo_dataset));
  ds->shortest = ~0ULL;
  return ds;
}

/* Dataset::readDataset (Dataset.cpp:110-193): FASTA records are a header line
 * then everything up to the next '>' with '\n' removed (:139-147); FASTQ
 * records are 4 lines, the sequence is the 2nd (:149-157). */
static int parse_file(mgo_dataset* ds, const char* path, uint64_t min_overlap) {
  FILE* f = fopen(path, "rb");
  if (!f) return -1;
  fseek(f, 0, SEEK_END);
  long sz = ftell(f);
  fseek(f, 0, SEEK_SET);
  char* buf = (char*)malloc(sz + 1);
  if (sz > 0 && fread(buf, 1, sz, f) != (size_t)sz) {
    fclose(f);
    free(buf);
    return -1;
  }
  fclose(f);
  buf[sz] = 0;
  if (sz == 0 || (buf[0] != '>' && buf[0] != '@')) {
    free(buf);
    return -2; /* "Unknown input file format." (Dataset.cpp:134-135) */
  }
  char* seq = (char*)malloc(sz + 1);
  long p = 0;
  if (buf[0] == '>') {
    while (p < sz) {
      while (p < sz && buf[p] != '\n') p++; /* header line */
      if (p < sz) p++;
      uint64_t n = 0;
      while (p < sz && buf[p] != '>') {
        if (buf[p] != '\n') seq[n++] = buf[p];
        p++;
      }
      if (p < sz) p++; /* consume '>' */
      add_read(ds, seq, n, min_overlap);
    }
  } else {
    long line = 0;
    while (p < sz) {
      long s = p;
      while (p < sz && buf[p] != '\n') p++;
      if (line % 4 == 1) add_read(ds, buf + s, (uint64_t)(p - s), min_overlap);
      if (p < sz) p++;
      line++;
    }
  }
  free(seq);
  free(buf);
  return 0;
}

mgo_dataset* mgo_dataset_from_files(const char* const* files, int nfiles, uint64_t min_overlap) {
  mgo_dataset* ds = new_dataset();
  for (int i = 0; i < nfiles; i++) {
    if (parse_file(ds, files[i], min_overlap)) {
      mgo_dataset_free(ds);
      return NULL;
    }
  }
  finish_dataset(ds);
  return ds;
}

mgo_dataset* mgo_dataset_from_seqs(const char* concat, const uint64_t* offsets, uint64_t n,
                                   uint64_t min_overlap) {
  mgo_dataset* ds = new_dataset();
  for (uint64_t i = 0; i < n; i++) add_read(ds, concat + offsets[i], offsets[i + 1] - offsets[i], min_overlap);
  finish_dataset(ds);
  return ds;
}

/* Same pipeline from 2-bit codes (0..3 = A C G T) of n reads, read i at
 * codes[i * stride, i * stride + lens[i]): the synthetic workloads' form. */
mgo_dataset* mgo_dataset_from_codes(const uint8_t* codes, uint64_t stride, const uint16_t* lens, uint64_t n,
                                    uint64_t min_overlap) {
  mgo_dataset* ds = new_dataset();
  char* s = (char*)malloc(stride + 1);
  for (uint64_t i = 0; i < n; i++) {
    const uint8_t* c = codes + i * stride;
    for (uint64_t k = 0; k < lens[i]; k++) s[k] = "ACGT"[c[k] & 3];
    add_read(ds, s, lens[i], min_overlap);
  }
  free(s);
  finish_dataset(ds);
  return ds;
}

static void free_table(mgo_dataset* ds) {
  if (ds->buckets) {
    for (uint64_t b = 0; b < ds->n_buckets; b++) free(ds->buckets[b].items);
    free(ds->buckets);
  }
  free(ds->slots);
  ds->buckets = NULL;
  ds->slots = NULL;
  ds->n_buckets = ds->bucket_cap = 0;
}

void mgo_dataset_free(mgo_dataset* ds) {
  if (!ds) return;
  for (uint64_t i = 0; i < ds->n_unique; i++) {
    free(ds->reads[i].fwd);
    free(ds->reads[i].rev);
  }
  free(ds->reads);
  free_table(ds);
  free(ds);
}

uint64_t mgo_num_reads(const mgo_dataset* ds) { return ds->n_reads; }
uint64_t mgo_num_unique(const mgo_dataset* ds) { return ds->n_unique; }
const char* mgo_read(const mgo_dataset* ds, uint64_t id, uint32_t* len) {
  if (id < 1 || id > ds->n_unique) return NULL; /* Dataset.cpp:484-490 */
  if (len) *len = ds->reads[id - 1].len;
  return ds->reads[id - 1].fwd;
}
uint32_t mgo_frequency(const mgo_dataset* ds, uint64_t id) {
  return (id < 1 || id > ds->n_unique) ? 0 : ds->reads[id - 1].freq;
}

/* --- exact-key multimap (HashTable.cpp:50-221).  The reference's own hash
 * (hashFunction, :135-155) only picks a probe start; bucket lists are exact-key
 * lists in insertion order, so any hash is equivalent. --- */
static uint64_t key_hash(const char* s, uint64_t h) {
  uint64_t x = 1469598103934665603ULL;
  for (uint64_t i = 0; i < h; i++) x = (x ^ (unsigned char)s[i]) * 1099511628211ULL;
  return x ^ (x >> 29);
}

static struct bucket* find_bucket(mgo_dataset* ds, const char* key, int create) {
  uint64_t i = key_hash(key, ds->h) & ds->slot_mask;
  for (;;) {
    int64_t b = ds->slots[i];
    if (b < 0) break;
    if (!memcmp(ds->buckets[b].key, key, ds->h)) return &ds->buckets[b];
    i = (i + 1) & ds->slot_mask;
  }
  if (!create) return NULL;
  if (ds->n_buckets == ds->bucket_cap) {
    ds->bucket_cap = ds->bucket_cap ? 2 * ds->bucket_cap : 1024;
    ds->buckets = (struct bucket*)realloc(ds->buckets, ds->bucket_cap * sizeof(struct bucket));
  }
  struct bucket* nb = &ds->buckets[ds->n_buckets];
  nb->key = key;
  nb->items = NULL;
  nb->n = nb->cap = 0;
  ds->slots[i] = (int64_t)ds->n_buckets++;
  return nb;
}

/* insertIntoTable (HashTable.cpp:163-195): append id | o << 62. */
static void insert_key(mgo_dataset* ds, const char* key, uint64_t id, uint64_t o) {
  struct bucket* b = find_bucket(ds, key, 1);
  if (b->n == b->cap) {
    b->cap = b->cap ? 2 * b->cap : 2;
    b->items = (uint64_t*)realloc(b->items, b->cap * sizeof(uint64_t));
  }
  b->items[b->n++] = id | (o << 62);
}

/* insertDataset + hashRead (HashTable.cpp:50-80, 88-104). */
static void build_table(mgo_dataset* ds, uint64_t min_overlap) {
  free_table(ds);
  ds->h = min_overlap - 1; /* :54 */
  uint64_t cap = 16;
  while (cap < 8 * ds->n_unique + 16) cap <<= 1;
  ds->slots = (int64_t*)malloc(cap * sizeof(int64_t));
  memset(ds->slots, 0xff, cap * sizeof(int64_t));
  ds->slot_mask = cap - 1;
  uint64_t h = ds->h;
  for (uint64_t i = 1; i <= ds->n_unique; i++) {
    oread* r = &ds->reads[i - 1];
    insert_key(ds, r->fwd, i, 0);               /* prefix of forward  */
    insert_key(ds, r->fwd + r->len - h, i, 1);  /* suffix of forward  */
    insert_key(ds, r->rev, i, 2);               /* prefix of reverse  */
    insert_key(ds, r->rev + r->len - h, i, 3);  /* suffix of reverse  */
  }
}

/* checkOverlapForContainedRead (OverlapGraph.cpp:302-340). */
static int contained_check(const oread* r1, const oread* r2, uint64_t o, uint64_t j, uint64_t h) {
  const char* s2 = (o == 0 || o == 1) ? r2->fwd : r2->rev;
  uint64_t n1 = r1->len, n2 = r2->len;
  if (o == 0 || o == 2) {
    uint64_t rem1 = n1 - j - h, rem2 = n2 - h;
    if (rem1 >= rem2) return !memcmp(r1->fwd + j + h, s2 + h, rem2);
  } else {
    uint64_t rem1 = j, rem2 = n2 - h;
    if (rem1 >= rem2) return !memcmp(r1->fwd + j - rem2, s2, rem2);
  }
  return 0;
}

/* checkOverlap (OverlapGraph.cpp:354-383). */
static int overlap_check(const oread* r1, const oread* r2, uint64_t o, uint64_t j, uint64_t h) {
  const char* s2 = (o == 0 || o == 1) ? r2->fwd : r2->rev;
  uint64_t n1 = r1->len, n2 = r2->len;
  if (o == 0 || o == 2) {
    if (n1 - j - h >= n2 - h) return 0; /* :367 */
    return !memcmp(r1->fwd + j + h, s2 + h, n1 - (j + h));
  }
  if (n2 - h < j) return 0; /* :379 */
  return !memcmp(r1->fwd, s2 + (n2 - h - j), j);
}

typedef struct {
  mgo_row* v;
  uint64_t n, cap;
} rowvec;

static void push_row(rowvec* rv, uint32_t s, uint32_t d, uint8_t o, uint16_t off) {
  if (rv->n == rv->cap) {
    rv->cap = rv->cap ? 2 * rv->cap : 4096;
    rv->v = (mgo_row*)realloc(rv->v, rv->cap * sizeof(mgo_row));
  }
  mgo_row* r = &rv->v[rv->n++];
  r->src = s;
  r->dst = d;
  r->offset = off;
  r->orient = o;
  r->pad = 0;
}

/* twinEdgeOrientation (OverlapGraph.cpp:841-855). */
static uint8_t twin_orient(uint8_t o) { return o == 0 ? 3 : (o == 3 ? 0 : o); }

int mgo_overlaps(mgo_dataset* ds, uint64_t min_overlap, uint64_t* super_out, mgo_row** rows_out,
                 uint64_t* nrows, double* t_hash, double* t_disc) {
  if (min_overlap < 2) return -1;
  uint64_t N = ds->n_unique, h = min_overlap - 1;
  double t0 = now_s();
  build_table(ds, min_overlap);
  double t1 = now_s();
  uint64_t* super = (uint64_t*)calloc(N + 1, sizeof(uint64_t));

  /* markContainedReads (OverlapGraph.cpp:225-290): skipped if all reads have
   * the same length (:228-233). */
  if (N && ds->longest != ds->shortest) {
    for (uint64_t i = 1; i <= N; i++) {
      oread* r1 = &ds->reads[i - 1];
      for (uint64_t j = 1; j < r1->len - h; j++) {
        struct bucket* b = find_bucket(ds, r1->fwd + j, 0);
        if (!b) continue;
        for (uint32_t k = 0; k < b->n; k++) {
          uint64_t data = b->items[k];
          uint64_t id2 = data & 0x3FFFFFFFFFFFFFFFULL, o = data >> 62;
          oread* r2 = &ds->reads[id2 - 1];
          if (r1->len > r2->len && contained_check(r1, r2, o, j, h)) {
            if (super[id2] == 0)
              super[id2] = i;
            else if (r1->len > ds->reads[super[id2] - 1].len) /* strictly longer (:266) */
              super[id2] = i;
          }
        }
      }
    }
  }

  /* ID-order exploration of insertAllEdgesOfRead (OverlapGraph.cpp:529-565);
   * the raw multiset does not depend on the order. */
  unsigned char* explored = (unsigned char*)calloc(N + 1, 1);
  rowvec rv = {0, 0, 0};
  for (uint64_t i = 1; i <= N; i++) {
    oread* r1 = &ds->reads[i - 1];
    uint64_t n1 = r1->len;
    for (uint64_t j = 1; j < n1 - h; j++) {
      struct bucket* b = find_bucket(ds, r1->fwd + j, 0);
      if (!b) continue;
      for (uint32_t k = 0; k < b->n; k++) {
        uint64_t data = b->items[k];
        uint64_t id2 = data & 0x3FFFFFFFFFFFFFFFULL, o = data >> 62;
        if (explored[id2]) continue; /* :546 */
        oread* r2 = &ds->reads[id2 - 1];
        if (super[i] == 0 && super[id2] == 0 && overlap_check(r1, r2, o, j, h)) {
          uint8_t orient;
          uint16_t ovl;
          switch (o) { /* :550-556 */
            case 0: orient = 3; ovl = (uint16_t)(n1 - j); break;
            case 1: orient = 0; ovl = (uint16_t)(h + j); break;
            case 2: orient = 2; ovl = (uint16_t)(n1 - j); break;
            default: orient = 1; ovl = (uint16_t)(h + j); break;
          }
          uint16_t off = (uint16_t)(n1 - ovl);                              /* :557 */
          uint16_t off_rev = (uint16_t)(r2->len + off - n1);                /* :410 */
          push_row(&rv, (uint32_t)i, (uint32_t)id2, orient, off);          /* insertEdge(Read*,..) */
          push_row(&rv, (uint32_t)id2, (uint32_t)i, twin_orient(orient), off_rev);
        }
      }
    }
    explored[i] = 1;
  }
  double t2 = now_s();
  free(explored);
  if (super_out) memcpy(super_out, super, (N + 1) * sizeof(uint64_t));
  free(super);
  *rows_out = rv.v;
  *nrows = rv.n;
  if (t_hash) *t_hash = t1 - t0;
  if (t_disc) *t_disc = t2 - t1;
  return 0;
}

uint64_t mgo_lookup(mgo_dataset* ds, uint64_t min_overlap, const char* key, uint64_t* out, uint64_t cap) {
  if (!ds->slots || ds->h != min_overlap - 1) build_table(ds, min_overlap);
  if (strlen(key) != ds->h) return 0;
  struct bucket* b = find_bucket(ds, key, 0);
  if (!b) return 0;
  for (uint32_t k = 0; k < b->n && k < cap; k++) out[k] = b->items[k];
  return b->n;
}

void mgo_free(void* p) { free(p); }

/* --- the same hot path, split over threads by source read, digests only ---
 *
 * For workloads whose row lists do not fit in memory (C5: 50M reads): the
 * loops are mgo_overlaps' loops, line for line, over source-read ranges.
 *  - markContainedReads (OverlapGraph.cpp:225-290): thread t runs the loop over
 *    sources [lo_t, hi_t) into its own superReadID array with the reference's
 *    rule (first containing read, replaced only by a strictly longer one,
 *    :259-268); the arrays are then folded in source order with the same rule,
 *    which is the rule applied to the whole sequence i = 1..N.
 *  - insertAllEdgesOfRead (OverlapGraph.cpp:529-565) in ID order: when read i
 *    is explored, the explored reads are exactly IDs 1..i-1, so the :546 test
 *    is id2 < i and every source is independent; rows go into additive digests
 *    (mg_digest.h) instead of a list. */
typedef struct {
  mgo_dataset* ds;
  uint64_t h, lo, hi;
  uint32_t* sup;          /* containment: this range's superReadIDs */
  const uint64_t* super;  /* discovery: the folded superReadIDs */
  uint64_t* next;         /* discovery: shared chunk cursor */
  uint64_t chunk;
  mgo_digest d;
} mgo_task;

static void* contain_range(void* arg) {
  mgo_task* t = (mgo_task*)arg;
  mgo_dataset* ds = t->ds;
  uint64_t h = t->h;
  for (uint64_t i = t->lo; i < t->hi; i++) {
    oread* r1 = &ds->reads[i - 1];
    for (uint64_t j = 1; j < r1->len - h; j++) {
      struct bucket* b = find_bucket(ds, r1->fwd + j, 0);
      if (!b) continue;
      for (uint32_t k = 0; k < b->n; k++) {
        uint64_t data = b->items[k];
        uint64_t id2 = data & 0x3FFFFFFFFFFFFFFFULL, o = data >> 62;
        oread* r2 = &ds->reads[id2 - 1];
        if (r1->len > r2->len && contained_check(r1, r2, o, j, h)) {
          if (t->sup[id2] == 0)
            t->sup[id2] = (uint32_t)i;
          else if (r1->len > ds->reads[t->sup[id2] - 1].len)
            t->sup[id2] = (uint32_t)i;
        }
      }
    }
  }
  return NULL;
}

static void* discover_chunks(void* arg) {
  mgo_task* t = (mgo_task*)arg;
  mgo_dataset* ds = t->ds;
  uint64_t h = t->h, N = ds->n_unique;
  for (;;) {
    uint64_t a = __atomic_fetch_add(t->next, t->chunk, __ATOMIC_RELAXED) + 1;
    if (a > N) break;
    uint64_t e = a + t->chunk > N + 1 ? N + 1 : a + t->chunk;
    for (uint64_t i = a; i < e; i++) {
      oread* r1 = &ds->reads[i - 1];
      uint64_t n1 = r1->len;
      for (uint64_t j = 1; j < n1 - h; j++) {
        struct bucket* b = find_bucket(ds, r1->fwd + j, 0);
        if (!b) continue;
        for (uint32_t k = 0; k < b->n; k++) {
          uint64_t data = b->items[k];
          uint64_t id2 = data & 0x3FFFFFFFFFFFFFFFULL, o = data >> 62;
          if (id2 < i) continue; /* explored (:546) */
          oread* r2 = &ds->reads[id2 - 1];
          if (t->super[i] == 0 && t->super[id2] == 0 && overlap_check(r1, r2, o, j, h)) {
            uint8_t orient;
            uint16_t ovl;
            switch (o) { /* :550-556 */
              case 0: orient = 3; ovl = (uint16_t)(n1 - j); break;
              case 1: orient = 0; ovl = (uint16_t)(h + j); break;
              case 2: orient = 2; ovl = (uint16_t)(n1 - j); break;
              default: orient = 1; ovl = (uint16_t)(h + j); break;
            }
            uint16_t off = (uint16_t)(n1 - ovl);               /* :557 */
            uint16_t off_rev = (uint16_t)(r2->len + off - n1); /* :410 */
            mgo_digest_add(&t->d, mgo_row_hash(i, id2, orient, off));
            mgo_digest_add(&t->d, mgo_row_hash(id2, i, twin_orient(orient), off_rev));
          }
        }
      }
    }
  }
  return NULL;
}

int mgo_overlaps_digest(mgo_dataset* ds, uint64_t min_overlap, int nthreads, uint64_t* rows_out,
                        uint64_t* super_digest_out, uint64_t* super_out, double* t_hash, double* t_contain,
                        double* t_disc) {
  if (min_overlap < 2 || nthreads < 1) return -1;
  uint64_t N = ds->n_unique, h = min_overlap - 1;
  double t0 = now_s();
  build_table(ds, min_overlap);
  double t1 = now_s();
  uint64_t* super = (uint64_t*)calloc(N + 1, sizeof(uint64_t));
  pthread_t* th = (pthread_t*)calloc((size_t)nthreads, sizeof(pthread_t));
  mgo_task* tk = (mgo_task*)calloc((size_t)nthreads, sizeof(mgo_task));
  if (N && ds->longest != ds->shortest) { /* :228-233 */
    for (int t = 0; t < nthreads; t++) {
      tk[t].ds = ds;
      tk[t].h = h;
      tk[t].lo = 1 + N * (uint64_t)t / (uint64_t)nthreads;
      tk[t].hi = 1 + N * (uint64_t)(t + 1) / (uint64_t)nthreads;
      tk[t].sup = (uint32_t*)calloc(N + 1, sizeof(uint32_t));
      pthread_create(&th[t], NULL, contain_range, &tk[t]);
    }
    for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
    for (int t = 0; t < nthreads; t++) { /* fold in source order, rule of :259-268 */
      for (uint64_t id = 1; id <= N; id++) {
        uint64_t s = tk[t].sup[id];
        if (!s) continue;
        if (super[id] == 0 || ds->reads[s - 1].len > ds->reads[super[id] - 1].len) super[id] = s;
      }
      free(tk[t].sup);
    }
  }
  double t2 = now_s();
  uint64_t next = 0;
  memset(tk, 0, (size_t)nthreads * sizeof(mgo_task));
  for (int t = 0; t < nthreads; t++) {
    tk[t].ds = ds;
    tk[t].h = h;
    tk[t].super = super;
    tk[t].next = &next;
    tk[t].chunk = 4096;
    pthread_create(&th[t], NULL, discover_chunks, &tk[t]);
  }
  mgo_digest d = {0, 0, 0, 0};
  for (int t = 0; t < nthreads; t++) {
    pthread_join(th[t], NULL);
    d.n += tk[t].d.n;
    d.sum += tk[t].d.sum;
    d.xr ^= tk[t].d.xr;
    d.sum2 += tk[t].d.sum2;
  }
  double t3 = now_s();
  rows_out[0] = d.n;
  rows_out[1] = d.sum;
  rows_out[2] = d.xr;
  rows_out[3] = d.sum2;
  mgo_super_digest(super, N, super_digest_out);
  if (super_out) memcpy(super_out, super, (N + 1) * sizeof(uint64_t));
  free(super);
  free(th);
  free(tk);
  if (t_hash) *t_hash = t1 - t0;
  if (t_contain) *t_contain = t2 - t1;
  if (t_disc) *t_disc = t3 - t2;
  return 0;
}

/* Digests of oracle/mg_digest.h over rows / a superReadID vector (the
 * checker's side of mg_rows_digest / mg_super_digest). */
void mgo_rows_digest(const mgo_row* rows, uint64_t n, uint64_t* out) {
  mgo_digest d = {0, 0, 0, 0};
  for (uint64_t i = 0; i < n; i++) mgo_digest_add(&d, mgo_row_hash(rows[i].src, rows[i].dst, rows[i].orient, rows[i].offset));
  out[0] = d.n;
  out[1] = d.sum;
  out[2] = d.xr;
  out[3] = d.sum2;
}

void mgo_super_digest(const uint64_t* super, uint64_t n_unique, uint64_t* out) {
  mgo_digest d = {0, 0, 0, 0};
  for (uint64_t i = 1; i <= n_unique; i++)
    if (super[i]) mgo_digest_add(&d, mgo_super_hash(i, super[i]));
  out[0] = d.n;
  out[1] = d.sum;
  out[2] = d.xr;
  out[3] = d.sum2;
}
