/* mg_oracle.h — TEST INFRASTRUCTURE ONLY (oracle/).
 *
 * A single-threaded plain-C restatement of the reference's overlap hot path
 * (SURVEY §8(a) rows a1-a14), used ONLY as the checker by tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg.  The product
 * (metagenomics_amd/) never links, loads or calls it.
 *
 * Parity of this restatement is pinned against the compiled reference itself
 * (oracle/_ref/ref_harness, golden fixtures in tests/golden/).
 */
#ifndef MG_ORACLE_H_
#define MG_ORACLE_H_
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

typedef struct mgo_dataset mgo_dataset;

/* One directed row of the overlap graph: Edge(source, destination,
 * overlapOrientation, overlapOffset)  (Edge.h:18-29). */
typedef struct {
  uint32_t src, dst;
  uint16_t offset;
  uint8_t orient;
  uint8_t pad;
} mgo_row;

/* Dataset::Dataset(pe, se, minOverlap) (Dataset.cpp:39-65): parse every
 * FASTA/FASTQ file, filter (testRead), canonicalise, sort, dedup, IDs 1..N.
 * Returns NULL on an unreadable / unknown-format file. */
mgo_dataset* mgo_dataset_from_files(const char* const* files, int nfiles, uint64_t min_overlap);
/* Same pipeline from n raw sequences given as one concatenated buffer plus
 * n+1 offsets (no parsing; upper-casing, filter, canonicalise, sort, dedup). */
mgo_dataset* mgo_dataset_from_seqs(const char* concat, const uint64_t* offsets, uint64_t n,
                                   uint64_t min_overlap);
/* Same pipeline from 2-bit codes (0..3 = A C G T): read i is
 * codes[i * stride, i * stride + lens[i]). */
mgo_dataset* mgo_dataset_from_codes(const uint8_t* codes, uint64_t stride, const uint16_t* lens, uint64_t n,
                                    uint64_t min_overlap);
void mgo_dataset_free(mgo_dataset* ds);
uint64_t mgo_num_reads(const mgo_dataset* ds);         /* good reads incl. duplicates */
uint64_t mgo_num_unique(const mgo_dataset* ds);
/* canonical forward string of read id (1-based), NUL-terminated. */
const char* mgo_read(const mgo_dataset* ds, uint64_t id, uint32_t* len);
uint32_t mgo_frequency(const mgo_dataset* ds, uint64_t id);

/* The hot path: HashTable::insertDataset (HashTable.cpp:50-80) then
 * markContainedReads (OverlapGraph.cpp:225-290) and the ID-order discovery
 * loop over insertAllEdgesOfRead (OverlapGraph.cpp:529-565).
 * super_out: N+1 entries (super_out[id] = superReadID, 0 = not contained).
 * *rows: malloc'd directed multiset (both twins of every insertEdge call).
 * t_hash / t_disc (optional): wall seconds of the two phases. */
int mgo_overlaps(mgo_dataset* ds, uint64_t min_overlap, uint64_t* super_out, mgo_row** rows,
                 uint64_t* nrows, double* t_hash, double* t_disc);

/* The same hot path over `nthreads` threads, for workloads whose rows do not
 * fit in memory: the containment loop over source ranges folded in source
 * order, the ID-order discovery loop with "explored" = ID below the source
 * (exactly the explored set when read i is explored), rows digested
 * (mg_digest.h) instead of listed.  rows_digest[4] / super_digest[4] as
 * mgo_rows_digest / mgo_super_digest; super_out (optional) N+1 entries. */
int mgo_overlaps_digest(mgo_dataset* ds, uint64_t min_overlap, int nthreads, uint64_t* rows_digest,
                        uint64_t* super_digest, uint64_t* super_out, double* t_hash, double* t_contain,
                        double* t_disc);

/* HashTable::getListOfReads(key) (HashTable.cpp:202-221) on a table built by
 * insertDataset: writes up to cap entries id|o<<62 in reference list order,
 * returns the list length. */
uint64_t mgo_lookup(mgo_dataset* ds, uint64_t min_overlap, const char* key, uint64_t* out, uint64_t cap);

void mgo_free(void* p);

/* Order-independent digests (oracle/mg_digest.h): out[4] = {n, sum, xor, sum2}. */
void mgo_rows_digest(const mgo_row* rows, uint64_t n, uint64_t* out);
void mgo_super_digest(const uint64_t* super, uint64_t n_unique, uint64_t* out);

#ifdef __cplusplus
}
#endif
#endif
