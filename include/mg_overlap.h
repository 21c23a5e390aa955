/* mg_overlap.h — the drop-in C-ABI for the read-overlap hot path on MI355X.
 *
 * The reference has no FFI: its boundary is the C++ class API that main.cpp
 * calls (main.cpp:45-47).  Each entry point below names the reference
 * interface it replaces (paths relative to /root/reference/MetaGenomics).
 * The host-side C++ mirror of those classes (metagenomics_amd/csrc/host/)
 * is implemented on top of these functions; INTEGRATION.md shows how a
 * maintainer wires them in.
 *
 * Conventions: plain pointers and sizes, int status (0 = ok,
 * <0 = error; never exit() across the ABI — the reference's MYEXIT calls
 * exit(0), Common.h:47), mg_last_error() for the message, all device buffers
 * owned by the context, one host thread per context, device chosen at create.
 *
 * Read model: reads are the Dataset's unique canonical forward strings in ID
 * order (ID = index + 1, Dataset.cpp:335-339), 2-bit packed A0 C1 G2 T3,
 * most-significant base first, `words_per_read` u64 words per read (bases
 * past the read's length are zero).
 */
#ifndef MG_OVERLAP_H_
#define MG_OVERLAP_H_
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct mg_ctx mg_ctx;

/* One directed row of the overlap graph, i.e. one Edge object
 * (Edge.h:18-29): source read ID, destination read ID, overlapOrientation
 * 0..3 (0 = u<-----<v, 1 = u<----->v, 2 = u>-----<v, 3 = u>----->v) and
 * overlapOffset (start of v relative to u).  12 bytes. */
typedef struct mg_edge {
  uint32_t src;
  uint32_t dst;
  uint16_t offset;
  uint8_t orient;
  uint8_t flags; /* 0 */
} mg_edge;

/* Device-side phase timings of the last call (HIP events on the context's
 * stream), milliseconds. */
typedef struct mg_timings {
  float pack_ms;        /* 2-bit encoding of ASCII reads            */
  float index_ms;       /* HashTable::insertDataset equivalent       */
  float contained_ms;   /* markContainedReads equivalent (0 if skipped) */
  float overlap_ms;     /* discovery = scan + probe (insertAllEdgesOfRead) */
  float total_ms;       /* index + contained + overlap               */
  float scan_ms;        /* minimizer-run scan kernel                 */
  float probe_ms;       /* probe + verify kernel                     */
} mg_timings;

/* Work counters of the last discovery launch (only with option "stats" = 1):
 * the units the roofline's algorithmic byte count is built from. */
typedef struct mg_counters {
  uint64_t sources;   /* source reads handled                         */
  uint64_t runs;      /* minimizer runs whose bucket was probed       */
  uint64_t entries;   /* bucket entries scanned                       */
  uint64_t verified;  /* partner reads fetched and compared           */
  uint64_t rows;      /* directed rows emitted                        */
} mg_counters;

/* --- context ------------------------------------------------------------ */
/* Creates a context on HIP device `device`.  Replaces nothing in the
 * reference (it is single-process); owns every device buffer below. */
int mg_create(mg_ctx** ctx, int device);
void mg_destroy(mg_ctx* ctx);
const char* mg_last_error(const mg_ctx* ctx);
/* Number of HIP devices visible (0 when no GPU). */
int mg_device_count(void);

/* --- reads (Dataset / Read) ---------------------------------------------- */
/* Upload the Dataset's unique reads, already 2-bit packed (the host mirror of
 * Dataset packs while it canonicalises/sorts, Dataset.cpp:158-202,316-345).
 * lens[i] = Read::getReadLength() of read ID i+1 (Read.h:62). */
int mg_upload_reads_packed(mg_ctx* ctx, const uint64_t* words, const uint16_t* lens, uint64_t n_reads,
                           uint32_t words_per_read);
/* Upload reads as ASCII (upper-case ACGT only, already filtered by
 * Dataset::testRead, Dataset.cpp:398-413): concat holds read i at
 * [offsets[i], offsets[i+1]).  The 2-bit encoding runs on the GPU
 * (replaces Read::setRead's string storage, Read.cpp:75-82). */
int mg_upload_reads_ascii(mg_ctx* ctx, const char* concat, const uint64_t* offsets, uint64_t n_reads);
uint64_t mg_num_reads(const mg_ctx* ctx);
/* Copy back the packed reads (words_per_read words each) for inspection. */
int mg_download_reads_packed(mg_ctx* ctx, uint64_t* words, uint16_t* lens, uint32_t* words_per_read);

/* --- index (HashTable) ---------------------------------------------------- */
/* HashTable::insertDataset(Dataset*, minOverlapLength) (HashTable.h:30,
 * HashTable.cpp:50-80): keys are the h = l-1 prefixes/suffixes of both
 * strands of every read (hashRead, HashTable.cpp:88-104).  The device index
 * files each key under its (seed_k)-mer minimizer (seed_k <= min(32, h);
 * 0 = min(31, h)); exact-key equality is re-established by verification, so
 * results equal the reference's exact-key buckets. */
int mg_build_index(mg_ctx* ctx, uint32_t min_overlap, uint32_t seed_k);
/* HashTable::getListOfReads(string) (HashTable.cpp:202-221): the exact-key
 * bucket of `key` (length h, ACGT), entries id | o << 62 in the reference's
 * list order (ID ascending, then o).  *n_out = list length (may exceed cap). */
int mg_lookup_key(mg_ctx* ctx, const char* key, uint32_t key_len, uint64_t* out, uint64_t cap,
                  uint64_t* n_out);

/* --- overlap discovery (OverlapGraph) ------------------------------------- */
/* markContainedReads (OverlapGraph.cpp:225-290).  Runs only when read lengths
 * differ (:228-233), as the reference does.  super_out (optional, n_reads+1
 * entries): superReadID per ID, 0 = not contained. */
int mg_mark_contained(mg_ctx* ctx, uint32_t* super_out);
/* The edge-discovery part of buildOverlapGraphFromHashTable
 * (OverlapGraph.cpp:144-204 via insertAllEdgesOfRead :529-565, checkOverlap
 * :354-383, insertEdge :407-419): produces the full directed multiset
 * (every Edge and its twin) on the device.  Calls mg_mark_contained first if
 * it has not run for the current index.  *n_rows = directed rows
 * (= 2 x insertEdge(Read*,...) calls). */
int mg_find_overlaps(mg_ctx* ctx, uint64_t* n_rows);
/* Copy the rows to the host (any order; the multiset is what the reference
 * defines).  cap in rows; returns rows copied via *n_copied. */
int mg_copy_rows(mg_ctx* ctx, mg_edge* out, uint64_t cap, uint64_t* n_copied);

/* --- sharding (multi-GPU, one process per GPU) ---------------------------- */
/* Restrict this context to index buckets owned by `rank` of `nranks`
 * (bucket-range sharding) and/or to source reads
 * [read_lo, read_hi) (0-based; read_hi = 0 means all).  Rows produced are
 * this shard's part of the multiset; the union over ranks is the whole. */
int mg_set_shard(mg_ctx* ctx, uint32_t rank, uint32_t nranks, uint64_t read_lo, uint64_t read_hi);

/* --- diagnostics ----------------------------------------------------------- */
int mg_get_timings(const mg_ctx* ctx, mg_timings* t);
int mg_get_counters(const mg_ctx* ctx, mg_counters* c);
/* Options: "nb_log2" (log2 directory buckets, 0 = auto), "rows_cap" (initial
 * row capacity, 0 = auto), "stats" (1 = count work units in the next launches). */
int mg_set_option(mg_ctx* ctx, const char* name, int64_t value);
/* HIP stream the context launches on (hipStream_t as void*), for callers that
 * time or capture it themselves. */
void* mg_stream(mg_ctx* ctx);

#ifdef __cplusplus
}
#endif
#endif /* MG_OVERLAP_H_ */
