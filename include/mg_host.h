/* mg_host.h — C-ABI over the host-side Dataset mirror (metagenomics_amd/csrc/host).
 *
 * The host Dataset mirror (the device version is mg_ingest_* in mg_overlap.h)
 * is the reference's Dataset semantics restated in C++ with packed reads:
 *   readDataset  Dataset.cpp:110-193  (FASTA/FASTQ parse, upper-case)
 *   testRead     Dataset.cpp:398-413  (only ACGT, no base >= floor(0.8 len))
 *   canonical    Dataset.cpp:163-167  (store min(s, revcomp(s)))
 *   sortReads    Dataset.cpp:197-202  (std::string order)
 *   removeDupicateReads Dataset.cpp:316-345 (frequency, IDs 1..N)
 * The result is handed to the device through mg_upload_reads_packed().
 */
#ifndef MG_HOST_H_
#define MG_HOST_H_
#include <stdint.h>

#include "mg_overlap.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct mgh_dataset mgh_dataset;

/* Dataset(pe, se, minOverlap) (Dataset.cpp:39-65).  Returns 0 on success,
 * -1 on an unreadable file, -2 on an unknown format (first byte not '>'/'@'). */
int mgh_dataset_from_files(const char* const* files, int nfiles, uint64_t min_overlap, mgh_dataset** out);
/* Same pipeline from in-memory reads: codes[i*stride + k] in {0:A,1:C,2:G,3:T,
 * anything else = not ACGT} for k < lens[i].  nthreads <= 0: hardware threads. */
int mgh_dataset_from_codes(const uint8_t* codes, uint64_t n, uint64_t stride, const uint16_t* lens,
                           uint64_t min_overlap, int nthreads, mgh_dataset** out);
void mgh_dataset_free(mgh_dataset* ds);

uint64_t mgh_num_reads(const mgh_dataset* ds);   /* Dataset::getNumberOfReads (good reads) */
uint64_t mgh_num_unique(const mgh_dataset* ds);  /* Dataset::getNumberOfUniqueReads */
uint64_t mgh_shortest(const mgh_dataset* ds);    /* Dataset::shortestReadLength */
uint64_t mgh_longest(const mgh_dataset* ds);     /* Dataset::longestReadLength */
/* Zero-copy views of the packed unique reads in ID order (ID = index + 1). */
int mgh_packed(const mgh_dataset* ds, const uint64_t** words, const uint16_t** lens, uint32_t* words_per_read);
/* Read::getStringForward() of read `id` into buf (NUL-terminated); returns its
 * length, or -1 if id is out of range (Dataset.cpp:484-490). */
int64_t mgh_read_string(const mgh_dataset* ds, uint64_t id, char* buf, uint64_t cap);
uint32_t mgh_frequency(const mgh_dataset* ds, uint64_t id); /* Read::getFrequency */
/* Dataset::getReadFromString (Dataset.cpp:421-455): ID of a read given either
 * strand, 0 if absent. */
uint64_t mgh_find_read(const mgh_dataset* ds, const char* s, uint64_t len);

/* --- HashTable API values (no device counterpart) --------------------------------
 * HashTable::getHashTableSize() after insertDataset: the first entry of the
 * reference's prime table greater than 8 N + 1 (getPrimeLargerThanNumber,
 * HashTable.cpp:20-29,56); N = unique reads.  HashTable::hashFunction(key)
 * (HashTable.cpp:135-155) for a table of `table_size` entries.  The device
 * index does not use either: its exact-key buckets do not depend on the hash
 * (SURVEY §8(a) a8). */
uint64_t mgh_hash_table_size(uint64_t n_unique);
uint64_t mgh_hash_function(const char* key, uint64_t len, uint64_t table_size);

/* --- record splitting -------------------------------------
 * Dataset::readDataset's record splitting (Dataset.cpp:110-193) on a
 * memory-mapped file with nthreads host threads (<= 0: all): FASTA = header
 * line, then everything up to the next '>' with '\n' removed; FASTQ = the 2nd
 * of every 4 lines.  Record i's raw sequence (bytes as in the file, before
 * upper-casing / testRead) is text[off[i] .. off[i+1]); n_records + 1 offsets.
 * The outputs are malloc'ed: release with mgh_parse_free.  They are the input
 * mg_ingest_ascii (include/mg_overlap.h) takes.  0 = ok, -1 = cannot open,
 * -2 = unknown format (first byte not '>' / '@'), -3 = out of memory. */
int mgh_parse_file(const char* path, int nthreads, char** text, uint64_t** offsets, uint64_t* n_records,
                   double* seconds);
/* several files, concatenated in order (Dataset.cpp:52-60 reads paired-end files first) */
int mgh_parse_files(const char* const* paths, int nfiles, int nthreads, char** text, uint64_t** offsets,
                    uint64_t* n_records, double* seconds);
int mgh_parse_buffer(const char* buf, uint64_t n, int nthreads, char** text, uint64_t** offsets,
                     uint64_t* n_records, double* seconds);
void mgh_parse_free(void* p);
/* smallest chunk one thread splits (default 1 MiB; 0 restores it) */
void mgh_parse_set_min_chunk(uint64_t bytes);

/* --- multi-process rendezvous (exchange mode over RCCL) ---------
 * Rank 0 serves the n-byte blob (the RCCL unique id) to the world - 1 other
 * ranks over TCP at addr:port; the others receive it into blob.  addr is a
 * dotted address or a host name (torchrun's MASTER_ADDR, e.g. "localhost").
 * Every wait is bounded by timeout_ms (<= 0: 10 minutes).  0 = ok, -1 bad
 * arguments, -2 addr does not resolve, -3 cannot listen (rank 0), -4 deadline
 * passed (a peer never connected / rank 0 never reachable), -5 I/O error.
 * Replaces torch.distributed's store for the C++ host (mg_overlap -xchg). */
int mgh_rendezvous(int rank, int world, const char* addr, int port, void* blob, uint64_t n, int timeout_ms);

/* --- graph construction order ----------------------------
 * Replays OverlapGraph::buildOverlapGraphFromHashTable's exploration and
 * transitive reduction (OverlapGraph.cpp:144-204, 574-661) on the device's
 * discovery multiset (mg_find_overlaps + mg_copy_rows, or the rows of every
 * rank in exchange mode): the resulting graph[u] lists, in list order, and the
 * numberOfNodes / numberOfEdges counters are the reference's just before its
 * contraction loop (:211-215).  lens[id - 1] = read lengths, h = l - 1. */
typedef struct mgh_graph mgh_graph;
/* 0 = ok; -1 bad arguments; -2 rows inconsistent with lens / h; -3 unpaired self rows */
int mgh_graph_replay(const mg_edge* rows, uint64_t n_rows, const uint16_t* lens, uint64_t n_reads, uint32_t h,
                     mgh_graph** out);
/* OverlapGraph::readGraphFromFile (OverlapGraph.cpp:1270-1367): a .unitig
 * checkpoint back into a graph (both edges of every record, twins rebuilt,
 * read locations updated); lens[id - 1] of the Dataset it was written for.
 * The handle then behaves as a contracted one (sort_edges, save_unitig,
 * save_lists, unitig_edges).  0 ok; -1 cannot open; -2 malformed or a read ID
 * out of range; -3 bad arguments. */
int mgh_graph_read_unitig(const char* path, const uint16_t* lens, uint64_t n_reads, mgh_graph** out);
void mgh_graph_free(mgh_graph* g);
uint64_t mgh_graph_nodes(const mgh_graph* g); /* OverlapGraph::getNumberOfNodes */
uint64_t mgh_graph_edges(const mgh_graph* g); /* OverlapGraph::getNumberOfEdges (directed) */
/* All lists concatenated in u order, each in list order (n_out = edges).
 * Returns the number of rows written (<= cap); cap = 0 returns the count. */
uint64_t mgh_graph_rows(const mgh_graph* g, mg_edge* out, uint64_t cap);

/* --- unitig contraction + .unitig checkpoint -------------
 * Runs the loop that ends new OverlapGraph(ht) (OverlapGraph.cpp:211-215):
 *   do { contractCompositePaths() :669-696; removeDeadEndNodes() :931-988 }
 *   while (anything merged or removed)
 * on the replayed graph, with the reference's mergeEdges / mergeList /
 * removeEdge list surgery and (track_locations != 0) the per-read location
 * lists of updateReadLocations / removeReadLocations (:1048-1115).  After it,
 * mgh_graph_nodes / mgh_graph_edges are the reference's counters after the
 * loop and mgh_graph_rows returns 0 (offsets of composite edges exceed 16 bits:
 * use mgh_graph_unitig_edges).  0 = ok; -1 bad handle / already contracted;
 * -4 an orientation pair mergedEdgeOrientation rejects (:830-833 MYEXIT). */
int mgh_graph_contract(mgh_graph* g, int track_locations, uint64_t* iterations, uint64_t* merged,
                       uint64_t* dead_end_nodes);
/* sortEdges (:2799-2808): every list sorted by destination ID (std::sort). */
int mgh_graph_sort_edges(mgh_graph* g);
/* saveGraphToFile (:1219-1261): the .unitig checkpoint of the current graph
 * (main.cpp:49-50 calls it after sortEdges).  0 = ok, -1 = open/write error. */
int mgh_graph_save_unitig(const mgh_graph* g, const char* path);
/* every list in list order as "u v orient offset nreads r:o:d ..." rows, then
 * the read location lists as "F|R read src dst orient offset location" rows
 * (the parity dump of oracle/ref_harness unitig). */
int mgh_graph_save_lists(const mgh_graph* g, const char* path);
typedef struct mgh_unitig_edge {
  uint32_t src, dst;  /* getSourceRead / getDestinationRead IDs */
  uint64_t offset;    /* getOverlapOffset (UINT64) */
  uint32_t n_reads;   /* getListOfReads()->size() */
  uint8_t orient;     /* getOrientation */
  uint8_t pad[3];
} mgh_unitig_edge;
/* contracted lists concatenated in u order, each in list order; the reads of
 * edge k are reads[read_start[k] .. read_start[k] + n_reads) (with their
 * listOfOverlapOffsets / listOfOrientations entries in offs / ors).  Any
 * output may be NULL.  Returns the number of edges; *n_reads_total the
 * length of reads/offs/ors.  Edges beyond edge_cap or reads beyond read_cap
 * are not written. */
uint64_t mgh_graph_unitig_edges(const mgh_graph* g, mgh_unitig_edge* edges, uint64_t edge_cap,
                                uint64_t* read_start, uint32_t* reads, uint16_t* offs, uint8_t* ors,
                                uint64_t read_cap, uint64_t* n_reads_total);

#ifdef __cplusplus
}
#endif
#endif /* MG_HOST_H_ */
