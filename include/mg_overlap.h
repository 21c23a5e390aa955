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
  float index_ms;       /* HashTable::insertDataset equivalent (with the window scan when fused) */
  float contained_ms;   /* markContainedReads equivalent (0 if skipped) */
  float overlap_ms;     /* discovery = scan + probe (insertAllEdgesOfRead) */
  float total_ms;       /* device wall of index + contained + overlap */
  float scan_ms;        /* minimizer-run scan kernel (unsharded: the index-building scan, part of index_ms) */
  float probe_ms;       /* probe kernel (fused path: probe + verify) */
  float verify_ms;      /* 0 (the probe verifies inline)                */
  float upload_ms;      /* H2D copy of raw reads (mg_ingest_*)        */
  float ingest_ms;      /* device Dataset ingest (mg_ingest_*)        */
  float sort_ms;        /* always 0 (no run sort since the clustered layout; field kept for ABI) */
  float layout_ms;      /* device layout of the last upload / ingest (clustered slots, option "layout") */
} mg_timings;

/* Work counters of the last discovery launch (only with option "stats" = 1):
 * the units the roofline's algorithmic byte count is built from. */
typedef struct mg_counters {
  uint64_t sources;   /* source reads handled                         */
  uint64_t runs;      /* minimizer runs whose bucket was probed       */
  uint64_t entries;   /* bucket entries scanned                       */
  uint64_t verified;  /* partner reads fetched and compared           */
  uint64_t rows;      /* directed rows emitted                        */
  uint64_t live_cells; /* cells of the discovery index of uncontained reads the probe
                          walked (option live_index); 0 = the full table */
  /* the last containment pass (markContainedReads), same units */
  uint64_t c_runs, c_entries, c_verified, c_contained;
  /* run records the last window scan wrote (every source read's windows; kept
   * without option "stats") */
  uint64_t scan_runs;
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
 * lens[i] = Read::getReadLength() of read ID i+1 (Read.h:62).  Any length up to
 * 65,535 (UINT16): reads up to 1,024 bp take the register-resident kernels,
 * longer ones the long-read kernels (the exchange mode refuses
 * them).  The same holds for every upload and ingest below. */
int mg_upload_reads_packed(mg_ctx* ctx, const uint64_t* words, const uint16_t* lens, uint64_t n_reads,
                           uint32_t words_per_read);
/* Upload reads as ASCII (upper-case ACGT only, already filtered by
 * Dataset::testRead, Dataset.cpp:398-413): concat holds read i at
 * [offsets[i], offsets[i+1]).  The 2-bit encoding runs on the GPU
 * (replaces Read::setRead's string storage, Read.cpp:75-82). */
int mg_upload_reads_ascii(mg_ctx* ctx, const char* concat, const uint64_t* offsets, uint64_t n_reads);
uint64_t mg_num_reads(const mg_ctx* ctx);
/* Dataset ingest ON THE DEVICE: raw reads in, the unique
 * canonical reads in ID order out, resident in the context exactly as
 * mg_upload_reads_packed would leave them.  Restates Dataset::Dataset's
 * per-read path (Dataset.cpp:39-65): upper-case (:158-159), testRead (length >
 * min_overlap, only ACGT, no base >= floor(0.8 len); :160, :398-413),
 * canonical strand min(s, revcomp(s)) (:163-167), sortReads in std::string
 * order (:197-202) and removeDupicateReads (frequency, IDs 1..N; :316-345).
 * ASCII: read i = concat[offsets[i], offsets[i+1]) (FASTA/FASTQ record text as
 * readDataset extracts it, Dataset.cpp:123-182); codes: codes[i*stride + k]
 * in {0:A,1:C,2:G,3:T, >3: not ACGT}, k < lens[i].  *n_unique = unique reads. */
int mg_ingest_ascii(mg_ctx* ctx, const char* concat, const uint64_t* offsets, uint64_t n_raw, uint32_t min_overlap,
                    uint64_t* n_unique);
int mg_ingest_codes(mg_ctx* ctx, const uint8_t* codes, uint64_t n_raw, uint64_t stride, const uint16_t* lens,
                    uint32_t min_overlap, uint64_t* n_unique);
/* Dataset::getNumberOfReads (reads that passed testRead) and
 * getNumberOfUniqueReads of the last device ingest. */
int mg_dataset_counts(const mg_ctx* ctx, uint64_t* n_good, uint64_t* n_unique);
/* Read::getFrequency of every unique read (n_reads entries, ID order). */
int mg_download_frequency(mg_ctx* ctx, uint32_t* freq);
/* Copy back the packed reads (words_per_read words each) for inspection. */
int mg_download_reads_packed(mg_ctx* ctx, uint64_t* words, uint16_t* lens, uint32_t* words_per_read);
/* Device slot of every read: slot_of_id[ID - 1] (the device stores the reads
 * clustered for locality, option "layout"; identity when it is off).  Only
 * diagnostics need it: every result leaves the device in reference IDs. */
int mg_read_slots(mg_ctx* ctx, uint32_t* slot_of_id);

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
/* Rows held by the context after the last mg_find_overlaps / mg_xchg_probe(0)
 * (the count mg_copy_rows copies and mg_rows_digest(rows = NULL) digests). */
uint64_t mg_num_rows(const mg_ctx* ctx);

/* --- sharding (multi-GPU, one process per GPU) ---------------------------- */
/* Restrict this context to index buckets owned by `rank` of `nranks`
 * (bucket-range sharding) and/or to the source reads with
 * reference IDs in [read_lo + 1, read_hi] (0-based range; read_hi = 0 means
 * all): every row this context produces then has its `src` in that range or
 * is the twin of such a row, so each rank holds the discoveries of its reads
 * (insertAllEdgesOfRead of its sources, OverlapGraph.cpp:529-565).  The union
 * over ranks is the whole multiset.  With the clustered slot layout the
 * range's reads are re-clustered into slots [read_lo, read_hi) at the next
 * mg_build_index.  A bucket range over every source (rank, nranks, 0, 0) with
 * one read length is the bucket mode (bench --multi bucket): mg_build_index's
 * one window scan reads every read, files the keys and keeps the runs of the
 * rank's buckets only, and mg_find_overlaps finds all of their discoveries. */
int mg_set_shard(mg_ctx* ctx, uint32_t rank, uint32_t nranks, uint64_t read_lo, uint64_t read_hi);

/* --- exchange mode: one process per GPU, SURVEY §8(e) ------------------------
 * Rank r of P (mg_set_shard(ctx, r, P, 0, 0)) owns the index buckets b with
 * floor(b P / 2^nb) == r and the source reads (IDs - 1) in
 * [floor(r N / P), floor((r+1) N / P)); every rank holds all packed reads.
 *
 * SLOT LAYOUT.  Records travel between ranks in caller-owned device buffers of
 * rounds * P * slot records (slot a multiple of 64).  The records a rank sends
 * to peer d -- or receives from peer s -- form one stream whose i-th record
 * sits at
 *     ((i / slot) * P + d) * slot + i % slot,      i < rounds * slot,
 * so round t of every peer is the contiguous block [t P slot, (t+1) P slot):
 * one equal-split all-to-all per round moves it (no split sizes on the host),
 * and one more moves the P per-peer counts (uint64 device arrays).  A stream
 * longer than rounds * slot is cut there but its count keeps the full length:
 * the caller reads the counts once at the end of the step (MAX over ranks),
 * and on an overflow grows the capacity and reruns the step.  Capacities must
 * be the same on every rank; mg_xchg_caps gives first estimates from global
 * quantities only.  Every call below only enqueues work on the context's
 * stream except mg_xchg_begin (one sync: the run count) and mg_xchg_probe(0)
 * (one sync: the row count); a caller that runs its collectives on the same
 * stream (metagenomics_amd/sharded.py) never waits on the host in between.
 *
 * One step (HashTable::insertDataset + OverlapGraph markContainedReads +
 * insertAllEdgesOfRead, distributed):
 *   mg_xchg_begin                 one window scan of this rank's sources: their
 *                                 index keys + minimizer runs (in scan order);
 *                                 keys first (mg_xchg_keys_first): the keys only
 *   mg_xchg_pack(MG_KEYS) -> a2a -> mg_xchg_insert_keys        (insertDataset;
 *                                 keys first: the window scan runs here)
 *   mg_xchg_pack(MG_RUNS) -> a2a   (the received runs serve both probes;
 *                                 one length: mg_xchg_probe_own meanwhile)
 *   mg_begin_contained(superkey)
 *   [lengths differ: (mg_xchg_prefix_marks -> all-reduce MAX of the marks)
 *                    mg_xchg_probe(1) -> all-reduce MAX of superkey]
 *   mg_finalize_contained                                       (markContainedReads)
 *   mg_xchg_probe(0) -> mg_xchg_pack(MG_ROWS) -> a2a             (insertAllEdgesOfRead)
 * and every rank ends with the rows whose src it owns (or, when the host skips
 * the last pack, with the rows it verified: the union over the ranks is the
 * same multiset).  Record sizes, mg_record_bytes(): keys 8 B (the index entry:
 * read slot | o | q | fingerprint | length), runs 8 B (the run meta: read slot
 * | minimizer position p | window range); the receiver recomputes the bucket
 * and fingerprint by hashing the minimizer m-mer of its own copy of the read
 * (every rank holds all reads), so they never travel; rows 12 B (mg_edge). */
enum { MG_KEYS = 0, MG_RUNS = 1, MG_ROWS = 2 };
uint32_t mg_record_bytes(int what);
/* First per-peer stream capacities (records) for keys, runs and rows:
 * caps[3], identical on every rank (global read count and lengths only). */
int mg_xchg_caps(mg_ctx* ctx, uint32_t min_overlap, uint32_t seed_k, uint64_t* caps);
/* Set up this rank's part of the index, then one scan of its source reads:
 * the index keys (hashRead, HashTable.cpp:88-104; the o = 1 key only when the
 * containment probe reads it) and the windows' minimizer runs
 * (OverlapGraph.cpp:534-537), in the scan's order. */
int mg_xchg_begin(mg_ctx* ctx, uint32_t min_overlap, uint32_t seed_k);
/* 1 when the current exchange build is KEYS FIRST (option xchg_keys_first,
 * default: several ranks and reads of one length): mg_xchg_begin then made the
 * key records only, and the window scan runs inside mg_xchg_insert_keys, which
 * CAS-inserts the received key records as it goes (k_scan<RECV>: no sort, no
 * separate cell build); MG_RUNS can be packed only after mg_xchg_insert_keys.
 * 0: one scan in mg_xchg_begin made keys and runs (MG_RUNS packable at once). */
int mg_xchg_keys_first(const mg_ctx* ctx);
/* Route what = MG_KEYS / MG_RUNS (after mg_xchg_begin) or MG_ROWS (after
 * mg_xchg_probe(0)) into dst in the slot layout; counts = P device uint64.
 * With one rank (P = 1) every stream is the rank's own: nothing is copied and
 * counts[0] = 0; mg_xchg_insert_keys and mg_xchg_probe then read the
 * context's own key records and run regions (recv / counts ignored), and the
 * rows stay in the context (mg_num_rows, mg_rows_digest, mg_copy_rows).
 * self_dst (optional): the stream bound for this rank itself is written there
 * instead -- the caller's receive buffer, whose slots for this rank sit at the
 * same offsets -- so it never travels (the all-to-all then moves only the
 * other peers' slots; dst may be NULL when P == 1). */
int mg_xchg_pack(mg_ctx* ctx, int what, void* dst, uint64_t slot, uint32_t rounds, uint64_t* counts,
                 void* self_dst);
/* File the received key records into the local cells (insertIntoTable,
 * HashTable.cpp:163-195); recv / counts as the all-to-all delivered them.  The
 * records are sorted by home cell and stored without atomics (a cell's 9th+
 * entries chain on); one host read of the counts.  Keys first
 * (mg_xchg_keys_first): the rank's window scan runs here instead and
 * CAS-inserts the received records between its windows, leaving the runs
 * (OverlapGraph.cpp:534-537) for mg_xchg_pack(MG_RUNS). */
int mg_xchg_insert_keys(mg_ctx* ctx, const void* recv, uint64_t slot, uint32_t rounds, const uint64_t* counts);
/* Probe the received runs against the local cells: contain = 1 atomicMax-es
 * containment keys into the buffer of mg_begin_contained; contain = 0 verifies
 * overlaps (sources with superReadID != 0 give none) and keeps the rows
 * (+ twins) for mg_xchg_pack(MG_ROWS).  The probes read the runs in place in
 * recv (pass the same recv / counts to both calls of a step); contain = 0
 * first compacts away, in place, the runs of contained sources, so recv is
 * the library's scratch until the step ends.  (Option xchg_sort_runs = 1: the
 * first call orders them by bucket into the context's own array instead.) */
int mg_xchg_probe(mg_ctx* ctx, int contain, const void* recv, uint64_t slot, uint32_t rounds, const uint64_t* counts);
/* Optional, after mg_finalize_contained and before mg_xchg_probe(0): the
 * discovery probe (insertAllEdgesOfRead's window loop + checkOverlap,
 * OverlapGraph.cpp:529-565, 354-383) of this rank's OWN run stream, which mg_xchg_pack(MG_RUNS)
 * wrote straight into recv (send_counts = that pack's counts; only this
 * rank's entry is read), so it runs while the peers' streams are still on the
 * links; mg_xchg_probe(0) then probes the peers' streams and appends its rows.
 * Same rows as one mg_xchg_probe(0).  A no-op (everything is left to
 * mg_xchg_probe(0)) with one rank, mixed lengths (the containment probe needs
 * every stream first) or option xchg_sort_runs. */
int mg_xchg_probe_own(mg_ctx* ctx, const void* recv, uint64_t slot, uint32_t rounds, const uint64_t* send_counts);
/* Containment: *needed = 1 when read lengths differ (OverlapGraph.cpp:228-233).
 * superkey = caller-owned device array of n_reads u64 (NULL: context-owned),
 * cleared here; the contain probe atomicMax-es (len << 32 | ~index) into it,
 * the host all-reduces it with MAX over the ranks, and mg_finalize_contained
 * turns it into superReadID (super_out optional, n_reads + 1 entries). */
int mg_begin_contained(mg_ctx* ctx, void* superkey, int* needed);
/* Optional, between mg_begin_contained and mg_xchg_probe(1) (lengths differ):
 * run this rank's offset-0 containments (checkOverlapForContainedRead at s = 0,
 * OverlapGraph.cpp:302-340, over the o = 0 key records it received) now and
 * write marks[i] = 1 for every read they found contained (n_reads bytes,
 * device; NULL: no marks).  The caller all-reduces marks with MAX over the
 * ranks on the context's stream; mg_xchg_probe(1) then folds them into the
 * key array, so that its contained-source skip (contain_skip) sees every
 * rank's offset-0 containments, not only this rank's.  marks stays the
 * caller's and must stay valid until mg_xchg_probe(1) is enqueued. */
int mg_xchg_prefix_marks(mg_ctx* ctx, void* marks);
int mg_finalize_contained(mg_ctx* ctx, uint32_t* super_out);

/* --- parity digests (no reference counterpart: test/bench support) ----------
 * Order-independent digests of the directed edge multiset and of the
 * superReadID vector, computed on the device, so that a 10^8-row result is
 * compared with the reference's (oracle/_ref/ref_harness digest) without a
 * multi-GB download.  out[4] = {count, sum h, xor h, sum mix64(h ^ SALT)}
 * mod 2^64, with mix64 the bijective finaliser (x ^= x>>31; x *= 0x7fb5d329728ea185;
 * x ^= x>>27; x *= 0x81dadef4bc2dd44d; x ^= x>>33), SALT = 0xD6E8FEB86659FD93 and
 *   row (u, v, orient, offset): h = mix64(((u << 32) | v) ^ mix64(((orient << 16) | offset)
 *                                   + 0x9E3779B97F4A7C15))
 *   contained read id:          h = mix64((id << 32) | superReadID)
 * Digests of disjoint parts combine by adding count/sum/sum2 and xor-ing xor.
 * mg_rows_digest: rows = NULL digests the context's rows of the last
 * mg_find_overlaps / mg_xchg_probe; else `rows` is a device array of n_rows
 * mg_edge records.  mg_slots_digest: rows received in the slot layout of the
 * exchange mode (counts = the P device uint64 per-peer counts). */
int mg_rows_digest(mg_ctx* ctx, const void* rows, uint64_t n_rows, uint64_t* out);
int mg_slots_digest(mg_ctx* ctx, const void* rows, uint64_t slot, uint32_t rounds, const uint64_t* counts,
                    uint64_t* out);
int mg_super_digest(mg_ctx* ctx, uint64_t* out);

/* --- diagnostics ----------------------------------------------------------- */
int mg_get_timings(const mg_ctx* ctx, mg_timings* t);
int mg_get_counters(const mg_ctx* ctx, mg_counters* c);
/* Options (results never depend on any of them):
 *  "nb_log2"        log2 directory buckets (0 = auto);
 *  "rows_cap"       initial row capacity (0 = auto);
 *  "stats"          1 = count work units (mg_get_counters) in the next launches;
 *  "layout"         1 = slots clustered by canonical global minimizer (default),
 *                   0 = ID order; takes effect at the next upload;
 *  "halving"        side of a self-symmetric o = 2/3 pair: 0 = parity-alternating
 *                   (default, even load over source IDs), 1 = lower ID;
 *  "prefix_contain" 1 = mixed-length sets find offset-0 containments with
 *                   k_prefix_contain and the containment probe skips suffix-key
 *                   hits (default); 0 = the probe verifies them itself;
 *  "contain_jcut", "contain_prune", "contain_skip"
 *                   containment pruning, all exact, default 1;
 *  "probe_share"    a discovery block's 4 wavefronts share its run regions (default 1);
 *  "probe_compact"  sparse run batches are compacted in the probe (default 1);
 *  "live_index"     mixed lengths: after mg_mark_contained the discovery probe
 *                   walks an index of the uncontained reads' keys only
 *                   (OverlapGraph.cpp:548; exact, default 1; the exchange mode
 *                   coarsens the rank's cells for it); with it, the full index
 *                   of a mixed-length set holds the o = 0 / 2 keys only;
 *  "xchg_sort_runs" exchange mode: order the received runs by bucket before
 *                   the probes (default 0: probed in place, arrival order);
 *  "xchg_keys_first" exchange mode, one read length, P > 1: key records first,
 *                   filed by CAS inside the receiver's window scan (default 1;
 *                   0: one scan makes keys and runs, the receiver sorts the keys);
 *  "xchg_scan_lds"  exchange mode, one read length: k_scan's LDS sliding minimum
 *                   (default 1) instead of the register scan;
 *  "xchg_split_max" mg_xchg_probe_own splits the discovery probe up to this many
 *                   ranks (default 4);
 *  "xchg_region"    records per probe region of the received runs (power of two,
 *                   default 512);
 *  "xchg_route_rows" exchange mode: the discovery probe counts its rows per src
 *                   owner for mg_xchg_pack(MG_ROWS) (default 1); 0 when the
 *                   host keeps the rows where they were verified;
 *  "xchg_windows"   exchange mode, mixed lengths: the scan takes length-ranked
 *                   windows of 256 reads (default 1);
 *  "layout_scratch" 0 = free the layout's double buffers after each layout
 *                   (many contexts on one device); default 1 keeps them;
 *  "cells_double"   1 = two cell tables: each build takes the one the previous
 *                   build cleared on the side stream and clears the table it
 *                   retires there (2x the cells' memory; measured slower: the
 *                   clear beside the scan slows the scan); 0 (default) = one
 *                   table, cleared at the start of each build;
 *  "chain_par"      sorted cell builds (exchange mode): records past their home
 *                   cell placed in parallel by their index in their fingerprint's
 *                   run (default 1); 0 = one thread walks each overflowing cell;
 *  "check_cells"    diagnostics: after each sorted cell build, walk every record
 *                   from its home and fail the call if one is not found;
 *  "xchg_fs"        diagnostics: fingerprint bits in the exchange sort key
 *                   (-1 = auto: what fills the sort's last 8-bit digit);
 *  "alloc_cap"      tests: a device allocation above this many bytes fails as
 *                   out of memory (0 = no cap); every failed allocation leaves
 *                   the buffer's name, its size and the HIP error in mg_last_error;
 *  "run_cap"        tests: initial run records per scan region (0 = sized from
 *                   the reads; overflowing regions are resized and rescanned);
 *  "phase_limit", "max_blocks"
 *                   diagnostics: stop the probe after a phase / cap its grid. */
int mg_set_option(mg_ctx* ctx, const char* name, int64_t value);
/* HIP stream the context launches on (hipStream_t as void*), for callers that
 * time or capture it themselves. */
void* mg_stream(mg_ctx* ctx);

#ifdef __cplusplus
}
#endif
#endif /* MG_OVERLAP_H_ */
