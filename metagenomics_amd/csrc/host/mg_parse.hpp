// mg_parse.hpp — INTERNAL: parallel FASTA/FASTQ record splitter with the
// reference's readDataset semantics (Dataset.cpp:110-193).  See mg_parse.cpp.
#ifndef MG_PARSE_HPP_
#define MG_PARSE_HPP_
#include <cstdint>
#include <string>
#include <vector>

namespace mg {

struct ParseStats {
  uint64_t bytes = 0;    // file size
  uint64_t records = 0;  // records split (good and bad)
  double seconds = 0;    // map + split + gather wall time
  int threads = 1;
};

// Records' raw sequences (bytes as in the file, '\n' removed), concatenated:
// record i is text[off[i] .. off[i + 1]).  malloc'ed; release() frees.
struct ParsedText {
  char* text = nullptr;
  uint64_t* off = nullptr;  // n_rec + 1 entries once n_rec > 0
  uint64_t n_text = 0, n_rec = 0;
  void release();
};

// Appends the file's records to `out`.  0 = ok, -1 = cannot open / map,
// -2 = first byte neither '>' nor '@' (the reference's "Unknown input file
// format.", Dataset.cpp:130-135), -3 = out of memory.
// nthreads <= 0: hardware threads.
int parse_file_parallel(const std::string& path, ParsedText& out, int nthreads, ParseStats* stats = nullptr);

// smallest chunk a thread gets (bytes; tests lower it to exercise the chunk seams)
extern uint64_t g_parse_min_chunk;

// The same on a buffer already in memory.
int parse_buffer_parallel(const char* buf, uint64_t n, ParsedText& out, int nthreads, ParseStats* stats = nullptr);

}  // namespace mg
#endif  // MG_PARSE_HPP_
