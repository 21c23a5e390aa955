// mg_parse.cpp — parallel FASTA/FASTQ record splitter.
// Paths relative to /root/reference/MetaGenomics.
//
// Dataset::readDataset (Dataset.cpp:110-193) reads records with getline:
//   * the format is fixed by the first byte of the file: '>' FASTA, '@' FASTQ,
//     anything else "Unknown input file format." (:126-135);
//   * FASTA: the header line, then everything up to the next '>' (wherever it
//     sits) with every '\n' removed is the sequence (:138-145);
//   * FASTQ: four lines per record, the sequence is the second (:147-154).
// This file produces the same record sequence (bytes as in the file) from a
// memory-mapped file with all host threads, in two passes over fixed chunks:
//
// FASTQ — a byte belongs to a sequence iff its line index is 1 mod 4.  Pass 1
//   counts '\n' per chunk; the prefix sum gives the line index at every chunk
//   start, so each chunk then owns the lines that START inside it.
// FASTA — a two-state machine (HDR: inside a header line, SEQ: inside a
//   sequence).  HDR --'\n'--> SEQ; SEQ --'>'--> HDR closes a record; the file
//   starts in HDR.  After any '\n' the state is SEQ whatever it was, so a chunk
//   that contains a '\n' ends in HDR iff a '>' follows its last '\n'
//   (independent of its start state); a chunk without '\n' ends in HDR iff it
//   started in HDR or contains a '>'.  Chunk start states are composed
//   sequentially from that (one value per chunk), then every chunk is split
//   independently.
// Pass 1 sizes every chunk without knowing its start (FASTQ: bytes and records
// per residue of the local line index; FASTA: for either start state); a
// sequential sweep over one value per chunk resolves them; pass 2 writes every
// chunk straight into its final place in an uninitialised (malloc'ed) buffer:
// two reads of the file and one write of the sequences in all.  The result
// equals the reference's record sequence (tests/test_parse.py).
#include "mg_parse.hpp"

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <thread>

namespace mg {

uint64_t g_parse_min_chunk = 1 << 20;

namespace {

int threads_for(int want) {
  if (want > 0) return want;
  const unsigned h = std::thread::hardware_concurrency();
  return h ? (int)std::min(h, 64u) : 4;
}

template <typename F>
void run_chunks(uint64_t nchunks, int T, F&& fn) {
  if (T <= 1 || nchunks <= 1) {
    for (uint64_t c = 0; c < nchunks; ++c) fn(c);
    return;
  }
  std::atomic<uint64_t> next{0};
  std::vector<std::thread> th;
  const int nt = (int)std::min<uint64_t>((uint64_t)T, nchunks);
  th.reserve(nt);
  for (int t = 0; t < nt; ++t)
    th.emplace_back([&] {
      for (uint64_t c; (c = next.fetch_add(1)) < nchunks;) fn(c);
    });
  for (auto& x : th) x.join();
}

inline const char* find(const char* p, const char* e, char ch) {
  const void* r = std::memchr(p, ch, (size_t)(e - p));
  return r ? static_cast<const char*>(r) : e;
}

struct ChunkOut {
  // pass 1: FASTQ line statistics per residue of the local line index
  uint64_t nl = 0;                      // '\n' inside the chunk
  uint64_t fq_bytes[4] = {0, 0, 0, 0};  // bytes of the lines starting here, by local index mod 4
  uint64_t fq_recs[4] = {0, 0, 0, 0};
  bool lead_nl = false;                 // the chunk's first line start follows a '\n' inside it
  // pass 1: FASTA, for either start state
  bool has_nl = false, end_hdr = false, any_gt = false;
  uint64_t fa_bytes_rest = 0, fa_close_rest = 0;  // from the first '\n' on (state SEQ there)
  uint64_t fa_bytes_pre = 0, fa_close_pre = 0;    // before the first '\n' if the chunk starts in SEQ
  // resolved
  uint64_t line_base = 0;  // FASTQ: '\n' before the chunk start
  bool start_hdr = false;  // FASTA: state at the chunk start
  uint64_t bytes = 0, records = 0, text_base = 0, rec_base = 0;
};

// first line start in [b, e) and its index relative to line_base; false = none
inline bool first_line(const char* buf, uint64_t b, uint64_t e, const char** p, uint64_t* rel) {
  if (b == 0 || buf[b - 1] == '\n') {
    *p = buf + b;
    *rel = 0;
    return b < e;
  }
  const char* q = find(buf + b, buf + e, '\n');
  if (q == buf + e) return false;
  *p = q + 1;
  *rel = 1;
  return true;
}

// FASTQ pass 1: newline count + line bytes by local index residue
void fastq_stats(const char* buf, uint64_t n, uint64_t b, uint64_t e, ChunkOut& c) {
  const char* end = buf + n;
  const char* ce = buf + e;
  const char* p;
  uint64_t rel;
  if (!first_line(buf, b, e, &p, &rel)) {
    c.nl = (uint64_t)std::count(buf + b, ce, '\n');  // (0 here)
    return;
  }
  c.lead_nl = rel == 1;
  uint64_t nl = rel, k = 0;
  while (p < ce) {
    const char* q = find(p, end, '\n');
    c.fq_bytes[k & 3] += (uint64_t)(q - p);
    c.fq_recs[k & 3]++;
    if (q < ce) nl++;
    p = q + 1;
    k++;
  }
  c.nl = nl;
}

// FASTQ pass 2: the sequence lines starting in [b, e) (global index 1 mod 4)
template <typename Emit>
void fastq_lines(const char* buf, uint64_t n, uint64_t b, uint64_t e, uint64_t line_base, Emit&& emit) {
  const char* end = buf + n;
  const char* p;
  uint64_t rel;
  if (!first_line(buf, b, e, &p, &rel)) return;
  uint64_t idx = line_base + rel;
  // jump to the first sequence line, then every 4th line
  while (p < buf + e) {
    const char* q = find(p, end, '\n');
    if ((idx & 3) == 1) emit(p, (uint64_t)(q - p));
    p = q + 1;
    idx++;
  }
}

// FASTA: split [b, e) from state `hdr`; seq(ptr, len) for sequence bytes,
// close() at every '>' seen in SEQ (a record ends)
template <typename Seq, typename Close>
void fasta_split(const char* buf, uint64_t b, uint64_t e, bool hdr, Seq&& seq, Close&& close) {
  const char* p = buf + b;
  const char* end = buf + e;
  while (p < end) {
    if (hdr) {
      const char* q = find(p, end, '\n');
      if (q == end) return;
      p = q + 1;
      hdr = false;
    } else {
      const char* gt = find(p, end, '>');
      while (p < gt) {  // sequence bytes up to the '>' with '\n' removed
        const char* nl = find(p, gt, '\n');
        if (nl > p) seq(p, (uint64_t)(nl - p));
        p = nl < gt ? nl + 1 : gt;
      }
      if (gt == end) return;
      close();
      p = gt + 1;
      hdr = true;
    }
  }
}

// FASTA pass 1: end state and sizes for either start state
void fasta_stats(const char* buf, uint64_t b, uint64_t e, ChunkOut& c) {
  const char* cb = buf + b;
  const char* ce = buf + e;
  const char* first_nl = find(cb, ce, '\n');
  c.has_nl = first_nl != ce;
  if (!c.has_nl) {
    c.any_gt = find(cb, ce, '>') != ce;
  } else {
    // prefix [b, first_nl) from SEQ: bytes up to the first '>', which closes
    const char* gt = find(cb, first_nl, '>');
    c.fa_bytes_pre = (uint64_t)(gt - cb);
    c.fa_close_pre = gt != first_nl;
  }
  // from SEQ after the first '\n' (or nothing)
  bool hdr = false;
  uint64_t bytes = 0, closes = 0;
  if (c.has_nl) {
    const char* p = first_nl + 1;
    while (p < ce) {
      if (hdr) {
        const char* q = find(p, ce, '\n');
        if (q == ce) break;
        p = q + 1;
        hdr = false;
      } else {
        const char* g = find(p, ce, '>');
        while (p < g) {
          const char* nl = find(p, g, '\n');
          bytes += (uint64_t)(nl - p);
          p = nl < g ? nl + 1 : g;
        }
        if (g == ce) break;
        closes++;
        p = g + 1;
        hdr = true;
      }
    }
  }
  c.end_hdr = hdr;
  c.fa_bytes_rest = bytes;
  c.fa_close_rest = closes;
}

}  // namespace

void ParsedText::release() {
  std::free(text);
  std::free(off);
  text = nullptr;
  off = nullptr;
  n_text = n_rec = 0;
}

int parse_buffer_parallel(const char* buf, uint64_t n, ParsedText& out, int nthreads, ParseStats* stats) {
  const auto t0 = std::chrono::steady_clock::now();
  if (n == 0 || (buf[0] != '>' && buf[0] != '@')) return -2;
  const bool fastq = buf[0] == '@';
  const int T = threads_for(nthreads);
  const uint64_t min_chunk = std::max<uint64_t>(1, g_parse_min_chunk);
  const uint64_t C = std::max<uint64_t>(1, std::min<uint64_t>(std::max<uint64_t>((uint64_t)T * 8, n / (64 << 20)),
                                                              n / min_chunk));
  std::vector<uint64_t> cs(C + 1);
  for (uint64_t c = 0; c <= C; ++c) cs[c] = (uint64_t)((__uint128_t)n * c / C);
  std::vector<ChunkOut> ch(C);
  bool final_hdr = false;  // FASTA: the file ends inside a header line

  // pass 1 (parallel) + the sequential composition of one value per chunk
  if (fastq) {
    run_chunks(C, T, [&](uint64_t c) { fastq_stats(buf, n, cs[c], cs[c + 1], ch[c]); });
    for (uint64_t c = 0; c < C; ++c) {
      if (c) ch[c].line_base = ch[c - 1].line_base + ch[c - 1].nl;
      const uint64_t first = ch[c].line_base + (ch[c].lead_nl ? 1 : 0);  // index of the first line start
      const uint64_t k = (1 - first) & 3;  // local residue of the sequence lines
      ch[c].bytes = ch[c].fq_bytes[k];
      ch[c].records = ch[c].fq_recs[k];
    }
  } else {
    run_chunks(C, T, [&](uint64_t c) { fasta_stats(buf, cs[c], cs[c + 1], ch[c]); });
    bool st = true;  // the file starts inside the first header line
    for (uint64_t c = 0; c < C; ++c) {
      ChunkOut& x = ch[c];
      x.start_hdr = st;
      x.bytes = x.fa_bytes_rest + (st ? 0 : x.fa_bytes_pre);
      x.records = x.fa_close_rest + (st ? 0 : x.fa_close_pre);
      if (!x.has_nl) {  // no '\n': the whole chunk is the prefix
        x.bytes = 0;
        x.records = 0;
        if (!st) {
          const char* cb = buf + cs[c];
          const char* ce = buf + cs[c + 1];
          const char* gt = find(cb, ce, '>');
          x.bytes = (uint64_t)(gt - cb);
          x.records = gt != ce;
        }
        st = st || x.any_gt;
      } else {
        st = x.end_hdr;
      }
    }
    final_hdr = st;
  }

  // bases; grow the (uninitialised) outputs; pass 2 writes in place
  uint64_t tb = 0, rb = 0;
  for (uint64_t c = 0; c < C; ++c) {
    ch[c].text_base = tb;
    ch[c].rec_base = rb;
    tb += ch[c].bytes;
    rb += ch[c].records;
  }
  const uint64_t nrec = fastq ? rb : rb + 1;  // FASTA: EOF closes the last record
  // the header-at-EOF case below may append up to n bytes
  const uint64_t text_cap = out.n_text + tb + (fastq ? 0 : n) + 1;
  char* nt = static_cast<char*>(std::realloc(out.text, text_cap));
  if (!nt) return -3;
  out.text = nt;
  uint64_t* no = static_cast<uint64_t*>(std::realloc(out.off, (out.n_rec + nrec + 1) * sizeof(uint64_t)));
  if (!no) return -3;
  out.off = no;
  if (out.n_rec == 0) out.off[0] = out.n_text;
  char* dst = out.text + out.n_text;
  uint64_t* o = out.off + out.n_rec + 1;
  const uint64_t start = out.n_text;
  if (fastq) {
    run_chunks(C, T, [&](uint64_t c) {
      uint64_t t = ch[c].text_base, r = ch[c].rec_base;
      fastq_lines(buf, n, cs[c], cs[c + 1], ch[c].line_base, [&](const char* p, uint64_t len) {
        std::memcpy(dst + t, p, len);
        t += len;
        o[r++] = start + t;
      });
    });
  } else {
    run_chunks(C, T, [&](uint64_t c) {
      uint64_t t = ch[c].text_base, r = ch[c].rec_base;
      fasta_split(
          buf, cs[c], cs[c + 1], ch[c].start_hdr,
          [&](const char* p, uint64_t len) {
            std::memcpy(dst + t, p, len);
            t += len;
          },
          [&] { o[r++] = start + t; });
    });
    o[nrec - 1] = start + tb;
    // The file ends inside a header line that has no '\n' (after the first
    // record): the reference's getline(text, '>') then fails without clearing
    // `text`, so the record's "sequence" is that header's text (Dataset.cpp:
    // 139-144 with libstdc++'s sentry semantics).  Only the last record can be
    // affected; its sequence is empty here in that case.
    if (final_hdr && nrec > 1) {
      const char* e = buf + n;
      const char* last_nl = nullptr;
      for (const char* p = e; p > buf;)
        if (*--p == '\n') {
          last_nl = p;
          break;
        }
      const char* gt = last_nl ? find(last_nl + 1, e, '>') : e;
      if (gt != e) {  // the header opened by this '>' runs to EOF
        const uint64_t len = (uint64_t)(e - (gt + 1));
        std::memcpy(dst + tb, gt + 1, len);
        tb += len;
        o[nrec - 1] = start + tb;
      }
    }
  }
  out.n_text += tb;
  out.n_rec += nrec;
  if (stats) {
    stats->bytes = n;
    stats->records = nrec;
    stats->threads = T;
    stats->seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  }
  return 0;
}

int parse_file_parallel(const std::string& path, ParsedText& out, int nthreads, ParseStats* stats) {
  const auto t0 = std::chrono::steady_clock::now();
  const int fd = ::open(path.c_str(), O_RDONLY);
  if (fd < 0) return -1;
  struct stat sb;
  if (::fstat(fd, &sb) != 0) {
    ::close(fd);
    return -1;
  }
  const uint64_t n = (uint64_t)sb.st_size;
  if (n == 0) {
    ::close(fd);
    return -2;
  }
  void* m = ::mmap(nullptr, n, PROT_READ, MAP_PRIVATE, fd, 0);
  ::close(fd);
  if (m == MAP_FAILED) return -1;
  ::madvise(m, n, MADV_WILLNEED);
  const int rc = parse_buffer_parallel(static_cast<const char*>(m), n, out, nthreads, stats);
  ::munmap(m, n);
  if (stats) stats->seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  return rc;
}

}  // namespace mg
