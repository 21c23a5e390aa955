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
// Each chunk is scanned twice with its start state known: once to size its
// sequence bytes and records, once to write them straight into their final
// place (no per-chunk staging copy).  The result equals the serial splitter's
// (tests/test_parse.py).
#include "mg_parse.hpp"

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
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
  uint64_t bytes = 0, records = 0;  // pass-1 sizes
  uint64_t text_base = 0, rec_base = 0;
  uint64_t line_base = 0;  // FASTQ: '\n' before the chunk start
  uint64_t nl = 0;         // FASTQ: '\n' inside the chunk
  bool start_hdr = false;  // FASTA: state at the chunk start
};

// FASTQ: the lines starting in [b, e); emit(ptr, len) for every sequence line
template <typename Emit>
void fastq_lines(const char* buf, uint64_t n, uint64_t b, uint64_t e, uint64_t line_base, Emit&& emit) {
  const char* end = buf + n;
  const char* p;
  uint64_t idx;
  if (b == 0) {
    p = buf;
    idx = 0;
  } else if (buf[b - 1] == '\n') {
    p = buf + b;
    idx = line_base;
  } else {
    const char* q = find(buf + b, buf + e, '\n');
    if (q == buf + e) return;  // no line starts in this chunk
    p = q + 1;
    idx = line_base + 1;
  }
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

}  // namespace

int parse_buffer_parallel(const char* buf, uint64_t n, std::string& text, std::vector<uint64_t>& off, int nthreads,
                          ParseStats* stats) {
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

  if (fastq) {
    run_chunks(C, T, [&](uint64_t c) {
      ch[c].nl = (uint64_t)std::count(buf + cs[c], buf + cs[c + 1], '\n');
    });
    for (uint64_t c = 1; c < C; ++c) ch[c].line_base = ch[c - 1].line_base + ch[c - 1].nl;
    run_chunks(C, T, [&](uint64_t c) {
      uint64_t bytes = 0, recs = 0;
      fastq_lines(buf, n, cs[c], cs[c + 1], ch[c].line_base, [&](const char*, uint64_t len) {
        bytes += len;
        recs++;
      });
      ch[c].bytes = bytes;
      ch[c].records = recs;
    });
  } else {
    // chunk end states, then start states composed in order
    std::vector<int8_t> end_has_nl(C), end_hdr(C), any_gt(C);
    run_chunks(C, T, [&](uint64_t c) {
      const char* b = buf + cs[c];
      const char* e = buf + cs[c + 1];
      const char* last_nl = nullptr;
      for (const char* p = e; p > b;)
        if (*--p == '\n') {
          last_nl = p;
          break;
        }
      end_has_nl[c] = last_nl != nullptr;
      if (last_nl)
        end_hdr[c] = find(last_nl + 1, e, '>') != e;
      else
        any_gt[c] = find(b, e, '>') != e;
    });
    bool st = true;  // the file starts inside the first header line
    for (uint64_t c = 0; c < C; ++c) {
      ch[c].start_hdr = st;
      st = end_has_nl[c] ? (bool)end_hdr[c] : (st || any_gt[c]);
    }
    final_hdr = st;
    run_chunks(C, T, [&](uint64_t c) {
      uint64_t bytes = 0, closes = 0;
      fasta_split(
          buf, cs[c], cs[c + 1], ch[c].start_hdr, [&](const char*, uint64_t len) { bytes += len; },
          [&] { closes++; });
      ch[c].bytes = bytes;
      ch[c].records = closes;
    });
  }

  // bases, then write in place
  const uint64_t text0 = text.size(), off0 = off.size();
  uint64_t tb = 0, rb = 0;
  for (uint64_t c = 0; c < C; ++c) {
    ch[c].text_base = tb;
    ch[c].rec_base = rb;
    tb += ch[c].bytes;
    rb += ch[c].records;
  }
  const uint64_t nrec = fastq ? rb : rb + 1;  // FASTA: EOF closes the last record
  text.resize(text0 + tb);
  off.resize(off0 + nrec);
  char* out = &text[0] + text0;
  uint64_t* o = off.data() + off0;
  const uint64_t start = text0;
  if (fastq) {
    run_chunks(C, T, [&](uint64_t c) {
      uint64_t t = ch[c].text_base, r = ch[c].rec_base;
      fastq_lines(buf, n, cs[c], cs[c + 1], ch[c].line_base, [&](const char* p, uint64_t len) {
        std::memcpy(out + t, p, len);
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
            std::memcpy(out + t, p, len);
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
      const char* from = last_nl ? last_nl + 1 : buf;
      const char* gt = find(from, e, '>');
      if (gt != e && last_nl) {  // the header opened by this '>' runs to EOF
        const uint64_t len = (uint64_t)(e - (gt + 1));
        text.resize(text0 + tb + len);
        std::memcpy(&text[0] + text0 + tb, gt + 1, len);
        off[off0 + nrec - 1] = start + tb + len;
      }
    }
  }
  if (stats) {
    stats->bytes = n;
    stats->records = nrec;
    stats->threads = T;
    stats->seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  }
  return 0;
}

int parse_file_parallel(const std::string& path, std::string& text, std::vector<uint64_t>& off, int nthreads,
                        ParseStats* stats) {
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
  const int rc = parse_buffer_parallel(static_cast<const char*>(m), n, text, off, nthreads, stats);
  ::munmap(m, n);
  if (stats) stats->seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  return rc;
}

}  // namespace mg
