// mg_overlap — command-line driver with main.cpp's argument surface
// (main.cpp:117-184: -se/-pe <n> <files...>, -f <prefix>, -l <minOverlap>)
// running main.cpp:33,45-50 with the overlap path on the GPU:
//   Dataset -> HashTable::insertDataset -> OverlapGraph(ht) (discovery on the
//   device; exploration order, transitive reduction and the contraction loop
//   replayed on the host) -> saveReads -> sortEdges -> saveGraphToFile
// writing <prefix>_sortedReads.fasta and <prefix>.unitig as the reference does.
// Extra flags: -k <seed k>, -d <device>;
//   -nocontract  stop before the contraction loop (OverlapGraph.cpp:211-215) and
//                write every graph[u] list in list order to <prefix>.graph
//                ("#C nodes edges" first) instead of the .unitig;
//   -raw         the raw discovery multiset to <prefix>.edges (sorted
//                "u v orient offset" lines);
//   -s           main.cpp:36-42's resume: OverlapGraph() -> setDataset ->
//                readGraphFromFile(<prefix>.unitig) -> sortEdges (no device
//                needed), then saveGraphToFile(<prefix>.resumed.unitig) and the
//                lists in list order to <prefix>.resumed.graph.
//   -xchg <K>    the exchange mode over RCCL: one
//                process per GPU (RANK / WORLD_SIZE / LOCAL_RANK / MASTER_ADDR /
//                MASTER_PORT as torchrun --no-python sets them; none set = one
//                rank), K timed steps of the distributed insertDataset +
//                markContainedReads + insertAllEdgesOfRead after one warm-up;
//                rank 0 prints the combined row digest (mg_rows_digest formula),
//                the superReadID digest and the max-over-ranks step time.
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "mg_api.hpp"
#include "mg_xchg.hpp"

static int env_int(const char* name, int dflt) {
  const char* v = std::getenv(name);
  return v && *v ? std::atoi(v) : dflt;
}

// -xchg: every rank parses the same files, uploads the whole read set and owns
// the buckets and source reads of mg_set_shard(rank, world, 0, 0).
struct XchgOpts {
  unsigned long long l = 0;
  int k = 0, steps = 0;
  double cap_scale = 1.0;  // -xchg-caps F: first capacity estimates x F (F < 1 forces the rerun path)
  bool shared_device = false;  // -xchg-sim: every rank's context on one device
};

static void hip_ok(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

static uint16_t max_read_length(Dataset* ds) {
  const uint16_t* len = ds->packedLengths();
  uint16_t m = 0;
  for (uint64_t i = 0; i < ds->getNumberOfUniqueReads(); ++i) m = std::max(m, len[i]);
  return m;
}

// One rank's part: upload, K timed steps (after one warm-up) of the exchange
// step over `x`, then the combined digests; rank 0 prints the JSON line.
// Reads over 1,024 bp: the exchange mode's kernels stop there
// (sharded.py EXCHANGE_MAX_BP), so the rank runs the replicated mode instead
// (whole index per rank, its source-read range, no data-path
// collective) -- the same fallback as sharded.py's _replicated_step.
static void run_rank(mg::Transport& x, Dataset* ds, int device, const XchgOpts& o) {
  const int rank = x.rank(), world = x.world();
  hip_ok(hipSetDevice(device), "hipSetDevice");
  mg_ctx* ctx = nullptr;
  if (mg_create(&ctx, device)) throw std::runtime_error("no HIP device available (no CPU fallback)");
  struct Destroy {
    mg_ctx* c;
    ~Destroy() { mg_destroy(c); }
  } destroy{ctx};
  auto ok = [&](int rc, const char* what) {
    if (rc) throw std::runtime_error(std::string(what) + ": " + mg_last_error(ctx));
  };
  const uint64_t n = ds->getNumberOfUniqueReads();
  const bool replicated = max_read_length(ds) > 1024;
  if (o.shared_device) ok(mg_set_option(ctx, "layout_scratch", 0), "mg_set_option");  // (P contexts on one device)
  ok(mg_upload_reads_packed(ctx, ds->packedWords(), ds->packedLengths(), n, ds->wordsPerRead()), "upload");
  const uint64_t lo = n * rank / world, hi = n * (rank + 1) / world;
  if (replicated)
    ok(mg_set_shard(ctx, 0, 1, lo, hi), "mg_set_shard");
  else
    ok(mg_set_shard(ctx, (uint32_t)rank, (uint32_t)world, 0, 0), "mg_set_shard");
  hipStream_t s = (hipStream_t)mg_stream(ctx);
  int reruns = 0;
  std::vector<double> ms;
  uint64_t mine[4] = {0, 0, 0, 0}, sup[4] = {0, 0, 0, 0}, held = 0;
  bool contained = false, rows_routed = false;
  std::vector<uint64_t> caps(3, 0);
  {
    mg::XchgStep step(ctx, x, (uint32_t)o.l, (uint32_t)o.k);
    if (o.cap_scale != 1.0) step.scale_caps(o.cap_scale);
    auto one = [&]() {
      if (!replicated) {
        reruns += step.run();
        return;
      }
      uint64_t rows = 0;
      ok(mg_build_index(ctx, (uint32_t)o.l, (uint32_t)o.k), "mg_build_index");
      ok(mg_mark_contained(ctx, nullptr), "mg_mark_contained");
      if (hi > lo) ok(mg_find_overlaps(ctx, &rows), "mg_find_overlaps");  // (read_hi == read_lo == 0 means all)
      hip_ok(hipStreamSynchronize(s), "hipStreamSynchronize");
    };
    one();  // warm-up: buffers sized, capacities grown
    double* dt = nullptr;
    hip_ok(hipMalloc(&dt, sizeof(double)), "hipMalloc");
    for (int i = 0; i < o.steps; ++i) {
      x.barrier(s);
      const auto t0 = std::chrono::steady_clock::now();
      one();
      hip_ok(hipStreamSynchronize(s), "hipStreamSynchronize");
      double v = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
      hip_ok(hipMemcpy(dt, &v, sizeof v, hipMemcpyHostToDevice), "hipMemcpy");
      x.allreduce_max_f64(dt, 1, s);  // the slowest rank's step
      hip_ok(hipMemcpyAsync(&v, dt, sizeof v, hipMemcpyDeviceToHost, s), "hipMemcpyAsync");
      hip_ok(hipStreamSynchronize(s), "hipStreamSynchronize");
      ms.push_back(v);
    }
    hip_ok(hipFree(dt), "hipFree");
    if (replicated) {
      contained = max_read_length(ds) != *std::min_element(ds->packedLengths(), ds->packedLengths() + n);
      if (hi > lo) ok(mg_rows_digest(ctx, nullptr, 0, mine), "mg_rows_digest");
      held = hi > lo ? mg_num_rows(ctx) : 0;
    } else {
      step.rows_digest(mine);
      contained = step.contained();
      held = step.rows_held();
      for (int kind = 0; kind < 3; ++kind) caps[kind] = step.caps()[kind];
      rows_routed = step.rows_routed();
    }
    if (contained) ok(mg_super_digest(ctx, sup), "mg_super_digest");
  }
  // combined digest: n, sum, sum2 add and xor xors over the ranks' rows
  uint64_t *d_in = nullptr, *d_all = nullptr;
  hip_ok(hipMalloc(&d_in, 5 * sizeof(uint64_t)), "hipMalloc");
  hip_ok(hipMalloc(&d_all, 5 * world * sizeof(uint64_t)), "hipMalloc");
  const uint64_t mine5[5] = {mine[0], mine[1], mine[2], mine[3], held};
  hip_ok(hipMemcpy(d_in, mine5, sizeof mine5, hipMemcpyHostToDevice), "hipMemcpy");
  x.allgather_u64(d_in, d_all, 5, s);
  std::vector<uint64_t> all(5 * world);
  hip_ok(hipMemcpyAsync(all.data(), d_all, all.size() * sizeof(uint64_t), hipMemcpyDeviceToHost, s), "hipMemcpyAsync");
  hip_ok(hipStreamSynchronize(s), "hipStreamSynchronize");
  hip_ok(hipFree(d_in), "hipFree");
  hip_ok(hipFree(d_all), "hipFree");
  uint64_t dg[4] = {0, 0, 0, 0};  // mg_rows_digest order: n, sum, xor, sum2
  std::string held_list;
  for (int r = 0; r < world; ++r) {
    dg[0] += all[5 * r];
    dg[1] += all[5 * r + 1];
    dg[2] ^= all[5 * r + 2];
    dg[3] += all[5 * r + 3];
    held_list += (r ? ", " : "") + std::to_string(all[5 * r + 4]);
  }
  x.barrier(s);
  if (rank == 0) {
    std::vector<double> sorted = ms;
    std::sort(sorted.begin(), sorted.end());
    const double best = sorted.empty() ? 0 : sorted.front(), med = sorted.empty() ? 0 : sorted[sorted.size() / 2];
    std::printf(
        "{\"mode\": \"%s\", \"world\": %d, \"unique_reads\": %llu, \"rows\": {\"n\": %llu, \"sum\": %llu, "
        "\"xor\": %llu, \"sum2\": %llu}, \"super\": {\"n\": %llu, \"sum\": %llu, \"xor\": %llu, \"sum2\": %llu}, "
        "\"contained\": %s, \"steps\": %d, \"best_ms\": %.3f, \"median_ms\": %.3f, \"reruns\": %d, "
        "\"rows_rank0\": %llu, \"rows_held\": [%s], \"caps\": [%llu, %llu, %llu], \"rows_routed\": %s}\n",
        replicated ? "replicated" : "xchg", world, (unsigned long long)n, (unsigned long long)dg[0],
        (unsigned long long)dg[1], (unsigned long long)dg[2], (unsigned long long)dg[3],
        (unsigned long long)sup[0], (unsigned long long)sup[1], (unsigned long long)sup[2],
        (unsigned long long)sup[3], contained ? "true" : "false", o.steps, best, med, reruns,
        (unsigned long long)held, held_list.c_str(), (unsigned long long)caps[0], (unsigned long long)caps[1],
        (unsigned long long)caps[2], rows_routed ? "true" : "false");
    std::fflush(stdout);
  }
}

// one process per GPU over RCCL (RANK / WORLD_SIZE / LOCAL_RANK / MASTER_* as torchrun sets them)
static int run_xchg(Dataset* ds, int dev, const XchgOpts& o) {
  const int rank = env_int("RANK", 0), world = env_int("WORLD_SIZE", 1);
  const int device = env_int("LOCAL_RANK", dev);
  const char* addr = std::getenv("MASTER_ADDR");
  const int port = env_int("MASTER_PORT", 29500) + 1;  // torchrun's own store holds MASTER_PORT
  mg::RcclExchange x(rank, world, device, addr && *addr ? addr : "127.0.0.1", port);
  run_rank(x, ds, device, o);
  return 0;
}

// -xchg-sim P: P ranks as threads of this process on one device, each with its
// own context and stream, the collectives by device copies (LocalTransport):
// the same XchgStep code as the N-GPU run, at P > 1 on one GPU.
static int run_xchg_sim(Dataset* ds, int dev, int P, XchgOpts o) {
  o.shared_device = true;
  mg::LocalGroup g(P);
  std::vector<std::string> err(P);
  std::vector<std::thread> th;
  for (int r = 0; r < P; ++r)
    th.emplace_back([&, r] {
      try {
        mg::LocalTransport x(g, r);
        run_rank(x, ds, dev, o);
      } catch (const std::exception& e) {
        err[r] = e.what();
        g.abort();
      }
    });
  for (std::thread& t : th) t.join();
  int rc = 0;
  for (int r = 0; r < P; ++r)
    if (!err[r].empty() && err[r] != "a peer rank failed") {
      std::fprintf(stderr, "mg_overlap: rank %d: %s\n", r, err[r].c_str());
      rc = 2;
    }
  if (!rc)
    for (int r = 0; r < P; ++r)
      if (!err[r].empty()) {
        std::fprintf(stderr, "mg_overlap: rank %d: %s\n", r, err[r].c_str());
        rc = 2;
      }
  return rc;
}

static void usage() {
  std::fprintf(stderr,
               "Usage: mg_overlap [-pe n f1..fn] [-se n f1..fn] -f prefix -l minOverlap [-k seedK] [-d device] [-nocontract | -raw | -s | -xchg K "
               "[-xchg-sim P] [-xchg-caps F]]\n");
}

int main(int argc, char** argv) {
  std::vector<std::string> pe, se;
  std::string prefix;
  unsigned long long l = 0;
  int k = 0, dev = 0;
  bool raw = false, nocontract = false, resume = false;
  int xchg_steps = -1, xchg_sim = 0;
  double xchg_caps = 1.0;
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    if ((a == "-pe" || a == "-se") && i + 1 < argc) {
      int n = std::atoi(argv[++i]);
      for (int j = 0; j < n && i + 1 < argc; ++j) (a == "-pe" ? pe : se).push_back(argv[++i]);
    } else if (a == "-f" && i + 1 < argc) {
      prefix = argv[++i];
    } else if (a == "-l" && i + 1 < argc) {
      l = std::strtoull(argv[++i], nullptr, 10);
    } else if (a == "-k" && i + 1 < argc) {
      k = std::atoi(argv[++i]);
    } else if (a == "-d" && i + 1 < argc) {
      dev = std::atoi(argv[++i]);
    } else if (a == "-raw") {
      raw = true;
    } else if (a == "-nocontract") {
      nocontract = true;
    } else if (a == "-s") {
      resume = true;
    } else if (a == "-xchg" && i + 1 < argc) {
      xchg_steps = std::max(0, std::atoi(argv[++i]));
    } else if (a == "-xchg-sim" && i + 1 < argc) {
      xchg_sim = std::atoi(argv[++i]);
    } else if (a == "-xchg-caps" && i + 1 < argc) {
      xchg_caps = std::atof(argv[++i]);
    } else {
      usage();
      return (a == "-h" || a == "--help") ? 0 : 1;
    }
  }
  if (l < 2 || prefix.empty() || (pe.empty() && se.empty()) || xchg_sim < 0 || xchg_sim > 16 || !(xchg_caps > 0)) {
    usage();
    return 1;
  }
  try {
    HashTable::setDefaultDevice(dev);
    HashTable::setDefaultSeedK((uint32_t)k);
    OverlapGraph::replayExploration = !raw;
    OverlapGraph::contractPaths = !nocontract;
    Dataset* ds = new Dataset(pe, se, l);
    if (xchg_steps >= 0) {
      XchgOpts o;
      o.l = l;
      o.k = k;
      o.steps = xchg_steps;
      o.cap_scale = xchg_caps;
      const int rc = xchg_sim > 0 ? run_xchg_sim(ds, dev, xchg_sim, o) : run_xchg(ds, dev, o);
      delete ds;
      return rc;
    }
    if (resume) {  // main.cpp:36-42
      OverlapGraph* g = new OverlapGraph();
      g->setDataset(ds);
      g->readGraphFromFile(prefix + ".unitig");
      g->sortEdges();
      g->saveGraphToFile(prefix + ".resumed.unitig");
      g->saveGraphLists(prefix + ".resumed.graph");
      std::printf("{\"unique_reads\": %llu, \"nodes\": %llu, \"directed_edges\": %llu}\n",
                  (unsigned long long)ds->getNumberOfUniqueReads(), (unsigned long long)g->getNumberOfNodes(),
                  (unsigned long long)g->getNumberOfEdges());
      delete g;
      delete ds;
      return 0;
    }
    HashTable* ht = new HashTable();
    ht->insertDataset(ds, l);
    OverlapGraph* g = new OverlapGraph(ht);  // deletes ht
    ds->saveReads(prefix + "_sortedReads.fasta");
    if (raw) {
      g->saveRawEdges(prefix + ".edges");
    } else if (nocontract) {
      g->saveGraphLists(prefix + ".graph");
    } else {
      g->sortEdges();  // main.cpp:49-50
      g->saveGraphToFile(prefix + ".unitig");
    }
    const mg_timings& t = g->timings();
    std::printf(
        "{\"reads\": %llu, \"unique_reads\": %llu, \"nodes\": %llu, \"directed_edges\": %llu, "
        "\"undirected_edges\": %llu, \"index_ms\": %.3f, \"contained_ms\": %.3f, \"overlap_ms\": %.3f}\n",
        (unsigned long long)ds->getNumberOfReads(), (unsigned long long)ds->getNumberOfUniqueReads(),
        (unsigned long long)g->getNumberOfNodes(), (unsigned long long)g->getNumberOfEdges(),
        (unsigned long long)g->getNumberOfEdges() / 2, t.index_ms, t.contained_ms, t.overlap_ms);
    delete g;
    delete ds;
  } catch (const std::exception& e) {
    std::fprintf(stderr, "mg_overlap: %s\n", e.what());
    return 2;
  }
  return 0;
}
