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
#include <vector>

#include "mg_api.hpp"
#include "mg_xchg.hpp"

static int env_int(const char* name, int dflt) {
  const char* v = std::getenv(name);
  return v && *v ? std::atoi(v) : dflt;
}

// -xchg: every rank parses the same files, uploads the whole read set and owns
// the buckets and source reads of mg_set_shard(rank, world, 0, 0).
static int run_xchg(Dataset* ds, unsigned long long l, int k, int dev, int steps) {
  const int rank = env_int("RANK", 0), world = env_int("WORLD_SIZE", 1);
  const int device = env_int("LOCAL_RANK", dev);
  const char* addr = std::getenv("MASTER_ADDR");
  const int port = env_int("MASTER_PORT", 29500) + 1;  // torchrun's own store holds MASTER_PORT
  mg::RcclExchange x(rank, world, device, addr && *addr ? addr : "127.0.0.1", port);
  mg_ctx* ctx = nullptr;
  if (mg_create(&ctx, device)) throw std::runtime_error("no HIP device available (no CPU fallback)");
  auto ok = [&](int rc, const char* what) {
    if (rc) throw std::runtime_error(std::string(what) + ": " + mg_last_error(ctx));
  };
  auto hip = [](hipError_t e, const char* what) {
    if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
  };
  ok(mg_upload_reads_packed(ctx, ds->packedWords(), ds->packedLengths(), ds->getNumberOfUniqueReads(),
                            ds->wordsPerRead()),
     "upload");
  ok(mg_set_shard(ctx, (uint32_t)rank, (uint32_t)world, 0, 0), "mg_set_shard");
  hipStream_t s = (hipStream_t)mg_stream(ctx);
  int reruns = 0;
  std::vector<double> ms;
  {
    mg::XchgStep step(ctx, x, (uint32_t)l, (uint32_t)k);
    reruns += step.run();  // warm-up: buffers sized, capacities grown
    double* dt = nullptr;
    hip(hipMalloc(&dt, sizeof(double)), "hipMalloc");
    for (int i = 0; i < steps; ++i) {
      x.barrier(s);
      const auto t0 = std::chrono::steady_clock::now();
      reruns += step.run();
      hip(hipStreamSynchronize(s), "hipStreamSynchronize");
      double v = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
      hip(hipMemcpy(dt, &v, sizeof v, hipMemcpyHostToDevice), "hipMemcpy");
      x.allreduce_max_f64(dt, 1, s);  // the slowest rank's step
      hip(hipMemcpyAsync(&v, dt, sizeof v, hipMemcpyDeviceToHost, s), "hipMemcpyAsync");
      hip(hipStreamSynchronize(s), "hipStreamSynchronize");
      ms.push_back(v);
    }
    hip(hipFree(dt), "hipFree");
    // combined digest: n, sum, sum2 add and xor xors over the ranks' rows
    uint64_t mine[4], sup[4] = {0, 0, 0, 0};
    step.rows_digest(mine);
    if (step.contained()) ok(mg_super_digest(ctx, sup), "mg_super_digest");
    uint64_t *d_in = nullptr, *d_all = nullptr;
    hip(hipMalloc(&d_in, 4 * sizeof(uint64_t)), "hipMalloc");
    hip(hipMalloc(&d_all, 4 * world * sizeof(uint64_t)), "hipMalloc");
    hip(hipMemcpy(d_in, mine, sizeof mine, hipMemcpyHostToDevice), "hipMemcpy");
    x.allgather_u64(d_in, d_all, 4, s);
    std::vector<uint64_t> all(4 * world);
    hip(hipMemcpyAsync(all.data(), d_all, all.size() * sizeof(uint64_t), hipMemcpyDeviceToHost, s), "hipMemcpyAsync");
    hip(hipStreamSynchronize(s), "hipStreamSynchronize");
    hip(hipFree(d_in), "hipFree");
    hip(hipFree(d_all), "hipFree");
    uint64_t dg[4] = {0, 0, 0, 0};  // mg_rows_digest order: n, sum, xor, sum2
    for (int r = 0; r < world; ++r) {
      dg[0] += all[4 * r];
      dg[1] += all[4 * r + 1];
      dg[2] ^= all[4 * r + 2];
      dg[3] += all[4 * r + 3];
    }
    if (rank == 0) {
      std::vector<double> sorted = ms;
      std::sort(sorted.begin(), sorted.end());
      const double best = sorted.empty() ? 0 : sorted.front(), med = sorted.empty() ? 0 : sorted[sorted.size() / 2];
      std::printf(
          "{\"mode\": \"xchg\", \"world\": %d, \"unique_reads\": %llu, \"rows\": {\"n\": %llu, \"sum\": %llu, "
          "\"xor\": %llu, \"sum2\": %llu}, \"super\": {\"n\": %llu, \"sum\": %llu, \"xor\": %llu, \"sum2\": %llu}, "
          "\"contained\": %s, \"steps\": %d, \"best_ms\": %.3f, \"median_ms\": %.3f, \"reruns\": %d, "
          "\"rows_rank0\": %llu}\n",
          world, (unsigned long long)ds->getNumberOfUniqueReads(), (unsigned long long)dg[0],
          (unsigned long long)dg[1], (unsigned long long)dg[2], (unsigned long long)dg[3],
          (unsigned long long)sup[0], (unsigned long long)sup[1], (unsigned long long)sup[2],
          (unsigned long long)sup[3], step.contained() ? "true" : "false", steps, best, med, reruns,
          (unsigned long long)step.rows_held());
    }
  }
  mg_destroy(ctx);
  return 0;
}

static void usage() {
  std::fprintf(stderr,
               "Usage: mg_overlap [-pe n f1..fn] [-se n f1..fn] -f prefix -l minOverlap [-k seedK] [-d device] [-nocontract | -raw | -s | -xchg K]\n");
}

int main(int argc, char** argv) {
  std::vector<std::string> pe, se;
  std::string prefix;
  unsigned long long l = 0;
  int k = 0, dev = 0;
  bool raw = false, nocontract = false, resume = false;
  int xchg_steps = -1;
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
    } else {
      usage();
      return (a == "-h" || a == "--help") ? 0 : 1;
    }
  }
  if (l < 2 || prefix.empty() || (pe.empty() && se.empty())) {
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
      const int rc = run_xchg(ds, l, k, dev, xchg_steps);
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
