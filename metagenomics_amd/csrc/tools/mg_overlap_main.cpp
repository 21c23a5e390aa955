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
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "mg_api.hpp"

static void usage() {
  std::fprintf(stderr,
               "Usage: mg_overlap [-pe n f1..fn] [-se n f1..fn] -f prefix -l minOverlap [-k seedK] [-d device] [-nocontract | -raw | -s]\n");
}

int main(int argc, char** argv) {
  std::vector<std::string> pe, se;
  std::string prefix;
  unsigned long long l = 0;
  int k = 0, dev = 0;
  bool raw = false, nocontract = false, resume = false;
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
