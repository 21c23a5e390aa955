// mg_explore — the reference's own exploration loop driven through the drop-in
// OverlapGraph's per-read methods (OverlapGraph.h:54,64-68).
//
// A caller that builds the graph itself, as buildOverlapGraphFromHashTable
// does (OverlapGraph.cpp:144-204), needs insertAllEdgesOfRead, the transitive
// reduction steps and, for its own checks, checkOverlap /
// checkOverlapForContainedRead.  This program is such a caller: it restates
// the component-by-component queue of :144-204 on top of
// OverlapGraph::beginBuildFromHashTable (the set-up of :111-142: lists,
// markContainedReads, the device discovery) and writes
//   <prefix>.graph   "#C nodes edges" + every graph[u] list in list order
//                    (the reference's graph before its contraction loop), and
//   <prefix>.unitig  after the contraction loop (:211-215), sortEdges and
//                    saveGraphToFile (main.cpp:49-50),
// which tests/test_gpu_parity.py compares with the reference's own (bfs /
// unitig goldens).  It also cross-checks checkOverlap and
// checkOverlapForContainedRead against the device's results: every listed
// edge passes checkOverlap at its (o, j) from the side that discovered it, and
// every contained read (up to 1,024 bp) passes checkOverlapForContainedRead
// against its superRead at some (o, j).
//   usage: mg_explore <fasta|fastq> <l> <prefix> [seed k]
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "mg_api.hpp"

namespace {
int g_fail = 0;
void check(bool ok, const char* what, UINT64 a, UINT64 b) {
  if (ok) return;
  if (g_fail++ < 10) std::fprintf(stderr, "mg_explore: %s failed for %llu %llu\n", what, a, b);
}

// key o and window j of an edge insertAllEdgesOfRead created (inverse of :550-557)
void key_of(Edge* e, UINT64 n1, UINT64 h, UINT64* o, UINT64* j) {
  const UINT8 t = e->getOrientation();
  *o = t == 3 ? 0 : t == 0 ? 1 : t == 2 ? 2 : 3;
  *j = (*o == 0 || *o == 2) ? e->getOverlapOffset() : n1 - h - e->getOverlapOffset();
}
}  // namespace

int main(int argc, char** argv) {
  if (argc < 4) {
    std::fprintf(stderr, "usage: %s <fasta|fastq> <l> <prefix> [seed k]\n", argv[0]);
    return 1;
  }
  const UINT64 l = std::strtoull(argv[2], nullptr, 10);
  const std::string prefix = argv[3];
  try {
    if (argc > 4) HashTable::setDefaultSeedK((uint32_t)std::atoi(argv[4]));
    Dataset* ds = new Dataset({}, {argv[1]}, l);
    HashTable* ht = new HashTable();
    ht->insertDataset(ds, l);
    OverlapGraph* g = new OverlapGraph();
    g->beginBuildFromHashTable(ht);  // :111-142
    const UINT64 N = ds->getNumberOfUniqueReads(), h = ht->getHashStringLength();
    auto list = [&](UINT64 r) { return g->getEdges(r); };
    std::vector<nodeType> explored(N + 1, UNEXPLORED);
    std::vector<markType> marked(N + 1, VACANT);
    std::vector<UINT64> queue(N + 1, 0);
    // the exploration of OverlapGraph.cpp:144-204, one component at a time
    for (UINT64 i = 1; i <= N; i++) {
      if (explored[i] != UNEXPLORED) continue;
      UINT64 start = 0, end = 0;
      queue[end++] = i;
      while (start < end) {
        const UINT64 read1 = queue[start++];
        if (explored[read1] == UNEXPLORED) {
          g->insertAllEdgesOfRead(read1, &explored);
          explored[read1] = EXPLORED;
        }
        if (list(read1)->empty()) continue;
        if (explored[read1] == EXPLORED) {  // unexplored neighbours first
          for (UINT64 a = 0; a < list(read1)->size(); a++) {
            const UINT64 read2 = list(read1)->at(a)->getDestinationRead()->getReadNumber();
            if (explored[read2] == UNEXPLORED) {
              queue[end++] = read2;
              g->insertAllEdgesOfRead(read2, &explored);
              explored[read2] = EXPLORED;
            }
          }
          g->markTransitiveEdges(read1, &marked);
          explored[read1] = EXPLORED_AND_TRANSITIVE_EDGES_MARKED;
        }
        if (explored[read1] == EXPLORED_AND_TRANSITIVE_EDGES_MARKED) {  // then the neighbours' neighbours
          for (UINT64 a = 0; a < list(read1)->size(); a++) {
            const UINT64 read2 = list(read1)->at(a)->getDestinationRead()->getReadNumber();
            if (explored[read2] != EXPLORED) continue;
            for (UINT64 b = 0; b < list(read2)->size(); b++) {
              const UINT64 read3 = list(read2)->at(b)->getDestinationRead()->getReadNumber();
              if (explored[read3] == UNEXPLORED) {
                queue[end++] = read3;
                g->insertAllEdgesOfRead(read3, &explored);
                explored[read3] = EXPLORED;
              }
            }
            g->markTransitiveEdges(read2, &marked);
            explored[read2] = EXPLORED_AND_TRANSITIVE_EDGES_MARKED;
          }
          g->removeTransitiveEdges(read1);
        }
      }
    }
    // checkOverlap / checkOverlapForContainedRead against the device's answers
    for (UINT64 u = 1; u <= N; u++) {
      Read* r1 = ds->getReadFromID(u);
      for (Edge* e : *list(u)) {
        Read* r2 = e->getDestinationRead();
        UINT64 o, j;
        key_of(e, r1->getReadLength(), h, &o, &j);
        // an edge of graph[u] was discovered from u (key o at window j) or is the
        // twin of one discovered from its destination: check whichever side holds
        UINT64 o2, j2;
        key_of(e->getReverseEdge(), r2->getReadLength(), h, &o2, &j2);
        const bool fwd = g->checkOverlap(r1, r2, o, j), rev = g->checkOverlap(r2, r1, o2, j2);
        check(fwd || rev, "checkOverlap", u, r2->getReadNumber());
      }
      if (r1->superReadID && r1->getReadLength() <= 1024) {
        Read* sup = ds->getReadFromID(r1->superReadID);
        bool found = false;
        for (UINT64 o = 0; o < 4 && !found; o++)
          for (UINT64 j = 0; j + h <= sup->getReadLength() && !found; j++)
            found = (o % 2 == 0 || j >= r1->getReadLength() - h) && g->checkOverlapForContainedRead(sup, r1, o, j);
        check(found, "checkOverlapForContainedRead", r1->superReadID, u);
      }
    }
    g->saveGraphLists(prefix + ".graph");
    delete ht;  // the caller's table (buildOverlapGraphFromHashTable frees its own, :210)
    UINT64 counter, iters = 0;
    do {  // OverlapGraph.cpp:211-215
      counter = g->contractCompositePaths();
      counter += g->removeDeadEndNodes();
      iters++;
    } while (counter > 0);
    g->sortEdges();
    g->saveGraphToFile(prefix + ".unitig");
    std::printf("{\"unique_reads\": %llu, \"nodes\": %llu, \"directed_edges\": %llu, \"iterations\": %llu, "
                "\"check_failures\": %d}\n",
                (unsigned long long)N, (unsigned long long)g->getNumberOfNodes(),
                (unsigned long long)g->getNumberOfEdges(), (unsigned long long)iters, g_fail);
    delete g;
    delete ds;
  } catch (const std::exception& e) {
    std::fprintf(stderr, "mg_explore: %s\n", e.what());
    return 2;
  }
  return g_fail ? 3 : 0;
}
