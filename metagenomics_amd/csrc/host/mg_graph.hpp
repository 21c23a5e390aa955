// mg_graph.hpp — INTERNAL: host replay of the reference's graph construction
// order (exploration + transitive reduction) on the device's discovery rows.
// See mg_graph.cpp.
#ifndef MG_GRAPH_HPP_
#define MG_GRAPH_HPP_
#include <cstdint>
#include <vector>

#include "mg_overlap.h"

namespace mg {

struct GraphEdge {  // Edge (Edge.h:18-44) without the contraction fields
  uint32_t src, dst;
  uint16_t offset;
  uint8_t orient;
  uint8_t trans;  // transitiveRemovalFlag
  uint32_t rev;   // reverseEdge (index into the pool)
};

// One discovery of read A: window j, partner r2, key o (HashTable's 2-bit
// orientation) and the edge insertEdge(A, r2, orient, offset) would create
// (OverlapGraph.cpp:550-557).
struct Disc {
  uint32_t j;
  uint32_t r2;
  uint8_t o;
  uint8_t orient;
  uint16_t offset;
};

// D(A) for every read A, in insertAllEdgesOfRead's loop order (window j
// ascending, then getListOfReads order: partner ID, then key o;
// OverlapGraph.cpp:534-547, HashTable.cpp:58-60), from the device's directed
// discovery multiset.  D(A) = disc[start[A] .. start[A + 1]).
struct Discoveries {
  std::vector<uint64_t> start;
  std::vector<Disc> disc;
  // rows: the full directed multiset (any order); lens[id - 1]; h = l - 1.
  // 0 = ok, < 0 = rows inconsistent with the lengths / h.
  int build(const mg_edge* rows, uint64_t n_rows, const uint16_t* lens, uint64_t n_reads, uint32_t h);
};

class GraphReplay {
 public:
  GraphReplay();
  ~GraphReplay();
  GraphReplay(const GraphReplay&) = delete;
  GraphReplay& operator=(const GraphReplay&) = delete;
  // rows: the full directed discovery multiset (any order); lens[id - 1]; h = l - 1.
  // 0 = ok, < 0 = rows inconsistent with the lengths / h.
  int build(const mg_edge* rows, uint64_t n_rows, const uint16_t* lens, uint64_t n_reads, uint32_t h);
  std::vector<GraphEdge> pool;               // every Edge ever created (removed ones stay, unlisted)
  std::vector<std::vector<uint32_t>> lists;  // graph[u]: pool indices in list order
  uint64_t nodes = 0, edges = 0;             // numberOfNodes, numberOfEdges

 private:
  struct Impl;
  Impl* impl;
};

}  // namespace mg
#endif  // MG_GRAPH_HPP_
