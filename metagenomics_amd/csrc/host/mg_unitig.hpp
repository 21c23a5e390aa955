// mg_unitig.hpp — INTERNAL: the reference's unitig contraction
// (OverlapGraph.cpp:211-215, 669-988, 1048-1115) and its checkpoint writer
// (:1219-1261, :2799-2808) on the replayed graph.  See mg_unitig.cpp.
#ifndef MG_UNITIG_HPP_
#define MG_UNITIG_HPP_
#include <cstdint>
#include <cstdio>
#include <memory>
#include <vector>

#include "mg_graph.hpp"

namespace mg {

struct UnitigEdge {  // Edge (Edge.h:18-44): the fields the contraction reads or writes
  uint32_t src, dst;
  uint32_t rev;      // reverseEdge (index into the pool)
  uint8_t orient;    // overlapOrientation
  uint8_t alive;     // still listed (the reference deletes the object)
  uint16_t flow;     // Edge::flow (UINT16)
  uint64_t offset;   // overlapOffset (UINT64)
};

struct EdgeReads {  // listOfReads / listOfOverlapOffsets / listOfOrientations (Edge.h:30-32)
  std::vector<uint32_t> reads;
  std::vector<uint16_t> offs;
  std::vector<uint8_t> ors;
};

struct ReadLoc {  // one entry of Read::listOfEdges{Forward,Reverse} + locationOnEdge* (Read.h:39-42)
  uint32_t edge;
  uint64_t loc;
};

class UnitigGraph {
 public:
  // Takes the replayed pre-contraction graph (buildOverlapGraphFromHashTable
  // up to :209).  track_locations = maintain the per-read location lists.
  void init(const GraphReplay& g, uint64_t n_reads, bool track_locations);
  // the same from any pre-contraction edge pool + lists (a caller-driven build
  // through OverlapGraph::insertAllEdgesOfRead & co.); pool in creation order
  void init(const std::vector<GraphEdge>& gpool, const std::vector<std::vector<uint32_t>>& glists, uint64_t gnodes,
            uint64_t gedges, uint64_t n_reads, bool track_locations);
  // readGraphFromFile (:1270-1367): the .unitig checkpoint back into lists
  // (both edges of every line, twins rebuilt, read locations updated);
  // lens[id - 1].  0 ok, -1 cannot open, -2 malformed / read ID out of range.
  int read_unitig(const char* path, const uint16_t* lens, uint64_t n_reads, bool track_locations);
  // do { contractCompositePaths(); removeDeadEndNodes(); } while (changed)
  // (:211-215).  Returns the number of loop iterations; < 0 on an
  // orientation the reference would MYEXIT on ("Unable to merge.").
  int64_t contract();
  uint64_t contract_composite_paths();  // :669-696
  uint64_t remove_dead_end_nodes();     // :931-988
  void sort_edges();                    // :2799-2808
  // saveGraphToFile (:1219-1261); 0 ok, -1 open/write failure
  int save_unitig(const char* path) const;
  // every list in list order as "u v orient offset nreads r:o:d ..." rows,
  // then the read location lists (the oracle harness's "unitig" dump)
  int save_lists(const char* path) const;

  std::vector<UnitigEdge> pool;
  std::vector<std::unique_ptr<EdgeReads>> reads;  // per pool entry; null = no reads (simple edge)
  std::vector<std::vector<uint32_t>> lists;        // graph[u]
  std::vector<std::vector<ReadLoc>> loc_fwd, loc_rev;
  uint64_t nodes = 0, edges = 0;
  uint64_t merged_total = 0, dead_end_total = 0;
  bool flow_computed = false;
  bool track = true;
  bool bad_merge = false;

 private:
  uint32_t new_edge(uint32_t src, uint32_t dst, uint8_t orient, uint64_t offset, std::unique_ptr<EdgeReads> r);
  void insert(uint32_t e);
  void remove(uint32_t e);
  bool edge_present(uint32_t s, uint32_t d) const;
  void merge(uint32_t e1, uint32_t e2);
  void merge_list(uint32_t e1, uint32_t e2, EdgeReads& out) const;
  void update_locations(uint32_t e);
  void remove_locations(uint32_t e);
  size_t list_size(uint32_t e) const { return reads[e] ? reads[e]->reads.size() : 0; }
};

}  // namespace mg
#endif  // MG_UNITIG_HPP_
