// mg_graph.cpp — host replay of OverlapGraph::buildOverlapGraphFromHashTable's
// exploration and transitive reduction on the discovery
// multiset the device produced.  Paths relative to /root/reference/MetaGenomics.
//
// The device computes every discovery of every read at once:
// the directed multiset M.  The reference builds its graph in a specific order
// instead: a queue per component (OverlapGraph.cpp:144-204), each read's
// discoveries inserted when it is explored (insertAllEdgesOfRead :529-565,
// skipping partners already explored), each list sorted by overlap offset with
// std::sort (:563, unstable), and Myers' transitive reduction interleaved
// (markTransitiveEdges :574-615, removeTransitiveEdges :623-661).  The list
// ORDER, and with it which edges the reduction removes, depends on that order.
// This file replays it exactly:
//   * D(A), A's discoveries in the reference's loop order (window j ascending,
//     then getListOfReads order = partner ID, then key o; HashTable.cpp:58-60),
//     are the rows of M with src = A: j and o follow from (orient, offset)
//     (:550-557); a self-overlap's rows come twice in M (discovery + twin of
//     the symmetric discovery), so each self row counts once;
//   * the exploration, insertEdge (:390-419), std::sort (same libstdc++
//     algorithm and comparator -> the same permutation) and the reduction run
//     as in the reference on compact edge records instead of Edge objects.
// tests/test_graph_replay.py pins the result (list order, numberOfNodes,
// numberOfEdges) to the reference's own graph (oracle/_ref/ref_harness bfs).
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <vector>

#include "mg_graph.hpp"

namespace mg {

namespace {

enum : uint8_t { UNEXPLORED = 0, EXPLORED = 1, EXPLORED_AND_MARKED = 2 };  // nodeType (OverlapGraph.h:20-25)
enum : uint8_t { VACANT = 0, INPLAY = 1, ELIMINATED = 2 };                // markType (OverlapGraph.h:26-30)

inline uint8_t orient_to_key(uint8_t orient) {  // inverse of the switch at OverlapGraph.cpp:550-556
  return orient == 3 ? 0 : orient == 0 ? 1 : orient == 2 ? 2 : 3;
}

inline uint8_t twin_orient(uint8_t o) { return o == 0 ? 3 : (o == 3 ? 0 : o); }  // :841-855

}  // namespace

struct GraphReplay::Impl {
  const uint16_t* len = nullptr;
  uint64_t n = 0;
  uint32_t h = 0;
  std::vector<uint64_t> dstart;  // D(A) = disc[dstart[A] .. dstart[A+1])
  std::vector<Disc> disc;
  std::vector<uint8_t> state, marks;

  GraphReplay* g = nullptr;

  uint16_t L(uint64_t id) const { return len[id - 1]; }

  void insert(uint32_t e) {  // insertEdge(Edge*) :390-400
    const uint32_t src = g->pool[e].src;
    if (g->lists[src].empty()) g->nodes++;
    g->lists[src].push_back(e);
    g->edges++;
  }

  void insert_pair(uint32_t r1, uint32_t r2, uint8_t orient, uint16_t off) {  // insertEdge(Read*, ...) :407-419
    const uint32_t e1 = (uint32_t)g->pool.size();
    const uint16_t rev = (uint16_t)(L(r2) + off - L(r1));  // UINT16 arithmetic (:410)
    g->pool.push_back({r1, r2, off, orient, 0, e1 + 1});
    g->pool.push_back({r2, r1, rev, twin_orient(orient), 0, e1});
    insert(e1);
    insert(e1 + 1);
  }

  void explore(uint32_t r) {  // insertAllEdgesOfRead :529-565
    for (uint64_t k = dstart[r]; k < dstart[r + 1]; ++k) {
      const Disc& d = disc[k];
      if (state[d.r2] != UNEXPLORED) continue;  // :546
      insert_pair(r, d.r2, d.orient, d.offset);
    }
    auto& lst = g->lists[r];
    if (!lst.empty()) {
      const GraphEdge* pool = g->pool.data();
      std::sort(lst.begin(), lst.end(), [pool](uint32_t a, uint32_t b) { return pool[a].offset < pool[b].offset; });
    }
  }

  void mark_transitive(uint32_t u) {  // markTransitiveEdges :574-615
    auto& lu = g->lists[u];
    for (uint32_t e : lu) marks[g->pool[e].dst] = INPLAY;
    for (size_t i = 0; i < lu.size(); ++i) {
      const uint32_t v = g->pool[lu[i]].dst;
      if (marks[v] != INPLAY) continue;
      const uint8_t t1 = g->pool[lu[i]].orient;
      for (uint32_t e2 : g->lists[v]) {
        const uint32_t w = g->pool[e2].dst;
        if (marks[w] != INPLAY) continue;
        const uint8_t t2 = g->pool[e2].orient;
        if ((t1 == 0 || t1 == 2) && (t2 == 0 || t2 == 1))
          marks[w] = ELIMINATED;
        else if ((t1 == 1 || t1 == 3) && (t2 == 2 || t2 == 3))
          marks[w] = ELIMINATED;
      }
    }
    for (uint32_t e : lu) {
      if (marks[g->pool[e].dst] == ELIMINATED) {
        g->pool[e].trans = 1;
        g->pool[g->pool[e].rev].trans = 1;
      }
    }
    for (uint32_t e : lu) marks[g->pool[e].dst] = VACANT;
    marks[u] = VACANT;
  }

  void remove_transitive(uint32_t u) {  // removeTransitiveEdges :623-661
    auto& lu = g->lists[u];
    for (size_t i = 0; i < lu.size(); ++i) {
      if (!g->pool[lu[i]].trans) continue;
      const uint32_t twin = g->pool[lu[i]].rev;
      auto& lt = g->lists[g->pool[twin].src];
      for (size_t k = 0; k < lt.size(); ++k) {
        if (lt[k] == twin) {  // move the last edge into its place
          lt[k] = lt.back();
          lt.pop_back();
          if (lt.empty()) g->nodes--;
          g->edges--;
          break;
        }
      }
    }
    size_t j = 0;
    for (size_t i = 0; i < lu.size(); ++i) {
      if (!g->pool[lu[i]].trans)
        lu[j++] = lu[i];
      else
        g->edges--;
    }
    lu.resize(j);
    if (lu.empty()) g->nodes--;
  }

  void run() {  // OverlapGraph.cpp:144-204
    state.assign(n + 1, UNEXPLORED);
    marks.assign(n + 1, VACANT);
    std::vector<uint32_t> queue(n + 1, 0);
    for (uint64_t seed = 1; seed <= n; ++seed) {
      if (state[seed] != UNEXPLORED) continue;
      uint64_t head = 0, tail = 0;
      queue[tail++] = (uint32_t)seed;
      while (head < tail) {
        const uint32_t r1 = queue[head++];
        if (state[r1] == UNEXPLORED) {
          explore(r1);
          state[r1] = EXPLORED;
        }
        if (g->lists[r1].empty()) continue;
        if (state[r1] == EXPLORED) {
          for (size_t a = 0; a < g->lists[r1].size(); ++a) {  // the list may grow inside explore()
            const uint32_t r2 = g->pool[g->lists[r1][a]].dst;
            if (state[r2] == UNEXPLORED) {
              queue[tail++] = r2;
              explore(r2);
              state[r2] = EXPLORED;
            }
          }
          mark_transitive(r1);
          state[r1] = EXPLORED_AND_MARKED;
        }
        if (state[r1] == EXPLORED_AND_MARKED) {
          for (size_t a = 0; a < g->lists[r1].size(); ++a) {
            const uint32_t r2 = g->pool[g->lists[r1][a]].dst;
            if (state[r2] != EXPLORED) continue;
            for (size_t b = 0; b < g->lists[r2].size(); ++b) {
              const uint32_t r3 = g->pool[g->lists[r2][b]].dst;
              if (state[r3] == UNEXPLORED) {
                queue[tail++] = r3;
                explore(r3);
                state[r3] = EXPLORED;
              }
            }
            mark_transitive(r2);
            state[r2] = EXPLORED_AND_MARKED;
          }
          remove_transitive(r1);
        }
      }
    }
  }
};

GraphReplay::GraphReplay() : impl(new Impl) { impl->g = this; }
GraphReplay::~GraphReplay() { delete impl; }

int Discoveries::build(const mg_edge* rows, uint64_t n_rows, const uint16_t* lens, uint64_t n_reads, uint32_t h) {
  // D(A) from the rows with src = A (counting sort by src)
  start.assign(n_reads + 2, 0);
  for (uint64_t i = 0; i < n_rows; ++i) {
    if (rows[i].src < 1 || rows[i].src > n_reads || rows[i].dst < 1 || rows[i].dst > n_reads) return -1;
    start[rows[i].src + 1]++;
  }
  for (uint64_t a = 1; a <= n_reads + 1; ++a) start[a] += start[a - 1];
  disc.assign(n_rows, Disc{});
  {
    std::vector<uint64_t> at(start.begin(), start.end() - 1);
    for (uint64_t i = 0; i < n_rows; ++i) {
      const mg_edge& r = rows[i];
      const uint8_t o = orient_to_key(r.orient);
      const int64_t n1 = lens[r.src - 1];
      // window j: offset = j for o = 0, 2; offset = n1 - h - j for o = 1, 3 (:550-557)
      const int64_t j = (o == 0 || o == 2) ? r.offset : n1 - (int64_t)h - r.offset;
      if (j < 1 || j >= n1 - (int64_t)h) return -2;
      disc[at[r.src]++] = Disc{(uint32_t)j, r.dst, o, r.orient, r.offset};
    }
  }
  // loop order; each self row is present twice in M and counts once
  for (uint64_t a = 1; a <= n_reads; ++a) {
    const uint64_t lo = start[a], hi = start[a + 1];
    std::sort(disc.begin() + lo, disc.begin() + hi, [](const Disc& x, const Disc& y) {
      if (x.j != y.j) return x.j < y.j;
      if (x.r2 != y.r2) return x.r2 < y.r2;
      return x.o < y.o;
    });
  }
  uint64_t w = 0;
  std::vector<uint64_t> ns(n_reads + 2, 0);
  for (uint64_t a = 1; a <= n_reads; ++a) {
    ns[a] = w;
    const uint64_t lo = start[a], hi = start[a + 1];
    for (uint64_t k = lo; k < hi; ++k) {
      const Disc& d = disc[k];
      if (d.r2 == a) {
        if (k + 1 >= hi || std::memcmp(&disc[k + 1], &d, sizeof(Disc)) != 0) return -3;  // must come in pairs
        disc[w++] = d;
        ++k;
      } else {
        disc[w++] = d;
      }
    }
  }
  ns[n_reads + 1] = w;
  ns[0] = 0;
  start.swap(ns);
  disc.resize(w);
  return 0;
}

int GraphReplay::build(const mg_edge* rows, uint64_t n_rows, const uint16_t* lens, uint64_t n_reads, uint32_t h) {
  Impl& I = *impl;
  I.len = lens;
  I.n = n_reads;
  I.h = h;
  pool.clear();
  lists.assign(n_reads + 1, {});
  nodes = edges = 0;
  Discoveries D;
  const int rc = D.build(rows, n_rows, lens, n_reads, h);
  if (rc) return rc;
  I.dstart.swap(D.start);
  I.disc.swap(D.disc);
  pool.reserve(n_rows);
  I.run();
  return 0;
}

}  // namespace mg
