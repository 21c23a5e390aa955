// mg_unitig.cpp — the reference's unitig contraction loop and its .unitig
// checkpoint writer on the replayed graph (mg_graph.cpp).
// Paths relative to /root/reference/MetaGenomics.
//
// new OverlapGraph(ht) ends with (OverlapGraph.cpp:211-215)
//     do { counter = contractCompositePaths(); counter += removeDeadEndNodes(); } while (counter > 0);
// and main.cpp:48-50 then calls sortEdges() and saveGraphToFile(prefix.unitig).
// The contraction is a sequential rewrite of the lists whose result depends on
// list order at every step (which two edges a degree-2 node holds, where
// swap-with-last removal moves an edge), so it runs here exactly as the
// reference runs it, on compact edge records instead of heap Edge objects:
//   * contractCompositePaths :669-696, mergeEdges :704-759, mergeList :766-794,
//     mergedEdgeOrientation :811-834, removeEdge :863-896;
//   * removeDeadEndNodes :931-988 (deadEndLength = 10, Common.h:42);
//   * updateReadLocations / removeReadLocations :1048-1115 (per-read lists of
//     the composite edges containing the read, with its distance on the edge);
//   * sortEdges :2799-2808 (std::sort by destination ID: the same libstdc++
//     algorithm on the same sequence gives the same permutation);
//   * saveGraphToFile :1219-1261.
// Widths follow the reference: overlapOffset is UINT64 (sums of merged edges do
// not wrap), listOfOverlapOffsets entries are UINT16 (mergeList's
// "edge1 offset - sum" is truncated), flow is UINT16.
// The one value the reference leaves to the allocator: a self-loop pair is
// written once, for the Edge object with the lower ADDRESS (:1236).  Here the
// lower pool index (the forward edge of mergeEdges, allocated first) is written.
// tests/test_unitig.py pins lists, counters, read locations and the .unitig
// file to the reference's own run (oracle/_ref/ref_harness unitig).
#include "mg_unitig.hpp"

#include <algorithm>
#include <cinttypes>
#include <cstring>

namespace mg {

namespace {

constexpr size_t kDeadEndLength = 10;  // Common.h:42

inline uint8_t twin_orient(uint8_t o) { return o == 0 ? 3 : (o == 3 ? 0 : o); }  // :841-855

// matchEdgeType (OverlapGraph.cpp:19-26)
inline bool match_edge_type(uint8_t t1, uint8_t t2) {
  if ((t1 == 1 || t1 == 3) && (t2 == 2 || t2 == 3)) return true;
  if ((t1 == 0 || t1 == 2) && (t2 == 0 || t2 == 1)) return true;
  return false;
}

// mergedEdgeOrientation (:811-834); 255 = the MYEXIT branch
inline uint8_t merged_orient(uint8_t a, uint8_t b) {
  if (a == 0 && b == 0) return 0;
  if (a == 0 && b == 1) return 1;
  if (a == 1 && b == 2) return 0;
  if (a == 1 && b == 3) return 1;
  if (a == 2 && b == 0) return 2;
  if (a == 2 && b == 1) return 3;
  if (a == 3 && b == 2) return 2;
  if (a == 3 && b == 3) return 3;
  return 255;
}

// buffered text writer for the checkpoint files
struct Out {
  FILE* f;
  std::vector<char> buf;
  size_t n = 0;
  bool ok = true;
  explicit Out(FILE* fp) : f(fp), buf(1 << 20) {}
  void flush() {
    if (n && std::fwrite(buf.data(), 1, n, f) != n) ok = false;
    n = 0;
  }
  void put(const char* s, size_t k) {
    if (n + k > buf.size()) flush();
    std::memcpy(buf.data() + n, s, k);
    n += k;
  }
  void u64(uint64_t v) {
    char t[24];
    int k = 0;
    do {
      t[k++] = (char)('0' + v % 10);
      v /= 10;
    } while (v);
    if (n + k + 1 > buf.size()) flush();
    while (k) buf[n++] = t[--k];
  }
  void ch(char c) {
    if (n + 1 > buf.size()) flush();
    buf[n++] = c;
  }
};

}  // namespace

void UnitigGraph::init(const GraphReplay& g, uint64_t n_reads, bool track_locations) {
  init(g.pool, g.lists, g.nodes, g.edges, n_reads, track_locations);
}

void UnitigGraph::init(const std::vector<GraphEdge>& gpool, const std::vector<std::vector<uint32_t>>& glists,
                       uint64_t gnodes, uint64_t gedges, uint64_t n_reads, bool track_locations) {
  track = track_locations;
  pool.clear();
  reads.clear();
  lists.assign(n_reads + 1, {});
  // keep only the listed edges (the transitive ones were deleted), renumbered
  // in creation order (insertEdge(Read*,...) allocates the edge before its twin)
  std::vector<uint32_t> id(gpool.size(), UINT32_MAX);
  uint64_t listed = 0;
  for (size_t u = 1; u < glists.size() && u <= n_reads; ++u) {
    listed += glists[u].size();
    for (uint32_t e : glists[u]) id[e] = 0;
  }
  pool.reserve(listed + listed / 2 + 16);
  for (size_t e = 0; e < gpool.size(); ++e) {
    if (id[e] == UINT32_MAX) continue;
    id[e] = (uint32_t)pool.size();
    const GraphEdge& x = gpool[e];
    pool.push_back(UnitigEdge{x.src, x.dst, UINT32_MAX, x.orient, 1, 0, x.offset});
  }
  for (size_t e = 0; e < gpool.size(); ++e)
    if (id[e] != UINT32_MAX) pool[id[e]].rev = id[gpool[e].rev];
  for (size_t u = 1; u < glists.size() && u <= n_reads; ++u)
    for (uint32_t e : glists[u]) lists[u].push_back(id[e]);
  reads.resize(pool.size());
  nodes = gnodes;
  edges = gedges;
  loc_fwd.clear();
  loc_rev.clear();
  if (track) {
    loc_fwd.resize(n_reads + 1);
    loc_rev.resize(n_reads + 1);
  }
  merged_total = dead_end_total = 0;
  bad_merge = false;
}

int UnitigGraph::read_unitig(const char* path, const uint16_t* lens, uint64_t n_reads, bool track_locations) {
  FILE* f = std::fopen(path, "rb");
  if (!f) return -1;  // "Unable to open file: " (:1276)
  std::vector<char> text;
  {
    char buf[1 << 16];
    size_t k;
    while ((k = std::fread(buf, 1, sizeof buf, f)) > 0) text.insert(text.end(), buf, buf + k);
    std::fclose(f);
  }
  // while (good()) { file >> temp; list.push_back(temp); } (:1289-1294): every
  // number, plus the value of the extraction that hits the end of the file
  // when the last number is followed by whitespace (or the file is empty)
  std::vector<uint64_t> vals;
  bool in_num = false, bad = false;
  uint64_t cur = 0;
  for (char c : text) {
    if (c >= '0' && c <= '9') {
      cur = cur * 10 + (uint64_t)(c - '0');
      in_num = true;
    } else if (c == ' ' || c == '\n' || c == '\t' || c == '\r' || c == '\v' || c == '\f') {
      if (in_num) vals.push_back(cur);
      in_num = false;
      cur = 0;
    } else {
      bad = true;
      break;
    }
  }
  if (bad) return -2;
  const bool trailing = !in_num;  // the last extraction failed at the end of the file
  if (in_num) vals.push_back(cur);
  const uint64_t size = vals.size() + (trailing ? 1 : 0);
  track = track_locations;
  pool.clear();
  reads.clear();
  lists.assign(n_reads + 1, {});
  loc_fwd.clear();
  loc_rev.clear();
  if (track) {
    loc_fwd.resize(n_reads + 1);
    loc_rev.resize(n_reads + 1);
  }
  nodes = edges = merged_total = dead_end_total = 0;
  bad_merge = false;
  flow_computed = false;
  auto at = [&](uint64_t i, uint64_t* v) {
    if (i >= vals.size()) return false;
    *v = vals[i];
    return true;
  };
  auto len = [&](uint64_t id) -> uint64_t { return lens[id - 1]; };
  for (uint64_t i = 0; i + 1 < size;) {  // (:1297-1363)
    uint64_t src, dst, orient, offset, nr;
    if (!at(i, &src) || !at(i + 1, &dst) || !at(i + 2, &orient) || !at(i + 3, &offset) || !at(i + 4, &nr))
      return -2;
    i += 5;
    if (src < 1 || src > n_reads || dst < 1 || dst > n_reads) return -2;  // getReadFromID's range check
    if (nr > (vals.size() - i) / 3) return -2;
    auto fr = std::make_unique<EdgeReads>();
    uint64_t length = 0;
    for (uint64_t j = 0; j < 3 * nr; j += 3) {
      fr->reads.push_back((uint32_t)vals[i + j]);
      fr->offs.push_back((uint16_t)vals[i + j + 1]);  // vector<UINT16>
      fr->ors.push_back((uint8_t)vals[i + j + 2]);    // vector<UINT8>
      length += vals[i + j + 1];
    }
    for (uint32_t r : fr->reads)
      if (r < 1 || r > n_reads) return -2;
    // the reverse edge's lists from the forward ones (:1322-1343)
    auto rr = std::make_unique<EdgeReads>();
    const uint64_t sz = fr->reads.size();
    for (uint64_t j = 0; j < sz; ++j) {
      rr->reads.push_back(fr->reads[sz - j - 1]);
      uint64_t length1, fwd;
      if (j == 0) {  // last / first read
        length1 = len(dst);
        fwd = offset - length;
      } else {
        length1 = len(fr->reads[sz - j]);
        fwd = fr->offs[sz - j];
      }
      const uint64_t length2 = len(fr->reads[sz - j - 1]);
      rr->offs.push_back((uint16_t)(length1 + fwd - length2));
      rr->ors.push_back((uint8_t)!fr->ors[sz - j - 1]);
    }
    const uint64_t rev_offset = offset + len(dst) - len(src);
    const uint32_t e1 = new_edge((uint32_t)src, (uint32_t)dst, (uint8_t)orient, offset, std::move(fr));
    const uint32_t e2 = new_edge((uint32_t)dst, (uint32_t)src, twin_orient((uint8_t)orient), rev_offset, std::move(rr));
    pool[e1].rev = e2;
    pool[e2].rev = e1;
    insert(e1);
    insert(e2);
    i += nr * 3;
  }
  return 0;
}

uint32_t UnitigGraph::new_edge(uint32_t src, uint32_t dst, uint8_t orient, uint64_t offset,
                               std::unique_ptr<EdgeReads> r) {  // Edge::makeEdge (Edge.cpp:103-116): flow = 0
  const uint32_t e = (uint32_t)pool.size();
  pool.push_back(UnitigEdge{src, dst, UINT32_MAX, orient, 1, 0, offset});
  if (r && r->reads.empty()) r.reset();
  reads.push_back(std::move(r));
  return e;
}

void UnitigGraph::insert(uint32_t e) {  // insertEdge(Edge*) :390-400
  auto& l = lists[pool[e].src];
  if (l.empty()) nodes++;
  l.push_back(e);
  edges++;
  update_locations(e);
}

void UnitigGraph::update_locations(uint32_t e) {  // updateReadLocations :1048-1073
  if (!track || !reads[e]) return;
  const EdgeReads& r = *reads[e];
  uint64_t distance = 0;
  for (size_t i = 0; i < r.reads.size(); ++i) {
    distance += r.offs[i];
    if (r.ors[i] == 1)
      loc_fwd[r.reads[i]].push_back(ReadLoc{e, distance});
    else
      loc_rev[r.reads[i]].push_back(ReadLoc{e, distance});
  }
}

void UnitigGraph::remove_locations(uint32_t e) {  // removeReadLocations :1081-1115
  if (!track || !reads[e]) return;
  const EdgeReads& r = *reads[e];
  for (size_t i = 0; i < r.reads.size(); ++i) {
    for (auto* lst : {&loc_fwd[r.reads[i]], &loc_rev[r.reads[i]]}) {
      // the reference advances j after moving the last entry into slot j, so
      // the moved entry is not looked at again in this pass
      for (size_t j = 0; j < lst->size(); ++j) {
        if ((*lst)[j].edge == e) {
          (*lst)[j] = lst->back();
          lst->pop_back();
        }
      }
    }
  }
}

void UnitigGraph::remove(uint32_t e) {  // removeEdge :863-896
  const uint32_t twin = pool[e].rev;
  remove_locations(e);
  remove_locations(twin);
  const uint32_t id1 = pool[e].src, id2 = pool[e].dst;
  for (int pass = 0; pass < 2; ++pass) {  // the twin first (in graph[ID2]), then the edge (in graph[ID1])
    const uint32_t target = pass == 0 ? twin : e;
    auto& l = lists[pass == 0 ? id2 : id1];
    for (size_t i = 0; i < l.size(); ++i) {
      if (l[i] == target) {
        l[i] = l.back();
        l.pop_back();
        if (l.empty()) nodes--;
        edges--;
        pool[target].alive = 0;
        reads[target].reset();  // delete
        break;
      }
    }
  }
}

bool UnitigGraph::edge_present(uint32_t s, uint32_t d) const {  // isEdgePresent :1599-1607
  for (uint32_t e : lists[s])
    if (pool[e].dst == d) return true;
  return false;
}

void UnitigGraph::merge_list(uint32_t e1, uint32_t e2, EdgeReads& out) const {  // mergeList :766-794
  uint64_t sum = 0;
  if (reads[e1]) {
    const EdgeReads& a = *reads[e1];
    out.reads = a.reads;
    out.offs = a.offs;
    out.ors = a.ors;
    for (uint16_t o : a.offs) sum += o;
  }
  out.reads.push_back(pool[e1].dst);  // the common node
  out.offs.push_back((uint16_t)(pool[e1].offset - sum));
  out.ors.push_back((pool[e1].orient == 1 || pool[e1].orient == 3) ? 1 : 0);
  if (reads[e2]) {
    const EdgeReads& b = *reads[e2];
    out.reads.insert(out.reads.end(), b.reads.begin(), b.reads.end());
    out.offs.insert(out.offs.end(), b.offs.begin(), b.offs.end());
    out.ors.insert(out.ors.end(), b.ors.begin(), b.ors.end());
  }
}

void UnitigGraph::merge(uint32_t e1, uint32_t e2) {  // mergeEdges :704-759
  const uint8_t of = merged_orient(pool[e1].orient, pool[e2].orient);
  if (of == 255) {
    bad_merge = true;
    return;
  }
  const uint8_t orr = twin_orient(of);
  const uint32_t r1 = pool[e1].src, r2 = pool[e2].dst;
  const uint32_t e1r = pool[e1].rev, e2r = pool[e2].rev;
  auto lf = std::make_unique<EdgeReads>();
  merge_list(e1, e2, *lf);
  auto lr = std::make_unique<EdgeReads>();
  merge_list(e2r, e1r, *lr);
  const uint64_t off_f = pool[e1].offset + pool[e2].offset;
  const uint64_t off_r = pool[e2r].offset + pool[e1r].offset;
  const uint32_t ef = new_edge(r1, r2, of, off_f, std::move(lf));
  const uint32_t er = new_edge(r2, r1, orr, off_r, std::move(lr));
  pool[ef].rev = er;
  pool[er].rev = ef;
  const uint16_t flow = std::min(pool[e1].flow, pool[e2].flow);
  pool[ef].flow = flow;
  pool[er].flow = flow;
  insert(ef);
  insert(er);
  pool[e1].flow = (uint16_t)(pool[e1].flow - flow);
  pool[pool[e1].rev].flow = pool[e1].flow;
  pool[e2].flow = (uint16_t)(pool[e2].flow - flow);
  pool[pool[e2].rev].flow = pool[e2].flow;
  if (pool[e1].flow == 0 || flow == 0) remove(e1);
  if (pool[e2].flow == 0 || flow == 0) remove(e2);
}

uint64_t UnitigGraph::contract_composite_paths() {  // :669-696
  uint64_t counter = 0;
  for (size_t index = 1; index < lists.size(); ++index) {
    if (lists[index].size() != 2) continue;
    const uint32_t a = lists[index][0], b = lists[index][1];
    if (flow_computed || !edge_present(pool[a].dst, pool[b].dst)) {
      if (match_edge_type(pool[pool[a].rev].orient, pool[b].orient) && pool[a].src != pool[a].dst) {
        merge(pool[a].rev, b);
        if (bad_merge) return counter;
        counter++;
      }
    }
  }
  merged_total += counter;
  return counter;
}

uint64_t UnitigGraph::remove_dead_end_nodes() {  // :931-988
  std::vector<uint32_t> nodes_out;
  for (size_t i = 1; i < lists.size(); ++i) {
    if (lists[i].empty()) continue;
    bool flag = false;
    uint64_t in = 0, out = 0;
    for (uint32_t e : lists[i]) {
      if (list_size(e) > kDeadEndLength || pool[e].src == pool[e].dst) {
        flag = true;
        break;
      }
      if (pool[e].orient == 0 || pool[e].orient == 1)
        in++;
      else
        out++;
    }
    if (!flag && ((in > 0 && out == 0) || (in == 0 && out > 0))) nodes_out.push_back((uint32_t)i);
  }
  std::vector<uint32_t> copy;
  for (uint32_t u : nodes_out) {
    if (lists[u].empty()) continue;
    copy = lists[u];
    for (uint32_t e : copy) remove(e);
  }
  dead_end_total += nodes_out.size();
  return nodes_out.size();
}

int64_t UnitigGraph::contract() {
  int64_t iters = 0;
  uint64_t counter = 0;
  do {
    counter = contract_composite_paths();
    if (bad_merge) return -1;
    counter += remove_dead_end_nodes();
    iters++;
  } while (counter > 0);
  return iters;
}

void UnitigGraph::sort_edges() {  // :2799-2808
  const UnitigEdge* p = pool.data();
  for (size_t i = 1; i < lists.size(); ++i)
    if (!lists[i].empty())
      std::sort(lists[i].begin(), lists[i].end(), [p](uint32_t a, uint32_t b) { return p[a].dst < p[b].dst; });
}

int UnitigGraph::save_unitig(const char* path) const {  // saveGraphToFile :1219-1261
  FILE* f = std::fopen(path, "w");
  if (!f) return -1;
  Out o(f);
  for (size_t i = 1; i < lists.size(); ++i) {
    for (uint32_t e : lists[i]) {
      const UnitigEdge& x = pool[e];
      if (!(x.src < x.dst || (x.src == x.dst && e < x.rev))) continue;
      o.u64(x.src), o.ch('\n');
      o.u64(x.dst), o.ch('\n');
      o.u64(x.orient), o.ch('\n');
      o.u64(x.offset), o.ch('\n');
      o.u64(list_size(e)), o.ch('\n');
      if (reads[e]) {
        const EdgeReads& r = *reads[e];
        for (size_t k = 0; k < r.reads.size(); ++k) {
          o.u64(r.reads[k]), o.ch('\n');
          o.u64(r.offs[k]), o.ch('\n');
          o.u64(r.ors[k]), o.ch('\n');
        }
      }
    }
  }
  o.flush();
  const bool ok = o.ok && std::fclose(f) == 0;
  return ok ? 0 : -1;
}

int UnitigGraph::save_lists(const char* path) const {
  FILE* f = std::fopen(path, "w");
  if (!f) return -1;
  Out o(f);
  for (size_t u = 1; u < lists.size(); ++u) {
    for (uint32_t e : lists[u]) {
      const UnitigEdge& x = pool[e];
      o.u64(u), o.ch(' '), o.u64(x.dst), o.ch(' '), o.u64(x.orient), o.ch(' '), o.u64(x.offset), o.ch(' ');
      o.u64(list_size(e));
      if (reads[e]) {
        const EdgeReads& r = *reads[e];
        for (size_t k = 0; k < r.reads.size(); ++k) {
          o.ch(' '), o.u64(r.reads[k]), o.ch(':'), o.u64(r.offs[k]), o.ch(':'), o.u64(r.ors[k]);
        }
      }
      o.ch('\n');
    }
  }
  if (track) {
    for (size_t r = 1; r < loc_fwd.size(); ++r) {
      for (int side = 0; side < 2; ++side) {
        for (const ReadLoc& L : side ? loc_rev[r] : loc_fwd[r]) {
          const UnitigEdge& x = pool[L.edge];
          o.ch(side ? 'R' : 'F'), o.ch(' '), o.u64(r), o.ch(' '), o.u64(x.src), o.ch(' '), o.u64(x.dst), o.ch(' ');
          o.u64(x.orient), o.ch(' '), o.u64(x.offset), o.ch(' '), o.u64(L.loc), o.ch('\n');
        }
      }
    }
  }
  o.flush();
  const bool ok = o.ok && std::fclose(f) == 0;
  return ok ? 0 : -1;
}

}  // namespace mg
