// ref_harness.cpp — TEST INFRASTRUCTURE ONLY (oracle/). Never linked into the product.
//
// Driver that runs the *reference* C++ classes (compiled in place from
// /root/reference/MetaGenomics by oracle/Makefile into oracle/_ref/) to produce
// golden vectors and the "reference" CPU baseline.  No reference source is
// copied: this file only #includes the reference headers where they lie.
//
// Modes
//   edges  <fasta> <l> <out>   : discovery harness (SURVEY §0 recipe):
//        Dataset(pe={}, se={fa}, l) -> HashTable::insertDataset(ds,l)
//        (HashTable.cpp:50-80) -> markContainedReads (OverlapGraph.cpp:225-290)
//        -> insertAllEdgesOfRead(i, explored) for i = 1..N in ID order,
//        marking i EXPLORED after each call (OverlapGraph.cpp:529-565).
//        Writes  "#N <n>", "#S <id> <super>" for every contained read,
//        "#R <id> <canonical forward string>" and one "u v orient offset"
//        row per directed Edge in graph[u].
//   time   <fasta> <l> <out>   : the shipped path timing used by SURVEY §6:
//        wall time of insertDataset + new OverlapGraph(ht)
//        (main.cpp:45-47, includes transitive reduction + contraction).
//   disc   <fasta> <l> <out>   : wall time of insertDataset + markContainedReads +
//        the ID-order discovery loop (no transitive reduction), plus the raw
//        directed edge count.  This is the apples-to-apples CPU figure for the
//        GPU path, which also stops at the raw edge multiset.
//   digest <fasta> <l> <out>   : as edges, but instead of dumping the rows it
//        folds every directed Edge of graph[u] into the order-independent
//        digest of oracle/mg_digest.h as soon as u is explored (graph[u] is
//        final then: later reads skip explored partners, :546) and frees it, so
//        10^8-row configs (C3) fit in host memory.  Writes one JSON line with
//        the row digest, the superReadID digest and the phase times.
//   hash   <fasta> <l> <out>   : HashTable::getHashTableSize() and
//        hashFunction(key) (HashTable.cpp:20-29,56,135-155) for the four keys
//        of the first 64 reads (hashRead's order, :88-104): "#P <size>" then
//        "<key> <hash>" lines.
//   lookup <fasta> <l> <out> <key>... : HashTable::getListOfReads(key)
//        (HashTable.cpp:202-221) for each key, in the reference list order.
//   bfs    <fasta> <l> <out>   : the graph as buildOverlapGraphFromHashTable
//        leaves it before its contraction loop (OverlapGraph.cpp:107-209):
//        markContainedReads, then the component-by-component exploration with
//        the reference's own insertAllEdgesOfRead / markTransitiveEdges /
//        removeTransitiveEdges (the driving loop of :144-204 restated here,
//        since the reference inlines it ahead of the contraction at :211-215).
//        Writes "#C <numberOfNodes> <numberOfEdges>" and every graph[u] list
//        IN LIST ORDER as "u v orient offset" rows.
//   dataset <fasta> <l> <out>  : Dataset(pe={}, se={fa}, l) only: "#N <unique>",
//        "#G <numberOfReads>", "#R <id> <string>" (Dataset.cpp:39-65,110-193).
//   dstime <fasta> <l> <out>   : "#T <seconds>" of the Dataset constructor alone.
//   unitig <fasta> <l> <out>   : as bfs, then the reference's own contraction
//        loop (OverlapGraph.cpp:211-215: contractCompositePaths +
//        removeDeadEndNodes until neither changes anything), i.e. the graph
//        new OverlapGraph(ht) returns (main.cpp:47).  Writes
//        "#C <numberOfNodes> <numberOfEdges>", "#I <loop iterations>", every
//        graph[u] list IN LIST ORDER as "u v orient offset nreads r:o:d ..."
//        rows (the edge's listOfReads / listOfOverlapOffsets /
//        listOfOrientations), then every read's location lists
//        (Read.h:39-42, maintained by :1048-1115) as
//        "F|R <read> <src> <dst> <orient> <offset> <location>" rows; then
//        sortEdges (:2799-2808) and saveGraphToFile (:1219-1261) into
//        <out>.unitig (main.cpp:49-50).
//   reread <fasta> <l> <out> <unitig> : main.cpp:36-42's resume from a
//        .unitig checkpoint: OverlapGraph() -> setDataset -> readGraphFromFile
//        (OverlapGraph.cpp:1270-1367); writes "#C", the lists and the read
//        location lists as the unitig mode does, then sortEdges and
//        saveGraphToFile into <out>.unitig.
#define private public
#include "Dataset.h"
#include "HashTable.h"
#include "OverlapGraph.h"
#undef private

#include <time.h>
#include <cstdio>

#include "mg_digest.h"
#include <cstring>

static double now_s() {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec + 1e-9 * ts.tv_nsec;
}

// Silence the reference's progress chatter (it writes to std::cout).
struct NullBuf : std::streambuf {
  int overflow(int c) { return c; }
};

static OverlapGraph* prepare_graph(Dataset* ds, HashTable* ht) {
  OverlapGraph* og = new OverlapGraph();
  og->hashTable = ht;
  og->dataSet = ds;
  og->graph = new vector<vector<Edge*>*>;
  for (UINT64 i = 0; i <= ds->getNumberOfUniqueReads(); i++) og->graph->push_back(new vector<Edge*>);
  return og;
}

static void discovery(OverlapGraph* og, Dataset* ds) {
  og->markContainedReads();
  vector<nodeType> explored(ds->getNumberOfUniqueReads() + 1, UNEXPLORED);
  for (UINT64 i = 1; i <= ds->getNumberOfUniqueReads(); i++) {
    og->insertAllEdgesOfRead(i, &explored);
    explored[i] = EXPLORED;
  }
}

// Exploration order of OverlapGraph.cpp:144-204: a queue per component; a
// popped read is explored if needed, its unexplored neighbours are explored
// and queued, its transitive edges marked; then each explored-but-unmarked
// neighbour queues its own unexplored neighbours and gets its transitive edges
// marked, and the popped read's transitive edges are removed.
static void explore_components(OverlapGraph* og, Dataset* ds) {
  const UINT64 N = ds->getNumberOfUniqueReads();
  vector<nodeType> state(N + 1, UNEXPLORED);
  vector<markType> marks(N + 1, VACANT);
  vector<UINT64> queue(N + 1, 0);
  og->markContainedReads();
  for (UINT64 seed = 1; seed <= N; seed++) {
    if (state[seed] != UNEXPLORED) continue;
    UINT64 head = 0, tail = 0;
    queue[tail++] = seed;
    while (head < tail) {
      const UINT64 u = queue[head++];
      if (state[u] == UNEXPLORED) {
        og->insertAllEdgesOfRead(u, &state);
        state[u] = EXPLORED;
      }
      if (og->graph->at(u)->empty()) continue;
      if (state[u] == EXPLORED) {
        for (UINT64 a = 0; a < og->graph->at(u)->size(); a++) {
          const UINT64 v = og->graph->at(u)->at(a)->getDestinationRead()->getReadNumber();
          if (state[v] == UNEXPLORED) {
            queue[tail++] = v;
            og->insertAllEdgesOfRead(v, &state);
            state[v] = EXPLORED;
          }
        }
        og->markTransitiveEdges(u, &marks);
        state[u] = EXPLORED_AND_TRANSITIVE_EDGES_MARKED;
      }
      if (state[u] == EXPLORED_AND_TRANSITIVE_EDGES_MARKED) {
        for (UINT64 a = 0; a < og->graph->at(u)->size(); a++) {
          const UINT64 v = og->graph->at(u)->at(a)->getDestinationRead()->getReadNumber();
          if (state[v] != EXPLORED) continue;
          for (UINT64 b = 0; b < og->graph->at(v)->size(); b++) {
            const UINT64 w = og->graph->at(v)->at(b)->getDestinationRead()->getReadNumber();
            if (state[w] == UNEXPLORED) {
              queue[tail++] = w;
              og->insertAllEdgesOfRead(w, &state);
              state[w] = EXPLORED;
            }
          }
          og->markTransitiveEdges(v, &marks);
          state[v] = EXPLORED_AND_TRANSITIVE_EDGES_MARKED;
        }
        og->removeTransitiveEdges(u);
      }
    }
  }
}

int main(int argc, char** argv) {
  if (argc < 5) {
    fprintf(stderr, "usage: %s edges|time|disc|lookup <fasta> <l> <out> [keys...]\n", argv[0]);
    return 2;
  }
  const char* mode = argv[1];
  string fasta = argv[2];
  UINT64 l = strtoull(argv[3], 0, 10);
  FILE* out = fopen(argv[4], "w");
  if (!out) { perror("open out"); return 2; }
  NullBuf nb;
  std::streambuf* old = std::cout.rdbuf(&nb);

  vector<string> pe, se;
  se.push_back(fasta);
  double t0 = now_s();
  Dataset* ds = new Dataset(pe, se, l);
  double t_ds = now_s() - t0;
  UINT64 N = ds->getNumberOfUniqueReads();

  if (!strcmp(mode, "dstime")) {
    fprintf(out, "#T %.6f\n", t_ds);
  } else if (!strcmp(mode, "dataset")) {
    fprintf(out, "#N %llu\n#G %llu\n", (unsigned long long)N, (unsigned long long)ds->getNumberOfReads());
    for (UINT64 i = 1; i <= N; i++)
      fprintf(out, "#R %llu %s\n", (unsigned long long)i, ds->getReadFromID(i)->getStringForward().c_str());
  } else if (!strcmp(mode, "time")) {
    double t1 = now_s();
    HashTable* ht = new HashTable();
    ht->insertDataset(ds, l);
    double t2 = now_s();
    OverlapGraph* og = new OverlapGraph(ht);  // deletes ht (OverlapGraph.cpp:210)
    double t3 = now_s();
    fprintf(out, "{\"n_unique\": %llu, \"dataset_s\": %.6f, \"hash_s\": %.6f, \"graph_s\": %.6f}\n",
            (unsigned long long)N, t_ds, t2 - t1, t3 - t2);
    (void)og;
  } else if (!strcmp(mode, "disc")) {
    double t1 = now_s();
    HashTable* ht = new HashTable();
    ht->insertDataset(ds, l);
    double t2 = now_s();
    OverlapGraph* og = prepare_graph(ds, ht);
    discovery(og, ds);
    double t3 = now_s();
    unsigned long long rows = 0;
    for (UINT64 u = 1; u <= N; u++) rows += og->graph->at(u)->size();
    fprintf(out, "{\"n_unique\": %llu, \"dataset_s\": %.6f, \"hash_s\": %.6f, \"discovery_s\": %.6f, \"directed_rows\": %llu}\n",
            (unsigned long long)N, t_ds, t2 - t1, t3 - t2, rows);
  } else if (!strcmp(mode, "digest")) {
    double t1 = now_s();
    HashTable* ht = new HashTable();
    ht->insertDataset(ds, l);
    double t2 = now_s();
    OverlapGraph* og = prepare_graph(ds, ht);
    og->markContainedReads();
    double t3 = now_s();
    mgo_digest sd = {0, 0, 0, 0}, rd = {0, 0, 0, 0};
    for (UINT64 i = 1; i <= N; i++) {
      Read* r = ds->getReadFromID(i);
      if (r->superReadID) mgo_digest_add(&sd, mgo_super_hash(i, r->superReadID));
    }
    vector<nodeType> explored(N + 1, UNEXPLORED);
    for (UINT64 u = 1; u <= N; u++) {
      og->insertAllEdgesOfRead(u, &explored);
      explored[u] = EXPLORED;
      vector<Edge*>* lst = og->graph->at(u);
      for (size_t k = 0; k < lst->size(); k++) {
        Edge* e = lst->at(k);
        mgo_digest_add(&rd, mgo_row_hash(u, e->getDestinationRead()->getReadNumber(), e->getOrientation(),
                                         e->getOverlapOffset()));
        delete e;  // its twin (in an unexplored list) is never dereferenced again
      }
      vector<Edge*>().swap(*lst);
    }
    double t4 = now_s();
    fprintf(out,
            "{\"n_unique\": %llu, \"n_reads\": %llu, \"directed_rows\": %llu, \"rows_sum\": %llu, "
            "\"rows_xor\": %llu, \"rows_sum2\": %llu, \"contained\": %llu, \"super_sum\": %llu, "
            "\"super_xor\": %llu, \"super_sum2\": %llu, \"dataset_s\": %.3f, \"hash_s\": %.3f, "
            "\"contain_s\": %.3f, \"discovery_s\": %.3f}\n",
            (unsigned long long)N, (unsigned long long)ds->getNumberOfReads(), (unsigned long long)rd.n,
            (unsigned long long)rd.sum, (unsigned long long)rd.xr, (unsigned long long)rd.sum2,
            (unsigned long long)sd.n, (unsigned long long)sd.sum, (unsigned long long)sd.xr,
            (unsigned long long)sd.sum2, t_ds, t2 - t1, t3 - t2, t4 - t3);
  } else if (!strcmp(mode, "hash")) {
    HashTable* ht = new HashTable();
    ht->insertDataset(ds, l);
    fprintf(out, "#P %llu\n", (unsigned long long)ht->getHashTableSize());
    const UINT64 h = ht->getHashStringLength();
    for (UINT64 i = 1; i <= N && i <= 64; i++) {
      Read* r = ds->getReadFromID(i);
      const string f = r->getStringForward(), b = r->getStringReverse();
      const string keys[4] = {f.substr(0, h), f.substr(f.length() - h, h), b.substr(0, h), b.substr(b.length() - h, h)};
      for (int o = 0; o < 4; o++)
        fprintf(out, "%s %llu\n", keys[o].c_str(), (unsigned long long)ht->hashFunction(keys[o]));
    }
  } else if (!strcmp(mode, "edges")) {
    HashTable* ht = new HashTable();
    ht->insertDataset(ds, l);
    OverlapGraph* og = prepare_graph(ds, ht);
    discovery(og, ds);
    fprintf(out, "#N %llu\n", (unsigned long long)N);
    for (UINT64 i = 1; i <= N; i++) {
      Read* r = ds->getReadFromID(i);
      fprintf(out, "#R %llu %s\n", (unsigned long long)i, r->getStringForward().c_str());
      if (r->superReadID)
        fprintf(out, "#S %llu %llu\n", (unsigned long long)i, (unsigned long long)r->superReadID);
    }
    for (UINT64 u = 1; u <= N; u++) {
      vector<Edge*>* lst = og->graph->at(u);
      for (size_t k = 0; k < lst->size(); k++) {
        Edge* e = lst->at(k);
        fprintf(out, "%llu %llu %u %llu\n", (unsigned long long)e->getSourceRead()->getReadNumber(),
                (unsigned long long)e->getDestinationRead()->getReadNumber(), (unsigned)e->getOrientation(),
                (unsigned long long)e->getOverlapOffset());
      }
    }
  } else if (!strcmp(mode, "bfs")) {
    HashTable* ht = new HashTable();
    ht->insertDataset(ds, l);
    OverlapGraph* og = prepare_graph(ds, ht);
    double t1 = now_s();
    explore_components(og, ds);
    double t2 = now_s();
    fprintf(out, "#C %llu %llu\n", (unsigned long long)og->numberOfNodes, (unsigned long long)og->numberOfEdges);
    fprintf(out, "#T %.6f\n", t2 - t1);
    for (UINT64 u = 1; u <= N; u++) {
      vector<Edge*>* lst = og->graph->at(u);
      for (size_t k = 0; k < lst->size(); k++) {
        Edge* e = lst->at(k);
        fprintf(out, "%llu %llu %u %llu\n", (unsigned long long)u,
                (unsigned long long)e->getDestinationRead()->getReadNumber(), (unsigned)e->getOrientation(),
                (unsigned long long)e->getOverlapOffset());
      }
    }
  } else if (!strcmp(mode, "unitig")) {
    HashTable* ht = new HashTable();
    ht->insertDataset(ds, l);
    OverlapGraph* og = prepare_graph(ds, ht);
    double t1 = now_s();
    explore_components(og, ds);
    double t2 = now_s();
    UINT64 counter = 0, iters = 0;
    do {  // OverlapGraph.cpp:211-215
      counter = og->contractCompositePaths();
      counter += og->removeDeadEndNodes();
      iters++;
    } while (counter > 0);
    double t3 = now_s();
    fprintf(out, "#C %llu %llu\n", (unsigned long long)og->numberOfNodes, (unsigned long long)og->numberOfEdges);
    fprintf(out, "#I %llu\n", (unsigned long long)iters);
    fprintf(out, "#T %.6f %.6f\n", t2 - t1, t3 - t2);
    for (UINT64 u = 1; u <= N; u++) {
      vector<Edge*>* lst = og->graph->at(u);
      for (size_t k = 0; k < lst->size(); k++) {
        Edge* e = lst->at(k);
        fprintf(out, "%llu %llu %u %llu %llu", (unsigned long long)u,
                (unsigned long long)e->getDestinationRead()->getReadNumber(), (unsigned)e->getOrientation(),
                (unsigned long long)e->getOverlapOffset(), (unsigned long long)e->getListOfReads()->size());
        for (size_t q = 0; q < e->getListOfReads()->size(); q++)
          fprintf(out, " %llu:%u:%u", (unsigned long long)e->getListOfReads()->at(q),
                  (unsigned)e->getListOfOverlapOffsets()->at(q), (unsigned)e->getListOfOrientations()->at(q));
        fprintf(out, "\n");
      }
    }
    for (UINT64 r = 1; r <= N; r++) {
      Read* rd = ds->getReadFromID(r);
      for (int side = 0; side < 2; side++) {
        vector<Edge*>* le = side ? rd->getListOfEdgesReverse() : rd->getListOfEdgesForward();
        vector<UINT64>* ll = side ? rd->getLocationOnEdgeReverse() : rd->getLocationOnEdgeForward();
        for (size_t q = 0; q < le->size(); q++) {
          Edge* e = le->at(q);
          fprintf(out, "%c %llu %llu %llu %u %llu %llu\n", side ? 'R' : 'F', (unsigned long long)r,
                  (unsigned long long)e->getSourceRead()->getReadNumber(),
                  (unsigned long long)e->getDestinationRead()->getReadNumber(), (unsigned)e->getOrientation(),
                  (unsigned long long)e->getOverlapOffset(), (unsigned long long)ll->at(q));
        }
      }
    }
    og->sortEdges();
    og->saveGraphToFile(string(argv[4]) + ".unitig");
  } else if (!strcmp(mode, "reread")) {
    if (argc < 6) {
      fprintf(stderr, "reread needs the .unitig file\n");
      return 2;
    }
    OverlapGraph* og = new OverlapGraph();
    og->setDataset(ds);
    og->readGraphFromFile(string(argv[5]));
    fprintf(out, "#C %llu %llu\n", (unsigned long long)og->numberOfNodes, (unsigned long long)og->numberOfEdges);
    for (UINT64 u = 1; u <= N; u++) {
      vector<Edge*>* lst = og->graph->at(u);
      for (size_t k = 0; k < lst->size(); k++) {
        Edge* e = lst->at(k);
        fprintf(out, "%llu %llu %u %llu %llu", (unsigned long long)u,
                (unsigned long long)e->getDestinationRead()->getReadNumber(), (unsigned)e->getOrientation(),
                (unsigned long long)e->getOverlapOffset(), (unsigned long long)e->getListOfReads()->size());
        for (size_t q = 0; q < e->getListOfReads()->size(); q++)
          fprintf(out, " %llu:%u:%u", (unsigned long long)e->getListOfReads()->at(q),
                  (unsigned)e->getListOfOverlapOffsets()->at(q), (unsigned)e->getListOfOrientations()->at(q));
        fprintf(out, "\n");
      }
    }
    for (UINT64 r = 1; r <= N; r++) {
      Read* rd = ds->getReadFromID(r);
      for (int side = 0; side < 2; side++) {
        vector<Edge*>* le = side ? rd->getListOfEdgesReverse() : rd->getListOfEdgesForward();
        vector<UINT64>* ll = side ? rd->getLocationOnEdgeReverse() : rd->getLocationOnEdgeForward();
        for (size_t q = 0; q < le->size(); q++) {
          Edge* e = le->at(q);
          fprintf(out, "%c %llu %llu %llu %u %llu %llu\n", side ? 'R' : 'F', (unsigned long long)r,
                  (unsigned long long)e->getSourceRead()->getReadNumber(),
                  (unsigned long long)e->getDestinationRead()->getReadNumber(), (unsigned)e->getOrientation(),
                  (unsigned long long)e->getOverlapOffset(), (unsigned long long)ll->at(q));
        }
      }
    }
    og->sortEdges();
    og->saveGraphToFile(string(argv[4]) + ".unitig");
  } else if (!strcmp(mode, "lookup")) {
    HashTable* ht = new HashTable();
    ht->insertDataset(ds, l);
    for (int a = 5; a < argc; a++) {
      vector<UINT64>* lst = ht->getListOfReads(string(argv[a]));
      fprintf(out, "%s", argv[a]);
      for (size_t k = 0; k < lst->size(); k++)
        fprintf(out, " %llu:%llu", (unsigned long long)(lst->at(k) & 0x3FFFFFFFFFFFFFFFULL),
                (unsigned long long)(lst->at(k) >> 62));
      fprintf(out, "\n");
    }
  } else {
    fprintf(stderr, "unknown mode %s\n", mode);
    return 2;
  }
  std::cout.rdbuf(old);
  fclose(out);
  return 0;
}
