// mg_api.hpp — drop-in C++ surface for the reference's overlap path.
//
// Same class names, method names and argument meaning as the reference's
// Read / Edge / Dataset / HashTable / OverlapGraph (Read.h:31-72,
// Edge.h:16-61, Dataset.h:18-51, HashTable.h:16-36, OverlapGraph.h:32-100 in
// /root/reference/MetaGenomics), so main.cpp:33,45-47 compiles against it:
//
//     Dataset *dataSet = new Dataset(pairedEndFileNames, singleEndFileNames, l);
//     HashTable *hashTable = new HashTable();
//     hashTable->insertDataset(dataSet, l);              // GPU index build
//     OverlapGraph *g = new OverlapGraph(hashTable);     // GPU discovery, deletes hashTable
//
// Differences, all deliberate:
//  * errors throw mg::Error instead of MYEXIT's exit(0) (Common.h:47);
//  * reads are stored 2-bit packed; getStringForward/Reverse decode on demand;
//  * OverlapGraph(ht) returns the reference's graph: discovery on the device,
//    then the reference's exploration order and transitive reduction
//     and its contraction loop (OverlapGraph.cpp:211-215,
//    row 3) replayed on the host; flow and scaffolding are out of scope
//    (SURVEY §2 rows 8-13);
//  * HashTable/OverlapGraph run on a HIP device through include/mg_overlap.h
//    and throw if no device is available (there is no CPU fallback).
#ifndef MG_API_HPP_
#define MG_API_HPP_

#include <cstdint>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "mg_overlap.h"

// The reference's integer names (Common.h:31-37); UINT32 is 64-bit on LP64 there.
typedef unsigned char UINT8;
typedef unsigned short UINT16;
typedef unsigned long UINT32;
typedef unsigned long long UINT64;
typedef long long INT64;

namespace mg {
class UnitigGraph;
struct Error : std::runtime_error {
  explicit Error(const std::string& s) : std::runtime_error(s) {}
};
struct PackedReads;
}  // namespace mg

class Dataset;
class Edge;

// The exploration state and the transitive-reduction marks (OverlapGraph.h:20-30).
enum nodeType { UNEXPLORED = 0, EXPLORED = 1, EXPLORED_AND_TRANSITIVE_EDGES_MARKED = 2 };
enum markType { VACANT = 0, INPLAY = 1, ELIMINATED = 2 };

class Read {
 public:
  UINT64 superReadID = 0;      // 0 = not contained, else ID of the super read (Read.h:50)
  bool isContainedRead = false;
  std::string getStringForward();
  std::string getStringReverse();
  UINT16 getReadLength();
  UINT64 getReadNumber() { return readNumber; }
  UINT32 getFrequency();
  // composite edges holding this read's forward / reverse string and the read's
  // distance on each (Read.h:39-42, maintained by OverlapGraph.cpp:1048-1115)
  std::vector<Edge*>* getListOfEdgesForward() { return &locations().edgesForward; }
  std::vector<UINT64>* getLocationOnEdgeForward() { return &locations().locationForward; }
  std::vector<Edge*>* getListOfEdgesReverse() { return &locations().edgesReverse; }
  std::vector<UINT64>* getLocationOnEdgeReverse() { return &locations().locationReverse; }

 private:
  friend class Dataset;
  friend class OverlapGraph;
  struct Locations {
    std::vector<Edge*> edgesForward, edgesReverse;
    std::vector<UINT64> locationForward, locationReverse;
  };
  Locations& locations() {
    if (!loc) loc.reset(new Locations());
    return *loc;
  }
  const Dataset* owner = nullptr;
  UINT64 readNumber = 0;
  std::unique_ptr<Locations> loc;  // allocated on first use (most reads are on no composite edge)
};

class Edge {
 public:
  Edge(Read* from, Read* to, UINT64 orient, UINT64 length)
      : source(from), destination(to), overlapOrientation((UINT8)orient), overlapOffset(length) {}
  Read* getSourceRead() { return source; }
  Read* getDestinationRead() { return destination; }
  UINT8 getOrientation() { return overlapOrientation; }
  UINT64 getOverlapOffset() { return overlapOffset; }
  Edge* getReverseEdge() { return reverseEdge; }
  bool setReverseEdge(Edge* e) {
    reverseEdge = e;
    return true;
  }
  // ordered reads inside a composite edge (Edge.h:30-32; empty for a simple edge)
  std::vector<UINT64>* getListOfReads() { return &listOfReads; }
  std::vector<UINT16>* getListOfOverlapOffsets() { return &listOfOverlapOffsets; }
  std::vector<UINT8>* getListOfOrientations() { return &listOfOrientations; }
  bool transitiveRemovalFlag = false;
  UINT16 flow = 0;  // Edge.h:42 (0 until flow is computed)

 private:
  friend class OverlapGraph;
  UINT64 serial = 0;  // creation order (insertEdge(Read*,...) makes the edge before its twin)
  Read* source;
  Read* destination;
  UINT8 overlapOrientation;  // 0 = u<---<v, 1 = u<--->v, 2 = u>---<v, 3 = u>--->v
  UINT64 overlapOffset;      // start of v relative to u
  Edge* reverseEdge = nullptr;
  std::vector<UINT64> listOfReads;
  std::vector<UINT16> listOfOverlapOffsets;
  std::vector<UINT8> listOfOrientations;
};

class Dataset {
 public:
  std::vector<std::string> pairedEndDatasetFileNames;
  std::vector<std::string> singleEndDatasetFileNames;
  UINT64 shortestReadLength = ~0ULL;
  UINT64 longestReadLength = 0;

  Dataset(std::vector<std::string> pairedEndFileNames, std::vector<std::string> singleEndFileNames,
          UINT64 minOverlap);
  ~Dataset();
  UINT64 getNumberOfReads() { return numberOfReads; }
  UINT64 getNumberOfUniqueReads() { return numberOfUniqueReads; }
  Read* getReadFromString(const std::string& read);
  Read* getReadFromID(UINT64 ID);
  void saveReads(std::string fileName);
  void readMatePairsFromFile() {}  // single-end only: mate pairs are out of scope

  // --- packed view (device upload) and bulk construction (bench / Python) ---
  static Dataset* fromCodes(const uint8_t* codes, uint64_t n, uint64_t stride, const uint16_t* lens,
                            UINT64 minOverlap, int nthreads);
  const uint64_t* packedWords() const;
  const uint16_t* packedLengths() const;
  uint32_t wordsPerRead() const;
  uint32_t frequencyOf(UINT64 id) const;
  std::string decode(UINT64 id, bool reverse) const;
  UINT64 minimumOverlapLength() const { return minOverlapLength; }

 private:
  Dataset() = default;
  void finalize(mg::PackedReads&& pr);
  mg::PackedReads* packed = nullptr;
  std::vector<Read> reads;
  UINT64 numberOfReads = 0, numberOfUniqueReads = 0, minOverlapLength = 0;
};

class HashTable {
 public:
  HashTable();
  explicit HashTable(Dataset* d) : HashTable() { dataSet = d; }
  ~HashTable();
  bool insertDataset(Dataset* d, UINT64 minOverlapLength);
  std::vector<UINT64>* getListOfReads(std::string subString);
  UINT64 hashFunction(std::string subString);  // the reference's index function (HashTable.cpp:135-155)
  UINT64 getHashTableSize() { return hashTableSize; }
  UINT64 getHashStringLength() { return hashStringLength; }
  Dataset* getDataset() { return dataSet; }

  // --- device controls (not in the reference) ---
  static void setDefaultDevice(int device);
  static void setDefaultSeedK(uint32_t k);
  mg_ctx* context() { return ctx; }

 private:
  Dataset* dataSet = nullptr;
  mg_ctx* ctx = nullptr;
  UINT64 hashTableSize = 0;
  UINT16 hashStringLength = 0;
  std::vector<std::vector<UINT64>*> lookups;  // lists handed out by getListOfReads
};

class OverlapGraph {
 public:
  OverlapGraph();
  explicit OverlapGraph(HashTable* ht);
  ~OverlapGraph();
  bool buildOverlapGraphFromHashTable(HashTable* ht);
  void markContainedReads();
  bool insertEdge(Edge* edge);
  bool insertEdge(Read* read1, Read* read2, UINT8 orient, UINT16 overlapOffset);

  // --- the reference's per-read build steps (OverlapGraph.h:54,64-68), for a
  // caller that drives its own exploration as buildOverlapGraphFromHashTable
  // does (OverlapGraph.cpp:144-204).  beginBuildFromHashTable(ht) does that
  // function's set-up (:111-142): counters, the N + 1 empty lists,
  // markContainedReads on the device, and the device discovery of every read's
  // D(A) (mg_find_overlaps), kept on the host in insertAllEdgesOfRead's loop
  // order; the caller keeps ownership of ht.  Then:
  //  * insertAllEdgesOfRead (:529-565) inserts D(readNumber) in that order,
  //    skipping partners that are not UNEXPLORED (:546), and sorts the list by
  //    overlap offset with the reference's comparator (:563);
  //  * markTransitiveEdges (:574-615) / removeTransitiveEdges (:623-661) on
  //    the Edge objects, statement for statement;
  //  * checkOverlap (:354-383) / checkOverlapForContainedRead (:302-340) are
  //    the reference's string predicates for any pair (the device answers the
  //    same questions in bulk);
  //  * the contraction steps, sortEdges and saveGraphToFile then apply to the
  //    caller-built graph as to buildOverlapGraphFromHashTable's.
  bool beginBuildFromHashTable(HashTable* ht);
  bool insertAllEdgesOfRead(UINT64 readNumber, std::vector<nodeType>* exploredReads);
  bool markTransitiveEdges(UINT64 readNumber, std::vector<markType>* markedNodes);
  bool removeTransitiveEdges(UINT64 readNumber);
  bool checkOverlap(Read* read1, Read* read2, UINT64 orient, UINT64 start);
  bool checkOverlapForContainedRead(Read* read1, Read* read2, UINT64 orient, UINT64 start);
  // the .unitig checkpoint back into the graph (:1270-1367; main.cpp:36-42's
  // -s resume: OverlapGraph() -> setDataset -> readGraphFromFile -> sortEdges)
  bool readGraphFromFile(const std::string& fileName);
  UINT64 getNumberOfEdges() { return numberOfEdges; }
  UINT64 getNumberOfNodes() { return numberOfNodes; }
  bool setDataset(Dataset* d) {
    dataSet = d;
    return true;
  }
  // graph[u] of the reference (private there): edges of read u, sorted by offset (:563)
  const std::vector<Edge*>* getEdges(UINT64 readNumber) const;
  // current edges as "u v orient offset" lines, sorted (checkpoint/parity dump)
  bool saveRawEdges(const std::string& fileName) const;
  // every graph[u] list in list order after "#C numberOfNodes numberOfEdges"
  bool saveGraphLists(const std::string& fileName) const;
  // true (default): buildOverlapGraphFromHashTable replays the reference's
  // exploration order and transitive reduction (OverlapGraph.cpp:144-204,
  // 574-661) on the device's discoveries; false: keep the raw discovery multiset.
  static bool replayExploration;
  // true (default, as the reference): then run the contraction loop
  // (OverlapGraph.cpp:211-215); false: stop just before it
  static bool contractPaths;
  // the contraction loop's steps (:669-696, :931-988) on the current graph
  // (available once the graph was built with replayExploration)
  UINT64 contractCompositePaths();
  UINT64 removeDeadEndNodes();
  void sortEdges();                                // :2799-2808
  bool saveGraphToFile(const std::string& fileName);  // the .unitig checkpoint (:1219-1261)
  const mg_timings& timings() const { return lastTimings; }

 private:
  Dataset* dataSet = nullptr;
  HashTable* hashTable = nullptr;
  std::vector<std::vector<Edge*>*>* graph = nullptr;
  UINT64 numberOfNodes = 0, numberOfEdges = 0;
  bool containedDone = false;
  mg_timings lastTimings{};
  mg::UnitigGraph* unitig = nullptr;  // the list state the contraction steps work on
  struct Manual;                      // a caller-driven build: D(A) lists + the hash string length
  Manual* manual = nullptr;
  UINT64 nextSerial = 0;
  void clear();
  void materialize();  // graph / Edge objects / read locations from `unitig`
  void adoptEdgeLists();  // `unitig` from the Edge lists of a caller-driven build
};

#endif  // MG_API_HPP_
