// mg_host.cpp — host-side mirror of the reference's Read / Dataset /
// HashTable / OverlapGraph API (include/mg_api.hpp) plus the mgh_* C-ABI
// (include/mg_host.h).  The hot path (index build, containment, overlap
// discovery) runs on the GPU through include/mg_overlap.h; this file only
// ingests reads (Dataset semantics) and shapes results into the reference's
// object model.  Reference citations are relative to /root/reference/MetaGenomics.
#include <algorithm>
#include <atomic>
#include <cctype>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iomanip>
#include <sstream>
#include <thread>
#include <unordered_map>

#include "mg_api.hpp"
#include "mg_parse.hpp"
#include "mg_unitig.hpp"
#include "mg_graph.hpp"
#include "mg_host.h"

namespace mg {

// Unique reads, 2-bit packed (A0 C1 G2 T3, most significant base first), ID order.
struct PackedReads {
  uint32_t wpr = 1;
  std::vector<uint64_t> words;
  std::vector<uint16_t> lens;
  std::vector<uint32_t> freq;
  uint64_t n_good = 0;
  uint64_t shortest = ~0ULL, longest = 0;
  uint64_t n() const { return lens.size(); }
  const uint64_t* rec(uint64_t i) const { return words.data() + i * wpr; }
};

namespace {

int hw_threads(int want) {
  int hc = (int)std::thread::hardware_concurrency();
  if (hc <= 0) hc = 4;
  if (want <= 0) want = hc;
  return std::max(1, std::min(want, 64));
}

template <typename F>
void parallel_for(uint64_t n, int nthreads, F&& fn) {
  const int T = (int)std::min<uint64_t>((uint64_t)nthreads, std::max<uint64_t>(1, n / 4096 + 1));
  if (T <= 1) {
    fn(0, 0, n);
    return;
  }
  std::vector<std::thread> th;
  for (int t = 0; t < T; ++t) {
    const uint64_t lo = n * t / T, hi = n * (t + 1) / T;
    th.emplace_back([&fn, t, lo, hi] { fn(t, lo, hi); });
  }
  for (auto& x : th) x.join();
}

// One raw read in upper-case 2-bit codes; returns false if not ACGT only.
struct Source {
  // ASCII source
  const char* text = nullptr;
  const uint64_t* off = nullptr;
  // code source
  const uint8_t* codes = nullptr;
  uint64_t stride = 0;
  const uint16_t* lens = nullptr;
  uint64_t n = 0;

  uint64_t length(uint64_t i) const { return text ? off[i + 1] - off[i] : lens[i]; }
  bool get(uint64_t i, std::vector<uint8_t>& out) const {
    const uint64_t L = length(i);
    out.resize(L);
    if (text) {
      const char* s = text + off[i];
      for (uint64_t k = 0; k < L; ++k) {
        switch (std::toupper((unsigned char)s[k])) {  // Dataset.cpp:158-159
          case 'A': out[k] = 0; break;
          case 'C': out[k] = 1; break;
          case 'G': out[k] = 2; break;
          case 'T': out[k] = 3; break;
          default: return false;  // testRead: only A, C, G, T (Dataset.cpp:405-406)
        }
      }
    } else {
      const uint8_t* c = codes + i * stride;
      for (uint64_t k = 0; k < L; ++k) {
        if (c[k] > 3) return false;
        out[k] = c[k];
      }
    }
    return true;
  }
};

// Dataset::testRead's 80 % rule (Dataset.cpp:409-411) on valid codes.
bool low_complexity(const std::vector<uint8_t>& c) {
  uint64_t cnt[4] = {0, 0, 0, 0};
  for (uint8_t x : c) cnt[x]++;
  const uint64_t threshold = (uint64_t)(c.size() * .8);
  return cnt[0] >= threshold || cnt[1] >= threshold || cnt[2] >= threshold || cnt[3] >= threshold;
}

void pack_codes(const uint8_t* c, uint64_t L, uint32_t wpr, uint64_t* dst) {
  for (uint32_t w = 0; w < wpr; ++w) {
    uint64_t x = 0;
    for (uint32_t k = 0; k < 32; ++k) {
      const uint64_t p = (uint64_t)w * 32 + k;
      x = (x << 2) | (p < L ? c[p] : 0);
    }
    dst[w] = x;
  }
}

// std::string order on packed reads: words (zero padded) then length.
inline int cmp_packed(const uint64_t* a, uint16_t la, const uint64_t* b, uint16_t lb, uint32_t wpr) {
  for (uint32_t k = 0; k < wpr; ++k)
    if (a[k] != b[k]) return a[k] < b[k] ? -1 : 1;
  return la == lb ? 0 : (la < lb ? -1 : 1);
}

template <typename Cmp>
void parallel_sort(std::vector<uint64_t>& idx, int nthreads, Cmp cmp) {
  const uint64_t n = idx.size();
  int T = 1;
  while (T * 2 <= nthreads && n / (uint64_t)(T * 2) > 65536) T *= 2;
  if (T == 1) {
    std::sort(idx.begin(), idx.end(), cmp);
    return;
  }
  std::vector<uint64_t> bounds(T + 1);
  for (int t = 0; t <= T; ++t) bounds[t] = n * t / T;
  {
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t)
      th.emplace_back([&, t] { std::sort(idx.begin() + bounds[t], idx.begin() + bounds[t + 1], cmp); });
    for (auto& x : th) x.join();
  }
  std::vector<uint64_t> tmp(n);
  for (int width = 1; width < T; width *= 2) {
    std::vector<std::thread> th;
    for (int t = 0; t < T; t += 2 * width) {
      const uint64_t lo = bounds[t], mid = bounds[std::min(t + width, T)], hi = bounds[std::min(t + 2 * width, T)];
      th.emplace_back([&, lo, mid, hi] {
        std::merge(idx.begin() + lo, idx.begin() + mid, idx.begin() + mid, idx.begin() + hi, tmp.begin() + lo, cmp);
      });
    }
    for (auto& x : th) x.join();
    idx.swap(tmp);
  }
}

// readDataset's per-read body + sortReads + removeDupicateReads
// (Dataset.cpp:158-181, 197-202, 316-345) over any read source.
PackedReads ingest(const Source& src, uint64_t min_overlap, int nthreads) {
  PackedReads pr;
  uint64_t maxlen = 0;
  for (uint64_t i = 0; i < src.n; ++i) maxlen = std::max(maxlen, src.length(i));
  pr.wpr = (uint32_t)std::max<uint64_t>(1, (maxlen + 31) / 32);
  const int T = hw_threads(nthreads);
  struct Part {
    std::vector<uint64_t> words;
    std::vector<uint16_t> lens;
    uint64_t shortest = ~0ULL, longest = 0;
  };
  std::vector<Part> parts(T);
  parallel_for(src.n, T, [&](int t, uint64_t lo, uint64_t hi) {
    Part& P = parts[t];
    std::vector<uint8_t> c, rc;
    for (uint64_t i = lo; i < hi; ++i) {
      const uint64_t L = src.length(i);
      if (!(L > min_overlap)) continue;  // Dataset.cpp:160
      if (L > 65535) continue;           // Read::getReadLength is UINT16
      if (!src.get(i, c) || low_complexity(c)) continue;
      rc.resize(L);
      for (uint64_t k = 0; k < L; ++k) rc[k] = (uint8_t)(3 - c[L - 1 - k]);  // Dataset.cpp:463-475
      // store the lexicographically smaller strand (Dataset.cpp:164-167)
      const bool fwd = std::lexicographical_compare(c.begin(), c.end(), rc.begin(), rc.end());
      const std::vector<uint8_t>& s = fwd ? c : rc;
      const size_t at = P.words.size();
      P.words.resize(at + pr.wpr);
      pack_codes(s.data(), L, pr.wpr, P.words.data() + at);
      P.lens.push_back((uint16_t)L);
      P.shortest = std::min(P.shortest, L);
      P.longest = std::max(P.longest, L);
    }
  });
  uint64_t ngood = 0;
  for (auto& P : parts) {
    ngood += P.lens.size();
    pr.shortest = std::min(pr.shortest, P.shortest);
    pr.longest = std::max(pr.longest, P.longest);
  }
  pr.n_good = ngood;
  std::vector<uint64_t> all_words;
  std::vector<uint16_t> all_lens;
  all_words.reserve(ngood * pr.wpr);
  all_lens.reserve(ngood);
  for (auto& P : parts) {
    all_words.insert(all_words.end(), P.words.begin(), P.words.end());
    all_lens.insert(all_lens.end(), P.lens.begin(), P.lens.end());
    std::vector<uint64_t>().swap(P.words);
  }
  // sort (std::string order) by index; the first word decides almost always
  std::vector<uint64_t> idx(ngood);
  for (uint64_t i = 0; i < ngood; ++i) idx[i] = i;
  const uint32_t wpr = pr.wpr;
  const uint64_t* W = all_words.data();
  const uint16_t* Ls = all_lens.data();
  parallel_sort(idx, T, [W, Ls, wpr](uint64_t a, uint64_t b) {
    return cmp_packed(W + a * wpr, Ls[a], W + b * wpr, Ls[b], wpr) < 0;
  });
  // dedup adjacent equal reads; frequency = multiplicity; ID = rank (Dataset.cpp:321-339)
  uint64_t nu = 0;
  for (uint64_t k = 0; k < ngood; ++k)
    if (k == 0 || cmp_packed(W + idx[k - 1] * wpr, Ls[idx[k - 1]], W + idx[k] * wpr, Ls[idx[k]], wpr) != 0) nu++;
  pr.words.resize(nu * wpr);
  pr.lens.resize(nu);
  pr.freq.assign(nu, 0);
  int64_t u = -1;
  for (uint64_t k = 0; k < ngood; ++k) {
    const uint64_t i = idx[k];
    if (k == 0 || cmp_packed(W + idx[k - 1] * wpr, Ls[idx[k - 1]], W + i * wpr, Ls[i], wpr) != 0) {
      ++u;
      std::memcpy(pr.words.data() + u * wpr, W + i * wpr, wpr * sizeof(uint64_t));
      pr.lens[u] = Ls[i];
    }
    pr.freq[u]++;
  }
  return pr;
}

std::string decode_packed(const uint64_t* w, uint16_t L, bool reverse) {
  static const char A[4] = {'A', 'C', 'G', 'T'};
  std::string s(L, 'A');
  for (uint32_t k = 0; k < L; ++k) {
    const uint32_t c = (uint32_t)(w[k >> 5] >> (62 - 2 * (k & 31))) & 3u;
    if (reverse)
      s[L - 1 - k] = A[3 - c];
    else
      s[k] = A[c];
  }
  return s;
}

int g_default_device = 0;
uint32_t g_default_seed_k = 0;

// getPrimeLargerThanNumber (HashTable.cpp:20-29): the first entry of the
// reference's fixed table of 450 primes that exceeds `number`, else number + 1.
// The table is data the API reports (getHashTableSize, hashFunction's modulus);
// the device index never uses it (its directory is a power of two).
const uint64_t kRefPrimes[450] = {
    1114523ULL, 1180043ULL, 1245227ULL, 1310759ULL, 1376447ULL, 1442087ULL, 1507379ULL, 1573667ULL,
    1638899ULL, 1704023ULL, 1769627ULL, 1835027ULL, 1900667ULL, 1966127ULL, 2031839ULL, 2228483ULL,
    2359559ULL, 2490707ULL, 2621447ULL, 2752679ULL, 2883767ULL, 3015527ULL, 3145739ULL, 3277283ULL,
    3408323ULL, 3539267ULL, 3670259ULL, 3801143ULL, 3932483ULL, 4063559ULL, 4456643ULL, 4718699ULL,
    4980827ULL, 5243003ULL, 5505239ULL, 5767187ULL, 6029603ULL, 6291563ULL, 6553979ULL, 6816527ULL,
    7079159ULL, 7340639ULL, 7602359ULL, 7864799ULL, 8126747ULL, 8913119ULL, 9437399ULL, 9962207ULL,
    10485767ULL, 11010383ULL, 11534819ULL, 12059123ULL, 12583007ULL, 13107923ULL, 13631819ULL, 14156543ULL,
    14680067ULL, 15204467ULL, 15729647ULL, 16253423ULL, 17825999ULL, 18874379ULL, 19923227ULL, 20971799ULL,
    22020227ULL, 23069447ULL, 24117683ULL, 25166423ULL, 26214743ULL, 27264047ULL, 28312007ULL, 29360147ULL,
    30410483ULL, 31457627ULL, 32505983ULL, 35651783ULL, 37749983ULL, 39845987ULL, 41943347ULL, 44040383ULL,
    46137887ULL, 48234623ULL, 50331707ULL, 52429067ULL, 54526019ULL, 56623367ULL, 58720307ULL, 60817763ULL,
    62915459ULL, 65012279ULL, 71303567ULL, 75497999ULL, 79691867ULL, 83886983ULL, 88080527ULL, 92275307ULL,
    96470447ULL, 100663439ULL, 104858387ULL, 109052183ULL, 113246699ULL, 117440699ULL, 121635467ULL, 125829239ULL,
    130023683ULL, 142606379ULL, 150994979ULL, 159383759ULL, 167772239ULL, 176160779ULL, 184549559ULL, 192938003ULL,
    201327359ULL, 209715719ULL, 218104427ULL, 226493747ULL, 234882239ULL, 243269639ULL, 251659139ULL, 260047367ULL,
    285215507ULL, 301989959ULL, 318767927ULL, 335544323ULL, 352321643ULL, 369100463ULL, 385876703ULL, 402654059ULL,
    419432243ULL, 436208447ULL, 452986103ULL, 469762067ULL, 486539519ULL, 503316623ULL, 520094747ULL, 570425399ULL,
    603979919ULL, 637534763ULL, 671089283ULL, 704643287ULL, 738198347ULL, 771752363ULL, 805307963ULL, 838861103ULL,
    872415239ULL, 905971007ULL, 939525143ULL, 973079279ULL, 1006633283ULL, 1040187419ULL, 1140852767ULL, 1207960679ULL,
    1275069143ULL, 1342177379ULL, 1409288183ULL, 1476395699ULL, 1543504343ULL, 1610613119ULL, 1677721667ULL, 1744830587ULL,
    1811940419ULL, 1879049087ULL, 1946157419ULL, 2013265967ULL, 2080375127ULL, 2281701827ULL, 2415920939ULL, 2550137039ULL,
    2684355383ULL, 2818572539ULL, 2952791147ULL, 3087008663ULL, 3221226167ULL, 3355444187ULL, 3489661079ULL, 3623878823ULL,
    3758096939ULL, 3892314659ULL, 4026532187ULL, 4160749883ULL, 4563403379ULL, 4831838783ULL, 5100273923ULL, 5368709219ULL,
    5637144743ULL, 5905580687ULL, 6174015503ULL, 6442452119ULL, 6710886467ULL, 6979322123ULL, 7247758307ULL, 7516193123ULL,
    7784629079ULL, 8053065599ULL, 8321499203ULL, 9126806147ULL, 9663676523ULL, 10200548819ULL, 10737418883ULL, 11274289319ULL,
    11811160139ULL, 12348031523ULL, 12884902223ULL, 13421772839ULL, 13958645543ULL, 14495515943ULL, 15032386163ULL, 15569257247ULL,
    16106127887ULL, 16642998803ULL, 18253612127ULL, 19327353083ULL, 20401094843ULL, 21474837719ULL, 22548578579ULL, 23622320927ULL,
    24696062387ULL, 25769803799ULL, 26843546243ULL, 27917287907ULL, 28991030759ULL, 30064772327ULL, 31138513067ULL, 32212254947ULL,
    33285996803ULL, 36507222923ULL, 38654706323ULL, 40802189423ULL, 42949673423ULL, 45097157927ULL, 47244640319ULL, 49392124247ULL,
    51539607599ULL, 53687092307ULL, 55834576979ULL, 57982058579ULL, 60129542339ULL, 62277026327ULL, 64424509847ULL, 66571993199ULL,
    73014444299ULL, 77309412407ULL, 81604379243ULL, 85899346727ULL, 90194314103ULL, 94489281203ULL, 98784255863ULL, 103079215439ULL,
    107374183703ULL, 111669150239ULL, 115964117999ULL, 120259085183ULL, 124554051983ULL, 128849019059ULL, 133143986399ULL, 146028888179ULL,
    154618823603ULL, 163208757527ULL, 171798693719ULL, 180388628579ULL, 188978561207ULL, 197568495647ULL, 206158430447ULL, 214748365067ULL,
    223338303719ULL, 231928234787ULL, 240518168603ULL, 249108103547ULL, 257698038539ULL, 266287975727ULL, 292057776239ULL, 309237645803ULL,
    326417515547ULL, 343597385507ULL, 360777253763ULL, 377957124803ULL, 395136991499ULL, 412316861267ULL, 429496730879ULL, 446676599987ULL,
    463856468987ULL, 481036337207ULL, 498216206387ULL, 515396078039ULL, 532575944723ULL, 584115552323ULL, 618475290887ULL, 652835029643ULL,
    687194768879ULL, 721554506879ULL, 755914244627ULL, 790273985219ULL, 824633721383ULL, 858993459587ULL, 893353198763ULL, 927712936643ULL,
    962072674643ULL, 996432414899ULL, 1030792152539ULL, 1065151889507ULL, 1168231105859ULL, 1236950582039ULL, 1305670059983ULL, 1374389535587ULL,
    1443109012607ULL, 1511828491883ULL, 1580547965639ULL, 1649267441747ULL, 1717986918839ULL, 1786706397767ULL, 1855425872459ULL, 1924145348627ULL,
    1992864827099ULL, 2061584304323ULL, 2130303780503ULL, 2336462210183ULL, 2473901164367ULL, 2611340118887ULL, 2748779070239ULL, 2886218024939ULL,
    3023656976507ULL, 3161095931639ULL, 3298534883999ULL, 3435973836983ULL, 3573412791647ULL, 3710851743923ULL, 3848290698467ULL, 3985729653707ULL,
    4123168604483ULL, 4260607557707ULL, 4672924419707ULL, 4947802331663ULL, 5222680234139ULL, 5497558138979ULL, 5772436047947ULL, 6047313952943ULL,
    6322191860339ULL, 6597069767699ULL, 6871947674003ULL, 7146825580703ULL, 7421703488567ULL, 7696581395627ULL, 7971459304163ULL, 8246337210659ULL,
    8521215117407ULL, 9345848837267ULL, 9895604651243ULL, 10445360463947ULL, 10995116279639ULL, 11544872100683ULL, 12094627906847ULL, 12644383722779ULL,
    13194139536659ULL, 13743895350023ULL, 14293651161443ULL, 14843406975659ULL, 15393162789503ULL, 15942918604343ULL, 16492674420863ULL, 17042430234443ULL,
    18691697672867ULL, 19791209300867ULL, 20890720927823ULL, 21990232555703ULL, 23089744183799ULL, 24189255814847ULL, 25288767440099ULL, 26388279068903ULL,
    27487790694887ULL, 28587302323787ULL, 29686813951463ULL, 30786325577867ULL, 31885837205567ULL, 32985348833687ULL, 34084860462083ULL, 37383395344739ULL,
    39582418600883ULL, 41781441856823ULL, 43980465111383ULL, 46179488367203ULL, 48378511622303ULL, 50577534878987ULL, 52776558134423ULL, 54975581392583ULL,
    57174604644503ULL, 59373627900407ULL, 61572651156383ULL, 63771674412287ULL, 65970697666967ULL, 68169720924167ULL, 74766790688867ULL, 79164837200927ULL,
    83562883712027ULL, 87960930223163ULL, 92358976733483ULL, 96757023247427ULL, 101155069756823ULL, 105553116266999ULL, 109951162779203ULL, 114349209290003ULL,
    118747255800179ULL, 123145302311783ULL, 127543348823027ULL, 131941395333479ULL, 136339441846019ULL, 149533581378263ULL, 158329674402959ULL, 167125767424739ULL,
    175921860444599ULL, 184717953466703ULL, 193514046490343ULL, 202310139514283ULL, 211106232536699ULL, 219902325558107ULL, 228698418578879ULL, 237494511600287ULL,
    246290604623279ULL, 255086697645023ULL, 263882790666959ULL, 272678883689987ULL, 299067162755363ULL, 316659348799919ULL, 334251534845303ULL, 351843720890723ULL,
    369435906934019ULL, 387028092977819ULL, 404620279022447ULL, 422212465067447ULL, 439804651111103ULL, 457396837157483ULL, 474989023199423ULL, 492581209246163ULL,
    510173395291199ULL, 527765581341227ULL, 545357767379483ULL, 598134325510343ULL, 633318697599023ULL, 668503069688723ULL, 703687441776707ULL, 738871813866287ULL,
    774056185954967ULL, 809240558043419ULL, 844424930134187ULL, 879609302222207ULL, 914793674313899ULL, 949978046398607ULL, 985162418489267ULL, 1020346790579903ULL,
    1055531162666507ULL, 1090715534754863ULL,
};

uint64_t prime_larger_than(uint64_t number) {
  for (uint64_t p : kRefPrimes)
    if (p > number) return p;
  return number + 1;
}

// hashFunction (HashTable.cpp:135-155): 2-bit codes (c >> 1) & 3 (A0 C1 G3 T2),
// the first 32 characters shifted into sum1, the rest into sum2, both seeded
// with 1; the product of the residues modulo the table size, in UINT64
// (wrapping like the reference's when the size exceeds 2^32).
uint64_t ref_hash(const char* s, uint64_t len, uint64_t size) {
  uint64_t sum1 = 1, sum2 = 1;
  for (uint64_t i = 0; i < len; ++i) {
    const uint64_t c = ((uint64_t)(int)s[i] >> 1) & 3ULL;
    if (i < 32)
      sum1 = (sum1 << 2) | c;
    else
      sum2 = (sum2 << 2) | c;
  }
  const uint64_t P = size ? size : 1;  // (the reference divides by zero before insertDataset)
  return ((sum1 % P) * (sum2 % P)) % P;
}

[[noreturn]] void fail(mg_ctx* ctx, const char* what) {
  throw mg::Error(std::string(what) + ": " + (ctx ? mg_last_error(ctx) : "no context"));
}

}  // namespace
}  // namespace mg

// ================================================================== Read ====
std::string Read::getStringForward() { return owner->decode(readNumber, false); }
std::string Read::getStringReverse() { return owner->decode(readNumber, true); }
UINT16 Read::getReadLength() { return owner->packedLengths()[readNumber - 1]; }
UINT32 Read::getFrequency() { return owner->frequencyOf(readNumber); }

// =============================================================== Dataset ====
Dataset::Dataset(std::vector<std::string> pe, std::vector<std::string> se, UINT64 minOverlap)
    : pairedEndDatasetFileNames(pe), singleEndDatasetFileNames(se), minOverlapLength(minOverlap) {
  mg::ParsedText parsed;
  std::vector<std::string> files(pe);
  files.insert(files.end(), se.begin(), se.end());  // paired-end first (Dataset.cpp:52-60)
  for (const auto& f : files) {
    const int rc = mg::parse_file_parallel(f, parsed, 0);  // Dataset.cpp:110-193
    if (rc) parsed.release();
    if (rc == -1) throw mg::Error("Unable to open file: " + f);
    if (rc == -2) throw mg::Error("Unknown input file format: " + f);
    if (rc) throw mg::Error("Out of memory reading " + f);
  }
  static const uint64_t kNoOffsets[1] = {0};
  mg::Source src;
  src.text = parsed.text;
  src.off = parsed.n_rec ? parsed.off : kNoOffsets;
  src.n = parsed.n_rec;
  try {
    finalize(mg::ingest(src, minOverlap, 0));
  } catch (...) {
    parsed.release();
    throw;
  }
  parsed.release();
}

Dataset* Dataset::fromCodes(const uint8_t* codes, uint64_t n, uint64_t stride, const uint16_t* lens,
                            UINT64 minOverlap, int nthreads) {
  mg::Source src;
  src.codes = codes;
  src.stride = stride;
  src.lens = lens;
  src.n = n;
  Dataset* d = new Dataset();
  d->minOverlapLength = minOverlap;
  d->finalize(mg::ingest(src, minOverlap, nthreads));
  return d;
}

void Dataset::finalize(mg::PackedReads&& pr) {
  packed = new mg::PackedReads(std::move(pr));
  numberOfReads = packed->n_good;
  numberOfUniqueReads = packed->n();
  shortestReadLength = packed->shortest;
  longestReadLength = packed->longest;
  reads.resize(numberOfUniqueReads);
  for (UINT64 i = 0; i < numberOfUniqueReads; ++i) {
    reads[i].owner = this;
    reads[i].readNumber = i + 1;
  }
}

Dataset::~Dataset() { delete packed; }

const uint64_t* Dataset::packedWords() const { return packed->words.data(); }
const uint16_t* Dataset::packedLengths() const { return packed->lens.data(); }
uint32_t Dataset::wordsPerRead() const { return packed->wpr; }
uint32_t Dataset::frequencyOf(UINT64 id) const { return packed->freq[id - 1]; }
std::string Dataset::decode(UINT64 id, bool reverse) const {
  return mg::decode_packed(packed->rec(id - 1), packed->lens[id - 1], reverse);
}

Read* Dataset::getReadFromID(UINT64 ID) {
  if (ID < 1 || ID > numberOfUniqueReads) {  // Dataset.cpp:484-490
    std::ostringstream ss;
    ss << "ID " << ID << " out of bound.";
    throw mg::Error(ss.str());
  }
  return &reads[ID - 1];
}

Read* Dataset::getReadFromString(const std::string& read) {
  // canonical strand, then binary search (Dataset.cpp:421-455)
  std::string rc(read.rbegin(), read.rend());
  for (char& c : rc) c = (c & 0x02) ? (char)(c ^ 0x04) : (char)(c ^ 0x15);
  const std::string& key = read.compare(rc) < 0 ? read : rc;
  std::vector<uint8_t> codes(key.size());
  for (size_t k = 0; k < key.size(); ++k) {
    switch (key[k]) {
      case 'A': codes[k] = 0; break;
      case 'C': codes[k] = 1; break;
      case 'G': codes[k] = 2; break;
      case 'T': codes[k] = 3; break;
      default: throw mg::Error("String not found in Dataset: " + read);
    }
  }
  const uint32_t wpr = packed->wpr;
  if (key.size() > 32ull * wpr || key.size() > 65535) throw mg::Error("String not found in Dataset: " + read);
  std::vector<uint64_t> q(wpr);
  mg::pack_codes(codes.data(), key.size(), wpr, q.data());
  uint64_t lo = 0, hi = numberOfUniqueReads;
  while (lo < hi) {
    const uint64_t mid = (lo + hi) / 2;
    const int c = mg::cmp_packed(packed->rec(mid), packed->lens[mid], q.data(), (uint16_t)key.size(), wpr);
    if (c == 0) return &reads[mid];
    if (c < 0)
      lo = mid + 1;
    else
      hi = mid;
  }
  throw mg::Error("String not found in Dataset: " + read);
}

void Dataset::saveReads(std::string fileName) {
  // Dataset.cpp:71-90 format
  std::ofstream out(fileName.c_str());
  if (!out) throw mg::Error("Unable to open file: " + fileName);
  for (UINT64 i = 1; i <= numberOfUniqueReads; ++i) {
    Read* r = &reads[i - 1];
    out << std::setw(10) << i << (r->superReadID ? " Contained in " : " Noncontained ") << std::setw(10)
        << r->superReadID << " " << r->getStringForward() << "\n";
  }
}

// ============================================================= HashTable ====
void HashTable::setDefaultDevice(int device) { mg::g_default_device = device; }
void HashTable::setDefaultSeedK(uint32_t k) { mg::g_default_seed_k = k; }

HashTable::HashTable() {}

HashTable::~HashTable() {
  for (auto* v : lookups) delete v;
  if (ctx) mg_destroy(ctx);
}

bool HashTable::insertDataset(Dataset* d, UINT64 minOverlapLength) {
  // HashTable::insertDataset (HashTable.cpp:50-80) on the device
  dataSet = d;
  hashStringLength = (UINT16)(minOverlapLength - 1);
  hashTableSize = mg::prime_larger_than(d->getNumberOfUniqueReads() * 8 + 1);  // HashTable.cpp:56
  if (!ctx) {
    const int rc = mg_create(&ctx, mg::g_default_device);
    if (rc) {
      ctx = nullptr;
      throw mg::Error(rc == -3 ? "no HIP device available (the overlap path has no CPU fallback)"
                               : "mg_create failed");
    }
  }
  if (mg_upload_reads_packed(ctx, d->packedWords(), d->packedLengths(), d->getNumberOfUniqueReads(),
                             d->wordsPerRead()))
    mg::fail(ctx, "upload");
  if (mg_build_index(ctx, (uint32_t)minOverlapLength, mg::g_default_seed_k)) mg::fail(ctx, "index");
  return true;
}

std::vector<UINT64>* HashTable::getListOfReads(std::string subString) {
  std::vector<UINT64>* v = new std::vector<UINT64>();
  lookups.push_back(v);
  uint64_t n = 0;
  std::vector<uint64_t> buf(64);
  for (;;) {
    if (mg_lookup_key(ctx, subString.data(), (uint32_t)subString.size(), buf.data(), buf.size(), &n))
      mg::fail(ctx, "getListOfReads");
    if (n <= buf.size()) break;
    buf.resize(n);
  }
  v->assign(buf.begin(), buf.begin() + n);
  return v;
}

UINT64 HashTable::hashFunction(std::string subString) {
  // the reference's index function (HashTable.cpp:135-155) modulo the
  // reference's table size (HashTable.cpp:56); the device index files keys
  // under minimizers instead, so this value only serves the API
  return mg::ref_hash(subString.data(), subString.size(), hashTableSize);
}

// ========================================================== OverlapGraph ====
OverlapGraph::OverlapGraph() {}

OverlapGraph::OverlapGraph(HashTable* ht) { buildOverlapGraphFromHashTable(ht); }

OverlapGraph::~OverlapGraph() { clear(); }

namespace {
void free_graph(std::vector<std::vector<Edge*>*>*& graph) {
  if (!graph) return;
  for (auto* lst : *graph) {
    for (auto* e : *lst) delete e;
    delete lst;
  }
  delete graph;
  graph = nullptr;
}
}  // namespace

struct OverlapGraph::Manual {
  mg::Discoveries D;  // D(A) of every read, in insertAllEdgesOfRead's loop order
  UINT64 h = 0;       // hashTable->getHashStringLength()
};

void OverlapGraph::clear() {
  free_graph(graph);
  delete unitig;
  unitig = nullptr;
  delete manual;
  manual = nullptr;
}

void OverlapGraph::materialize() {
  // Edge objects for the current lists of `unitig`, in list order, with their
  // read lists; the read location lists point at them (Read.h:39-42)
  const mg::UnitigGraph& ug = *unitig;
  free_graph(graph);
  const UINT64 N = dataSet->getNumberOfUniqueReads();
  for (UINT64 i = 1; i <= N; ++i) dataSet->getReadFromID(i)->loc.reset();
  graph = new std::vector<std::vector<Edge*>*>();
  graph->reserve(N + 1);
  for (UINT64 i = 0; i <= N; ++i) graph->push_back(new std::vector<Edge*>());
  std::vector<Edge*> made(ug.pool.size(), nullptr);
  for (UINT64 u = 1; u <= N && u < ug.lists.size(); ++u)
    for (uint32_t e : ug.lists[u]) {
      const mg::UnitigEdge& x = ug.pool[e];
      Edge* ed = new Edge(dataSet->getReadFromID(x.src), dataSet->getReadFromID(x.dst), x.orient, x.offset);
      ed->flow = x.flow;
      if (const mg::EdgeReads* r = ug.reads[e].get()) {
        ed->getListOfReads()->assign(r->reads.begin(), r->reads.end());
        *ed->getListOfOverlapOffsets() = r->offs;
        *ed->getListOfOrientations() = r->ors;
      }
      made[e] = ed;
    }
  for (UINT64 u = 1; u <= N && u < ug.lists.size(); ++u)
    for (uint32_t e : ug.lists[u]) {
      made[e]->setReverseEdge(made[ug.pool[e].rev]);
      (*graph)[u]->push_back(made[e]);
    }
  if (ug.track) {
    for (UINT64 i = 1; i <= N && i < ug.loc_fwd.size(); ++i) {
      if (ug.loc_fwd[i].empty() && ug.loc_rev[i].empty()) continue;
      Read::Locations& L = dataSet->getReadFromID(i)->locations();
      for (const mg::ReadLoc& l : ug.loc_fwd[i]) {
        L.edgesForward.push_back(made[l.edge]);
        L.locationForward.push_back(l.loc);
      }
      for (const mg::ReadLoc& l : ug.loc_rev[i]) {
        L.edgesReverse.push_back(made[l.edge]);
        L.locationReverse.push_back(l.loc);
      }
    }
  }
  numberOfNodes = ug.nodes;
  numberOfEdges = ug.edges;
}

void OverlapGraph::adoptEdgeLists() {
  // the Edge lists of a caller-driven build as compact records, numbered in
  // creation order (the .unitig writer's self-loop rule, mg_unitig.cpp)
  if (unitig || !graph) return;
  const UINT64 N = dataSet->getNumberOfUniqueReads();
  std::vector<Edge*> live;
  for (UINT64 u = 1; u <= N; ++u)
    for (Edge* e : *(*graph)[u]) live.push_back(e);
  std::sort(live.begin(), live.end(), [](Edge* a, Edge* b) { return a->serial < b->serial; });
  std::unordered_map<const Edge*, uint32_t> idx;
  idx.reserve(live.size() * 2);
  for (size_t i = 0; i < live.size(); ++i) idx[live[i]] = (uint32_t)i;
  std::vector<mg::GraphEdge> pool(live.size());
  for (size_t i = 0; i < live.size(); ++i) {
    Edge* e = live[i];
    auto it = idx.find(e->getReverseEdge());
    if (it == idx.end()) throw mg::Error("graph edge without its listed twin");
    pool[i] = mg::GraphEdge{(uint32_t)e->getSourceRead()->getReadNumber(),
                            (uint32_t)e->getDestinationRead()->getReadNumber(), (uint16_t)e->getOverlapOffset(),
                            e->getOrientation(), 0, it->second};
  }
  std::vector<std::vector<uint32_t>> lists(N + 1);
  for (UINT64 u = 1; u <= N; ++u)
    for (Edge* e : *(*graph)[u]) lists[u].push_back(idx[e]);
  unitig = new mg::UnitigGraph();
  unitig->init(pool, lists, numberOfNodes, numberOfEdges, N, true);
  materialize();
}

UINT64 OverlapGraph::contractCompositePaths() {
  adoptEdgeLists();
  if (!unitig) throw mg::Error("contractCompositePaths: no replayed graph");
  const UINT64 n = unitig->contract_composite_paths();
  if (unitig->bad_merge) throw mg::Error("Unable to merge.");  // OverlapGraph.cpp:830-833
  materialize();
  return n;
}

UINT64 OverlapGraph::removeDeadEndNodes() {
  adoptEdgeLists();
  if (!unitig) throw mg::Error("removeDeadEndNodes: no replayed graph");
  const UINT64 n = unitig->remove_dead_end_nodes();
  materialize();
  return n;
}

void OverlapGraph::sortEdges() {
  // :2799-2808; the Edge lists and the list state stay in step
  if (unitig) {
    unitig->sort_edges();
    materialize();
  } else if (graph) {
    for (size_t i = 1; i < graph->size(); ++i)
      std::sort((*graph)[i]->begin(), (*graph)[i]->end(), [](Edge* a, Edge* b) {
        return a->getDestinationRead()->getReadNumber() < b->getDestinationRead()->getReadNumber();
      });
  }
}

bool OverlapGraph::saveGraphToFile(const std::string& fileName) {
  adoptEdgeLists();
  if (!unitig) throw mg::Error("saveGraphToFile: no replayed graph");
  if (unitig->save_unitig(fileName.c_str())) throw mg::Error("Unable to open file: " + fileName);
  return true;
}

void OverlapGraph::markContainedReads() {
  // OverlapGraph.cpp:225-290 on the device; superReadID written back to Read
  if (!hashTable) throw mg::Error("markContainedReads: no hash table (the build released it)");
  mg_ctx* ctx = hashTable->context();
  const UINT64 N = dataSet->getNumberOfUniqueReads();
  std::vector<uint32_t> super(N + 1, 0);
  if (mg_mark_contained(ctx, super.data())) mg::fail(ctx, "markContainedReads");
  for (UINT64 i = 1; i <= N; ++i) {
    Read* r = dataSet->getReadFromID(i);
    r->superReadID = super[i];
    r->isContainedRead = super[i] != 0;
  }
  containedDone = true;
}

bool OverlapGraph::insertEdge(Edge* edge) {
  // OverlapGraph.cpp:390-400
  const UINT64 id = edge->getSourceRead()->getReadNumber();
  if ((*graph)[id]->empty()) numberOfNodes++;
  (*graph)[id]->push_back(edge);
  numberOfEdges++;
  return true;
}

bool OverlapGraph::insertEdge(Read* read1, Read* read2, UINT8 orient, UINT16 overlapOffset) {
  // OverlapGraph.cpp:407-419, twin orientation :841-855
  Edge* e1 = new Edge(read1, read2, orient, overlapOffset);
  const UINT16 rev = (UINT16)(read2->getReadLength() + overlapOffset - read1->getReadLength());
  const UINT8 tw = orient == 0 ? 3 : (orient == 3 ? 0 : orient);
  Edge* e2 = new Edge(read2, read1, tw, rev);
  e1->serial = nextSerial++;
  e2->serial = nextSerial++;
  e1->setReverseEdge(e2);
  e2->setReverseEdge(e1);
  insertEdge(e1);
  insertEdge(e2);
  return true;
}

bool OverlapGraph::buildOverlapGraphFromHashTable(HashTable* ht) {
  // OverlapGraph.cpp:107-218 up to the end of edge discovery: containment,
  // then every insertEdge of the exploration, on the device
  clear();
  hashTable = ht;
  dataSet = ht->getDataset();
  numberOfNodes = numberOfEdges = 0;
  const UINT64 N = dataSet->getNumberOfUniqueReads();
  graph = new std::vector<std::vector<Edge*>*>();
  graph->reserve(N + 1);
  for (UINT64 i = 0; i <= N; ++i) graph->push_back(new std::vector<Edge*>());
  markContainedReads();
  mg_ctx* ctx = ht->context();
  uint64_t nrows = 0;
  if (mg_find_overlaps(ctx, &nrows)) mg::fail(ctx, "buildOverlapGraphFromHashTable");
  std::vector<mg_edge> rows(nrows);
  uint64_t got = 0;
  if (mg_copy_rows(ctx, rows.data(), nrows, &got)) mg::fail(ctx, "copy rows");
  mg_get_timings(ctx, &lastTimings);
  if (!replayExploration) {
    // the raw discovery multiset: rows come in (edge, twin) pairs, as
    // insertEdge(Read*,...) creates them
    for (uint64_t k = 0; k + 1 < got; k += 2) {
      Read* u = dataSet->getReadFromID(rows[k].src);
      Read* v = dataSet->getReadFromID(rows[k].dst);
      Edge* e1 = new Edge(u, v, rows[k].orient, rows[k].offset);
      Edge* e2 = new Edge(v, u, rows[k + 1].orient, rows[k + 1].offset);
      e1->setReverseEdge(e2);
      e2->setReverseEdge(e1);
      insertEdge(e1);
      insertEdge(e2);
    }
    for (UINT64 i = 1; i <= N; ++i) {  // :562-563
      auto* lst = (*graph)[i];
      std::stable_sort(lst->begin(), lst->end(),
                       [](Edge* a, Edge* b) { return a->getOverlapOffset() < b->getOverlapOffset(); });
    }
  } else {
    // the reference's exploration order + transitive reduction (:144-204,
    // 574-661) replayed on the rows: same lists, same order, same counters
    mg::GraphReplay rp;
    const int rc = rp.build(rows.data(), got, dataSet->packedLengths(), N, (uint32_t)ht->getHashStringLength());
    if (rc) throw mg::Error("graph replay: rows inconsistent with the Dataset (" + std::to_string(rc) + ")");
    unitig = new mg::UnitigGraph();
    unitig->init(rp, N, true);
    if (contractPaths && unitig->contract() < 0) throw mg::Error("Unable to merge.");  // :211-215
    materialize();
  }
  delete ht;  // the graph owns and frees the table (:210)
  hashTable = nullptr;
  return true;
}

bool OverlapGraph::beginBuildFromHashTable(HashTable* ht) {
  // buildOverlapGraphFromHashTable's set-up (OverlapGraph.cpp:111-142); the
  // caller then explores (:144-204) through insertAllEdgesOfRead & co.
  clear();
  hashTable = ht;
  dataSet = ht->getDataset();
  numberOfNodes = numberOfEdges = 0;
  nextSerial = 0;
  const UINT64 N = dataSet->getNumberOfUniqueReads();
  graph = new std::vector<std::vector<Edge*>*>();
  graph->reserve(N + 1);
  for (UINT64 i = 0; i <= N; ++i) graph->push_back(new std::vector<Edge*>());
  markContainedReads();
  mg_ctx* ctx = ht->context();
  uint64_t nrows = 0;
  if (mg_find_overlaps(ctx, &nrows)) mg::fail(ctx, "beginBuildFromHashTable");
  std::vector<mg_edge> rows(nrows);
  uint64_t got = 0;
  if (mg_copy_rows(ctx, rows.data(), nrows, &got)) mg::fail(ctx, "copy rows");
  mg_get_timings(ctx, &lastTimings);
  manual = new Manual();
  manual->h = ht->getHashStringLength();
  const int rc = manual->D.build(rows.data(), got, dataSet->packedLengths(), N, (uint32_t)manual->h);
  if (rc) throw mg::Error("discoveries inconsistent with the Dataset (" + std::to_string(rc) + ")");
  // the table stays the caller's, who frees it after the build as the reference
  // does (:210, mg_explore_main.cpp): nothing here reads it again (h is captured)
  hashTable = nullptr;
  return true;
}

bool OverlapGraph::insertAllEdgesOfRead(UINT64 readNumber, std::vector<nodeType>* exploredReads) {
  // OverlapGraph.cpp:529-565: D(readNumber) in the loop order (j, then the
  // getListOfReads list: partner ID, then o); the device verified each one
  // (checkOverlap with both superReadIDs 0, :548)
  if (!manual) throw mg::Error("insertAllEdgesOfRead: call beginBuildFromHashTable first");
  Read* read1 = dataSet->getReadFromID(readNumber);
  const mg::Discoveries& D = manual->D;
  for (uint64_t k = D.start[readNumber]; k < D.start[readNumber + 1]; ++k) {
    const mg::Disc& d = D.disc[k];
    if (exploredReads->at(d.r2) != UNEXPLORED) continue;  // :546
    insertEdge(read1, dataSet->getReadFromID(d.r2), d.orient, d.offset);
  }
  std::vector<Edge*>* lst = (*graph)[readNumber];
  if (!lst->empty())  // compareEdges (:42-45): overlap offset ascending, std::sort as :563
    std::sort(lst->begin(), lst->end(), [](Edge* a, Edge* b) { return a->getOverlapOffset() < b->getOverlapOffset(); });
  return true;
}

bool OverlapGraph::markTransitiveEdges(UINT64 readNumber, std::vector<markType>* markedNodes) {
  // OverlapGraph.cpp:574-615 (Myers' transitive reduction, one read)
  std::vector<Edge*>& lu = *(*graph)[readNumber];
  for (Edge* e : lu) markedNodes->at(e->getDestinationRead()->getReadNumber()) = INPLAY;
  for (size_t i = 0; i < lu.size(); ++i) {
    const UINT64 read2 = lu[i]->getDestinationRead()->getReadNumber();
    if (markedNodes->at(read2) != INPLAY) continue;
    const UINT8 t1 = lu[i]->getOrientation();
    for (Edge* e2 : *(*graph)[read2]) {
      const UINT64 read3 = e2->getDestinationRead()->getReadNumber();
      if (markedNodes->at(read3) != INPLAY) continue;
      const UINT8 t2 = e2->getOrientation();
      if ((t1 == 0 || t1 == 2) && (t2 == 0 || t2 == 1))
        markedNodes->at(read3) = ELIMINATED;
      else if ((t1 == 1 || t1 == 3) && (t2 == 2 || t2 == 3))
        markedNodes->at(read3) = ELIMINATED;
    }
  }
  for (Edge* e : lu) {
    if (markedNodes->at(e->getDestinationRead()->getReadNumber()) == ELIMINATED) {
      e->transitiveRemovalFlag = true;
      e->getReverseEdge()->transitiveRemovalFlag = true;
    }
  }
  for (Edge* e : lu) markedNodes->at(e->getDestinationRead()->getReadNumber()) = VACANT;
  markedNodes->at(readNumber) = VACANT;
  return true;
}

bool OverlapGraph::removeTransitiveEdges(UINT64 readNumber) {
  // OverlapGraph.cpp:623-661: the twins first (the last edge of their list
  // moved into their place), then this read's marked edges, order kept
  std::vector<Edge*>& lu = *(*graph)[readNumber];
  for (size_t index = 0; index < lu.size(); ++index) {
    if (!lu[index]->transitiveRemovalFlag) continue;
    Edge* twin = lu[index]->getReverseEdge();
    std::vector<Edge*>& lt = *(*graph)[twin->getSourceRead()->getReadNumber()];
    for (size_t k = 0; k < lt.size(); ++k) {
      if (lt[k] == twin) {
        delete twin;
        lt[k] = lt.back();
        lt.pop_back();
        if (lt.empty()) numberOfNodes--;
        numberOfEdges--;
        break;
      }
    }
  }
  size_t j = 0;
  for (size_t index = 0; index < lu.size(); ++index) {
    if (!lu[index]->transitiveRemovalFlag) {
      lu[j++] = lu[index];
    } else {
      numberOfEdges--;
      delete lu[index];
    }
  }
  lu.resize(j);
  if (lu.empty()) numberOfNodes--;
  return true;
}

namespace {
UINT64 hash_string_length(HashTable* ht, UINT64 manual_h) {
  if (manual_h) return manual_h;  // captured by beginBuildFromHashTable (the table may be freed since)
  if (ht) return ht->getHashStringLength();
  throw mg::Error("checkOverlap: no hash table (the graph was built and its table freed)");
}
}  // namespace

bool OverlapGraph::checkOverlap(Read* read1, Read* read2, UINT64 orient, UINT64 start) {
  // OverlapGraph.cpp:354-383, the same unsigned arithmetic and substrings
  const std::string string1 = read1->getStringForward();
  const UINT64 h = hash_string_length(hashTable, manual ? manual->h : 0);
  const std::string string2 = (orient == 0 || orient == 1) ? read2->getStringForward() : read2->getStringReverse();
  if (orient == 0 || orient == 2) {
    if (string1.length() - start - h >= string2.length() - h) return false;  // :367
    return string1.substr(start + h, string1.length() - (start + h)) == string2.substr(h, string1.length() - (start + h));
  }
  if (string2.length() - h < start) return false;  // :379
  return string1.substr(0, start) == string2.substr(string2.length() - h - start, start);
}

bool OverlapGraph::checkOverlapForContainedRead(Read* read1, Read* read2, UINT64 orient, UINT64 start) {
  // OverlapGraph.cpp:302-340
  const std::string string1 = read1->getStringForward();
  const UINT64 h = hash_string_length(hashTable, manual ? manual->h : 0);
  const std::string string2 = (orient == 0 || orient == 1) ? read2->getStringForward() : read2->getStringReverse();
  if (orient == 0 || orient == 2) {
    const UINT64 rem1 = string1.length() - start - h, rem2 = string2.length() - h;
    if (rem1 >= rem2) return string1.substr(start + h, rem2) == string2.substr(h, rem2);
  } else {
    const UINT64 rem1 = start, rem2 = string2.length() - h;
    if (rem1 >= rem2) return string1.substr(start - rem2, rem2) == string2.substr(0, rem2);
  }
  return false;
}

bool OverlapGraph::readGraphFromFile(const std::string& fileName) {
  // OverlapGraph.cpp:1270-1367 (the -s resume of main.cpp:36-42)
  if (!dataSet) throw mg::Error("readGraphFromFile: setDataset first");
  clear();
  numberOfNodes = numberOfEdges = 0;
  unitig = new mg::UnitigGraph();
  const int rc = unitig->read_unitig(fileName.c_str(), dataSet->packedLengths(), dataSet->getNumberOfUniqueReads(), true);
  if (rc == -1) throw mg::Error("Unable to open file: " + fileName);
  if (rc) throw mg::Error("readGraphFromFile: malformed unitig file " + fileName);
  materialize();
  return true;
}

const std::vector<Edge*>* OverlapGraph::getEdges(UINT64 readNumber) const {
  if (!graph || readNumber >= graph->size()) return nullptr;
  return (*graph)[readNumber];
}

bool OverlapGraph::replayExploration = true;
bool OverlapGraph::contractPaths = true;

bool OverlapGraph::saveGraphLists(const std::string& fileName) const {
  if (!graph) return false;
  FILE* f = std::fopen(fileName.c_str(), "w");
  if (!f) return false;
  std::fprintf(f, "#C %llu %llu\n", (unsigned long long)numberOfNodes, (unsigned long long)numberOfEdges);
  for (size_t u = 1; u < graph->size(); ++u)
    for (Edge* e : *(*graph)[u])
      std::fprintf(f, "%llu %llu %u %llu\n", (unsigned long long)u,
                   (unsigned long long)e->getDestinationRead()->getReadNumber(), (unsigned)e->getOrientation(),
                   (unsigned long long)e->getOverlapOffset());
  std::fclose(f);
  return true;
}

bool OverlapGraph::saveRawEdges(const std::string& fileName) const {
  if (!graph) return false;
  struct Row {
    UINT64 u, v, o, off;
  };
  std::vector<Row> all;
  for (size_t u = 1; u < graph->size(); ++u)
    for (Edge* e : *(*graph)[u])
      all.push_back({e->getSourceRead()->getReadNumber(), e->getDestinationRead()->getReadNumber(),
                     e->getOrientation(), e->getOverlapOffset()});
  std::sort(all.begin(), all.end(), [](const Row& a, const Row& b) {
    if (a.u != b.u) return a.u < b.u;
    if (a.v != b.v) return a.v < b.v;
    if (a.o != b.o) return a.o < b.o;
    return a.off < b.off;
  });
  FILE* f = std::fopen(fileName.c_str(), "w");
  if (!f) return false;
  for (const Row& r : all) std::fprintf(f, "%llu %llu %llu %llu\n", r.u, r.v, r.o, r.off);
  std::fclose(f);
  return true;
}

// ================================================================ C-ABI ====
extern "C" {

struct mgh_dataset {
  Dataset* d;
};

int mgh_dataset_from_files(const char* const* files, int nfiles, uint64_t min_overlap, mgh_dataset** out) {
  if (!out) return -3;
  *out = nullptr;
  std::vector<std::string> se;
  for (int i = 0; i < nfiles; ++i) {
    std::ifstream f(files[i]);
    if (!f) return -1;
    int c = f.peek();
    if (c != '>' && c != '@') return -2;
    se.emplace_back(files[i]);
  }
  try {
    *out = new mgh_dataset{new Dataset({}, se, min_overlap)};
  } catch (const std::exception&) {
    return -1;
  }
  return 0;
}

int mgh_dataset_from_codes(const uint8_t* codes, uint64_t n, uint64_t stride, const uint16_t* lens,
                           uint64_t min_overlap, int nthreads, mgh_dataset** out) {
  if (!out) return -3;
  try {
    *out = new mgh_dataset{Dataset::fromCodes(codes, n, stride, lens, min_overlap, nthreads)};
  } catch (const std::exception&) {
    *out = nullptr;
    return -1;
  }
  return 0;
}

void mgh_dataset_free(mgh_dataset* ds) {
  if (!ds) return;
  delete ds->d;
  delete ds;
}

uint64_t mgh_num_reads(const mgh_dataset* ds) { return ds ? ds->d->getNumberOfReads() : 0; }
uint64_t mgh_num_unique(const mgh_dataset* ds) { return ds ? ds->d->getNumberOfUniqueReads() : 0; }
uint64_t mgh_shortest(const mgh_dataset* ds) { return ds ? ds->d->shortestReadLength : 0; }
uint64_t mgh_longest(const mgh_dataset* ds) { return ds ? ds->d->longestReadLength : 0; }

int mgh_packed(const mgh_dataset* ds, const uint64_t** words, const uint16_t** lens, uint32_t* wpr) {
  if (!ds) return -1;
  if (words) *words = ds->d->packedWords();
  if (lens) *lens = ds->d->packedLengths();
  if (wpr) *wpr = ds->d->wordsPerRead();
  return 0;
}

int64_t mgh_read_string(const mgh_dataset* ds, uint64_t id, char* buf, uint64_t cap) {
  if (!ds || id < 1 || id > ds->d->getNumberOfUniqueReads()) return -1;
  const std::string s = ds->d->decode(id, false);
  if (buf && cap) {
    const uint64_t c = std::min<uint64_t>(cap - 1, s.size());
    std::memcpy(buf, s.data(), c);
    buf[c] = 0;
  }
  return (int64_t)s.size();
}

uint32_t mgh_frequency(const mgh_dataset* ds, uint64_t id) {
  if (!ds || id < 1 || id > ds->d->getNumberOfUniqueReads()) return 0;
  return ds->d->frequencyOf(id);
}

uint64_t mgh_find_read(const mgh_dataset* ds, const char* s, uint64_t len) {
  if (!ds) return 0;
  try {
    return ds->d->getReadFromString(std::string(s, len))->getReadNumber();
  } catch (const std::exception&) {
    return 0;
  }
}

struct mgh_graph {
  mg::GraphReplay g;
  std::unique_ptr<mg::UnitigGraph> u;  // set once contracted
};

int mgh_graph_replay(const mg_edge* rows, uint64_t n_rows, const uint16_t* lens, uint64_t n_reads, uint32_t h,
                     mgh_graph** out) {
  if (!out || (n_rows && !rows) || (n_reads && !lens)) return -1;
  *out = nullptr;
  try {
    mgh_graph* g = new mgh_graph();
    const int rc = g->g.build(rows, n_rows, lens, n_reads, h);
    if (rc) {
      delete g;
      return rc;
    }
    *out = g;
  } catch (const std::exception&) {
    return -1;
  }
  return 0;
}

int mgh_graph_read_unitig(const char* path, const uint16_t* lens, uint64_t n_reads, mgh_graph** out) {
  if (!out || !path || (n_reads && !lens)) return -3;
  *out = nullptr;
  try {
    std::unique_ptr<mgh_graph> g(new mgh_graph());
    g->u.reset(new mg::UnitigGraph());
    const int rc = g->u->read_unitig(path, lens, n_reads, true);
    if (rc) return rc;
    *out = g.release();
  } catch (const std::exception&) {
    return -3;
  }
  return 0;
}

void mgh_graph_free(mgh_graph* g) { delete g; }
uint64_t mgh_graph_nodes(const mgh_graph* g) { return g ? (g->u ? g->u->nodes : g->g.nodes) : 0; }
uint64_t mgh_graph_edges(const mgh_graph* g) { return g ? (g->u ? g->u->edges : g->g.edges) : 0; }

uint64_t mgh_graph_rows(const mgh_graph* g, mg_edge* out, uint64_t cap) {
  if (!g || g->u) return 0;
  uint64_t n = 0;
  for (size_t u = 1; u < g->g.lists.size(); ++u) {
    for (uint32_t e : g->g.lists[u]) {
      if (out && n < cap) {
        const mg::GraphEdge& x = g->g.pool[e];
        out[n] = mg_edge{x.src, x.dst, x.offset, x.orient, 0};
      }
      n++;
    }
  }
  return out ? std::min(n, cap) : n;
}

int mgh_graph_contract(mgh_graph* g, int track_locations, uint64_t* iterations, uint64_t* merged,
                       uint64_t* dead_end_nodes) {
  if (!g || g->u) return -1;
  try {
    auto u = std::make_unique<mg::UnitigGraph>();
    u->init(g->g, g->g.lists.empty() ? 0 : g->g.lists.size() - 1, track_locations != 0);
    const int64_t it = u->contract();
    if (it < 0) return -4;
    if (iterations) *iterations = (uint64_t)it;
    if (merged) *merged = u->merged_total;
    if (dead_end_nodes) *dead_end_nodes = u->dead_end_total;
    g->u = std::move(u);
    // the pre-contraction graph is no longer needed
    std::vector<mg::GraphEdge>().swap(g->g.pool);
    std::vector<std::vector<uint32_t>>().swap(g->g.lists);
  } catch (const std::exception&) {
    return -1;
  }
  return 0;
}

int mgh_graph_sort_edges(mgh_graph* g) {
  if (!g || !g->u) return -1;
  g->u->sort_edges();
  return 0;
}

int mgh_graph_save_unitig(const mgh_graph* g, const char* path) {
  if (!g || !g->u || !path) return -1;
  return g->u->save_unitig(path);
}

int mgh_graph_save_lists(const mgh_graph* g, const char* path) {
  if (!g || !g->u || !path) return -1;
  return g->u->save_lists(path);
}

uint64_t mgh_graph_unitig_edges(const mgh_graph* g, mgh_unitig_edge* edges, uint64_t edge_cap,
                                uint64_t* read_start, uint32_t* reads, uint16_t* offs, uint8_t* ors,
                                uint64_t read_cap, uint64_t* n_reads_total) {
  if (!g || !g->u) return 0;
  const mg::UnitigGraph& u = *g->u;
  uint64_t k = 0, r = 0;
  for (size_t v = 1; v < u.lists.size(); ++v) {
    for (uint32_t e : u.lists[v]) {
      const mg::UnitigEdge& x = u.pool[e];
      const mg::EdgeReads* lr = u.reads[e].get();
      const uint32_t nr = lr ? (uint32_t)lr->reads.size() : 0;
      if (k < edge_cap) {
        if (edges) edges[k] = mgh_unitig_edge{x.src, x.dst, x.offset, nr, x.orient, {0, 0, 0}};
        if (read_start) read_start[k] = r;
      }
      for (uint32_t q = 0; q < nr; ++q, ++r) {
        if (r >= read_cap) continue;
        if (reads) reads[r] = lr->reads[q];
        if (offs) offs[r] = lr->offs[q];
        if (ors) ors[r] = lr->ors[q];
      }
      k++;
    }
  }
  if (n_reads_total) *n_reads_total = r;
  return k;
}

namespace {
int parse_out(int rc, mg::ParsedText& pt, const mg::ParseStats& st, char** text_out, uint64_t** off_out,
              uint64_t* n_records, double* seconds) {
  if (rc) {
    pt.release();
    return rc;
  }
  if (!pt.off) {  // no record at all
    pt.off = static_cast<uint64_t*>(std::calloc(1, sizeof(uint64_t)));
    if (!pt.off) return -3;
  }
  if (!pt.text) pt.text = static_cast<char*>(std::malloc(1));
  *text_out = pt.text;  // ownership passes to the caller (mgh_parse_free)
  *off_out = pt.off;
  *n_records = pt.n_rec;
  if (seconds) *seconds = st.seconds;
  return 0;
}
}  // namespace

int mgh_parse_file(const char* path, int nthreads, char** text_out, uint64_t** off_out, uint64_t* n_records,
                   double* seconds) {
  return mgh_parse_files(&path, 1, nthreads, text_out, off_out, n_records, seconds);
}

int mgh_parse_files(const char* const* paths, int nfiles, int nthreads, char** text_out, uint64_t** off_out,
                    uint64_t* n_records, double* seconds) {
  if (!paths || nfiles < 0 || !text_out || !off_out || !n_records) return -1;
  mg::ParsedText pt;
  mg::ParseStats st;
  double total = 0;
  try {
    for (int i = 0; i < nfiles; ++i) {
      if (!paths[i]) return parse_out(-1, pt, st, text_out, off_out, n_records, seconds);
      const int rc = mg::parse_file_parallel(paths[i], pt, nthreads, &st);
      total += st.seconds;
      if (rc) return parse_out(rc, pt, st, text_out, off_out, n_records, seconds);
    }
  } catch (const std::exception&) {
    return parse_out(-3, pt, st, text_out, off_out, n_records, seconds);
  }
  st.seconds = total;
  return parse_out(0, pt, st, text_out, off_out, n_records, seconds);
}

int mgh_parse_buffer(const char* buf, uint64_t n, int nthreads, char** text_out, uint64_t** off_out,
                     uint64_t* n_records, double* seconds) {
  if ((!buf && n) || !text_out || !off_out || !n_records) return -1;
  mg::ParsedText pt;
  mg::ParseStats st;
  int rc;
  try {
    rc = mg::parse_buffer_parallel(buf, n, pt, nthreads, &st);
  } catch (const std::exception&) {
    rc = -3;
  }
  return parse_out(rc, pt, st, text_out, off_out, n_records, seconds);
}

void mgh_parse_free(void* p) { std::free(p); }

void mgh_parse_set_min_chunk(uint64_t bytes) { mg::g_parse_min_chunk = bytes ? bytes : (1 << 20); }

}  // extern "C"

// ======================================================== HashTable C-ABI ====
extern "C" uint64_t mgh_hash_table_size(uint64_t n_unique) { return mg::prime_larger_than(n_unique * 8 + 1); }

extern "C" uint64_t mgh_hash_function(const char* key, uint64_t len, uint64_t table_size) {
  return mg::ref_hash(key, len, table_size);
}
