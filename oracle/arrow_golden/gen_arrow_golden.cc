// gen_arrow_golden.cc — golden-vector generator for the blocked Bloom filter spec.
//
// TEST INFRASTRUCTURE ONLY. Runs in the build container, never on the GPU box and never as part
// of the product. It links the Arrow Acero BlockedBloomFilter shipped with the pyarrow 25.0.0
// wheel (libarrow_acero.so.2500) — the filter the reference's README says it ported
// (/root/reference/README.md:23-32) and the spec north_star names — and dumps:
//   * the 136-byte BloomFilterMasks table (bloom_filter.h:42-91),
//   * filter sizing (log_num_blocks) for a list of row counts (BlockedBloomFilter::CreateEmpty),
//   * full filter words + Find() bit-vectors for seeded inputs (bloom_filter.h:113-125,163-193),
//   * Fold() results (bloom_filter.h:135-158),
// into tests/golden/ as raw little-endian .bin files plus golden_manifest.json.
//
// Key -> hash uses the restated DuckDB hash (MurmurHash64 finalizer, NULL -> NULL_HASH). DuckDB is
// absent from the container, so that step is NOT pinned by Arrow; it is restated identically in
// oracle/rpt_oracle.cpp and in the HIP kernels. Only the hash -> filter-bits step is pinned here.
//
// Private members are exposed ONLY in this harness, to dump the filter words.
#define private public
#include "arrow/acero/bloom_filter.h"
#undef private
#include "arrow/memory_pool.h"

#include <cinttypes>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

using arrow::acero::BlockedBloomFilter;
using arrow::acero::BloomFilterBuilder;
using arrow::acero::BloomFilterBuildStrategy;
using arrow::acero::BloomFilterMasks;

static std::string g_out;

static inline uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}
// Indexable splitmix64 stream: element i of stream `seed`.
static inline uint64_t sm64(uint64_t seed, uint64_t i) {
  return mix64(seed + (i + 1) * 0x9e3779b97f4a7c15ULL);
}
// Restated DuckDB hash (unpinned, see header).
static inline uint64_t murmur64(uint64_t x) {
  x ^= x >> 32;
  x *= 0xd6e8feb86659fd93ULL;
  x ^= x >> 32;
  x *= 0xd6e8feb86659fd93ULL;
  x ^= x >> 32;
  return x;
}
static const uint64_t kNullHash = 0xbf58476d1ce4e5b9ULL;

static uint64_t fnv1a(const void* p, size_t n) {
  const uint8_t* b = static_cast<const uint8_t*>(p);
  uint64_t h = 0xcbf29ce484222325ULL;
  for (size_t i = 0; i < n; i++) {
    h ^= b[i];
    h *= 0x100000001b3ULL;
  }
  return h;
}

static void write_bin(const std::string& name, const void* p, size_t n) {
  std::ofstream f(g_out + "/" + name, std::ios::binary);
  f.write(static_cast<const char*>(p), static_cast<std::streamsize>(n));
  if (!f) {
    fprintf(stderr, "write failed: %s\n", name.c_str());
    exit(1);
  }
}

static void check(const arrow::Status& st) {
  if (!st.ok()) {
    fprintf(stderr, "arrow error: %s\n", st.ToString().c_str());
    exit(1);
  }
}

static void build(BlockedBloomFilter* bf, int64_t size_rows, const std::vector<uint64_t>& hashes,
                  int64_t batch) {
  auto builder = BloomFilterBuilder::Make(BloomFilterBuildStrategy::SINGLE_THREADED);
  int64_t nb = hashes.empty() ? 1 : (static_cast<int64_t>(hashes.size()) + batch - 1) / batch;
  check(builder->Begin(1, 0, arrow::default_memory_pool(), size_rows, nb, bf));
  for (size_t i = 0; i < hashes.size(); i += static_cast<size_t>(batch)) {
    int64_t cnt = std::min<int64_t>(batch, static_cast<int64_t>(hashes.size() - i));
    check(builder->PushNextBatch(0, cnt, hashes.data() + i));
  }
}

static std::vector<uint8_t> find_bits(const BlockedBloomFilter& bf, const std::vector<uint64_t>& h) {
  std::vector<uint8_t> bv((h.size() + 7) / 8 + 8, 0);
  // 2048-row batches like DuckDB vectors; Find writes whole bytes so keep batches byte-aligned.
  for (size_t i = 0; i < h.size(); i += 2048) {
    int64_t cnt = std::min<int64_t>(2048, static_cast<int64_t>(h.size() - i));
    bf.Find(0, cnt, h.data() + i, bv.data() + i / 8, true);
  }
  bv.resize((h.size() + 7) / 8);
  // Cross-check the batched form against the scalar Find.
  for (size_t i = 0; i < h.size(); i++) {
    bool a = (bv[i / 8] >> (i % 8)) & 1;
    if (a != bf.Find(h[i])) {
      fprintf(stderr, "batched/scalar Find disagree at %zu\n", i);
      exit(1);
    }
  }
  return bv;
}

static std::ostringstream g_cases;
static bool g_first_case = true;

static void emit_case(const std::string& name, const std::string& inputs_json,
                      const BlockedBloomFilter& bf, const std::vector<uint64_t>* probe_h) {
  size_t nwords = static_cast<size_t>(bf.num_blocks_);
  write_bin(name + ".words.bin", bf.blocks_, nwords * 8);
  std::string find_json = "null";
  if (probe_h) {
    auto bv = find_bits(bf, *probe_h);
    write_bin(name + ".find.bin", bv.data(), bv.size());
    int64_t pass = 0;
    for (size_t i = 0; i < probe_h->size(); i++) pass += (bv[i / 8] >> (i % 8)) & 1;
    char buf[128];
    snprintf(buf, sizeof buf, "{\"file\": \"%s.find.bin\", \"pass\": %" PRId64 "}", name.c_str(), pass);
    find_json = buf;
  }
  if (!g_first_case) g_cases << ",\n";
  g_first_case = false;
  char buf[512];
  snprintf(buf, sizeof buf,
           "    \"%s\": {\"inputs\": %s,\n      \"log_num_blocks\": %d, \"num_hash_bits_used\": %d, "
           "\"num_bits_set\": %" PRId64 ", \"words\": \"%s.words.bin\", \"words_fnv1a\": \"%016" PRIx64
           "\", \"find\": ",
           name.c_str(), inputs_json.c_str(), bf.log_num_blocks(), bf.NumHashBitsUsed(), bf.NumBitsSet(),
           name.c_str(), fnv1a(bf.blocks_, nwords * 8));
  g_cases << buf << find_json << "}";
}

// Key streams (documented in tests/golden/README.md):
//   build key i            = (int64) sm64(seed, i)              [int32 cases: low 32 bits]
//   probe row r            = build key sm64(seed+2000, r) % n   if sm64(seed+1000, r) % 2 == 0
//                            (int64) sm64(seed+3000, r)          otherwise
//   null rows (if nulls=k) = rows with index % k == k-1 (both build and probe)
struct KeyCase {
  const char* name;
  uint64_t seed;
  int64_t n;
  int64_t m;
  int width;  // 64 or 32
  int nulls;  // 0 = none
  int64_t size_rows;  // rows passed to Begin (sizing); -1 => n
};

static uint64_t key_hash(int64_t key_bits, int width, bool is_null) {
  if (is_null) return kNullHash;
  if (width == 32) return murmur64(static_cast<uint64_t>(static_cast<uint32_t>(key_bits)));
  return murmur64(static_cast<uint64_t>(key_bits));
}

static void run_key_case(const KeyCase& c) {
  std::vector<uint64_t> h(static_cast<size_t>(c.n)), ph(static_cast<size_t>(c.m));
  for (int64_t i = 0; i < c.n; i++) {
    bool is_null = c.nulls && (i % c.nulls == c.nulls - 1);
    h[i] = key_hash(static_cast<int64_t>(sm64(c.seed, i)), c.width, is_null);
  }
  for (int64_t r = 0; r < c.m; r++) {
    int64_t k;
    if (sm64(c.seed + 1000, r) % 2 == 0 && c.n > 0) {
      k = static_cast<int64_t>(sm64(c.seed, sm64(c.seed + 2000, r) % c.n));
    } else {
      k = static_cast<int64_t>(sm64(c.seed + 3000, r));
    }
    bool is_null = c.nulls && (r % c.nulls == c.nulls - 1);
    ph[r] = key_hash(k, c.width, is_null);
  }
  BlockedBloomFilter bf;
  int64_t size_rows = c.size_rows < 0 ? c.n : c.size_rows;
  build(&bf, size_rows, h, 2048);
  char in[256];
  snprintf(in, sizeof in,
           "{\"kind\": \"keys\", \"seed\": %" PRIu64 ", \"n\": %" PRId64 ", \"m\": %" PRId64
           ", \"width\": %d, \"nulls\": %d, \"size_rows\": %" PRId64 "}",
           c.seed, c.n, c.m, c.width, c.nulls, size_rows);
  emit_case(c.name, in, bf, &ph);
}

int main(int argc, char** argv) {
  g_out = argc > 1 ? argv[1] : ".";

  // 1. mask table
  BloomFilterMasks masks;
  write_bin("masks.bin", masks.masks_, BloomFilterMasks::kTotalBytes);
  std::vector<uint64_t> mask_vals(BloomFilterMasks::kNumMasks);
  for (int i = 0; i < BloomFilterMasks::kNumMasks; i++) mask_vals[i] = masks.mask(i);
  write_bin("mask_values.bin", mask_vals.data(), mask_vals.size() * 8);

  // 2. sizing
  std::ostringstream sizing;
  const int64_t ns[] = {0, 1, 2, 63, 64, 65, 100, 127, 128, 129, 1000, 4096, 100000, 1000000,
                        10000000, 100000000, 1000000000LL, 8000000000LL};
  bool first = true;
  for (int64_t n : ns) {
    // CreateEmpty only sizes/allocates; for the huge counts size without allocating by computing
    // through a tiny builder run only where the allocation is affordable.
    int lnb;
    if (n <= 100000000) {
      BlockedBloomFilter bf;
      check(bf.CreateEmpty(n, arrow::default_memory_pool()));
      lnb = bf.log_num_blocks();
    } else {
      lnb = -1;  // not allocated here; the test derives it from the rule and checks the rest
    }
    if (lnb < 0) continue;
    if (!first) sizing << ", ";
    first = false;
    sizing << "[" << n << ", " << lnb << "]";
  }

  // 3. known-answer case
  {
    BlockedBloomFilter bf;
    std::vector<uint64_t> h = {1, 2, 0x0123456789abcdefULL};
    build(&bf, 16, h, 2048);
    std::vector<uint64_t> p = {1, 2, 3, 4, 0x0123456789abcdefULL, 5, 6, 7};
    emit_case("kat16", "{\"kind\": \"hashes\", \"size_rows\": 16, \"hashes\": [\"1\", \"2\", \"0x0123456789abcdef\"], "
              "\"probe\": [\"1\",\"2\",\"3\",\"4\",\"0x0123456789abcdef\",\"5\",\"6\",\"7\"]}",
              bf, &p);
  }

  // 4. raw-hash case: hashes are splitmix64 values directly (independent of the key hash)
  {
    const int64_t n = 100000, m = 50000;
    std::vector<uint64_t> h(n), p(m);
    for (int64_t i = 0; i < n; i++) h[i] = sm64(0xABC, i);
    for (int64_t r = 0; r < m; r++) p[r] = (r % 3 == 0) ? h[sm64(0xABD, r) % n] : sm64(0xABE, r);
    BlockedBloomFilter bf;
    build(&bf, n, h, 1000);  // odd batch size: batching must not matter
    emit_case("raw_hash_100k",
              "{\"kind\": \"raw\", \"n\": 100000, \"m\": 50000, \"build\": \"sm64(0xABC,i)\", "
              "\"probe\": \"r%3==0 ? build[sm64(0xABD,r)%n] : sm64(0xABE,r)\"}",
              bf, &p);
  }

  // 5. key cases (int64/int32, nulls, sizes on both sides of the 256 KB prefetch limit)
  const KeyCase kc[] = {
      {"k64_n1", 11, 1, 4096, 64, 0, -1},
      {"k64_n100", 12, 100, 4096, 64, 0, -1},
      {"k64_n1000", 13, 1000, 20000, 64, 0, -1},
      {"k64_n50000", 14, 50000, 20000, 64, 0, -1},
      {"k64_n300000", 15, 300000, 20000, 64, 0, -1},
      {"k32_n5000", 31, 5000, 20000, 32, 0, -1},
      {"k64_n3000_nulls7", 41, 3000, 10000, 64, 7, -1},
      {"k32_n3000_nulls5", 42, 3000, 10000, 32, 5, -1},
      {"k64_n20000_over", 51, 20000, 20000, 64, 0, 1000},  // undersized: 20k keys in a 1k-row filter
  };
  for (const auto& c : kc) run_key_case(c);

  // 6. fold cases
  {
    // 200k pushes of only 1000 distinct keys into a filter sized for 200k rows -> sparse -> folds.
    const int64_t n = 200000;
    std::vector<uint64_t> h(n);
    for (int64_t i = 0; i < n; i++) h[i] = murmur64(sm64(21, i % 1000));
    BlockedBloomFilter bf;
    build(&bf, n, h, 2048);
    int before = bf.log_num_blocks();
    bf.Fold();
    std::vector<uint64_t> p(20000);
    for (int64_t r = 0; r < 20000; r++)
      p[r] = murmur64(r % 2 ? sm64(21, sm64(22, r) % 1000) : sm64(23, r));
    char in[256];
    snprintf(in, sizeof in,
             "{\"kind\": \"fold\", \"n\": 200000, \"size_rows\": 200000, \"build\": \"murmur64(sm64(21, i %% 1000))\", "
             "\"probe\": \"murmur64(r%%2 ? sm64(21, sm64(22,r)%%1000) : sm64(23,r))\", \"log_num_blocks_before\": %d}",
             before);
    emit_case("fold_200k_dup1000", in, bf, &p);
  }
  {
    // 3 keys into a 100k-row filter -> folds down to the 2^4-block floor.
    std::vector<uint64_t> h = {murmur64(1), murmur64(2), murmur64(3)};
    BlockedBloomFilter bf;
    build(&bf, 100000, h, 2048);
    int before = bf.log_num_blocks();
    bf.Fold();
    std::vector<uint64_t> p;
    for (uint64_t k = 0; k < 4096; k++) p.push_back(murmur64(k));
    char in[256];
    snprintf(in, sizeof in,
             "{\"kind\": \"fold\", \"n\": 3, \"size_rows\": 100000, \"build\": \"murmur64(1..3)\", "
             "\"probe\": \"murmur64(0..4095)\", \"log_num_blocks_before\": %d}",
             before);
    emit_case("fold_100k_3keys", in, bf, &p);
  }
  {
    // Dense filter: Fold must be a no-op (SURVEY §8c known answer).
    const int64_t n = 100000;
    std::vector<uint64_t> h(n);
    for (int64_t i = 0; i < n; i++) h[i] = sm64(0xABC, i);
    BlockedBloomFilter bf;
    build(&bf, n, h, 2048);
    int before = bf.log_num_blocks();
    bf.Fold();
    char in[256];
    snprintf(in, sizeof in,
             "{\"kind\": \"fold\", \"n\": 100000, \"size_rows\": 100000, \"build\": \"sm64(0xABC,i)\", "
             "\"log_num_blocks_before\": %d}",
             before);
    emit_case("fold_dense_noop", in, bf, nullptr);
  }

  std::ofstream mf(g_out + "/golden_manifest.json");
  mf << "{\n  \"generator\": \"oracle/arrow_golden/gen_arrow_golden.cc\",\n"
     << "  \"arrow\": \"pyarrow 25.0.0 libarrow_acero.so.2500 (BlockedBloomFilter, SINGLE_THREADED builder)\",\n"
     << "  \"masks\": {\"file\": \"masks.bin\", \"bytes\": " << BloomFilterMasks::kTotalBytes
     << ", \"fnv1a\": \"";
  char hb[32];
  snprintf(hb, sizeof hb, "%016" PRIx64, fnv1a(masks.masks_, BloomFilterMasks::kTotalBytes));
  mf << hb << "\", \"values\": \"mask_values.bin\"},\n"
     << "  \"sizing\": [" << sizing.str() << "],\n"
     << "  \"cases\": {\n" << g_cases.str() << "\n  }\n}\n";
  printf("golden vectors written to %s\n", g_out.c_str());
  return 0;
}
