// cpu_crosscheck.cc — per-core speed of the CPU restatement (oracle/rpt_oracle.cpp, the bench's
// cpu_baseline "port") against Arrow Acero's own BlockedBloomFilter::Find, on the same hashes and the
// same filter (SURVEY §8d "CPU baseline ... cross-check: time libarrow_acero Find against the
// restatement per core").
//
// TEST INFRASTRUCTURE ONLY: runs in the build container (pyarrow 25.0.0's libarrow_acero.so.2500),
// never on the GPU box. Built and run by cpu_crosscheck.sh.
//
// Per filter size (1e5 / 1e7 / 1e8 build rows: the 128 KiB JOB-sized filter, C2, C3): build the Arrow
// filter from the hashes of the synthetic build keys (SURVEY §8d streams), copy its words into the
// oracle's layout (identical by the golden tests), then probe 2^24 synthetic probe hashes with
//   arrow   BlockedBloomFilter::Find(hardware_flags = 0, n, hashes, bitvec, prefetch) in 2048-row batches
//   port    rpt_oracle_find_hashes (the restatement) in 2048-row batches
// on ONE thread; the two bit vectors must be identical. Median of 5 timed runs after 1 warm-up.
#define private public
#include "arrow/acero/bloom_filter.h"
#undef private
#include "arrow/memory_pool.h"

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

using arrow::acero::BlockedBloomFilter;
using arrow::acero::BloomFilterBuilder;
using arrow::acero::BloomFilterBuildStrategy;

extern "C" {
uint64_t rpt_oracle_murmur64(uint64_t x);
void rpt_oracle_synth_build_keys(uint64_t start, uint64_t n, int64_t* out);
void rpt_oracle_synth_probe_keys(uint64_t n_build, uint32_t p_permille, uint64_t start, uint64_t n, int64_t* out);
void rpt_oracle_find_hashes(const uint64_t* words, int log_nb, const uint64_t* h, uint64_t n, uint8_t* bv);
double rpt_oracle_probe_mt(const uint64_t* words, int log_nb, const int64_t* keys, uint64_t n, int threads,
                           uint64_t* out_count);
}

static void check(const arrow::Status& st) {
  if (!st.ok()) {
    fprintf(stderr, "arrow error: %s\n", st.ToString().c_str());
    exit(1);
  }
}

template <typename F>
static double median_ms(F&& f) {
  f();  // warm-up
  std::vector<double> t;
  for (int r = 0; r < 5; r++) {
    const auto a = std::chrono::steady_clock::now();
    f();
    t.push_back(std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - a).count());
  }
  std::sort(t.begin(), t.end());
  return t[2];
}

int main() {
  const uint64_t n_probe = 1ULL << 24;
  constexpr int64_t kBatch = 2048;  // DuckDB vector size
  printf("# one thread; %llu probe hashes (p = 0.1) per run, 2048-row batches; ns per key, median of 5\n",
         static_cast<unsigned long long>(n_probe));
  for (uint64_t n_build : {100000ULL, 10000000ULL, 100000000ULL}) {
    std::vector<int64_t> keys(n_build);
    rpt_oracle_synth_build_keys(0, n_build, keys.data());
    std::vector<uint64_t> h(n_build);
    for (uint64_t i = 0; i < n_build; i++) h[i] = rpt_oracle_murmur64(static_cast<uint64_t>(keys[i]));
    BlockedBloomFilter bf;
    auto builder = BloomFilterBuilder::Make(BloomFilterBuildStrategy::SINGLE_THREADED);
    const int64_t nb = (static_cast<int64_t>(n_build) + kBatch - 1) / kBatch;
    check(builder->Begin(1, 0, arrow::default_memory_pool(), static_cast<int64_t>(n_build), nb, &bf));
    for (uint64_t i = 0; i < n_build; i += kBatch)
      check(builder->PushNextBatch(0, std::min<int64_t>(kBatch, static_cast<int64_t>(n_build - i)), h.data() + i));
    const int log_nb = bf.log_num_blocks();
    const uint64_t* words = reinterpret_cast<const uint64_t*>(bf.blocks_);
    std::vector<int64_t> pk(n_probe);
    rpt_oracle_synth_probe_keys(n_build, 100, 0, n_probe, pk.data());
    std::vector<uint64_t> ph(n_probe);
    for (uint64_t i = 0; i < n_probe; i++) ph[i] = rpt_oracle_murmur64(static_cast<uint64_t>(pk[i]));
    std::vector<uint8_t> bv_a(n_probe / 8 + 8, 0), bv_p(n_probe / 8 + 8, 0);
    const double ms_a = median_ms([&] {
      for (uint64_t i = 0; i < n_probe; i += kBatch)
        bf.Find(0, kBatch, ph.data() + i, bv_a.data() + i / 8, /*enable_prefetch=*/true);
    });
    const double ms_p = median_ms([&] {
      for (uint64_t i = 0; i < n_probe; i += kBatch)
        rpt_oracle_find_hashes(words, log_nb, ph.data() + i, kBatch, bv_p.data() + i / 8);
    });
    // with the key hash inside the timed loop: Arrow (hash a 2048-row vector, Find) against the bench's
    // cpu_baseline routine (rpt_oracle_probe_mt on one thread: hash + prefetch + LookupSel per vector)
    std::vector<uint64_t> hb(kBatch);
    const double ms_ah = median_ms([&] {
      for (uint64_t i = 0; i < n_probe; i += kBatch) {
        for (int64_t j = 0; j < kBatch; j++) hb[j] = rpt_oracle_murmur64(static_cast<uint64_t>(pk[i + j]));
        bf.Find(0, kBatch, hb.data(), bv_a.data() + i / 8, /*enable_prefetch=*/true);
      }
    });
    uint64_t survivors_mt = 0;
    const double ms_b = median_ms([&] { rpt_oracle_probe_mt(words, log_nb, pk.data(), n_probe, 1, &survivors_mt); });
    const bool same = memcmp(bv_a.data(), bv_p.data(), n_probe / 8) == 0;
    uint64_t pass = 0;
    for (uint64_t i = 0; i < n_probe / 8; i++) pass += __builtin_popcount(bv_p[i]);
    printf("build %9llu rows (2^%d blocks, %6.1f MiB): hashes given: arrow Find %5.2f, port find %5.2f ns/key | "
           "hash included: arrow %5.2f, cpu_baseline routine %5.2f ns/key (baseline/arrow %.2f); survivors %llu (%llu), "
           "bit vectors %s\n",
           static_cast<unsigned long long>(n_build), log_nb, (8.0 * (1ULL << log_nb)) / (1 << 20), ms_a * 1e6 / n_probe,
           ms_p * 1e6 / n_probe, ms_ah * 1e6 / n_probe, ms_b * 1e6 / n_probe, ms_b / ms_ah,
           static_cast<unsigned long long>(pass), static_cast<unsigned long long>(survivors_mt), same ? "identical" : "DIFFER");
    if (!same || survivors_mt != pass) return 1;
  }
  return 0;
}
