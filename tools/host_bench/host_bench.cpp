// host_bench.cpp — PCIe-inclusive throughput of the C++ host mirror (include/rpt_host.hpp): host-resident
// 2048-row DuckDB-style chunks are staged to the device, probed, and their selection vectors copied
// back, for batches of 1 .. 8192 chunks per device call (LookupSelBatch), plus the batched build.
// This is the rate a DuckDB shim calling the mirror would see; it is never the bench's `value`.
#include <chrono>
#include <cstdio>
#include <random>
#include <vector>

#include "rpt_host.hpp"

int main() {
  const int dev = 0;
  const size_t n_build = 10000000, n_probe = 1ULL << 25;  // 33.5M probe rows = 16384 chunks
  std::mt19937_64 rng(42);
  std::vector<int64_t> build(n_build), probe(n_probe);
  for (auto& k : build) k = static_cast<int64_t>(rng() >> 1);
  for (size_t i = 0; i < n_probe; i++) probe[i] = (rng() % 10 == 0) ? build[rng() % n_build] : static_cast<int64_t>(rng() >> 1);
  auto chunks_of = [](std::vector<int64_t>& v) {
    std::vector<rpt::DataChunk> cs;
    for (size_t lo = 0; lo < v.size(); lo += 2048) {
      rpt::DataChunk c;
      c.count = std::min<size_t>(2048, v.size() - lo);
      rpt::Vector x;
      x.key_type = rpt::KeyType::I64;
      x.data = v.data() + lo;
      c.data.push_back(x);
      cs.push_back(c);
    }
    return cs;
  };
  auto bchunks = chunks_of(build), pchunks = chunks_of(probe);
  rpt::DeviceContext ctx(dev);
  rpt::PTBloomFilter bf;
  bf.Initialize(dev, static_cast<uint32_t>(n_build));
  using clk = std::chrono::steady_clock;
  {
    std::vector<const rpt::DataChunk*> all;
    for (auto& c : bchunks) all.push_back(&c);
    bf.InsertBatch(ctx, all, {0});  // warm-up
    auto t0 = clk::now();
    bf.InsertBatch(ctx, all, {0});
    const double s = std::chrono::duration<double>(clk::now() - t0).count();
    printf("{\"op\": \"InsertBatch\", \"rows\": %zu, \"chunks_per_call\": %zu, \"rows_per_s\": %.4g}\n", n_build,
           all.size(), n_build / s);
  }
  bf.finalized_ = true;
  for (size_t per_call : {1, 16, 128, 1024, 8192}) {
    std::vector<rpt::SelectionVector> sels;
    size_t rows = 0, calls = 0, survivors = 0;
    const size_t max_calls = per_call == 1 ? 2000 : pchunks.size() / per_call;
    // warm-up call
    {
      std::vector<const rpt::DataChunk*> b;
      for (size_t k = 0; k < per_call; k++) b.push_back(&pchunks[k]);
      bf.LookupSelBatch(ctx, b, sels, {0});
    }
    auto t0 = clk::now();
    for (size_t c = 0; c < max_calls; c++) {
      std::vector<const rpt::DataChunk*> b;
      for (size_t k = 0; k < per_call; k++) b.push_back(&pchunks[c * per_call + k]);
      bf.LookupSelBatch(ctx, b, sels, {0});
      for (size_t k = 0; k < per_call; k++) {
        rows += pchunks[c * per_call + k].count;
        survivors += sels[k].size();
      }
      calls++;
    }
    const double s = std::chrono::duration<double>(clk::now() - t0).count();
    printf("{\"op\": \"LookupSelBatch\", \"chunks_per_call\": %zu, \"rows\": %zu, \"calls\": %zu, \"us_per_call\": %.1f, "
           "\"rows_per_s\": %.4g, \"pass_fraction\": %.4f}\n",
           per_call, rows, calls, s / calls * 1e6, rows / s, static_cast<double>(survivors) / rows);
  }
  return 0;
}
