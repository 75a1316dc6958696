// host_bench.cpp — PCIe-inclusive throughput of the C++ host mirror (include/rpt_host.hpp): host-resident
// 2048-row DuckDB-style chunks are staged to the device, probed, and their selection vectors copied
// back, for batches of 1 .. 16384 chunks per device call (LookupSelBatch, unpipelined and pipelined in
// stages of 0.5-4 Mi rows), plus the batched build and
// CREATE_BF end to end (parallel sink, Combine, Finalize's rehash from HBM vs from host chunks).
// This is the rate a DuckDB shim calling the mirror would see; it is never the bench's `value`.
#include <chrono>
#include <cstdio>
#include <memory>
#include <random>
#include <thread>
#include <vector>

#include <cstdlib>
#include <cstring>

#include <hip/hip_runtime_api.h>

#include "rpt_host.hpp"

int main(int argc, char** argv) {
  const int dev = 0;
  // --spin: host threads spin (hipDeviceScheduleSpin) instead of the runtime's default wait while a
  // synchronize waits for the device (per-vector call latency experiment)
  if (argc > 1 && std::strcmp(argv[1], "--spin") == 0) {
    if (hipSetDevice(dev) != hipSuccess || hipSetDeviceFlags(hipDeviceScheduleSpin) != hipSuccess) return 3;
    printf("{\"op\": \"config\", \"device_flags\": \"hipDeviceScheduleSpin\"}\n");
  }
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
    for (uint64_t pr : {uint64_t(~0ULL), uint64_t(1) << 20, uint64_t(1) << 21}) {
      ctx.pipeline_rows = pr;
      bf.InsertBatch(ctx, all, {0});  // warm-up
      auto t0 = clk::now();
      bf.InsertBatch(ctx, all, {0});
      const double s = std::chrono::duration<double>(clk::now() - t0).count();
      printf("{\"op\": \"InsertBatch\", \"rows\": %zu, \"chunks_per_call\": %zu, \"pipeline_rows\": %lld, \"rows_per_s\": %.4g}\n",
             n_build, all.size(), pr == ~0ULL ? -1LL : static_cast<long long>(pr), n_build / s);
    }
  }
  {  // per-vector Insert (an unbatched Sink): 2000 single 2048-row chunks
    rpt::PTBloomFilter one;
    one.Initialize(dev, static_cast<uint32_t>(n_build));
    one.Insert(ctx, bchunks[0], {0});  // warm-up
    auto t0 = clk::now();
    for (size_t c = 0; c < 2000; c++) one.Insert(ctx, bchunks[c], {0});
    const double s = std::chrono::duration<double>(clk::now() - t0).count();
    printf("{\"op\": \"Insert\", \"chunks_per_call\": 1, \"calls\": 2000, \"us_per_call\": %.1f, \"rows_per_s\": %.4g}\n",
           s / 2000 * 1e6, 2000 * 2048 / s);
  }
  bf.finalized_ = true;
  struct Case {
    size_t per_call;
    uint64_t pipeline_rows;  // ~0: one staged copy per call (no pipeline)
    unsigned threads = 8;    // flatten threads
  };
  std::vector<Case> cases = {{1, ~0ULL}, {8, ~0ULL}, {16, ~0ULL}, {128, ~0ULL}, {1024, ~0ULL}, {8192, ~0ULL}, {16384, ~0ULL}};
  for (size_t per_call : {8192, 16384})
    for (uint64_t pr : {uint64_t(1) << 20, uint64_t(1) << 21, uint64_t(1) << 22}) cases.push_back({per_call, pr});
  for (unsigned th : {4u, 12u, 16u}) cases.push_back({16384, uint64_t(1) << 22, th});
  for (const Case& cs : cases) {
    const size_t per_call = cs.per_call;
    ctx.pipeline_rows = cs.pipeline_rows;
    ctx.flatten_threads = cs.threads;
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
    printf("{\"op\": \"LookupSelBatch\", \"chunks_per_call\": %zu, \"pipeline_rows\": %lld, \"flatten_threads\": %u, \"rows\": %zu, "
           "\"calls\": %zu, \"us_per_call\": %.1f, \"rows_per_s\": %.4g, \"pass_fraction\": %.4f}\n",
           per_call, cs.pipeline_rows == ~0ULL ? -1LL : static_cast<long long>(cs.pipeline_rows), cs.threads, rows, calls,
           s / calls * 1e6, rows / s, static_cast<double>(survivors) / rows);
  }
  // USE_BF as DuckDB runs it: T operator threads, each with its own DeviceContext (stream + staging),
  // each calling LookupSel on one 2048-row vector at a time
  for (int T : {1, 4, 8, 16}) {
    const size_t per_thread = 1000;
    std::vector<std::unique_ptr<rpt::DeviceContext>> ctxs;
    for (int t = 0; t < T; t++) ctxs.push_back(std::make_unique<rpt::DeviceContext>(dev));
    for (int t = 0; t < T; t++) {  // warm-up: staging buffers
      rpt::SelectionVector sv;
      bf.LookupSel(*ctxs[t], pchunks[t], sv, {0});
    }
    std::vector<size_t> surv(T, 0);
    auto t0 = clk::now();
    std::vector<std::thread> th;
    for (int t = 0; t < T; t++)
      th.emplace_back([&, t] {
        rpt::SelectionVector sv;
        for (size_t c = 0; c < per_thread; c++) {
          bf.LookupSel(*ctxs[t], pchunks[(t * per_thread + c) % pchunks.size()], sv, {0});
          surv[t] += sv.size();
        }
      });
    for (auto& x : th) x.join();
    const double s = std::chrono::duration<double>(clk::now() - t0).count();
    const double rows = static_cast<double>(T) * per_thread * 2048;
    printf("{\"op\": \"LookupSel\", \"threads\": %d, \"calls_per_thread\": %zu, \"us_per_call\": %.1f, \"rows_per_s\": %.4g}\n",
           T, per_thread, s / per_thread * 1e6, rows / s);
  }
  // USE_BF's filter chain on one 2048-row vector per call: UseBF::Execute (K filters in one launch,
  // rpt_bf_probe_chain) against K LookupSel calls one after another (one launch + sync each: the
  // filter-by-filter loop's cost without its slicing), one operator thread
  {
    auto shared = std::shared_ptr<rpt::PTBloomFilter>(&bf, [](rpt::PTBloomFilter*) {});
    for (size_t K : {1, 2, 3, 4}) {
      rpt::UseBF ub(std::vector<std::shared_ptr<rpt::PTBloomFilter>>(K, shared), std::vector<uint64_t>(K, 0));
      const size_t calls = 2000;
      rpt::SelectionVector sv;
      ub.Execute(ctx, pchunks[0], sv);  // warm-up
      auto t0 = clk::now();
      for (size_t c = 0; c < calls; c++) ub.Execute(ctx, pchunks[c % pchunks.size()], sv);
      const double s_chain = std::chrono::duration<double>(clk::now() - t0).count();
      t0 = clk::now();
      for (size_t c = 0; c < calls; c++)
        for (size_t k = 0; k < K; k++) bf.LookupSel(ctx, pchunks[c % pchunks.size()], sv, {0});
      const double s_seq = std::chrono::duration<double>(clk::now() - t0).count();
      printf("{\"op\": \"UseBF::Execute\", \"filters\": %zu, \"calls\": %zu, \"us_per_call\": %.1f, "
             "\"us_per_call_filter_by_filter\": %.1f}\n",
             K, calls, s_chain / calls * 1e6, s_seq / calls * 1e6);
    }
  }
  // a caching USE_BF: UseBF::ExecuteBatch over 16 .. 1024 chunks per call (one filter)
  {
    rpt::UseBF ub({std::shared_ptr<rpt::PTBloomFilter>(&bf, [](rpt::PTBloomFilter*) {})}, {0});
    for (size_t per_call : {16, 128, 1024}) {
      std::vector<rpt::SelectionVector> outs;
      std::vector<const rpt::DataChunk*> b;
      for (size_t k = 0; k < per_call; k++) b.push_back(&pchunks[k]);
      ub.ExecuteBatch(ctx, b, outs);  // warm-up
      const size_t calls = std::min<size_t>(pchunks.size() / per_call, 256);
      auto t0 = clk::now();
      for (size_t c = 0; c < calls; c++) {
        b.clear();
        for (size_t k = 0; k < per_call; k++) b.push_back(&pchunks[c * per_call + k]);
        ub.ExecuteBatch(ctx, b, outs);
      }
      const double s = std::chrono::duration<double>(clk::now() - t0).count();
      printf("{\"op\": \"UseBF::ExecuteBatch\", \"chunks_per_call\": %zu, \"calls\": %zu, \"us_per_call\": %.1f, \"rows_per_s\": %.4g}\n",
             per_call, calls, s / calls * 1e6, static_cast<double>(calls) * per_call * 2048 / s);
    }
  }
  // CREATE_BF end to end on a 1e8-row build: 8 sink threads over 2048-row chunks (sink batches staged
  // to HBM), Combine, then Finalize with an under-estimated cardinality so the filter is resized and
  // rehashed -- from the HBM key segments -- versus the same rehash re-staging the materialized host
  // chunks over PCIe (each with a fresh DeviceContext, as Finalize has).
  {
    const size_t n_cb = 100000000;
    std::vector<int64_t> cb(n_cb);
    for (auto& k : cb) k = static_cast<int64_t>(rng() >> 1);
    auto cchunks = chunks_of(cb);
    for (uint64_t flush : {uint64_t(1) << 20, rpt::CreateBF::kDefaultSinkFlushRows, uint64_t(1) << 24}) {
      rpt::CreateBF create(dev, /*estimated_cardinality=*/1000, {0}, flush);
      const int T = 8;
      std::vector<std::unique_ptr<rpt::CreateBF::LocalState>> locals;
      for (int t = 0; t < T; t++) locals.push_back(create.MakeLocalState());
      auto t0 = clk::now();
      std::vector<std::thread> th;
      for (int t = 0; t < T; t++)
        th.emplace_back([&, t] {  // each thread sinks its chunks, then combines (as DuckDB's pipeline does)
          for (size_t k = t; k < cchunks.size(); k += T) create.Sink(*locals[t], cchunks[k]);
          create.Combine(*locals[t]);
        });
      for (auto& x : th) x.join();
      const double sink_s = std::chrono::duration<double>(clk::now() - t0).count();
      t0 = clk::now();
      create.Finalize();
      const double fin_s = std::chrono::duration<double>(clk::now() - t0).count();
      auto bfh = create.GetBloomFilter(0);
      const auto words = bfh->ExportWords();
      double hbm_s, host_s;
      {
        t0 = clk::now();
        rpt::DeviceContext c2(dev);
        bfh->ReinitializeAndRehash(c2, n_cb, create.DeviceKeys(0));
        hbm_s = std::chrono::duration<double>(clk::now() - t0).count();
      }
      std::vector<rpt::DataChunk> host_chunks;
      {
        auto gs = create.GetGlobalSourceState(1);
        rpt::CreateBF::LocalSourceState ls;
        rpt::DataChunk c;
        while (create.GetData(*gs, ls, c)) host_chunks.push_back(c);
      }
      {
        t0 = clk::now();
        rpt::DeviceContext c3(dev);
        bfh->ReinitializeAndRehash(c3, n_cb, host_chunks, {0});
        host_s = std::chrono::duration<double>(clk::now() - t0).count();
      }
      printf("{\"op\": \"CreateBF\", \"rows\": %zu, \"sink_threads\": %d, \"sink_flush_rows\": %llu, "
             "\"segments\": %zu, \"sink_combine_rows_per_s\": %.4g, \"finalize_ms\": %.2f, "
             "\"rehash_hbm_ms\": %.2f, \"rehash_from_host_ms\": %.2f, \"resized\": %s, \"same_words\": %s}\n",
             n_cb, T, static_cast<unsigned long long>(flush), create.DeviceKeys(0).segments().size(), n_cb / sink_s,
             fin_s * 1e3, hbm_s * 1e3, host_s * 1e3, create.Resized(0) ? "true" : "false",
             bfh->ExportWords() == words ? "true" : "false");
    }
  }
  return 0;
}
