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

namespace {
using clk = std::chrono::steady_clock;
double since(clk::time_point t0) { return std::chrono::duration<double>(clk::now() - t0).count(); }

void print_stats(const char* what, const rpt::DeviceContext::PipelineStats& ps, double calls) {
  printf("\"%s\": {\"stages_per_call\": %.1f, \"narrow_stages_per_call\": %.1f, \"flatten_ms\": %.3f, \"enqueue_ms\": %.3f, "
         "\"wait_copy_ms\": %.3f, \"wait_count_ms\": %.3f, \"wait_sel_ms\": %.3f, \"split_ms\": %.3f, \"total_ms\": %.3f}",
         what, ps.stages / calls, ps.narrow_stages / calls, ps.flatten_s / calls * 1e3, ps.enqueue_s / calls * 1e3,
         ps.wait_copy_s / calls * 1e3, ps.wait_count_s / calls * 1e3, ps.wait_sel_s / calls * 1e3, ps.split_s / calls * 1e3,
         ps.total_s / calls * 1e3);
}

// Narrow BIGINT keys (DeviceContext::narrow_keys): C2's shape (1e7 build keys, 2^25 probe rows in 2048-row FLAT
// chunks, p = 0.1) with keys below 2^32 (4-B low words over PCIe) and with random 63-bit keys (the narrow attempt
// fails on the first stage), InsertBatch and LookupSelBatch (4 Mi-row stages, 8 workers) with narrow_keys on / off.
int host_narrow(int dev) {
  const size_t n_build = 10000000, n_probe = 1ULL << 25;
  for (int ids : {1, 0}) {
    std::mt19937_64 rng(17);
    const uint64_t mask = ids ? 0xFFFFFFFFULL : (~0ULL >> 1);
    std::vector<int64_t> b(n_build), q(n_probe);
    for (auto& k : b) k = static_cast<int64_t>(rng() & mask);
    for (size_t i = 0; i < n_probe; i++) q[i] = (rng() % 10 == 0) ? b[rng() % n_build] : static_cast<int64_t>(rng() & mask);
    auto chunks = [](const std::vector<int64_t>& v) {
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
    auto bch = chunks(b), pch = chunks(q);
    std::vector<const rpt::DataChunk*> ball, pall;
    for (auto& c : bch) ball.push_back(&c);
    for (auto& c : pch) pall.push_back(&c);
    std::vector<uint64_t> words[2];
    std::vector<rpt::SelectionVector> sels[2];
    for (int cfg = 0; cfg < 3; cfg++) {
      const int on = cfg > 0 ? 1 : 0;
      const unsigned workers = cfg == 2 ? 16 : 8;
      rpt::DeviceContext ctx(dev);
      ctx.narrow_keys = on != 0;
      ctx.flatten_threads = workers;
      rpt::PTBloomFilter bf;
      bf.Initialize(dev, static_cast<uint32_t>(n_build));
      bf.InsertBatch(ctx, ball, {0});  // warm-up
      const int calls = 4;
      ctx.stats = {};
      double ins = 0;
      for (int c = 0; c < calls; c++) {
        const auto t0 = clk::now();
        bf.InsertBatch(ctx, ball, {0});
        ins += since(t0);
      }
      const auto ins_stats = ctx.stats;
      words[on] = bf.ExportWords();
      bf.finalized_ = true;
      bf.LookupSelBatch(ctx, pall, sels[on], {0});  // warm-up
      ctx.stats = {};
      double sec = 0;
      for (int c = 0; c < calls; c++) {
        const auto t0 = clk::now();
        bf.LookupSelBatch(ctx, pall, sels[on], {0});
        sec += since(t0);
      }
      size_t surv = 0;
      for (auto& sv : sels[on]) surv += sv.size();
      printf("{\"op\": \"host_path.narrow\", \"keys\": \"%s\", \"narrow_keys\": %s, \"workers\": %u, \"insert_rows_per_s\": %.4g, "
             "\"lookup_rows_per_s\": %.4g, \"pass_fraction\": %.4f, ",
             ids ? "int64 below 2^32" : "int64 random 63-bit", on ? "true" : "false", workers, calls * double(n_build) / ins,
             calls * double(n_probe) / sec, surv / double(n_probe));
      print_stats("insert_phases_per_call", ins_stats, calls);
      printf(", ");
      print_stats("lookup_phases_per_call", ctx.stats, calls);
      printf("}\n");
      fflush(stdout);
    }
    if (words[0] != words[1] || sels[0] != sels[1]) {
      fprintf(stderr, "narrow and plain results differ (%s)\n", ids ? "ids" : "random");
      return 1;
    }
  }
  return 0;
}

// Result bits back instead of sels (DeviceContext::bits_back): LookupSelBatch (2^25 rows, 4 Mi-row stages, 8
// workers) of BIGINT and INTEGER keys against C2's filter at pass fractions 0.1 / 0.5 / 0.9, on / off, compared.
int host_bits(int dev) {
  const size_t n_build = 10000000, n_probe = 1ULL << 25;
  std::mt19937_64 rng(23);
  std::vector<int64_t> b(n_build);
  for (auto& k : b) k = static_cast<int64_t>(rng() >> 1);
  std::vector<int32_t> b32(n_build);
  for (size_t i = 0; i < n_build; i++) b32[i] = static_cast<int32_t>(b[i]);
  for (int i32 = 0; i32 < 2; i32++) {
    auto chunks = [&](size_t n, const void* data) {
      std::vector<rpt::DataChunk> cs;
      for (size_t lo = 0; lo < n; lo += 2048) {
        rpt::DataChunk c;
        c.count = std::min<size_t>(2048, n - lo);
        rpt::Vector x;
        x.key_type = i32 ? rpt::KeyType::I32 : rpt::KeyType::I64;
        x.data = i32 ? static_cast<const void*>(static_cast<const int32_t*>(data) + lo)
                     : static_cast<const void*>(static_cast<const int64_t*>(data) + lo);
        c.data.push_back(x);
        cs.push_back(c);
      }
      return cs;
    };
    auto bch = chunks(n_build, i32 ? static_cast<const void*>(b32.data()) : static_cast<const void*>(b.data()));
    std::vector<const rpt::DataChunk*> ball;
    for (auto& c : bch) ball.push_back(&c);
    rpt::DeviceContext ctx(dev);
    rpt::PTBloomFilter bf;
    bf.Initialize(dev, static_cast<uint32_t>(n_build));
    bf.InsertBatch(ctx, ball, {0});
    bf.finalized_ = true;
    for (int pct : {10, 50, 90}) {
      std::vector<int64_t> q(n_probe);
      for (size_t i = 0; i < n_probe; i++) q[i] = (rng() % 100 < static_cast<uint64_t>(pct)) ? b[rng() % n_build] : static_cast<int64_t>(rng() >> 1);
      std::vector<int32_t> q32(i32 ? n_probe : 0);
      for (size_t i = 0; i < q32.size(); i++) q32[i] = static_cast<int32_t>(q[i]);
      auto pch = chunks(n_probe, i32 ? static_cast<const void*>(q32.data()) : static_cast<const void*>(q.data()));
      std::vector<const rpt::DataChunk*> pall;
      for (auto& c : pch) pall.push_back(&c);
      std::vector<rpt::SelectionVector> sels[2];
      for (int on : {0, 1}) {
        ctx.bits_back = on != 0;
        bf.LookupSelBatch(ctx, pall, sels[on], {0});  // warm-up
        ctx.stats = {};
        const int calls = 4;
        double sec = 0;
        for (int c = 0; c < calls; c++) {
          const auto t0 = clk::now();
          bf.LookupSelBatch(ctx, pall, sels[on], {0});
          sec += since(t0);
        }
        size_t surv = 0;
        for (auto& sv : sels[on]) surv += sv.size();
        printf("{\"op\": \"host_path.bits_back\", \"keys\": \"%s\", \"bits_back\": %s, \"lookup_rows_per_s\": %.4g, \"pass_fraction\": %.4f, ",
               i32 ? "int32" : "int64", on ? "true" : "false", calls * double(n_probe) / sec, surv / double(n_probe));
        print_stats("phases_per_call", ctx.stats, calls);
        printf("}\n");
        fflush(stdout);
      }
      if (sels[0] != sels[1]) {
        fprintf(stderr, "bits_back on / off differ\n");
        return 1;
      }
    }
  }
  return 0;
}

// Mid-size batches (a caching USE_BF flushing every 128 .. 4096 chunks): UseBF::ExecuteBatch with the default
// stages (4 Mi rows: batches under 8 Mi rows run unpipelined) against stages of a quarter of the batch (>= 128 Ki
// rows), one operator thread, 8 workers, C2's filter, p = 0.1.
int host_batch_sizes(int dev) {
  const size_t n_build = 10000000, n_probe = 1ULL << 24;
  std::mt19937_64 rng(29);
  std::vector<int64_t> b(n_build), q(n_probe);
  for (auto& k : b) k = static_cast<int64_t>(rng() >> 1);
  for (size_t i = 0; i < n_probe; i++) q[i] = (rng() % 10 == 0) ? b[rng() % n_build] : static_cast<int64_t>(rng() >> 1);
  auto chunks = [](const std::vector<int64_t>& v) {
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
  auto bch = chunks(b), pch = chunks(q);
  std::vector<const rpt::DataChunk*> ball;
  for (auto& c : bch) ball.push_back(&c);
  rpt::DeviceContext ctx(dev);
  auto bf = std::make_shared<rpt::PTBloomFilter>();
  bf->Initialize(dev, static_cast<uint32_t>(n_build));
  bf->InsertBatch(ctx, ball, {0});
  bf->finalized_ = true;
  // a second filter on a second (INTEGER, 50 % hits) column for the two-filter chain below
  std::vector<int32_t> b1(n_build), q1(n_probe);
  for (auto& k : b1) k = static_cast<int32_t>(rng());
  for (size_t i = 0; i < n_probe; i++) q1[i] = (rng() % 2 == 0) ? b1[rng() % n_build] : static_cast<int32_t>(rng());
  for (size_t i = 0; i < bch.size(); i++) {
    rpt::Vector x;
    x.key_type = rpt::KeyType::I32;
    x.data = b1.data() + 2048 * i;
    bch[i].data.push_back(x);
  }
  for (size_t i = 0; i < pch.size(); i++) {
    rpt::Vector x;
    x.key_type = rpt::KeyType::I32;
    x.data = q1.data() + 2048 * i;
    pch[i].data.push_back(x);
  }
  auto bf1 = std::make_shared<rpt::PTBloomFilter>();
  bf1->Initialize(dev, static_cast<uint32_t>(n_build));
  bf1->InsertBatch(ctx, ball, {1});
  bf1->finalized_ = true;
  rpt::UseBF ub2({bf, bf1}, {0, 1});
  for (size_t per : {128, 512, 1024, 2048}) {
    const size_t calls = pch.size() / per;
    std::vector<rpt::SelectionVector> outs;
    std::vector<const rpt::DataChunk*> bt;
    for (size_t k = 0; k < per; k++) bt.push_back(&pch[k]);
    ub2.ExecuteBatch(ctx, bt, outs);  // warm-up
    double best = 0;
    for (int rep = 0; rep < 3; rep++) {  // best of 3 passes (small calls are latency-bound and noisy)
      const auto t0 = clk::now();
      for (size_t c = 0; c < calls; c++) {
        bt.clear();
        for (size_t k = 0; k < per; k++) bt.push_back(&pch[c * per + k]);
        ub2.ExecuteBatch(ctx, bt, outs);
      }
      best = std::max(best, static_cast<double>(calls) * per * 2048 / since(t0));
    }
    printf("{\"op\": \"host_path.batch_size.chain2\", \"chunks_per_call\": %zu, \"rows_per_s\": %.4g}\n", per, best);
    fflush(stdout);
  }
  rpt::UseBF ub({bf}, {0});
  for (size_t per : {128, 512, 1024, 2048, 4096}) {
    const size_t calls = pch.size() / per;
    double rate[2];
    for (int quarter = 0; quarter < 2; quarter++) {
      ctx.pipeline_rows = quarter ? std::max<uint64_t>(1u << 17, per * 2048 / 4) : (1ULL << 22);
      std::vector<rpt::SelectionVector> outs;
      std::vector<const rpt::DataChunk*> bt;
      for (size_t k = 0; k < per; k++) bt.push_back(&pch[k]);
      ub.ExecuteBatch(ctx, bt, outs);  // warm-up
      rate[quarter] = 0;
      for (int rep = 0; rep < 3; rep++) {  // best of 3 passes
        const auto t0 = clk::now();
        for (size_t c = 0; c < calls; c++) {
          bt.clear();
          for (size_t k = 0; k < per; k++) bt.push_back(&pch[c * per + k]);
          ub.ExecuteBatch(ctx, bt, outs);
        }
        rate[quarter] = std::max(rate[quarter], static_cast<double>(calls) * per * 2048 / since(t0));
      }
    }
    printf("{\"op\": \"host_path.batch_size\", \"chunks_per_call\": %zu, \"default_stages_rows_per_s\": %.4g, "
           "\"quarter_stages_rows_per_s\": %.4g}\n", per, rate[0], rate[1]);
    fflush(stdout);
  }
  ctx.pipeline_rows = 1ULL << 22;
  return 0;
}

// The host -> device path of a DuckDB shim for JOB's INTEGER keys and for BIGINT keys:
// FLAT int64, FLAT int32 and DICTIONARY int32 2048-row chunks through LookupSelBatch's pipeline (4 Mi-row
// stages) with 1..16 worker threads per call, the host-side time of each phase per call (DeviceContext::
// stats), then T operator threads each driving its own DeviceContext through UseBF::ExecuteBatch.
int host_path(int dev, bool trace) {
  const size_t n_build = 10000000, n_probe = 1ULL << 25;  // C2's filter; 33.5M probe rows = 16384 chunks
  std::mt19937_64 rng(7);
  std::vector<int64_t> b64(n_build), p64(n_probe);
  for (auto& k : b64) k = static_cast<int64_t>(rng() >> 1);
  for (size_t i = 0; i < n_probe; i++) p64[i] = (rng() % 10 == 0) ? b64[rng() % n_build] : static_cast<int64_t>(rng() >> 1);
  std::vector<int32_t> b32(n_build), p32(n_probe);
  for (size_t i = 0; i < n_build; i++) b32[i] = static_cast<int32_t>(b64[i]);
  for (size_t i = 0; i < n_probe; i++) p32[i] = static_cast<int32_t>(p64[i]);
  // DICTIONARY int32 chunks: a 64 Ki-entry dictionary (a tenth of it build keys) and a random selection
  const size_t n_dict = 1 << 16;
  std::vector<int32_t> dict(n_dict);
  for (size_t i = 0; i < n_dict; i++) dict[i] = (i % 10 == 0) ? b32[rng() % n_build] : static_cast<int32_t>(rng());
  std::vector<uint32_t> dsel(n_probe);
  for (auto& x : dsel) x = static_cast<uint32_t>(rng() % n_dict);
  auto make = [&](const char* kind) {
    std::vector<rpt::DataChunk> cs;
    for (size_t lo = 0; lo < n_probe; lo += 2048) {
      rpt::DataChunk c;
      c.count = std::min<size_t>(2048, n_probe - lo);
      rpt::Vector x;
      if (std::strcmp(kind, "i64_flat") == 0) {
        x.key_type = rpt::KeyType::I64;
        x.data = p64.data() + lo;
      } else if (std::strcmp(kind, "i32_flat") == 0) {
        x.key_type = rpt::KeyType::I32;
        x.data = p32.data() + lo;
      } else {
        x.type = rpt::VectorType::DICTIONARY;
        x.key_type = rpt::KeyType::I32;
        x.data = dict.data();
        x.sel = dsel.data() + lo;
        x.dict_size = n_dict;
      }
      c.data.push_back(x);
      cs.push_back(c);
    }
    return cs;
  };
  auto build_chunks = [&](bool i32) {
    std::vector<rpt::DataChunk> cs;
    for (size_t lo = 0; lo < n_build; lo += 2048) {
      rpt::DataChunk c;
      c.count = std::min<size_t>(2048, n_build - lo);
      rpt::Vector x;
      x.key_type = i32 ? rpt::KeyType::I32 : rpt::KeyType::I64;
      x.data = i32 ? static_cast<const void*>(b32.data() + lo) : static_cast<const void*>(b64.data() + lo);
      c.data.push_back(x);
      cs.push_back(c);
    }
    return cs;
  };
  const std::vector<const char*> kinds = trace ? std::vector<const char*>{"i64_flat", "i32_flat"}
                                               : std::vector<const char*>{"i64_flat", "i32_flat", "i32_dict"};
  for (const char* kind : kinds) {
    const bool i32 = kind[1] == '3';
    const size_t key_bytes = i32 ? 4 : 8;
    auto pch = make(kind);
    auto bch = build_chunks(i32);
    rpt::DeviceContext ctx(dev);
    auto bf = std::make_shared<rpt::PTBloomFilter>();
    bf->Initialize(dev, static_cast<uint32_t>(n_build));
    {
      std::vector<const rpt::DataChunk*> all;
      for (auto& c : bch) all.push_back(&c);
      bf->InsertBatch(ctx, all, {0});  // warm-up
      ctx.stats = {};
      const auto t0 = clk::now();
      bf->InsertBatch(ctx, all, {0});
      const double sec = since(t0);
      printf("{\"op\": \"host_path.InsertBatch\", \"keys\": \"%s\", \"rows\": %zu, \"rows_per_s\": %.4g, ", i32 ? "i32_flat" : "i64_flat",
             n_build, n_build / sec);
      print_stats("phases", ctx.stats, 1);
      printf("}\n");
    }
    bf->finalized_ = true;
    std::vector<const rpt::DataChunk*> all;
    for (auto& c : pch) all.push_back(&c);
    std::vector<rpt::SelectionVector> sels;
    for (uint64_t stage : {uint64_t(1) << 21, uint64_t(1) << 22, uint64_t(1) << 23})
      for (unsigned th : {1u, 2u, 4u, 8u, 16u}) {
        if (stage != (uint64_t(1) << 22) && th != 8) continue;
        if (trace && (stage != (uint64_t(1) << 22) || th != 8)) continue;
        ctx.pipeline_rows = stage;
        ctx.flatten_threads = th;
        bf->LookupSelBatch(ctx, all, sels, {0});  // warm-up (pool, staging)
        ctx.stats = {};
        const int calls = 4;
        size_t surv = 0;
        double sec = 0;
        for (int c = 0; c < calls; c++) {
          // --host-path-trace: 20 ms of idle between calls, so a copy trace shows each call on its own
          if (trace) std::this_thread::sleep_for(std::chrono::milliseconds(20));
          const auto t0 = clk::now();
          bf->LookupSelBatch(ctx, all, sels, {0});
          sec += since(t0);
          for (auto& sv : sels) surv += sv.size();
        }
        const double rows = static_cast<double>(calls) * n_probe;
        printf("{\"op\": \"host_path.LookupSelBatch\", \"keys\": \"%s\", \"chunks_per_call\": %zu, \"pipeline_rows\": %llu, "
               "\"worker_threads\": %u, \"rows_per_s\": %.4g, \"h2d_GBps\": %.1f, \"pass_fraction\": %.4f, ",
               kind, all.size(), static_cast<unsigned long long>(stage), th, rows / sec, rows * key_bytes / sec / 1e9,
               surv / rows);
        print_stats("phases_per_call", ctx.stats, calls);
        printf("}\n");
        fflush(stdout);
      }
    // T operator threads (DuckDB's parallel USE_BF), each with its own DeviceContext, each calling
    // UseBF::ExecuteBatch on 4096-chunk (8 Mi-row) batches of the column
    for (int T : {1, 2, 4, 8, 16}) {
      if (trace) break;
      const unsigned per_ctx = std::max(1, 16 / T);
      std::vector<std::unique_ptr<rpt::DeviceContext>> ctxs;
      std::vector<std::unique_ptr<rpt::UseBF>> ops;
      for (int t = 0; t < T; t++) {
        ctxs.push_back(std::make_unique<rpt::DeviceContext>(dev));
        ctxs.back()->flatten_threads = per_ctx;
        ops.push_back(std::make_unique<rpt::UseBF>(std::vector<std::shared_ptr<rpt::PTBloomFilter>>{bf}, std::vector<uint64_t>{0}));
      }
      const size_t per_batch = 4096, batches_per_thread = 4;
      auto batch = [&](int t, size_t k) {
        std::vector<const rpt::DataChunk*> b;
        const size_t first = ((static_cast<size_t>(t) * batches_per_thread + k) * per_batch) % pch.size();
        for (size_t j = 0; j < per_batch; j++) b.push_back(&pch[(first + j) % pch.size()]);
        return b;
      };
      for (int t = 0; t < T; t++) {  // warm-up
        std::vector<rpt::SelectionVector> outs;
        ops[t]->ExecuteBatch(*ctxs[t], batch(t, 0), outs);
      }
      std::vector<size_t> surv(T, 0);
      const auto t0 = clk::now();
      std::vector<std::thread> th;
      for (int t = 0; t < T; t++)
        th.emplace_back([&, t] {
          std::vector<rpt::SelectionVector> outs;
          for (size_t k = 0; k < batches_per_thread; k++) surv[t] += ops[t]->ExecuteBatch(*ctxs[t], batch(t, k), outs);
        });
      for (auto& x : th) x.join();
      const double sec = since(t0);
      const double rows = static_cast<double>(T) * batches_per_thread * per_batch * 2048;
      size_t s_all = 0;
      for (size_t x : surv) s_all += x;
      printf("{\"op\": \"host_path.ExecuteBatch\", \"keys\": \"%s\", \"operator_threads\": %d, \"worker_threads_per_context\": %u, "
             "\"chunks_per_call\": %zu, \"rows_per_s\": %.4g, \"h2d_GBps\": %.1f, \"pass_fraction\": %.4f}\n",
             kind, T, per_ctx, per_batch, rows / sec, rows * key_bytes / sec / 1e9, s_all / rows);
      fflush(stdout);
    }
  }
  return 0;
}
// USE_BF's filter chain over large batches (UseBF::ExecuteBatch with 1..3 applicable filters on three key
// columns: BIGINT 10% hits, INTEGER 50% hits, BIGINT 50% hits): the pipelined chain (4 Mi-row stages, 8 worker
// threads) beside the filter-by-filter path (the whole batch per filter, pipeline_rows beyond the batch), both
// checked equal.
int host_chain(int dev, bool ids) {
  const size_t n_build = 10000000, n_probe = 1ULL << 25;
  std::mt19937_64 rng(11);
  const uint64_t m64 = ids ? 0xFFFFFFFFULL : ~0ULL;  // --chain-ids: BIGINT keys below 2^32 (narrow over PCIe)
  std::vector<int64_t> b0(n_build), b2(n_build), p0(n_probe), p2(n_probe);
  std::vector<int32_t> b1(n_build), p1(n_probe);
  for (size_t i = 0; i < n_build; i++) {
    b0[i] = static_cast<int64_t>((rng() >> 1) & m64);
    b1[i] = static_cast<int32_t>(rng());
    b2[i] = static_cast<int64_t>((rng() >> 1) & m64);
  }
  for (size_t i = 0; i < n_probe; i++) {
    p0[i] = (rng() % 10 == 0) ? b0[rng() % n_build] : static_cast<int64_t>((rng() >> 1) & m64);
    p1[i] = (rng() % 2 == 0) ? b1[rng() % n_build] : static_cast<int32_t>(rng());
    p2[i] = (rng() % 2 == 0) ? b2[rng() % n_build] : static_cast<int64_t>((rng() >> 1) & m64);
  }
  auto chunks = [](size_t n, const int64_t* c0, const int32_t* c1, const int64_t* c2) {
    std::vector<rpt::DataChunk> cs;
    for (size_t lo = 0; lo < n; lo += 2048) {
      rpt::DataChunk c;
      c.count = std::min<size_t>(2048, n - lo);
      c.data.resize(3);
      c.data[0].key_type = rpt::KeyType::I64;
      c.data[0].data = c0 + lo;
      c.data[1].key_type = rpt::KeyType::I32;
      c.data[1].data = c1 + lo;
      c.data[2].key_type = rpt::KeyType::I64;
      c.data[2].data = c2 + lo;
      cs.push_back(c);
    }
    return cs;
  };
  auto bch = chunks(n_build, b0.data(), b1.data(), b2.data());
  auto pch = chunks(n_probe, p0.data(), p1.data(), p2.data());
  std::vector<const rpt::DataChunk*> ball, pall;
  for (auto& c : bch) ball.push_back(&c);
  for (auto& c : pch) pall.push_back(&c);
  rpt::DeviceContext ctx(dev);
  ctx.flatten_threads = 8;
  std::vector<std::shared_ptr<rpt::PTBloomFilter>> fs;
  for (uint64_t col = 0; col < 3; col++) {
    auto f = std::make_shared<rpt::PTBloomFilter>();
    f->Initialize(dev, static_cast<uint32_t>(n_build));
    f->InsertBatch(ctx, ball, {col});
    f->finalized_ = true;
    fs.push_back(f);
  }
  const double rows = static_cast<double>(n_probe);
  for (size_t k = 1; k <= 3; k++) {
    rpt::UseBF ub(std::vector<std::shared_ptr<rpt::PTBloomFilter>>(fs.begin(), fs.begin() + k),
                  k == 1 ? std::vector<uint64_t>{0} : k == 2 ? std::vector<uint64_t>{0, 1} : std::vector<uint64_t>{0, 1, 2});
    std::vector<rpt::SelectionVector> ref, outs;
    const int calls = 4;
    uint64_t surv = 0;
    double sec_ref = 0;
    ctx.pipeline_rows = ~0ULL / 4;  // filter by filter: the whole batch per filter
    ub.ExecuteBatch(ctx, pall, ref);  // warm-up
    for (int c = 0; c < calls; c++) {
      const auto t0 = clk::now();
      surv = ub.ExecuteBatch(ctx, pall, ref);
      sec_ref += since(t0);
    }
    for (uint64_t stage : {uint64_t(1) << 21, uint64_t(1) << 22}) {
      ctx.pipeline_rows = stage;
      ub.ExecuteBatch(ctx, pall, outs);  // warm-up
      ctx.stats = {};
      double sec = 0;
      for (int c = 0; c < calls; c++) {
        const auto t0 = clk::now();
        ub.ExecuteBatch(ctx, pall, outs);
        sec += since(t0);
      }
      size_t bad = 0;
      for (size_t i = 0; i < pall.size(); i++) bad += outs[i] != ref[i];
      if (bad) {
        fprintf(stderr, "chain of %zu: pipelined and filter-by-filter sels differ in %zu chunks\n", k, bad);
        return 1;
      }
      printf("{\"op\": \"host_path.ExecuteBatch.chain\", \"keys\": \"%s\", \"filters\": %zu, \"chunks_per_call\": %zu, \"worker_threads\": 8, "
             "\"pass_fraction\": %.4f, \"filter_by_filter_rows_per_s\": %.4g, \"pipelined_rows_per_s\": %.4g, \"pipeline_rows\": %llu, ",
             ids ? "BIGINT below 2^32" : "BIGINT random 63-bit", k, pall.size(), surv / rows, calls * rows / sec_ref,
             calls * rows / sec, static_cast<unsigned long long>(stage));
      print_stats("phases_per_call", ctx.stats, calls);
      printf("}\n");
      fflush(stdout);
    }
  }
  return 0;
}
// CREATE_BF end to end on a 1e8-row build: 8 sink threads over 2048-row chunks (sink batches staged
// to HBM), Combine, then Finalize with an under-estimated cardinality so the filter is resized and
// rehashed -- from the HBM key segments -- versus the same rehash re-staging the materialized host
// chunks over PCIe (each with a fresh DeviceContext, as Finalize has); every flush size with the sink's
// flushes synchronous and asynchronous (LocalState::async_flush).
int create_bf(int dev) {
  std::mt19937_64 rng(43);
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
  {
    const size_t n_cb = 100000000;
    std::vector<int64_t> cb(n_cb);
    for (auto& k : cb) k = static_cast<int64_t>(rng() >> 1);
    auto cchunks = chunks_of(cb);
    {  // what pinning costs: hipHostMalloc + hipHostFree of a 32 MiB staging buffer
      const int reps = 8;
      double ms = 0, free_ms = 0;
      for (int r = 0; r < reps; r++) {
        void* p = nullptr;
        auto t0 = clk::now();
        if (hipHostMalloc(&p, size_t(32) << 20, hipHostMallocDefault) != hipSuccess) return 3;
        ms += since(t0) * 1e3;
        t0 = clk::now();
        (void)hipHostFree(p);
        free_ms += since(t0) * 1e3;
      }
      double dms = 0;
      for (int r = 0; r < reps; r++) {
        void* p = nullptr;
        auto t0 = clk::now();
        if (hipMalloc(&p, size_t(32) << 20) != hipSuccess) return 3;
        dms += since(t0) * 1e3;
        (void)hipFree(p);
      }
      printf("{\"op\": \"hipHostMalloc\", \"bytes\": %zu, \"malloc_ms\": %.3f, \"free_ms\": %.3f, \"hipMalloc_ms\": %.3f}\n",
             size_t(32) << 20, ms / reps, free_ms / reps, dms / reps);
    }
    for (uint64_t flush : {uint64_t(1) << 20, rpt::CreateBF::kDefaultSinkFlushRows, uint64_t(1) << 24})
    for (bool async : {false, true})
    for (bool warm : {false, true})
    for (unsigned workers : {8u, 2u}) {
      if (flush != rpt::CreateBF::kDefaultSinkFlushRows && (!warm || workers != 2)) continue;
      if (!warm) rpt::ReleasePinnedCache();  // cold: every sink state pins its staging afresh
      rpt::CreateBF create(dev, /*estimated_cardinality=*/1000, {0}, flush);
      const int T = 8;
      std::vector<std::unique_ptr<rpt::CreateBF::LocalState>> locals;
      for (int t = 0; t < T; t++) {
        locals.push_back(create.MakeLocalState());
        locals.back()->async_flush = async;
        locals.back()->ctx.flatten_threads = workers;
      }
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
      double mat_s = 0, fl_s = 0;
      for (auto& l : locals) {
        mat_s += l->materialize_s;
        fl_s += l->flush_s;
      }
      printf("{\"op\": \"CreateBF\", \"rows\": %zu, \"sink_threads\": %d, \"sink_flush_rows\": %llu, \"async_flush\": %s, \"pinned_cache\": \"%s\", \"workers_per_state\": %u, "
             "\"segments\": %zu, \"sink_combine_rows_per_s\": %.4g, \"materialize_ms_per_thread\": %.2f, "
             "\"flush_ms_per_thread\": %.2f, \"finalize_ms\": %.2f, "
             "\"rehash_hbm_ms\": %.2f, \"rehash_from_host_ms\": %.2f, \"resized\": %s, \"same_words\": %s}\n",
             n_cb, T, static_cast<unsigned long long>(flush), async ? "true" : "false", warm ? "warm" : "cold", workers,
             create.DeviceKeys(0).segments().size(),
             n_cb / sink_s, mat_s / T * 1e3, fl_s / T * 1e3, fin_s * 1e3, hbm_s * 1e3, host_s * 1e3,
             create.Resized(0) ? "true" : "false", bfh->ExportWords() == words ? "true" : "false");
      fflush(stdout);
    }
  }
  return 0;
}

// Where CREATE_BF's sink time goes: per sink thread, when its Sink loop ends and when its Combine returns
// (ms from the start), for an under-estimated filter (tiny: atomic inserts, resized at Finalize) and a
// right-sized one (128 MiB: partitioned inserts), flushes synchronous and asynchronous.
int create_split(int dev) {
  const size_t n_cb = 100000000;
  std::mt19937_64 rng(43);
  std::vector<int64_t> cb(n_cb);
  for (auto& k : cb) k = static_cast<int64_t>(rng() >> 1);
  std::vector<rpt::DataChunk> cchunks;
  for (size_t lo = 0; lo < cb.size(); lo += 2048) {
    rpt::DataChunk c;
    c.count = std::min<size_t>(2048, cb.size() - lo);
    rpt::Vector x;
    x.key_type = rpt::KeyType::I64;
    x.data = cb.data() + lo;
    c.data.push_back(x);
    cchunks.push_back(c);
  }
  for (int rep = 0; rep < 2; rep++)
  for (uint64_t est : {uint64_t(1000), uint64_t(n_cb)})
  for (bool async : {false, true}) {
    rpt::CreateBF create(dev, est, {0});
    const int T = 8;
    std::vector<std::unique_ptr<rpt::CreateBF::LocalState>> locals;
    for (int t = 0; t < T; t++) {
      locals.push_back(create.MakeLocalState());
      locals.back()->async_flush = async;
      locals.back()->ctx.flatten_threads = 2;
    }
    const int log_blocks0 = create.GetBloomFilter(0)->LogNumBlocks();
    std::vector<double> sink_end(T), comb_end(T);
    auto t0 = clk::now();
    std::vector<std::thread> th;
    for (int t = 0; t < T; t++)
      th.emplace_back([&, t] {
        for (size_t k = t; k < cchunks.size(); k += T) create.Sink(*locals[t], cchunks[k]);
        sink_end[t] = since(t0) * 1e3;
        create.Combine(*locals[t]);
        comb_end[t] = since(t0) * 1e3;
      });
    for (auto& x : th) x.join();
    const double total_ms = since(t0) * 1e3;
    t0 = clk::now();
    create.Finalize();
    const double fin_ms = since(t0) * 1e3;
    // Finalize's parts: the rehash from HBM with a warm context, and the reinitialization alone
    double rehash_warm_ms = 0, reinit_ms = 0;
    {
      rpt::DeviceContext c2(dev);
      auto bfh = create.GetBloomFilter(0);
      bfh->ReinitializeAndRehash(c2, n_cb, create.DeviceKeys(0));  // warm-up
      auto t1 = clk::now();
      bfh->ReinitializeAndRehash(c2, n_cb, create.DeviceKeys(0));
      rehash_warm_ms = since(t1) * 1e3;
      rpt::DeviceKeyColumn none(dev);
      t1 = clk::now();
      bfh->ReinitializeAndRehash(c2, n_cb, none);
      reinit_ms = since(t1) * 1e3;
      bfh->ReinitializeAndRehash(c2, n_cb, create.DeviceKeys(0));
    }
    // a short-lived context's own costs: create, two large device buffers (the rehash's sizes), destroy
    double ctor_ms, alloc_ms, dtor_ms;
    {
      auto t1 = clk::now();
      auto c3 = std::make_unique<rpt::DeviceContext>(dev);
      ctor_ms = since(t1) * 1e3;
      t1 = clk::now();
      (void)c3->dev(6, size_t(1) << 30);
      (void)c3->dev(7, n_cb * 8);
      alloc_ms = since(t1) * 1e3;
      t1 = clk::now();
      c3.reset();
      dtor_ms = since(t1) * 1e3;
    }
    double mat = 0, fl = 0, se = 0, ce = 0, se_max = 0;
    for (int t = 0; t < T; t++) {
      mat += locals[t]->materialize_s * 1e3 / T;
      fl += locals[t]->flush_s * 1e3 / T;
      se += sink_end[t] / T;
      ce += comb_end[t] / T;
      se_max = std::max(se_max, sink_end[t]);
    }
    printf("{\"op\": \"CreateBF split\", \"rep\": %d, \"rows\": %zu, \"estimated_cardinality\": %llu, \"async_flush\": %s, "
           "\"resized\": %s, \"log_blocks_during_sink\": %d, \"sink_combine_rows_per_s\": %.4g, \"total_ms\": %.2f, "
           "\"sink_loop_end_ms_avg\": %.2f, \"sink_loop_end_ms_max\": %.2f, \"combine_end_ms_avg\": %.2f, "
           "\"materialize_ms_per_thread\": %.2f, \"flush_ms_per_thread\": %.2f, \"finalize_ms\": %.2f, "
           "\"segments\": %zu, \"rehash_warm_ctx_ms\": %.2f, \"reinit_only_ms\": %.2f, \"ctx_create_ms\": %.2f, "
           "\"ctx_alloc_1g_800m_ms\": %.2f, \"ctx_destroy_ms\": %.2f}\n",
           rep, n_cb, static_cast<unsigned long long>(est), async ? "true" : "false", create.Resized(0) ? "true" : "false",
           log_blocks0,
           n_cb / (total_ms * 1e-3), total_ms, se, se_max, ce, mat, fl, fin_ms, create.DeviceKeys(0).segments().size(),
           rehash_warm_ms, reinit_ms, ctor_ms, alloc_ms, dtor_ms);
    fflush(stdout);
  }
  return 0;
}

}  // namespace

int main(int argc, char** argv) {
  const int dev = 0;
  // --host-path: only the host -> device path section above (int64 / int32 / dictionary keys)
  if (argc > 1 && std::strcmp(argv[1], "--host-path") == 0) return host_path(dev, false);
  // --host-path-trace: int64 / int32 FLAT through the pipeline only (8 worker threads, 4 Mi-row stages), the
  // calls 20 ms apart: the run to take under rocprofv3 --memory-copy-trace (copy-engine busy time per call)
  if (argc > 1 && std::strcmp(argv[1], "--host-path-trace") == 0) return host_path(dev, true);
  // --chain: UseBF::ExecuteBatch with 1..3 filters, pipelined chain vs filter by filter
  if (argc > 1 && std::strcmp(argv[1], "--chain") == 0) return host_chain(dev, false);
  if (argc > 1 && std::strcmp(argv[1], "--chain-ids") == 0) return host_chain(dev, true);
  // --narrow: narrow BIGINT keys on / off
  if (argc > 1 && std::strcmp(argv[1], "--narrow") == 0) return host_narrow(dev);
  // --bits: result bits back vs sels back at pass fractions 0.1 / 0.5 / 0.9
  if (argc > 1 && std::strcmp(argv[1], "--bits") == 0) return host_bits(dev);
  // --batch-sizes: mid-size batches, default stages vs quarter-batch stages
  if (argc > 1 && std::strcmp(argv[1], "--batch-sizes") == 0) return host_batch_sizes(dev);
  // --create: only the CREATE_BF section
  if (argc > 1 && std::strcmp(argv[1], "--create") == 0) return create_bf(dev);
  // --create-split: CREATE_BF sink loop vs Combine wait per thread, tiny vs right-sized filter
  if (argc > 1 && std::strcmp(argv[1], "--create-split") == 0) return create_split(dev);
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
  return create_bf(dev);
}
