// rpt_gpu.hip — the C-ABI of librpt_gpu.so (include/rpt_gpu.h) and its host runtime; the gfx950
// kernels live in kernels/*.hpp, included below into this one translation unit.
//
// Hot path: PTBloomFilter::Insert / LookupSel (reference src/bloom_filter.cpp:60-78),
// called per DataChunk by PhysicalCreateBF::Sink (physical_create_bf.cpp:221-227) and
// PhysicalUseBF::ExecuteInternal (physical_use_bf.cpp:163). Re-designed for MI355X:
//
//   probe   : phase 1 = hash + filter test -> result bit vector (Arrow Find layout) + one survivor
//             count per 512-row segment, by one of four strategies (rpt_probe_strategy):
//               GATHER       probe_direct.hpp  one 8-B gather per key
//               LDS          probe_direct.hpp  filters <= 64 KiB staged whole in LDS
//               PARTITIONED  partitioned.hpp   rows routed by 128 KiB filter slice; slices in LDS
//               BUCKETED     bucketed.hpp      two levels for filters of 32 MiB..16 GiB
//             phase 2 = two-level scan + expansion into an ascending uint32 sel (compaction.hpp).
//   insert  : atomic OR per key (misc.hpp), or the partitioned / bucketed routing with the slices
//             ORed in LDS; the build's key min/max is folded in on the way.
//   merge   : OR of partial filters / peer slices;  fold;  popcount (misc.hpp).
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>  // ncclConfig_t / NCCL_CONFIG_INITIALIZER only: librccl itself is dlopened, never linked

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <list>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <type_traits>
#include <vector>

#include "rpt_bloom_device.hpp"
#include "rpt_gpu.h"
#include "rpt_gpu_synth.h"
#include "rpt_gpu_testing.h"  // the RCCL entry-point table type; its setter exists in the test build only

#include "kernels/common.hpp"
#include "kernels/probe_direct.hpp"
#include "kernels/partitioned.hpp"
#include "kernels/bucketed.hpp"
#include "kernels/compaction.hpp"
#include "kernels/misc.hpp"

// Host-side tuning macros (the kernels' own are in kernels/*.hpp).
#ifndef RPT_FUSED_SEL
#define RPT_FUSED_SEL 1  // rpt_bf_probe, PARTITIONED: the unpermute writes the selection vector itself
#endif
#ifndef RPT_L1_FIXED_PCT
// Fixed chunks per list, in % of an even split's (+ 1). Measured (C5 probe ms, same box): 0 -> 8.70-8.75,
// 110 / 125 -> 8.82-8.85: fixed ids spare the scatter its extent atomics and waits (3.15 -> 3.06 ms), but
// the larger workspace (+6 GB at 1e9 rows: the overflow pool stays sized for the worst case) costs the
// slice probe, partition and unpermute more (slice probe 2.32 -> 2.48 ms).
#define RPT_L1_FIXED_PCT 0
#endif

#ifndef RPT_LOOKBACK_TAIL
#define RPT_LOOKBACK_TAIL 0  // 1: the direct strategies' sel tail in one look-back launch (measured slower, DESIGN §5 rejected list)
#endif
#ifndef RPT_LDS_HYBRID_MAX_LOG
#define RPT_LDS_HYBRID_MAX_LOG 17  // the LDS strategy up to 2^this blocks; above 2^14 the first 128 KiB in LDS, the rest
                                   // gathered from L2 (probe_direct.hpp). ms per 1e9 keys against AUTO's previous pick
                                   // (partitioned) with 2-segment int64 groups: 256 KiB int64 2.77 vs 3.81, int32 2.27 vs
                                   // 3.43; 512 KiB int64 3.64 vs 3.81, int32 3.23 vs 3.43 (gather: 4.66 / 4.27); 1 MiB
                                   // slower than partitioned but faster than the gather from 4 Mi rows (1 MiB,
                                   // 16 Mi rows: 107 vs 112 us int64, 99 vs 106 us int32; profiles/r06/ab_hybrid2.txt,
                                   // ab_hybrid_1m.txt, first pass ab_hybrid.txt)
#endif
#ifndef RPT_SUMSCAN_TAIL
#define RPT_SUMSCAN_TAIL 0  // 1: the direct strategies' group sums and their scan in one launch (measured: no gain)
#endif

// The product build runs the tuning macros at the defaults the GPU suite tests. Other values exist for
// A/B timing only (tools/build_variants.sh builds them under other names, without RPT_PRODUCT_BUILD);
// several were never run through the parity suite (tuning macros).
#if defined(RPT_PRODUCT_BUILD)
static_assert(RPT_SLICE_LOG == 14 && RPT_RUN_ALIGN == 8 && RPT_BUCKET_SLICE_LOG == 8 && RPT_L1_TILE_ROWS == 16384 &&
                  RPT_L1_FIXED_PCT == 0 && RPT_BUCKET_UNPERMUTE_THREADS == 256 && RPT_SLICE_UNROLL == 4 &&
                  RPT_PARTITION_MIN_WAVES == 8 && RPT_PROBE_PREFETCH == 2 && RPT_SEL_BALLOT_MIN == 192 &&
                  RPT_COMPACT_BALLOT_MIN == 384 && RPT_COMPACT_STAGE == 3072 && RPT_LDS_I64_GROUP == 1 &&
                  RPT_PROBE_RING == 2 && RPT_LOOKBACK_TAIL == 0 && RPT_COMPACT_V16 == 0 && RPT_SUMSCAN_TAIL == 0 &&
                  RPT_PROBE_BUFSTORE == 0 && RPT_PROBE_SCHED_BARRIER == 0 && RPT_LDS_HYBRID_MAX_LOG == 17 &&
                  RPT_HYBRID_I64_GROUP == 2,
              "product build: tuning macros must keep their tested defaults (use tools/build_variants.sh)");
static_assert(RPT_FUSED_SEL == 1 && RPT_NT_KEY_LOADS == 1 && RPT_NT_PART_STORES == 1 && RPT_NT_PROBE_LOADS == 1 &&
                  RPT_NT_REC_LOADS == 0 && RPT_NT_SLICE_LOADS == 1 && RPT_PARK_LANE_MAJOR == 1 && RPT_SLICE_XCD_MAP == 1 &&
                  RPT_PARTITION_SMALL_P == 1 && RPT_VALU_INTERLEAVE == 1 && RPT_SEL_BALLOT_EXPAND == 1 &&
                  RPT_DPP_MINMAX == 1 && RPT_DPP_SCAN == 1 && RPT_PART_NOPARK == 1 && RPT_SCATTER_POS_PACK == 2 &&
                  RPT_MM_TOURNAMENT == 1,
              "product build: tuning switches must keep their tested defaults (use tools/build_variants.sh)");
#endif

// =================================================================================================
// Host side
// =================================================================================================
struct rpt_bf {
  int device = 0;
  int log_num_blocks = 0;
  uint64_t* words = nullptr;
  uint64_t alloc_words = 0;
  int64_t* stats = nullptr;  // device {min, max} of the inserted I32/I64 keys (min/max dynamic filter)
  uint64_t sized_for_rows = 0;
  std::atomic<int> has_data{0};
  std::atomic<int> finalized{0};
  std::atomic<int> probe_strategy{RPT_PROBE_AUTO};
  std::atomic<int> insert_strategy{RPT_INSERT_AUTO};
  // Device order of the operations that write the words (inserts, clear, merges, copies): each waits
  // for the previous one's event, whatever host thread or stream enqueued it, so concurrent inserts
  // compose (OR) even where the slice insert updates words with plain read-modify-write stores.
  // `pristine`: every word is zero once the last ordered write completes (create / clear /
  // reinitialize, no write since): the next slice insert may then store its slices outright.
  std::mutex order_mu;
  hipEvent_t order_ev = nullptr;
  bool order_pending = false;
  bool pristine = true;
  // Deferred clear: rpt_bf_clear leaves the zeroing of the words to the next operation on them
  // (settle_for_read / zero_pending_locked; an insert that stores every slice whole does it as part of
  // its stores). Written under order_mu; readers test it without the lock first.
  std::atomic<bool> clear_pending{false};
  // A reader that settled the clear recorded zero_ev after its memset: readers on other streams wait on
  // it (no host sync) until it has completed (zero_unsynced then drops).
  hipEvent_t zero_ev = nullptr;
  std::atomic<bool> zero_unsynced{false};
};

namespace {

thread_local std::string t_last_error;
thread_local bool t_merge_stuck = false;  // the last merge on this thread aborted without draining its streams

int fail(int status, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  t_last_error = buf;
  return status;
}

#define RPT_HIP(expr)                                                                              \
  do {                                                                                             \
    hipError_t e_ = (expr);                                                                        \
    if (e_ != hipSuccess) return fail(RPT_ERR_HIP, "%s failed: %s", #expr, hipGetErrorString(e_)); \
  } while (0)

#define RPT_LAUNCHED(name)                                                                          \
  do {                                                                                              \
    hipError_t e_ = hipGetLastError();                                                              \
    if (e_ != hipSuccess) return fail(RPT_ERR_HIP, "launch of %s failed: %s", name, hipGetErrorString(e_)); \
  } while (0)

// Run device work on `device` and restore the caller's current device afterwards.
struct DeviceGuard {
  int prev = -1, target;
  hipError_t err = hipSuccess;
  explicit DeviceGuard(int d) : target(d) {
    err = hipGetDevice(&prev);
    if (err == hipSuccess && prev != d) err = hipSetDevice(d);
  }
  ~DeviceGuard() {
    if (prev >= 0 && prev != target) (void)hipSetDevice(prev);
  }
};

#define RPT_ON_DEVICE(dev)                                                                        \
  DeviceGuard guard_(dev);                                                                        \
  if (guard_.err != hipSuccess)                                                                   \
    return fail(RPT_ERR_HIP, "hipSetDevice(%d) failed: %s", (dev), hipGetErrorString(guard_.err))


// ---- kernel timing (rpt_profiling_*; mirrors rpt_profiling.hpp's counters at kernel granularity) ----
struct ProfRecord {
  const char* name;
  hipEvent_t start, end;
};
struct ProfStat {
  uint64_t launches = 0;
  double total_ms = 0.0;
};
std::atomic<int> g_prof_enabled{0};
std::mutex g_prof_mu;
std::vector<ProfRecord> g_prof_pending;
std::vector<hipEvent_t> g_prof_free;
std::vector<std::pair<std::string, ProfStat>> g_prof_stats;

hipEvent_t prof_event() {
  if (!g_prof_free.empty()) {
    hipEvent_t e = g_prof_free.back();
    g_prof_free.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  if (hipEventCreate(&e) != hipSuccess) return nullptr;
  return e;
}

// Brackets one kernel launch with events on its stream when profiling is enabled.
struct ProfScope {
  const char* name;
  hipStream_t stream;
  hipEvent_t start = nullptr;
  ProfScope(const char* n, hipStream_t s) : name(n), stream(s) {
    if (!g_prof_enabled.load(std::memory_order_relaxed)) return;
    std::lock_guard<std::mutex> lk(g_prof_mu);
    start = prof_event();
    if (start && hipEventRecord(start, stream) != hipSuccess) start = nullptr;
  }
  void end() {
    if (!start) return;
    std::lock_guard<std::mutex> lk(g_prof_mu);
    hipEvent_t e = prof_event();
    if (e && hipEventRecord(e, stream) == hipSuccess) {
      g_prof_pending.push_back({name, start, e});
    } else {
      g_prof_free.push_back(start);
      if (e) g_prof_free.push_back(e);
    }
    start = nullptr;
  }
};

// Profiling name of a kernel template instantiation, spelled as tools/pmc_summary.py short() spells
// rocprofv3's kernel names ("partition_kernel<0,true,false,1,0>"), so bench.py can match the PMC
// counters of exactly the instantiation that ran. Interned once per (instantiation, base name).
template <typename T>
std::string targ_str(T v) {
  if constexpr (std::is_same_v<T, bool>) return v ? "true" : "false";
  else return std::to_string(v);
}
template <auto... A>
const char* inst_name(const char* base) {
  static std::mutex mu;
  static std::list<std::pair<const char*, std::string>> names;  // list: c_str() pointers stay valid
  std::lock_guard<std::mutex> lk(mu);
  for (const auto& e : names)
    if (e.first == base) return e.second.c_str();
  std::string s = base;
  s += '<';
  ((s += targ_str(A), s += ','), ...);
  s.back() = '>';
  names.emplace_back(base, std::move(s));
  return names.back().second.c_str();
}

bool stream_capturing(hipStream_t s) {
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  return hipStreamIsCapturing(s, &cs) == hipSuccess && cs != hipStreamCaptureStatusNone;
}

// Has `ev` (recorded outside any capture) completed, asked while the calling thread's stream is capturing?
// Querying an event is a potentially unsafe call under hipStreamCaptureModeGlobal (torch.cuda.graph's default)
// and would invalidate the caller's capture, so the thread's capture mode is relaxed around the query and
// restored after it.
bool event_done_during_capture(hipEvent_t ev) {
  hipStreamCaptureMode mode = hipStreamCaptureModeRelaxed;
  const bool swapped = hipThreadExchangeStreamCaptureMode(&mode) == hipSuccess;
  const bool done = hipEventQuery(ev) == hipSuccess;
  if (swapped) (void)hipThreadExchangeStreamCaptureMode(&mode);
  return done;
}

// Writes captured into a graph. A graph replays its kernels, not this library's host-side
// bookkeeping, so a captured write must not depend on host state that changes between replays:
// * a deferred clear (clear_pending) would be settled by a memset (or whole-slice stores) recorded in the
//   graph and dropped once, at capture time: every replay would then wipe the bits inserted since the last
//   one. A capture that would have to settle it is refused; rpt_bf_settle() before capturing settles it;
// * rpt_bf_clear itself only flips that flag, which a replay cannot redo: refused inside a capture;
// * the cross-stream write order (order_ev) cannot be waited on from inside the capture, so an earlier
//   write still in flight refuses the capture too (synchronize it first). A captured write takes no part in
//   that order: replays are ordered by the stream the caller launches the graph on;
// * the slice insert's plain-store merges rely on the words being zero (pristine / store-all): inside a
//   capture it merges with atomics, correct whatever the words hold at replay time.
// The C-ABI entry points that write words call this before enqueueing anything.
int refuse_capture_write(rpt_bf* bf, hipStream_t s, const char* what) {
  if (!stream_capturing(s)) return RPT_OK;
  if (bf->clear_pending.load() || bf->zero_unsynced.load())
    return fail(RPT_ERR_INVALID_ARGUMENT,
                "%s of a cleared filter inside stream capture: call rpt_bf_settle() before capturing", what);
  std::lock_guard<std::mutex> lk(bf->order_mu);
  if (bf->order_pending && !event_done_during_capture(bf->order_ev))
    return fail(RPT_ERR_INVALID_ARGUMENT,
                "%s inside stream capture while an earlier write to the filter is in flight: synchronize it (or "
                "call rpt_bf_settle()) before capturing", what);
  return RPT_OK;
}
#define RPT_REFUSE_IN_FLIGHT(order, what)                                                                     \
  do {                                                                                                        \
    if ((order).in_flight)                                                                                    \
      return fail(RPT_ERR_INVALID_ARGUMENT,                                                                   \
                  "%s inside stream capture while an earlier write to the filter is in flight: synchronize " \
                  "it (or call rpt_bf_settle()) before capturing", what);                                      \
  } while (0)
#define RPT_REFUSE_CAPTURE_WRITE(bf, s, what)                  \
  do {                                                         \
    const int st_cap_ = refuse_capture_write(bf, s, what);     \
    if (st_cap_ != RPT_OK) return st_cap_;                     \
  } while (0)

// Scope of one word-writing operation on a filter (see rpt_bf::order_mu): waits on `s` for the previous
// write's completion event, and records this one's when done() is called (after the launches). Inside a
// stream capture (refuse_capture_write has checked the previous write completed) it neither waits nor
// records: the graph's replays are ordered by the caller's stream.
struct WriteOrder {
  rpt_bf* bf;
  hipStream_t s;
  std::unique_lock<std::mutex> lk;
  bool captured;
  // captured, but a write another thread enqueued since refuse_capture_write looked is still in flight:
  // the caller refuses (RPT_REFUSE_IN_FLIGHT) before enqueueing anything
  bool in_flight = false;
  WriteOrder(rpt_bf* b, hipStream_t st) : bf(b), s(st), lk(b->order_mu), captured(stream_capturing(st)) {
    if (!bf->order_pending) return;
    if (!captured) (void)hipStreamWaitEvent(s, bf->order_ev, 0);
    else in_flight = !event_done_during_capture(bf->order_ev);
  }
  // pristine_after: every word is zero once this operation completes
  void done(bool pristine_after) {
    if (captured) {
      bf->order_pending = false;  // the previous write completed (refuse_capture_write); nothing recorded
      bf->pristine = false;       // a replay may run at any later time
      return;
    }
    if (!bf->order_ev && hipEventCreateWithFlags(&bf->order_ev, hipEventDisableTiming) != hipSuccess) bf->order_ev = nullptr;
    bf->order_pending = bf->order_ev != nullptr && hipEventRecord(bf->order_ev, s) == hipSuccess;
    if (!bf->order_pending) (void)hipStreamSynchronize(s);  // no event: order by waiting here
    bf->pristine = pristine_after;
  }
};

// The deferred clear (rpt_bf::clear_pending), settled by a writer inside its WriteOrder scope: zero the
// words on the writer's stream, before its own launches.
hipError_t zero_pending_locked(rpt_bf* bf, hipStream_t s) {
  if (!bf->clear_pending.load()) return hipSuccess;
  const hipError_t e = hipMemsetAsync(bf->words, 0, (1ULL << bf->log_num_blocks) * 8, s);
  if (e == hipSuccess) bf->clear_pending.store(false);
  return e;
}

// ... and by a reader: zero the words as an ordered write on the reader's stream and record zero_ev after
// the memset, so a reader on another stream that finds the clear already settled waits for that event
// instead of overtaking the zeroing. Reading a cleared filter before any insert is rare: the fast path is
// two atomic loads.
// Not inside stream capture: a captured memset would run at every replay of the graph (wiping
// bits inserted between replays), while the flags would drop once, at capture time; and querying or waiting
// on an event recorded outside the capture is illegal there. A capture that reads a filter with a clear
// still pending is refused; rpt_bf_settle() before the capture settles it.
int settle_for_read(const rpt_bf* cbf, hipStream_t s) {
  rpt_bf* bf = const_cast<rpt_bf*>(cbf);
  if (!bf->clear_pending.load() && !bf->zero_unsynced.load()) return RPT_OK;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(s, &cs) == hipSuccess && cs != hipStreamCaptureStatusNone)
    return fail(RPT_ERR_INVALID_ARGUMENT,
                "read of a cleared filter inside stream capture: call rpt_bf_settle() before capturing");
  std::lock_guard<std::mutex> lk(bf->order_mu);
  if (bf->clear_pending.load()) {
    // both events exist before anything is enqueued, so no early return leaves the memset unordered
    if (!bf->zero_ev) RPT_HIP(hipEventCreateWithFlags(&bf->zero_ev, hipEventDisableTiming));
    if (!bf->order_ev) RPT_HIP(hipEventCreateWithFlags(&bf->order_ev, hipEventDisableTiming));
    if (bf->order_pending) RPT_HIP(hipStreamWaitEvent(s, bf->order_ev, 0));
    RPT_HIP(hipMemsetAsync(bf->words, 0, (1ULL << bf->log_num_blocks) * 8, s));
    bf->pristine = true;
    bf->zero_unsynced.store(true);  // before the flag drops: a reader seeing neither may skip both
    bf->clear_pending.store(false);
    if (hipEventRecord(bf->zero_ev, s) != hipSuccess || hipEventRecord(bf->order_ev, s) != hipSuccess) {
      // the memset is enqueued but cannot be ordered by events: order it by waiting for it here
      const hipError_t e = hipStreamSynchronize(s);
      bf->order_pending = false;
      bf->zero_unsynced.store(false);
      if (e != hipSuccess) return fail(RPT_ERR_HIP, "settling a cleared filter: %s", hipGetErrorString(e));
      return RPT_OK;
    }
    bf->order_pending = true;  // later writes are ordered after the zeroing too
    return RPT_OK;
  }
  if (bf->zero_unsynced.load()) {
    if (hipEventQuery(bf->zero_ev) == hipSuccess) bf->zero_unsynced.store(false);
    else RPT_HIP(hipStreamWaitEvent(s, bf->zero_ev, 0));
  }
  return RPT_OK;
}
#define RPT_SETTLE(bf, s)                        \
  do {                                           \
    const int st_settle_ = settle_for_read(bf, s); \
    if (st_settle_ != RPT_OK) return st_settle_;   \
  } while (0)

int num_cus(int device) {
  static std::mutex mu;
  static std::vector<int> cache;
  std::lock_guard<std::mutex> lk(mu);
  if (device >= static_cast<int>(cache.size())) cache.resize(device + 1, 0);
  if (cache[device] == 0) {
    int c = 0;
    if (hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || c <= 0) c = 256;
    cache[device] = c;
  }
  return cache[device];
}

inline hipStream_t as_stream(rpt_stream_t s) { return reinterpret_cast<hipStream_t>(s); }
inline uint64_t ceil_div(uint64_t a, uint64_t b) { return (a + b - 1) / b; }
inline size_t align256(size_t x) { return (x + 255) & ~static_cast<size_t>(255); }

int log_blocks_for_rows(uint64_t n_rows) {
  const uint64_t bits = std::max<uint64_t>(512, n_rows > (UINT64_MAX >> 4) ? (UINT64_MAX >> 1) : n_rows * 8);
  int lg = 0;
  while (lg < 63 && (1ULL << lg) < bits) lg++;
  return lg - 6;
}

struct ProbeWorkspace {
  uint64_t* bits;
  uint32_t* seg_counts;
  uint32_t* group_sums;
  uint32_t* group_offs;
  // partitioned strategy (and level 2 of the bucketed one)
  uint32_t* recs;
  uint16_t* pos;
  uint8_t* passb;
  uint32_t* runs;     // slice-major [slice][tile]
  uint32_t* runs_tm;  // tile-major [tile][slice] (partition kernel output)
  // bucketed strategy, level 1 (bucketed.hpp)
  uint32_t* counts_tm;     // [tile1][bucket] rows of the tile's run
  uint32_t* pre_tm;        // [tile1][bucket] the run's start in its list
  uint64_t* list_base;     // [group][bucket] w-space row of the list's first row
  uint32_t* bucket_tiles;  // [bucket + 1] first level-2 tile of the bucket; [nb] = level-2 tile count
  uint32_t* chunk_map;     // [level-2 tile][4] chunk ids
  uint32_t* lists;         // cursors, pool counters, error flag (L1Lists)
  uint32_t* ext_dir;       // L1Lists::ext_dir
  uint32_t* hash_lo;       // level-2 array (kKeySplit) in 4 Ki-row chunks: hash bits 0..31
  uint8_t* hash_hi;        // and bits 32..39
  uint16_t* pos1;          // row -> position in its level-1 tile's bucket-sorted order
  uint64_t* bits2;         // level-2 result bits (w-space order)
  uint32_t* heavy;         // partitioned: [slice] epoch stamp of a slice skewed probe keys overload (rpt::SkewItems)
  uint64_t* lb_state;      // gather / LDS: [group] look-back states + [n_groups] ticket (compact_lookback_kernel),
                           // or group_sum_scan_kernel's flagged group sums (u32); cleared by the probe kernel
};

uint32_t slice_count(int log_num_blocks) {
  return log_num_blocks <= rpt::kSliceLog ? 1u : (1u << (log_num_blocks - rpt::kSliceLog));
}

// 32 MiB buckets of the bucketed strategy (1 for smaller filters).
uint32_t bucket_count(int log_num_blocks) {
  return 1u << std::max(0, log_num_blocks - rpt::kSliceLog - rpt::kBucketSliceLog);
}

// (slice, split) work items of the slice probe: RPT_SLICE_SPLIT_MULT x one resident round (the grid stays one round
// and walks them)
#ifndef RPT_SLICE_SPLIT_MULT
#define RPT_SLICE_SPLIT_MULT 1
#endif
// Work items of a slice skewed probe keys overload: RPT_SLICE_SKEW_MULT x finer (1: off; rpt::SkewItems)
#ifndef RPT_SLICE_SKEW_MULT
#define RPT_SLICE_SKEW_MULT 32
#endif
std::atomic<uint32_t> g_skew_epoch{0};
int strategy_supported(int strategy, int log_num_blocks) {
  constexpr int kBucketLog = rpt::kSliceLog + rpt::kBucketSliceLog;  // log2 blocks per bucket (22)
  switch (strategy) {
    case RPT_PROBE_GATHER: return 1;
    case RPT_PROBE_LDS: return log_num_blocks <= std::max(rpt::kLdsDirectMaxLog, RPT_LDS_HYBRID_MAX_LOG);
    case RPT_PROBE_PARTITIONED:
      return log_num_blocks >= rpt::kSliceLog && slice_count(log_num_blocks) <= static_cast<uint32_t>(rpt::kMaxSliceCount);
    case RPT_PROBE_BUCKETED:  // 1..512 buckets of 32 MiB (filters of 32 MiB..16 GiB)
      return log_num_blocks >= kBucketLog && log_num_blocks <= rpt::kMaxBucketedLog &&
             bucket_count(log_num_blocks) <= rpt::kMaxBuckets;
    default: return 0;
  }
}

// AUTO, from measured crossovers (tools/strategy_crossover.py, profiles/r01/strategy_crossover.jsonl):
//   <= 128 KiB  LDS: the whole filter in each workgroup's LDS;
//   256-512 KiB LDS, hybrid (r06), for batches of >= 4 Mi rows: the first 128 KiB in LDS, the rest gathered from
//               L2 -- faster than the gather and than the partitioned probe (tools/ab_hybrid.sh,
//               profiles/r06/ab_hybrid2.txt). Below 4 Mi rows its 128 KiB staging per workgroup costs more than it
//               saves: GATHER (1 Mi rows: 37.5 vs 35.7 us, 4 Mi: 43.8 vs 51.6 us, profiles/r06/ab_hybrid_small.txt);
//   1 MiB       LDS, hybrid, for 4 Mi .. 32 Mi rows (over the gather: 1-8 %, profiles/r06/ab_hybrid_1m.txt); the
//               partitioned probe from 32 Mi rows as below (1e9 keys: 3.89 vs 4.22 ms);
//   <= 128 MiB  PARTITIONED for batches of >= 4 Mi rows (>= 32 Mi below 8 MiB filters, where the L2
//               still serves the gather well), else GATHER: routing has ~50 us of fixed cost;
//   <= 16 GiB   BUCKETED for batches of >= max(blocks/8, 32 Mi) rows (it stages the whole filter in
//               LDS once), else GATHER.
// n = ~0 is "a batch of unknown, large size" (rpt_bf_probe_strategy).
constexpr uint64_t kHybridMinRows = 1ULL << 22;
int resolve_strategy(int requested, int log_num_blocks, uint64_t n) {
  if (requested != RPT_PROBE_AUTO) return requested;
  const int L = log_num_blocks;
  if (L <= rpt::kLdsDirectMaxLog) return RPT_PROBE_LDS;
  if (L <= RPT_LDS_HYBRID_MAX_LOG && n >= kHybridMinRows && (L <= 16 || n < (1ULL << 25))) return RPT_PROBE_LDS;
  if (L <= 16 && L <= RPT_LDS_HYBRID_MAX_LOG) return RPT_PROBE_GATHER;  // 256 / 512 KiB below 4 Mi rows
  // measured crossovers (tools/strategy_crossover.py --mid, profiles/r01/strategy_crossover_mid.jsonl):
  // the partitioned probe overtakes the (partly L2-resident) gather from 2^25 rows for 256 KiB..2 MiB
  // filters and from 2^22 rows above
  if (strategy_supported(RPT_PROBE_PARTITIONED, L))
    return n >= (L >= 19 ? (1ULL << 22) : (1ULL << 25)) ? RPT_PROBE_PARTITIONED : RPT_PROBE_GATHER;
  if (strategy_supported(RPT_PROBE_BUCKETED, L))
    return n >= std::max<uint64_t>((1ULL << L) >> 3, 1ULL << 25) ? RPT_PROBE_BUCKETED : RPT_PROBE_GATHER;
  return RPT_PROBE_GATHER;
}

// Geometry of the bucketed level 1 for a batch of n rows (bucketed.hpp): 8 list groups (one per XCD
// share) for large batches, 1 below RPT_L1_GROUPS_MIN_ROWS (8 lists per bucket would pad too much); K
// fixed chunks per list, then overflow extents from per-group pool shards; the level-2 tile bound.
constexpr uint64_t kL1GroupsMinRows = 1ULL << 27;
struct L1Geom {
  uint64_t t1;           // level-1 tiles
  uint32_t nb, groups;   // buckets, list groups
  uint64_t n_lists;      // groups * nb
  uint64_t k_fixed;      // chunks with fixed ids per list
  uint64_t n_ext;        // overflow extents per list (bound)
  uint64_t shard_ext;    // extents per pool shard (bound)
  uint64_t pool_chunks;  // chunk ids: n_lists * k_fixed fixed ones, then groups * shard_ext extents
  uint64_t t2max;        // level-2 tiles (bound)
};
L1Geom l1_geom(uint64_t n, int log_num_blocks) {
  static const uint64_t min_rows = [] {
#if defined(RPT_PRODUCT_BUILD)
    return kL1GroupsMinRows;  // the product runs the geometry the GPU suite tests
#else
    const char* e = std::getenv("RPT_L1_GROUPS_MIN_ROWS");  // tuning variants only (tools/build_variants.sh)
    return e ? static_cast<uint64_t>(std::strtoull(e, nullptr, 10)) : kL1GroupsMinRows;
#endif
  }();
  L1Geom g;
  g.t1 = ceil_div(n, rpt::kL1TileRows);
  g.nb = bucket_count(log_num_blocks);
  g.groups = n >= min_rows ? rpt::kL1Groups : 1u;
  g.n_lists = static_cast<uint64_t>(g.groups) * g.nb;
  const uint64_t even = ceil_div(ceil_div(n, g.n_lists), rpt::kChunkRows);  // chunks per list of an even split
  g.k_fixed = ceil_div(even * RPT_L1_FIXED_PCT, 100) + 1;
  const uint64_t group_chunks = ceil_div(g.t1, g.groups) * (rpt::kL1TileRows / rpt::kChunkRows);  // rows of one group
  const uint64_t cmax = group_chunks + 1;  // chunks of one list
  g.n_ext = cmax > g.k_fixed ? ceil_div(cmax - g.k_fixed, rpt::kExtentChunks) : 0;
  g.shard_ext = ceil_div(group_chunks + g.nb, rpt::kExtentChunks) + g.nb;  // + one part-used extent per list
  g.pool_chunks = g.n_lists * g.k_fixed + g.groups * g.shard_ext * rpt::kExtentChunks;
  g.t2max = ceil_div(ceil_div(n, rpt::kChunkRows) + g.n_lists, rpt::kChunksPerTile) + g.nb;  // + one part tile per bucket
  return g;
}
uint64_t level2_tiles_max(uint64_t n, int log_num_blocks) { return l1_geom(n, log_num_blocks).t2max; }

// rpt::tile_mult, with its slice threshold overridable in tuning variants (RPT_TILE_MULT_SLICES: tiles
// double above that many slices).
uint32_t tile_mult_of(uint32_t n_slices) {
  static const uint32_t above = [] {
#if defined(RPT_PRODUCT_BUILD)
    return 0u;  // the product keeps rpt::tile_mult
#else
    const char* e = std::getenv("RPT_TILE_MULT_SLICES");  // tuning variants only
    return e ? static_cast<uint32_t>(std::strtoul(e, nullptr, 10)) : 0u;
#endif
  }();
  return above ? (n_slices > above ? 2u : 1u) : rpt::tile_mult(n_slices);
}

// Layout (all 256-aligned): bits | seg_counts | group_sums | group_offs, then for the partitioned
// strategy recs | pos | passb | runs | runs_tm (whole 16 Ki-row tiles), and for the bucketed one the
// same level-2 arrays over level2_tiles_max tiles of 256 slices plus the level-1 arrays.
// RPT_LOOKBACK_TAIL = 1 runs the direct strategies' selection-vector tail as one look-back launch
// (compact_lookback_kernel) instead of group sums + their scan + the compaction; measured slower, so off.
bool lookback_tail(int strategy) {
  return RPT_LOOKBACK_TAIL && (strategy == RPT_PROBE_GATHER || strategy == RPT_PROBE_LDS);
}
// RPT_SUMSCAN_TAIL: the direct strategies' group sums + scan as one launch whose highest-numbered workgroup scans
// (flagged group sums the probe kernel clears), then the compaction: two dependent launches after the probe, not three.
bool sumscan_tail(int strategy) {
  return RPT_SUMSCAN_TAIL && !lookback_tail(strategy) && (strategy == RPT_PROBE_GATHER || strategy == RPT_PROBE_LDS);
}

size_t workspace_layout(uint64_t n, int log_num_blocks, int strategy, void* base, ProbeWorkspace* ws) {
  const uint64_t n_segs = ceil_div(n, rpt::kSegRows);
  const uint64_t n_groups = ceil_div(n_segs, rpt::kGroupSegs);
  const uint64_t T = rpt::kTileRows;
  constexpr int kParts = 22;
  size_t sz[kParts] = {align256(n_segs * rpt::kWordsPerSeg * 8), align256(n_groups * rpt::kGroupSegs * 4),
                       align256(n_groups * 4), align256(n_groups * 4)};
  const bool part = strategy == RPT_PROBE_PARTITIONED, buck = strategy == RPT_PROBE_BUCKETED;
  if (lookback_tail(strategy)) sz[21] = align256((n_groups + 1) * 8);
  if (sumscan_tail(strategy)) sz[21] = align256(n_groups * 4);
  if (part || buck) {
    const uint32_t slices = part ? slice_count(log_num_blocks) : rpt::kBucketSlices;
    const uint32_t tm = part ? tile_mult_of(slices) : 1u;
    const uint64_t tiles = part ? ceil_div(n, T * tm) : level2_tiles_max(n, log_num_blocks);
    const uint64_t cap = rpt::tile_cap_for(slices, tm);
    sz[4] = align256(tiles * cap * 4);
    sz[5] = align256(tiles * T * tm * 2);
    sz[6] = align256(tiles * cap / 8);
    sz[7] = align256(static_cast<uint64_t>(slices) * tiles * 4);
    sz[8] = sz[7];
    if (part) sz[20] = align256(static_cast<uint64_t>(slices) * 4);
  }
  if (buck) {
    const L1Geom g = l1_geom(n, log_num_blocks);
    sz[9] = sz[10] = align256(g.t1 * g.nb * 4);
    sz[11] = align256(static_cast<uint64_t>(g.groups) * g.nb * 8);
    sz[12] = align256((g.nb + 1) * 4);
    sz[13] = align256(g.t2max * rpt::kChunksPerTile * 4);
    sz[14] = align256((g.n_lists + g.groups + 1) * 4);
    sz[15] = align256(g.n_lists * g.n_ext * 4);
    sz[16] = align256(g.pool_chunks * rpt::kChunkRows * 4);
    sz[17] = align256(g.t1 * rpt::kL1TileRows * 2);
    sz[18] = align256(g.t2max * T / 8);
    sz[19] = align256(g.pool_chunks * rpt::kChunkRows);
  }
  size_t off[kParts], total = 0;
  for (int i = 0; i < kParts; i++) {
    off[i] = total;
    total += sz[i];
  }
  if (ws) {
    char* p = static_cast<char*>(base);
    auto at = [&](int i) -> void* { return sz[i] ? p + off[i] : nullptr; };
    ws->bits = static_cast<uint64_t*>(at(0));
    ws->seg_counts = static_cast<uint32_t*>(at(1));
    ws->group_sums = static_cast<uint32_t*>(at(2));
    ws->group_offs = static_cast<uint32_t*>(at(3));
    ws->recs = static_cast<uint32_t*>(at(4));
    ws->pos = static_cast<uint16_t*>(at(5));
    ws->passb = static_cast<uint8_t*>(at(6));
    ws->runs = static_cast<uint32_t*>(at(7));
    ws->runs_tm = static_cast<uint32_t*>(at(8));
    ws->counts_tm = static_cast<uint32_t*>(at(9));
    ws->pre_tm = static_cast<uint32_t*>(at(10));
    ws->list_base = static_cast<uint64_t*>(at(11));
    ws->bucket_tiles = static_cast<uint32_t*>(at(12));
    ws->chunk_map = static_cast<uint32_t*>(at(13));
    ws->lists = static_cast<uint32_t*>(at(14));
    ws->ext_dir = static_cast<uint32_t*>(at(15));
    ws->hash_lo = static_cast<uint32_t*>(at(16));
    ws->pos1 = static_cast<uint16_t*>(at(17));
    ws->bits2 = static_cast<uint64_t*>(at(18));
    ws->hash_hi = static_cast<uint8_t*>(at(19));
    ws->heavy = static_cast<uint32_t*>(at(20));
    ws->lb_state = static_cast<uint64_t*>(at(21));
  }
  return total;
}

// Build workspace: records | runs (slice-major) | runs (tile-major) (partitioned, or level 2 of the
// bucketed insert), then the bucketed level-1 arrays.
struct InsertWorkspace {
  uint32_t* recs;
  uint32_t* runs;
  uint32_t* runs_tm;
  uint32_t* bucket_tiles;
  uint32_t* chunk_map;
  uint32_t* lists;
  uint32_t* ext_dir;
  uint32_t* hash_lo;
  uint8_t* hash_hi;
  uint64_t* list_base;
};

// rpt_bf_insert_ws runs a bucketed insert of more rows in batches of this many (level-1 list positions are
// 32-bit); the test build batches from 2^20 rows so that the batching runs at test sizes
#ifdef RPT_TESTING_HOOKS
constexpr uint64_t kBucketedInsertBatch = 1ULL << 20;
#else
constexpr uint64_t kBucketedInsertBatch = 1ULL << 31;
#endif

size_t insert_workspace_layout(uint64_t n, int log_num_blocks, int strategy, void* base, InsertWorkspace* ws) {
  const bool buck = strategy == RPT_INSERT_BUCKETED;
  if (strategy != RPT_INSERT_PARTITIONED && !buck) return 0;
  if (buck) n = std::min(n, kBucketedInsertBatch);
  const uint64_t T = rpt::kTileRows;
  const uint32_t slices = buck ? rpt::kBucketSlices : slice_count(log_num_blocks);
  const uint32_t tm = buck ? 1u : tile_mult_of(slices);
  const uint64_t tiles = buck ? level2_tiles_max(n, log_num_blocks) : ceil_div(n, T * tm);
  constexpr int kParts = 10;
  size_t sz[kParts] = {align256(tiles * rpt::tile_cap_for(slices, tm) * 4), align256(static_cast<uint64_t>(slices) * tiles * 4),
                       align256(static_cast<uint64_t>(slices) * tiles * 4)};
  if (buck) {
    const L1Geom g = l1_geom(n, log_num_blocks);
    sz[3] = align256((g.nb + 1) * 4);
    sz[4] = align256(g.t2max * rpt::kChunksPerTile * 4);
    sz[5] = align256((g.n_lists + g.groups + 1) * 4);
    sz[6] = align256(g.n_lists * g.n_ext * 4);
    sz[7] = align256(g.pool_chunks * rpt::kChunkRows * 4);
    sz[8] = align256(g.pool_chunks * rpt::kChunkRows);
    sz[9] = align256(static_cast<uint64_t>(g.groups) * g.nb * 8);
  }
  size_t off[kParts], total = 0;
  for (int i = 0; i < kParts; i++) {
    off[i] = total;
    total += sz[i];
  }
  if (ws) {
    char* p = static_cast<char*>(base);
    auto at = [&](int i) -> void* { return sz[i] ? p + off[i] : nullptr; };
    ws->recs = static_cast<uint32_t*>(at(0));
    ws->runs = static_cast<uint32_t*>(at(1));
    ws->runs_tm = static_cast<uint32_t*>(at(2));
    ws->bucket_tiles = static_cast<uint32_t*>(at(3));
    ws->chunk_map = static_cast<uint32_t*>(at(4));
    ws->lists = static_cast<uint32_t*>(at(5));
    ws->ext_dir = static_cast<uint32_t*>(at(6));
    ws->hash_lo = static_cast<uint32_t*>(at(7));
    ws->hash_hi = static_cast<uint8_t*>(at(8));
    ws->list_base = static_cast<uint64_t*>(at(9));
  }
  return total;
}

// AUTO insert, from the measured crossovers (profiles/r03/strategy_crossover_insert.jsonl): memory-side
// atomics cost ~40 ps/key at any filter size; the partitioned insert ~4-9 ps/key plus ~40-80 us, so it
// overtakes between 1 and 2 Mi rows (2-4 Mi above 128 slices, where it partitions 32 Ki-row tiles: at 2 Mi
// rows into 128 MiB, 0.103 vs 0.088 ms atomic); the bucketed insert ~9 ps/key plus a pass over the whole
// filter (~2 ms per 8 GiB), so from ~blocks/16 rows.
uint64_t partitioned_insert_min_rows(int L) { return L > rpt::kSliceLog + 7 ? (1ULL << 22) : (1ULL << 21); }
int resolve_insert_strategy(int requested, int log_num_blocks, uint64_t n) {
  if (requested != RPT_INSERT_AUTO) return requested;
  const int L = log_num_blocks;
  if (strategy_supported(RPT_PROBE_PARTITIONED, L))
    return n >= partitioned_insert_min_rows(L) ? RPT_INSERT_PARTITIONED : RPT_INSERT_ATOMIC;
  if (strategy_supported(RPT_PROBE_BUCKETED, L) && n >= std::max<uint64_t>((1ULL << L) >> 4, 1ULL << 23))
    return RPT_INSERT_BUCKETED;
  return RPT_INSERT_ATOMIC;
}

int check_col(const rpt_key_column* col) {
  if (!col) return fail(RPT_ERR_INVALID_ARGUMENT, "null key column");
  if (col->key_type < RPT_KEY_I64 || col->key_type > RPT_KEY_HASH)
    return fail(RPT_ERR_INVALID_ARGUMENT, "bad key_type %d", col->key_type);
  if (!col->keys) return fail(RPT_ERR_INVALID_ARGUMENT, "null keys pointer");
  return RPT_OK;
}

bool dense_ok(const rpt_key_column* col, const uint32_t* row_sel) {
  return row_sel == nullptr && col->key_sel == nullptr && (reinterpret_cast<uintptr_t>(col->keys) & 15) == 0;
}

unsigned persistent_grid(int device, uint64_t n_segs) {
  const uint64_t want = ceil_div(n_segs, rpt::kWavesPerBlock);
  const uint64_t cap = static_cast<uint64_t>(num_cus(device)) * rpt::kBlocksPerCU;
  return static_cast<unsigned>(std::max<uint64_t>(1, std::min(want, cap)));
}

template <int K, bool D>
void launch_probe_bits_t(unsigned grid, hipStream_t s, const rpt_bf* bf, const rpt::KeyArgs& a, uint64_t n,
                         uint64_t n_segs, uint64_t* bits, uint32_t* counts, uint64_t* zero = nullptr,
                         uint32_t n_zero = 0) {
  ProfScope prof(inst_name<K, D, false, rpt::kBlockThreads>("probe_bits_kernel"), s);
  hipLaunchKernelGGL((rpt::probe_bits_kernel<K, D, false>), dim3(grid), dim3(rpt::kBlockThreads), 0, s, bf->words,
                     (1ULL << bf->log_num_blocks) - 1, a, n, n_segs, bits, counts, zero, n_zero);
  prof.end();
}

template <int K, bool D>
void launch_probe_small_t(hipStream_t s, const rpt_bf* bf, const rpt::KeyArgs& a, uint64_t n, const uint32_t* row_sel,
                          uint32_t* out_sel, uint64_t* out_count) {
  ProfScope prof(inst_name<K, D>("probe_small_kernel"), s);
  hipLaunchKernelGGL((rpt::probe_small_kernel<K, D>), dim3(1), dim3(rpt::kSmallThreads), 0, s, bf->words,
                     (1ULL << bf->log_num_blocks) - 1, a, n, row_sel, out_sel, out_count);
  prof.end();
}

// Whole filter in LDS (dynamic LDS = filter bytes), 1024-thread workgroups (16 waves): as many per CU as
// LDS allows. Measured against 256-thread workgroups: 16 KiB 1.79 -> 1.67 ms, 64 KiB 2.07 -> 1.73 ms per
// 1e9 int64 keys (int32: 1.71 -> 1.26 ms); a 128 KiB filter fits one workgroup per CU either way.
void allow_dynamic_lds(const void* fn);
template <int K, bool D>
void launch_probe_bits_lds_t(unsigned grid, hipStream_t s, const rpt_bf* bf, const rpt::KeyArgs& a, uint64_t n,
                             uint64_t n_segs, uint64_t* bits, uint32_t* counts, uint64_t* zero, uint32_t n_zero) {
  if (bf->log_num_blocks > rpt::kLdsDirectMaxLog) {  // hybrid: the first 128 KiB in LDS, the rest from L2
    const size_t lds = 8ULL << rpt::kLdsDirectMaxLog;
    static std::once_flag once_h;
    std::call_once(once_h, [] {
      allow_dynamic_lds(reinterpret_cast<const void*>(&rpt::probe_bits_hybrid_kernel<K, D>));
    });
    ProfScope prof(inst_name<K, D>("probe_bits_hybrid_kernel"), s);
    hipLaunchKernelGGL((rpt::probe_bits_hybrid_kernel<K, D>), dim3(grid),
                       dim3(rpt::kLdsProbeThreads), lds, s, bf->words, (1ULL << bf->log_num_blocks) - 1, a, n, n_segs,
                       bits, counts, zero, n_zero);
    prof.end();
    return;
  }
  const size_t lds = 8ULL << bf->log_num_blocks;
  static std::once_flag once;  // > 64 KiB of dynamic LDS must be opted into
  std::call_once(once, [] { allow_dynamic_lds(reinterpret_cast<const void*>(&rpt::probe_bits_kernel<K, D, true, rpt::kLdsProbeThreads>)); });
  ProfScope prof(inst_name<K, D, true, rpt::kLdsProbeThreads>("probe_bits_kernel"), s);
  hipLaunchKernelGGL((rpt::probe_bits_kernel<K, D, true, rpt::kLdsProbeThreads>), dim3(grid), dim3(rpt::kLdsProbeThreads), lds,
                     s, bf->words, (1ULL << bf->log_num_blocks) - 1, a, n, n_segs, bits, counts, zero, n_zero);
  prof.end();
}

// Let `fn` use all of the CU's 160 KiB of LDS: dynamic allowance = 160 KiB - its static LDS.
void allow_dynamic_lds(const void* fn) {
  hipFuncAttributes at{};
  size_t stat = 0;
  if (hipFuncGetAttributes(&at, fn) == hipSuccess) stat = at.sharedSizeBytes;
  (void)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>((160u << 10) - stat));
  (void)hipGetLastError();
}

template <int K, bool D, bool MM, int TM, int SP = 0>
void launch_partition_tm(unsigned grid, hipStream_t s, const rpt::KeyArgs& a, uint64_t n, uint32_t slice_mask,
                         uint64_t n_tiles, uint32_t* recs, uint16_t* pos, uint32_t* runs, int64_t* stats,
                         const uint32_t* dev_n_tiles, const uint32_t* chunk_map) {
  if constexpr (TM == 1 && SP == 0) {
    if (RPT_PARTITION_SMALL_P && slice_mask + 1 <= 4) {  // few slices: wave-aggregated slice counters
      launch_partition_tm<K, D, MM, 1, 4>(grid, s, a, n, slice_mask, n_tiles, recs, pos, runs, stats, dev_n_tiles, chunk_map);
      return;
    }
  }
  const size_t lds = rpt::partition_lds_bytes(slice_mask + 1, TM);
  static std::once_flag once;  // per instantiation; > 64 KiB of dynamic LDS must be opted into
  std::call_once(once, [] { allow_dynamic_lds(reinterpret_cast<const void*>(&rpt::partition_kernel<K, D, MM, TM, SP>)); });
  ProfScope prof(inst_name<K, D, MM, TM, SP>("partition_kernel"), s);
  hipLaunchKernelGGL((rpt::partition_kernel<K, D, MM, TM, SP>), dim3(grid), dim3(rpt::kTileThreads), lds, s, a, n,
                     slice_mask, n_tiles, recs, pos, runs, stats, dev_n_tiles, chunk_map);
  prof.end();
}

// Tiles of tm * kTileRows rows (rpt::tile_mult; the bucketed level 2 always passes tm = 1).
template <int K, bool D, bool MM>
void launch_partition_mm(unsigned grid, hipStream_t s, const rpt::KeyArgs& a, uint64_t n, uint32_t slice_mask,
                         uint64_t n_tiles, uint32_t* recs, uint16_t* pos, uint32_t* runs, int64_t* stats,
                         const uint32_t* dev_n_tiles, uint32_t tm) {
  if (tm == 2)
    launch_partition_tm<K, D, MM, 2>(grid, s, a, n, slice_mask, n_tiles, recs, pos, runs, stats, dev_n_tiles, nullptr);
  else
    launch_partition_tm<K, D, MM, 1>(grid, s, a, n, slice_mask, n_tiles, recs, pos, runs, stats, dev_n_tiles, nullptr);
}

// stats == nullptr: probe (no min/max); otherwise the build's key min/max is folded into stats.
template <int K, bool D>
void launch_partition_t(unsigned grid, hipStream_t s, const rpt::KeyArgs& a, uint64_t n, uint32_t slice_mask,
                        uint64_t n_tiles, uint32_t* recs, uint16_t* pos, uint32_t* runs, int64_t* stats,
                        const uint32_t* dev_n_tiles, uint32_t tm) {
  if (rpt::KeyTraits<K>::kValues && stats != nullptr)
    launch_partition_mm<K, D, true>(grid, s, a, n, slice_mask, n_tiles, recs, pos, runs, stats, dev_n_tiles, tm);
  else
    launch_partition_mm<K, D, false>(grid, s, a, n, slice_mask, n_tiles, recs, pos, runs, nullptr, dev_n_tiles, tm);
}

// Level 2 of the bucketed strategies: the partition over the level-2 hash array, tile t = chunks
// chunk_map[4t ..] (bucketed.hpp).
void launch_partition_level2(unsigned grid, hipStream_t s, const rpt::KeyArgs& a, uint64_t n, uint64_t n_tiles,
                             uint32_t* recs, uint16_t* pos, uint32_t* runs, const uint32_t* dev_n_tiles,
                             const uint32_t* chunk_map) {
  launch_partition_tm<rpt::kKeySplit, true, false, 1>(grid, s, a, n, rpt::kBucketSlices - 1, n_tiles, recs, pos, runs,
                                                      nullptr, dev_n_tiles, chunk_map);
}

template <int K, bool D>
void launch_insert_t(unsigned grid, hipStream_t s, rpt_bf* bf, const rpt::KeyArgs& a, uint64_t n, uint64_t n_segs) {
  ProfScope prof(inst_name<K, D>("insert_kernel"), s);
  hipLaunchKernelGGL((rpt::insert_kernel<K, D>), dim3(grid), dim3(rpt::kBlockThreads), 0, s, bf->words,
                     (1ULL << bf->log_num_blocks) - 1, a, n, n_segs, bf->stats);
  prof.end();
}

template <int K, bool D>
void launch_bucket_scatter_t(unsigned grid, hipStream_t s, const rpt::KeyArgs& a, uint64_t n, uint32_t bucket_mask,
                             const rpt::L1Lists& lists, uint32_t* hash_lo, uint8_t* hash_hi, uint16_t* pos1,
                             uint32_t* counts_tm, uint32_t* pre_tm, int64_t* stats) {
  const size_t lds = rpt::kL1TileRows * 8;  // the tile's hashes
  if (rpt::KeyTraits<K>::kValues && stats != nullptr) {
    static std::once_flag once;  // > 64 KiB of dynamic LDS must be opted into (160 KiB minus the static part)
    std::call_once(once, [] { allow_dynamic_lds(reinterpret_cast<const void*>(&rpt::bucket_scatter_kernel<K, D, true>)); });
    ProfScope prof(inst_name<K, D, true>("bucket_scatter_kernel"), s);
    hipLaunchKernelGGL((rpt::bucket_scatter_kernel<K, D, true>), dim3(grid), dim3(rpt::kTileThreads), lds, s, a, n,
                       bucket_mask, lists, hash_lo, hash_hi, pos1, counts_tm, pre_tm, stats);
    prof.end();
  } else {
    static std::once_flag once;
    std::call_once(once, [] { allow_dynamic_lds(reinterpret_cast<const void*>(&rpt::bucket_scatter_kernel<K, D, false>)); });
    ProfScope prof(inst_name<K, D, false>("bucket_scatter_kernel"), s);
    hipLaunchKernelGGL((rpt::bucket_scatter_kernel<K, D, false>), dim3(grid), dim3(rpt::kTileThreads), lds, s, a, n,
                       bucket_mask, lists, hash_lo, hash_hi, pos1, counts_tm, pre_tm, static_cast<int64_t*>(nullptr));
    prof.end();
  }
}

#define RPT_DISPATCH_KD(fn, kt, dense, ...)                  \
  do {                                                       \
    switch (kt) {                                            \
      case RPT_KEY_I64:                                      \
        if (dense) fn<rpt::kKeyI64, true>(__VA_ARGS__);      \
        else fn<rpt::kKeyI64, false>(__VA_ARGS__);           \
        break;                                               \
      case RPT_KEY_I32:                                      \
        if (dense) fn<rpt::kKeyI32, true>(__VA_ARGS__);      \
        else fn<rpt::kKeyI32, false>(__VA_ARGS__);           \
        break;                                               \
      default:                                               \
        if (dense) fn<rpt::kKeyHash, true>(__VA_ARGS__);     \
        else fn<rpt::kKeyHash, false>(__VA_ARGS__);          \
        break;                                               \
    }                                                        \
  } while (0)

// [rows][cols] u32 matrix -> [cols][rows] (the run-table transpose kernel).
int transpose_u32(hipStream_t s, const uint32_t* in, uint64_t rows, uint64_t cols, uint32_t* out, uint32_t* heavy = nullptr,
                  uint32_t heavy_run = 0, uint32_t epoch = 0) {
  if (ceil_div(cols, 64) > 65535) return fail(RPT_ERR_INVALID_ARGUMENT, "transpose of %llu columns", (unsigned long long)cols);
  ProfScope prof_t("runs_transpose_kernel", s);
  hipLaunchKernelGGL(rpt::runs_transpose_kernel, dim3(static_cast<unsigned>(ceil_div(rows, 64)), static_cast<unsigned>(ceil_div(cols, 64))),
                     dim3(rpt::kBlockThreads), 0, s, in, static_cast<uint32_t>(cols), rows, out, heavy, heavy_run, epoch);
  prof_t.end();
  RPT_LAUNCHED("runs_transpose_kernel");
  return RPT_OK;
}

// Level 1 of the bucketed strategies (bucketed.hpp): one pass over the keys appends every row's hash to
// its (group, bucket) list of chunks [+ the build's min/max; + the probe's row map and run tables], then
// the lists are laid out as level-2 tiles (chunk_map, bucket_tiles, list_base) and padded.
struct BucketLevel1 {
  uint32_t* lists;      // cursors | pool counters | error flag
  uint32_t* ext_dir;
  uint32_t* chunk_map;
  uint32_t* bucket_tiles;
  uint64_t* list_base;
  uint32_t* hash_lo;
  uint8_t* hash_hi;
  uint16_t* pos1;       // probe only
  uint32_t* counts_tm;  // probe only
  uint32_t* pre_tm;     // probe only
};
// The level-1 error flag (L1Lists::error) inside the lists block.
uint32_t* l1_error_flag(uint32_t* lists, const L1Geom& g) { return lists + g.n_lists + g.groups; }
#ifdef RPT_TESTING_HOOKS
std::atomic<int> g_force_l1_error{0};  // rpt_testing_force_l1_error
#endif
int run_bucket_level1(hipStream_t s, int key_type, const rpt::KeyArgs& a, bool dense, uint64_t n, int L,
                      const BucketLevel1& w, int64_t* stats) {
  const L1Geom g = l1_geom(n, L);
  const uint64_t n_lists = g.n_lists;
  if (g.pool_chunks >= (1ULL << 32) - rpt::kExtentChunks)
    return fail(RPT_ERR_INVALID_ARGUMENT, "bucketed batch of %llu rows too large", static_cast<unsigned long long>(n));
  RPT_HIP(hipMemsetAsync(w.lists, 0, (n_lists + g.groups + 1) * 4, s));
  if (g.n_ext)
    RPT_HIP(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(w.ext_dir), static_cast<int>(rpt::kChunkEmpty),
                              n_lists * g.n_ext, s));
  rpt::L1Lists lists{w.lists, w.lists + n_lists, l1_error_flag(w.lists, g), w.ext_dir,
                     static_cast<uint32_t>(g.k_fixed), static_cast<uint32_t>(g.n_ext),
                     static_cast<uint32_t>(g.shard_ext), g.groups, static_cast<uint32_t>(n_lists)};
#ifdef RPT_TESTING_HOOKS
  if (g_force_l1_error.load()) lists.k_fixed = lists.n_ext = 0;  // every chunk past the bound: the error path
#endif
  RPT_DISPATCH_KD(launch_bucket_scatter_t, key_type, dense, static_cast<unsigned>(g.t1), s, a, n, g.nb - 1, lists, w.hash_lo,
                  w.hash_hi, w.pos1, w.counts_tm, w.pre_tm, stats);
  RPT_LAUNCHED("bucket_scatter_kernel");
  ProfScope prof("bucket_lists_kernel", s);
  hipLaunchKernelGGL(rpt::bucket_lists_kernel, dim3(g.nb), dim3(rpt::kListsThreads), 0, s, lists, g.nb, w.chunk_map,
                     w.list_base, w.bucket_tiles, w.hash_lo, w.hash_hi);
  prof.end();
  RPT_LAUNCHED("bucket_lists_kernel");
  return RPT_OK;
}

int alloc_words(rpt_bf* bf, int log_nb) {
  const uint64_t nw = 1ULL << log_nb;
  void* p = nullptr;
  hipError_t e = hipMalloc(&p, nw * 8);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    return fail(RPT_ERR_OUT_OF_MEMORY, "hipMalloc(%llu bytes) failed: %s", static_cast<unsigned long long>(nw * 8),
                hipGetErrorString(e));
  }
  e = hipMemset(p, 0, nw * 8);
  if (e != hipSuccess) {
    (void)hipFree(p);
    return fail(RPT_ERR_HIP, "hipMemset failed: %s", hipGetErrorString(e));
  }
  bf->words = static_cast<uint64_t*>(p);
  bf->alloc_words = nw;
  bf->log_num_blocks = log_nb;
  return RPT_OK;
}

const int64_t kStatsInit[2] = {INT64_MAX, INT64_MIN};

int alloc_stats(rpt_bf* bf) {
  void* p = nullptr;
  hipError_t e = hipMalloc(&p, sizeof kStatsInit);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    return fail(RPT_ERR_OUT_OF_MEMORY, "hipMalloc(stats) failed: %s", hipGetErrorString(e));
  }
  bf->stats = static_cast<int64_t*>(p);
  e = hipMemcpy(bf->stats, kStatsInit, sizeof kStatsInit, hipMemcpyHostToDevice);
  if (e != hipSuccess) return fail(RPT_ERR_HIP, "stats init failed: %s", hipGetErrorString(e));
  return RPT_OK;
}

// {min, max} reset on the stream (after the caller's earlier work on it)
__global__ void stats_reset_kernel(int64_t* stats) {
  stats[0] = INT64_MAX;
  stats[1] = INT64_MIN;
}
__global__ void stats_merge_kernel(int64_t* dst, const int64_t* src) {
  if (src[0] < dst[0]) dst[0] = src[0];
  if (src[1] > dst[1]) dst[1] = src[1];
}

}  // namespace

namespace {
template <bool COMBINE>
int launch_hash(const rpt_key_column* col, uint64_t n, uint64_t* out_hashes, rpt_stream_t stream) {
  if (!out_hashes) return fail(RPT_ERR_INVALID_ARGUMENT, "null out");
  if (n == 0) return RPT_OK;
  int st = check_col(col);
  if (st != RPT_OK) return st;
  const unsigned grid = static_cast<unsigned>(std::min<uint64_t>(ceil_div(n, rpt::kBlockThreads), 4096));
  const rpt::KeyArgs a{col->keys, col->key_sel, col->validity, nullptr};
  hipStream_t s = as_stream(stream);
  switch (col->key_type) {
    case RPT_KEY_I64: {
      ProfScope prof_(inst_name<rpt::kKeyI64, COMBINE>("hash_kernel"), s);
      hipLaunchKernelGGL((rpt::hash_kernel<rpt::kKeyI64, COMBINE>), dim3(grid), dim3(rpt::kBlockThreads), 0, s, a, n, out_hashes);
      prof_.end();
      break;
    }
    case RPT_KEY_I32: {
      ProfScope prof_(inst_name<rpt::kKeyI32, COMBINE>("hash_kernel"), s);
      hipLaunchKernelGGL((rpt::hash_kernel<rpt::kKeyI32, COMBINE>), dim3(grid), dim3(rpt::kBlockThreads), 0, s, a, n, out_hashes);
      prof_.end();
      break;
    }
    default: {
      ProfScope prof_(inst_name<rpt::kKeyHash, COMBINE>("hash_kernel"), s);
      hipLaunchKernelGGL((rpt::hash_kernel<rpt::kKeyHash, COMBINE>), dim3(grid), dim3(rpt::kBlockThreads), 0, s, a, n, out_hashes);
      prof_.end();
      break;
    }
  }
  RPT_LAUNCHED("hash_kernel");
  return RPT_OK;
}
}  // namespace

extern "C" {

int rpt_abi_version(void) { return RPT_GPU_ABI_VERSION; }

const char* rpt_status_string(int status) {
  switch (status) {
    case RPT_OK: return "ok";
    case RPT_ERR_INVALID_ARGUMENT: return "invalid argument";
    case RPT_ERR_HIP: return "HIP runtime error";
    case RPT_ERR_OUT_OF_MEMORY: return "out of device memory";
    case RPT_ERR_WORKSPACE: return "workspace too small";
    case RPT_ERR_SHAPE_MISMATCH: return "filter shape mismatch";
    case RPT_ERR_COLLECTIVE: return "collective (RCCL) failed";
    default: return "unknown status";
  }
}

const char* rpt_last_error(void) { return t_last_error.c_str(); }

int rpt_bf_log_num_blocks_for_rows(uint64_t n_rows) { return log_blocks_for_rows(n_rows); }

int rpt_bf_needs_resize(uint64_t sized_for_rows, uint64_t actual_rows) {
  if (actual_rows == 0) return 0;
  const uint64_t min_bits = std::max<uint64_t>(512, sized_for_rows * 12);
  uint64_t alloc = 1;
  while (alloc < min_bits) alloc <<= 1;
  return actual_rows * 8 > alloc ? 1 : 0;
}

int rpt_bf_needs_resize_alloc(const rpt_bf* bf, uint64_t actual_rows) {
  if (!bf) return -fail(RPT_ERR_INVALID_ARGUMENT, "null filter");
  if (actual_rows == 0) return 0;
  return actual_rows > (64ULL << bf->log_num_blocks) / 8 ? 1 : 0;
}

size_t rpt_probe_workspace_bytes(uint64_t n_rows, int log_num_blocks) {
  // enough for any strategy the filter may run
  size_t m = 0;
  for (int st : {RPT_PROBE_GATHER, RPT_PROBE_LDS, RPT_PROBE_PARTITIONED, RPT_PROBE_BUCKETED})
    if (strategy_supported(st, log_num_blocks)) m = std::max(m, workspace_layout(n_rows, log_num_blocks, st, nullptr, nullptr));
  return m;
}

int rpt_bf_probe_strategy_for(const rpt_bf* bf, uint64_t n_rows) {
  if (!bf) return -fail(RPT_ERR_INVALID_ARGUMENT, "null filter");
  return resolve_strategy(bf->probe_strategy.load(), bf->log_num_blocks, n_rows);
}

size_t rpt_bf_probe_workspace_bytes(const rpt_bf* bf, uint64_t n_rows) {
  if (!bf) return 0;
  const int st = resolve_strategy(bf->probe_strategy.load(), bf->log_num_blocks, n_rows);
  return workspace_layout(n_rows, bf->log_num_blocks, st, nullptr, nullptr);
}

int rpt_probe_strategy_supported(int strategy, int log_num_blocks) {
  return strategy == RPT_PROBE_AUTO ? 1 : strategy_supported(strategy, log_num_blocks);
}

int rpt_bf_set_probe_strategy(rpt_bf* bf, int strategy) {
  if (!bf) return fail(RPT_ERR_INVALID_ARGUMENT, "null filter");
  if (strategy < RPT_PROBE_AUTO || strategy > RPT_PROBE_BUCKETED)
    return fail(RPT_ERR_INVALID_ARGUMENT, "unknown probe strategy %d", strategy);
  bf->probe_strategy.store(strategy);
  return RPT_OK;
}

int rpt_bf_probe_strategy(const rpt_bf* bf) {
  if (!bf) return -fail(RPT_ERR_INVALID_ARGUMENT, "null filter");
  return resolve_strategy(bf->probe_strategy.load(), bf->log_num_blocks, ~0ULL);
}

int rpt_bf_create_log_blocks(int device, int log_num_blocks, rpt_bf** out) {
  if (!out) return fail(RPT_ERR_INVALID_ARGUMENT, "null out");
  *out = nullptr;
  if (log_num_blocks < 0 || log_num_blocks > 40) return fail(RPT_ERR_INVALID_ARGUMENT, "log_num_blocks %d", log_num_blocks);
  RPT_ON_DEVICE(device);
  rpt_bf* bf = new rpt_bf();
  bf->device = device;
  int st = alloc_words(bf, log_num_blocks);
  if (st == RPT_OK) st = alloc_stats(bf);
  if (st != RPT_OK) {
    if (bf->words) (void)hipFree(bf->words);
    delete bf;
    return st;
  }
  *out = bf;
  return RPT_OK;
}

int rpt_bf_create(int device, uint64_t est_num_rows, rpt_bf** out) {
  int st = rpt_bf_create_log_blocks(device, log_blocks_for_rows(est_num_rows), out);
  if (st == RPT_OK) (*out)->sized_for_rows = est_num_rows;
  return st;
}

int rpt_bf_destroy(rpt_bf* bf) {
  if (!bf) return RPT_OK;
  {
    DeviceGuard g(bf->device);
    if (bf->words) (void)hipFree(bf->words);
    if (bf->stats) (void)hipFree(bf->stats);
    if (bf->order_ev) (void)hipEventDestroy(bf->order_ev);
    if (bf->zero_ev) (void)hipEventDestroy(bf->zero_ev);
  }
  delete bf;
  return RPT_OK;
}

int rpt_bf_get_info(const rpt_bf* bf, rpt_bf_info* out) {
  if (!bf || !out) return fail(RPT_ERR_INVALID_ARGUMENT, "null argument");
  out->device = bf->device;
  out->log_num_blocks = bf->log_num_blocks;
  out->num_blocks = 1ULL << bf->log_num_blocks;
  out->sized_for_rows = bf->sized_for_rows;
  out->has_data = bf->has_data.load();
  out->finalized = bf->finalized.load();
  out->words = bf->words;
  return RPT_OK;
}

int rpt_bf_reinitialize(rpt_bf* bf, uint64_t actual_rows) {
  if (!bf) return fail(RPT_ERR_INVALID_ARGUMENT, "null filter");
  RPT_ON_DEVICE(bf->device);
  RPT_HIP(hipDeviceSynchronize());
  if (bf->words) RPT_HIP(hipFree(bf->words));
  bf->words = nullptr;
  int st = alloc_words(bf, log_blocks_for_rows(actual_rows));
  if (st != RPT_OK) return st;
  bf->sized_for_rows = actual_rows;
  bf->has_data.store(0);
  RPT_HIP(hipMemcpy(bf->stats, kStatsInit, sizeof kStatsInit, hipMemcpyHostToDevice));
  std::lock_guard<std::mutex> lk(bf->order_mu);
  bf->order_pending = false;  // the device is idle
  bf->pristine = true;
  bf->clear_pending.store(false);  // alloc_words zeroed the new words
  bf->zero_unsynced.store(false);
  return RPT_OK;
}

int rpt_bf_set_finalized(rpt_bf* bf, int value) {
  if (!bf) return fail(RPT_ERR_INVALID_ARGUMENT, "null filter");
  bf->finalized.store(value ? 1 : 0);
  return RPT_OK;
}

int rpt_bf_set_has_data(rpt_bf* bf, int value) {
  if (!bf) return fail(RPT_ERR_INVALID_ARGUMENT, "null filter");
  bf->has_data.store(value ? 1 : 0);
  return RPT_OK;
}

int rpt_bf_clear(rpt_bf* bf, rpt_stream_t stream) {
  if (!bf) return fail(RPT_ERR_INVALID_ARGUMENT, "null filter");
  RPT_ON_DEVICE(bf->device);
  if (stream_capturing(as_stream(stream)))  // the deferred clear is a host-side flag a replay cannot redo
    return fail(RPT_ERR_INVALID_ARGUMENT, "rpt_bf_clear inside stream capture: clear outside the capture");
  WriteOrder order(bf, as_stream(stream));
  RPT_REFUSE_IN_FLIGHT(order, "write");
  // the words are zeroed by the next operation on them (rpt_bf::clear_pending): a slice insert that
  // stores every slice whole needs no separate pass over the filter (8 GiB C5 filter: 1.35 ms)
  bf->clear_pending.store(true);
  hipLaunchKernelGGL(stats_reset_kernel, dim3(1), dim3(1), 0, as_stream(stream), bf->stats);
  order.done(true);
  RPT_LAUNCHED("stats_reset_kernel");
  bf->has_data.store(0);
  return RPT_OK;
}

int rpt_bf_settle(rpt_bf* bf, rpt_stream_t stream) {
  if (!bf) return fail(RPT_ERR_INVALID_ARGUMENT, "null filter");
  RPT_ON_DEVICE(bf->device);
  RPT_SETTLE(bf, as_stream(stream));
  if (bf->zero_unsynced.load()) {
    std::lock_guard<std::mutex> lk(bf->order_mu);
    if (bf->zero_unsynced.load()) {
      RPT_HIP(hipEventSynchronize(bf->zero_ev));
      bf->zero_unsynced.store(false);
    }
  }
  return RPT_OK;
}

int rpt_bf_get_minmax(const rpt_bf* bf, int64_t* out_min, int64_t* out_max, int* out_has_value, rpt_stream_t stream) {
  if (!bf || !out_min || !out_max || !out_has_value) return fail(RPT_ERR_INVALID_ARGUMENT, "null argument");
  RPT_ON_DEVICE(bf->device);
  int64_t v[2];
  RPT_HIP(hipMemcpyAsync(v, bf->stats, sizeof v, hipMemcpyDeviceToHost, as_stream(stream)));
  RPT_HIP(hipStreamSynchronize(as_stream(stream)));
  *out_has_value = v[0] <= v[1] ? 1 : 0;
  *out_min = *out_has_value ? v[0] : 0;
  *out_max = *out_has_value ? v[1] : 0;
  return RPT_OK;
}

int rpt_bf_set_minmax(rpt_bf* bf, int64_t min_value, int64_t max_value, int has_value, rpt_stream_t stream) {
  if (!bf) return fail(RPT_ERR_INVALID_ARGUMENT, "null filter");
  if (has_value && min_value > max_value) return fail(RPT_ERR_INVALID_ARGUMENT, "min > max");
  RPT_ON_DEVICE(bf->device);
  static thread_local int64_t v[2];  // pageable source: hipMemcpyAsync copies it before returning
  v[0] = has_value ? min_value : INT64_MAX;
  v[1] = has_value ? max_value : INT64_MIN;
  RPT_HIP(hipMemcpyAsync(bf->stats, v, sizeof v, hipMemcpyHostToDevice, as_stream(stream)));
  RPT_HIP(hipStreamSynchronize(as_stream(stream)));
  return RPT_OK;
}

int rpt_bf_insert(rpt_bf* bf, const rpt_key_column* col, uint64_t n, rpt_stream_t stream) {
  if (!bf) return fail(RPT_ERR_INVALID_ARGUMENT, "null filter");
  if (n == 0) return RPT_OK;  // bloom_filter.cpp:72-74
  int st = check_col(col);
  if (st != RPT_OK) return st;
  RPT_ON_DEVICE(bf->device);
  RPT_REFUSE_CAPTURE_WRITE(bf, as_stream(stream), "insert");
  bf->has_data.store(1);  // bloom_filter.cpp:75
  const uint64_t n_segs = ceil_div(n, rpt::kSegRows);
  const unsigned grid = persistent_grid(bf->device, n_segs);
  const rpt::KeyArgs a{col->keys, col->key_sel, col->validity, nullptr};
  WriteOrder order(bf, as_stream(stream));
  RPT_REFUSE_IN_FLIGHT(order, "write");
  const hipError_t ez = zero_pending_locked(bf, as_stream(stream));
  if (ez != hipSuccess) return fail(RPT_ERR_HIP, "hipMemsetAsync failed: %s", hipGetErrorString(ez));
  RPT_DISPATCH_KD(launch_insert_t, col->key_type, dense_ok(col, nullptr), grid, as_stream(stream), bf, a, n, n_segs);
  order.done(false);
  RPT_LAUNCHED("insert_kernel");
  return RPT_OK;
}

size_t rpt_insert_workspace_bytes(uint64_t n_rows, int log_num_blocks) {
  size_t m = 0;
  if (strategy_supported(RPT_PROBE_PARTITIONED, log_num_blocks))
    m = std::max(m, insert_workspace_layout(n_rows, log_num_blocks, RPT_INSERT_PARTITIONED, nullptr, nullptr));
  if (strategy_supported(RPT_PROBE_BUCKETED, log_num_blocks))
    m = std::max(m, insert_workspace_layout(n_rows, log_num_blocks, RPT_INSERT_BUCKETED, nullptr, nullptr));
  return m;
}

int rpt_bf_insert_strategy_for(const rpt_bf* bf, uint64_t n_rows) {
  if (!bf) return -fail(RPT_ERR_INVALID_ARGUMENT, "null filter");
  return resolve_insert_strategy(bf->insert_strategy.load(), bf->log_num_blocks, n_rows);
}

size_t rpt_bf_insert_workspace_bytes(const rpt_bf* bf, uint64_t n_rows) {
  if (!bf) return 0;
  const int st = resolve_insert_strategy(bf->insert_strategy.load(), bf->log_num_blocks, n_rows);
  return insert_workspace_layout(n_rows, bf->log_num_blocks, st, nullptr, nullptr);
}

int rpt_bf_set_insert_strategy(rpt_bf* bf, int strategy) {
  if (!bf) return fail(RPT_ERR_INVALID_ARGUMENT, "null filter");
  if (strategy < RPT_INSERT_AUTO || strategy > RPT_INSERT_BUCKETED)
    return fail(RPT_ERR_INVALID_ARGUMENT, "unknown insert strategy %d", strategy);
  bf->insert_strategy.store(strategy);
  return RPT_OK;
}

int rpt_bf_insert_ws(rpt_bf* bf, const rpt_key_column* col, uint64_t n, void* workspace, size_t workspace_bytes,
                     rpt_stream_t stream) {
  if (!bf) return fail(RPT_ERR_INVALID_ARGUMENT, "null filter");
  if (n == 0) return RPT_OK;  // bloom_filter.cpp:72-74
  const int L = bf->log_num_blocks;
  const int strategy = resolve_insert_strategy(bf->insert_strategy.load(), L, n);
  if (strategy == RPT_INSERT_ATOMIC) return rpt_bf_insert(bf, col, n, stream);
  const bool buck = strategy == RPT_INSERT_BUCKETED;
  if (!strategy_supported(buck ? RPT_PROBE_BUCKETED : RPT_PROBE_PARTITIONED, L))
    return fail(RPT_ERR_INVALID_ARGUMENT, "%s insert unsupported for a 2^%d-block filter",
                buck ? "bucketed" : "partitioned", L);
  int st = check_col(col);
  if (st != RPT_OK) return st;
  if (buck && n > kBucketedInsertBatch) {  // level-1 list positions are 32-bit: batches of 2^31 rows
    const size_t elem = col->key_type == RPT_KEY_I32 ? 4 : 8;
    for (uint64_t off = 0; off < n; off += kBucketedInsertBatch) {
      rpt_key_column sub = *col;
      if (col->key_sel) {
        sub.key_sel = col->key_sel + off;  // dictionary: the selection indexes the whole key array
      } else {
        sub.keys = static_cast<const char*>(col->keys) + off * elem;
        if (col->validity) sub.validity = col->validity + off / 64;  // off is a multiple of 64
      }
      st = rpt_bf_insert_ws(bf, &sub, std::min(kBucketedInsertBatch, n - off), workspace, workspace_bytes, stream);
      if (st != RPT_OK) return st;
    }
    return RPT_OK;
  }
  const size_t need = insert_workspace_layout(n, L, strategy, nullptr, nullptr);
  if (!workspace || workspace_bytes < need)
    return fail(RPT_ERR_WORKSPACE, "workspace %zu bytes < required %zu", workspace_bytes, need);
  RPT_ON_DEVICE(bf->device);
  hipStream_t s = as_stream(stream);
  RPT_REFUSE_CAPTURE_WRITE(bf, s, "insert");
  const bool captured = stream_capturing(s);
  bf->has_data.store(1);  // bloom_filter.cpp:75
  InsertWorkspace ws;
  insert_workspace_layout(n, L, strategy, workspace, &ws);
  // the first kernels below fold the keys' min/max into bf->stats: they must land after the filter's
  // previous write (e.g. a clear's stats reset enqueued on another stream), so wait for its event now;
  // only the slice merge at the end takes the write order for the words (inside a capture the previous
  // write has completed: refuse_capture_write)
  if (!captured) {
    std::lock_guard<std::mutex> lk(bf->order_mu);
    if (bf->order_pending) RPT_HIP(hipStreamWaitEvent(s, bf->order_ev, 0));
  }
  const int cus = num_cus(bf->device);
  const rpt::KeyArgs a{col->keys, col->key_sel, col->validity, nullptr};
  const bool dense = dense_ok(col, nullptr);
  // the partition input: the key column itself, or (bucketed) the level-2 hash array
  uint32_t tile_slices = slice_count(L), tm = tile_mult_of(tile_slices);
  uint64_t n_tiles = ceil_div(n, rpt::kTileRows * tm), n_part = n;
  rpt::KeyArgs pa = a;
  const uint32_t* bucket_tiles = nullptr;
  const uint32_t* dev_n_tiles = nullptr;
  uint32_t grid_slices = tile_slices;
  if (buck) {  // (the key min/max comes from level 1's key read)
    const BucketLevel1 l1{ws.lists, ws.ext_dir, ws.chunk_map, ws.bucket_tiles, ws.list_base, ws.hash_lo, ws.hash_hi,
                          nullptr, nullptr, nullptr};
    st = run_bucket_level1(s, col->key_type, a, dense, n, L, l1, bf->stats);
    if (st != RPT_OK) return st;
    tile_slices = rpt::kBucketSlices;
    tm = 1;
    n_tiles = level2_tiles_max(n, L);
    n_part = n_tiles * rpt::kTileRows;
    pa = rpt::KeyArgs{ws.hash_lo, nullptr, nullptr, nullptr, ws.hash_hi};
    bucket_tiles = ws.bucket_tiles;
    dev_n_tiles = ws.bucket_tiles + bucket_count(L);
    grid_slices = bucket_count(L) * rpt::kBucketSlices;
  }
  if (buck)
    launch_partition_level2(static_cast<unsigned>(n_tiles), s, pa, n_part, n_tiles, ws.recs, nullptr, ws.runs_tm, dev_n_tiles,
                            ws.chunk_map);
  else
    RPT_DISPATCH_KD(launch_partition_t, col->key_type, dense, static_cast<unsigned>(n_tiles), s, pa, n_part, tile_slices - 1,
                    n_tiles, ws.recs, static_cast<uint16_t*>(nullptr), ws.runs_tm, bf->stats, dev_n_tiles, tm);
  RPT_LAUNCHED("partition_kernel");
  st = transpose_u32(s, ws.runs_tm, n_tiles, tile_slices, ws.runs);
  if (st != RPT_OK) return st;
  const uint32_t splits = static_cast<uint32_t>(
      std::max<uint64_t>(1, std::min<uint64_t>(n_tiles, static_cast<uint64_t>(cus) / grid_slices)));
  // only the slice merge writes the words: it alone is ordered after the filter's previous writes
  WriteOrder order(bf, s);
  RPT_REFUSE_IN_FLIGHT(order, "write");
  // one workgroup per slice: every slice stored whole (a deferred clear), plain stores of the non-zero
  // pieces (a pristine filter) or a per-slice choice of read-modify-write vs atomic ORs; several
  // workgroups per slice must merge with atomics (after the deferred clear's memset, if any)
  // (inside a stream capture: atomics, whatever the words hold when the graph replays; no clear is pending)
  const bool store_all = splits == 1 && bf->clear_pending.load() && !captured;
  if (!store_all) {
    const hipError_t ez = zero_pending_locked(bf, s);
    if (ez != hipSuccess) return fail(RPT_ERR_HIP, "hipMemsetAsync failed: %s", hipGetErrorString(ez));
  }
  const int mode = store_all ? rpt::kSliceMergeStoreAll
                   : (splits > 1 || captured) ? rpt::kSliceMergeAtomic
                                : (bf->pristine ? rpt::kSliceMergeStore : rpt::kSliceMergeAdaptive);
  ProfScope prof_i("slice_insert_kernel", s);
  hipLaunchKernelGGL(rpt::slice_insert_kernel, dim3(grid_slices * splits), dim3(rpt::kSliceThreads), 0, s, bf->words, splits,
                     n_tiles, ws.recs, ws.runs, static_cast<uint32_t>(rpt::tile_cap_for(tile_slices, tm)), bucket_tiles, mode);
  prof_i.end();
  if (buck) {  // a level-1 bound hit (never expected): every bit set instead of keys missing
    const uint64_t n_words = 1ULL << L;
    hipLaunchKernelGGL(rpt::l1_error_fill_kernel, dim3(static_cast<unsigned>(std::min<uint64_t>(ceil_div(n_words, rpt::kErrorFillThreads * 8ULL), 4096))),
                       dim3(rpt::kErrorFillThreads), 0, s, bf->words, n_words, l1_error_flag(ws.lists, l1_geom(n, L)));
  }
  const hipError_t el = hipGetLastError();
  if (store_all && el == hipSuccess) bf->clear_pending.store(false);  // the slice stores zeroed the words
  order.done(false);
  if (el != hipSuccess) return fail(RPT_ERR_HIP, "slice_insert_kernel launch: %s", hipGetErrorString(el));
  RPT_LAUNCHED("slice_insert_kernel");
  return RPT_OK;
}

int rpt_bf_find_bits(const rpt_bf* bf, const rpt_key_column* col, uint64_t n, uint64_t* out_bits,
                     rpt_stream_t stream) {
  if (!bf || !out_bits) return fail(RPT_ERR_INVALID_ARGUMENT, "null argument");
  if (n == 0) return RPT_OK;
  int st = check_col(col);
  if (st != RPT_OK) return st;
  RPT_ON_DEVICE(bf->device);
  RPT_SETTLE(bf, as_stream(stream));
  const uint64_t n_segs = ceil_div(n, rpt::kSegRows);
  const unsigned grid = persistent_grid(bf->device, n_segs);
  const rpt::KeyArgs a{col->keys, col->key_sel, col->validity, nullptr};
  RPT_DISPATCH_KD(launch_probe_bits_t, col->key_type, dense_ok(col, nullptr), grid, as_stream(stream), bf, a, n,
                  n_segs, out_bits, static_cast<uint32_t*>(nullptr));
  RPT_LAUNCHED("probe_bits_kernel");
  return RPT_OK;
}


// Phase 1 of rpt_bf_probe. With out_sel (rpt_bf_probe only) the plain PARTITIONED pipeline ends in the
// fused selection-vector tail instead of the result bits, and *done is set: phase 2 is skipped.
static int probe_phase1_impl(const rpt_bf* bf, const rpt_key_column* col, const uint32_t* row_sel, uint64_t n,
                             void* workspace, size_t workspace_bytes, rpt_stream_t stream, uint32_t* out_sel,
                             uint64_t* out_count_dev, bool* done, uint64_t* bits_out = nullptr) {
  if (!bf) return fail(RPT_ERR_INVALID_ARGUMENT, "null filter");
  if (n >= (1ULL << 32)) return fail(RPT_ERR_INVALID_ARGUMENT, "n=%llu rows exceeds uint32 sel_t", (unsigned long long)n);
  if (n == 0) return RPT_OK;
  int st = check_col(col);
  if (st != RPT_OK) return st;
  const int L = bf->log_num_blocks;
  const int strategy = resolve_strategy(bf->probe_strategy.load(), L, n);
  if (!strategy_supported(strategy, L))
    return fail(RPT_ERR_INVALID_ARGUMENT, "probe strategy %d unsupported for a 2^%d-block filter", strategy, L);
  const size_t need = workspace_layout(n, L, strategy, nullptr, nullptr);
  if (!workspace || workspace_bytes < need)
    return fail(RPT_ERR_WORKSPACE, "workspace %zu bytes < required %zu", workspace_bytes, need);
  RPT_ON_DEVICE(bf->device);
  ProbeWorkspace ws;
  workspace_layout(n, L, strategy, workspace, &ws);
  if (bits_out) ws.bits = bits_out;  // rpt_bf_probe_bits: the result bits go to the caller's buffer
  hipStream_t s = as_stream(stream);
  RPT_SETTLE(bf, s);
  const uint64_t n_segs = ceil_div(n, rpt::kSegRows);
  const rpt::KeyArgs a{col->keys, col->key_sel, col->validity, row_sel};
  const bool dense = dense_ok(col, row_sel);
  // the look-back tail's group states and ticket (compact_lookback_kernel) or the sum+scan tail's flagged group
  // sums (group_sum_scan_kernel), cleared by the probe kernel (64-bit words)
  const uint64_t n_groups = ceil_div(n_segs, rpt::kGroupSegs);
  const uint32_t lb_words = !ws.lb_state ? 0u
                            : lookback_tail(strategy) ? static_cast<uint32_t>(n_groups + 1)
                                                      : static_cast<uint32_t>(ceil_div(n_groups, 2));
  if (strategy == RPT_PROBE_GATHER) {
    const unsigned grid = persistent_grid(bf->device, n_segs);
    RPT_DISPATCH_KD(launch_probe_bits_t, col->key_type, dense, grid, s, bf, a, n, n_segs, ws.bits, ws.seg_counts,
                    ws.lb_state, lb_words);
    RPT_LAUNCHED("probe_bits_kernel");
  } else if (strategy == RPT_PROBE_LDS) {
    const uint64_t lds = (8ULL << std::min(L, rpt::kLdsDirectMaxLog)) + 8ULL * rpt::kNumMasks;
    const uint64_t per_cu = std::max<uint64_t>(1, std::min<uint64_t>(rpt::kBlocksPerCU, (160ULL << 10) / lds));
    const uint64_t waves = rpt::kLdsProbeThreads / 64;  // launch_probe_bits_lds_t
    const unsigned grid = static_cast<unsigned>(
        std::max<uint64_t>(1, std::min(ceil_div(n_segs, waves), num_cus(bf->device) * per_cu)));
    RPT_DISPATCH_KD(launch_probe_bits_lds_t, col->key_type, dense, grid, s, bf, a, n, n_segs, ws.bits, ws.seg_counts,
                    ws.lb_state, lb_words);
    RPT_LAUNCHED("probe_bits_kernel<lds>");
  } else {
    // PARTITIONED: the key column, tiles of slice_count(L) slices. BUCKETED: level 1 first, then the
    // same pipeline over the level-2 hash array (tiles of 256 slices, bucket by bucket), then level 1's
    // unpermute.
    const bool buck = strategy == RPT_PROBE_BUCKETED;
    uint32_t tile_slices = slice_count(L), grid_slices = tile_slices, tm = tile_mult_of(tile_slices);
    uint64_t n_tiles = ceil_div(n, rpt::kTileRows * tm), n_part = n;
    rpt::KeyArgs pa = a;
    const uint32_t* bucket_tiles = nullptr;
    const uint32_t* dev_n_tiles = nullptr;
    uint64_t* part_bits = ws.bits;
    uint32_t* part_counts = ws.seg_counts;
    if (buck) {
      const BucketLevel1 l1{ws.lists, ws.ext_dir, ws.chunk_map, ws.bucket_tiles, ws.list_base, ws.hash_lo, ws.hash_hi,
                            ws.pos1, ws.counts_tm, ws.pre_tm};
      int st1 = run_bucket_level1(s, col->key_type, a, dense, n, L, l1, nullptr);
      if (st1 != RPT_OK) return st1;
      tile_slices = rpt::kBucketSlices;
      tm = 1;
      grid_slices = bucket_count(L) * rpt::kBucketSlices;
      n_tiles = level2_tiles_max(n, L);
      n_part = n_tiles * rpt::kTileRows;
      pa = rpt::KeyArgs{ws.hash_lo, nullptr, nullptr, nullptr, ws.hash_hi};
      bucket_tiles = ws.bucket_tiles;
      dev_n_tiles = ws.bucket_tiles + bucket_count(L);
      part_bits = ws.bits2;
      part_counts = nullptr;
    }
    const int cus = num_cus(bf->device);
    if (buck)
      launch_partition_level2(static_cast<unsigned>(n_tiles), s, pa, n_part, n_tiles, ws.recs, ws.pos, ws.runs_tm, dev_n_tiles,
                              ws.chunk_map);
    else
      RPT_DISPATCH_KD(launch_partition_t, col->key_type, dense, static_cast<unsigned>(n_tiles), s, pa, n_part, tile_slices - 1,
                      n_tiles, ws.recs, ws.pos, ws.runs_tm, static_cast<int64_t*>(nullptr), dev_n_tiles, tm);
    RPT_LAUNCHED("partition_kernel");
    // skewed probe keys: slices whose run in some tile is over 4x the mean get mult x finer work items
    rpt::SkewItems skew;
    const bool skewed = !buck && RPT_SLICE_SKEW_MULT > 1 && tile_slices >= 16 && ws.heavy != nullptr;
    if (skewed) {
      skew.heavy = ws.heavy;
      skew.mult = RPT_SLICE_SKEW_MULT;
      if (stream_capturing(s)) {
        // a graph replays the epoch it was captured with: the stamps are reset by a captured
        // memset instead, so every replay stamps only the slices its own keys overload
        skew.epoch = 1;
        RPT_HIP(hipMemsetAsync(ws.heavy, 0, sizeof(uint32_t) * tile_slices, s));
      } else {
        skew.epoch = g_skew_epoch.fetch_add(1) + 1;  // a fresh stamp per call: nothing to clear
      }
    }
    int st2 = transpose_u32(s, ws.runs_tm, n_tiles, tile_slices, ws.runs, skewed ? ws.heavy : nullptr,
                            static_cast<uint32_t>(4 * rpt::kTileRows * tm / tile_slices), skew.epoch);
    if (st2 != RPT_OK) return st2;
    // exactly one resident round of slice workgroups (LDS decides how many fit per CU), never more
    // splits than tiles
    const uint64_t slice_lds = rpt::kSliceWords * 8 + 8ULL * rpt::kRotMasks;
    const uint64_t per_cu = std::max<uint64_t>(1, (160ULL << 10) / slice_lds);
    const uint64_t resident = static_cast<uint64_t>(cus) * per_cu;
    const uint32_t splits = static_cast<uint32_t>(
        std::max<uint64_t>(1, std::min<uint64_t>(n_tiles, RPT_SLICE_SPLIT_MULT * resident / grid_slices)));
    skew.base = grid_slices * splits;
    const uint32_t n_items = skew.base * (skewed ? 1 + skew.mult : 1);
    ProfScope prof6_("slice_probe_kernel", s);
    hipLaunchKernelGGL(rpt::slice_probe_kernel, dim3(static_cast<unsigned>(std::min<uint64_t>(skew.base, resident))),
                       dim3(rpt::kSliceThreads), 0, s, bf->words, splits, n_tiles, ws.recs, ws.runs, ws.passb,
                       static_cast<uint32_t>(rpt::tile_cap_for(tile_slices, tm)), bucket_tiles, n_items, skew);
    prof6_.end();
    RPT_LAUNCHED("slice_probe_kernel");
    const uint64_t cap = rpt::tile_cap_for(tile_slices, tm);
    if (RPT_FUSED_SEL && !buck && out_sel != nullptr && out_count_dev != nullptr) {
      // tile survivor counts (in seg_counts; then their prefix inside blocks of 256 tiles) -> block sums and
      // block offsets (in the unused result-bit area) -> sel
      uint32_t* tile_counts = ws.seg_counts;
      const uint64_t n_blocks = ceil_div(n_tiles, rpt::kTileBlock);
      uint32_t* block_sums = reinterpret_cast<uint32_t*>(ws.bits);
      uint32_t* block_offs = block_sums + n_blocks;
      ProfScope prof7a_("tile_count_kernel", s);
      hipLaunchKernelGGL(rpt::tile_count_kernel, dim3(static_cast<unsigned>(ceil_div(n_tiles, rpt::kTileCountThreads / 64))),
                         dim3(rpt::kTileCountThreads), 0, s, ws.passb, ws.runs_tm, tile_slices, n_tiles, cap, tile_counts);
      prof7a_.end();
      RPT_LAUNCHED("tile_count_kernel");
      ProfScope prof7b_("tile_block_scan_kernel", s);
      hipLaunchKernelGGL(rpt::tile_block_scan_kernel, dim3(static_cast<unsigned>(n_blocks)), dim3(rpt::kTileBlock), 0, s,
                         tile_counts, n_tiles, block_sums);
      prof7b_.end();
      ProfScope prof7d_("group_scan_kernel", s);
      hipLaunchKernelGGL(rpt::group_scan_kernel, dim3(1), dim3(1024), 0, s, block_sums, static_cast<uint32_t>(n_blocks),
                         block_offs, out_count_dev);
      prof7d_.end();
      RPT_LAUNCHED("group_scan_kernel");
      ProfScope prof7c_(tm == 2 ? "unpermute_sel_kernel<2>" : "unpermute_sel_kernel<1>", s);
      if (tm == 2)
        hipLaunchKernelGGL(rpt::unpermute_sel_kernel<2>, dim3(static_cast<unsigned>(n_tiles)), dim3(rpt::kUnpermuteSelThreads<2>),
                           0, s, ws.pos, ws.passb, n, cap, tile_counts, block_offs, row_sel, out_sel);
      else
        hipLaunchKernelGGL(rpt::unpermute_sel_kernel<1>, dim3(static_cast<unsigned>(n_tiles)), dim3(rpt::kUnpermuteSelThreads<1>),
                           0, s, ws.pos, ws.passb, n, cap, tile_counts, block_offs, row_sel, out_sel);
      prof7c_.end();
      RPT_LAUNCHED("unpermute_sel_kernel");
      *done = true;
      return RPT_OK;
    }
    ProfScope prof7_(tm == 2 ? "unpermute_kernel<2>" : "unpermute_kernel<1>", s);
    if (tm == 2)
      hipLaunchKernelGGL(rpt::unpermute_kernel<2>, dim3(static_cast<unsigned>(n_tiles)), dim3(rpt::kUnpermuteThreads), 0,
                         s, ws.pos, ws.passb, n_part, cap, part_bits, part_counts, dev_n_tiles);
    else
      hipLaunchKernelGGL(rpt::unpermute_kernel<1>, dim3(static_cast<unsigned>(n_tiles)), dim3(rpt::kUnpermuteThreads), 0,
                         s, ws.pos, ws.passb, n_part, cap, part_bits, part_counts, dev_n_tiles);
    prof7_.end();
    RPT_LAUNCHED("unpermute_kernel");
    if (buck) {
      ProfScope prof8b_("bucket_unpermute_kernel", s);
      hipLaunchKernelGGL(rpt::bucket_unpermute_kernel, dim3(static_cast<unsigned>(ceil_div(n, rpt::kL1TileRows))),
                         dim3(rpt::kBucketUnpermuteThreads), 0, s, ws.pos1, ws.bits2, n, bucket_count(L) - 1,
                         ws.counts_tm, ws.pre_tm, ws.list_base, l1_geom(n, L).groups, l1_error_flag(ws.lists, l1_geom(n, L)),
                         ws.bits, ws.seg_counts);
      prof8b_.end();
      RPT_LAUNCHED("bucket_unpermute_kernel");
    }
  }
  return RPT_OK;
}

int rpt_bf_probe_phase1(const rpt_bf* bf, const rpt_key_column* col, const uint32_t* row_sel, uint64_t n,
                        void* workspace, size_t workspace_bytes, rpt_stream_t stream) {
  bool done = false;
  return probe_phase1_impl(bf, col, row_sel, n, workspace, workspace_bytes, stream, nullptr, nullptr, &done);
}

int rpt_bf_probe_bits(const rpt_bf* bf, const rpt_key_column* col, const uint32_t* row_sel, uint64_t n,
                      uint64_t* out_bits, void* workspace, size_t workspace_bytes, rpt_stream_t stream) {
  if (!bf || !out_bits) return fail(RPT_ERR_INVALID_ARGUMENT, "null argument");
  bool done = false;
  return probe_phase1_impl(bf, col, row_sel, n, workspace, workspace_bytes, stream, nullptr, nullptr, &done, out_bits);
}

int rpt_bf_probe_phase2(const rpt_bf* bf, const uint32_t* row_sel, uint64_t n, uint32_t* out_sel,
                        uint64_t* out_count_dev, void* workspace, size_t workspace_bytes, rpt_stream_t stream) {
  if (!bf || !out_count_dev) return fail(RPT_ERR_INVALID_ARGUMENT, "null argument");
  if (n >= (1ULL << 32)) return fail(RPT_ERR_INVALID_ARGUMENT, "n=%llu rows exceeds uint32 sel_t", (unsigned long long)n);
  RPT_ON_DEVICE(bf->device);
  hipStream_t s = as_stream(stream);
  if (n == 0) {  // bloom_filter.cpp:63-65
    RPT_HIP(hipMemsetAsync(out_count_dev, 0, sizeof(uint64_t), s));
    return RPT_OK;
  }
  if (!out_sel) return fail(RPT_ERR_INVALID_ARGUMENT, "null out_sel");
  const int L = bf->log_num_blocks;
  const int strategy = resolve_strategy(bf->probe_strategy.load(), L, n);
  const size_t need = workspace_layout(n, L, strategy, nullptr, nullptr);
  if (!workspace || workspace_bytes < need)
    return fail(RPT_ERR_WORKSPACE, "workspace %zu bytes < required %zu", workspace_bytes, need);
  ProbeWorkspace ws;
  workspace_layout(n, L, strategy, workspace, &ws);
  const uint64_t n_segs = ceil_div(n, rpt::kSegRows);
  const uint64_t n_groups = ceil_div(n_segs, rpt::kGroupSegs);
  if (lookback_tail(strategy)) {
    // one launch: group offsets by look-back (phase 1's probe kernel cleared the states and the ticket)
    ProfScope prof10_("compact_lookback_kernel", s);
    hipLaunchKernelGGL(rpt::compact_lookback_kernel, dim3(static_cast<unsigned>(n_groups)), dim3(rpt::kBlockThreads), 0, s,
                       ws.bits, ws.seg_counts, n_segs, static_cast<uint32_t>(n_groups), ws.lb_state, row_sel, out_sel,
                       out_count_dev);
    prof10_.end();
    RPT_LAUNCHED("compact_lookback_kernel");
    return RPT_OK;
  }
  if (sumscan_tail(strategy)) {
    // group sums + scan in one launch (phase 1's probe kernel cleared the done counter), then the compaction
    ProfScope prof8_("group_sum_scan_kernel", s);
    hipLaunchKernelGGL(rpt::group_sum_scan_kernel, dim3(static_cast<unsigned>(n_groups)), dim3(rpt::kBlockThreads), 0, s,
                       ws.seg_counts, n_segs, static_cast<uint32_t>(n_groups), reinterpret_cast<uint32_t*>(ws.lb_state),
                       ws.group_offs, out_count_dev);
    prof8_.end();
    RPT_LAUNCHED("group_sum_scan_kernel");
    ProfScope prof10_("compact_kernel", s);
    hipLaunchKernelGGL(rpt::compact_kernel, dim3(static_cast<unsigned>(n_groups)), dim3(rpt::kBlockThreads), 0, s,
                       ws.bits, ws.seg_counts, n_segs, ws.group_offs, row_sel, out_sel);
    prof10_.end();
    RPT_LAUNCHED("compact_kernel");
    return RPT_OK;
  }
  ProfScope prof8_("group_sum_kernel", s);
  hipLaunchKernelGGL(rpt::group_sum_kernel, dim3(static_cast<unsigned>(n_groups)), dim3(rpt::kBlockThreads), 0, s,
                     ws.seg_counts, n_segs, ws.group_sums);
  prof8_.end();
  RPT_LAUNCHED("group_sum_kernel");
  ProfScope prof9_("group_scan_kernel", s);
  hipLaunchKernelGGL(rpt::group_scan_kernel, dim3(1), dim3(1024), 0, s, ws.group_sums,
                     static_cast<uint32_t>(n_groups), ws.group_offs, out_count_dev);
  prof9_.end();
  RPT_LAUNCHED("group_scan_kernel");
  ProfScope prof10_("compact_kernel", s);
  hipLaunchKernelGGL(rpt::compact_kernel, dim3(static_cast<unsigned>(n_groups)), dim3(rpt::kBlockThreads), 0, s,
                     ws.bits, ws.seg_counts, n_segs, ws.group_offs, row_sel, out_sel);
  prof10_.end();
  RPT_LAUNCHED("compact_kernel");
  return RPT_OK;
}

int rpt_bf_probe_is_fused(const rpt_bf* bf, uint64_t n_rows) {
  if (!bf) return -fail(RPT_ERR_INVALID_ARGUMENT, "null filter");
  return n_rows > 0 && n_rows <= rpt::kSmallRows && bf->probe_strategy.load() == RPT_PROBE_AUTO;
}

int rpt_bf_probe(const rpt_bf* bf, const rpt_key_column* col, const uint32_t* row_sel, uint64_t n,
                 uint32_t* out_sel, uint64_t* out_count_dev, void* workspace, size_t workspace_bytes,
                 rpt_stream_t stream) {
  if (!bf || !out_count_dev) return fail(RPT_ERR_INVALID_ARGUMENT, "null argument");
  RPT_ON_DEVICE(bf->device);
  if (rpt_bf_probe_is_fused(bf, n) == 1) {
    // small batch: one fused launch, no workspace
    int st = check_col(col);
    if (st != RPT_OK) return st;
    if (!out_sel) return fail(RPT_ERR_INVALID_ARGUMENT, "null out_sel");
    hipStream_t s = as_stream(stream);
    RPT_SETTLE(bf, s);
    const rpt::KeyArgs a{col->keys, col->key_sel, col->validity, row_sel};
    RPT_DISPATCH_KD(launch_probe_small_t, col->key_type, dense_ok(col, row_sel), s, bf, a, n, row_sel, out_sel,
                    out_count_dev);
    RPT_LAUNCHED("probe_small_kernel");
    return RPT_OK;
  }
  bool done = false;
  int st = probe_phase1_impl(bf, col, row_sel, n, workspace, workspace_bytes, stream, out_sel, out_count_dev, &done);
  if (st != RPT_OK || done) return st;
  return rpt_bf_probe_phase2(bf, row_sel, n, out_sel, out_count_dev, workspace, workspace_bytes, stream);
}

int rpt_bf_probe_chain(const rpt_bf* const* filters, const rpt_key_column* cols, uint32_t n_filters,
                       const uint32_t* row_sel, uint64_t n, uint32_t* out_sel, uint64_t* out_count_dev,
                       rpt_stream_t stream) {
  if (!filters || !cols || !out_count_dev) return fail(RPT_ERR_INVALID_ARGUMENT, "null argument");
  if (n_filters == 0 || n_filters > RPT_MAX_CHAIN)
    return fail(RPT_ERR_INVALID_ARGUMENT, "n_filters=%u outside 1..%d", n_filters, RPT_MAX_CHAIN);
  if (n > rpt::kSmallRows)
    return fail(RPT_ERR_INVALID_ARGUMENT, "n=%llu rows exceeds RPT_SMALL_PROBE_ROWS", (unsigned long long)n);
  rpt::ChainArgs c{};
  for (uint32_t f = 0; f < n_filters; f++) {
    if (!filters[f]) return fail(RPT_ERR_INVALID_ARGUMENT, "null filter %u", f);
    if (filters[f]->device != filters[0]->device) return fail(RPT_ERR_INVALID_ARGUMENT, "filters on different devices");
    const int st = check_col(&cols[f]);
    if (st != RPT_OK) return st;
    c.words[f] = filters[f]->words;
    c.block_mask[f] = (1ULL << filters[f]->log_num_blocks) - 1;
    c.a[f] = rpt::KeyArgs{cols[f].keys, cols[f].key_sel, cols[f].validity, row_sel};
    c.key_type[f] = cols[f].key_type;
  }
  c.k = n_filters;
  RPT_ON_DEVICE(filters[0]->device);
  hipStream_t s = as_stream(stream);
  if (n == 0) {
    RPT_HIP(hipMemsetAsync(out_count_dev, 0, sizeof(uint64_t), s));
    return RPT_OK;
  }
  if (!out_sel) return fail(RPT_ERR_INVALID_ARGUMENT, "null out_sel");
  for (uint32_t f = 0; f < n_filters; f++) RPT_SETTLE(filters[f], s);
  ProfScope prof("probe_chain_small_kernel", s);
  hipLaunchKernelGGL(rpt::probe_chain_small_kernel, dim3(1), dim3(rpt::kSmallThreads), 0, s, c, n, row_sel, out_sel,
                     out_count_dev);
  prof.end();
  RPT_LAUNCHED("probe_chain_small_kernel");
  return RPT_OK;
}


int rpt_hash_combine(const rpt_key_column* col, uint64_t n, uint64_t* inout_hashes, rpt_stream_t stream) {
  return launch_hash<true>(col, n, inout_hashes, stream);
}

int rpt_hash_keys(const rpt_key_column* col, uint64_t n, uint64_t* out_hashes, rpt_stream_t stream) {
  return launch_hash<false>(col, n, out_hashes, stream);
}

int rpt_keys_widen(const uint32_t* lo, const uint32_t* chunk_hi, const uint32_t* chunk_row0, uint64_t n_chunks,
                   uint64_t* out, rpt_stream_t stream) {
  if (n_chunks == 0) return RPT_OK;
  if (!lo || !chunk_hi || !chunk_row0 || !out) return fail(RPT_ERR_INVALID_ARGUMENT, "null argument");
  if (n_chunks > 0x7FFFFFFFu) return fail(RPT_ERR_INVALID_ARGUMENT, "too many chunks");
  ProfScope prof_w("widen_keys_kernel", as_stream(stream));
  hipLaunchKernelGGL(rpt::widen_keys_kernel, dim3(static_cast<unsigned>(n_chunks)), dim3(rpt::kWidenThreads), 0,
                     as_stream(stream), lo, chunk_hi, chunk_row0, out);
  prof_w.end();
  RPT_LAUNCHED("widen_keys_kernel");
  return RPT_OK;
}

int rpt_words_or_slices(uint64_t* dst, const uint64_t* srcs, uint32_t k, uint64_t n_words, rpt_stream_t stream) {
  if (!dst || (!srcs && k > 0)) return fail(RPT_ERR_INVALID_ARGUMENT, "null argument");
  if (n_words == 0) return RPT_OK;
  const unsigned grid = static_cast<unsigned>(std::max<uint64_t>(1, std::min<uint64_t>(ceil_div(n_words / 2, rpt::kBlockThreads), 8192)));
  ProfScope prof12_("or_slices_kernel", as_stream(stream));
  hipLaunchKernelGGL(rpt::or_slices_kernel, dim3(grid), dim3(rpt::kBlockThreads), 0, as_stream(stream), dst, srcs, k,
                     n_words, n_words, 0);
  prof12_.end();
  RPT_LAUNCHED("or_slices_kernel");
  return RPT_OK;
}

int rpt_words_or(uint64_t* dst, const uint64_t* src, uint64_t n_words, rpt_stream_t stream) {
  if (!dst || !src) return fail(RPT_ERR_INVALID_ARGUMENT, "null argument");
  if (n_words == 0) return RPT_OK;
  const unsigned grid = static_cast<unsigned>(std::max<uint64_t>(1, std::min<uint64_t>(ceil_div(n_words / 2, rpt::kBlockThreads), 8192)));
  ProfScope prof13_("or_slices_kernel", as_stream(stream));
  hipLaunchKernelGGL(rpt::or_slices_kernel, dim3(grid), dim3(rpt::kBlockThreads), 0, as_stream(stream), dst, src, 1u,
                     n_words, n_words, 1);
  prof13_.end();
  RPT_LAUNCHED("or_slices_kernel");
  return RPT_OK;
}

int rpt_bf_merge_or(rpt_bf* dst, const rpt_bf* src, rpt_stream_t stream) {
  if (!dst || !src) return fail(RPT_ERR_INVALID_ARGUMENT, "null filter");
  if (dst->log_num_blocks != src->log_num_blocks || dst->device != src->device)
    return fail(RPT_ERR_SHAPE_MISMATCH, "merge of log_num_blocks %d (dev %d) with %d (dev %d)", dst->log_num_blocks,
                dst->device, src->log_num_blocks, src->device);
  RPT_ON_DEVICE(dst->device);
  RPT_REFUSE_CAPTURE_WRITE(dst, as_stream(stream), "merge");
  if (src != dst) RPT_SETTLE(src, as_stream(stream));
  WriteOrder order(dst, as_stream(stream));
  RPT_REFUSE_IN_FLIGHT(order, "write");
  const hipError_t ez = zero_pending_locked(dst, as_stream(stream));
  if (ez != hipSuccess) return fail(RPT_ERR_HIP, "hipMemsetAsync failed: %s", hipGetErrorString(ez));
  int st = rpt_words_or(dst->words, src->words, 1ULL << dst->log_num_blocks, stream);
  if (st == RPT_OK) {
    // inside the write order: a later clear's stats reset must not be overtaken by this merge
    hipLaunchKernelGGL(stats_merge_kernel, dim3(1), dim3(1), 0, as_stream(stream), dst->stats, src->stats);
    const hipError_t el = hipGetLastError();
    if (el != hipSuccess) st = fail(RPT_ERR_HIP, "launch of stats_merge_kernel failed: %s", hipGetErrorString(el));
  }
  order.done(false);
  if (st != RPT_OK) return st;
  if (src->has_data.load()) dst->has_data.store(1);
  return RPT_OK;
}

// ---- multi-GPU Combine over RCCL ------------------------------------------------------------------
}  // extern "C"
namespace {
// The RCCL entry points rpt_bf_allreduce_or uses, resolved from librccl on first use (rccl.h types:
// ncclResult_t = int, ncclComm_t = opaque pointer, ncclDataType_t / ncclRedOp_t = int enums).
struct RcclApi {
  rpt_rccl_api_table fn{};
  std::string load_error;
};
constexpr int kNcclInt64 = 4, kNcclUint64 = 5, kNcclMin = 3;  // rccl.h ncclDataType_t / ncclRedOp_t

std::shared_ptr<const RcclApi> load_librccl() {
  auto a = std::make_shared<RcclApi>();
  void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
  if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_LOCAL);
  if (!h) {
    const char* e = dlerror();
    a->load_error = e ? e : "dlopen(librccl) failed";
    return a;
  }
  auto sym = [&](auto& fn, const char* name) {
    fn = reinterpret_cast<std::remove_reference_t<decltype(fn)>>(dlsym(h, name));
    if (!fn && a->load_error.empty()) a->load_error = std::string("librccl lacks ") + name;
  };
  sym(a->fn.get_unique_id, "ncclGetUniqueId");
  sym(a->fn.comm_init_rank, "ncclCommInitRank");
  sym(a->fn.comm_destroy, "ncclCommDestroy");
  sym(a->fn.group_start, "ncclGroupStart");
  sym(a->fn.group_end, "ncclGroupEnd");
  sym(a->fn.send, "ncclSend");
  sym(a->fn.recv, "ncclRecv");
  sym(a->fn.all_reduce, "ncclAllReduce");
  sym(a->fn.comm_count, "ncclCommCount");
  sym(a->fn.comm_user_rank, "ncclCommUserRank");
  sym(a->fn.error_string, "ncclGetErrorString");
  sym(a->fn.comm_abort, "ncclCommAbort");
  sym(a->fn.get_async_error, "ncclCommGetAsyncError");
  sym(a->fn.comm_init_rank_config, "ncclCommInitRankConfig");
  // optional: only rpt_rccl_comm_destroy of a non-blocking communicator uses it (abort if absent)
  a->fn.comm_finalize = reinterpret_cast<decltype(a->fn.comm_finalize)>(dlsym(h, "ncclCommFinalize"));
  return a;
}

// librccl; the test build (RPT_TESTING_HOOKS, csrc/rpt_gpu_testing.h) can swap in a loopback table.
std::mutex g_rccl_mu;
std::shared_ptr<const RcclApi> g_rccl, g_librccl;
std::shared_ptr<const RcclApi> rccl_api() {
  std::lock_guard<std::mutex> lk(g_rccl_mu);
  if (!g_rccl) {
    if (!g_librccl) g_librccl = load_librccl();
    g_rccl = g_librccl;
  }
  return g_rccl;
}

// {min, max, has_data} -> {min, ~max, ~has}: bit complement reverses the order without overflow, so one
// MIN all-reduce gives the global min, max and has_data (an empty partial holds {INT64_MAX, INT64_MIN}).
__global__ void minmax_pack_kernel(const int64_t* stats, int has, int64_t* v) {
  v[0] = stats[0];
  v[1] = ~stats[1];
  v[2] = ~static_cast<int64_t>(has != 0);
}
__global__ void minmax_unpack_kernel(const int64_t* v, int64_t* stats, int* has) {
  stats[0] = v[0];
  stats[1] = ~v[1];
  *has = static_cast<int>(~v[2]);
}

// Word ranges of the OR all-reduce: rank j owns words [lo(j), lo(j + 1)), starts rounded down to 32 words
// (256 B) so every slice, and every round's piece of it, is 16-B aligned for the OR kernel; the last rank
// takes the rest. The reduce-scatter runs in rounds of at most `round` words per peer (the staging bound);
// every rank derives the same round count, so the grouped sends and receives pair up round by round.
struct MergeGeom {
  uint64_t nw;
  int world;
  uint64_t lo(int j) const { return j >= world ? nw : ((nw * static_cast<uint64_t>(j)) / world) & ~31ULL; }
  uint64_t len(int j) const { return lo(j + 1) - lo(j); }
  uint64_t max_len() const {
    uint64_t m = 0;
    for (int j = 0; j < world; j++) m = std::max(m, len(j));
    return m;
  }
  uint64_t round_words() const { return std::max<uint64_t>(2, std::min<uint64_t>(RPT_ALLREDUCE_ROUND_WORDS, (max_len() + 1) & ~1ULL)); }
  uint64_t rounds() const { return ceil_div(max_len(), round_words()); }
  // words of slice j sent in round r
  uint64_t piece(int j, uint64_t r) const {
    const uint64_t R = round_words(), l = len(j);
    return r * R >= l ? 0 : std::min(R, l - r * R);
  }
  // workspace: {min, ~max, ~has, has} scratch, then two staging buffers of (world - 1) round pieces
  size_t workspace_bytes() const {
    return 256 + (world > 1 ? 2 * static_cast<size_t>(world - 1) * round_words() * 8 : 0);
  }
};

// A helper stream + events per concurrent all-reduce: the OR kernel of round r runs there while the
// transfers of round r + 1 run on the caller's stream. Pooled per device (never destroyed).
struct MergeHelper {
  int device;
  hipStream_t s = nullptr;
  hipEvent_t rx[2] = {nullptr, nullptr}, ored[2] = {nullptr, nullptr}, join = nullptr;
};
std::mutex g_helper_mu;
std::vector<MergeHelper*> g_helper_free;
MergeHelper* take_helper(int device) {
  {
    std::lock_guard<std::mutex> lk(g_helper_mu);
    for (size_t i = 0; i < g_helper_free.size(); i++)
      if (g_helper_free[i]->device == device) {
        MergeHelper* h = g_helper_free[i];
        g_helper_free.erase(g_helper_free.begin() + static_cast<long>(i));
        return h;
      }
  }
  auto* h = new MergeHelper{device};
  bool ok = hipStreamCreateWithFlags(&h->s, hipStreamNonBlocking) == hipSuccess;
  for (hipEvent_t* e : {&h->rx[0], &h->rx[1], &h->ored[0], &h->ored[1], &h->join})
    ok = ok && hipEventCreateWithFlags(e, hipEventDisableTiming) == hipSuccess;
  if (!ok) {
    (void)hipGetLastError();
    return nullptr;  // leaks what was created: only after a HIP failure
  }
  return h;
}
void give_helper(MergeHelper* h) {
  std::lock_guard<std::mutex> lk(g_helper_mu);
  g_helper_free.push_back(h);
}

// ---- bounded waits (rpt_collective_set_timeout_ms) ----
// A peer that dies mid-merge never posts its side of a grouped send/recv: RCCL's kernels on this rank's
// stream then wait for it forever, and ncclGroupEnd has already returned success. So the merge never blocks
// on the stream blindly: it polls the stream and ncclCommGetAsyncError until the deadline, and on an error or
// timeout aborts the communicator (ncclCommAbort: RCCL's kernels leave), then drains the streams, bounded too.
constexpr int kNcclInProgress = 7;  // rccl.h ncclInProgress (a non-blocking communicator's pending call)
std::atomic<uint64_t> g_coll_timeout_ms{RPT_COLLECTIVE_TIMEOUT_MS_DEFAULT};
// Communicators this library made (rpt_rccl_comm_init_rank[_nonblocking]; the flag: non-blocking), and
// those of them a failed merge aborted: ncclCommAbort frees a communicator, so rpt_rccl_comm_destroy must
// not. A caller-owned communicator (one the caller made and passed in) is never recorded: the merge tells
// its owner by RPT_ERR_COMM_ABORTED, and nothing here grows with such failures.
std::mutex g_aborted_mu;
std::vector<void*> g_aborted;
std::vector<std::pair<void*, bool>> g_made;
std::atomic<int> g_abort_on_error{1};  // rpt_collective_set_abort_on_error

using Clock = std::chrono::steady_clock;
Clock::time_point coll_deadline() { return Clock::now() + std::chrono::milliseconds(g_coll_timeout_ms.load()); }

// Sleep between polls: 10 us doubling to 200 us (an 8 GiB merge takes ~0.1 s, a 16 MiB one ~1 ms).
struct Backoff {
  unsigned us = 10;
  void pause() {
    std::this_thread::sleep_for(std::chrono::microseconds(us));
    us = std::min(us * 2, 200u);
  }
};

// RPT_OK once every stream in `ss` has completed; otherwise a status and the reason in *why. With a
// communicator, its asynchronous error is polled too (an error other than ncclInProgress ends the wait).
int poll_streams(const rpt_rccl_api_table* api, void* comm, std::initializer_list<hipStream_t> ss,
                 Clock::time_point deadline, std::string* why) {
  Backoff b;
  for (;;) {
    bool all = true;
    for (hipStream_t x : ss) {
      const hipError_t q = hipStreamQuery(x);
      if (q == hipErrorNotReady) {
        all = false;
      } else if (q != hipSuccess) {
        *why = std::string("stream error: ") + hipGetErrorString(q);
        return RPT_ERR_HIP;
      }
    }
    if (all) return RPT_OK;
    if (api && comm) {
      int ae = 0;
      const int rc = api->get_async_error(comm, &ae);
      if (rc != 0 || (ae != 0 && ae != kNcclInProgress)) {
        *why = std::string("RCCL asynchronous error: ") + api->error_string(rc != 0 ? rc : ae);
        return RPT_ERR_COLLECTIVE;
      }
    }
    if (Clock::now() >= deadline) {
      *why = "no progress within " + std::to_string(g_coll_timeout_ms.load()) + " ms (a peer that never posted its side?)";
      return RPT_ERR_COLLECTIVE;
    }
    b.pause();
  }
}

// A call that returned ncclInProgress (non-blocking communicator): poll ncclCommGetAsyncError until it
// settles or the deadline passes. Other results pass through.
int settle_nccl(const rpt_rccl_api_table& api, void* comm, int rc, Clock::time_point deadline) {
  Backoff b;
  while (rc == kNcclInProgress) {
    if (Clock::now() >= deadline) return kNcclInProgress;
    b.pause();
    int ae = 0;
    const int q = api.get_async_error(comm, &ae);
    rc = q != 0 ? q : ae;
  }
  return rc;
}

void abort_comm(const rpt_rccl_api_table& api, void* comm) {
  {
    std::lock_guard<std::mutex> lk(g_aborted_mu);
    for (const auto& m : g_made)
      if (m.first == comm) {
        g_aborted.push_back(comm);
        break;
      }
  }
  (void)api.comm_abort(comm);
}

bool take_aborted(void* comm) {
  std::lock_guard<std::mutex> lk(g_aborted_mu);
  auto it = std::find(g_aborted.begin(), g_aborted.end(), comm);
  if (it == g_aborted.end()) return false;
  g_aborted.erase(it);
  return true;
}

// A communicator made here: (re)registered at its address (a new one at an aborted one's address is live).
void note_made(void* comm, bool nonblocking) {
  std::lock_guard<std::mutex> lk(g_aborted_mu);
  g_aborted.erase(std::remove(g_aborted.begin(), g_aborted.end(), comm), g_aborted.end());
  for (auto& m : g_made)
    if (m.first == comm) {
      m.second = nonblocking;
      return;
    }
  g_made.emplace_back(comm, nonblocking);
}

// Forget a communicator made here; returns {was made here, non-blocking}.
std::pair<bool, bool> forget_made(void* comm) {
  std::lock_guard<std::mutex> lk(g_aborted_mu);
  for (size_t i = 0; i < g_made.size(); i++)
    if (g_made[i].first == comm) {
      const bool nb = g_made[i].second;
      g_made.erase(g_made.begin() + static_cast<long>(i));
      return {true, nb};
    }
  return {false, false};
}
}  // namespace
extern "C" {

#define RPT_NCCL(call)                                                                          \
  do {                                                                                         \
    const int rc_ = (call);                                                                    \
    if (rc_ != 0) return fail(RPT_ERR_COLLECTIVE, "%s: %s", #call, api.error_string(rc_));      \
  } while (0)
// inside ncclGroupStart/End: close the group before returning (rpt_bf_allreduce_or_ws then aborts the
// communicator: peers may already depend on this rank's earlier groups)
#define RPT_NCCL_IN_GROUP(call)                                                                 \
  do {                                                                                         \
    const int rc_ = (call);                                                                    \
    if (rc_ != 0) {                                                                            \
      (void)api.group_end();                                                                   \
      return fail(RPT_ERR_COLLECTIVE, "%s: %s", #call, api.error_string(rc_));                 \
    }                                                                                          \
  } while (0)
// a merge call: a non-blocking communicator's ncclInProgress is polled to completion by the deadline
#define RPT_NCCL_MERGE(call)                                                                    \
  do {                                                                                         \
    const int rc_ = settle_nccl(api, nccl_comm, (call), deadline);                             \
    if (rc_ != 0) return fail(RPT_ERR_COLLECTIVE, "%s: %s", #call, api.error_string(rc_));      \
  } while (0)

size_t rpt_allreduce_workspace_bytes(int world, int log_num_blocks) {
  if (world < 1 || log_num_blocks < 0 || log_num_blocks > 40) return 0;
  return MergeGeom{1ULL << log_num_blocks, world}.workspace_bytes();
}

int rpt_bf_allreduce_or_ws(rpt_bf* bf, void* nccl_comm, void* workspace, size_t workspace_bytes,
                           rpt_stream_t stream) {
  t_merge_stuck = false;
  if (!bf || !nccl_comm) return fail(RPT_ERR_INVALID_ARGUMENT, "null argument");
  const std::shared_ptr<const RcclApi> api_p = rccl_api();
  const rpt_rccl_api_table& api = api_p->fn;
  if (!api_p->load_error.empty()) return fail(RPT_ERR_COLLECTIVE, "RCCL unavailable: %s", api_p->load_error.c_str());
  RPT_ON_DEVICE(bf->device);
  hipStream_t s = as_stream(stream);
  int world = 1, me = 0;
  RPT_NCCL(api.comm_count(nccl_comm, &world));
  RPT_NCCL(api.comm_user_rank(nccl_comm, &me));
  const MergeGeom g{1ULL << bf->log_num_blocks, world};
  if (!workspace || workspace_bytes < g.workspace_bytes())
    return fail(RPT_ERR_WORKSPACE, "all-reduce workspace %zu bytes < required %zu", workspace_bytes, g.workspace_bytes());
  int64_t* v = static_cast<int64_t*>(workspace);  // {min, ~max, ~has} then has_data (as int) in v[3]
  uint64_t* stage = reinterpret_cast<uint64_t*>(static_cast<char*>(workspace) + 256);
  if (stream_capturing(s))  // it polls the stream from the host: nothing of it can be replayed
    return fail(RPT_ERR_INVALID_ARGUMENT, "rpt_bf_allreduce_or inside stream capture");
  MergeHelper* h = nullptr;
  WriteOrder order(bf, s);
  RPT_REFUSE_IN_FLIGHT(order, "write");
  if (zero_pending_locked(bf, s) != hipSuccess) {
    order.done(false);
    return fail(RPT_ERR_HIP, "hipMemsetAsync failed");
  }
  // every RCCL call below, and the wait for the stream, ends by this deadline (rpt_collective_set_timeout_ms)
  const Clock::time_point deadline = coll_deadline();
  bool posted = false;          // a collective call was issued: peers may now depend on this rank
  bool helper_pending = false;  // OR kernels enqueued on the helper stream and not yet joined into s
  auto join_helper = [&]() -> hipError_t {
    if (!helper_pending) return hipSuccess;
    helper_pending = false;
    hipError_t e = hipEventRecord(h->join, h->s);
    if (e == hipSuccess) e = hipStreamWaitEvent(s, h->join, 0);
    return e;
  };
  auto run = [&]() -> int {
    if (world > 1) {
      h = take_helper(bf->device);
      if (!h) return fail(RPT_ERR_HIP, "all-reduce helper stream creation failed");
      const uint64_t R = g.round_words(), nr = g.rounds();
      bool ored[2] = {false, false};
      // reduce-scatter by OR: rank `me` owns words [lo(me), lo(me + 1)); in round r every peer sends its
      // r-th piece of that range into staging buffer r % 2, and the OR kernel folds the pieces in on the
      // helper stream while round r + 1 transfers
      for (uint64_t r = 0; r < nr; r++) {
        const int b = static_cast<int>(r & 1);
        uint64_t* buf = stage + static_cast<uint64_t>(b) * (world - 1) * R;
        const uint64_t cnt = g.piece(me, r), stride = (cnt + 1) & ~1ULL;
        if (ored[b]) RPT_HIP(hipStreamWaitEvent(s, h->ored[b], 0));  // round r - 2's OR has read buf
        posted = true;
        RPT_NCCL_MERGE(api.group_start());
        for (int p = 0, k = 0; p < world; p++) {
          if (p == me) continue;
          const uint64_t out = g.piece(p, r);
          if (out) RPT_NCCL_IN_GROUP(api.send(bf->words + g.lo(p) + r * R, out, kNcclUint64, p, nccl_comm, s));
          if (cnt) RPT_NCCL_IN_GROUP(api.recv(buf + static_cast<uint64_t>(k) * stride, cnt, kNcclUint64, p, nccl_comm, s));
          k++;
        }
        RPT_NCCL_MERGE(api.group_end());
        if (cnt) {
          RPT_HIP(hipEventRecord(h->rx[b], s));
          RPT_HIP(hipStreamWaitEvent(h->s, h->rx[b], 0));
          helper_pending = true;
          const unsigned grid = static_cast<unsigned>(std::max<uint64_t>(1, std::min<uint64_t>(ceil_div(cnt / 2 + 1, rpt::kBlockThreads), 2048)));
          ProfScope prof_or("or_slices_kernel(allreduce)", h->s);
          hipLaunchKernelGGL(rpt::or_slices_kernel, dim3(grid), dim3(rpt::kBlockThreads), 0, h->s,
                             bf->words + g.lo(me) + r * R, buf, static_cast<uint32_t>(world - 1), cnt, stride, 1);
          prof_or.end();
          RPT_LAUNCHED("or_slices_kernel");
          RPT_HIP(hipEventRecord(h->ored[b], h->s));
          ored[b] = true;
        }
      }
      // all-gather: every rank's merged words to every peer, once its OR kernels are done
      RPT_HIP(join_helper());
      RPT_NCCL_MERGE(api.group_start());
      for (int p = 0; p < world; p++) {
        if (p == me) continue;
        if (g.len(me)) RPT_NCCL_IN_GROUP(api.send(bf->words + g.lo(me), g.len(me), kNcclUint64, p, nccl_comm, s));
        if (g.len(p)) RPT_NCCL_IN_GROUP(api.recv(bf->words + g.lo(p), g.len(p), kNcclUint64, p, nccl_comm, s));
      }
      RPT_NCCL_MERGE(api.group_end());
    }
    hipLaunchKernelGGL(minmax_pack_kernel, dim3(1), dim3(1), 0, s, bf->stats, bf->has_data.load(), v);
    RPT_LAUNCHED("minmax_pack_kernel");
    posted = true;
    RPT_NCCL_MERGE(api.all_reduce(v, v, 3, kNcclInt64, kNcclMin, nccl_comm, s));
    hipLaunchKernelGGL(minmax_unpack_kernel, dim3(1), dim3(1), 0, s, v, bf->stats, reinterpret_cast<int*>(v + 3));
    RPT_LAUNCHED("minmax_unpack_kernel");
    // bounded wait for everything enqueued above (never a blind hipStreamSynchronize: see poll_streams)
    std::string why;
    const int ws = poll_streams(&api, nccl_comm, {s}, deadline, &why);
    if (ws != RPT_OK) return fail(ws, "OR all-reduce (rank %d of %d): %s", me, world, why.c_str());
    int has = 0;
    RPT_HIP(hipMemcpyAsync(&has, v + 3, sizeof(int), hipMemcpyDeviceToHost, s));  // s is idle: returns at once
    RPT_HIP(hipStreamSynchronize(s));
    bf->has_data.store(has ? 1 : 0);
    return RPT_OK;
  };
  int st = run();
  const std::string err = t_last_error;
  bool drained = true;
  if (st != RPT_OK && posted && g_abort_on_error.load()) {
    // peers may be blocked on this rank, or this rank on a dead peer: the communicator cannot be reused.
    // Abort it (RCCL's kernels on s leave), then drain s and the helper stream, bounded again, so the
    // workspace is free on return. The distinct status tells a caller that owns the communicator that it
    // is gone (ncclCommAbort freed it: never destroy or use it again).
    abort_comm(api, nccl_comm);
    (void)join_helper();
    std::string why;
    drained = poll_streams(nullptr, nullptr, {s}, coll_deadline(), &why) == RPT_OK &&
              (!h || poll_streams(nullptr, nullptr, {h->s}, coll_deadline(), &why) == RPT_OK);
    t_merge_stuck = !drained;
    t_last_error = err + "; communicator aborted" +
                   (drained ? "" : "; streams did not drain (" + why + "): the workspace is still in use");
    st = RPT_ERR_COMM_ABORTED;
  } else if (st != RPT_OK && posted) {
    // rpt_collective_set_abort_on_error(0): the communicator stays its owner's to abort. RCCL's kernels may
    // still hold `stream` (a dead peer): until the owner aborts the communicator, the stream, the helper
    // stream and the workspace stay in use, so none of them is released here.
    (void)join_helper();
    drained = hipStreamQuery(s) == hipSuccess && (!h || hipStreamQuery(h->s) == hipSuccess);
    t_merge_stuck = !drained;
    t_last_error = err + "; communicator NOT aborted (rpt_collective_set_abort_on_error(0))" +
                   (drained ? "" : ": the streams are still blocked; abort the communicator (ncclCommAbort) "
                                   "before reusing the stream, the workspace or the filter");
  } else if (h) {
    // on an error before any collective call the helper may still hold OR kernels: the caller's stream
    // waits for them, so the workspace is free once `stream` is
    if (join_helper() != hipSuccess) (void)hipStreamSynchronize(h->s);
  }
  if (h && drained) give_helper(h);  // a helper stream that did not drain is leaked, never reused
  order.done(false);
  return st;
}

int rpt_collective_set_timeout_ms(uint64_t ms) {
  if (ms == 0) return fail(RPT_ERR_INVALID_ARGUMENT, "collective timeout of 0 ms");
  g_coll_timeout_ms.store(ms);
  return RPT_OK;
}

uint64_t rpt_collective_timeout_ms(void) { return g_coll_timeout_ms.load(); }

int rpt_collective_set_abort_on_error(int abort_on_error) {
  g_abort_on_error.store(abort_on_error ? 1 : 0);
  return RPT_OK;
}

int rpt_collective_abort_on_error(void) { return g_abort_on_error.load(); }

int rpt_bf_allreduce_or(rpt_bf* bf, void* nccl_comm, rpt_stream_t stream) {
  if (!bf || !nccl_comm) return fail(RPT_ERR_INVALID_ARGUMENT, "null argument");
  int world = 1;
  {
    const std::shared_ptr<const RcclApi> api_p = rccl_api();
    const rpt_rccl_api_table& api = api_p->fn;
    if (!api_p->load_error.empty()) return fail(RPT_ERR_COLLECTIVE, "RCCL unavailable: %s", api_p->load_error.c_str());
    RPT_NCCL(api.comm_count(nccl_comm, &world));
  }
  RPT_ON_DEVICE(bf->device);
  const size_t bytes = MergeGeom{1ULL << bf->log_num_blocks, world}.workspace_bytes();
  void* ws = nullptr;
  if (hipMalloc(&ws, bytes) != hipSuccess) {
    (void)hipGetLastError();
    return fail(RPT_ERR_OUT_OF_MEMORY, "all-reduce workspace of %zu bytes", bytes);
  }
  const int st = rpt_bf_allreduce_or_ws(bf, nccl_comm, ws, bytes, stream);
  if (t_merge_stuck) return st;  // aborted and still not drained: the workspace is leaked, never freed in use
  (void)hipStreamSynchronize(as_stream(stream));  // nothing may still use the workspace
  (void)hipFree(ws);
  return st;
}

int rpt_rccl_available(int device) {
  const std::shared_ptr<const RcclApi> api_p = rccl_api();
  if (!api_p->load_error.empty()) return fail(RPT_ERR_COLLECTIVE, "RCCL unavailable: %s", api_p->load_error.c_str());
  RPT_ON_DEVICE(device);
  return RPT_OK;
}

int rpt_rccl_get_unique_id(uint8_t* out_id) {
  if (!out_id) return fail(RPT_ERR_INVALID_ARGUMENT, "null argument");
  const std::shared_ptr<const RcclApi> api_p = rccl_api();
  const rpt_rccl_api_table& api = api_p->fn;
  if (!api_p->load_error.empty()) return fail(RPT_ERR_COLLECTIVE, "RCCL unavailable: %s", api_p->load_error.c_str());
  rpt_rccl_unique_id id{};
  RPT_NCCL(api.get_unique_id(&id));
  std::memcpy(out_id, id.internal, RPT_RCCL_UNIQUE_ID_BYTES);
  return RPT_OK;
}

int rpt_rccl_comm_init_rank(int device, int world, const uint8_t* id, int rank, void** out_comm) {
  if (!id || !out_comm || world < 1 || rank < 0 || rank >= world)
    return fail(RPT_ERR_INVALID_ARGUMENT, "bad communicator arguments (world %d, rank %d)", world, rank);
  const std::shared_ptr<const RcclApi> api_p = rccl_api();
  const rpt_rccl_api_table& api = api_p->fn;
  if (!api_p->load_error.empty()) return fail(RPT_ERR_COLLECTIVE, "RCCL unavailable: %s", api_p->load_error.c_str());
  RPT_ON_DEVICE(device);
  rpt_rccl_unique_id uid{};
  std::memcpy(uid.internal, id, RPT_RCCL_UNIQUE_ID_BYTES);
  void* comm = nullptr;
  RPT_NCCL(api.comm_init_rank(&comm, world, uid, rank));
  note_made(comm, false);  // (a new communicator at an aborted one's address is live)
  *out_comm = comm;
  return RPT_OK;
}

int rpt_rccl_comm_init_rank_nonblocking(int device, int world, const uint8_t* id, int rank, void** out_comm) {
  if (!id || !out_comm || world < 1 || rank < 0 || rank >= world)
    return fail(RPT_ERR_INVALID_ARGUMENT, "bad communicator arguments (world %d, rank %d)", world, rank);
  const std::shared_ptr<const RcclApi> api_p = rccl_api();
  const rpt_rccl_api_table& api = api_p->fn;
  if (!api_p->load_error.empty()) return fail(RPT_ERR_COLLECTIVE, "RCCL unavailable: %s", api_p->load_error.c_str());
  RPT_ON_DEVICE(device);
  rpt_rccl_unique_id uid{};
  std::memcpy(uid.internal, id, RPT_RCCL_UNIQUE_ID_BYTES);
  ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
  cfg.blocking = 0;  // every call may return ncclInProgress; the merge polls it against its deadline
  void* comm = nullptr;
  int rc = api.comm_init_rank_config(&comm, world, uid, rank, &cfg);
  if (rc == kNcclInProgress && comm) rc = settle_nccl(api, comm, rc, coll_deadline());
  if (rc != 0) {
    if (comm) (void)api.comm_abort(comm);  // never handed out: nothing to record
    return fail(RPT_ERR_COLLECTIVE, "ncclCommInitRankConfig (non-blocking): %s",
                rc == kNcclInProgress ? "no completion within the collective timeout" : api.error_string(rc));
  }
  note_made(comm, true);
  *out_comm = comm;
  return RPT_OK;
}

int rpt_rccl_comm_destroy(void* comm) {
  if (!comm) return RPT_OK;
  const bool aborted = take_aborted(comm);
  const std::pair<bool, bool> made = forget_made(comm);
  if (aborted) return RPT_OK;  // a failed merge aborted it: ncclCommAbort already freed it
  const std::shared_ptr<const RcclApi> api_p = rccl_api();
  const rpt_rccl_api_table& api = api_p->fn;
  if (!api_p->load_error.empty()) return fail(RPT_ERR_COLLECTIVE, "RCCL unavailable: %s", api_p->load_error.c_str());
  if (made.second) {
    // non-blocking: ncclCommDestroy would return ncclInProgress and tear down in the background,
    // so the caller could exit or reuse the device under it. Finalize first and poll it to completion, bounded
    // by the collective timeout; a finalize that does not complete (or a library without ncclCommFinalize)
    // ends in an abort, which tears down synchronously.
    int rc = api.comm_finalize ? settle_nccl(api, comm, api.comm_finalize(comm), coll_deadline()) : kNcclInProgress;
    if (rc != 0) {
      (void)api.comm_abort(comm);
      if (api.comm_finalize)
        return fail(RPT_ERR_COLLECTIVE, "ncclCommFinalize: %s; communicator aborted",
                    rc == kNcclInProgress ? "no completion within the collective timeout" : api.error_string(rc));
      return RPT_OK;
    }
  }
  const int rc = api.comm_destroy(comm);
  if (rc != 0 && !(made.second && rc == kNcclInProgress))
    return fail(RPT_ERR_COLLECTIVE, "ncclCommDestroy: %s", api.error_string(rc));
  return RPT_OK;
}
#undef RPT_NCCL_IN_GROUP
#undef RPT_NCCL_MERGE
#undef RPT_NCCL

#ifdef RPT_TESTING_HOOKS
// Test build only (rpt_gpu_testing.h): the product library has no such entry point.
int rpt_testing_set_rccl_api(const rpt_rccl_api_table* table) {
  std::shared_ptr<const RcclApi> a;
  if (table) {
    const void* const* e = reinterpret_cast<const void* const*>(table);
    for (size_t i = 0; i < sizeof(rpt_rccl_api_table) / sizeof(void*); i++)
      if (!e[i]) return fail(RPT_ERR_INVALID_ARGUMENT, "RCCL table entry %zu is null", i);
    auto t = std::make_shared<RcclApi>();
    t->fn = *table;
    a = std::move(t);
  }
  std::lock_guard<std::mutex> lk(g_rccl_mu);
  g_rccl = std::move(a);  // null: rccl_api() returns to librccl
  return RPT_OK;
}
uint64_t rpt_testing_bucketed_insert_batch(void) { return kBucketedInsertBatch; }
void rpt_testing_force_l1_error(int on) { g_force_l1_error.store(on != 0); }
#endif  // RPT_TESTING_HOOKS

int rpt_bf_count_bits(const rpt_bf* bf, uint64_t* out) {
  if (!bf || !out) return fail(RPT_ERR_INVALID_ARGUMENT, "null argument");
  RPT_ON_DEVICE(bf->device);
  RPT_SETTLE(bf, nullptr);
  unsigned long long* d = nullptr;
  RPT_HIP(hipMalloc(&d, sizeof(unsigned long long)));
  hipError_t e = hipMemset(d, 0, sizeof(unsigned long long));
  const uint64_t nw = 1ULL << bf->log_num_blocks;
  const unsigned grid = static_cast<unsigned>(std::max<uint64_t>(1, std::min<uint64_t>(ceil_div(nw, rpt::kBlockThreads), 4096)));
  if (e == hipSuccess) {
    hipLaunchKernelGGL(rpt::popcount_kernel, dim3(grid), dim3(rpt::kBlockThreads), 0, nullptr, bf->words, nw, d);
    e = hipGetLastError();
  }
  unsigned long long h = 0;
  if (e == hipSuccess) e = hipMemcpy(&h, d, sizeof h, hipMemcpyDeviceToHost);
  (void)hipFree(d);
  if (e != hipSuccess) return fail(RPT_ERR_HIP, "count_bits: %s", hipGetErrorString(e));
  *out = h;
  return RPT_OK;
}

int rpt_bf_is_same_as(const rpt_bf* a, const rpt_bf* b, int* out_same, uint64_t* out_diff_words) {
  if (!a || !b || !out_same) return fail(RPT_ERR_INVALID_ARGUMENT, "null argument");
  *out_same = 0;
  if (out_diff_words) *out_diff_words = 0;
  if (a->device != b->device) return fail(RPT_ERR_SHAPE_MISMATCH, "filters on devices %d and %d", a->device, b->device);
  if (a->log_num_blocks != b->log_num_blocks) {  // Arrow IsSameAs: different geometry is simply not the same
    if (out_diff_words) *out_diff_words = ~0ULL;
    return RPT_OK;
  }
  RPT_ON_DEVICE(a->device);
  RPT_SETTLE(a, nullptr);
  RPT_SETTLE(b, nullptr);
  RPT_HIP(hipDeviceSynchronize());  // every stream's writes to either filter have landed
  unsigned long long* d = nullptr;
  RPT_HIP(hipMalloc(&d, sizeof(unsigned long long)));
  hipError_t e = hipMemset(d, 0, sizeof(unsigned long long));
  const uint64_t nw = 1ULL << a->log_num_blocks;
  const unsigned grid =
      static_cast<unsigned>(std::max<uint64_t>(1, std::min<uint64_t>(ceil_div(nw / 2, rpt::kBlockThreads),
                                                                      static_cast<uint64_t>(num_cus(a->device)) * rpt::kBlocksPerCU)));
  if (e == hipSuccess) {
    hipLaunchKernelGGL(rpt::diff_count_kernel, dim3(grid), dim3(rpt::kBlockThreads), 0, nullptr, a->words, b->words, nw, d);
    e = hipGetLastError();
  }
  unsigned long long h = 0;
  if (e == hipSuccess) e = hipMemcpy(&h, d, sizeof h, hipMemcpyDeviceToHost);
  (void)hipFree(d);
  if (e != hipSuccess) return fail(RPT_ERR_HIP, "is_same_as: %s", hipGetErrorString(e));
  *out_same = h == 0;
  if (out_diff_words) *out_diff_words = h;
  return RPT_OK;
}

int rpt_bf_fold(rpt_bf* bf, int* out_new_log_num_blocks) {
  if (!bf) return fail(RPT_ERR_INVALID_ARGUMENT, "null filter");
  RPT_ON_DEVICE(bf->device);
  RPT_SETTLE(bf, nullptr);
  RPT_HIP(hipDeviceSynchronize());
  {
    std::lock_guard<std::mutex> lk(bf->order_mu);
    bf->order_pending = false;  // the device is idle; fold writes synchronously below
    bf->pristine = false;
  }
  constexpr int kMinLog = 4;  // bloom_filter.h Fold: log_num_blocks_min
  for (;;) {
    if (bf->log_num_blocks <= kMinLog) break;
    uint64_t set = 0;
    int st = rpt_bf_count_bits(bf, &set);
    if (st != RPT_OK) return st;
    const uint64_t nb = 1ULL << bf->log_num_blocks;
    const uint64_t num_bits = nb * 64;
    if (4 * set >= num_bits) break;
    int folds = 1;
    while ((bf->log_num_blocks - folds) > kMinLog && (4 * set) < (num_bits >> folds)) ++folds;
    const uint64_t slice = nb >> folds;
    // target slice 0 accumulates slices 1 .. 2^folds-1 (they never overlap the target)
    const unsigned grid = static_cast<unsigned>(std::max<uint64_t>(1, std::min<uint64_t>(ceil_div(slice / 2, rpt::kBlockThreads), 8192)));
    ProfScope prof14_("or_slices_kernel(fold)", nullptr);
    hipLaunchKernelGGL(rpt::or_slices_kernel, dim3(grid), dim3(rpt::kBlockThreads), 0, nullptr, bf->words,
                       bf->words + slice, static_cast<uint32_t>((1u << folds) - 1), slice, slice, 1);
    prof14_.end();
    RPT_LAUNCHED("or_slices_kernel(fold)");
    RPT_HIP(hipDeviceSynchronize());
    bf->log_num_blocks -= folds;
  }
  if (out_new_log_num_blocks) *out_new_log_num_blocks = bf->log_num_blocks;
  return RPT_OK;
}

int rpt_bf_export_words(const rpt_bf* bf, uint64_t* host_words, uint64_t n_words) {
  if (!bf || !host_words) return fail(RPT_ERR_INVALID_ARGUMENT, "null argument");
  if (n_words != (1ULL << bf->log_num_blocks))
    return fail(RPT_ERR_SHAPE_MISMATCH, "export of %llu words from a %llu-word filter", (unsigned long long)n_words,
                (unsigned long long)(1ULL << bf->log_num_blocks));
  RPT_ON_DEVICE(bf->device);
  RPT_SETTLE(bf, nullptr);
  RPT_HIP(hipDeviceSynchronize());
  RPT_HIP(hipMemcpy(host_words, bf->words, n_words * 8, hipMemcpyDeviceToHost));
  return RPT_OK;
}

int rpt_bf_import_words(rpt_bf* bf, const uint64_t* host_words, uint64_t n_words) {
  if (!bf || !host_words) return fail(RPT_ERR_INVALID_ARGUMENT, "null argument");
  if (n_words != (1ULL << bf->log_num_blocks))
    return fail(RPT_ERR_SHAPE_MISMATCH, "import of %llu words into a %llu-word filter", (unsigned long long)n_words,
                (unsigned long long)(1ULL << bf->log_num_blocks));
  RPT_ON_DEVICE(bf->device);
  RPT_HIP(hipDeviceSynchronize());
  {
    std::lock_guard<std::mutex> lk(bf->order_mu);
    bf->order_pending = false;
    bf->pristine = false;
    bf->clear_pending.store(false);  // every word is overwritten
  }
  RPT_HIP(hipMemcpy(bf->words, host_words, n_words * 8, hipMemcpyHostToDevice));
  int any = 0;
  for (uint64_t i = 0; i < n_words && !any; i++) any = host_words[i] != 0;
  bf->has_data.store(any);
  return RPT_OK;
}

int rpt_bf_copy_words_to(const rpt_bf* bf, uint64_t* dst_dev, uint64_t n_words, rpt_stream_t stream) {
  if (!bf || !dst_dev) return fail(RPT_ERR_INVALID_ARGUMENT, "null argument");
  if (n_words != (1ULL << bf->log_num_blocks))
    return fail(RPT_ERR_SHAPE_MISMATCH, "copy of %llu words from a %llu-word filter", (unsigned long long)n_words,
                (unsigned long long)(1ULL << bf->log_num_blocks));
  RPT_ON_DEVICE(bf->device);
  RPT_SETTLE(bf, as_stream(stream));
  RPT_HIP(hipMemcpyAsync(dst_dev, bf->words, n_words * 8, hipMemcpyDeviceToDevice, as_stream(stream)));
  return RPT_OK;
}

int rpt_bf_copy_words_from(rpt_bf* bf, const uint64_t* src_dev, uint64_t n_words, rpt_stream_t stream) {
  if (!bf || !src_dev) return fail(RPT_ERR_INVALID_ARGUMENT, "null argument");
  if (n_words != (1ULL << bf->log_num_blocks))
    return fail(RPT_ERR_SHAPE_MISMATCH, "copy of %llu words into a %llu-word filter", (unsigned long long)n_words,
                (unsigned long long)(1ULL << bf->log_num_blocks));
  RPT_ON_DEVICE(bf->device);
  RPT_REFUSE_CAPTURE_WRITE(bf, as_stream(stream), "copy into the filter");
  WriteOrder order(bf, as_stream(stream));
  RPT_REFUSE_IN_FLIGHT(order, "write");
  const hipError_t e = hipMemcpyAsync(bf->words, src_dev, n_words * 8, hipMemcpyDeviceToDevice, as_stream(stream));
  if (e == hipSuccess) bf->clear_pending.store(false);  // every word is overwritten
  order.done(false);
  if (e != hipSuccess) return fail(RPT_ERR_HIP, "hipMemcpyAsync failed: %s", hipGetErrorString(e));
  return RPT_OK;
}


int rpt_profiling_enable(int enable) {
  g_prof_enabled.store(enable ? 1 : 0);
  return RPT_OK;
}

int rpt_profiling_reset(void) {
  std::lock_guard<std::mutex> lk(g_prof_mu);
  for (auto& r : g_prof_pending) {
    (void)hipEventSynchronize(r.end);
    g_prof_free.push_back(r.start);
    g_prof_free.push_back(r.end);
  }
  g_prof_pending.clear();
  g_prof_stats.clear();
  return RPT_OK;
}

int rpt_profiling_read(rpt_kernel_stat* out, int capacity) {
  std::lock_guard<std::mutex> lk(g_prof_mu);
  for (auto& r : g_prof_pending) {
    float ms = 0.f;
    if (hipEventSynchronize(r.end) != hipSuccess || hipEventElapsedTime(&ms, r.start, r.end) != hipSuccess)
      return -fail(RPT_ERR_HIP, "profiling: event query failed");
    auto it = std::find_if(g_prof_stats.begin(), g_prof_stats.end(), [&](const auto& p) { return p.first == r.name; });
    if (it == g_prof_stats.end()) {
      g_prof_stats.push_back({std::string(r.name), ProfStat{}});
      it = g_prof_stats.end() - 1;
    }
    it->second.launches++;
    it->second.total_ms += ms;
    g_prof_free.push_back(r.start);
    g_prof_free.push_back(r.end);
  }
  g_prof_pending.clear();
  const int n = static_cast<int>(g_prof_stats.size());
  for (int i = 0; i < n && i < capacity && out; i++) {
    memset(out[i].name, 0, sizeof out[i].name);
    strncpy(out[i].name, g_prof_stats[i].first.c_str(), sizeof out[i].name - 1);
    out[i].launches = g_prof_stats[i].second.launches;
    out[i].total_ms = g_prof_stats[i].second.total_ms;
  }
  return n;
}

// ---- bench / test workload generators (include/rpt_gpu_synth.h) ---------------------------------
int rpt_synth_build_keys(int64_t* out, uint64_t start, uint64_t n, rpt_stream_t stream) {
  if (!out) return fail(RPT_ERR_INVALID_ARGUMENT, "null out");
  if (n == 0) return RPT_OK;
  const unsigned grid = static_cast<unsigned>(std::min<uint64_t>(ceil_div(n, rpt::kBlockThreads), 8192));
  ProfScope prof15_("synth_build_kernel", as_stream(stream));
  hipLaunchKernelGGL(rpt::synth_build_kernel, dim3(grid), dim3(rpt::kBlockThreads), 0, as_stream(stream), out, start, n);
  prof15_.end();
  RPT_LAUNCHED("synth_build_kernel");
  return RPT_OK;
}

int rpt_synth_probe_keys(int64_t* out, uint64_t n_build, uint32_t p_permille, uint64_t start, uint64_t n,
                         rpt_stream_t stream) {
  if (!out) return fail(RPT_ERR_INVALID_ARGUMENT, "null out");
  if (p_permille > 1000) return fail(RPT_ERR_INVALID_ARGUMENT, "p_permille %u > 1000", p_permille);
  if (n == 0) return RPT_OK;
  const unsigned grid = static_cast<unsigned>(std::min<uint64_t>(ceil_div(n, rpt::kBlockThreads), 8192));
  ProfScope prof16_("synth_probe_kernel", as_stream(stream));
  hipLaunchKernelGGL(rpt::synth_probe_kernel, dim3(grid), dim3(rpt::kBlockThreads), 0, as_stream(stream), out, n_build,
                     p_permille, start, n);
  prof16_.end();
  RPT_LAUNCHED("synth_probe_kernel");
  return RPT_OK;
}

uint64_t rpt_stream_sink_words(int device) { return static_cast<uint64_t>(num_cus(device)) * rpt::kStreamBlocksPerCU; }

static int stream_check(const void* p, uint64_t bytes, int* dev) {
  if (!p) return fail(RPT_ERR_INVALID_ARGUMENT, "null pointer");
  if ((reinterpret_cast<uintptr_t>(p) & 15) || (bytes & 15))
    return fail(RPT_ERR_INVALID_ARGUMENT, "stream calibration needs 16-B aligned pointers and sizes");
  RPT_HIP(hipGetDevice(dev));
  return RPT_OK;
}

int rpt_stream_read(const void* src, uint64_t bytes, uint64_t* sink, rpt_stream_t stream) {
  int dev = 0;
  int st = stream_check(src, bytes, &dev);
  if (st != RPT_OK) return st;
  if (!sink) return fail(RPT_ERR_INVALID_ARGUMENT, "null sink");
  if (bytes == 0) return RPT_OK;
  ProfScope prof_("stream_read_kernel", as_stream(stream));
  hipLaunchKernelGGL(rpt::stream_read_kernel, dim3(static_cast<unsigned>(rpt_stream_sink_words(dev))),
                     dim3(rpt::kBlockThreads), 0, as_stream(stream), static_cast<const rpt::u64x2*>(src), bytes / 16, sink);
  prof_.end();
  RPT_LAUNCHED("stream_read_kernel");
  return RPT_OK;
}

int rpt_stream_copy(void* dst, const void* src, uint64_t bytes, rpt_stream_t stream) {
  int dev = 0;
  int st = stream_check(src, bytes, &dev);
  if (st == RPT_OK) st = stream_check(dst, bytes, &dev);
  if (st != RPT_OK) return st;
  if (bytes == 0) return RPT_OK;
  if (ceil_div(bytes / 16, rpt::kBlockThreads) > 0x7fffffffULL) return fail(RPT_ERR_INVALID_ARGUMENT, "copy too large");
  ProfScope prof_("stream_copy_kernel", as_stream(stream));
  hipLaunchKernelGGL(rpt::stream_copy_kernel, dim3(static_cast<unsigned>(ceil_div(bytes / 16, rpt::kBlockThreads))),
                     dim3(rpt::kBlockThreads), 0, as_stream(stream), static_cast<const rpt::u64x2*>(src), bytes / 16,
                     static_cast<rpt::u64x2*>(dst));
  prof_.end();
  RPT_LAUNCHED("stream_copy_kernel");
  return RPT_OK;
}

}  // extern "C"
