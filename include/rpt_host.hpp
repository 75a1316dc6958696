// rpt_host.hpp — C++ host mirror of the predicate-transfer hot path over librpt_gpu.so.
//
// What a DuckDB-side shim links against (C++17, no DuckDB types): the reference's PTBloomFilter
// (src/include/bloom_filter.hpp:22-57) and the hot-path logic of PhysicalCreateBF
// (src/operators/physical_create_bf.cpp:201-419) and PhysicalUseBF::ExecuteInternal
// (src/operators/physical_use_bf.cpp:60-198), operating on DuckDB-shaped key vectors. Errors are
// C++ exceptions (GpuError), as in the reference (DuckDB exceptions); nothing throws across the
// C-ABI underneath.
//
// Vectors are HOST-resident (DuckDB DataChunks live in host memory). Each call stages its rows
// to the device through pinned buffers on the caller's HIP stream; callers that own device-resident
// columns should use the C-ABI (rpt_gpu.h) directly. The *Batch entry points concatenate many
// 2048-row chunks into one device call, which is how the shim amortises PCIe latency.
#pragma once

#include <atomic>
#include <cstdint>
#include <functional>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "rpt_gpu.h"

namespace rpt {

class GpuError : public std::runtime_error {
 public:
  GpuError(int status, const std::string& what) : std::runtime_error(what), status_(status) {}
  int status() const { return status_; }

 private:
  int status_;
};

// DuckDB VectorType subset the hot path sees (HashColumns flattens CONSTANT, bloom_filter.cpp:19-21;
// VectorOperations::Hash reads the others through their unified format).
enum class VectorType { FLAT, CONSTANT, DICTIONARY, SEQUENCE };
// DuckDB physical key types. I32 (INTEGER, DATE) and I64 (BIGINT, TIMESTAMP) go to the device as they are.
// The others are converted while the column is staged, to the value DuckDB's Hash<T> hashes (restated, parity
// unpinned like the int32 rule): I8 / I16 (TINYINT, SMALLINT) sign-extended and U8 / U16 (UTINYINT,
// USMALLINT) zero-extended to I32 (Hash<T> casts to uint32_t); U32 (UINTEGER) zero-extended to I64 (same hash,
// and the key min/max stays exact); U64 (UBIGINT) as its bits; F32 / F64 (FLOAT, DOUBLE) as their bits after
// DuckDB's equality transform (-0.0 -> 0.0, every NaN -> the quiet NaN), F32's zero-extended like a uint32.
// The key min/max (MinMax) is exact for I8..U32 and not kept for U64 / F32 / F64 (their device values do not
// order like the keys): there the shim keeps the reference's host UpdateMinMax.
enum class KeyType { I32 = RPT_KEY_I32, I64 = RPT_KEY_I64, I8 = 16, I16, U8, U16, U32, U64, F32, F64 };

// One key column of a DataChunk.
//   FLAT:       data[row], validity indexed by row
//   CONSTANT:   data[0] for every row, validity bit 0 for every row
//   DICTIONARY: data[sel[row]] (dictionary of dict_size entries), validity indexed by sel[row]
//   SEQUENCE:   seq_start + row * seq_increment (DuckDB SEQUENCE_VECTOR, e.g. range() keys), never NULL;
//               no data pointer (INTEGER sequences wrap to int32 as DuckDB's do)
struct Vector {
  VectorType type = VectorType::FLAT;
  KeyType key_type = KeyType::I64;
  const void* data = nullptr;
  const uint32_t* sel = nullptr;       // DICTIONARY only
  uint64_t dict_size = 0;              // DICTIONARY only
  const uint64_t* validity = nullptr;  // DuckDB ValidityMask words; nullptr = all valid
  int64_t seq_start = 0;               // SEQUENCE only
  int64_t seq_increment = 1;           // SEQUENCE only
};

struct DataChunk {
  std::vector<Vector> data;
  uint64_t count = 0;  // <= 2048 in DuckDB; any size here
};

using SelectionVector = std::vector<uint32_t>;  // sel_t

// Pinned host staging of DeviceContexts that grow a slot or are destroyed goes to a process-wide cache (up to
// `bytes`, default 4 GiB) and is handed to the next context that needs that size, so per-query operator states
// do not pin fresh pages (hipHostMalloc) every query. ReleasePinnedCache frees what is cached now.
void SetPinnedCacheLimit(size_t bytes);
size_t PinnedCacheBytes();
void ReleasePinnedCache();

// Device stream + pinned/device staging owned by one host thread (DuckDB thread-local state).
class DeviceContext {
 public:
  explicit DeviceContext(int device);
  ~DeviceContext();
  DeviceContext(const DeviceContext&) = delete;
  DeviceContext& operator=(const DeviceContext&) = delete;
  int device() const { return device_; }
  void* stream() const { return stream_; }
  void synchronize();  // every stream

  // internal: grow-on-demand buffers (host slots 16..31: UseBF::Execute's chained key columns; 32..63: the
  // pipelined filter chain of UseBF::ExecuteBatch; 56..59 and 64..72: narrow BIGINT staging)
  static constexpr int kSlots = 80;
  void* host(int slot, size_t bytes);
  void* dev(int slot, size_t bytes);
  // the device address of host slot `slot`'s pinned buffer (kernels read / write it in place), cached
  // until the slot grows
  void* host_device_ptr(int slot);
  // internal: the device-to-host stream of pipelined batches, the host-to-device stream that feeds them
  // (created on first use), and their events
  void* copy_stream();
  void* h2d_stream();
  // internal: further compute streams (created on first use): the pipelined filter chain runs successive
  // stages' chains on stream() and these, so one stage's next filter never queues behind a later stage's copy
  static constexpr int kAuxStreams = 2;
  void* aux_stream(int i);
  static constexpr int kEvents = 16;
  void* event(int i);
  // internal: run fn(0) .. fn(n - 1) on this context's worker threads (flatten_threads of them, the caller
  // included; created on first use and kept, so a stage costs no thread start-up); rethrows the first
  // exception a task threw, after every task has finished.
  void parallel_for(size_t n, const std::function<void(size_t)>& fn);

  // Batches of at least 2 Mi rows (or 2 * pipeline_rows when that is smaller) are staged in stages of a quarter of
  // the batch, at least 512 Ki rows and at most pipeline_rows (whole chunks): flattening stage i+1 on the host
  // overlaps the copy of stage i, the probe of stage i-1 and the copy back of stage i-2's result.
  uint64_t pipeline_rows = 1ULL << 22;
  // Host threads (the calling one included) that flatten a batch or stage of >= 128 Ki rows into pinned
  // memory and split a stage's selection vector into per-chunk ones. DuckDB's operator threads each own a
  // DeviceContext, so with many of them 1-2 per context is enough.
  unsigned flatten_threads = 8;
  // Pipelined BIGINT batches whose chunks each share their keys' high 32 bits (ids below 2^32, or any 2^32-aligned
  // window) cross PCIe as 4-B low words and are widened on the device (rpt_keys_widen): half the bytes of the
  // shim's bound. A stage that does not qualify is flattened as 8-B keys and the rest of the batch stays plain.
  bool narrow_keys = true;
  // Pipelined lookups bring each stage's result bits back (rows / 8 bytes; rpt_bf_probe_bits) and the workers
  // expand them into the chunks' sels, instead of copying the survivors' sel (4 B each) after a count round trip.
  bool bits_back = true;

  // Host-side time of the pipelined batch paths by phase (accumulated; reset by assigning {}): where a
  // host-resident batch's time goes (tools/host_bench reports it).
  struct PipelineStats {
    uint64_t stages = 0, rows = 0;
    double flatten_s = 0;     // chunks -> pinned staging (worker threads)
    double enqueue_s = 0;     // copy / probe / insert launches
    double wait_copy_s = 0;   // waiting for a pinned buffer's previous copy to finish before refilling it
    double wait_count_s = 0;  // waiting for a stage's survivor count (probe done)
    double wait_sel_s = 0;    // waiting for a stage's selection vector to arrive on the host
    double split_s = 0;       // stage sel -> per-chunk sels (worker threads)
    uint64_t narrow_stages = 0;  // stages sent as narrow BIGINT keys
    double total_s = 0;
  };
  PipelineStats stats;

 private:
  int device_;
  void* stream_ = nullptr;
  void* copy_stream_ = nullptr;
  void* h2d_stream_ = nullptr;
  void* aux_streams_[kAuxStreams] = {};
  struct Buf {
    void* p = nullptr;
    size_t cap = 0;
    void* dp = nullptr;  // host slots: device address of p (0 until asked for)
  };
  Buf host_[kSlots], dev_[kSlots];
  void* events_[kEvents] = {};
  struct Pool;
  std::unique_ptr<Pool> pool_;
};

// One key column kept in HBM, one segment per staged batch: the device half of CREATE_BF's
// materialization (physical_create_bf.cpp:211-218; the full rows stay in host memory). Finalize's
// rehash (bloom_filter.cpp:34-58) re-inserts from these segments instead of re-staging every host
// chunk over PCIe.
class DeviceKeyColumn {
 public:
  struct Segment {
    rpt_key_column col;  // device keys (+ validity words when the batch had NULLs)
    uint64_t rows;
  };
  explicit DeviceKeyColumn(int device) : device_(device) {}
  ~DeviceKeyColumn();
  DeviceKeyColumn(DeviceKeyColumn&& o) noexcept;
  DeviceKeyColumn& operator=(DeviceKeyColumn&& o) noexcept;
  DeviceKeyColumn(const DeviceKeyColumn&) = delete;
  DeviceKeyColumn& operator=(const DeviceKeyColumn&) = delete;

  // Flatten column `col` of `chunks` (FLAT / CONSTANT / DICTIONARY) into a new device segment, through the
  // context's pinned slots `slot` / `slot + 1`; the copy is enqueued on the context's stream (it has not
  // necessarily finished when Append returns: synchronize before reusing those slots).
  const Segment& Append(DeviceContext& ctx, const std::vector<const DataChunk*>& chunks, uint64_t col, int slot = 0);
  // Take over `other`'s segments (CREATE_BF Combine).
  void Splice(DeviceKeyColumn&& other);
  const std::vector<Segment>& segments() const { return segs_; }
  uint64_t rows() const;

 private:
  void release();
  int device_;
  std::vector<Segment> segs_;
};

// PTBloomFilter (bloom_filter.hpp:22-57) with the filter on the device.
class PTBloomFilter {
 public:
  PTBloomFilter() = default;
  ~PTBloomFilter();
  PTBloomFilter(const PTBloomFilter&) = delete;
  PTBloomFilter& operator=(const PTBloomFilter&) = delete;

  // bloom_filter.cpp:27-32 (est_num_rows is uint32 as in physical_create_bf.cpp:187)
  void Initialize(int device, uint32_t est_num_rows);
  // bloom_filter.cpp:70-78: thread-safe (device atomic OR); no-op on an empty chunk. Several `cols`
  // form a composite key (HashColumns' CombineHash, bloom_filter.cpp:15-17), as in LookupSel.
  void Insert(DeviceContext& ctx, const DataChunk& chunk, const std::vector<uint64_t>& cols);
  void InsertBatch(DeviceContext& ctx, const std::vector<const DataChunk*>& chunks, const std::vector<uint64_t>& cols);
  // bloom_filter.cpp:60-68: ascending surviving row ids; returns the count
  uint64_t LookupSel(DeviceContext& ctx, const DataChunk& chunk, SelectionVector& sel,
                     const std::vector<uint64_t>& cols) const;
  // many chunks in one device call (pipelined in stages for large single-column batches, see
  // DeviceContext::pipeline_rows); sels[i] holds chunk i's survivors (ids relative to chunk i)
  void LookupSelBatch(DeviceContext& ctx, const std::vector<const DataChunk*>& chunks,
                      std::vector<SelectionVector>& sels, const std::vector<uint64_t>& cols) const;
  // Insert a device-resident key column (large batches take the routed inserts; same bits). synchronize =
  // false: the insert is only enqueued on the context's stream (col and the context's workspace slot 6 stay in
  // use until the caller synchronizes).
  void InsertDevice(DeviceContext& ctx, const rpt_key_column& col, uint64_t n, bool synchronize = true);
  // bloom_filter.cpp:34-58: reallocate for actual_rows and re-insert the materialized chunks
  void ReinitializeAndRehash(DeviceContext& ctx, uint64_t actual_rows, const std::vector<DataChunk>& data,
                             const std::vector<uint64_t>& cols);
  // ... or re-insert a key column already in HBM (no PCIe traffic); NULL-free segments are inserted in groups
  // of up to kRehashGroupRows rows, copied back to back into one device buffer (context slot 7)
  void ReinitializeAndRehash(DeviceContext& ctx, uint64_t actual_rows, const DeviceKeyColumn& keys);
  static constexpr uint64_t kRehashGroupRows = 1ULL << 27;

  uint64_t SizedForRows() const;
  // Finalize's resize predicate on this filter's real allocation (rpt_bf_needs_resize_alloc)
  bool NeedsResize(uint64_t actual_rows) const;
  bool IsEmpty() const;
  int LogNumBlocks() const;
  // Min/max of the valid keys inserted (the min/max dynamic filter), as int64 (I8..U32 values exactly);
  // false: none yet, or a U64 / F32 / F64 column was inserted (KeyType).
  bool MinMax(int64_t& min_value, int64_t& max_value) const;
  // A host column of this type is inserted (Insert / InsertBatch / CreateBF note it themselves; callers that
  // stage their own device columns from such keys call it).
  void NoteKeyType(KeyType t);
  std::vector<uint64_t> ExportWords() const;
  // Multi-GPU Combine: OR all-reduce of every rank's partial filter over an RCCL communicator
  // (ncclComm_t, one rank per GPU; collective: every rank calls it). rpt_bf_allreduce_or.
  void AllReduceOr(DeviceContext& ctx, void* nccl_comm);
  rpt_bf* native() const { return bf_; }

  bool finalized_ = false;

 private:
  struct PipelineBuffers;
  void InsertPipelined(DeviceContext& ctx, const std::vector<const DataChunk*>& chunks, uint64_t col);
  void LookupSelPipelined(DeviceContext& ctx, const std::vector<const DataChunk*>& chunks,
                          std::vector<SelectionVector>& sels, uint64_t col) const;
  void LookupSelMapped(DeviceContext& ctx, const std::vector<const DataChunk*>& chunks,
                       std::vector<SelectionVector>& sels, uint64_t col, uint64_t total) const;
  rpt_bf* bf_ = nullptr;
  std::atomic<bool> minmax_kept_{true};  // no U64 / F32 / F64 column inserted since Initialize
};

// The hot-path part of PhysicalCreateBF: parallel Sink (materialize + insert), Combine, Finalize
// (resize rule + rehash, finalized_), one filter per build column (bloom_filter_map,
// physical_create_bf.hpp:73), and the parallel source that re-emits the materialized chunks
// (physical_create_bf.cpp:441-557).
//
// Sink materializes every column of the chunk on the host (the reference's local
// ColumnDataCollection, physical_create_bf.cpp:211-218) and stages the build columns to the device
// in batches of `sink_flush_rows` rows (one PCIe transfer + one insert per batch instead of one per
// 2048-row chunk; the filters are only read after Finalize, so deferring the inserts is unobservable).
// The staged key columns stay in HBM (DeviceKeyColumn), so Finalize's rehash never re-reads the host.
class CreateBF {
 public:
  static constexpr uint64_t kDefaultSinkFlushRows = 1ULL << 22;

  struct LocalState {
    LocalState(int device, size_t n_cols) : ctx(device) {
      for (size_t i = 0; i < n_cols; i++) keys.emplace_back(device);
    }
    DeviceContext ctx;
    std::vector<DataChunk> chunks;                      // materialized chunks (views of owned storage)
    std::vector<std::unique_ptr<uint64_t[]>> storage;   // owned blocks backing `chunks` (bump-allocated)
    uint64_t* arena = nullptr;                          // the current block's free words
    size_t arena_left = 0;
    std::vector<DeviceKeyColumn> keys;                  // build columns already staged to HBM
    size_t pending_from = 0;                            // chunks[pending_from..] not yet inserted
    uint64_t pending_rows = 0;
    uint64_t flushes = 0;
    // A flush's copy and insert overlap the next chunks' materialization (two pinned buffers per build column,
    // up to kAsyncFlushColumns columns); false: every flush waits for its insert.
    bool async_flush = true;
    double materialize_s = 0, flush_s = 0;  // host time in Sink's materialization / in the flushes
  };
  static constexpr size_t kAsyncFlushColumns = 12;
  static constexpr size_t kSinkBlockWords = size_t(1) << 17;  // materialization blocks of 1 MiB
  // CreateBFGlobalSourceState (physical_create_bf.cpp:441-485): chunk ranges, one per source thread
  struct GlobalSourceState {
    std::vector<std::pair<size_t, size_t>> chunks_todo;
    std::atomic<size_t> partition_id{0};
  };
  struct LocalSourceState {
    bool initial = true;
    size_t chunk_from = 0, chunk_to = 0, current = 0;
  };

  // Finalize's resize predicate (physical_create_bf.cpp:383-398). kOnAllocation (default): the stated
  // intent "< 8 bits per actual row" on the filter actually allocated (Arrow sizing, 8 bits per estimated
  // row: rpt_bf_needs_resize_alloc). kReferenceFormula: the reference's formula verbatim, which prices the
  // allocation as DuckDB's native filter would (NextPow2(max(512, 12 * sized_for)): rpt_bf_needs_resize);
  // on this filter it keeps e.g. 2048 rows in a filter sized for 1000 (4 bits per key) where the default
  // resizes. Results differ from the reference's only in which of the two rules decides.
  enum class ResizeRule { kOnAllocation, kReferenceFormula };
  CreateBF(int device, uint64_t estimated_cardinality, std::vector<uint64_t> bound_column_indices,
           uint64_t sink_flush_rows = kDefaultSinkFlushRows, ResizeRule resize_rule = ResizeRule::kOnAllocation);
  std::unique_ptr<LocalState> MakeLocalState() const { return std::make_unique<LocalState>(device_, cols_.size()); }
  void Sink(LocalState& local, const DataChunk& chunk) const;  // physical_create_bf.cpp:201-242
  void Combine(LocalState& local);                             // physical_create_bf.cpp:244-275
  void Finalize();                                             // physical_create_bf.cpp:352-419
  std::shared_ptr<PTBloomFilter> GetBloomFilter(size_t build_column) const { return filters_.at(build_column); }
  uint64_t MaterializedRows() const { return total_rows_; }
  size_t ChunkCount() const { return all_chunks_.size(); }
  bool Resized(size_t build_column) const { return resized_.at(build_column); }
  // The build column's keys in HBM (after Combine): a device-side consumer can read them directly.
  const DeviceKeyColumn& DeviceKeys(size_t build_column) const { return all_keys_.at(build_column); }
  // Rows whose sink-time insert was skipped because the rows flushed so far already make Finalize resize the
  // filter (the resize rule is monotone in the row count), so Finalize's rehash from HBM inserts them instead;
  // the finalized filter is the same either way.
  uint64_t SkippedInsertRows() const { return skipped_insert_rows_.load(); }
  // CreateBFGlobalSinkState::column_min_max[i] (physical_create_bf.cpp:229-272): min / max of the
  // valid keys of build column i, computed by the insert kernels; false when no valid key was seen.
  bool MinMax(size_t build_column, int64_t& min_value, int64_t& max_value) const;
  // The parallel source (physical_create_bf.cpp:453-557): ceil(chunks / num_threads) chunks per
  // range; each LocalSourceState claims one range and walks it. GetData returns false when its range
  // is done (SourceResultType::FINISHED); `chunk` is a view of the materialized chunk.
  std::unique_ptr<GlobalSourceState> GetGlobalSourceState(size_t num_threads) const;
  bool GetData(GlobalSourceState& global, LocalSourceState& local, DataChunk& chunk) const;

 private:
  void Flush(LocalState& local) const;  // stage + insert the pending chunks' build columns
  bool WillResize(size_t build_column, uint64_t actual_rows) const;  // Finalize's resize predicate

  int device_;
  uint64_t estimated_cardinality_;
  ResizeRule resize_rule_;
  std::vector<uint64_t> cols_;
  uint64_t sink_flush_rows_;
  std::vector<std::shared_ptr<PTBloomFilter>> filters_;
  std::vector<bool> resized_;
  std::mutex lock_;
  std::vector<DataChunk> all_chunks_;
  std::vector<std::unique_ptr<uint64_t[]>> all_storage_;
  std::vector<DeviceKeyColumn> all_keys_;
  uint64_t total_rows_ = 0;
  mutable std::atomic<uint64_t> flushed_rows_{0};        // rows handed to Flush by every sink state so far
  mutable std::atomic<uint64_t> skipped_insert_rows_{0};
};

// Where a CREATE_BF's filter is applied: the reference's forward pass pushes its filter into the
// probe table's scan (PhysicalCreateBF::Finalize -> PushDynamicFilters, physical_create_bf.cpp:282-350: a
// BFTableFilter wrapped in SelectivityOptionalFilter(.., 1, 1000000), min/max ConstantFilters, always-false for an
// empty build) and marks that forward USE_BF passthrough (SetupDynamicFilterPushdown, rpt_optimizer.cpp:1493-1494),
// so those probes run inside DuckDB's CPU scan. The GPU mode (the `rpt_device` setting) keeps the BF
// probe in USE_BF, on the device, and pushes only the cheap scan filters. A DuckDB shim calls PlanPushdown in
// SetupDynamicFilterPushdown (to decide is_passthrough) and in PushDynamicFilters (to decide what to push).
enum class FilterType { kAll, kBfOnly, kMinMaxOnly };  // rpt_filter_type ('all' | 'bf_only' | 'minmax_only')
enum class Device { kCpu, kGpu };                       // rpt_device ('cpu' = the reference | 'gpu')
struct PushdownPlan {
  bool use_bf_passthrough = false;  // the USE_BF operator references its input unchanged (physical_use_bf.cpp:62-66)
  bool push_always_false = false;   // empty build side: every target scan gets `col > MAX` (cpp:288-297)
  bool push_bf = false;             // BFTableFilter into the target scans (cpp:321-333)
  bool push_minmax = false;         // `col >= min` and `col <= max` into the target scans (cpp:335-345)
  bool bf_probed_in_use_bf = true;  // the BF probe runs in USE_BF (rpt::UseBF): false when the scan runs it, or
                                    // when nothing probes it (minmax_only drops the forward BF, as the reference)
};
// is_forward_pass / has_targets: the CREATE_BF's pass and whether SetupDynamicFilterPushdown found scan targets for
// it; build_rows == 0: the build side was empty; bf_empty: the filter holds no key (IsEmpty); has_minmax: the build
// column kept a min/max (CreateBF::MinMax).
PushdownPlan PlanPushdown(Device device, FilterType filter_type, bool is_forward_pass, bool has_targets,
                          uint64_t build_rows, bool bf_empty, bool has_minmax);

// PhysicalUseBF::ExecuteInternal (physical_use_bf.cpp:60-198): AND of the filters over the chunk,
// in filter order, with its early exits (empty filter -> 0 rows, 0 survivors -> stop) and skips
// (filter not finalized). Returns the surviving row ids of the input chunk (ascending). A chunk of at
// most RPT_SMALL_PROBE_ROWS rows whose applicable filters number 1..RPT_MAX_CHAIN runs the whole chain
// as one launch (rpt_bf_probe_chain, one sync); otherwise filter by filter.
class UseBF {
 public:
  UseBF(std::vector<std::shared_ptr<PTBloomFilter>> filters, std::vector<uint64_t> bound_column_indices,
        bool passthrough = false);
  uint64_t Execute(DeviceContext& ctx, const DataChunk& input, SelectionVector& out) const;
  // The same filter chain over many chunks at once (a caching USE_BF): each filter probes the whole
  // batch's surviving rows in one device call (the survivors stay on the device between filters);
  // outs[i] == Execute(inputs[i]). Returns the batch's surviving rows.
  uint64_t ExecuteBatch(DeviceContext& ctx, const std::vector<const DataChunk*>& inputs,
                        std::vector<SelectionVector>& outs) const;
  uint64_t rows_in() const { return rows_in_; }
  uint64_t rows_out() const { return rows_out_; }

 private:
  // ExecuteBatch for 2+ applicable filters over a large batch: the first filter's column goes through
  // LookupSelBatch's pipeline; each further filter gets only the previous one's survivors (their keys gathered on
  // the host), and successive stages overlap.
  uint64_t ExecuteChainPipelined(DeviceContext& ctx, const std::vector<const DataChunk*>& inputs,
                                 std::vector<SelectionVector>& outs, const std::vector<size_t>& act) const;
  std::vector<std::shared_ptr<PTBloomFilter>> filters_;
  std::vector<uint64_t> cols_;
  bool passthrough_;
  mutable uint64_t rows_in_ = 0, rows_out_ = 0;  // UseBFStats (rpt_profiling.hpp) counters
};

}  // namespace rpt
