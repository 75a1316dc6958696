/*
 * rpt_gpu.h — C-ABI of the MI355X-native predicate-transfer Bloom filter (librpt_gpu.so).
 *
 * This is the drop-in boundary for the reference's PTBloomFilter seam
 * (/root/reference/src/include/bloom_filter.hpp:22-57, src/bloom_filter.cpp:11-78): the DuckDB
 * operators PhysicalCreateBF::Sink/Finalize (src/operators/physical_create_bf.cpp:201-242,352-419)
 * and PhysicalUseBF::ExecuteInternal (src/operators/physical_use_bf.cpp:60-198) call these entry
 * points instead of the DuckDB-native BloomFilter. Plain pointers and sizes only; no exceptions
 * cross the ABI (every entry point returns an rpt_status); device work is enqueued on the caller's
 * HIP stream and is asynchronous unless stated otherwise.
 *
 * Filter spec: the Arrow Acero BlockedBloomFilter the reference README ports (README.md:23-32):
 * 2^k 64-bit blocks, a 1024-entry table of 57-bit masks (4-5 bits set), mask rotation by hash bits
 * 10..15, block id from hash bits 16... Key hash: DuckDB VectorOperations::Hash semantics
 * (MurmurHash64 finalizer; int32 zero-extended through uint32; NULL rows hash to NULL_HASH).
 *
 * Key columns follow DuckDB's Vector model (see rpt_key_column):
 *   FLAT        keys[row]
 *   DICTIONARY  keys[key_sel[row]]        (validity indexed by the physical index key_sel[row])
 *   CONSTANT    flatten on the host first (PTBloomFilter's HashColumns flattens, bloom_filter.cpp:19-21)
 * Validity is DuckDB's ValidityMask layout: uint64 words, bit (i % 64) of word (i / 64) set = valid;
 * NULL pointer = all rows valid.
 */
#ifndef RPT_GPU_H
#define RPT_GPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RPT_GPU_ABI_VERSION 1

typedef enum rpt_status {
  RPT_OK = 0,
  RPT_ERR_INVALID_ARGUMENT = 1, /* null handle/pointer, bad key type, n too large for uint32 sel */
  RPT_ERR_HIP = 2,              /* a HIP runtime call failed; rpt_last_error() has the text */
  RPT_ERR_OUT_OF_MEMORY = 3,    /* device allocation failed */
  RPT_ERR_WORKSPACE = 4,        /* caller workspace smaller than rpt_probe_workspace_bytes() */
  RPT_ERR_SHAPE_MISMATCH = 5,   /* merge of filters with different log_num_blocks / devices */
  RPT_ERR_COLLECTIVE = 6,       /* librccl could not be loaded, or an RCCL call failed */
  RPT_ERR_COMM_ABORTED = 7      /* an OR all-reduce failed after its first collective call and ABORTED the
                                   communicator (ncclCommAbort freed it: never use or destroy it again) */
} rpt_status;

typedef enum rpt_key_type {
  RPT_KEY_I64 = 0,  /* BIGINT / int64 keys */
  RPT_KEY_I32 = 1,  /* INTEGER / int32 keys (JOB join keys) */
  RPT_KEY_HASH = 2  /* pre-computed 64-bit hashes (HashColumns output); validity/NULLs not applied */
} rpt_key_type;

/* How a probe reaches the filter blocks (rpt_bf_set_probe_strategy). All give identical results. */
typedef enum rpt_probe_strategy {
  RPT_PROBE_AUTO = 0,        /* by filter and batch size (measured crossovers): LDS (<= 128 KiB, and
                                256 / 512 KiB for n >= 4 Mi, 1 MiB for 4 Mi <= n < 32 Mi);
                                PARTITIONED (<= 128 MiB) for n >= 32 Mi (256 KiB..2 MiB) or n >= 4 Mi
                                (4 MiB and up); BUCKETED (<= 16 GiB, n >= max(blocks/8, 32 Mi));
                                otherwise GATHER */
  RPT_PROBE_GATHER = 1,      /* one random 8-byte gather per key from L2 / Infinity Cache / HBM */
  RPT_PROBE_LDS = 2,         /* filter staged in each workgroup's LDS: whole (<= 128 KiB), or its first 128 KiB
                                with the rest gathered from L2 (256 KiB .. 1 MiB) */
  RPT_PROBE_PARTITIONED = 3, /* rows bucketed per 16 Ki-row tile by 128 KiB filter slice; each slice is
                                probed from LDS, then row order is restored (filters 128 KiB..128 MiB) */
  RPT_PROBE_BUCKETED = 4     /* two levels: rows first bucketed by 32 MiB filter region into contiguous
                                hash arrays, then PARTITIONED per region (filters 32 MiB..16 GiB) */
} rpt_probe_strategy;

/* How an insert reaches the filter (rpt_bf_set_insert_strategy). All give identical filters. */
typedef enum rpt_insert_strategy {
  RPT_INSERT_AUTO = 0,        /* by filter and batch size (measured crossovers): PARTITIONED (<= 128 MiB,
                                 n >= 1 Mi), BUCKETED (larger, n >= max(blocks/16, 8 Mi)), else ATOMIC */
  RPT_INSERT_ATOMIC = 1,      /* one device-scope 64-bit atomic OR per key */
  RPT_INSERT_PARTITIONED = 2, /* rows bucketed by 128 KiB filter slice; each slice ORed in LDS, then
                                 merged with coalesced atomic ORs (filters 128 KiB..128 MiB) */
  RPT_INSERT_BUCKETED = 3     /* two levels as RPT_PROBE_BUCKETED (filters 32 MiB..16 GiB) */
} rpt_insert_strategy;

/* A hipStream_t, passed opaquely so this header needs no HIP include. NULL = the null stream. */
typedef void* rpt_stream_t;

/* Opaque filter handle: owns its device memory (PTBloomFilter + its BufferManager allocation,
 * bloom_filter.hpp:27-28,56; bloom_filter.cpp:27-32). */
typedef struct rpt_bf rpt_bf;

/* A key column on the device (DuckDB Vector shape; see header comment). */
typedef struct rpt_key_column {
  int32_t key_type;         /* rpt_key_type */
  const void* keys;         /* device pointer */
  const uint32_t* key_sel;  /* device pointer or NULL (DICTIONARY selection) */
  const uint64_t* validity; /* device pointer or NULL (all valid) */
} rpt_key_column;

typedef struct rpt_bf_info {
  int32_t device;          /* HIP device ordinal the words live on */
  int32_t log_num_blocks;  /* filter has 2^log_num_blocks uint64 blocks */
  uint64_t num_blocks;
  uint64_t sized_for_rows; /* PTBloomFilter::SizedForRows (bloom_filter.hpp:41-43) */
  int32_t has_data;        /* !PTBloomFilter::IsEmpty (bloom_filter.hpp:45-47) */
  int32_t finalized;       /* PTBloomFilter::finalized_ (bloom_filter.hpp:30) */
  uint64_t* words;         /* device pointer to the blocks (after rpt_bf_clear they read as zero only once
                              another operation on the filter has run: see rpt_bf_clear) */
} rpt_bf_info;

/* ---- library ---------------------------------------------------------------------------- */
int rpt_abi_version(void);
const char* rpt_status_string(int status);
/* Text of the last error raised on the calling thread ("" if none). */
const char* rpt_last_error(void);

/* ---- host-only sizing rules (no device work) ----------------------------------------------- */
/* log2 of the block count for a filter sized for n rows: log2ceil(max(512, 8n)) - 6 (Arrow
 * BlockedBloomFilter::CreateEmpty; the filter PTBloomFilter::Initialize allocates, bloom_filter.cpp:27-32). */
int rpt_bf_log_num_blocks_for_rows(uint64_t n_rows);
/* PhysicalCreateBF::Finalize resize rule, verbatim (physical_create_bf.cpp:394-398):
 * 1 iff actual_rows > 0 and actual_rows*8 > NextPow2(max(512, sized_for_rows*12)). */
int rpt_bf_needs_resize(uint64_t sized_for_rows, uint64_t actual_rows);
/* The resize predicate CREATE_BF's Finalize applies here: the reference's stated intent ("resize iff
 * allocated_bits / actual_rows < 8", physical_create_bf.cpp:383) evaluated on the filter actually
 * allocated (64 * 2^log_num_blocks bits, Arrow sizing at 8 bits per estimated row): 1 iff
 * actual_rows * 8 > 64 << log_num_blocks. The verbatim rule above assumes DuckDB's native 12-bit
 * allocation and would leave an Arrow-sized filter at 4 bits per key (sized_for 1000, actual 2048);
 * DESIGN.md §2. Negative rpt_status on error. */
int rpt_bf_needs_resize_alloc(const rpt_bf* bf, uint64_t actual_rows);
/* Device workspace a probe of n rows against a 2^log_num_blocks-block filter needs, for any
 * strategy (bytes, 256-aligned). rpt_bf_probe_workspace_bytes: for the strategy a probe of n rows
 * of this filter runs now (AUTO resolved), usually far less for very large filters. */
size_t rpt_probe_workspace_bytes(uint64_t n_rows, int log_num_blocks);

/* ---- lifecycle --------------------------------------------------------------------------- */
/* PTBloomFilter::Initialize(context, est_num_rows) (bloom_filter.cpp:27-32): allocate and zero a
 * filter sized for est_num_rows on `device`. Synchronous. */
int rpt_bf_create(int device, uint64_t est_num_rows, rpt_bf** out);
/* Same with an explicit size (2^log_num_blocks blocks, 0 <= log_num_blocks <= 40). */
int rpt_bf_create_log_blocks(int device, int log_num_blocks, rpt_bf** out);
int rpt_bf_destroy(rpt_bf* bf);
int rpt_bf_get_info(const rpt_bf* bf, rpt_bf_info* out);
/* First half of PTBloomFilter::ReinitializeAndRehash (bloom_filter.cpp:34-43): reallocate for
 * actual_rows, zero, sized_for_rows = actual_rows, has_data = 0. The caller then re-inserts the
 * materialized rows with rpt_bf_insert. Synchronous. */
int rpt_bf_reinitialize(rpt_bf* bf, uint64_t actual_rows);
/* PTBloomFilter::finalized_ = value (physical_create_bf.cpp:409-413). */
int rpt_bf_set_finalized(rpt_bf* bf, int value);
/* Select the probe strategy (rpt_probe_strategy); rpt_bf_probe_strategy returns the one a probe
 * will run now (AUTO resolved), or a negative status. */
int rpt_bf_set_probe_strategy(rpt_bf* bf, int strategy);
/* 1 if `strategy` can probe a 2^log_num_blocks-block filter, else 0. */
int rpt_probe_strategy_supported(int strategy, int log_num_blocks);
int rpt_bf_probe_strategy(const rpt_bf* bf);
/* The strategy a probe / insert of n rows runs now (AUTO resolved with n), or a negative status. */
int rpt_bf_probe_strategy_for(const rpt_bf* bf, uint64_t n_rows);
int rpt_bf_insert_strategy_for(const rpt_bf* bf, uint64_t n_rows);
size_t rpt_bf_probe_workspace_bytes(const rpt_bf* bf, uint64_t n_rows);
/* Zero every block and clear has_data (stream-ordered). The zeroing is deferred to the next operation on
 * the filter: a partitioned / bucketed insert that owns every slice stores the slices whole (so a rebuild
 * is one pass over the filter, not a memset and then the insert's stores); any other insert, merge,
 * probe, copy or export zeroes the words first, ordered like any other write. Only a direct read through
 * rpt_bf_info::words can see the words before that. */
int rpt_bf_clear(rpt_bf* bf, rpt_stream_t stream);
/* Settle a deferred clear now: zero the words on `stream` and wait until that zeroing has completed (a
 * no-op if no clear is pending). Needed before a stream capture (graph) reads or writes a cleared filter:
 * a read or write inside a capture that would have to settle the clear is refused with
 * RPT_ERR_INVALID_ARGUMENT (the zeroing would be replayed with the graph, wiping what was inserted between
 * replays). Synchronous.
 * Stream capture in general: probes capture freely once no clear is pending. A write (insert, merge, copy
 * into the filter) captures when no clear is pending and the filter's previous write has completed
 * (otherwise RPT_ERR_INVALID_ARGUMENT: synchronize first); a captured insert merges with atomics, so each
 * replay ORs its keys in whatever the filter holds by then, and replays are ordered by the stream the
 * graph is launched on (a captured write takes no part in the filter's cross-stream write order).
 * rpt_bf_clear and rpt_bf_allreduce_or[_ws] are refused inside a capture. Any capture mode works: the one event
 * query a captured write makes runs with the thread's capture mode relaxed around it. Under
 * hipStreamCaptureModeGlobal (torch.cuda.graph's default) no thread of the process may make an unsafe HIP call
 * while the capture is open, and rpt_bf_destroy / rpt_bf_create / rpt_bf_reinitialize are such calls (hipFree /
 * hipMalloc): create and destroy filters outside capture windows (collect garbage that may hold filters first,
 * as torch.cuda.graph does). */
int rpt_bf_settle(rpt_bf* bf, rpt_stream_t stream);

/* ---- build ------------------------------------------------------------------------------- */
/* PTBloomFilter::Insert (bloom_filter.cpp:70-78): hash each of n rows of `col` and OR its mask into
 * its block with a device-scope atomic OR. Thread-safe: any number of host threads / streams may
 * insert into one filter concurrently (parallel Sink, physical_create_bf.hpp:43-45). n == 0 is a
 * no-op; otherwise has_data becomes 1. */
int rpt_bf_insert(rpt_bf* bf, const rpt_key_column* col, uint64_t n, rpt_stream_t stream);

/* rpt_bf_insert with a caller workspace, which enables the partitioned / bucketed inserts for large
 * batches (same result, same thread-safety). workspace: rpt_insert_workspace_bytes(n,
 * log_num_blocks) bytes of device memory (the largest any insert strategy needs; 0 when the filter
 * only supports atomic inserts), or rpt_bf_insert_workspace_bytes(bf, n) for the strategy this
 * insert will run (0 = atomic, no workspace needed). */
size_t rpt_insert_workspace_bytes(uint64_t n_rows, int log_num_blocks);
size_t rpt_bf_insert_workspace_bytes(const rpt_bf* bf, uint64_t n_rows);
int rpt_bf_insert_ws(rpt_bf* bf, const rpt_key_column* col, uint64_t n, void* workspace, size_t workspace_bytes,
                     rpt_stream_t stream);
int rpt_bf_set_insert_strategy(rpt_bf* bf, int strategy);

/* Min/max dynamic filter (PhysicalCreateBF::Sink/Combine, physical_create_bf.cpp:82-176, 229-272;
 * pushed as >= min / <= max scan filters at :335-345): every insert of an I32/I64 column also folds
 * the min and max of its valid (non-NULL) key values into the filter, fused into the insert kernels
 * (HASH columns carry no values and are skipped). I32 values are sign-extended. Reset by
 * rpt_bf_create / rpt_bf_clear / rpt_bf_reinitialize; rpt_bf_merge_or merges them. get: stream-ordered
 * read, then synchronizes `stream`; *out_has_value = 0 (and min = max = 0) when no valid key was
 * inserted. set: overwrite (the multi-GPU merge writes the all-reduced values back). */
int rpt_bf_get_minmax(const rpt_bf* bf, int64_t* out_min, int64_t* out_max, int* out_has_value, rpt_stream_t stream);
int rpt_bf_set_minmax(rpt_bf* bf, int64_t min_value, int64_t max_value, int has_value, rpt_stream_t stream);

/* ---- probe ------------------------------------------------------------------------------- */
/* PTBloomFilter::LookupSel (bloom_filter.cpp:60-68) for a batch of rows: writes the ids of rows
 * whose key may be in the filter to out_sel in ASCENDING order and the survivor count to
 * *out_count_dev (device uint64). Rows are 0..n-1, or row_sel[0..n) when row_sel != NULL (the
 * already-sliced chunk of PhysicalUseBF's multi-filter loop, physical_use_bf.cpp:137-183); the
 * written ids are then the row_sel values. n must be < 2^32 (sel_t is uint32). out_sel capacity n.
 * workspace: device memory of rpt_probe_workspace_bytes(n, log_num_blocks) bytes, exclusively owned by this call
 * until it completes on `stream`. Batches of at most RPT_SMALL_PROBE_ROWS rows under the AUTO strategy
 * run one fused single-workgroup kernel (probe + compaction: one launch instead of four) and leave
 * the workspace untouched. */
#define RPT_SMALL_PROBE_ROWS 16384
/* 1 if rpt_bf_probe of n_rows rows runs the fused small-batch kernel now (AUTO strategy, 1 <= n_rows <=
 * RPT_SMALL_PROBE_ROWS), else 0; negative rpt_status on error. Its key, validity, row_sel and output
 * buffers may then be device-mapped pinned host memory (hipHostGetDevicePointer): one launch and no
 * copies per call. */
int rpt_bf_probe_is_fused(const rpt_bf* bf, uint64_t n_rows);
int rpt_bf_probe(const rpt_bf* bf, const rpt_key_column* col, const uint32_t* row_sel, uint64_t n,
                 uint32_t* out_sel, uint64_t* out_count_dev, void* workspace, size_t workspace_bytes,
                 rpt_stream_t stream);
/* PhysicalUseBF::ExecuteInternal's filter chain (physical_use_bf.cpp:127-179: each LookupSel over the rows
 * the previous filters kept, i.e. the AND of the filters) over one small batch in ONE launch: out_sel gets
 * the ascending ids of the rows that pass every filters[i], probed on its own key column cols[i] (each
 * column may have its own key type, dictionary, validity), and *out_count_dev their count. Rows are
 * 0..n-1, or row_sel[0..n) as in rpt_bf_probe. 1 <= n_filters <= RPT_MAX_CHAIN, n <= RPT_SMALL_PROBE_ROWS,
 * every filter on one device; no workspace. The skips and early exits of the reference loop (a filter not
 * yet finalized is skipped, an empty filter passes nothing) are the caller's: pass the filters that
 * apply. Buffers may be device-mapped pinned host memory, as for the fused rpt_bf_probe. */
#define RPT_MAX_CHAIN 8
int rpt_bf_probe_chain(const rpt_bf* const* filters, const rpt_key_column* cols, uint32_t n_filters,
                       const uint32_t* row_sel, uint64_t n, uint32_t* out_sel, uint64_t* out_count_dev,
                       rpt_stream_t stream);
/* rpt_bf_probe in its two stream-ordered phases (same filter, workspace and stream), for callers that
 * time or overlap them. GATHER / LDS: phase 1 = hash + gather + result bits + per-segment counts,
 * phase 2 = scan + expansion into out_sel. PARTITIONED: phase 1 = partition rows by filter slice +
 * probe each slice from LDS + restore row order into the result bits, phase 2 = as above.
 * (rpt_bf_probe itself runs the PARTITIONED strategy without the result bits: per-tile survivor counts
 * give each tile's offset and the row-order restore writes out_sel directly. Same sel and count.) */
int rpt_bf_probe_phase1(const rpt_bf* bf, const rpt_key_column* col, const uint32_t* row_sel, uint64_t n,
                        void* workspace, size_t workspace_bytes, rpt_stream_t stream);
int rpt_bf_probe_phase2(const rpt_bf* bf, const uint32_t* row_sel, uint64_t n, uint32_t* out_sel,
                        uint64_t* out_count_dev, void* workspace, size_t workspace_bytes, rpt_stream_t stream);
/* rpt_bf_probe's result as bits instead of a selection vector: bit i (LSB-first in uint64 words) of out_bits = the
 * i-th probed row (row i, or row_sel[i]) passes; out_bits (device memory) holds ceil(n/512)*8 words, bits past n
 * are 0. Same strategies and workspace (rpt_bf_probe_workspace_bytes) as rpt_bf_probe; stream-ordered, no sync. A
 * host-resident caller copies n/8 bytes back instead of 4 bytes per survivor (the C++ host mirror's pipelined
 * lookups do, DeviceContext::bits_back). */
int rpt_bf_probe_bits(const rpt_bf* bf, const rpt_key_column* col, const uint32_t* row_sel, uint64_t n,
                      uint64_t* out_bits, void* workspace, size_t workspace_bytes, rpt_stream_t stream);
/* Arrow BlockedBloomFilter::Find(…, result_bit_vector) shape: bit i (LSB-first in uint64 words) of
 * out_bits = row i passes. out_bits must hold ceil(n/512)*8 words. */
int rpt_bf_find_bits(const rpt_bf* bf, const rpt_key_column* col, uint64_t n, uint64_t* out_bits,
                     rpt_stream_t stream);
/* Key hashes exactly as the filter sees them (DuckDB HashColumns restatement). */
int rpt_hash_keys(const rpt_key_column* col, uint64_t n, uint64_t* out_hashes, rpt_stream_t stream);
/* HashColumns' CombineHash step for composite keys (bloom_filter.cpp:15-17): inout_hashes[i] =
 * CombineHashScalar(inout_hashes[i], Hash(row i of col)) with DuckDB v1.1+'s form (a ^= a >> 32;
 * a *= 0xd6e8feb86659fd93; a ^ b; restated, parity unpinned). rpt_hash_keys(col_0) followed by
 * rpt_hash_combine(col_j) for j = 1, 2, ... is the composite-key hash; insert / probe it as an
 * RPT_KEY_HASH column. */
int rpt_hash_combine(const rpt_key_column* col, uint64_t n, uint64_t* inout_hashes, rpt_stream_t stream);
/* Narrow BIGINT keys (device memory): out[r] = (uint64_t)chunk_hi[c] << 32 | lo[r] for the rows r of chunk c,
 * [chunk_row0[c], chunk_row0[c + 1]), c < n_chunks (chunk_row0 ascending; out and lo hold chunk_row0[n_chunks]
 * entries). A host-resident batch whose chunks each share their keys' high 32 bits crosses PCIe as 4-B low words
 * plus one high word per chunk and is widened here before the insert / probe (the C++ host mirror does this by
 * itself). Stream-ordered; n_chunks == 0 is a no-op. */
int rpt_keys_widen(const uint32_t* lo, const uint32_t* chunk_hi, const uint32_t* chunk_row0, uint64_t n_chunks,
                   uint64_t* out, rpt_stream_t stream);

/* ---- merge / fold / export ----------------------------------------------------------------- */
/* dst |= src (same log_num_blocks, same device): merging per-thread or per-GPU partial filters
 * built over disjoint row ranges gives the filter of the union, bit-identical to one build. */
int rpt_bf_merge_or(rpt_bf* dst, const rpt_bf* src, rpt_stream_t stream);
/* Multi-GPU CREATE_BF Combine: OR all-reduce of every rank's partial filter over an RCCL
 * communicator (`comm` is an ncclComm_t, one rank per GPU; every rank's filter has the same
 * log_num_blocks). It is composed as a reduce-scatter by OR (grouped ncclSend/ncclRecv of 1/W of the
 * words, then an OR kernel) and an all-gather (grouped ncclSend/ncclRecv). RCCL has no bitwise-OR
 * ncclRedOp_t. The key min/max and has_data are reduced too, in one ncclAllReduce(MIN). Collective:
 * every rank of the communicator must call it. Stream-ordered on `stream`; returns after has_data is
 * known (one stream sync). librccl is loaded on first use (dlopen), so the library itself does not
 * depend on it.
 * Rank j owns words [lo(j), lo(j+1)), lo(j) = (num_blocks * j / world) rounded down to 32 words (W need not
 * divide the block count). The reduce-scatter runs in rounds of at most RPT_ALLREDUCE_ROUND_WORDS words
 * per peer through two staging buffers: the OR kernel of round r runs on a library helper stream while
 * round r + 1 transfers on `stream`. rpt_bf_allreduce_or_ws takes that staging from the caller
 * (rpt_allreduce_workspace_bytes(world, log_num_blocks) bytes of device memory, exclusively owned until
 * the call returns; <= 2 (W-1) * 32 MiB + 256 B whatever the filter size); rpt_bf_allreduce_or allocates
 * and frees it itself.
 * Failure (the cross-GPU analogue of a Combine that cannot finish, physical_create_bf.cpp:244-275): the
 * call never blocks on the stream blindly. It polls the stream and ncclCommGetAsyncError until every
 * transfer completed or the collective timeout (rpt_collective_set_timeout_ms) passed; a non-blocking
 * communicator's ncclInProgress results are polled against the same deadline. A peer that dies mid-merge
 * never posts its side, so its peers' streams would wait forever: on a timeout, an asynchronous RCCL error
 * or any error after the first collective call, the call ABORTS the communicator (ncclCommAbort, which
 * frees it), drains the streams (bounded again) and returns RPT_ERR_COMM_ABORTED: never use the
 * communicator again, and do not ncclCommDestroy it (rpt_rccl_comm_destroy accepts one this library made
 * and does nothing). An error before any collective call returns RPT_ERR_COLLECTIVE (or another status)
 * with the communicator intact. The filter then holds its own partial plus possibly some peers' bits
 * (never fewer bits than before the call): rebuild it, or merge again on a new communicator.
 * If even the aborted streams do not drain by the second deadline, the message says "streams did not
 * drain": the workspace, `stream` and the filter stay in use by work that may never finish (later work
 * ordered after them may never run; rpt_bf_allreduce_or then leaks its workspace rather than free it).
 * A caller that owns its communicator and wants to abort it itself sets rpt_collective_set_abort_on_error(0):
 * the merge then never aborts; after a failure past the first collective call it returns
 * RPT_ERR_COLLECTIVE with the communicator untouched, and, when RCCL's kernels still hold the streams (the
 * message says "streams are still blocked"), `stream`, the workspace and the filter stay in use until the
 * owner calls ncclCommAbort. Not inside a stream capture (RPT_ERR_INVALID_ARGUMENT): it waits on the host. */
#define RPT_ALLREDUCE_ROUND_WORDS (4ULL << 20)
size_t rpt_allreduce_workspace_bytes(int world, int log_num_blocks);
int rpt_bf_allreduce_or_ws(rpt_bf* bf, void* nccl_comm, void* workspace, size_t workspace_bytes,
                           rpt_stream_t stream);
int rpt_bf_allreduce_or(rpt_bf* bf, void* nccl_comm, rpt_stream_t stream);
/* Bound of one OR all-reduce's waits (process-wide; default RPT_COLLECTIVE_TIMEOUT_MS_DEFAULT). An 8 GiB
 * filter merges in well under a second over xGMI; the bound only has to outlast RCCL's first connection
 * setup between the ranks. 0 is rejected. */
#define RPT_COLLECTIVE_TIMEOUT_MS_DEFAULT 120000ULL
int rpt_collective_set_timeout_ms(uint64_t ms);
uint64_t rpt_collective_timeout_ms(void);
/* Process-wide: 1 (default) = a failed merge aborts its communicator (RPT_ERR_COMM_ABORTED above); 0 = it
 * leaves the communicator to its owner (RPT_ERR_COLLECTIVE). */
int rpt_collective_set_abort_on_error(int abort_on_error);
int rpt_collective_abort_on_error(void);
/* RCCL communicator for callers that bring none (bench.py, tests; a DuckDB shim that owns an
 * ncclComm_t passes it to rpt_bf_allreduce_or directly). Rank 0 calls rpt_rccl_get_unique_id, the
 * caller broadcasts the RPT_RCCL_UNIQUE_ID_BYTES bytes out of band (torch.distributed, MPI, a file),
 * then every rank calls rpt_rccl_comm_init_rank for its own GPU (collective; blocks until all ranks
 * joined) — ncclGetUniqueId / ncclCommInitRank / ncclCommDestroy of the dlopened librccl. */
#define RPT_RCCL_UNIQUE_ID_BYTES 128
/* RPT_OK if librccl loads with every entry point the merge uses and `device` can be made current (no
 * collective call): every rank checks it, and the ranks agree, before the collective init, so a rank
 * that cannot join never leaves the others blocked in ncclCommInitRank. */
int rpt_rccl_available(int device);
int rpt_rccl_get_unique_id(uint8_t* out_id);
int rpt_rccl_comm_init_rank(int device, int world, const uint8_t* id, int rank, void** out_comm);
/* The same as a NON-BLOCKING communicator (ncclCommInitRankConfig, blocking = 0): every RCCL call on it returns
 * at once (ncclInProgress) and rpt_bf_allreduce_or[_ws] polls ncclCommGetAsyncError against the collective
 * timeout, so even RCCL's host-side connection setup with a peer that died cannot block the caller past the
 * bound (a blocking communicator's ncclGroupEnd can). Init itself completes within the timeout or fails. */
int rpt_rccl_comm_init_rank_nonblocking(int device, int world, const uint8_t* id, int rank, void** out_comm);
/* Destroy a communicator made by rpt_rccl_comm_init_rank[_nonblocking] (one a failed merge aborted: nothing to
 * do). A non-blocking one is finalized first (ncclCommFinalize, polled to completion against the collective
 * timeout; aborted if it does not complete), so its teardown has finished when this returns. */
int rpt_rccl_comm_destroy(void* comm);
/* dst[i] |= src[i] for n_words words (device pointers): the local step of the multi-GPU
 * OR all-reduce (reduce-scatter slices). */
int rpt_words_or(uint64_t* dst, const uint64_t* src, uint64_t n_words, rpt_stream_t stream);
/* dst[i] = src_0[i] | src_1[i] | ... | src_{k-1}[i], srcs given as k contiguous slices of
 * n_words words starting at `srcs` (a receive buffer of k peer slices). */
int rpt_words_or_slices(uint64_t* dst, const uint64_t* srcs, uint32_t k, uint64_t n_words, rpt_stream_t stream);
/* BlockedBloomFilter::IsSameAs (pyarrow 25 arrow/acero/bloom_filter.h:131): *out_same = 1 iff both filters
 * have the same log_num_blocks and every word is equal, compared on the device (no host copy of either
 * filter; bench.py's multi-GPU merge check of C5's 8 GiB filters). *out_diff_words (nullable) = the number of
 * differing words (~0 for different geometry). Filters on one device. Synchronous (waits for the device). */
int rpt_bf_is_same_as(const rpt_bf* a, const rpt_bf* b, int* out_same, uint64_t* out_diff_words);
/* Number of set bits (BlockedBloomFilter::NumBitsSet). Synchronous. */
int rpt_bf_count_bits(const rpt_bf* bf, uint64_t* out);
/* BlockedBloomFilter::Fold (bloom_filter.h:135-158): while fewer than 1/4 of the bits are set and
 * the filter has more than 2^4 blocks, OR its upper slices into the lowest one. Synchronous. */
int rpt_bf_fold(rpt_bf* bf, int* out_new_log_num_blocks);
/* Copy the blocks to/from host memory (parity, checkpoint of a finished filter). Synchronous.
 * import sets has_data = (any bit set). */
int rpt_bf_export_words(const rpt_bf* bf, uint64_t* host_words, uint64_t n_words);
int rpt_bf_import_words(rpt_bf* bf, const uint64_t* host_words, uint64_t n_words);
/* Stream-ordered device-to-device copies of all 2^log_num_blocks blocks to / from a caller buffer
 * (the staging buffer of the multi-GPU OR all-reduce). n_words must equal the block count. */
int rpt_bf_copy_words_to(const rpt_bf* bf, uint64_t* dst_dev, uint64_t n_words, rpt_stream_t stream);
int rpt_bf_copy_words_from(rpt_bf* bf, const uint64_t* src_dev, uint64_t n_words, rpt_stream_t stream);
/* Mark has_data after words were filled by a device-side exchange (multi-GPU merge). */
int rpt_bf_set_has_data(rpt_bf* bf, int value);

/* ---- kernel timing ----------------------------------------------------------------------- */
/* The reference's per-operator profiling counters (src/include/rpt_profiling.hpp:16-217), at kernel
 * granularity: while enabled, every kernel the library launches is bracketed by HIP events on its
 * own stream. rpt_profiling_read resolves pending events (waits for them), fills up to `capacity`
 * entries and returns the number of distinct kernels (negative status on error). */
typedef struct rpt_kernel_stat {
  char name[48];
  uint64_t launches;
  double total_ms;
} rpt_kernel_stat;
int rpt_profiling_enable(int enable);
int rpt_profiling_reset(void);
int rpt_profiling_read(rpt_kernel_stat* out, int capacity);

#ifdef __cplusplus
}
#endif

#endif /* RPT_GPU_H */
