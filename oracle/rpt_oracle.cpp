// rpt_oracle.cpp — CPU restatement of the predicate-transfer Bloom-filter hot path.
//
// ***************************************************************************************
// TEST INFRASTRUCTURE ONLY. This file is the parity checker and the reported CPU baseline.
// Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it. The
// product (librpt_gpu.so) never links, loads or falls back to it.
// ***************************************************************************************
//
// What it restates, and from where:
//   * PTBloomFilter (reference src/bloom_filter.cpp:11-78, src/include/bloom_filter.hpp:22-57):
//     HashColumns -> native BloomFilter::InsertHashes / LookupHashes. Insert sets has_data_
//     (bloom_filter.cpp:75); LookupSel writes ascending surviving row ids (bloom_filter.cpp:60-68).
//   * The filter arithmetic is the Arrow Acero BlockedBloomFilter the reference README ports
//     (README.md:23-32; pyarrow 25.0.0 arrow/acero/bloom_filter.h:42-240):
//       mask(h)     = ROTL64(masks.mask(h & 1023), (h >> 10) & 63)         (bloom_filter.h:172-185)
//       block_id(h) = (h >> 16) & (num_blocks - 1)                            (bloom_filter.h:187-193)
//       Insert      = blocks[block_id] |= mask                                 (bloom_filter.h:163-167)
//       Find        = (blocks[block_id] & mask) == mask                        (bloom_filter.h:113-117)
//       sizing      = log2_ceil(max(512, 8 * n)) - 6 blocks                    (CreateEmpty)
//       Fold        = OR slices while density < 1/4, floor 2^4 blocks          (bloom_filter.h:135-158)
//     PINNED against golden vectors produced by the real Arrow library (tests/golden/).
//   * Key hash: DuckDB VectorOperations::Hash (third-party, DuckDB v1.4.4, source absent from the
//     container): MurmurHash64 finalizer, int32 zero-extended through uint32, NULL -> NULL_HASH.
//     UNPINNED (no DuckDB here); restated identically in the HIP kernels.
//   * Resize rule of PhysicalCreateBF::Finalize (physical_create_bf.cpp:386-406).
//   * Composite-key CombineHash (bloom_filter.cpp:15-17; UNPINNED) and the build's min/max dynamic
//     filter (TypedUpdateMinMax, physical_create_bf.cpp:86-119) for INTEGER / BIGINT keys.
//   * CPU baseline: morsel-parallel build/probe in 2048-row vectors, like DuckDB's parallel sink
//     (physical_create_bf.hpp:43-45) and parallel operator (physical_use_bf.hpp:47-49), with an
//     atomic fetch_or insert (README.md:32).
#include <pthread.h>
#include <sched.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstring>
#include <random>
#include <thread>
#include <vector>

namespace {

constexpr int kBitsPerMask = 57;
constexpr uint64_t kFullMask = (1ULL << kBitsPerMask) - 1;
constexpr int kMinBitsSet = 4;
constexpr int kMaxBitsSet = 5;
constexpr int kLogNumMasks = 10;
constexpr int kNumMasks = 1 << kLogNumMasks;
constexpr int kTotalBytes = (kNumMasks + 64) / 8;
constexpr uint64_t kNullHash = 0xbf58476dULL << 32 | 0x1ce4e5b9ULL;
constexpr uint64_t kVectorSize = 2048;  // DuckDB STANDARD_VECTOR_SIZE

inline bool get_bit(const uint8_t* b, int64_t i) { return (b[i >> 3] >> (i & 7)) & 1; }
inline void set_bit(uint8_t* b, int64_t i) { b[i >> 3] |= static_cast<uint8_t>(1u << (i & 7)); }

// Restatement of arrow::acero::BloomFilterMasks::BloomFilterMasks() (bloom_filter.h:42-48):
// a sliding 57-bit window over one 1088-bit vector, every window holding 4 or 5 set bits,
// driven by mt19937 seeded with seed_seq{0 x 8}.
struct Masks {
  uint8_t bytes[kTotalBytes];
  uint64_t values[kNumMasks];
  Masks() {
    std::seed_seq seed{0, 0, 0, 0, 0, 0, 0, 0};
    std::mt19937 re(seed);
    std::uniform_int_distribution<uint64_t> rd;
    auto random = [&](int lo, int hi) -> int64_t {
      return lo + static_cast<int64_t>(rd(re) % static_cast<uint64_t>(hi - lo + 1));
    };
    memset(bytes, 0, sizeof bytes);
    int num_bits_set = static_cast<int>(random(kMinBitsSet, kMaxBitsSet));
    for (int i = 0; i < num_bits_set; ++i) {
      for (;;) {
        int pos = static_cast<int>(random(0, kBitsPerMask - 1));
        if (!get_bit(bytes, pos)) {
          set_bit(bytes, pos);
          break;
        }
      }
    }
    const int64_t total = kNumMasks + kBitsPerMask - 1;
    for (int64_t i = kBitsPerMask; i < total; ++i) {
      int leaving = get_bit(bytes, i - kBitsPerMask) ? 1 : 0;
      if (leaving == 1 && num_bits_set == kMinBitsSet) {
        set_bit(bytes, i);
        continue;
      }
      if (leaving == 0 && num_bits_set == kMaxBitsSet) continue;
      if (random(0, kBitsPerMask * 2 - 1) < kMinBitsSet + kMaxBitsSet) {
        set_bit(bytes, i);
        if (leaving == 0) ++num_bits_set;
      } else if (leaving == 1) {
        --num_bits_set;
      }
    }
    for (int id = 0; id < kNumMasks; id++) {
      uint64_t w;
      memcpy(&w, bytes + id / 8, 8);  // little-endian unaligned load (bloom_filter.h:50-60)
      values[id] = (w >> (id % 8)) & kFullMask;
    }
  }
};

const Masks& masks() {
  static const Masks m;
  return m;
}

inline uint64_t rotl64(uint64_t x, int n) { return (x << n) | (x >> ((-n) & 63)); }

inline uint64_t mask_of(uint64_t h) {
  return rotl64(masks().values[h & (kNumMasks - 1)], static_cast<int>((h >> kLogNumMasks) & 63));
}

inline uint64_t block_of(uint64_t h, uint64_t nb) { return (h >> (kLogNumMasks + 6)) & (nb - 1); }

inline uint64_t murmur64(uint64_t x) {
  x ^= x >> 32;
  x *= 0xd6e8feb86659fd93ULL;
  x ^= x >> 32;
  x *= 0xd6e8feb86659fd93ULL;
  x ^= x >> 32;
  return x;
}

inline bool row_valid(const uint64_t* validity, uint64_t idx) {
  return !validity || ((validity[idx >> 6] >> (idx & 63)) & 1);
}

// DuckDB HashOp::Operation(input, is_null) over a FLAT or DICTIONARY vector: the physical index
// is key_sel[i] (dictionary) or i (flat); validity is indexed by the physical index.
template <typename T>
inline uint64_t key_hash(const T* keys, const uint32_t* key_sel, const uint64_t* validity, uint64_t i) {
  uint64_t idx = key_sel ? key_sel[i] : i;
  if (!row_valid(validity, idx)) return kNullHash;
  if (sizeof(T) == 4) return murmur64(static_cast<uint64_t>(static_cast<uint32_t>(keys[idx])));
  return murmur64(static_cast<uint64_t>(keys[idx]));
}

inline uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}
inline uint64_t sm64(uint64_t seed, uint64_t i) { return mix64(seed + (i + 1) * 0x9e3779b97f4a7c15ULL); }

constexpr uint64_t kSeedBuild = 0x5EED0001ULL;
constexpr uint64_t kSeedProbeSel = 0x5EED0002ULL;
constexpr uint64_t kSeedProbeMiss = 0x5EED0003ULL;

inline int64_t synth_probe_key(uint64_t n_build, uint32_t p_permille, uint64_t r) {
  uint64_t u = sm64(kSeedProbeSel, r);
  if (n_build > 0 && (u % 1000) < p_permille) {
    return static_cast<int64_t>(sm64(kSeedBuild, (u >> 20) % n_build));
  }
  return static_cast<int64_t>(sm64(kSeedProbeMiss, r));
}

template <typename T>
uint64_t probe_keys(const uint64_t* words, int log_nb, const T* keys, const uint32_t* key_sel,
                    const uint64_t* validity, uint64_t n, uint32_t* sel) {
  const uint64_t nb = 1ULL << log_nb;
  uint64_t cnt = 0;
  for (uint64_t i = 0; i < n; i++) {
    uint64_t h = key_hash(keys, key_sel, validity, i);
    uint64_t m = mask_of(h);
    sel[cnt] = static_cast<uint32_t>(i);
    cnt += (words[block_of(h, nb)] & m) == m;
  }
  return cnt;
}

template <typename T>
void insert_keys(uint64_t* words, int log_nb, const T* keys, const uint32_t* key_sel,
                 const uint64_t* validity, uint64_t n) {
  const uint64_t nb = 1ULL << log_nb;
  for (uint64_t i = 0; i < n; i++) {
    uint64_t h = key_hash(keys, key_sel, validity, i);
    words[block_of(h, nb)] |= mask_of(h);
  }
}

}  // namespace

// DuckDB CombineHashScalar as of v1.1+ (the hash rework that also introduced this MurmurHash64
// finalizer): a ^= a >> 32; a *= 0xd6e8feb86659fd93; return a ^ b. Restated from memory (v0.x-1.0 used
// (a * 0xbf58476d1ce4e5b9) ^ b); no DuckDB source in the image: parity unpinned.
inline uint64_t combine_hash(uint64_t a, uint64_t b) {
  a ^= a >> 32;
  a *= 0xd6e8feb86659fd93ULL;
  return a ^ b;
}

// TypedUpdateMinMax (reference physical_create_bf.cpp:86-119) for INTEGER / BIGINT: min and max of
// the valid rows (row -> physical index through key_sel, validity by physical index). Returns 0 and
// leaves out2 untouched when no row is valid.
template <typename T>
int minmax(const T* keys, const uint32_t* key_sel, const uint64_t* validity, uint64_t n, int64_t* out2) {
  bool has = false;
  T lo{}, hi{};
  for (uint64_t r = 0; r < n; r++) {
    const uint64_t idx = key_sel ? key_sel[r] : r;
    if (!row_valid(validity, idx)) continue;
    const T v = keys[idx];
    if (!has) {
      lo = hi = v;
      has = true;
    } else {
      if (v < lo) lo = v;
      if (v > hi) hi = v;
    }
  }
  if (!has) return 0;
  out2[0] = static_cast<int64_t>(lo);
  out2[1] = static_cast<int64_t>(hi);
  return 1;
}

extern "C" {

// ---- spec pieces --------------------------------------------------------------------------
void rpt_oracle_mask_table(uint8_t* out136) { memcpy(out136, masks().bytes, kTotalBytes); }
uint64_t rpt_oracle_mask(uint32_t id) { return masks().values[id & (kNumMasks - 1)]; }
uint64_t rpt_oracle_mask_of_hash(uint64_t h) { return mask_of(h); }

// BlockedBloomFilter::CreateEmpty sizing: log2_ceil(max(512, 8n)) - 6.
int rpt_oracle_log_num_blocks(uint64_t n_rows) {
  uint64_t bits = std::max<uint64_t>(512, n_rows * 8);
  int lg = 0;
  while ((1ULL << lg) < bits) lg++;
  return lg - 6;
}

// PhysicalCreateBF::Finalize resize predicate (physical_create_bf.cpp:394-398), verbatim:
// min_bits = max(512, sized_for * 12); allocated = NextPowerOfTwo(min_bits); resize iff actual*8 > allocated.
int rpt_oracle_needs_resize(uint64_t sized_for_rows, uint64_t actual_rows) {
  if (actual_rows == 0) return 0;
  uint64_t min_bits = std::max<uint64_t>(512, sized_for_rows * 12);
  uint64_t alloc = 1;
  while (alloc < min_bits) alloc <<= 1;
  return actual_rows * 8 > alloc ? 1 : 0;
}

// The same predicate against the filter actually allocated (the reference's stated intent,
// physical_create_bf.cpp:383: "resize iff allocated_bits / actual_rows < 8"): the filter holds
// 64 * 2^log_num_blocks bits (Arrow sizing, 8 bits per estimated row), so resize iff
// actual * 8 > 64 << log_num_blocks.
int rpt_oracle_needs_resize_alloc(int log_num_blocks, uint64_t actual_rows) {
  if (actual_rows == 0) return 0;
  const uint64_t alloc_bits = 64ULL << log_num_blocks;
  return actual_rows > alloc_bits / 8 ? 1 : 0;
}

uint64_t rpt_oracle_murmur64(uint64_t x) { return murmur64(x); }
uint64_t rpt_oracle_null_hash(void) { return kNullHash; }

void rpt_oracle_hash_i64(const int64_t* keys, const uint32_t* key_sel, const uint64_t* validity, uint64_t n,
                         uint64_t* out) {
  for (uint64_t i = 0; i < n; i++) out[i] = key_hash(keys, key_sel, validity, i);
}
void rpt_oracle_hash_i32(const int32_t* keys, const uint32_t* key_sel, const uint64_t* validity, uint64_t n,
                         uint64_t* out) {
  for (uint64_t i = 0; i < n; i++) out[i] = key_hash(keys, key_sel, validity, i);
}

// HashColumns' CombineHash (reference src/bloom_filter.cpp:15-17) for composite keys: DuckDB
// CombineHashScalar(a, b) (combine_hash above, the v1.1+ form) with b = Hash(row of col_j). Restated
// from DuckDB (vector_hash.cpp; source absent): UNPINNED, like the key hash.
void rpt_oracle_hash_combine_i64(const int64_t* keys, const uint32_t* key_sel, const uint64_t* validity, uint64_t n,
                                 uint64_t* inout) {
  for (uint64_t i = 0; i < n; i++) inout[i] = combine_hash(inout[i], key_hash(keys, key_sel, validity, i));
}
void rpt_oracle_hash_combine_i32(const int32_t* keys, const uint32_t* key_sel, const uint64_t* validity, uint64_t n,
                                 uint64_t* inout) {
  for (uint64_t i = 0; i < n; i++) inout[i] = combine_hash(inout[i], key_hash(keys, key_sel, validity, i));
}

int rpt_oracle_minmax_i64(const int64_t* keys, const uint32_t* key_sel, const uint64_t* validity, uint64_t n,
                          int64_t* out2) {
  return minmax(keys, key_sel, validity, n, out2);
}
int rpt_oracle_minmax_i32(const int32_t* keys, const uint32_t* key_sel, const uint64_t* validity, uint64_t n,
                          int64_t* out2) {
  return minmax(keys, key_sel, validity, n, out2);
}

// ---- filter ops ---------------------------------------------------------------------------
void rpt_oracle_insert_hashes(uint64_t* words, int log_nb, const uint64_t* h, uint64_t n) {
  const uint64_t nb = 1ULL << log_nb;
  for (uint64_t i = 0; i < n; i++) words[block_of(h[i], nb)] |= mask_of(h[i]);
}
void rpt_oracle_insert_i64(uint64_t* words, int log_nb, const int64_t* keys, const uint32_t* key_sel,
                           const uint64_t* validity, uint64_t n) {
  insert_keys(words, log_nb, keys, key_sel, validity, n);
}
void rpt_oracle_insert_i32(uint64_t* words, int log_nb, const int32_t* keys, const uint32_t* key_sel,
                           const uint64_t* validity, uint64_t n) {
  insert_keys(words, log_nb, keys, key_sel, validity, n);
}

// Arrow Find(…, result_bit_vector): LSB-first bit per row.
void rpt_oracle_find_hashes(const uint64_t* words, int log_nb, const uint64_t* h, uint64_t n, uint8_t* bv) {
  const uint64_t nb = 1ULL << log_nb;
  memset(bv, 0, (n + 7) / 8);
  for (uint64_t i = 0; i < n; i++) {
    uint64_t m = mask_of(h[i]);
    if ((words[block_of(h[i], nb)] & m) == m) bv[i >> 3] |= static_cast<uint8_t>(1u << (i & 7));
  }
}

// LookupHashes-shaped: ascending surviving row ids, returns count.
uint64_t rpt_oracle_lookup_sel_hashes(const uint64_t* words, int log_nb, const uint64_t* h, uint64_t n,
                                      uint32_t* sel) {
  const uint64_t nb = 1ULL << log_nb;
  uint64_t cnt = 0;
  for (uint64_t i = 0; i < n; i++) {
    uint64_t m = mask_of(h[i]);
    sel[cnt] = static_cast<uint32_t>(i);
    cnt += (words[block_of(h[i], nb)] & m) == m;
  }
  return cnt;
}
uint64_t rpt_oracle_probe_i64(const uint64_t* words, int log_nb, const int64_t* keys, const uint32_t* key_sel,
                              const uint64_t* validity, uint64_t n, uint32_t* sel) {
  return probe_keys(words, log_nb, keys, key_sel, validity, n, sel);
}
uint64_t rpt_oracle_probe_i32(const uint64_t* words, int log_nb, const int32_t* keys, const uint32_t* key_sel,
                              const uint64_t* validity, uint64_t n, uint32_t* sel) {
  return probe_keys(words, log_nb, keys, key_sel, validity, n, sel);
}

uint64_t rpt_oracle_count_bits(const uint64_t* words, uint64_t nwords) {
  uint64_t c = 0;
  for (uint64_t i = 0; i < nwords; i++) c += static_cast<uint64_t>(__builtin_popcountll(words[i]));
  return c;
}

// BlockedBloomFilter::Fold (bloom_filter.h:135-158): returns the new log_num_blocks; the folded
// filter occupies words[0 .. 2^new).
int rpt_oracle_fold(uint64_t* words, int log_nb) {
  constexpr int kMinLog = 4;
  for (;;) {
    if (log_nb <= kMinLog) break;
    const int64_t nb = 1LL << log_nb;
    const int64_t num_bits = nb * 64;
    const int64_t set = static_cast<int64_t>(rpt_oracle_count_bits(words, static_cast<uint64_t>(nb)));
    if (4 * set >= num_bits) break;
    int folds = 1;
    while ((log_nb - folds) > kMinLog && (4 * set) < (num_bits >> folds)) ++folds;
    const int64_t slices = 1LL << folds;
    const int64_t slice_blocks = nb >> folds;
    for (int64_t s = 1; s < slices; ++s)
      for (int64_t i = 0; i < slice_blocks; ++i) words[i] |= words[s * slice_blocks + i];
    log_nb -= folds;
  }
  return log_nb;
}

// ---- synthetic workload --------------------------------------------------------
uint64_t rpt_oracle_sm64(uint64_t seed, uint64_t i) { return sm64(seed, i); }
void rpt_oracle_synth_build_keys(uint64_t start, uint64_t n, int64_t* out) {
  for (uint64_t i = 0; i < n; i++) out[i] = static_cast<int64_t>(sm64(kSeedBuild, start + i));
}
void rpt_oracle_synth_probe_keys(uint64_t n_build, uint32_t p_permille, uint64_t start, uint64_t n, int64_t* out) {
  for (uint64_t i = 0; i < n; i++) out[i] = synth_probe_key(n_build, p_permille, start + i);
}

// ---- CPU baseline: morsel-parallel build / probe (2048-row vectors) -------------------------
// Keys are a pre-generated host array (the sample); hashing is inside the timed region, as in
// PTBloomFilter::Insert / LookupSel (bloom_filter.cpp:66-67,76-77). Returns wall seconds.
// Filters above 256 KiB prefetch each row's block while the vector is hashed, as Arrow's Find does
// (bloom_filter.h:220-224): per core this matches libarrow_acero's Find (cpu_crosscheck.sh), so the
// baseline is not a strawman.
// Thread placement of the CPU baseline: 0 = the OS places the threads (the default); 1 = thread
// t is pinned to the t-th CPU of the process's affinity mask, in mask order (on the GPU box's EPYC: consecutive
// physical cores of one CCD, then the next); 2 = thread t to the (t * stride)-th CPU, spreading the threads over the
// whole mask. The box grants 16 CPUs of quota with an affinity of all 256 hardware threads.
static std::atomic<int> g_pin_mode{0};
void rpt_oracle_set_pin_mode(int mode) { g_pin_mode.store(mode); }
static void pin_thread(int t, int threads) {
  const int mode = g_pin_mode.load();
  if (mode == 0) return;
  cpu_set_t all;
  CPU_ZERO(&all);
  if (sched_getaffinity(0, sizeof all, &all) != 0) return;
  std::vector<int> cpus;
  for (int c = 0; c < CPU_SETSIZE; c++)
    if (CPU_ISSET(c, &all)) cpus.push_back(c);
  if (cpus.empty()) return;
  const size_t stride = mode == 2 ? std::max<size_t>(1, cpus.size() / static_cast<size_t>(std::max(1, threads))) : 1;
  cpu_set_t one;
  CPU_ZERO(&one);
  CPU_SET(cpus[(static_cast<size_t>(t) * stride) % cpus.size()], &one);
  (void)pthread_setaffinity_np(pthread_self(), sizeof one, &one);
}

constexpr uint64_t kPrefetchMinWords = (256u << 10) / 8;
double rpt_oracle_build_mt(uint64_t* words, int log_nb, const int64_t* keys, uint64_t n, int threads) {
  const uint64_t nb = 1ULL << log_nb;
  std::atomic<uint64_t> next{0};
  auto t0 = std::chrono::steady_clock::now();
  std::vector<std::thread> ts;
  for (int t = 0; t < std::max(1, threads); t++) {
    ts.emplace_back([&, t] {
      pin_thread(t, threads);
      uint64_t hashes[kVectorSize];
      for (;;) {
        uint64_t base = next.fetch_add(kVectorSize, std::memory_order_relaxed);
        if (base >= n) break;
        uint64_t cnt = std::min<uint64_t>(kVectorSize, n - base);
        for (uint64_t i = 0; i < cnt; i++) {
          hashes[i] = murmur64(static_cast<uint64_t>(keys[base + i]));
          if (nb > kPrefetchMinWords) __builtin_prefetch(&words[block_of(hashes[i], nb)], 1);
        }
        for (uint64_t i = 0; i < cnt; i++) {
          uint64_t h = hashes[i];
          __atomic_fetch_or(&words[block_of(h, nb)], mask_of(h), __ATOMIC_RELAXED);
        }
      }
    });
  }
  for (auto& t : ts) t.join();
  return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}

// Probe: per 2048-row vector hash -> LookupHashes into a per-thread SelectionVector
// (physical_use_bf.hpp:16,23): the filter loop below with one filter. Until r05 it had a loop of its own, the
// shape of rpt_oracle_set_probe_lag(2048), which ran at half this rate at 16 threads on r05's box; on r06's boxes it
// is 1.4-1.8x faster. Which distance wins depends on the host's thread placement and neighbours, not on the loop
// ("Why the CPU baseline moved 2x"), so bench.py runs both. The survivors are counted (*out_count).
double rpt_oracle_probe_chain_mt(const uint64_t* const* words, const int* log_nb, const int64_t* const* keys, int k,
                                 uint64_t n, int threads, uint64_t* out_count);
double rpt_oracle_probe_mt(const uint64_t* words, int log_nb, const int64_t* keys, uint64_t n, int threads,
                           uint64_t* out_count) {
  return rpt_oracle_probe_chain_mt(&words, &log_nb, &keys, 1, n, threads, out_count);
}

// USE_BF's filter loop per vector (physical_use_bf.cpp:137-183): filter 0 over every row of the vector, each
// further filter over the previous one's survivors (its own key column, same rows), stopping when none are left;
// per 2048-row vector on `threads` threads, hash included. The final survivors are counted (*out_count).
// Rows between a row's hash + prefetch and its filter test (default 24; set for the prefetch-distance sweep of
// 2048 = the whole vector hashed and prefetched before any row is tested, the pre-r05 loop).
static std::atomic<uint64_t> g_probe_lag{24};
void rpt_oracle_set_probe_lag(uint64_t lag) { g_probe_lag.store(lag ? lag : 24); }
uint64_t rpt_oracle_probe_lag(void) { return g_probe_lag.load(); }

double rpt_oracle_probe_chain_mt(const uint64_t* const* words, const int* log_nb, const int64_t* const* keys, int k,
                                 uint64_t n, int threads, uint64_t* out_count) {
  const uint64_t kLag = g_probe_lag.load();
  std::atomic<uint64_t> next{0};
  std::atomic<uint64_t> total{0};
  auto t0 = std::chrono::steady_clock::now();
  std::vector<std::thread> ts;
  for (int t = 0; t < std::max(1, threads); t++) {
    ts.emplace_back([&, t] {
      pin_thread(t, threads);
      uint64_t hashes[kVectorSize];
      uint32_t sel[kVectorSize];
      uint64_t local = 0;
      for (;;) {
        const uint64_t base = next.fetch_add(kVectorSize, std::memory_order_relaxed);
        if (base >= n) break;
        uint64_t cnt = std::min<uint64_t>(kVectorSize, n - base);
        for (uint32_t i = 0; i < cnt; i++) sel[i] = i;
        for (int f = 0; f < k && cnt > 0; f++) {
          const uint64_t nb = 1ULL << log_nb[f];
          const uint64_t* w = words[f];
          const int64_t* kf = keys[f] + base;
          uint64_t c = 0;
          auto test = [&](uint64_t j) {  // j: index into the current survivors
            const uint64_t h = hashes[j], m = mask_of(h);
            sel[c] = sel[j];
            c += (w[block_of(h, nb)] & m) == m;
          };
          for (uint64_t j = 0; j < cnt; j++) {
            hashes[j] = murmur64(static_cast<uint64_t>(kf[sel[j]]));
            __builtin_prefetch(&w[block_of(hashes[j], nb)]);
            if (j >= kLag) test(j - kLag);
          }
          for (uint64_t j = cnt > kLag ? cnt - kLag : 0; j < cnt; j++) test(j);
          cnt = c;
        }
        local += cnt;
        asm volatile("" ::"r"(sel) : "memory");
      }
      total.fetch_add(local);
    });
  }
  for (auto& t : ts) t.join();
  double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  if (out_count) *out_count = total.load();
  return s;
}

}  // extern "C"
