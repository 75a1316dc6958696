// rpt_host.cpp — C++ host mirror of PTBloomFilter / PhysicalCreateBF / PhysicalUseBF over the
// C-ABI (include/rpt_host.hpp). Host-side only: every device operation goes through rpt_gpu.h.
#include "rpt_host.hpp"

#include <hip/hip_runtime_api.h>
#include <emmintrin.h>  // SSE2 streaming stores (x86-64 baseline) for the pinned staging copies
#include <immintrin.h>  // AVX-512 / AVX2 paths (runtime-dispatched): narrow-key packing, bit expansion

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <exception>
#include <limits>
#include <map>
#include <thread>
#include <utility>

namespace rpt {

namespace {

void check(int status) {
  if (status != RPT_OK) throw GpuError(status, std::string("librpt_gpu: ") + rpt_last_error());
}

void check_hip(hipError_t e, const char* what) {
  if (e != hipSuccess) throw GpuError(RPT_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
}

struct DeviceScope {
  int prev = -1, dev;
  explicit DeviceScope(int d) : dev(d) {
    check_hip(hipGetDevice(&prev), "hipGetDevice");
    if (prev != d) check_hip(hipSetDevice(d), "hipSetDevice");
  }
  ~DeviceScope() {
    if (prev >= 0 && prev != dev) (void)hipSetDevice(prev);
  }
};

// Bytes per key of a device column (I32 / I64) or of a host column of any KeyType.
size_t key_size(KeyType t) { return t == KeyType::I32 ? 4 : 8; }
size_t source_size(KeyType t) {
  switch (t) {
    case KeyType::I8:
    case KeyType::U8: return 1;
    case KeyType::I16:
    case KeyType::U16: return 2;
    case KeyType::I32:
    case KeyType::U32:
    case KeyType::F32: return 4;
    default: return 8;
  }
}
// The device key type a host column is staged as (rpt_host.hpp, KeyType).
KeyType device_type(KeyType t) {
  switch (t) {
    case KeyType::I8:
    case KeyType::I16:
    case KeyType::U8:
    case KeyType::U16:
    case KeyType::I32:
    case KeyType::F32: return KeyType::I32;
    default: return KeyType::I64;
  }
}
bool keeps_minmax(KeyType t) { return t != KeyType::U64 && t != KeyType::F32 && t != KeyType::F64; }

// One host key (its source bytes) -> its device value: what DuckDB's Hash<T> hashes (rpt_host.hpp KeyType).
uint64_t device_value(KeyType t, const uint8_t* p) {
  switch (t) {
    case KeyType::I8: { int8_t v; std::memcpy(&v, p, 1); return static_cast<uint32_t>(static_cast<int32_t>(v)); }
    case KeyType::I16: { int16_t v; std::memcpy(&v, p, 2); return static_cast<uint32_t>(static_cast<int32_t>(v)); }
    case KeyType::U8: return p[0];
    case KeyType::U16: { uint16_t v; std::memcpy(&v, p, 2); return v; }
    case KeyType::I32:
    case KeyType::U32: { uint32_t v; std::memcpy(&v, p, 4); return v; }
    case KeyType::F32: {
      float v;
      std::memcpy(&v, p, 4);
      if (v == 0.0f) v = 0.0f;                                        // -0.0 -> 0.0
      else if (v != v) v = std::numeric_limits<float>::quiet_NaN();   // every NaN -> the quiet NaN
      uint32_t b;
      std::memcpy(&b, &v, 4);
      return b;
    }
    case KeyType::F64: {
      double v;
      std::memcpy(&v, p, 8);
      if (v == 0.0) v = 0.0;
      else if (v != v) v = std::numeric_limits<double>::quiet_NaN();
      uint64_t b;
      std::memcpy(&b, &v, 8);
      return b;
    }
    default: { uint64_t v; std::memcpy(&v, p, 8); return v; }
  }
}

bool valid_bit(const uint64_t* validity, uint64_t idx) {
  return validity == nullptr || ((validity[idx >> 6] >> (idx & 63)) & 1ULL);
}

// Clear the validity bits of the NULL rows in `nulls` (LSB = row g0) at rows [g0, g0 + n), n <= 64, in
// words preset to all-valid. Words at a chunk's edges may be shared with a neighbouring chunk that
// another thread flattens: those ANDs are atomic.
void clear_bits(uint64_t* words, uint64_t g0, uint64_t nulls, uint32_t n) {
  if (n < 64) nulls &= (1ULL << n) - 1;
  if (!nulls) return;
  const uint64_t w = g0 >> 6, sh = g0 & 63;
  __atomic_fetch_and(&words[w], ~(nulls << sh), __ATOMIC_RELAXED);
  if (sh && sh + n > 64) __atomic_fetch_and(&words[w + 1], ~(nulls >> (64 - sh)), __ATOMIC_RELAXED);
}

// Bits [r, r + n) (n <= 64) of a DuckDB validity mask (nullptr = all valid).
uint64_t mask_bits(const uint64_t* validity, uint64_t r, uint32_t n) {
  if (!validity) return n >= 64 ? ~0ULL : (1ULL << n) - 1;
  const uint64_t w = r >> 6, sh = r & 63;
  uint64_t b = validity[w] >> sh;
  if (sh && sh + n > 64) b |= validity[w + 1] << (64 - sh);
  return n >= 64 ? b : b & ((1ULL << n) - 1);
}

// A column whose keys must be converted on the way to the device (everything but I32 / I64) into `keys` as
// device values, its NULL rows cleared in `valid_words` as flatten_column does.
bool flatten_converted(const Vector& v, uint64_t count, uint8_t* keys, uint64_t* valid_words, uint64_t row0) {
  const size_t ss = source_size(v.key_type), ds = key_size(device_type(v.key_type));
  const uint8_t* src = static_cast<const uint8_t*>(v.data);
  bool any_null = false;
  for (uint64_t r = 0; r < count; r += 64) {
    const uint32_t n = static_cast<uint32_t>(std::min<uint64_t>(64, count - r));
    uint64_t nulls = 0;
    for (uint32_t e = 0; e < n; e++) {
      uint64_t idx = r + e, x = 0;
      uint8_t seq[8];
      const uint8_t* p;
      if (v.type == VectorType::SEQUENCE) {  // start + row * increment, wrapped to the column's width
        x = static_cast<uint64_t>(v.seq_start) + static_cast<uint64_t>(v.seq_increment) * idx;
        std::memcpy(seq, &x, 8);             // little-endian: the low bytes are the narrower value
        p = seq;
      } else {
        if (v.type == VectorType::CONSTANT) idx = 0;
        else if (v.type == VectorType::DICTIONARY) {
          idx = v.sel[r + e];
          if (idx >= v.dict_size) throw GpuError(RPT_ERR_INVALID_ARGUMENT, "dictionary index out of range");
        }
        p = src + idx * ss;
        nulls |= static_cast<uint64_t>(!valid_bit(v.validity, idx)) << e;
      }
      const uint64_t d = device_value(v.key_type, p);
      std::memcpy(keys + (r + e) * ds, &d, ds);  // little-endian: an I32 device value is the low 4 bytes
    }
    any_null |= nulls != 0;
    clear_bits(valid_words, row0 + r, nulls, n);
  }
  return any_null;
}

// A FLAT vector's bytes into pinned staging memory the device will read by DMA: streaming (non-temporal)
// 16-B stores, which skip the read-for-ownership of every destination line a plain memcpy of a 16 KiB vector
// does (the staging buffer is not read back by the host), then a store fence so the DMA sees the bytes.
void copy_to_staging(uint8_t* dst, const void* src_v, size_t bytes) {
  const uint8_t* src = static_cast<const uint8_t*>(src_v);
  const size_t head = std::min(bytes, static_cast<size_t>((16 - (reinterpret_cast<uintptr_t>(dst) & 15)) & 15));
  if (bytes < 256) {
    std::memcpy(dst, src, bytes);
    return;
  }
  std::memcpy(dst, src, head);
  dst += head;
  src += head;
  bytes -= head;
  size_t i = 0;
  for (; i + 64 <= bytes; i += 64) {
    const __m128i a = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + i));
    const __m128i b = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + i + 16));
    const __m128i c = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + i + 32));
    const __m128i d = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + i + 48));
    _mm_stream_si128(reinterpret_cast<__m128i*>(dst + i), a);
    _mm_stream_si128(reinterpret_cast<__m128i*>(dst + i + 16), b);
    _mm_stream_si128(reinterpret_cast<__m128i*>(dst + i + 32), c);
    _mm_stream_si128(reinterpret_cast<__m128i*>(dst + i + 48), d);
  }
  std::memcpy(dst + i, src + i, bytes - i);
  _mm_sfence();
}

// A DICTIONARY vector's keys gathered through its selection (element type T: the column's own width), 64 rows
// per step: the index bound is checked once per step (the largest index), NULLs only when the dictionary has a
// validity mask.
template <typename T>
bool flatten_dictionary(const Vector& v, uint64_t count, uint8_t* keys, uint64_t* valid_words, uint64_t row0) {
  const T* src = static_cast<const T*>(v.data);
  T* dst = reinterpret_cast<T*>(keys);
  bool any_null = false;
  for (uint64_t r = 0; r < count; r += 64) {
    const uint32_t n = static_cast<uint32_t>(std::min<uint64_t>(64, count - r));
    const uint32_t* sel = v.sel + r;
    uint32_t kmax = 0;
    for (uint32_t e = 0; e < n; e++) kmax = std::max(kmax, sel[e]);
    if (kmax >= v.dict_size) throw GpuError(RPT_ERR_INVALID_ARGUMENT, "dictionary index out of range");
    for (uint32_t e = 0; e < n; e++) {
      T x;
      std::memcpy(&x, src + sel[e], sizeof(T));
      std::memcpy(dst + r + e, &x, sizeof(T));
    }
    if (v.validity) {
      uint64_t nulls = 0;
      for (uint32_t e = 0; e < n; e++) nulls |= static_cast<uint64_t>(!valid_bit(v.validity, sel[e])) << e;
      any_null |= nulls != 0;
      clear_bits(valid_words, row0 + r, nulls, n);
    }
  }
  return any_null;
}

// Flatten one column of `chunk` (FLAT / CONSTANT / DICTIONARY / SEQUENCE) into `keys` and clear the bits of
// its NULL rows at row offset `row0` of `valid_words` (preset to all-valid: a chunk without NULLs touches
// no validity word), 64 rows per step. Returns true if any row was NULL. to_device: keys are device values
// (key_size(device_type) bytes each: converted for the non-I32/I64 types); else the column's own values
// (source_size bytes: the materialized copy the CREATE_BF source re-emits).
bool flatten_column(const Vector& v, uint64_t count, uint8_t* keys, uint64_t* valid_words, uint64_t row0,
                    bool to_device = true) {
  if (to_device && device_type(v.key_type) != v.key_type) return flatten_converted(v, count, keys, valid_words, row0);
  const size_t es = source_size(v.key_type);
  bool any_null = false;
  switch (v.type) {
    case VectorType::FLAT:
      copy_to_staging(keys, v.data, count * es);
      if (v.validity) {
        for (uint64_t r = 0; r < count; r += 64) {
          const uint32_t n = static_cast<uint32_t>(std::min<uint64_t>(64, count - r));
          const uint64_t nulls = ~mask_bits(v.validity, r, n) & (n == 64 ? ~0ULL : (1ULL << n) - 1);
          any_null |= nulls != 0;
          clear_bits(valid_words, row0 + r, nulls, n);
        }
      }
      break;
    case VectorType::CONSTANT: {
      for (uint64_t r = 0; r < count; r++) std::memcpy(keys + r * es, v.data, es);
      if (!valid_bit(v.validity, 0) && count > 0) {
        any_null = true;
        for (uint64_t r = 0; r < count; r += 64) clear_bits(valid_words, row0 + r, ~0ULL, static_cast<uint32_t>(std::min<uint64_t>(64, count - r)));
      }
      break;
    }
    case VectorType::DICTIONARY:
      switch (es) {  // a fixed-size element per row: the gather compiles to plain loads and stores
        case 1: any_null = flatten_dictionary<uint8_t>(v, count, keys, valid_words, row0); break;
        case 2: any_null = flatten_dictionary<uint16_t>(v, count, keys, valid_words, row0); break;
        case 4: any_null = flatten_dictionary<uint32_t>(v, count, keys, valid_words, row0); break;
        default: any_null = flatten_dictionary<uint64_t>(v, count, keys, valid_words, row0); break;
      }
      break;
    case VectorType::SEQUENCE: {  // start + r * increment in two's complement (wraps as DuckDB's)
      uint64_t x = static_cast<uint64_t>(v.seq_start);
      const uint64_t inc = static_cast<uint64_t>(v.seq_increment);
      for (uint64_t r = 0; r < count; r++, x += inc) std::memcpy(keys + r * es, &x, es);  // little-endian
      break;
    }
  }
  return any_null;
}

// Column `col` of `chunks` flattened into the context's pinned staging buffers (slots 0/1).
struct Flattened {
  KeyType key_type;
  const uint8_t* keys;
  const uint64_t* valid;
  bool any_null;
  // narrow: BIGINT keys as 4-B low words, meta = each chunk's high word [n_chunks] then the chunks' first rows
  // [n_chunks + 1] (uint32), widened on the device (rpt_keys_widen)
  bool narrow = false;
  const uint32_t* meta = nullptr;
  uint64_t n_chunks = 0;
};

// FLAT BIGINT keys src[0 .. count) -> their low words at lo; returns true when they all share one high word
// (every bit of the high words equal: their OR equals their AND), which *hi then holds. One pass: the check
// accumulates while the low words are stored. AVX-512 (vpmovqd) or AVX2 where the host has them (runtime
// dispatch; the GPU box's EPYC 9575F has both), SSE2 otherwise.
__attribute__((target("avx512f"))) bool narrow_flat_avx512(const int64_t* src, uint64_t count, uint32_t* lo, uint32_t* hi) {
  __m512i o = _mm512_setzero_si512(), n = _mm512_set1_epi64(-1);
  const bool aligned = (reinterpret_cast<uintptr_t>(lo) & 31) == 0;
  uint64_t r = 0;
  for (; r + 8 <= count; r += 8) {
    const __m512i v = _mm512_loadu_si512(src + r);
    o = _mm512_or_si512(o, v);
    n = _mm512_and_si512(n, v);
    const __m256i packed = _mm512_cvtepi64_epi32(v);  // the low dwords
    if (aligned) _mm256_stream_si256(reinterpret_cast<__m256i*>(lo + r), packed);
    else _mm256_storeu_si256(reinterpret_cast<__m256i*>(lo + r), packed);
  }
  uint64_t so = static_cast<uint64_t>(_mm512_reduce_or_epi64(o)), sn = static_cast<uint64_t>(_mm512_reduce_and_epi64(n));
  for (; r < count; r++) {
    const uint64_t k = static_cast<uint64_t>(src[r]);
    so |= k;
    sn &= k;
    lo[r] = static_cast<uint32_t>(k);
  }
  if (aligned) _mm_sfence();
  *hi = static_cast<uint32_t>(so >> 32);
  return (so >> 32) == (sn >> 32);
}

__attribute__((target("avx2"))) bool narrow_flat_avx2(const int64_t* src, uint64_t count, uint32_t* lo, uint32_t* hi) {
  const __m256i even = _mm256_setr_epi32(0, 2, 4, 6, 1, 3, 5, 7);
  __m256i o = _mm256_setzero_si256(), n = _mm256_set1_epi64x(-1);
  const bool aligned = (reinterpret_cast<uintptr_t>(lo) & 31) == 0;
  uint64_t r = 0;
  for (; r + 8 <= count; r += 8) {
    const __m256i a = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(src + r));
    const __m256i b = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(src + r + 4));
    o = _mm256_or_si256(o, _mm256_or_si256(a, b));
    n = _mm256_and_si256(n, _mm256_and_si256(a, b));
    // low dwords of a into the low 128 bits, of b into the high 128 bits
    const __m256i packed = _mm256_permute2x128_si256(_mm256_permutevar8x32_epi32(a, even),
                                                     _mm256_permutevar8x32_epi32(b, even), 0x20);
    if (aligned) _mm256_stream_si256(reinterpret_cast<__m256i*>(lo + r), packed);
    else _mm256_storeu_si256(reinterpret_cast<__m256i*>(lo + r), packed);
  }
  alignas(32) uint64_t ov[4], nv[4];
  _mm256_store_si256(reinterpret_cast<__m256i*>(ov), o);
  _mm256_store_si256(reinterpret_cast<__m256i*>(nv), n);
  uint64_t so = ov[0] | ov[1] | ov[2] | ov[3], sn = nv[0] & nv[1] & nv[2] & nv[3];
  for (; r < count; r++) {
    const uint64_t k = static_cast<uint64_t>(src[r]);
    so |= k;
    sn &= k;
    lo[r] = static_cast<uint32_t>(k);
  }
  if (aligned) _mm_sfence();
  *hi = static_cast<uint32_t>(so >> 32);
  return (so >> 32) == (sn >> 32);
}

bool narrow_flat_sse2(const int64_t* src, uint64_t count, uint32_t* lo, uint32_t* hi) {
  __m128i o = _mm_setzero_si128(), n = _mm_set1_epi64x(-1);
  const bool aligned = (reinterpret_cast<uintptr_t>(lo) & 15) == 0;
  uint64_t r = 0;
  for (; r + 4 <= count; r += 4) {
    const __m128i a = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + r));
    const __m128i b = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + r + 2));
    o = _mm_or_si128(o, _mm_or_si128(a, b));
    n = _mm_and_si128(n, _mm_and_si128(a, b));
    // the low dwords of a and b -> one 16-B store
    const __m128i packed = _mm_unpacklo_epi64(_mm_shuffle_epi32(a, _MM_SHUFFLE(2, 0, 2, 0)),
                                              _mm_shuffle_epi32(b, _MM_SHUFFLE(2, 0, 2, 0)));
    if (aligned) _mm_stream_si128(reinterpret_cast<__m128i*>(lo + r), packed);
    else _mm_storeu_si128(reinterpret_cast<__m128i*>(lo + r), packed);
  }
  alignas(16) uint64_t ov[2], nv[2];
  _mm_store_si128(reinterpret_cast<__m128i*>(ov), o);
  _mm_store_si128(reinterpret_cast<__m128i*>(nv), n);
  uint64_t so = ov[0] | ov[1], sn = nv[0] & nv[1];
  for (; r < count; r++) {
    const uint64_t k = static_cast<uint64_t>(src[r]);
    so |= k;
    sn &= k;
    lo[r] = static_cast<uint32_t>(k);
  }
  if (aligned) _mm_sfence();
  *hi = static_cast<uint32_t>(so >> 32);
  return (so >> 32) == (sn >> 32);
}

// 2: AVX-512F, 1: AVX2, 0: SSE2 (cpu_init first: a static initializer may run before the runtime's)
int simd_level() {
  static const int level = [] {
    __builtin_cpu_init();
    return __builtin_cpu_supports("avx512f") ? 2 : __builtin_cpu_supports("avx2") ? 1 : 0;
  }();
  return level;
}

// One chunk's BIGINT keys as their low 32-bit words at `lo` and the high word they all share in *hi, NULL rows
// cleared in `valid_words` from bit row0 on (as flatten_column). False when the keys do not share their high word:
// `lo` and the validity bits are then partly written and the caller re-flattens.
bool narrow_column(const Vector& v, uint64_t count, uint32_t* lo, uint32_t* hi, uint64_t* valid_words, uint64_t row0,
                   bool& any_null) {
  if (v.key_type != KeyType::I64 || count == 0) return count == 0 && v.key_type == KeyType::I64;
  const int64_t* src = static_cast<const int64_t*>(v.data);
  switch (v.type) {
    case VectorType::FLAT: {
      const int lvl = simd_level();
      if (!(lvl == 2 ? narrow_flat_avx512(src, count, lo, hi)
                     : lvl == 1 ? narrow_flat_avx2(src, count, lo, hi) : narrow_flat_sse2(src, count, lo, hi)))
        return false;
      if (v.validity) {
        for (uint64_t q = 0; q < count; q += 64) {
          const uint32_t n = static_cast<uint32_t>(std::min<uint64_t>(64, count - q));
          const uint64_t nulls = ~mask_bits(v.validity, q, n) & (n == 64 ? ~0ULL : (1ULL << n) - 1);
          any_null |= nulls != 0;
          clear_bits(valid_words, row0 + q, nulls, n);
        }
      }
      return true;
    }
    case VectorType::CONSTANT: {
      const uint64_t k = static_cast<uint64_t>(src[0]);
      std::fill(lo, lo + count, static_cast<uint32_t>(k));
      *hi = static_cast<uint32_t>(k >> 32);
      if (!valid_bit(v.validity, 0)) {
        any_null = true;
        for (uint64_t q = 0; q < count; q += 64) clear_bits(valid_words, row0 + q, ~0ULL, static_cast<uint32_t>(std::min<uint64_t>(64, count - q)));
      }
      return true;
    }
    case VectorType::DICTIONARY: {
      if (v.dict_size == 0) throw GpuError(RPT_ERR_INVALID_ARGUMENT, "dictionary index out of range");
      const uint64_t v0 = static_cast<uint64_t>(src[v.sel[0] < v.dict_size ? v.sel[0] : 0]);
      uint64_t acc = 0;
      for (uint64_t q = 0; q < count; q += 64) {
        const uint32_t n = static_cast<uint32_t>(std::min<uint64_t>(64, count - q));
        const uint32_t* sel = v.sel + q;
        uint32_t kmax = 0;
        for (uint32_t e = 0; e < n; e++) kmax = std::max(kmax, sel[e]);
        if (kmax >= v.dict_size) throw GpuError(RPT_ERR_INVALID_ARGUMENT, "dictionary index out of range");
        for (uint32_t e = 0; e < n; e++) {
          const uint64_t k = static_cast<uint64_t>(src[sel[e]]);
          acc |= (k ^ v0) >> 32;
          lo[q + e] = static_cast<uint32_t>(k);
        }
        if (v.validity) {
          uint64_t nulls = 0;
          for (uint32_t e = 0; e < n; e++) nulls |= static_cast<uint64_t>(!valid_bit(v.validity, sel[e])) << e;
          any_null |= nulls != 0;
          clear_bits(valid_words, row0 + q, nulls, n);
        }
      }
      if (acc != 0) return false;
      *hi = static_cast<uint32_t>(v0 >> 32);
      return true;
    }
    case VectorType::SEQUENCE: {  // start + r * increment in two's complement, never NULL
      const uint64_t v0 = static_cast<uint64_t>(v.seq_start), inc = static_cast<uint64_t>(v.seq_increment);
      uint64_t acc = 0, k = v0;
      for (uint64_t r = 0; r < count; r++, k += inc) {
        acc |= (k ^ v0) >> 32;
        lo[r] = static_cast<uint32_t>(k);
      }
      if (acc != 0) return false;
      *hi = static_cast<uint32_t>(v0 >> 32);
      return true;
    }
    default:
      return false;
  }
}

// Column `col` of chunks[0 .. n_chunks) (total rows) into pinned slots `slot` (keys) and `valid_slot` (validity
// words; default slot + 1).
Flattened flatten_pinned(DeviceContext& ctx, const DataChunk* const* chunks, size_t n_chunks, uint64_t col,
                         uint64_t total, int slot, int valid_slot = -1, int narrow_slot = -1) {
  if (valid_slot < 0) valid_slot = slot + 1;
  if (n_chunks == 0) throw GpuError(RPT_ERR_INVALID_ARGUMENT, "no chunks");
  const Vector& v0 = chunks[0]->data.at(col);
  const size_t es = key_size(device_type(v0.key_type));
  const uint64_t nwords = (total + 63) / 64;
  auto* hkeys = static_cast<uint8_t*>(ctx.host(slot, std::max<size_t>(total * es, 16)));
  auto* hvalid = static_cast<uint64_t*>(ctx.host(valid_slot, std::max<size_t>(nwords * 8, 8)));
  std::vector<uint64_t> row0(n_chunks + 1, 0);
  for (size_t i = 0; i < n_chunks; i++) {
    if (chunks[i]->data.at(col).key_type != v0.key_type)
      throw GpuError(RPT_ERR_INVALID_ARGUMENT, "mixed key types in one column");
    row0[i + 1] = row0[i] + chunks[i]->count;
  }
  const bool big = total >= (1u << 17) && n_chunks >= 16 && ctx.flatten_threads > 1;  // from 128 Ki rows (a ramp stage)
  const size_t n_tasks = big ? std::min<size_t>(n_chunks / 4, 4 * static_cast<size_t>(ctx.flatten_threads)) : 1;
  // narrow BIGINT keys: every chunk's keys share their high word -> 4 B per key over PCIe (else the plain flatten
  // below, after this attempt's partial writes)
  if (narrow_slot >= 0 && v0.key_type == KeyType::I64 && total < (1ULL << 32)) {
    std::memset(hvalid, 0xFF, nwords * 8);
    auto* lo = reinterpret_cast<uint32_t*>(hkeys);
    auto* meta = static_cast<uint32_t*>(ctx.host(narrow_slot, (2 * n_chunks + 1) * 4));
    for (size_t i = 0; i <= n_chunks; i++) meta[n_chunks + i] = static_cast<uint32_t>(row0[i]);
    std::atomic<bool> ok{true};
    std::vector<char> nulls(n_tasks, 0);
    auto range = [&](size_t t) {
      bool nl = false;
      for (size_t i = n_chunks * t / n_tasks; i < n_chunks * (t + 1) / n_tasks && ok.load(std::memory_order_relaxed); i++)
        if (!narrow_column(chunks[i]->data.at(col), chunks[i]->count, lo + row0[i], meta + i, hvalid, row0[i], nl))
          ok.store(false, std::memory_order_relaxed);
      nulls[t] = nl ? 1 : 0;
    };
    if (n_tasks == 1) range(0);
    else ctx.parallel_for(n_tasks, range);
    if (ok.load()) {
      Flattened f{KeyType::I64, hkeys, hvalid, false};
      for (char c : nulls) f.any_null |= c != 0;
      f.narrow = true;
      f.meta = meta;
      f.n_chunks = n_chunks;
      return f;
    }
  }
  std::memset(hvalid, 0xFF, nwords * 8);  // all valid; flatten_column clears the NULL rows
  // Flattening into the pinned staging buffer is the host side's bottleneck for large batches; big
  // batches are split over ctx.flatten_threads threads by chunk.
  auto flatten_range = [&](size_t lo, size_t hi) {
    bool nulls = false;
    for (size_t i = lo; i < hi; i++)
      nulls |= flatten_column(chunks[i]->data.at(col), chunks[i]->count, hkeys + row0[i] * es, hvalid, row0[i]);
    return nulls;
  };
  bool any_null = false;
  if (!big) {
    any_null = flatten_range(0, n_chunks);
  } else {
    // several ranges per worker thread, so uneven chunks (dictionaries, conversions) still balance
    std::vector<char> nulls(n_tasks, 0);
    ctx.parallel_for(n_tasks, [&](size_t t) {
      nulls[t] = flatten_range(n_chunks * t / n_tasks, n_chunks * (t + 1) / n_tasks) ? 1 : 0;
    });
    for (char c : nulls) any_null |= c != 0;
  }
  return Flattened{device_type(v0.key_type), hkeys, hvalid, any_null};
}

// Copy a flattened column to device buffers (dvalid is only written when the batch had NULLs), on `stream`
// (default: the context's).
rpt_key_column copy_flattened(DeviceContext& ctx, const Flattened& f, uint64_t total, void* dkeys, void* dvalid,
                              void* stream = nullptr, void* d_lo = nullptr, void* d_meta = nullptr) {
  auto s = static_cast<hipStream_t>(stream ? stream : ctx.stream());
  if (f.narrow) {  // 4-B low words + the chunks' high words and first rows, widened into dkeys
    if (!d_lo || !d_meta) throw GpuError(RPT_ERR_INVALID_ARGUMENT, "narrow keys without device staging");
    check_hip(hipMemcpyAsync(d_lo, f.keys, total * 4, hipMemcpyHostToDevice, s), "stage keys");
    check_hip(hipMemcpyAsync(d_meta, f.meta, (2 * f.n_chunks + 1) * 4, hipMemcpyHostToDevice, s), "stage chunk words");
    const auto* m = static_cast<const uint32_t*>(d_meta);
    check(rpt_keys_widen(static_cast<const uint32_t*>(d_lo), m, m + f.n_chunks, f.n_chunks, static_cast<uint64_t*>(dkeys), s));
  } else {
    check_hip(hipMemcpyAsync(dkeys, f.keys, total * key_size(f.key_type), hipMemcpyHostToDevice, s), "stage keys");
  }
  if (f.any_null)
    check_hip(hipMemcpyAsync(dvalid, f.valid, (total + 63) / 64 * 8, hipMemcpyHostToDevice, s), "stage validity");
  rpt_key_column kc;
  kc.key_type = static_cast<int32_t>(f.key_type);
  kc.keys = dkeys;
  kc.key_sel = nullptr;
  kc.validity = f.any_null ? static_cast<const uint64_t*>(dvalid) : nullptr;
  return kc;
}

// Stage column `col` of `chunks` to the device as one flat key column (slots 0/1 of the context).
rpt_key_column stage(DeviceContext& ctx, const std::vector<const DataChunk*>& chunks, uint64_t col, uint64_t total) {
  const Flattened f = flatten_pinned(ctx, chunks.data(), chunks.size(), col, total, 0);
  void* dkeys = ctx.dev(0, std::max<size_t>(total * key_size(f.key_type), 16));
  void* dvalid = ctx.dev(1, std::max<size_t>((total + 63) / 64 * 8, 8));
  return copy_flattened(ctx, f, total, dkeys, dvalid);
}

uint64_t total_rows(const std::vector<const DataChunk*>& chunks) {
  uint64_t t = 0;
  for (const DataChunk* c : chunks) t += c->count;
  return t;
}

// The key column(s) of a filter on the device. One column (the hot path: physical_create_bf.cpp:225,
// 403, physical_use_bf.cpp:163) is staged as is and hashed inside the insert / probe kernels. Several
// columns are HashColumns' composite key (bloom_filter.cpp:11-24): Hash(col_0), then CombineHash
// with each further column, into a device hash column (slot 5) that is inserted / probed as
// RPT_KEY_HASH.
rpt_key_column stage_key(DeviceContext& ctx, const std::vector<const DataChunk*>& chunks,
                         const std::vector<uint64_t>& cols, uint64_t total) {
  if (cols.empty()) throw GpuError(RPT_ERR_INVALID_ARGUMENT, "no key columns");
  if (cols.size() == 1) return stage(ctx, chunks, cols[0], total);
  auto* dh = static_cast<uint64_t*>(ctx.dev(5, total * 8));
  for (size_t j = 0; j < cols.size(); j++) {
    rpt_key_column kc = stage(ctx, chunks, cols[j], total);
    check(j == 0 ? rpt_hash_keys(&kc, total, dh, ctx.stream()) : rpt_hash_combine(&kc, total, dh, ctx.stream()));
    ctx.synchronize();  // the next column reuses the staging slots
  }
  rpt_key_column hc;
  hc.key_type = RPT_KEY_HASH;
  hc.keys = dh;
  hc.key_sel = nullptr;
  hc.validity = nullptr;
  return hc;
}


// Batches up to this many rows copy the count and the whole sel capacity back in one copy.
constexpr uint64_t kSingleCopyRows = RPT_SMALL_PROBE_ROWS;

// Whole-chunk stages of about `target` rows for the pipelined batch paths (a short tail joins the
// previous stage). Every chunk's key column must have the same key type. (Stages ramping up from target / 8 at
// the start of a batch and down at its end, to shorten the pipeline's fill and drain, were measured in r05 and
// lost: more stages cost more in per-stage fixed costs than the shorter fill and drain saved)
struct StageRange {
  size_t c_lo, c_hi;
  uint64_t rows;
};
std::vector<StageRange> pipeline_stages(const std::vector<const DataChunk*>& chunks, uint64_t col, uint64_t target) {
  std::vector<StageRange> st;
  StageRange cur{0, 0, 0};
  const KeyType kt = chunks.at(0)->data.at(col).key_type;
  for (size_t i = 0; i < chunks.size(); i++) {
    if (chunks[i]->data.at(col).key_type != kt) throw GpuError(RPT_ERR_INVALID_ARGUMENT, "mixed key types in one column");
    cur.rows += chunks[i]->count;
    cur.c_hi = i + 1;
    if (cur.rows >= target) {
      st.push_back(cur);
      cur = StageRange{i + 1, i + 1, 0};
    }
  }
  if (cur.rows > 0) {
    if (!st.empty() && cur.rows < target / 2) {
      st.back().c_hi = cur.c_hi;
      st.back().rows += cur.rows;
    } else {
      st.push_back(cur);
    }
  }
  return st;
}

// Rows per stage of a pipelined batch of `total` rows, 0 = one piece: a quarter of the batch, at least 512 Ki and at
// most DeviceContext::pipeline_rows; batches under 2 Mi rows (or two stages) run in one piece. Mid-size batches
// gain from the overlap (r05, tools/host_bench --batch-sizes, profiles/r05/host_batch_sizes.jsonl: 4 Mi-row batches
// 3.1 -> 4.0e9 rows/s, 8 Mi-row 4.1 -> 4.7e9); 1 Mi-row batches in 256 Ki stages lose to the single piece.
uint64_t stage_rows_for(const DeviceContext& ctx, uint64_t total) {
  const uint64_t cap = std::max<uint64_t>(ctx.pipeline_rows, 1), floor_rows = 1u << 19;
  const uint64_t st = std::min(cap, std::max(floor_rows, total / 4));
  return (total >= 2 * st && total >= std::min(4 * floor_rows, 2 * cap)) ? st : 0;
}

}  // namespace

// Double-buffered staging of the pipelined batch paths, sized once for the largest stage (a slot that
// grows synchronizes both streams, which must not happen mid-pipeline).
struct PTBloomFilter::PipelineBuffers {
  static constexpr int kHostKeys = 8;  // host slots 8..11: keys / validity of buffers 0 and 1
  void* d_keys[2];
  void* d_valid[2];
  uint32_t* d_sel[2];
  uint64_t* d_cnt[2];
  uint32_t* h_sel[2];
  uint64_t* h_cnt[2];
  // narrow BIGINT stages (max_chunks > 0): device slots 56 + b (4-B low words), 58 + b and host slot 56 + b (the
  // chunks' high words and first rows)
  void* d_lo[2] = {nullptr, nullptr};
  void* d_meta[2] = {nullptr, nullptr};
  static constexpr int kNarrowMeta = 56;
  DeviceContext& ctx;
  PipelineBuffers(DeviceContext& c, uint64_t max_rows, size_t key_bytes, size_t max_chunks = 0) : ctx(c) {
    const size_t words = (max_rows + 63) / 64 * 8;
    for (int b = 0; max_chunks && b < 2; b++) {
      d_lo[b] = ctx.dev(56 + b, std::max<size_t>(max_rows * 4, 16));
      d_meta[b] = ctx.dev(58 + b, (2 * max_chunks + 1) * 4);
      (void)ctx.host(kNarrowMeta + b, (2 * max_chunks + 1) * 4);
    }
    for (int b = 0; b < 2; b++) {
      (void)ctx.host(kHostKeys + 2 * b, std::max<size_t>(max_rows * key_bytes, 16));
      (void)ctx.host(kHostKeys + 2 * b + 1, std::max<size_t>(words, 8));
      h_cnt[b] = static_cast<uint64_t*>(ctx.host(12 + b, 8));
      h_sel[b] = static_cast<uint32_t*>(ctx.host(14 + b, std::max<size_t>(max_rows * 4, 4)));
      d_keys[b] = ctx.dev(8 + 2 * b, std::max<size_t>(max_rows * key_bytes, 16));
      d_valid[b] = ctx.dev(9 + 2 * b, std::max<size_t>(words, 8));
      d_sel[b] = static_cast<uint32_t*>(ctx.dev(12 + b, std::max<size_t>(max_rows * 4, 4)));
      d_cnt[b] = static_cast<uint64_t*>(ctx.dev(14 + b, 8));
    }
  }
  // stage of buffer b copied to the device (the pinned buffer may be refilled) / probed or inserted (the
  // device key buffer may be overwritten; the count is on its way back) / sel back on the host
  hipEvent_t copied(int b) { return static_cast<hipEvent_t>(ctx.event(b)); }
  hipEvent_t probed(int b) { return static_cast<hipEvent_t>(ctx.event(2 + b)); }
  hipEvent_t returned(int b) { return static_cast<hipEvent_t>(ctx.event(4 + b)); }
};

namespace {
using Clock = std::chrono::steady_clock;

// n empty selection vectors that keep the capacity a caller's earlier batch gave them: a caching operator
// calls with the same vector every batch, and re-allocating ~16 Ki small vectors per call (then growing them
// as survivors arrive) cost more than the copy of the batch itself (tools/host_bench: 21 ms of 35 per 2^25
// rows on the GPU box, where fresh pages fault expensively).
void reset_sels(std::vector<SelectionVector>& sels, size_t n) {
  sels.resize(n);
  for (SelectionVector& v : sels) v.clear();
}
double secs_since(Clock::time_point t0) { return std::chrono::duration<double>(Clock::now() - t0).count(); }

// A stage's ascending sel (ids relative to the stage) -> per-chunk sels (ids relative to each chunk), over
// the context's worker threads: each chunk's survivors are one contiguous range of the stage's sel.
void split_sel(DeviceContext& ctx, const std::vector<const DataChunk*>& chunks, size_t c_lo, size_t c_hi,
               const uint32_t* h_sel, uint64_t cnt, std::vector<SelectionVector>& sels) {
  const size_t n_chunks = c_hi - c_lo;
  std::vector<uint64_t> start(n_chunks + 1, 0);
  for (size_t c = 0; c < n_chunks; c++) start[c + 1] = start[c] + chunks[c_lo + c]->count;
  const uint32_t* const end = h_sel + cnt;
  // the first id >= bound at or after p: galloping from p (a chunk's survivors are a few hundred ids on,
  // so the search stays on lines the copy reads anyway; a binary search over the whole rest of the stage
  // missed the cache at nearly every step: 21 ms per 2^25 rows on the GPU box)
  auto next_at_least = [end](const uint32_t* p, uint32_t bound) {
    size_t step = 16;
    while (static_cast<size_t>(end - p) > step && p[step] < bound) {
      p += step;
      step *= 2;
    }
    return std::lower_bound(p, static_cast<size_t>(end - p) > step ? p + step + 1 : end, bound);
  };
  auto range = [&](size_t lo, size_t hi) {
    const uint32_t* p = std::lower_bound(h_sel, end, static_cast<uint32_t>(start[lo]));
    for (size_t c = lo; c < hi; c++) {
      const uint32_t* e = next_at_least(p, static_cast<uint32_t>(start[c + 1]));
      SelectionVector& out = sels[c_lo + c];
      out.resize(static_cast<size_t>(e - p));
      const uint32_t base = static_cast<uint32_t>(start[c]);
      for (size_t x = 0; x < out.size(); x++) out[x] = p[x] - base;
      p = e;
    }
  };
  if (cnt < (1u << 13) || n_chunks < 64 || ctx.flatten_threads <= 1) {
    range(0, n_chunks);
    return;
  }
  const size_t n_tasks = std::min<size_t>(n_chunks / 16, 4 * static_cast<size_t>(ctx.flatten_threads));
  ctx.parallel_for(n_tasks, [&](size_t t) { range(n_chunks * t / n_tasks, n_chunks * (t + 1) / n_tasks); });
}

// The set bits of x as base + bit index into tmp (room for 64 + 16), their count returned: AVX-512 compress where
// the host has it, else branchless (every bit writes, the cursor moves by the bit). For the dense words of a high
// pass fraction, where a ctz loop's branch on every survivor mispredicts.
__attribute__((target("avx512f"))) uint32_t expand_word_avx512(uint64_t x, uint32_t base, uint32_t* tmp) {
  const __m512i iota = _mm512_setr_epi32(0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15);
  uint32_t k = 0;
  for (int q = 0; q < 4; q++) {
    const __mmask16 m = static_cast<__mmask16>(x >> (16 * q));
    const __m512i idx = _mm512_add_epi32(iota, _mm512_set1_epi32(static_cast<int>(base + 16 * q)));
    _mm512_storeu_si512(tmp + k, _mm512_maskz_compress_epi32(m, idx));
    k += static_cast<uint32_t>(__builtin_popcount(static_cast<uint32_t>(m)));
  }
  return k;
}
uint32_t expand_word_scalar(uint64_t x, uint32_t base, uint32_t* tmp) {
  uint32_t k = 0;
  for (uint32_t j = 0; j < 64; j++) {
    tmp[k] = base + j;
    k += static_cast<uint32_t>((x >> j) & 1);
  }
  return k;
}
bool host_has_avx512() {
  static const bool v = [] {
    __builtin_cpu_init();
    return __builtin_cpu_supports("avx512f") != 0;
  }();
  return v;
}

// A stage's result bits (bit r = stage row r passes) -> per-chunk sels (ids relative to each chunk), over the
// context's worker threads: each chunk's rows are one bit range.
void split_bits(DeviceContext& ctx, const std::vector<const DataChunk*>& chunks, size_t c_lo, size_t c_hi,
                const uint64_t* h_bits, std::vector<SelectionVector>& sels) {
  const size_t n_chunks = c_hi - c_lo;
  std::vector<uint64_t> start(n_chunks + 1, 0);
  for (size_t c = 0; c < n_chunks; c++) start[c + 1] = start[c] + chunks[c_lo + c]->count;
  auto word = [&](uint64_t w, uint64_t r, uint64_t e) {  // bits of word w inside rows [r, e)
    uint64_t x = h_bits[w];
    const uint64_t lo = w << 6;
    if (lo < r) x &= ~0ULL << (r - lo);
    if (e - lo < 64) x &= (1ULL << (e - lo)) - 1;
    return x;
  };
  const bool avx512 = host_has_avx512();
  auto range = [&](size_t lo_c, size_t hi_c) {
    for (size_t c = lo_c; c < hi_c; c++) {
      const uint64_t r = start[c], e = start[c + 1];
      SelectionVector& out = sels[c_lo + c];
      if (r == e) {
        out.clear();
        continue;
      }
      size_t cnt = 0;
      for (uint64_t w = r >> 6; (w << 6) < e; w++) cnt += static_cast<size_t>(__builtin_popcountll(word(w, r, e)));
      out.resize(cnt);
      size_t k = 0;
      alignas(64) uint32_t tmp[64 + 16];
      for (uint64_t w = r >> 6; (w << 6) < e; w++) {
        uint64_t x = word(w, r, e);
        const uint32_t base = static_cast<uint32_t>((w << 6) - r);  // wraps below r: the sums do not
        if (__builtin_popcountll(x) > 12) {  // dense word
          const uint32_t m = avx512 ? expand_word_avx512(x, base, tmp) : expand_word_scalar(x, base, tmp);
          std::memcpy(out.data() + k, tmp, m * 4);
          k += m;
        } else {
          while (x) {
            out[k++] = base + static_cast<uint32_t>(__builtin_ctzll(x));
            x &= x - 1;
          }
        }
      }
    }
  };
  if (start[n_chunks] < (1u << 16) || n_chunks < 64 || ctx.flatten_threads <= 1) {
    range(0, n_chunks);
  } else {
    const size_t n_tasks = std::min<size_t>(n_chunks / 16, 4 * static_cast<size_t>(ctx.flatten_threads));
    ctx.parallel_for(n_tasks, [&](size_t t) { range(n_chunks * t / n_tasks, n_chunks * (t + 1) / n_tasks); });
  }
}
}  // namespace

// Persistent worker threads of a DeviceContext (parallel_for): workers sleep on a condition variable
// between jobs; a job hands out task indices through an atomic counter, the caller works too.
struct DeviceContext::Pool {
  explicit Pool(unsigned n_workers) {
    for (unsigned i = 0; i < n_workers; i++) workers.emplace_back([this] { loop(); });
  }
  ~Pool() {
    {
      std::lock_guard<std::mutex> lk(mu);
      stop = true;
    }
    wake.notify_all();
    for (auto& t : workers) t.join();
  }
  void loop() {
    uint64_t seen = 0;
    for (;;) {
      std::unique_lock<std::mutex> lk(mu);
      wake.wait(lk, [&] { return stop || gen != seen; });
      if (stop) return;
      seen = gen;
      lk.unlock();
      work();
      lk.lock();
      if (--active == 0) done.notify_all();
    }
  }
  void work() {
    for (;;) {
      const size_t t = next.fetch_add(1);
      if (t >= n) return;
      try {
        (*fn)(t);
      } catch (...) {
        std::lock_guard<std::mutex> g(err_mu);
        if (!err) err = std::current_exception();
      }
    }
  }
  // every worker takes part in every job, so a job cannot start before the previous one is done
  void run(size_t n_tasks, const std::function<void(size_t)>& f) {
    {
      std::lock_guard<std::mutex> lk(mu);
      fn = &f;
      n = n_tasks;
      next.store(0);
      active = workers.size();
      err = nullptr;
      gen++;
    }
    wake.notify_all();
    work();
    std::unique_lock<std::mutex> lk(mu);
    done.wait(lk, [&] { return active == 0; });
    fn = nullptr;
    if (err) {
      std::exception_ptr e = err;
      err = nullptr;
      std::rethrow_exception(e);
    }
  }
  std::vector<std::thread> workers;
  std::mutex mu, err_mu;
  std::condition_variable wake, done;
  const std::function<void(size_t)>* fn = nullptr;
  size_t n = 0, active = 0;
  std::atomic<size_t> next{0};
  uint64_t gen = 0;
  bool stop = false;
  std::exception_ptr err;
};

void DeviceContext::parallel_for(size_t n, const std::function<void(size_t)>& fn) {
  const unsigned threads = std::min<unsigned>(std::max(flatten_threads, 1u), std::max(1u, std::thread::hardware_concurrency()));
  if (n <= 1 || threads <= 1) {
    for (size_t t = 0; t < n; t++) fn(t);
    return;
  }
  if (!pool_ || pool_->workers.size() != threads - 1) {
    pool_.reset();
    pool_ = std::make_unique<Pool>(threads - 1);
  }
  pool_->run(n, fn);
}

// ---- DeviceContext -----------------------------------------------------------------------------
// ---- pinned host buffer cache ----------------------------------------------------------------------
// Pinned buffers of contexts that grow a slot or die, kept for the next context of that device that asks for that
// size (powers of two from 64 KiB): hipHostMalloc pins every page (12.7 ms per 32 MiB on the GPU box), which
// per-query operator states would otherwise pay on every query. Never freed at exit (the HIP runtime may be gone
// by then); ReleasePinnedCache frees what is cached.
namespace {
struct PinnedCache {
  std::mutex mu;
  std::map<std::pair<int, size_t>, std::vector<void*>> free;  // by (device, capacity)
  size_t cached = 0, limit = size_t(4) << 30;
};
PinnedCache& pinned_cache() {
  static PinnedCache* c = new PinnedCache;  // intentionally leaked (see above)
  return *c;
}
size_t pinned_class(size_t bytes) {
  size_t c = size_t(1) << 16;
  while (c < bytes) c <<= 1;
  return c;
}
void* pinned_take(int device, size_t cap) {
  PinnedCache& c = pinned_cache();
  {
    std::lock_guard<std::mutex> lk(c.mu);
    auto it = c.free.find({device, cap});
    if (it != c.free.end() && !it->second.empty()) {
      void* p = it->second.back();
      it->second.pop_back();
      c.cached -= cap;
      return p;
    }
  }
  void* p = nullptr;
  DeviceScope ds(device);
  check_hip(hipHostMalloc(&p, cap, hipHostMallocDefault), "hipHostMalloc");
  return p;
}
void pinned_give(int device, void* p, size_t cap) {  // p is no longer used by any stream
  PinnedCache& c = pinned_cache();
  {
    std::lock_guard<std::mutex> lk(c.mu);
    if (c.cached + cap <= c.limit) {
      c.free[{device, cap}].push_back(p);
      c.cached += cap;
      return;
    }
  }
  (void)hipHostFree(p);
}

// Streams and events of ended contexts, per device, for the next context: hipStreamCreate and hipStreamDestroy
// cost ~2 ms each on this runtime (profiles/r05/host_create_split.jsonl: ctx_create_ms / ctx_destroy_ms), which
// every short-lived context (a query's operator-thread states, Finalize) paid. A stream is returned drained and
// not capturing; the pool is bounded by the most contexts ever alive at once. Intentionally leaked, as the
// pinned cache.
struct HandlePool {
  std::mutex mu;
  std::map<int, std::vector<hipStream_t>> streams;
  std::map<int, std::vector<hipEvent_t>> events;
};
HandlePool& handle_pool() {
  static HandlePool* p = new HandlePool;
  return *p;
}
hipStream_t stream_take(int device) {
  HandlePool& p = handle_pool();
  {
    std::lock_guard<std::mutex> lk(p.mu);
    auto& v = p.streams[device];
    if (!v.empty()) {
      hipStream_t s = v.back();
      v.pop_back();
      return s;
    }
  }
  DeviceScope ds(device);
  hipStream_t s;
  check_hip(hipStreamCreateWithFlags(&s, hipStreamNonBlocking), "hipStreamCreate");
  return s;
}
void stream_give(int device, hipStream_t s) {  // s is drained
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(s, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone || hipStreamQuery(s) != hipSuccess) {
    (void)hipStreamDestroy(s);  // a stream left capturing or failed is not handed on
    return;
  }
  HandlePool& p = handle_pool();
  std::lock_guard<std::mutex> lk(p.mu);
  p.streams[device].push_back(s);
}
hipEvent_t event_take(int device) {
  HandlePool& p = handle_pool();
  {
    std::lock_guard<std::mutex> lk(p.mu);
    auto& v = p.events[device];
    if (!v.empty()) {
      hipEvent_t e = v.back();
      v.pop_back();
      return e;
    }
  }
  DeviceScope ds(device);
  hipEvent_t e;
  check_hip(hipEventCreateWithFlags(&e, hipEventDisableTiming), "hipEventCreate");
  return e;
}
void event_give(int device, hipEvent_t e) {  // its stream is drained: the event has completed
  HandlePool& p = handle_pool();
  std::lock_guard<std::mutex> lk(p.mu);
  p.events[device].push_back(e);
}
}  // namespace

void SetPinnedCacheLimit(size_t bytes) {
  PinnedCache& c = pinned_cache();
  std::vector<std::pair<void*, size_t>> drop;
  {
    std::lock_guard<std::mutex> lk(c.mu);
    c.limit = bytes;
    for (auto it = c.free.rbegin(); it != c.free.rend() && c.cached > c.limit; ++it)
      while (!it->second.empty() && c.cached > c.limit) {
        drop.emplace_back(it->second.back(), it->first.second);
        it->second.pop_back();
        c.cached -= it->first.second;
      }
  }
  for (auto& d : drop) (void)hipHostFree(d.first);
}

size_t PinnedCacheBytes() {
  PinnedCache& c = pinned_cache();
  std::lock_guard<std::mutex> lk(c.mu);
  return c.cached;
}

void ReleasePinnedCache() {
  PinnedCache& c = pinned_cache();
  std::map<std::pair<int, size_t>, std::vector<void*>> all;
  {
    std::lock_guard<std::mutex> lk(c.mu);
    all.swap(c.free);
    c.cached = 0;
  }
  for (auto& kv : all)
    for (void* p : kv.second) (void)hipHostFree(p);
}

DeviceContext::DeviceContext(int device) : device_(device) { stream_ = stream_take(device_); }

DeviceContext::~DeviceContext() {
  pool_.reset();
  DeviceScope ds(device_);
  for (void* st : {stream_, copy_stream_, h2d_stream_, aux_streams_[0], aux_streams_[1]})
    if (st) (void)hipStreamSynchronize(static_cast<hipStream_t>(st));
  for (auto& b : host_)
    if (b.p) pinned_give(device_, b.p, b.cap);  // the streams are drained above
  for (auto& b : dev_)
    if (b.p) (void)hipFree(b.p);
  for (void* e : events_)
    if (e) event_give(device_, static_cast<hipEvent_t>(e));
  for (void* st : {aux_streams_[1], aux_streams_[0], h2d_stream_, copy_stream_, stream_})
    if (st) stream_give(device_, static_cast<hipStream_t>(st));
}

void DeviceContext::synchronize() {
  DeviceScope ds(device_);
  check_hip(hipStreamSynchronize(static_cast<hipStream_t>(stream_)), "hipStreamSynchronize");
  if (copy_stream_) check_hip(hipStreamSynchronize(static_cast<hipStream_t>(copy_stream_)), "hipStreamSynchronize");
  if (h2d_stream_) check_hip(hipStreamSynchronize(static_cast<hipStream_t>(h2d_stream_)), "hipStreamSynchronize");
  for (void* st : aux_streams_)
    if (st) check_hip(hipStreamSynchronize(static_cast<hipStream_t>(st)), "hipStreamSynchronize");
}

void* DeviceContext::copy_stream() {
  if (!copy_stream_) copy_stream_ = stream_take(device_);
  return copy_stream_;
}

void* DeviceContext::h2d_stream() {
  if (!h2d_stream_) h2d_stream_ = stream_take(device_);
  return h2d_stream_;
}

void* DeviceContext::aux_stream(int i) {
  if (i < 0 || i >= kAuxStreams) throw GpuError(RPT_ERR_INVALID_ARGUMENT, "aux stream index out of range");
  if (!aux_streams_[i]) aux_streams_[i] = stream_take(device_);
  return aux_streams_[i];
}

void* DeviceContext::event(int i) {
  if (i < 0 || i >= kEvents) throw GpuError(RPT_ERR_INVALID_ARGUMENT, "event index out of range");
  void*& e = events_[i];
  if (!e) e = event_take(device_);
  return e;
}

void* DeviceContext::host(int slot, size_t bytes) {
  Buf& b = host_[slot];
  if (b.cap < bytes) {
    synchronize();
    if (b.p) pinned_give(device_, b.p, b.cap);
    b.p = nullptr;
    b.dp = nullptr;
    const size_t cap = pinned_class(std::max(bytes, 2 * b.cap));
    b.p = pinned_take(device_, cap);
    b.cap = cap;
  }
  return b.p;
}

void* DeviceContext::host_device_ptr(int slot) {
  Buf& b = host_[slot];
  if (!b.p) throw GpuError(RPT_ERR_INVALID_ARGUMENT, "host slot not allocated");
  if (!b.dp) check_hip(hipHostGetDevicePointer(&b.dp, b.p, 0), "hipHostGetDevicePointer");
  return b.dp;
}

void* DeviceContext::dev(int slot, size_t bytes) {
  Buf& b = dev_[slot];
  if (b.cap < bytes) {
    synchronize();
    DeviceScope ds(device_);
    if (b.p) check_hip(hipFree(b.p), "hipFree");
    b.p = nullptr;
    const size_t cap = std::max(bytes, 2 * b.cap);
    check_hip(hipMalloc(&b.p, cap), "hipMalloc");
    b.cap = cap;
  }
  return b.p;
}

// ---- DeviceKeyColumn ---------------------------------------------------------------------------
DeviceKeyColumn::~DeviceKeyColumn() { release(); }

DeviceKeyColumn::DeviceKeyColumn(DeviceKeyColumn&& o) noexcept : device_(o.device_), segs_(std::move(o.segs_)) {
  o.segs_.clear();
}

DeviceKeyColumn& DeviceKeyColumn::operator=(DeviceKeyColumn&& o) noexcept {
  if (this != &o) {
    release();
    device_ = o.device_;
    segs_ = std::move(o.segs_);
    o.segs_.clear();
  }
  return *this;
}

void DeviceKeyColumn::release() {
  if (segs_.empty()) return;
  DeviceScope ds(device_);
  for (auto& g : segs_) {
    (void)hipFree(const_cast<void*>(g.col.keys));
    if (g.col.validity) (void)hipFree(const_cast<uint64_t*>(g.col.validity));
  }
  segs_.clear();
}

const DeviceKeyColumn::Segment& DeviceKeyColumn::Append(DeviceContext& ctx, const std::vector<const DataChunk*>& chunks,
                                                        uint64_t col, int slot) {
  const uint64_t total = total_rows(chunks);
  if (total == 0) throw GpuError(RPT_ERR_INVALID_ARGUMENT, "empty batch");
  const Flattened f = flatten_pinned(ctx, chunks.data(), chunks.size(), col, total, slot);
  DeviceScope ds(device_);
  void* dkeys = nullptr;
  void* dvalid = nullptr;
  check_hip(hipMalloc(&dkeys, total * key_size(f.key_type)), "hipMalloc key segment");
  if (f.any_null) {
    if (hipMalloc(&dvalid, (total + 63) / 64 * 8) != hipSuccess) {
      (void)hipFree(dkeys);
      throw GpuError(RPT_ERR_HIP, "hipMalloc validity segment");
    }
  }
  segs_.push_back(Segment{copy_flattened(ctx, f, total, dkeys, dvalid), total});
  return segs_.back();
}

void DeviceKeyColumn::Splice(DeviceKeyColumn&& other) {
  if (other.device_ != device_) throw GpuError(RPT_ERR_INVALID_ARGUMENT, "key columns on different devices");
  for (auto& g : other.segs_) segs_.push_back(g);
  other.segs_.clear();
}

uint64_t DeviceKeyColumn::rows() const {
  uint64_t r = 0;
  for (const auto& g : segs_) r += g.rows;
  return r;
}

// ---- PTBloomFilter -------------------------------------------------------------------------------
PTBloomFilter::~PTBloomFilter() {
  if (bf_) rpt_bf_destroy(bf_);
}

void PTBloomFilter::Initialize(int device, uint32_t est_num_rows) {
  if (bf_) {
    rpt_bf_destroy(bf_);
    bf_ = nullptr;
  }
  check(rpt_bf_create(device, est_num_rows, &bf_));
  minmax_kept_.store(true);
}

void PTBloomFilter::Insert(DeviceContext& ctx, const DataChunk& chunk, const std::vector<uint64_t>& cols) {
  InsertBatch(ctx, {&chunk}, cols);
}

void PTBloomFilter::InsertBatch(DeviceContext& ctx, const std::vector<const DataChunk*>& chunks,
                                const std::vector<uint64_t>& cols) {
  const uint64_t total = total_rows(chunks);
  if (total == 0) return;  // bloom_filter.cpp:72-74
  if (cols.size() == 1) NoteKeyType(chunks[0]->data.at(cols[0]).key_type);  // (composite keys carry no min/max)
  if (cols.size() == 1 && stage_rows_for(ctx, total)) {
    InsertPipelined(ctx, chunks, cols[0]);
    return;
  }
  if (cols.size() == 1 && total <= kSingleCopyRows && rpt_bf_insert_workspace_bytes(bf_, total) == 0) {
    // small batch, atomic insert: the kernel reads the flattened keys from the pinned staging buffer
    // through device-mapped pointers (no copy)
    const Flattened f = flatten_pinned(ctx, chunks.data(), chunks.size(), cols[0], total, 0);
    rpt_key_column kc;
    kc.key_type = static_cast<int32_t>(f.key_type);
    kc.keys = ctx.host_device_ptr(0);  // flatten_pinned: keys at the start of slot 0, validity of slot 1
    kc.key_sel = nullptr;
    kc.validity = f.any_null ? static_cast<const uint64_t*>(ctx.host_device_ptr(1)) : nullptr;
    check(rpt_bf_insert(bf_, &kc, total, ctx.stream()));
    ctx.synchronize();  // the staging buffer is reused by the next call
    return;
  }
  InsertDevice(ctx, stage_key(ctx, chunks, cols, total), total);
}

// Stage by stage: the host flattens stage i into pinned buffer i % 2 while the host-to-device stream copies
// stage i-1 and the context's stream inserts stage i-2 (inserts stay serial in stream order). A pinned
// buffer is refilled once its copy has finished, a device key buffer once the insert that read it has.
void PTBloomFilter::InsertPipelined(DeviceContext& ctx, const std::vector<const DataChunk*>& chunks, uint64_t col) {
  const Clock::time_point t_begin = Clock::now();
  DeviceContext::PipelineStats& ps = ctx.stats;
  const std::vector<StageRange> st = pipeline_stages(chunks, col, stage_rows_for(ctx, total_rows(chunks)));
  uint64_t max_rows = 0, total = 0;
  size_t ws_bytes = 0;
  for (const StageRange& r : st) {
    max_rows = std::max(max_rows, r.rows);
    total += r.rows;
    ws_bytes = std::max(ws_bytes, rpt_bf_insert_workspace_bytes(bf_, r.rows));
  }
  const KeyType kt = chunks[st[0].c_lo]->data.at(col).key_type;
  const size_t es = key_size(device_type(kt));
  bool narrow = ctx.narrow_keys && kt == KeyType::I64;  // until a stage's keys are not narrow
  size_t max_chunks = 0;
  for (const StageRange& r : st) max_chunks = std::max(max_chunks, r.c_hi - r.c_lo);
  PipelineBuffers pb(ctx, max_rows, es, narrow ? max_chunks : 0);
  void* ws = ws_bytes ? ctx.dev(6, ws_bytes) : nullptr;
  auto s = static_cast<hipStream_t>(ctx.stream());
  auto h = static_cast<hipStream_t>(ctx.h2d_stream());
  try {
    for (size_t i = 0; i < st.size(); i++) {
      const int b = static_cast<int>(i & 1);
      Clock::time_point t0 = Clock::now();
      if (i >= 2) check_hip(hipEventSynchronize(pb.copied(b)), "hipEventSynchronize");
      ps.wait_copy_s += secs_since(t0);
      t0 = Clock::now();
      const Flattened f = flatten_pinned(ctx, chunks.data() + st[i].c_lo, st[i].c_hi - st[i].c_lo, col, st[i].rows,
                                         PipelineBuffers::kHostKeys + 2 * b, -1,
                                         narrow ? PipelineBuffers::kNarrowMeta + b : -1);
      narrow = f.narrow;
      ps.narrow_stages += f.narrow;
      ps.flatten_s += secs_since(t0);
      t0 = Clock::now();
      if (i >= 2) check_hip(hipStreamWaitEvent(h, pb.probed(b), 0), "hipStreamWaitEvent");  // insert i-2 read it
      const rpt_key_column kc = copy_flattened(ctx, f, st[i].rows, pb.d_keys[b], pb.d_valid[b], h, pb.d_lo[b], pb.d_meta[b]);
      check_hip(hipEventRecord(pb.copied(b), h), "hipEventRecord");
      check_hip(hipStreamWaitEvent(s, pb.copied(b), 0), "hipStreamWaitEvent");
      if (rpt_bf_insert_workspace_bytes(bf_, st[i].rows)) check(rpt_bf_insert_ws(bf_, &kc, st[i].rows, ws, ws_bytes, s));
      else check(rpt_bf_insert(bf_, &kc, st[i].rows, s));
      check_hip(hipEventRecord(pb.probed(b), s), "hipEventRecord");
      ps.enqueue_s += secs_since(t0);
    }
  } catch (...) {
    (void)hipStreamSynchronize(h);  // nothing may still read the staging buffers
    (void)hipStreamSynchronize(s);
    throw;
  }
  ctx.synchronize();
  ps.stages += st.size();
  ps.rows += total;
  ps.total_s += secs_since(t_begin);
}

void PTBloomFilter::InsertDevice(DeviceContext& ctx, const rpt_key_column& col, uint64_t n, bool synchronize) {
  if (n == 0) return;
  // large batches take the partitioned / bucketed insert (same filter bits)
  const size_t ws_bytes = rpt_bf_insert_workspace_bytes(bf_, n);
  if (ws_bytes) check(rpt_bf_insert_ws(bf_, &col, n, ctx.dev(6, ws_bytes), ws_bytes, ctx.stream()));
  else check(rpt_bf_insert(bf_, &col, n, ctx.stream()));
  if (synchronize) ctx.synchronize();  // the staging buffers are reused by the next call
}

uint64_t PTBloomFilter::LookupSel(DeviceContext& ctx, const DataChunk& chunk, SelectionVector& sel,
                                  const std::vector<uint64_t>& cols) const {
  std::vector<SelectionVector> sels;
  LookupSelBatch(ctx, {&chunk}, sels, cols);
  sel.swap(sels[0]);
  return sel.size();
}

void PTBloomFilter::LookupSelBatch(DeviceContext& ctx, const std::vector<const DataChunk*>& chunks,
                                   std::vector<SelectionVector>& sels, const std::vector<uint64_t>& cols) const {
  reset_sels(sels, chunks.size());
  const uint64_t total = total_rows(chunks);
  if (total == 0) return;  // bloom_filter.cpp:63-65
  if (cols.size() == 1 && stage_rows_for(ctx, total)) {
    LookupSelPipelined(ctx, chunks, sels, cols[0]);
    return;
  }
  if (cols.size() == 1 && rpt_bf_probe_is_fused(bf_, total) == 1) {
    LookupSelMapped(ctx, chunks, sels, cols[0], total);
    return;
  }
  rpt_key_column kc = stage_key(ctx, chunks, cols, total);
  const size_t ws_bytes = rpt_bf_probe_workspace_bytes(bf_, total);  // for the strategy this batch runs
  void* ws = ctx.dev(2, ws_bytes);
  // [count (8 B) | sel]: small batches bring both back in ONE copy (one sync per call); larger ones
  // copy the count first and then exactly `count` ids
  auto s = static_cast<hipStream_t>(ctx.stream());
  if (ctx.bits_back && total > kSingleCopyRows) {  // the result bits back in one copy, one sync (no count first)
    const size_t bits_bytes = (total + 511) / 512 * 64;
    auto* d_bits = static_cast<uint64_t*>(ctx.dev(3, bits_bytes));
    check(rpt_bf_probe_bits(bf_, &kc, nullptr, total, d_bits, ws, ws_bytes, s));
    auto* h_bits = static_cast<uint64_t*>(ctx.host(3, bits_bytes));
    check_hip(hipMemcpyAsync(h_bits, d_bits, bits_bytes, hipMemcpyDeviceToHost, s), "copy bits");
    ctx.synchronize();
    split_bits(ctx, chunks, 0, chunks.size(), h_bits, sels);
    return;
  }
  auto* d_out = static_cast<uint8_t*>(ctx.dev(3, 8 + total * 4));
  auto* d_cnt = reinterpret_cast<uint64_t*>(d_out);
  auto* d_sel = reinterpret_cast<uint32_t*>(d_out + 8);
  check(rpt_bf_probe(bf_, &kc, nullptr, total, d_sel, d_cnt, ws, ws_bytes, s));
  const bool one_copy = total <= kSingleCopyRows;
  auto* h_out = static_cast<uint8_t*>(ctx.host(2, one_copy ? 8 + total * 4 : 8));
  check_hip(hipMemcpyAsync(h_out, d_out, one_copy ? 8 + total * 4 : 8, hipMemcpyDeviceToHost, s), "copy count");
  ctx.synchronize();
  const uint64_t cnt = *reinterpret_cast<const uint64_t*>(h_out);
  const uint32_t* h_sel = reinterpret_cast<const uint32_t*>(h_out + 8);
  if (!one_copy) {
    auto* hs = static_cast<uint32_t*>(ctx.host(3, std::max<uint64_t>(cnt, 1) * 4));
    if (cnt) check_hip(hipMemcpyAsync(hs, d_sel, cnt * 4, hipMemcpyDeviceToHost, s), "copy sel");
    ctx.synchronize();
    h_sel = hs;
  }
  split_sel(ctx, chunks, 0, chunks.size(), h_sel, cnt, sels);  // batch-wide ascending sel -> per-chunk sels
}

// Per-vector calls (one fused kernel): the kernel reads the flattened keys straight from the pinned
// staging buffer and writes [count | sel] straight into pinned memory through device-mapped pointers,
// so a call is one launch and one sync with no copies.
void PTBloomFilter::LookupSelMapped(DeviceContext& ctx, const std::vector<const DataChunk*>& chunks,
                                    std::vector<SelectionVector>& sels, uint64_t col, uint64_t total) const {
  const Flattened f = flatten_pinned(ctx, chunks.data(), chunks.size(), col, total, 0);
  auto* h_out = static_cast<uint8_t*>(ctx.host(2, 8 + total * 4));
  void* d_keys = ctx.host_device_ptr(0);  // flatten_pinned: keys at the start of slot 0, validity of slot 1
  void* d_valid = f.any_null ? ctx.host_device_ptr(1) : nullptr;
  void* d_out = ctx.host_device_ptr(2);
  rpt_key_column kc;
  kc.key_type = static_cast<int32_t>(f.key_type);
  kc.keys = d_keys;
  kc.key_sel = nullptr;
  kc.validity = static_cast<const uint64_t*>(d_valid);
  auto* d_cnt = static_cast<uint64_t*>(d_out);
  auto* d_sel = reinterpret_cast<uint32_t*>(static_cast<uint8_t*>(d_out) + 8);
  check(rpt_bf_probe(bf_, &kc, nullptr, total, d_sel, d_cnt, nullptr, 0, ctx.stream()));
  ctx.synchronize();
  const uint64_t cnt = *reinterpret_cast<const volatile uint64_t*>(h_out);
  const uint32_t* h_sel = reinterpret_cast<const uint32_t*>(h_out + 8);
  uint64_t k = 0, start = 0;
  for (size_t i = 0; i < chunks.size(); i++) {
    const uint64_t end = start + chunks[i]->count;
    SelectionVector& out = sels[i];
    while (k < cnt && h_sel[k] < end) out.push_back(static_cast<uint32_t>(h_sel[k++] - start));
    start = end;
  }
}

// Four stages in flight on three streams: while the host flattens stage i into pinned buffer i % 2, the
// host-to-device stream copies stage i-1 to the device, the context's stream probes it once it is there (and
// copies its count back), and the copy stream brings stage i-2's selection vector back (its exact length is
// known once that stage's count has arrived); the host splits each stage's sel into per-chunk sels. Copies
// in the two directions and the probes overlap, so the copy engine feeding the device is the limit when the
// host keeps up. A pinned buffer is refilled once its copy has finished, a device key buffer once the probe
// that read it has, a device sel buffer once its copy back has.
void PTBloomFilter::LookupSelPipelined(DeviceContext& ctx, const std::vector<const DataChunk*>& chunks,
                                       std::vector<SelectionVector>& sels, uint64_t col) const {
  const Clock::time_point t_begin = Clock::now();
  DeviceContext::PipelineStats& ps = ctx.stats;
  const std::vector<StageRange> st = pipeline_stages(chunks, col, stage_rows_for(ctx, total_rows(chunks)));
  uint64_t max_rows = 0, total = 0;
  size_t ws_bytes = 16;
  for (const StageRange& r : st) {
    max_rows = std::max(max_rows, r.rows);
    total += r.rows;
    ws_bytes = std::max(ws_bytes, rpt_bf_probe_workspace_bytes(bf_, r.rows));
  }
  const KeyType kt = chunks[st[0].c_lo]->data.at(col).key_type;
  const size_t es = key_size(device_type(kt));
  bool narrow = ctx.narrow_keys && kt == KeyType::I64;  // until a stage's keys are not narrow
  size_t max_chunks = 0;
  for (const StageRange& r : st) max_chunks = std::max(max_chunks, r.c_hi - r.c_lo);
  PipelineBuffers pb(ctx, max_rows, es, narrow ? max_chunks : 0);
  void* ws = ctx.dev(2, ws_bytes);
  auto s = static_cast<hipStream_t>(ctx.stream());
  auto d = static_cast<hipStream_t>(ctx.copy_stream());
  auto h = static_cast<hipStream_t>(ctx.h2d_stream());
  // bits_back: each stage's result bits come back (rows / 8 bytes, no count round trip) and the workers turn them
  // into the chunks' sels; else the survivors' sel (4 B each) after its count. Device / host slots 60 + b.
  const bool bits = ctx.bits_back;
  const size_t bits_bytes = (max_rows + 511) / 512 * 64;
  uint64_t* d_bits[2] = {nullptr, nullptr};
  uint64_t* h_bits[2] = {nullptr, nullptr};
  for (int b = 0; bits && b < 2; b++) {
    d_bits[b] = static_cast<uint64_t*>(ctx.dev(60 + b, bits_bytes));
    h_bits[b] = static_cast<uint64_t*>(ctx.host(60 + b, bits_bytes));
  }
  uint64_t counts[2] = {0, 0};
  auto count_arrived = [&](size_t j) {  // stage j's count is on the host: copy its sel back exactly
    const int b = static_cast<int>(j & 1);
    const Clock::time_point t0 = Clock::now();
    check_hip(hipEventSynchronize(pb.probed(b)), "hipEventSynchronize");
    ps.wait_count_s += secs_since(t0);
    counts[b] = *pb.h_cnt[b];
    if (counts[b]) {
      check_hip(hipStreamWaitEvent(d, pb.probed(b), 0), "hipStreamWaitEvent");
      check_hip(hipMemcpyAsync(pb.h_sel[b], pb.d_sel[b], counts[b] * 4, hipMemcpyDeviceToHost, d), "copy sel");
    }
    check_hip(hipEventRecord(pb.returned(b), d), "hipEventRecord");
  };
  auto split = [&](size_t j) {  // stage j's ascending sel -> per-chunk sels (ids relative to each chunk)
    const int b = static_cast<int>(j & 1);
    Clock::time_point t0 = Clock::now();
    check_hip(hipEventSynchronize(pb.returned(b)), "hipEventSynchronize");
    ps.wait_sel_s += secs_since(t0);
    t0 = Clock::now();
    if (bits) split_bits(ctx, chunks, st[j].c_lo, st[j].c_hi, h_bits[b], sels);
    else split_sel(ctx, chunks, st[j].c_lo, st[j].c_hi, pb.h_sel[b], counts[b], sels);
    ps.split_s += secs_since(t0);
  };
  try {
    for (size_t i = 0; i < st.size(); i++) {
      const int b = static_cast<int>(i & 1);
      Clock::time_point t0 = Clock::now();
      if (i >= 2) check_hip(hipEventSynchronize(pb.copied(b)), "hipEventSynchronize");
      ps.wait_copy_s += secs_since(t0);
      t0 = Clock::now();
      const Flattened f = flatten_pinned(ctx, chunks.data() + st[i].c_lo, st[i].c_hi - st[i].c_lo, col, st[i].rows,
                                         PipelineBuffers::kHostKeys + 2 * b, -1,
                                         narrow ? PipelineBuffers::kNarrowMeta + b : -1);
      narrow = f.narrow;
      ps.narrow_stages += f.narrow;
      ps.flatten_s += secs_since(t0);
      t0 = Clock::now();
      if (i >= 2) check_hip(hipStreamWaitEvent(h, pb.probed(b), 0), "hipStreamWaitEvent");  // probe i-2 read it
      const rpt_key_column kc = copy_flattened(ctx, f, st[i].rows, pb.d_keys[b], pb.d_valid[b], h, pb.d_lo[b], pb.d_meta[b]);
      check_hip(hipEventRecord(pb.copied(b), h), "hipEventRecord");
      check_hip(hipStreamWaitEvent(s, pb.copied(b), 0), "hipStreamWaitEvent");
      if (i >= 2) check_hip(hipStreamWaitEvent(s, pb.returned(b), 0), "hipStreamWaitEvent");  // d_sel[b] free
      if (bits) {
        check(rpt_bf_probe_bits(bf_, &kc, nullptr, st[i].rows, d_bits[b], ws, ws_bytes, s));
      } else {
        check(rpt_bf_probe(bf_, &kc, nullptr, st[i].rows, pb.d_sel[b], pb.d_cnt[b], ws, ws_bytes, s));
        check_hip(hipMemcpyAsync(pb.h_cnt[b], pb.d_cnt[b], 8, hipMemcpyDeviceToHost, s), "copy count");
      }
      check_hip(hipEventRecord(pb.probed(b), s), "hipEventRecord");
      ps.enqueue_s += secs_since(t0);
      if (!bits && i >= 1) count_arrived(i - 1);
      if (i >= 2) split(i - 2);  // frees h_bits[b] / h_sel[b] for stage i
      if (bits) {  // stage i's bits back as soon as its probe is done
        check_hip(hipStreamWaitEvent(d, pb.probed(b), 0), "hipStreamWaitEvent");
        check_hip(hipMemcpyAsync(h_bits[b], d_bits[b], (st[i].rows + 511) / 512 * 64, hipMemcpyDeviceToHost, d), "copy bits");
        check_hip(hipEventRecord(pb.returned(b), d), "hipEventRecord");
      }
    }
    const size_t n = st.size();
    if (!bits) count_arrived(n - 1);
    if (n >= 2) split(n - 2);
    split(n - 1);
  } catch (...) {
    for (hipStream_t x : {h, s, d}) (void)hipStreamSynchronize(x);  // nothing may still use the staging buffers
    throw;
  }
  ps.stages += st.size();
  ps.rows += total;
  ps.total_s += secs_since(t_begin);
}

void PTBloomFilter::ReinitializeAndRehash(DeviceContext& ctx, uint64_t actual_rows, const std::vector<DataChunk>& data,
                                          const std::vector<uint64_t>& cols) {
  check(rpt_bf_reinitialize(bf_, actual_rows));
  std::vector<const DataChunk*> ptrs;
  for (const DataChunk& c : data)
    if (c.count) ptrs.push_back(&c);
  if (!ptrs.empty()) InsertBatch(ctx, ptrs, cols);
}

void PTBloomFilter::ReinitializeAndRehash(DeviceContext& ctx, uint64_t actual_rows, const DeviceKeyColumn& keys) {
  check(rpt_bf_reinitialize(bf_, actual_rows));
  const auto& segs = keys.segments();
  auto s = static_cast<hipStream_t>(ctx.stream());
  // Segments without NULLs are inserted in groups of up to kRehashGroupRows rows: their keys are copied back to
  // back into one buffer (HBM to HBM) and inserted by one call. One partitioned insert per 4 Mi-row sink segment
  // costs ~0.13 ms, mostly per-call work (1e8 rows: 24 calls 3.3 ms, one call ~0.5 ms).
  auto groupable = [&segs](size_t k) {
    return segs[k].col.validity == nullptr && segs[k].col.key_sel == nullptr && segs[k].col.key_type == segs[0].col.key_type;
  };
  const size_t es = segs.empty() ? 8 : (segs[0].col.key_type == RPT_KEY_I32 ? 4 : 8);
  size_t ws_max = 0, cat_max = 0;
  for (size_t k = 0; k < segs.size();) {  // pass 1: the groups' sizes -> one workspace and one copy buffer
    uint64_t rows = segs[k].rows;
    size_t e = k + 1;
    if (groupable(k))
      while (e < segs.size() && groupable(e) && rows + segs[e].rows <= kRehashGroupRows) rows += segs[e++].rows;
    if (e - k > 1) cat_max = std::max<size_t>(cat_max, rows * es);
    ws_max = std::max(ws_max, rpt_bf_insert_workspace_bytes(bf_, rows));
    k = e;
  }
  void* ws = ws_max ? ctx.dev(6, ws_max) : nullptr;
  auto* cat = static_cast<uint8_t*>(cat_max ? ctx.dev(7, cat_max) : nullptr);
  for (size_t k = 0; k < segs.size();) {
    rpt_key_column col = segs[k].col;
    uint64_t rows = segs[k].rows;
    size_t e = k + 1;
    if (groupable(k))
      while (e < segs.size() && groupable(e) && rows + segs[e].rows <= kRehashGroupRows) rows += segs[e++].rows;
    if (e - k > 1) {
      uint64_t off = 0;
      for (size_t j = k; j < e; j++) {
        check_hip(hipMemcpyAsync(cat + off * es, segs[j].col.keys, segs[j].rows * es, hipMemcpyDeviceToDevice, s),
                  "hipMemcpyAsync (rehash group)");
        off += segs[j].rows;
      }
      col.keys = cat;
    }
    const size_t b = rpt_bf_insert_workspace_bytes(bf_, rows);
    if (b) check(rpt_bf_insert_ws(bf_, &col, rows, ws, b, s));
    else check(rpt_bf_insert(bf_, &col, rows, s));
    k = e;
  }
  ctx.synchronize();
}

uint64_t PTBloomFilter::SizedForRows() const {
  rpt_bf_info i;
  check(rpt_bf_get_info(bf_, &i));
  return i.sized_for_rows;
}

bool PTBloomFilter::NeedsResize(uint64_t actual_rows) const {
  const int r = rpt_bf_needs_resize_alloc(bf_, actual_rows);
  if (r < 0) check(-r);
  return r == 1;
}

bool PTBloomFilter::IsEmpty() const {
  rpt_bf_info i;
  check(rpt_bf_get_info(bf_, &i));
  return !i.has_data;
}

int PTBloomFilter::LogNumBlocks() const {
  rpt_bf_info i;
  check(rpt_bf_get_info(bf_, &i));
  return i.log_num_blocks;
}

bool PTBloomFilter::MinMax(int64_t& min_value, int64_t& max_value) const {
  int has = 0;
  check(rpt_bf_get_minmax(bf_, &min_value, &max_value, &has, nullptr));
  return has != 0 && minmax_kept_.load();
}

void PTBloomFilter::NoteKeyType(KeyType t) {
  if (!keeps_minmax(t)) minmax_kept_.store(false);
}

std::vector<uint64_t> PTBloomFilter::ExportWords() const {
  rpt_bf_info i;
  check(rpt_bf_get_info(bf_, &i));
  std::vector<uint64_t> w(i.num_blocks);
  check(rpt_bf_export_words(bf_, w.data(), w.size()));
  return w;
}

void PTBloomFilter::AllReduceOr(DeviceContext& ctx, void* nccl_comm) {
  check(rpt_bf_allreduce_or(bf_, nccl_comm, ctx.stream()));
}

// ---- CreateBF ------------------------------------------------------------------------------------
CreateBF::CreateBF(int device, uint64_t estimated_cardinality, std::vector<uint64_t> bound_column_indices,
                   uint64_t sink_flush_rows, ResizeRule resize_rule)
    : device_(device),
      estimated_cardinality_(estimated_cardinality),
      resize_rule_(resize_rule),
      cols_(std::move(bound_column_indices)),
      sink_flush_rows_(std::max<uint64_t>(1, sink_flush_rows)) {
  for (size_t i = 0; i < cols_.size(); i++) {
    auto bf = std::make_shared<PTBloomFilter>();
    // CreateBFGlobalSinkState: Initialize(context, op.estimated_cardinality) -> uint32 (cpp:179-186)
    bf->Initialize(device_, static_cast<uint32_t>(estimated_cardinality_));
    filters_.push_back(std::move(bf));
    resized_.push_back(false);
    all_keys_.emplace_back(device_);
  }
}

void CreateBF::Sink(LocalState& local, const DataChunk& chunk) const {
  // materialize the chunk (every column, flattened, owned): the source re-emits it
  // (physical_create_bf.cpp:211-218). The copies are bump-allocated from 1 MiB blocks the state owns (one
  // allocation per ~64 chunks, nothing zero-filled first; 4 MiB blocks advised as transparent huge pages
  // measured no faster).
  const Clock::time_point t0 = Clock::now();
  auto alloc = [&local](size_t words) {
    if (words > local.arena_left) {
      const size_t blk = std::max<size_t>(words, kSinkBlockWords);
      local.storage.emplace_back(new uint64_t[blk]);
      local.arena = local.storage.back().get();
      local.arena_left = blk;
    }
    uint64_t* p = local.arena;
    local.arena += words;
    local.arena_left -= words;
    return p;
  };
  DataChunk m;
  m.count = chunk.count;
  m.data.resize(chunk.data.size());
  for (size_t c = 0; c < chunk.data.size(); c++) {
    const Vector& v = chunk.data[c];
    if (v.data == nullptr && v.type != VectorType::SEQUENCE) continue;  // a column this mirror does not carry
    const size_t es = source_size(v.key_type);
    const size_t nvalid = (chunk.count + 63) / 64 + 1;
    uint64_t* keys = alloc((chunk.count * es + 7) / 8 + 1);
    uint64_t* valid = alloc(nvalid);
    std::fill(valid, valid + nvalid, ~0ULL);  // all valid; NULL rows cleared
    const bool any_null = flatten_column(v, chunk.count, reinterpret_cast<uint8_t*>(keys), valid, 0, /*to_device=*/false);
    Vector f;
    f.type = VectorType::FLAT;
    f.key_type = v.key_type;
    f.data = keys;
    f.validity = any_null ? valid : nullptr;
    m.data[c] = f;
  }
  local.chunks.push_back(std::move(m));
  local.pending_rows += chunk.count;
  local.materialize_s += secs_since(t0);
  // insert into one filter per build column (physical_create_bf.cpp:221-227), a batch at a time
  if (local.pending_rows >= sink_flush_rows_) Flush(local);
}

void CreateBF::Flush(LocalState& local) const {
  if (local.pending_rows == 0) {
    local.pending_from = local.chunks.size();
    return;
  }
  const Clock::time_point t0 = Clock::now();
  std::vector<const DataChunk*> batch;
  for (size_t k = local.pending_from; k < local.chunks.size(); k++)
    if (local.chunks[k].count) batch.push_back(&local.chunks[k]);
  // async: flush k stages through pinned buffer k % 2 (host slots 8 + 4 i + 2 b / + 1 for build column i) and
  // leaves its copies and inserts running; flush k + 2 first waits for them (event b)
  const bool async = local.async_flush && cols_.size() <= kAsyncFlushColumns;
  const int b = async ? static_cast<int>(local.flushes & 1) : 0;
  auto done = static_cast<hipEvent_t>(local.ctx.event(b));
  if (async && local.flushes >= 2) check_hip(hipEventSynchronize(done), "hipEventSynchronize");
  // Once the rows flushed by all states make Finalize's resize certain (its predicate only grows with the row
  // count), inserting into this filter is wasted: Finalize reinitializes it and rehashes every row from HBM. An
  // under-estimated filter is also the small one whose atomic inserts contend on a few words (1e8 rows into the
  // 1 KiB filter of an estimate of 1000: 26 ms of the sink's 64; profiles/r05/host_create_split.jsonl).
  const uint64_t flushed = flushed_rows_.fetch_add(local.pending_rows) + local.pending_rows;
  for (size_t i = 0; i < cols_.size(); i++) {
    const int slot = async ? 8 + 4 * static_cast<int>(i) + 2 * b : 0;
    const DeviceKeyColumn::Segment& g = local.keys[i].Append(local.ctx, batch, cols_[i], slot);
    filters_[i]->NoteKeyType(batch[0]->data.at(cols_[i]).key_type);
    if (WillResize(i, flushed)) {
      skipped_insert_rows_.fetch_add(g.rows);
      if (!async) local.ctx.synchronize();  // the copy out of staging slot 0 is done before the slot is refilled
    } else {
      filters_[i]->InsertDevice(local.ctx, g.col, g.rows, /*synchronize=*/!async);
    }
  }
  if (async) check_hip(hipEventRecord(done, static_cast<hipStream_t>(local.ctx.stream())), "hipEventRecord");
  local.flushes++;
  local.pending_from = local.chunks.size();
  local.pending_rows = 0;
  local.flush_s += secs_since(t0);
}

void CreateBF::Combine(LocalState& local) {
  Flush(local);
  local.ctx.synchronize();  // the state's inserts are done (Finalize and the source read what they wrote)
  std::lock_guard<std::mutex> lk(lock_);
  for (auto& c : local.chunks) {
    total_rows_ += c.count;
    all_chunks_.push_back(std::move(c));
  }
  for (auto& s : local.storage) all_storage_.push_back(std::move(s));
  for (size_t i = 0; i < cols_.size(); i++) all_keys_[i].Splice(std::move(local.keys[i]));
  local.chunks.clear();
  local.storage.clear();
  local.arena = nullptr;
  local.arena_left = 0;
  local.pending_from = 0;
}

bool CreateBF::WillResize(size_t i, uint64_t actual_rows) const {
  const PTBloomFilter& bf = *filters_[i];
  return resize_rule_ == ResizeRule::kReferenceFormula ? rpt_bf_needs_resize(bf.SizedForRows(), actual_rows) == 1
                                                       : bf.NeedsResize(actual_rows);
}

void CreateBF::Finalize() {
  const uint64_t actual_rows = total_rows_;
  // The sink skipped inserts once the rows flushed by every state made the resize certain (Flush). Those rows
  // reach the filter only through the rehash below, so a filter is rehashed whenever any insert was skipped,
  // even if the rows actually combined no longer call for the resize (a state that flushed but never combined:
  // flushed_rows_ > total_rows_). Fail safe: a false negative is never possible.
  const bool skipped = skipped_insert_rows_.load() > 0;
  if (actual_rows > 0) {
    std::unique_ptr<DeviceContext> ctx;  // made only when a filter is rehashed
    for (size_t i = 0; i < filters_.size(); i++) {
      auto& bf = *filters_[i];
      // physical_create_bf.cpp:383-398: resize iff the allocated filter gives < 8 bits per actual row,
      // on this filter's real allocation (default) or by the reference's formula verbatim (ResizeRule);
      // the rehash reads the build column from HBM
      const bool resize = WillResize(i, actual_rows);
      if (resize || skipped) {
        if (!ctx) ctx = std::make_unique<DeviceContext>(device_);
        // no resize: rehash into a filter of the same size (reinitialized for the estimate it was sized for)
        bf.ReinitializeAndRehash(*ctx, resize ? actual_rows : bf.SizedForRows(), all_keys_[i]);
        resized_[i] = resize;
      }
    }
  }
  for (auto& bf : filters_) bf->finalized_ = true;  // physical_create_bf.cpp:409-413
}

std::unique_ptr<CreateBF::GlobalSourceState> CreateBF::GetGlobalSourceState(size_t num_threads) const {
  auto g = std::make_unique<GlobalSourceState>();
  const size_t chunk_count = all_chunks_.size();
  num_threads = std::max<size_t>(1, num_threads);
  const size_t per = std::max<size_t>((chunk_count + num_threads - 1) / num_threads, 1);
  for (size_t t = 0, k = 0; t < num_threads && k < chunk_count; t++) {
    const size_t to = std::min(k + per, chunk_count);
    g->chunks_todo.emplace_back(k, to);
    k = to;
  }
  return g;
}

bool CreateBF::GetData(GlobalSourceState& global, LocalSourceState& local, DataChunk& chunk) const {
  if (local.initial) {
    local.initial = false;
    const size_t id = global.partition_id.fetch_add(1);
    if (id >= global.chunks_todo.size()) {
      local.current = local.chunk_to = 0;
      return false;
    }
    local.chunk_from = global.chunks_todo[id].first;
    local.chunk_to = global.chunks_todo[id].second;
    local.current = local.chunk_from;
  }
  if (local.current >= local.chunk_to) return false;
  chunk = all_chunks_[local.current++];
  return true;
}

bool CreateBF::MinMax(size_t build_column, int64_t& min_value, int64_t& max_value) const {
  return filters_.at(build_column)->MinMax(min_value, max_value);
}

// ---- where the filter runs: scan pushdown or USE_BF ---------------------------------
PushdownPlan PlanPushdown(Device device, FilterType filter_type, bool is_forward_pass, bool has_targets,
                          uint64_t build_rows, bool bf_empty, bool has_minmax) {
  PushdownPlan p;
  // backward-pass CREATE_BFs and forward ones without scan targets push nothing; their USE_BF probes
  // (PushDynamicFilters' early return, physical_create_bf.cpp:284-286; only forward USE_BFs with targets are
  // marked passthrough, rpt_optimizer.cpp:1436-1440,1493-1494)
  if (!is_forward_pass || !has_targets) return p;
  const bool bf = filter_type == FilterType::kAll || filter_type == FilterType::kBfOnly;
  const bool minmax = filter_type == FilterType::kAll || filter_type == FilterType::kMinMaxOnly;
  if (device == Device::kCpu) {
    // the reference: the forward USE_BF passes through and the scan filters do the work
    p.use_bf_passthrough = true;
    p.bf_probed_in_use_bf = false;
    if (build_rows == 0) {
      p.push_always_false = true;  // cpp:288-297 (and nothing else)
      return p;
    }
    p.push_bf = bf && !bf_empty;  // cpp:321-323: the filter of a non-empty build
    p.push_minmax = minmax && has_minmax;
    return p;
  }
  // GPU mode: no BFTableFilter (it would run the filter in DuckDB's CPU scan); the forward USE_BF keeps the probe on
  // the device unless the filter type leaves the BF out (minmax_only: passthrough, as the reference drops it too).
  // Min/max and the empty build's always-false filter stay in the scan: they skip row groups for nothing.
  p.use_bf_passthrough = !bf;
  p.bf_probed_in_use_bf = bf;
  if (build_rows == 0) {
    p.push_always_false = true;
    return p;
  }
  p.push_minmax = minmax && has_minmax;
  return p;
}

// ---- UseBF ---------------------------------------------------------------------------------------
UseBF::UseBF(std::vector<std::shared_ptr<PTBloomFilter>> filters, std::vector<uint64_t> bound_column_indices,
             bool passthrough)
    : filters_(std::move(filters)), cols_(std::move(bound_column_indices)), passthrough_(passthrough) {
  if (filters_.size() != cols_.size()) throw GpuError(RPT_ERR_INVALID_ARGUMENT, "one bound column per filter");
}

uint64_t UseBF::Execute(DeviceContext& ctx, const DataChunk& input, SelectionVector& out) const {
  const uint64_t n = input.count;
  out.resize(n);
  for (uint64_t r = 0; r < n; r++) out[r] = static_cast<uint32_t>(r);
  if (passthrough_) return n;  // physical_use_bf.cpp:62-66
  rows_in_ += n;
  if (filters_.empty() || n == 0) {  // cpp:113-121
    rows_out_ += n;
    return n;
  }
  // The filters that apply (cpp:139-155): not finalized -> skipped; an empty one -> no rows. The AND of
  // the rest over a DuckDB-sized chunk is one launch (its result equals the loop below: each LookupSel
  // sees the previous survivors, and stopping at 0 survivors changes nothing).
  std::vector<size_t> act;
  for (size_t i = 0; i < filters_.size(); i++) {
    const auto& bf = filters_[i];
    if (!bf || !bf->finalized_) continue;
    if (bf->IsEmpty()) {
      out.clear();
      return 0;
    }
    act.push_back(i);
  }
  if (!act.empty() && act.size() <= RPT_MAX_CHAIN && n <= RPT_SMALL_PROBE_ROWS) {
    const DataChunk* in = &input;
    std::vector<const rpt_bf*> bfs;
    std::vector<rpt_key_column> kcs;
    for (size_t k = 0; k < act.size(); k++) {
      const int slot = 16 + 2 * static_cast<int>(k);
      const Flattened f = flatten_pinned(ctx, &in, 1, cols_[act[k]], n, slot);
      rpt_key_column kc;
      kc.key_type = static_cast<int32_t>(f.key_type);
      kc.keys = ctx.host_device_ptr(slot);
      kc.key_sel = nullptr;
      kc.validity = f.any_null ? static_cast<const uint64_t*>(ctx.host_device_ptr(slot + 1)) : nullptr;
      kcs.push_back(kc);
      bfs.push_back(filters_[act[k]]->native());
    }
    auto* h_out = static_cast<uint8_t*>(ctx.host(2, 8 + n * 4));
    void* d_out = ctx.host_device_ptr(2);
    check(rpt_bf_probe_chain(bfs.data(), kcs.data(), static_cast<uint32_t>(act.size()), nullptr, n,
                             reinterpret_cast<uint32_t*>(static_cast<uint8_t*>(d_out) + 8), static_cast<uint64_t*>(d_out),
                             ctx.stream()));
    ctx.synchronize();
    const uint64_t cnt = *reinterpret_cast<const volatile uint64_t*>(h_out);
    const uint32_t* h_sel = reinterpret_cast<const uint32_t*>(h_out + 8);
    out.assign(h_sel, h_sel + cnt);
    rows_out_ += cnt;
    return cnt;
  }
  for (size_t i : act) {
    const auto& bf = filters_[i];
    // LookupSel over the current slice of the input (physical_use_bf.cpp:163,176-179)
    DataChunk sliced;
    sliced.count = out.size();
    sliced.data.resize(input.data.size());
    const Vector& v = input.data.at(cols_[i]);
    Vector sv = v;
    std::vector<uint32_t> composed;
    std::vector<uint64_t> seq_vals;  // SEQUENCE: the selected rows' values (as FLAT)
    if (v.type == VectorType::SEQUENCE) {
      const size_t es = source_size(v.key_type);
      seq_vals.resize((out.size() * es + 7) / 8 + 1);
      uint8_t* dst = reinterpret_cast<uint8_t*>(seq_vals.data());
      for (size_t r = 0; r < out.size(); r++) {
        const uint64_t x = static_cast<uint64_t>(v.seq_start) + static_cast<uint64_t>(v.seq_increment) * out[r];
        std::memcpy(dst + r * es, &x, es);  // little-endian: the low 4 bytes are the int32 value
      }
      sv.type = VectorType::FLAT;
      sv.data = seq_vals.data();
    } else if (v.type == VectorType::FLAT) {
      sv.type = VectorType::DICTIONARY;
      sv.sel = out.data();
      sv.dict_size = n;
    } else if (v.type == VectorType::DICTIONARY) {
      composed.resize(out.size());
      for (size_t r = 0; r < out.size(); r++) composed[r] = v.sel[out[r]];
      sv.sel = composed.data();
    }
    sliced.data[cols_[i]] = sv;
    SelectionVector sel;
    const uint64_t cnt = bf->LookupSel(ctx, sliced, sel, {cols_[i]});
    if (cnt == 0) {  // cpp:166-173
      out.clear();
      return 0;
    }
    SelectionVector next(cnt);
    for (uint64_t r = 0; r < cnt; r++) next[r] = out[sel[r]];
    out.swap(next);
  }
  rows_out_ += out.size();
  return out.size();
}

uint64_t UseBF::ExecuteBatch(DeviceContext& ctx, const std::vector<const DataChunk*>& inputs,
                             std::vector<SelectionVector>& outs) const {
  reset_sels(outs, inputs.size());
  const uint64_t total = total_rows(inputs);
  auto all_rows = [&] {
    for (size_t i = 0; i < inputs.size(); i++) {
      outs[i].resize(inputs[i]->count);
      for (uint64_t r = 0; r < inputs[i]->count; r++) outs[i][r] = static_cast<uint32_t>(r);
    }
    return total;
  };
  if (passthrough_) return all_rows();  // physical_use_bf.cpp:62-66
  rows_in_ += total;
  if (filters_.empty() || total == 0) {  // cpp:113-121
    rows_out_ += total;
    return all_rows();
  }
  if (total >= (1ULL << 32)) throw GpuError(RPT_ERR_INVALID_ARGUMENT, "batch exceeds uint32 row ids");
  {
    // one applicable filter: LookupSelBatch (fused, one piece with the result bits back, or pipelined, by size);
    // several over a large batch: the chained pipeline (flatten, copy, probe and copy back of successive stages
    // overlap); same per-chunk sels as the filter loop below
    std::vector<size_t> act;
    for (size_t i = 0; i < filters_.size(); i++) {
      const auto& bf = filters_[i];
      if (!bf || !bf->finalized_) continue;  // cpp:139-142
      if (bf->IsEmpty()) return 0;           // cpp:145-155
      act.push_back(i);
    }
    if (act.size() == 1 || (!act.empty() && stage_rows_for(ctx, total))) {
      uint64_t count = 0;
      if (act.size() == 1) {  // any size: LookupSelBatch picks the fused, single-piece or pipelined route
        filters_[act[0]]->LookupSelBatch(ctx, inputs, outs, {cols_[act[0]]});
        for (const SelectionVector& o : outs) count += o.size();
      } else {
        count = ExecuteChainPipelined(ctx, inputs, outs, act);
      }
      rows_out_ += count;
      return count;
    }
  }
  auto s = static_cast<hipStream_t>(ctx.stream());
  uint32_t* d_rows = nullptr;  // surviving row ids (ascending, over the batch); nullptr = every row
  uint64_t count = total;
  int cur = 12;  // device slots 12 / 13: the survivors before and after a filter, 14: the count
  auto* d_cnt = static_cast<uint64_t*>(ctx.dev(14, 8));
  auto* h_cnt = static_cast<uint64_t*>(ctx.host(2, 8));
  for (size_t i = 0; i < filters_.size(); i++) {
    const auto& bf = filters_[i];
    if (!bf || !bf->finalized_) continue;  // cpp:139-142
    if (bf->IsEmpty()) return 0;           // cpp:145-155
    // this filter's key column for the whole batch; the probe reads only the surviving rows
    // (row_sel, physical_use_bf.cpp:163,176-179)
    const rpt_key_column kc = stage(ctx, inputs, cols_[i], total);
    const size_t ws_bytes = rpt_bf_probe_workspace_bytes(bf->native(), count);
    void* ws = ctx.dev(2, std::max<size_t>(ws_bytes, 16));
    auto* d_next = static_cast<uint32_t*>(ctx.dev(cur == 12 ? 13 : 12, std::max<uint64_t>(count, 1) * 4));
    check(rpt_bf_probe(bf->native(), &kc, d_rows, count, d_next, d_cnt, ws, ws_bytes, s));
    check_hip(hipMemcpyAsync(h_cnt, d_cnt, 8, hipMemcpyDeviceToHost, s), "copy count");
    ctx.synchronize();  // the next filter needs the count (and reuses the staging slots)
    count = *h_cnt;
    if (count == 0) return 0;  // cpp:166-173
    d_rows = d_next;
    cur = cur == 12 ? 13 : 12;
  }
  rows_out_ += count;
  if (d_rows == nullptr) return all_rows();  // every filter skipped
  auto* h_rows = static_cast<uint32_t*>(ctx.host(3, count * 4));
  check_hip(hipMemcpyAsync(h_rows, d_rows, count * 4, hipMemcpyDeviceToHost, s), "copy sel");
  ctx.synchronize();
  split_sel(ctx, inputs, 0, inputs.size(), h_rows, count, outs);
  return count;
}

// A FLAT / DICTIONARY vector of I32 / I64 keys (element T) at rows rows[0 .. n) - base (ascending): the keys as
// they are, NULLs cleared in `valid_words` from bit `out0` on, 64 rows per step.
template <typename T, bool kDict>
bool gather_typed(const Vector& v, const uint32_t* rows, uint64_t base, uint64_t n, uint8_t* keys, uint64_t* valid_words,
                  uint64_t out0) {
  const T* src = static_cast<const T*>(v.data);
  T* dst = reinterpret_cast<T*>(keys);
  bool any_null = false;
  for (uint64_t j0 = 0; j0 < n; j0 += 64) {
    const uint32_t m = static_cast<uint32_t>(std::min<uint64_t>(64, n - j0));
    uint64_t nulls = 0;
    if (kDict) {
      uint32_t kmax = 0;
      for (uint32_t e = 0; e < m; e++) kmax = std::max(kmax, v.sel[rows[j0 + e] - base]);
      if (kmax >= v.dict_size) throw GpuError(RPT_ERR_INVALID_ARGUMENT, "dictionary index out of range");
    }
    for (uint32_t e = 0; e < m; e++) {
      if (!kDict && j0 + e + 32 < n) __builtin_prefetch(src + (rows[j0 + e + 32] - base));  // the survivors' lines
      const uint64_t r = rows[j0 + e] - base;
      const uint64_t idx = kDict ? v.sel[r] : r;
      std::memcpy(dst + j0 + e, src + idx, sizeof(T));
      if (v.validity) nulls |= static_cast<uint64_t>(!valid_bit(v.validity, idx)) << e;
    }
    any_null |= nulls != 0;
    clear_bits(valid_words, out0 + j0, nulls, m);
  }
  return any_null;
}

// Rows rows[0 .. n) - base (ascending, chunk-local) of one vector gathered as device values into `keys`, their NULLs
// cleared in `valid_words` (preset to all-valid) from bit `out0` on; the same conversions and NULL rules as
// flatten_column. Returns true if any gathered row was NULL.
bool gather_column(const Vector& v, const uint32_t* rows, uint64_t base, uint64_t n, uint8_t* keys,
                   uint64_t* valid_words, uint64_t out0) {
  const KeyType dt = device_type(v.key_type);
  if (dt == v.key_type && (v.type == VectorType::FLAT || v.type == VectorType::DICTIONARY)) {
    const bool dict = v.type == VectorType::DICTIONARY;
    if (dt == KeyType::I32)
      return dict ? gather_typed<uint32_t, true>(v, rows, base, n, keys, valid_words, out0)
                  : gather_typed<uint32_t, false>(v, rows, base, n, keys, valid_words, out0);
    return dict ? gather_typed<uint64_t, true>(v, rows, base, n, keys, valid_words, out0)
                : gather_typed<uint64_t, false>(v, rows, base, n, keys, valid_words, out0);
  }
  const size_t ss = source_size(v.key_type), ds = key_size(dt);
  const uint8_t* src = static_cast<const uint8_t*>(v.data);
  bool any_null = false;
  for (uint64_t j0 = 0; j0 < n; j0 += 64) {
    const uint32_t m = static_cast<uint32_t>(std::min<uint64_t>(64, n - j0));
    uint64_t nulls = 0;
    for (uint32_t e = 0; e < m; e++) {
      const uint64_t r = rows[j0 + e] - base;
      uint8_t seq[8];
      const uint8_t* p;
      switch (v.type) {
        case VectorType::SEQUENCE: {  // never NULL
          const uint64_t x = static_cast<uint64_t>(v.seq_start) + static_cast<uint64_t>(v.seq_increment) * r;
          std::memcpy(seq, &x, 8);
          p = seq;
          break;
        }
        case VectorType::CONSTANT:
          p = src;
          nulls |= static_cast<uint64_t>(!valid_bit(v.validity, 0)) << e;
          break;
        case VectorType::DICTIONARY: {
          const uint32_t idx = v.sel[r];
          if (idx >= v.dict_size) throw GpuError(RPT_ERR_INVALID_ARGUMENT, "dictionary index out of range");
          p = src + static_cast<uint64_t>(idx) * ss;
          nulls |= static_cast<uint64_t>(!valid_bit(v.validity, idx)) << e;
          break;
        }
        default:
          p = src + r * ss;
          nulls |= static_cast<uint64_t>(!valid_bit(v.validity, r)) << e;
          break;
      }
      const uint64_t d = dt == v.key_type ? 0 : device_value(v.key_type, p);
      std::memcpy(keys + (j0 + e) * ds, dt == v.key_type ? static_cast<const void*>(p) : &d, ds);
    }
    any_null |= nulls != 0;
    clear_bits(valid_words, out0 + j0, nulls, m);
  }
  return any_null;
}

// The survivors of a filter as stage rows: out[x] = rows[idx[x]] for x in [0, n) (idx ascending), on the
// context's workers for large n.
void map_survivors(DeviceContext& ctx, const uint32_t* rows, const uint32_t* idx, uint64_t n, uint32_t* out) {
  auto range = [&](uint64_t lo, uint64_t hi) {
    for (uint64_t x = lo; x < hi; x++) out[x] = rows[idx[x]];
  };
  if (n < (1u << 16) || ctx.flatten_threads <= 1) {
    range(0, n);
  } else {
    const size_t n_tasks = std::min<size_t>(n >> 14, 4 * static_cast<size_t>(ctx.flatten_threads));
    ctx.parallel_for(n_tasks, [&](size_t t) { range(n * t / n_tasks, n * (t + 1) / n_tasks); });
  }
}

// Column `col` of a stage's chunks (chunk i starting at stage row row0[i]) at stage rows into pinned slots `slot`
// (keys) / `valid_slot` (validity), on the context's workers for large n. The rows are rows[0 .. n), or, with idx,
// rows[idx[x]] (the previous filter's survivors mapped through its sel, idx ascending), written to mapped[x].
Flattened gather_pinned(DeviceContext& ctx, const DataChunk* const* chunks, const std::vector<uint64_t>& row0,
                        uint64_t col, const uint32_t* rows_in, const uint32_t* idx, uint32_t* mapped, uint64_t n,
                        int slot, int valid_slot) {
  const uint32_t* rows = idx ? mapped : rows_in;
  const KeyType kt = chunks[0]->data.at(col).key_type;
  const size_t es = key_size(device_type(kt));
  const uint64_t nwords = (n + 63) / 64;
  auto* hkeys = static_cast<uint8_t*>(ctx.host(slot, std::max<size_t>(n * es, 16)));
  auto* hvalid = static_cast<uint64_t*>(ctx.host(valid_slot, std::max<size_t>(nwords * 8, 8)));
  std::memset(hvalid, 0xFF, nwords * 8);
  const size_t n_chunks = row0.size() - 1;
  auto range = [&](uint64_t lo, uint64_t hi) {  // rows[lo .. hi): a run per chunk
    if (idx)
      for (uint64_t x = lo; x < hi; x++) mapped[x] = rows_in[idx[x]];
    bool nulls = false;
    size_t c = static_cast<size_t>(std::upper_bound(row0.begin(), row0.end(), static_cast<uint64_t>(rows[lo])) -
                                   row0.begin()) - 1;
    for (uint64_t j = lo; j < hi;) {
      while (c < n_chunks && rows[j] >= row0[c + 1]) c++;
      if (c >= n_chunks) throw GpuError(RPT_ERR_INVALID_ARGUMENT, "survivor row beyond the stage");
      // the chunk's end among the survivors: galloping from j (a chunk holds a few hundred of them)
      const uint32_t bound = static_cast<uint32_t>(row0[c + 1]);
      const uint32_t* p = rows + j;
      const uint32_t* const end = rows + hi;
      size_t step = 16;
      while (static_cast<size_t>(end - p) > step && p[step] < bound) {
        p += step;
        step *= 2;
      }
      const uint32_t* e = std::lower_bound(p, static_cast<size_t>(end - p) > step ? p + step + 1 : end, bound);
      const uint64_t m = static_cast<uint64_t>(e - rows) - j;
      nulls |= gather_column(chunks[c]->data.at(col), rows + j, row0[c], m, hkeys + j * es, hvalid, j);
      j += m;
    }
    return nulls;
  };
  bool any_null = false;
  if (n < (1u << 16) || ctx.flatten_threads <= 1) {
    if (n) any_null = range(0, n);
  } else {
    const size_t n_tasks = std::min<size_t>(n >> 14, 4 * static_cast<size_t>(ctx.flatten_threads));
    std::vector<char> nulls(n_tasks, 0);
    ctx.parallel_for(n_tasks, [&](size_t t) { nulls[t] = range(n * t / n_tasks, n * (t + 1) / n_tasks) ? 1 : 0; });
    for (char c : nulls) any_null |= c != 0;
  }
  return Flattened{device_type(kt), hkeys, hvalid, any_null};
}

// The reference's filter loop (physical_use_bf.cpp:127-179) over a pipelined batch, with the survivors compacted
// on the host between filters. Stage i's first applicable filter's column is flattened into pinned buffer
// b = i % 3, copied on the host-to-device stream and probed over every row on compute stream b (the context's
// stream or one of its aux streams). Each further filter gets only the previous one's survivors: their selection
// vector comes back, the host gathers the next column's keys at those rows and sends them, and the probe's sel
// (indices into the gathered keys) maps back through the survivor list. Against the filter-by-filter path this
// sends a later column's keys for the survivors only (p x the bytes) instead of for every row. Three stages are in
// flight: the chains of stages i-1 and i-2 advance on their own streams, between the host's other work, while the
// copy engine moves stage i. A stage whose survivors run out stops its chain (cpp:166-173); the final survivor list
// is split per chunk.
uint64_t UseBF::ExecuteChainPipelined(DeviceContext& ctx, const std::vector<const DataChunk*>& inputs,
                                      std::vector<SelectionVector>& outs, const std::vector<size_t>& act) const {
  const Clock::time_point t_begin = Clock::now();
  DeviceContext::PipelineStats& ps = ctx.stats;
  const size_t k = act.size();
  std::vector<StageRange> st = pipeline_stages(inputs, cols_[act[0]], stage_rows_for(ctx, total_rows(inputs)));
  for (size_t f = 1; f < k; f++) (void)pipeline_stages(inputs, cols_[act[f]], ~0ULL);  // every column one key type
  uint64_t max_rows = 0;
  size_t ws_bytes = 16;
  for (const StageRange& r : st) {
    max_rows = std::max(max_rows, r.rows);
    for (size_t f = 0; f < k; f++) ws_bytes = std::max(ws_bytes, rpt_bf_probe_workspace_bytes(filters_[act[f]]->native(), r.rows));
  }
  // kNB stages in flight, stage i in buffer b = i % kNB: private slots 32.. (DeviceContext::kSlots) per buffer:
  // host / device 32 + b (the first column's keys), 35 + b (its validity), 38 + b / 41 + b (a later column's
  // gathered keys / validity); host 44 + b / 47 + b (the survivor lists, ping-pong), 50 + b (a later probe's sel),
  // 53 + b (the count); device 50 + b (the probe's sel), 53 (the counts), 54 + b (the probe workspaces); narrow
  // BIGINT first columns: device 64 + b (low words), 67 + b and host 70 + b (the chunks' high words and first rows)
  constexpr int kNB = 3;
  static_assert(kNB == DeviceContext::kAuxStreams + 1 && 73 <= DeviceContext::kSlots, "chain pipeline slots");
  const size_t words = (max_rows + 63) / 64 * 8;
  const size_t es0 = key_size(device_type(inputs[0]->data.at(cols_[act[0]]).key_type));
  void* d_keys[2][kNB];
  void* d_valid[2][kNB];
  uint32_t* d_sel[kNB];
  uint32_t* h_sel[kNB];
  uint32_t* surv[kNB][2];
  uint64_t* h_cnt[kNB];
  void* ws[kNB];
  hipStream_t cs[kNB];
  auto* d_cnt = static_cast<uint64_t*>(ctx.dev(53, kNB * 8));
  for (int b = 0; b < kNB; b++) {
    for (int g = 0; g < 2; g++) {
      (void)ctx.host(32 + 6 * g + b, std::max<size_t>(max_rows * (g ? 8 : es0), 16));
      (void)ctx.host(35 + 6 * g + b, std::max<size_t>(words, 8));
      d_keys[g][b] = ctx.dev(32 + 6 * g + b, std::max<size_t>(max_rows * (g ? 8 : es0), 16));
      d_valid[g][b] = ctx.dev(35 + 6 * g + b, std::max<size_t>(words, 8));
    }
    for (int v = 0; v < 2; v++) surv[b][v] = static_cast<uint32_t*>(ctx.host(44 + 3 * v + b, std::max<size_t>(max_rows * 4, 4)));
    h_sel[b] = static_cast<uint32_t*>(ctx.host(50 + b, std::max<size_t>(max_rows * 4, 4)));
    h_cnt[b] = static_cast<uint64_t*>(ctx.host(53 + b, 8));
    d_sel[b] = static_cast<uint32_t*>(ctx.dev(50 + b, std::max<size_t>(max_rows * 4, 4)));
    ws[b] = ctx.dev(54 + b, ws_bytes);
    cs[b] = static_cast<hipStream_t>(b == 0 ? ctx.stream() : ctx.aux_stream(b - 1));
  }
  bool narrow = ctx.narrow_keys && inputs[0]->data.at(cols_[act[0]]).key_type == KeyType::I64;  // until a stage is not
  void* d_lo[kNB] = {};
  void* d_meta[kNB] = {};
  if (narrow) {
    size_t max_chunks = 0;
    for (const StageRange& r : st) max_chunks = std::max(max_chunks, r.c_hi - r.c_lo);
    for (int b = 0; b < kNB; b++) {
      d_lo[b] = ctx.dev(64 + b, std::max<size_t>(max_rows * 4, 16));
      d_meta[b] = ctx.dev(67 + b, (2 * max_chunks + 1) * 4);
      (void)ctx.host(70 + b, (2 * max_chunks + 1) * 4);
    }
  }
  auto h = static_cast<hipStream_t>(ctx.h2d_stream());
  auto copied = [&](int b) { return static_cast<hipEvent_t>(ctx.event(b)); };
  auto arrived = [&](int b) { return static_cast<hipEvent_t>(ctx.event(kNB + b)); };  // a count (+ sel) on the host
  auto probed = [&](int b) { return static_cast<hipEvent_t>(ctx.event(2 * kNB + b)); };  // the first probe read its keys
  rpt_key_column kc0[kNB];
  uint64_t count = 0;
  // A stage's chain as a state machine, so its round trips overlap the next stage's flatten: phase 0 = the first
  // probe's count and the head of its sel are on their way (the head sized from the previous stage's survivors,
  // so one round trip usually brings the whole sel), 1 = the rest of that sel, 2 = filter `lev`'s count and sel
  // (indices into its input list surv[b][sv]); advance() takes every step whose event has fired (all of them,
  // waiting, when `block`).
  struct Chain {
    size_t j = 0;
    int phase = 0;
    size_t lev = 0;
    int sv = 0;
    uint64_t n = 0, head = 0;
    bool live = false;
    std::vector<uint64_t> row0;
  } ch[kNB];
  double head_frac = 0.25;  // the first probe's pass fraction expected (the last stage's)
  // probe filter `lev` over n keys, its count and `sel_rows` sel entries back to the host (a later filter's count
  // is <= n, so one copy of n brings its whole sel)
  auto probe = [&](int b, size_t lev, const rpt_key_column* kc, uint64_t n, uint32_t* sel_to, uint64_t sel_rows) {
    check(rpt_bf_probe(filters_[act[lev]]->native(), kc, nullptr, n, d_sel[b], d_cnt + b, ws[b], ws_bytes, cs[b]));
    check_hip(hipMemcpyAsync(h_cnt[b], d_cnt + b, 8, hipMemcpyDeviceToHost, cs[b]), "copy count");
    if (sel_rows) check_hip(hipMemcpyAsync(sel_to, d_sel[b], sel_rows * 4, hipMemcpyDeviceToHost, cs[b]), "copy sel");
    check_hip(hipEventRecord(arrived(b), cs[b]), "hipEventRecord");
  };
  // gather filter c.lev's column at the survivors (mapped through the previous filter's sel when `idx`) and probe it
  auto next_filter = [&](Chain& c, int b, const uint32_t* idx) {
    Clock::time_point t0 = Clock::now();
    const Flattened g = gather_pinned(ctx, inputs.data() + st[c.j].c_lo, c.row0, cols_[act[c.lev]], surv[b][c.sv], idx,
                                      surv[b][c.sv ^ 1], c.n, 38 + b, 41 + b);
    if (idx) c.sv ^= 1;
    ps.flatten_s += secs_since(t0);
    t0 = Clock::now();
    const rpt_key_column kc = copy_flattened(ctx, g, c.n, d_keys[1][b], d_valid[1][b], cs[b]);
    probe(b, c.lev, &kc, c.n, h_sel[b], c.n);
    ps.enqueue_s += secs_since(t0);
    c.phase = 2;
  };
  auto advance = [&](Chain& c, bool block) {
    const int b = static_cast<int>(c.j % kNB);
    while (c.live) {
      if (block) {
        const Clock::time_point t0 = Clock::now();
        check_hip(hipEventSynchronize(arrived(b)), "hipEventSynchronize");
        ps.wait_count_s += secs_since(t0);
      } else {
        const hipError_t q = hipEventQuery(arrived(b));
        if (q == hipErrorNotReady) return;
        check_hip(q, "hipEventQuery");
      }
      bool done = false;
      if (c.phase == 0) {
        c.n = *h_cnt[b];
        head_frac = static_cast<double>(c.n) / static_cast<double>(st[c.j].rows);
        if (c.n == 0) {
          done = true;
        } else if (c.n > c.head) {  // the rest of the first filter's sel (stage row ids)
          check_hip(hipMemcpyAsync(surv[b][0] + c.head, d_sel[b] + c.head, (c.n - c.head) * 4, hipMemcpyDeviceToHost, cs[b]),
                    "copy sel");
          check_hip(hipEventRecord(arrived(b), cs[b]), "hipEventRecord");
          c.phase = 1;
        } else {
          c.lev = 1;
          next_filter(c, b, nullptr);
        }
      } else if (c.phase == 1) {
        c.lev = 1;
        next_filter(c, b, nullptr);
      } else {
        const uint64_t m = *h_cnt[b];
        c.n = m;
        if (m == 0) {
          done = true;
        } else if (++c.lev == k) {  // the last filter's survivors as stage rows
          const Clock::time_point t0 = Clock::now();
          map_survivors(ctx, surv[b][c.sv], h_sel[b], m, surv[b][c.sv ^ 1]);
          c.sv ^= 1;
          ps.split_s += secs_since(t0);
          done = true;
        } else {
          next_filter(c, b, h_sel[b]);
        }
      }
      if (done) {
        const Clock::time_point t0 = Clock::now();
        split_sel(ctx, inputs, st[c.j].c_lo, st[c.j].c_hi, surv[b][c.sv], c.n, outs);
        count += c.n;
        ps.split_s += secs_since(t0);
        c.live = false;
      }
    }
  };
  try {
    for (size_t i = 0; i < st.size(); i++) {
      const int b = static_cast<int>(i % kNB);
      advance(ch[b], true);  // stage i - kNB: its buffers are about to be reused
      for (int o = 1; o < kNB; o++) advance(ch[(b + o) % kNB], false);
      Clock::time_point t0 = Clock::now();
      if (i >= kNB) check_hip(hipEventSynchronize(copied(b)), "hipEventSynchronize");
      ps.wait_copy_s += secs_since(t0);
      t0 = Clock::now();
      const Flattened f = flatten_pinned(ctx, inputs.data() + st[i].c_lo, st[i].c_hi - st[i].c_lo, cols_[act[0]],
                                         st[i].rows, 32 + b, 35 + b, narrow ? 70 + b : -1);
      narrow = f.narrow;
      ps.narrow_stages += f.narrow;
      ps.flatten_s += secs_since(t0);
      t0 = Clock::now();
      if (i >= kNB) check_hip(hipStreamWaitEvent(h, probed(b), 0), "hipStreamWaitEvent");  // stage i - kNB read them
      kc0[b] = copy_flattened(ctx, f, st[i].rows, d_keys[0][b], d_valid[0][b], h, d_lo[b], d_meta[b]);
      check_hip(hipEventRecord(copied(b), h), "hipEventRecord");
      check_hip(hipStreamWaitEvent(cs[b], copied(b), 0), "hipStreamWaitEvent");
      Chain& c = ch[b];
      c.head = std::min<uint64_t>(st[i].rows, static_cast<uint64_t>(head_frac * 1.25 * static_cast<double>(st[i].rows)) + 4096);
      probe(b, 0, &kc0[b], st[i].rows, surv[b][0], c.head);
      check_hip(hipEventRecord(probed(b), cs[b]), "hipEventRecord");
      ps.enqueue_s += secs_since(t0);
      c.j = i;
      c.phase = 0;
      c.sv = 0;
      c.live = true;
      c.row0.assign(st[i].c_hi - st[i].c_lo + 1, 0);
      for (size_t x = st[i].c_lo; x < st[i].c_hi; x++) c.row0[x - st[i].c_lo + 1] = c.row0[x - st[i].c_lo] + inputs[x]->count;
      for (int o = 1; o < kNB; o++) advance(ch[(b + o) % kNB], false);
    }
    for (size_t i = st.size() > kNB ? st.size() - kNB : 0; i < st.size(); i++) advance(ch[i % kNB], true);
  } catch (...) {
    // nothing may still use the staging buffers: the copy stream and EVERY stage stream (the third
    // stage's stream was left running, so its late copies could land in the next call's pinned buffers)
    (void)hipStreamSynchronize(h);
    for (int b = 0; b < kNB; b++) (void)hipStreamSynchronize(cs[b]);
    throw;
  }
  ps.stages += st.size();
  ps.rows += total_rows(inputs);
  ps.total_s += secs_since(t_begin);
  return count;
}

}  // namespace rpt
