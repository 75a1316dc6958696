// test_host_mirror.cpp — the C++ host mirror (include/rpt_host.hpp) end to end on the GPU, checked
// against the CPU restatement (oracle/librpt_oracle.so, test infrastructure).
//
// CREATE_BF: 4 sink threads, 2048-row chunks (last one ragged), FLAT/CONSTANT/DICTIONARY vectors with
// NULLs, sink batches staged to HBM, an under-estimated cardinality so Finalize must
// ReinitializeAndRehash (from the HBM key segments); the parallel source re-emitting the materialized
// chunks; then USE_BF with two filters (chain = AND: one launch per chunk, and the filter-by-filter loop
// over a chunk beyond RPT_SMALL_PROBE_ROWS), the empty-build early exit, the not-finalized
// skip and passthrough; the build's min/max dynamic filter; a composite (two-column) key filter; a 256 MiB filter whose
// batched insert and lookup take the bucketed strategy.
#include <climits>
#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <iterator>
#include <limits>
#include <type_traits>
#include <cstring>
#include <random>
#include <thread>
#include <vector>

#include "rpt_host.hpp"

extern "C" {
int rpt_oracle_needs_resize(uint64_t sized_for_rows, uint64_t actual_rows);
int rpt_oracle_needs_resize_alloc(int log_num_blocks, uint64_t actual_rows);
int rpt_oracle_log_num_blocks(uint64_t n_rows);
void rpt_oracle_insert_i64(uint64_t* words, int log_nb, const int64_t* keys, const uint32_t* key_sel,
                           const uint64_t* validity, uint64_t n);
void rpt_oracle_insert_i32(uint64_t* words, int log_nb, const int32_t* keys, const uint32_t* key_sel,
                           const uint64_t* validity, uint64_t n);
uint64_t rpt_oracle_probe_i64(const uint64_t* words, int log_nb, const int64_t* keys, const uint32_t* key_sel,
                              const uint64_t* validity, uint64_t n, uint32_t* sel);
uint64_t rpt_oracle_probe_i32(const uint64_t* words, int log_nb, const int32_t* keys, const uint32_t* key_sel,
                              const uint64_t* validity, uint64_t n, uint32_t* sel);
void rpt_oracle_hash_i64(const int64_t* keys, const uint32_t* key_sel, const uint64_t* validity, uint64_t n,
                         uint64_t* out);
void rpt_oracle_hash_combine_i32(const int32_t* keys, const uint32_t* key_sel, const uint64_t* validity, uint64_t n,
                                 uint64_t* inout);
void rpt_oracle_insert_hashes(uint64_t* words, int log_nb, const uint64_t* h, uint64_t n);
uint64_t rpt_oracle_lookup_sel_hashes(const uint64_t* words, int log_nb, const uint64_t* h, uint64_t n, uint32_t* sel);
int rpt_oracle_minmax_i64(const int64_t* keys, const uint32_t* key_sel, const uint64_t* validity, uint64_t n,
                          int64_t* out2);
int rpt_oracle_minmax_i32(const int32_t* keys, const uint32_t* key_sel, const uint64_t* validity, uint64_t n,
                          int64_t* out2);
}

static int g_fail = 0;
#define EXPECT(cond, ...)                        \
  do {                                           \
    if (!(cond)) {                               \
      fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
      fprintf(stderr, __VA_ARGS__);              \
      fprintf(stderr, "\n");                     \
      g_fail++;                                  \
    }                                            \
  } while (0)

// A host-side "table" of two key columns, with per-chunk vector shapes.
struct Table {
  std::vector<int64_t> c0;   // BIGINT keys
  std::vector<bool> v0;      // validity of c0
  std::vector<int32_t> c1;   // INTEGER keys
  std::vector<bool> v1;
};

static std::vector<uint64_t> pack(const std::vector<bool>& v, size_t lo, size_t n) {
  std::vector<uint64_t> w((n + 63) / 64 + 1, 0);
  for (size_t i = 0; i < n; i++)
    if (v[lo + i]) w[i / 64] |= 1ULL << (i % 64);
  return w;
}

// Chunk storage: keeps the buffers each rpt::Vector points into alive.
struct ChunkStore {
  std::vector<std::vector<int64_t>> i64;
  std::vector<std::vector<int32_t>> i32;
  std::vector<std::vector<uint32_t>> sel;
  std::vector<std::vector<uint64_t>> valid;
  std::vector<rpt::DataChunk> chunks;
};

// Cut rows [0, n) into 2048-row chunks; chunk k uses shape k % 3 for column 0 (FLAT, DICTIONARY, and
// CONSTANT when the chunk's c0 values are all equal) and DICTIONARY for column 1 on odd chunks.
static void make_chunks(const Table& t, size_t n, ChunkStore& st, bool allow_constant) {
  for (size_t lo = 0, k = 0; lo < n; lo += 2048, k++) {
    const size_t cnt = std::min<size_t>(2048, n - lo);
    rpt::DataChunk ch;
    ch.count = cnt;
    ch.data.resize(3);
    // column 0
    rpt::Vector a;
    a.key_type = rpt::KeyType::I64;
    bool all_same = true;
    for (size_t i = 1; i < cnt; i++) all_same &= (t.c0[lo + i] == t.c0[lo] && t.v0[lo + i] == t.v0[lo]);
    if (allow_constant && all_same) {
      st.i64.push_back({t.c0[lo]});
      st.valid.push_back({t.v0[lo] ? 1ULL : 0ULL});
      a.type = rpt::VectorType::CONSTANT;
      a.data = st.i64.back().data();
      a.validity = st.valid.back().data();
    } else if (k % 3 == 1) {
      // dictionary: reversed distinct copy + selection
      std::vector<int64_t> dict(cnt);
      std::vector<uint32_t> sel(cnt);
      std::vector<bool> dv(cnt);
      for (size_t i = 0; i < cnt; i++) {
        dict[cnt - 1 - i] = t.c0[lo + i];
        dv[cnt - 1 - i] = t.v0[lo + i];
        sel[i] = static_cast<uint32_t>(cnt - 1 - i);
      }
      std::vector<uint64_t> w((cnt + 63) / 64 + 1, 0);
      for (size_t i = 0; i < cnt; i++)
        if (dv[i]) w[i / 64] |= 1ULL << (i % 64);
      st.i64.push_back(std::move(dict));
      st.sel.push_back(std::move(sel));
      st.valid.push_back(std::move(w));
      a.type = rpt::VectorType::DICTIONARY;
      a.data = st.i64.back().data();
      a.sel = st.sel.back().data();
      a.dict_size = cnt;
      a.validity = st.valid.back().data();
    } else {
      st.i64.push_back(std::vector<int64_t>(t.c0.begin() + lo, t.c0.begin() + lo + cnt));
      st.valid.push_back(pack(t.v0, lo, cnt));
      a.type = rpt::VectorType::FLAT;
      a.data = st.i64.back().data();
      a.validity = st.valid.back().data();
    }
    ch.data[0] = a;
    // column 1 (INTEGER)
    rpt::Vector b;
    b.key_type = rpt::KeyType::I32;
    if (k % 2) {
      std::vector<int32_t> dict(cnt);
      std::vector<uint32_t> sel(cnt);
      for (size_t i = 0; i < cnt; i++) {
        dict[i] = t.c1[lo + i];
        sel[i] = static_cast<uint32_t>(i);
      }
      st.i32.push_back(std::move(dict));
      st.sel.push_back(std::move(sel));
      st.valid.push_back(pack(t.v1, lo, cnt));
      b.type = rpt::VectorType::DICTIONARY;
      b.data = st.i32.back().data();
      b.sel = st.sel.back().data();
      b.dict_size = cnt;
      b.validity = st.valid.back().data();
    } else {
      st.i32.push_back(std::vector<int32_t>(t.c1.begin() + lo, t.c1.begin() + lo + cnt));
      st.valid.push_back(pack(t.v1, lo, cnt));
      b.type = rpt::VectorType::FLAT;
      b.data = st.i32.back().data();
      b.validity = st.valid.back().data();
    }
    ch.data[1] = b;
    ch.data[2] = rpt::Vector();  // an unrelated payload column the operators never touch
    st.chunks.push_back(std::move(ch));
  }
}

static Table make_table(size_t n, uint64_t seed, int null_every, size_t const_run) {
  std::mt19937_64 rng(seed);
  Table t;
  t.c0.resize(n);
  t.v0.resize(n);
  t.c1.resize(n);
  t.v1.resize(n);
  for (size_t i = 0; i < n; i++) {
    t.c0[i] = static_cast<int64_t>(rng() % 200000) - 100000;
    t.v0[i] = null_every == 0 || (i % null_every) != 0;
    t.c1[i] = static_cast<int32_t>(rng() % 300000) - 7;
    t.v1[i] = null_every == 0 || (i % (null_every + 2)) != 1;
  }
  // a constant chunk (chunk 3) for the CONSTANT vector path
  for (size_t i = 3 * 2048; i < std::min(n, 3 * 2048 + const_run); i++) {
    t.c0[i] = 4242;
    t.v0[i] = true;
  }
  return t;
}


// ---------------- key types beyond INTEGER / BIGINT (rpt_host.hpp KeyType) -------------------------
// The conversion restated independently of the mirror: what DuckDB's Hash<T> hashes, as an I32 / I64 device
// value (Hash<T> casts narrow integers to uint32_t; FLOAT / DOUBLE hash their bits after -0.0 -> 0.0 and
// NaN -> the quiet NaN; parity unpinned, like the int32 rule).
template <typename T>
static uint64_t expect_device(T v) {
  if constexpr (std::is_floating_point<T>::value) {
    if (v == T(0)) v = T(0);
    else if (v != v) v = std::numeric_limits<T>::quiet_NaN();
    if constexpr (sizeof(T) == 4) {
      uint32_t b;
      std::memcpy(&b, &v, 4);
      return b;
    } else {
      uint64_t b;
      std::memcpy(&b, &v, 8);
      return b;
    }
  } else if constexpr (sizeof(T) == 8) {
    return static_cast<uint64_t>(v);
  } else {
    return static_cast<uint32_t>(v);  // sign-extends signed types, as static_cast<uint32_t> in Hash<T>
  }
}

// One key type end to end: FLAT (with NULLs), DICTIONARY and CONSTANT chunks (+ SEQUENCE for integers)
// inserted through PTBloomFilter::InsertBatch and through CreateBF; filter words and LookupSel against the
// oracle fed the restated device values; min/max exact or absent per KeyType; the CREATE_BF source
// re-emits the original values.
template <typename T>
static void typed_keys_case(int dev, rpt::KeyType kt, const std::vector<T>& vals, bool minmax_kept, const char* name) {
  const size_t n = vals.size();
  const bool dev64 = kt == rpt::KeyType::U32 || kt == rpt::KeyType::U64 || kt == rpt::KeyType::F64;
  std::vector<bool> valid(n);
  for (size_t i = 0; i < n; i++) valid[i] = i % 13 != 5;
  // chunks: [0, 2048) FLAT, [2048, n) DICTIONARY (reversed), plus one CONSTANT and (integers) one SEQUENCE chunk
  std::vector<uint64_t> vw0 = pack(valid, 0, 2048), vw1;
  std::vector<T> dict(vals.begin() + 2048, vals.end());
  std::reverse(dict.begin(), dict.end());
  std::vector<uint32_t> dsel(n - 2048);
  std::vector<bool> dvalid(n - 2048);
  for (size_t i = 0; i < n - 2048; i++) {
    dsel[i] = static_cast<uint32_t>(n - 2048 - 1 - i);
    dvalid[n - 2048 - 1 - i] = valid[2048 + i];
  }
  vw1 = pack(dvalid, 0, n - 2048);
  const T cval = vals[7];
  const uint64_t cvalid = 1;
  std::vector<rpt::DataChunk> chunks(3);
  chunks[0].count = 2048;
  chunks[0].data.resize(1);
  chunks[0].data[0].key_type = kt;
  chunks[0].data[0].data = vals.data();
  chunks[0].data[0].validity = vw0.data();
  chunks[1].count = n - 2048;
  chunks[1].data.resize(1);
  chunks[1].data[0].key_type = kt;
  chunks[1].data[0].type = rpt::VectorType::DICTIONARY;
  chunks[1].data[0].data = dict.data();
  chunks[1].data[0].sel = dsel.data();
  chunks[1].data[0].dict_size = dict.size();
  chunks[1].data[0].validity = vw1.data();
  chunks[2].count = 100;
  chunks[2].data.resize(1);
  chunks[2].data[0].key_type = kt;
  chunks[2].data[0].type = rpt::VectorType::CONSTANT;
  chunks[2].data[0].data = &cval;
  chunks[2].data[0].validity = &cvalid;
  const bool integer = !std::is_floating_point<T>::value;
  if (integer) {  // a SEQUENCE chunk whose values wrap at the column's width
    rpt::DataChunk q;
    q.count = 300;
    q.data.resize(1);
    q.data[0].key_type = kt;
    q.data[0].type = rpt::VectorType::SEQUENCE;
    q.data[0].seq_start = -150;
    q.data[0].seq_increment = 97;
    chunks.push_back(q);
  }
  // the same rows flattened by hand: device values + validity
  std::vector<uint64_t> dv;
  std::vector<bool> ok;
  std::vector<T> orig;
  for (size_t i = 0; i < 2048; i++) { dv.push_back(expect_device(vals[i])); ok.push_back(valid[i]); orig.push_back(vals[i]); }
  for (size_t i = 0; i < n - 2048; i++) {
    dv.push_back(expect_device(dict[dsel[i]]));
    ok.push_back(dvalid[dsel[i]]);
    orig.push_back(dict[dsel[i]]);
  }
  for (size_t i = 0; i < 100; i++) { dv.push_back(expect_device(cval)); ok.push_back(true); orig.push_back(cval); }
  if (integer)
    for (size_t i = 0; i < 300; i++) {
      const T x = static_cast<T>(static_cast<uint64_t>(-150) + 97ULL * i);
      dv.push_back(expect_device(x));
      ok.push_back(true);
      orig.push_back(x);
    }
  const size_t total = dv.size();
  const std::vector<uint64_t> vwall = pack(ok, 0, total);
  rpt::PTBloomFilter f;
  f.Initialize(dev, static_cast<uint32_t>(total));
  const int lnb = f.LogNumBlocks();
  std::vector<uint64_t> w(1ULL << lnb, 0);
  std::vector<int64_t> d64(total);
  std::vector<int32_t> d32(total);
  for (size_t i = 0; i < total; i++) {
    d64[i] = static_cast<int64_t>(dv[i]);
    d32[i] = static_cast<int32_t>(static_cast<uint32_t>(dv[i]));
  }
  if (dev64) rpt_oracle_insert_i64(w.data(), lnb, d64.data(), nullptr, vwall.data(), total);
  else rpt_oracle_insert_i32(w.data(), lnb, d32.data(), nullptr, vwall.data(), total);
  rpt::DeviceContext ctx(dev);
  std::vector<const rpt::DataChunk*> ptrs;
  for (const auto& c : chunks) ptrs.push_back(&c);
  f.InsertBatch(ctx, ptrs, {0});
  EXPECT(f.ExportWords() == w, "%s: filter words differ from the oracle", name);
  // LookupSel of every chunk == the oracle's probe of the device values
  size_t base = 0;
  std::vector<uint32_t> exp(total);
  for (const auto& c : chunks) {
    rpt::SelectionVector sel;
    f.LookupSel(ctx, c, sel, {0});
    const std::vector<uint64_t> vwc = pack(ok, base, c.count);
    const uint64_t ne = dev64 ? rpt_oracle_probe_i64(w.data(), lnb, d64.data() + base, nullptr, vwc.data(), c.count, exp.data())
                              : rpt_oracle_probe_i32(w.data(), lnb, d32.data() + base, nullptr, vwc.data(), c.count, exp.data());
    EXPECT(sel == std::vector<uint32_t>(exp.begin(), exp.begin() + ne), "%s: LookupSel chunk at row %zu", name, base);
    base += c.count;
  }
  // min/max: exact for the integer types up to 32 bits, absent for U64 / F32 / F64
  int64_t mn = 0, mx = 0;
  const bool has = f.MinMax(mn, mx);
  if (minmax_kept) {
    int64_t emn = INT64_MAX, emx = INT64_MIN;
    for (size_t i = 0; i < total; i++)
      if (ok[i]) {
        emn = std::min<int64_t>(emn, static_cast<int64_t>(orig[i]));
        emx = std::max<int64_t>(emx, static_cast<int64_t>(orig[i]));
      }
    EXPECT(has && mn == emn && mx == emx, "%s: min/max %lld %lld, expected %lld %lld", name, (long long)mn, (long long)mx,
           (long long)emn, (long long)emx);
  } else {
    EXPECT(!has, "%s: min/max must not be reported", name);
  }
  // CREATE_BF over the same chunks: the same filter words; the source re-emits the original values
  rpt::CreateBF cb(dev, total, {0});
  auto l = cb.MakeLocalState();
  for (const auto& c : chunks) cb.Sink(*l, c);
  cb.Combine(*l);
  cb.Finalize();
  EXPECT(cb.GetBloomFilter(0)->ExportWords() == w, "%s: CREATE_BF filter words differ", name);
  EXPECT(cb.MinMax(0, mn, mx) == minmax_kept, "%s: CREATE_BF min/max presence", name);
  auto gs = cb.GetGlobalSourceState(1);
  rpt::CreateBF::LocalSourceState ls;
  rpt::DataChunk out;
  size_t r = 0;
  bool same = true;
  while (cb.GetData(*gs, ls, out)) {
    const T* p = static_cast<const T*>(out.data[0].data);
    for (size_t i = 0; i < out.count; i++, r++)
      if (ok[r] && std::memcmp(&p[i], &orig[r], sizeof(T)) != 0) same = false;
  }
  EXPECT(same && r == total, "%s: CREATE_BF source re-emits the original values", name);
}

static void typed_keys(int dev) {
  std::mt19937_64 rng(77);
  const size_t n = 5000;
  auto gen = [&](auto zero) {
    using T = decltype(zero);
    std::vector<T> v(n);
    for (auto& x : v) x = static_cast<T>(rng());
    return v;
  };
  typed_keys_case(dev, rpt::KeyType::I8, gen(int8_t{}), true, "TINYINT");
  typed_keys_case(dev, rpt::KeyType::I16, gen(int16_t{}), true, "SMALLINT");
  typed_keys_case(dev, rpt::KeyType::U8, gen(uint8_t{}), true, "UTINYINT");
  typed_keys_case(dev, rpt::KeyType::U16, gen(uint16_t{}), true, "USMALLINT");
  typed_keys_case(dev, rpt::KeyType::U32, gen(uint32_t{}), true, "UINTEGER");  // values >= 2^31 included
  typed_keys_case(dev, rpt::KeyType::U64, gen(uint64_t{}), false, "UBIGINT");
  std::vector<float> fv(n);
  std::vector<double> dv(n);
  for (size_t i = 0; i < n; i++) {
    fv[i] = static_cast<float>(static_cast<int64_t>(rng() % 2000001) - 1000000) / 7.0f;
    dv[i] = static_cast<double>(static_cast<int64_t>(rng() % 2000001) - 1000000) / 7.0;
  }
  uint32_t fnan = 0x7FC01234u;  // a NaN with a payload, and its sign-flipped twin
  uint64_t dnan = 0xFFF0000000000042ULL;
  std::memcpy(&fv[10], &fnan, 4);
  fnan ^= 0x80000000u;
  std::memcpy(&fv[11], &fnan, 4);
  std::memcpy(&dv[10], &dnan, 8);
  fv[12] = -0.0f;
  dv[12] = -0.0;
  fv[13] = std::numeric_limits<float>::infinity();
  dv[13] = -std::numeric_limits<double>::infinity();
  typed_keys_case(dev, rpt::KeyType::F32, fv, false, "FLOAT");
  typed_keys_case(dev, rpt::KeyType::F64, dv, false, "DOUBLE");
  // the equality transform: -0.0 finds 0.0, a NaN finds any other NaN
  rpt::PTBloomFilter f;
  f.Initialize(dev, 100);
  rpt::DeviceContext ctx(dev);
  const double ins[2] = {-0.0, std::numeric_limits<double>::quiet_NaN()};
  uint64_t other_nan = 0x7FF0000000000001ULL;  // signalling, another payload
  double probe[3] = {0.0, 0.0, 1.5};
  std::memcpy(&probe[1], &other_nan, 8);
  rpt::DataChunk a, b;
  a.count = 2;
  a.data.resize(1);
  a.data[0].key_type = rpt::KeyType::F64;
  a.data[0].data = ins;
  b = a;
  b.count = 3;
  b.data[0].data = probe;
  f.Insert(ctx, a, {0});
  rpt::SelectionVector sel;
  f.LookupSel(ctx, b, sel, {0});
  EXPECT(sel.size() >= 2 && sel[0] == 0 && sel[1] == 1, "DOUBLE: -0.0 / NaN equality transform");
}

// Pipelined batches big enough for the context's worker threads (stages of >= 1 Mi rows are flattened, and
// stage sels of >= 64 Ki survivors split, on flatten_threads threads): FLAT / DICTIONARY chunks with NULLs,
// both key columns, the selection vectors reused across calls (their capacity is kept), UseBF::ExecuteBatch's
// single-filter route through the pipeline; every chunk against the oracle.
static void pipelined_workers(int dev) {
  const size_t nb = (2u << 20) + 777, np = (3u << 20) + 1234;  // both pipelined (>= 2 stages of 1 Mi rows)
  Table bt = make_table(nb, 11, 53, 0), pt = make_table(np, 12, 41, 0);
  ChunkStore bst, pst;
  make_chunks(bt, nb, bst, false);
  make_chunks(pt, np, pst, false);
  std::vector<const rpt::DataChunk*> bptrs, pptrs;
  for (const auto& ch : bst.chunks) bptrs.push_back(&ch);
  for (const auto& ch : pst.chunks) pptrs.push_back(&ch);
  for (int c = 0; c < 2; c++) {
    rpt::DeviceContext ctx(dev);
    ctx.pipeline_rows = 1u << 20;
    ctx.flatten_threads = 4;
    auto f = std::make_shared<rpt::PTBloomFilter>();
    f->Initialize(dev, static_cast<uint32_t>(nb));
    f->InsertBatch(ctx, bptrs, {static_cast<uint64_t>(c)});
    const int lnb = f->LogNumBlocks();
    std::vector<uint64_t> w(1ULL << lnb, 0);
    const std::vector<uint64_t> vb = pack(c == 0 ? bt.v0 : bt.v1, 0, nb);
    if (c == 0) rpt_oracle_insert_i64(w.data(), lnb, bt.c0.data(), nullptr, vb.data(), nb);
    else rpt_oracle_insert_i32(w.data(), lnb, bt.c1.data(), nullptr, vb.data(), nb);
    EXPECT(f->ExportWords() == w, "worker-thread pipelined insert (column %d) differs from the oracle", c);
    f->finalized_ = true;
    // expected sels per chunk (chunk k = rows [2048 k, ...))
    std::vector<rpt::SelectionVector> want(pptrs.size());
    size_t total = 0;
    for (size_t k = 0; k < pptrs.size(); k++) {
      const size_t lo = 2048 * k, cnt = pptrs[k]->count;
      const std::vector<uint64_t> vp = pack(c == 0 ? pt.v0 : pt.v1, lo, cnt);
      want[k].resize(cnt);
      const uint64_t ne = c == 0 ? rpt_oracle_probe_i64(w.data(), lnb, pt.c0.data() + lo, nullptr, vp.data(), cnt, want[k].data())
                                 : rpt_oracle_probe_i32(w.data(), lnb, pt.c1.data() + lo, nullptr, vp.data(), cnt, want[k].data());
      want[k].resize(ne);
      total += ne;
    }
    EXPECT(total > (1u << 17), "column %d: %zu survivors (the split must run on the workers)", c, total);
    std::vector<rpt::SelectionVector> sels;
    for (int rep = 0; rep < 3; rep++) {  // the second call reuses the vectors the first one filled; the third copies sels back
      ctx.stats = {};
      ctx.bits_back = rep < 2;
      f->LookupSelBatch(ctx, pptrs, sels, {static_cast<uint64_t>(c)});
      EXPECT(sels.size() == pptrs.size() && ctx.stats.stages >= 3 && ctx.stats.rows == np, "pipeline stats (column %d)", c);
      size_t bad = 0;
      for (size_t k = 0; k < pptrs.size(); k++) bad += sels[k] != want[k];
      EXPECT(bad == 0, "worker-thread pipelined lookup (column %d, call %d): %zu chunks differ", c, rep, bad);
    }
    ctx.bits_back = true;
    rpt::UseBF ub({f}, {static_cast<uint64_t>(c)});
    std::vector<rpt::SelectionVector> outs(5, rpt::SelectionVector(7, 9));  // stale contents must not leak
    const uint64_t got = ub.ExecuteBatch(ctx, pptrs, outs);
    size_t bad = 0;
    for (size_t k = 0; k < pptrs.size(); k++) bad += outs[k] != want[k];
    EXPECT(got == total && outs.size() == pptrs.size() && bad == 0, "ExecuteBatch through the pipeline (column %d): %zu chunks differ", c, bad);
    // a dictionary index out of range in a chunk of the third stage: the worker thread that flattens it throws,
    // the pipeline drains its streams and LookupSelBatch raises INVALID_ARGUMENT; the context stays usable
    if (c == 0) {
      std::vector<uint32_t> bad_sel(2048, 0);
      bad_sel[777] = 1u << 30;
      std::vector<int64_t> dict(16, 5);
      rpt::DataChunk broken;
      broken.count = 2048;
      broken.data.resize(1);
      broken.data[0].type = rpt::VectorType::DICTIONARY;
      broken.data[0].key_type = rpt::KeyType::I64;
      broken.data[0].data = dict.data();
      broken.data[0].sel = bad_sel.data();
      broken.data[0].dict_size = dict.size();
      std::vector<const rpt::DataChunk*> with_bad = pptrs;
      with_bad[with_bad.size() / 2 + 10] = &broken;
      bool threw = false;
      try {
        f->LookupSelBatch(ctx, with_bad, sels, {0});
      } catch (const rpt::GpuError& e) {
        threw = e.status() == RPT_ERR_INVALID_ARGUMENT;
      }
      EXPECT(threw, "an out-of-range dictionary index inside a worker's flatten raises INVALID_ARGUMENT");
      f->LookupSelBatch(ctx, pptrs, sels, {0});
      size_t bad2 = 0;
      for (size_t k = 0; k < pptrs.size(); k++) bad2 += sels[k] != want[k];
      EXPECT(bad2 == 0, "the context after a failed pipelined batch: %zu chunks differ", bad2);
    }
  }
}

// UseBF::ExecuteBatch with 2..5 applicable filters over a pipelined batch (ExecuteChainPipelined): per stage the
// first filter probes every row, each further one the previous one's survivors, their keys gathered on the host
// from FLAT / DICTIONARY / CONSTANT chunks with NULLs; BIGINT and INTEGER columns mixed, a non-finalized filter
// skipped, a stage whose column-1 keys all miss f1 (its chain stops there); every chunk against the oracle's
// intersection of per-row hits, pipelined and filter by filter (pipeline_rows beyond the batch).
static void pipelined_chain(int dev) {
  const size_t nb = 96 * 2048, np = (3u << 20) + 1234;
  Table bt = make_table(nb, 21, 53, 0), pt = make_table(np, 22, 41, 2048);  // chunk 3's column 0: CONSTANT
  ChunkStore bst, pst;
  make_chunks(bt, nb, bst, false);
  std::vector<const rpt::DataChunk*> pptrs;
  rpt::DeviceContext ctx(dev);
  ctx.pipeline_rows = 1u << 20;
  ctx.flatten_threads = 4;
  // f0: column 0 of build chunks [0, 48); f1: column 1 of [0, 80); f2: column 0 of [48, 96)
  struct Spec { int col; size_t c_lo, c_hi; };
  const Spec specs[3] = {{0, 0, 48}, {1, 0, 80}, {0, 48, 96}};
  std::vector<std::shared_ptr<rpt::PTBloomFilter>> fs;
  std::vector<std::vector<uint64_t>> words;
  for (const Spec& sp : specs) {
    std::vector<const rpt::DataChunk*> part;
    for (size_t k = sp.c_lo; k < sp.c_hi; k++) part.push_back(&bst.chunks[k]);
    const size_t lo = sp.c_lo * 2048, n = (sp.c_hi - sp.c_lo) * 2048;
    auto f = std::make_shared<rpt::PTBloomFilter>();
    f->Initialize(dev, static_cast<uint32_t>(n));
    f->InsertBatch(ctx, part, {static_cast<uint64_t>(sp.col)});
    f->finalized_ = true;
    const int lnb = f->LogNumBlocks();
    std::vector<uint64_t> w(1ULL << lnb, 0);
    const std::vector<uint64_t> vb = pack(sp.col == 0 ? bt.v0 : bt.v1, lo, n);
    if (sp.col == 0) rpt_oracle_insert_i64(w.data(), lnb, bt.c0.data() + lo, nullptr, vb.data(), n);
    else rpt_oracle_insert_i32(w.data(), lnb, bt.c1.data() + lo, nullptr, vb.data(), n);
    EXPECT(f->ExportWords() == w, "chain filter on column %d differs from the oracle", sp.col);
    words.push_back(std::move(w));
    fs.push_back(f);
  }
  // stage 1 (rows [1 Mi, 2 Mi)): every column-1 key one value f1 rejects (NULLs would not do: their hash is a
  // value like any other, and the build's NULLs put it in f1)
  int32_t miss = -1000000;
  for (;; miss--) {
    uint64_t one = 1;
    uint32_t sel1;
    if (rpt_oracle_probe_i32(words[1].data(), fs[1]->LogNumBlocks(), &miss, nullptr, &one, 1, &sel1) == 0) break;
  }
  for (size_t i = 1u << 20; i < (2u << 20); i++) {
    pt.c1[i] = miss;
    pt.v1[i] = true;
  }
  make_chunks(pt, np, pst, true);
  for (const auto& ch : pst.chunks) pptrs.push_back(&ch);
  EXPECT(pptrs[3]->data[0].type == rpt::VectorType::CONSTANT, "chunk 3 column 0 CONSTANT");
  std::vector<std::vector<uint8_t>> hit;  // per filter: does probe row i pass it
  for (size_t i = 0; i < 3; i++) {
    const Spec& sp = specs[i];
    const std::vector<uint64_t> vp = pack(sp.col == 0 ? pt.v0 : pt.v1, 0, np);
    std::vector<uint32_t> sel(np);
    const int lnb = fs[i]->LogNumBlocks();
    const uint64_t ne = sp.col == 0 ? rpt_oracle_probe_i64(words[i].data(), lnb, pt.c0.data(), nullptr, vp.data(), np, sel.data())
                                    : rpt_oracle_probe_i32(words[i].data(), lnb, pt.c1.data(), nullptr, vp.data(), np, sel.data());
    std::vector<uint8_t> h(np, 0);
    for (uint64_t j = 0; j < ne; j++) h[sel[j]] = 1;
    hit.push_back(std::move(h));
  }
  auto unfinished = std::make_shared<rpt::PTBloomFilter>();  // never finalized: UseBF skips it (cpp:139-142)
  unfinished->Initialize(dev, 1000);
  struct Case { std::vector<int> order; };
  const Case cases[] = {{{0, 1}}, {{0, 1, 2}}, {{1, 0, 2, 1}}, {{2, -1, 0}}, {{0, 1, 2, 0, 1}}};
  for (const Case& cs : cases) {
    std::vector<std::shared_ptr<rpt::PTBloomFilter>> use;
    std::vector<uint64_t> cols;
    for (int i : cs.order) {
      use.push_back(i < 0 ? unfinished : fs[i]);
      cols.push_back(i < 0 ? 0 : static_cast<uint64_t>(specs[i].col));
    }
    std::vector<rpt::SelectionVector> want(pptrs.size());
    size_t total = 0, stage1 = 0;
    for (size_t k = 0; k < pptrs.size(); k++) {
      for (size_t r = 0; r < pptrs[k]->count; r++) {
        bool pass = true;
        for (int i : cs.order) pass = pass && (i < 0 || hit[i][2048 * k + r]);
        if (pass) want[k].push_back(static_cast<uint32_t>(r));
      }
      total += want[k].size();
      if (2048 * k >= (1u << 20) && 2048 * k < (2u << 20)) stage1 += want[k].size();
    }
    const bool with_f1 = std::find(cs.order.begin(), cs.order.end(), 1) != cs.order.end();
    EXPECT(total > 10000 && (stage1 == 0) == with_f1, "chain of %zu: %zu survivors, %zu in stage 1", cs.order.size(), total, stage1);
    rpt::UseBF ub(use, cols);
    std::vector<rpt::SelectionVector> outs(3, rpt::SelectionVector(5, 1));  // stale contents must not leak
    for (int rep = 0; rep < 3; rep++) {  // pipelined twice (outs reused), then filter by filter
      ctx.stats = {};
      ctx.pipeline_rows = rep < 2 ? (1u << 20) : ~0ULL / 4;
      const uint64_t got = ub.ExecuteBatch(ctx, pptrs, outs);
      size_t bad = 0;
      for (size_t k = 0; k < pptrs.size(); k++) bad += outs[k] != want[k];
      EXPECT(got == total && outs.size() == pptrs.size() && bad == 0, "chain of %zu filters (call %d): %zu chunks differ, %llu vs %zu rows",
             cs.order.size(), rep, bad, (unsigned long long)got, total);
      if (rep < 2)
        EXPECT(ctx.stats.stages >= 3 && ctx.stats.rows == np, "chain of %zu: %llu pipeline stages", cs.order.size(),
               (unsigned long long)ctx.stats.stages);
    }
  }
  ctx.pipeline_rows = 1u << 20;
  // a chunk whose column-1 dictionary indices are out of range: the gather for f1 (on a worker thread, mid
  // chain) throws, the pipeline drains its streams and ExecuteBatch raises INVALID_ARGUMENT; the context stays
  // usable
  // (with every stage stream synchronized before the error leaves, including the third stage's) at
  // several positions, with stages of 256 Ki rows so all three stage streams are busy when the gather throws
  ctx.pipeline_rows = 1u << 18;
  for (const size_t victim : {pptrs.size() / 2 + 7, size_t(300), pptrs.size() - 2, size_t(1400)}) {
    rpt::DataChunk broken = *pptrs[victim];
    std::vector<uint32_t> bad_sel(broken.count, 1u << 30);
    std::vector<int32_t> dict(4, 1);
    broken.data[1].type = rpt::VectorType::DICTIONARY;
    broken.data[1].data = dict.data();
    broken.data[1].sel = bad_sel.data();
    broken.data[1].dict_size = dict.size();
    broken.data[1].validity = nullptr;
    std::vector<const rpt::DataChunk*> with_bad = pptrs;
    with_bad[victim] = &broken;
    rpt::UseBF ub({fs[0], fs[1]}, {0, 1});
    std::vector<rpt::SelectionVector> outs;
    bool threw = false;
    try {
      ub.ExecuteBatch(ctx, with_bad, outs);
    } catch (const rpt::GpuError& e) {
      threw = e.status() == RPT_ERR_INVALID_ARGUMENT;
    }
    EXPECT(threw, "an out-of-range dictionary index in a gathered column raises INVALID_ARGUMENT");
    const uint64_t got = ub.ExecuteBatch(ctx, pptrs, outs);
    size_t bad = 0, total = 0;
    for (size_t k = 0; k < pptrs.size(); k++) {
      rpt::SelectionVector w;
      for (size_t r = 0; r < pptrs[k]->count; r++)
        if (hit[0][2048 * k + r] && hit[1][2048 * k + r]) w.push_back(static_cast<uint32_t>(r));
      total += w.size();
      bad += outs[k] != w;
    }
    EXPECT(bad == 0 && got == total, "the context after a failed chain (bad chunk %zu): %zu chunks differ", victim, bad);
  }
  ctx.pipeline_rows = 1u << 20;
}

// The process-wide pinned staging cache: a destroyed context's buffers are cached and handed to the next
// context of that size class (the same address), the limit bounds what is kept, ReleasePinnedCache empties it.
static void pinned_cache(int dev) {
  rpt::ReleasePinnedCache();
  EXPECT(rpt::PinnedCacheBytes() == 0, "cache empty after release");
  void* first = nullptr;
  {
    rpt::DeviceContext a(dev);
    first = a.host(3, 3u << 20);  // a 4 MiB class
  }
  EXPECT(rpt::PinnedCacheBytes() == (4u << 20), "destroyed context's buffer cached: %zu", rpt::PinnedCacheBytes());
  {
    rpt::DeviceContext b(dev);
    void* again = b.host(7, 4u << 20);
    EXPECT(again == first && rpt::PinnedCacheBytes() == 0, "the cached buffer is reused");
    void* bigger = b.host(7, 5u << 20);  // grows: the 4 MiB buffer goes back, an 8 MiB one is pinned
    EXPECT(bigger != nullptr && rpt::PinnedCacheBytes() == (4u << 20), "growth returns the old buffer");
    std::memset(bigger, 1, 5u << 20);
  }
  rpt::SetPinnedCacheLimit(6u << 20);  // keeps 4 MiB, not 4 + 8
  EXPECT(rpt::PinnedCacheBytes() <= (6u << 20), "limit applied: %zu", rpt::PinnedCacheBytes());
  rpt::SetPinnedCacheLimit(size_t(4) << 30);
  rpt::ReleasePinnedCache();
  EXPECT(rpt::PinnedCacheBytes() == 0, "released");
  // streams and events of an ended context serve the next one (drained, not capturing)
  // (every later test's contexts run on pooled streams)
  void *s0 = nullptr, *e0 = nullptr;
  {
    rpt::DeviceContext a(dev);
    s0 = a.stream();
    e0 = a.event(0);
  }
  {
    rpt::DeviceContext b(dev);
    EXPECT(b.stream() == s0 && b.event(0) == e0, "pooled stream / event reused");
  }
}

// Narrow BIGINT keys (DeviceContext::narrow_keys): chunks whose keys share their high 32 bits (0, 5 and 0xFFFFFFFF,
// i.e. negative keys, by chunk) cross PCIe as 4-B low words and are widened on the device; FLAT / DICTIONARY /
// CONSTANT chunks with NULLs, pipelined insert and lookup against the oracle, the same with narrow_keys off, and
// a batch whose chunks mix high words (stays plain after its first stage's attempt).
static void narrow_keys(int dev) {
  const size_t nb = (2u << 20) + 333, np = (3u << 20) + 555;
  Table bt = make_table(nb, 31, 47, 0), pt = make_table(np, 32, 43, 2048);
  const uint32_t his[3] = {0u, 5u, 0xFFFFFFFFu};
  auto narrowed = [&](Table& t, size_t n) {
    for (size_t i = 0; i < n; i++)
      t.c0[i] = static_cast<int64_t>((static_cast<uint64_t>(his[(i / 2048) % 3]) << 32) |
                                     static_cast<uint32_t>(t.c0[i] & 0x3FFFF));
  };
  narrowed(bt, nb);
  narrowed(pt, np);
  ChunkStore bst, pst;
  make_chunks(bt, nb, bst, false);
  make_chunks(pt, np, pst, true);
  std::vector<const rpt::DataChunk*> bptrs, pptrs;
  for (const auto& ch : bst.chunks) bptrs.push_back(&ch);
  for (const auto& ch : pst.chunks) pptrs.push_back(&ch);
  EXPECT(pptrs[3]->data[0].type == rpt::VectorType::CONSTANT, "chunk 3 column 0 CONSTANT");
  const int lnb = rpt_oracle_log_num_blocks(nb);
  std::vector<uint64_t> w(1ULL << lnb, 0);
  {
    const std::vector<uint64_t> vb = pack(bt.v0, 0, nb);
    rpt_oracle_insert_i64(w.data(), lnb, bt.c0.data(), nullptr, vb.data(), nb);
  }
  std::vector<rpt::SelectionVector> want(pptrs.size());
  for (size_t k = 0; k < pptrs.size(); k++) {
    const size_t lo = 2048 * k, cnt = pptrs[k]->count;
    const std::vector<uint64_t> vp = pack(pt.v0, lo, cnt);
    want[k].resize(cnt);
    want[k].resize(rpt_oracle_probe_i64(w.data(), lnb, pt.c0.data() + lo, nullptr, vp.data(), cnt, want[k].data()));
  }
  for (int on = 1; on >= 0; on--) {
    rpt::DeviceContext ctx(dev);
    ctx.pipeline_rows = 1u << 20;
    ctx.flatten_threads = 4;
    ctx.narrow_keys = on != 0;
    auto f = std::make_shared<rpt::PTBloomFilter>();
    f->Initialize(dev, static_cast<uint32_t>(nb));
    f->InsertBatch(ctx, bptrs, {0});
    EXPECT(f->ExportWords() == w, "pipelined insert of narrow keys (narrow_keys %d) differs from the oracle", on);
    EXPECT(on ? ctx.stats.narrow_stages >= 2 : ctx.stats.narrow_stages == 0, "insert: %llu narrow stages (narrow_keys %d)",
           (unsigned long long)ctx.stats.narrow_stages, on);
    f->finalized_ = true;
    ctx.stats = {};
    std::vector<rpt::SelectionVector> sels;
    f->LookupSelBatch(ctx, pptrs, sels, {0});
    size_t bad = 0;
    for (size_t k = 0; k < pptrs.size(); k++) bad += sels[k] != want[k];
    EXPECT(bad == 0, "pipelined lookup of narrow keys (narrow_keys %d): %zu chunks differ", on, bad);
    EXPECT(on ? ctx.stats.narrow_stages == ctx.stats.stages : ctx.stats.narrow_stages == 0,
           "lookup: %llu of %llu stages narrow (narrow_keys %d)", (unsigned long long)ctx.stats.narrow_stages,
           (unsigned long long)ctx.stats.stages, on);
  }
  // the pipelined chain's first column narrow too: f (column 0) then an INTEGER filter on column 1
  {
    rpt::DeviceContext ctx(dev);
    ctx.pipeline_rows = 1u << 20;
    ctx.flatten_threads = 4;
    auto f0 = std::make_shared<rpt::PTBloomFilter>(), f1 = std::make_shared<rpt::PTBloomFilter>();
    f0->Initialize(dev, static_cast<uint32_t>(nb));
    f1->Initialize(dev, static_cast<uint32_t>(nb));
    f0->InsertBatch(ctx, bptrs, {0});
    f1->InsertBatch(ctx, bptrs, {1});
    f0->finalized_ = f1->finalized_ = true;
    const int lnb1 = f1->LogNumBlocks();
    const std::vector<uint64_t> w1 = f1->ExportWords();
    rpt::UseBF ub({f0, f1}, {0, 1});
    std::vector<rpt::SelectionVector> outs;
    ctx.stats = {};
    const uint64_t got = ub.ExecuteBatch(ctx, pptrs, outs);
    size_t bad = 0, total = 0;
    for (size_t k = 0; k < pptrs.size(); k++) {
      const size_t lo = 2048 * k, cnt = pptrs[k]->count;
      const std::vector<uint64_t> vp = pack(pt.v1, lo, cnt);
      rpt::SelectionVector s1(cnt), both;
      s1.resize(rpt_oracle_probe_i32(w1.data(), lnb1, pt.c1.data() + lo, nullptr, vp.data(), cnt, s1.data()));
      std::set_intersection(want[k].begin(), want[k].end(), s1.begin(), s1.end(), std::back_inserter(both));
      total += both.size();
      bad += outs[k] != both;
    }
    EXPECT(bad == 0 && got == total && ctx.stats.narrow_stages == ctx.stats.stages && ctx.stats.stages >= 3,
           "narrow first column in the chain: %zu chunks differ, %llu of %llu stages narrow", bad,
           (unsigned long long)ctx.stats.narrow_stages, (unsigned long long)ctx.stats.stages);
  }
  // a batch whose chunks' keys straddle high words (BIGINT keys around 0: both signs in one chunk)
  {
    Table mt = make_table(np, 33, 0, 0);
    ChunkStore mst;
    make_chunks(mt, np, mst, false);
    std::vector<const rpt::DataChunk*> mptrs;
    for (const auto& ch : mst.chunks) mptrs.push_back(&ch);
    rpt::DeviceContext ctx(dev);
    ctx.pipeline_rows = 1u << 20;
    auto f = std::make_shared<rpt::PTBloomFilter>();
    f->Initialize(dev, static_cast<uint32_t>(nb));
    f->InsertBatch(ctx, bptrs, {0});
    f->finalized_ = true;
    ctx.stats = {};
    std::vector<rpt::SelectionVector> sels;
    f->LookupSelBatch(ctx, mptrs, sels, {0});
    size_t bad = 0;
    for (size_t k = 0; k < mptrs.size(); k++) {
      const size_t lo = 2048 * k, cnt = mptrs[k]->count;
      const std::vector<uint64_t> vp = pack(mt.v0, lo, cnt);
      rpt::SelectionVector e(cnt);
      e.resize(rpt_oracle_probe_i64(w.data(), lnb, mt.c0.data() + lo, nullptr, vp.data(), cnt, e.data()));
      bad += sels[k] != e;
    }
    EXPECT(bad == 0 && ctx.stats.narrow_stages == 0 && ctx.stats.stages >= 3, "mixed high words: %zu chunks differ, %llu narrow stages",
           bad, (unsigned long long)ctx.stats.narrow_stages);
  }
}

// Randomized batches through every pipelined path: ragged chunks (0..2048 rows), FLAT / DICTIONARY / CONSTANT /
// SEQUENCE vectors, NULLs at random rates, BIGINT keys in narrow and wide ranges, small stages (many per batch),
// 1..8 workers, narrow_keys and bits_back on / off; InsertBatch against the oracle's words, LookupSelBatch and UseBF::ExecuteBatch
// chains of 1..3 filters against the oracle's per-row hits.
struct FuzzCol {
  std::vector<int64_t> v64;  // logical value per row (column 0)
  std::vector<int32_t> v32;  // (column 1)
  std::vector<bool> ok0, ok1;
};
static void fuzz_chunks(std::mt19937_64& rng, size_t n_chunks, bool narrow64, FuzzCol& fc, ChunkStore& st) {
  for (size_t k = 0; k < n_chunks; k++) {
    const size_t cnt = (rng() % 7 == 0) ? rng() % 3 : (rng() % 2 ? 2048 : 1 + rng() % 2048);
    const size_t lo = fc.v64.size();
    const uint64_t hi = narrow64 ? (rng() % 3 == 0 ? 0xFFFFFFFFULL : rng() % 4) : 0;
    const int null_rate = static_cast<int>(rng() % 4);  // 0: none, else 1 in (8 << rate)
    rpt::DataChunk ch;
    ch.count = cnt;
    ch.data.resize(2);
    for (int c = 0; c < 2; c++) {
      const int shape = static_cast<int>(rng() % 6);  // 0-2 FLAT, 3 DICTIONARY, 4 CONSTANT, 5 SEQUENCE
      rpt::Vector x;
      x.key_type = c == 0 ? rpt::KeyType::I64 : rpt::KeyType::I32;
      std::vector<int64_t> vals(cnt);
      std::vector<bool> valid(cnt, true);
      auto draw = [&]() -> int64_t {
        const uint64_t r = rng() % 60000;
        if (c == 1) return static_cast<int64_t>(static_cast<int32_t>(r) - 30000);
        return narrow64 ? static_cast<int64_t>((hi << 32) | r) : static_cast<int64_t>(r * 0x9E3779B97F4A7C15ULL);
      };
      if (shape == 5 && cnt) {  // SEQUENCE: never NULL
        x.type = rpt::VectorType::SEQUENCE;
        x.seq_start = c == 0 ? static_cast<int64_t>((hi << 32) | (rng() % 50000)) : static_cast<int64_t>(rng() % 50000) - 25000;
        x.seq_increment = static_cast<int64_t>(rng() % 5);
        for (size_t i = 0; i < cnt; i++) {
          const uint64_t v = static_cast<uint64_t>(x.seq_start) + static_cast<uint64_t>(x.seq_increment) * i;
          vals[i] = c == 0 ? static_cast<int64_t>(v) : static_cast<int64_t>(static_cast<int32_t>(v));
        }
      } else if (shape == 4 && cnt) {  // CONSTANT
        x.type = rpt::VectorType::CONSTANT;
        const int64_t v = draw();
        const bool ok = null_rate == 0 || rng() % 4 != 0;
        for (size_t i = 0; i < cnt; i++) {
          vals[i] = v;
          valid[i] = ok;
        }
        if (c == 0) st.i64.push_back({v});
        else st.i32.push_back({static_cast<int32_t>(v)});
        st.valid.push_back({ok ? 1ULL : 0ULL});
        x.data = c == 0 ? static_cast<const void*>(st.i64.back().data()) : static_cast<const void*>(st.i32.back().data());
        x.validity = st.valid.back().data();
      } else if (shape == 3 && cnt) {  // DICTIONARY over a small dictionary with NULL entries
        x.type = rpt::VectorType::DICTIONARY;
        const size_t nd = 1 + rng() % 300;
        std::vector<int64_t> dict(nd);
        std::vector<uint64_t> dv((nd + 63) / 64 + 1, ~0ULL);
        for (size_t d = 0; d < nd; d++) {
          dict[d] = draw();
          if (null_rate && rng() % (8u << null_rate) == 0) dv[d / 64] &= ~(1ULL << (d % 64));
        }
        std::vector<uint32_t> sel(cnt);
        for (size_t i = 0; i < cnt; i++) {
          sel[i] = static_cast<uint32_t>(rng() % nd);
          vals[i] = dict[sel[i]];
          valid[i] = (dv[sel[i] / 64] >> (sel[i] % 64)) & 1;
        }
        if (c == 0) st.i64.push_back(dict);
        else st.i32.push_back(std::vector<int32_t>(dict.begin(), dict.end()));
        st.sel.push_back(std::move(sel));
        st.valid.push_back(std::move(dv));
        x.data = c == 0 ? static_cast<const void*>(st.i64.back().data()) : static_cast<const void*>(st.i32.back().data());
        x.sel = st.sel.back().data();
        x.dict_size = nd;
        x.validity = st.valid.back().data();
      } else {  // FLAT (also every empty chunk)
        x.type = rpt::VectorType::FLAT;
        std::vector<uint64_t> vw((cnt + 63) / 64 + 1, ~0ULL);
        for (size_t i = 0; i < cnt; i++) {
          vals[i] = draw();
          if (null_rate && rng() % (8u << null_rate) == 0) {
            valid[i] = false;
            vw[i / 64] &= ~(1ULL << (i % 64));
          }
        }
        if (c == 0) st.i64.push_back(vals);
        else st.i32.push_back(std::vector<int32_t>(vals.begin(), vals.end()));
        st.valid.push_back(std::move(vw));
        x.data = c == 0 ? static_cast<const void*>(st.i64.back().data()) : static_cast<const void*>(st.i32.back().data());
        x.validity = null_rate ? st.valid.back().data() : nullptr;
      }
      ch.data[c] = x;
      for (size_t i = 0; i < cnt; i++) {
        if (c == 0) {
          fc.v64.push_back(vals[i]);
          fc.ok0.push_back(valid[i]);
        } else {
          fc.v32.push_back(static_cast<int32_t>(vals[i]));
          fc.ok1.push_back(valid[i]);
        }
      }
    }
    (void)lo;
    st.chunks.push_back(std::move(ch));
  }
}

static std::vector<uint64_t> pack_all(const std::vector<bool>& v) { return pack(v, 0, v.size()); }

static void fuzz_pipelines(int dev) {
  std::mt19937_64 rng(2026);
  uint64_t stages = 0, narrow = 0;
  int create_skipped = 0;
  const int iters = 30;
  for (int it = 0; it < iters; it++) {
    const bool narrow64 = rng() % 2;
    FuzzCol bc, pc;
    ChunkStore bst, pst;
    fuzz_chunks(rng, 150 + rng() % 100, narrow64, bc, bst);
    fuzz_chunks(rng, 200 + rng() % 150, narrow64, pc, pst);
    std::vector<const rpt::DataChunk*> bptrs, pptrs;
    for (const auto& ch : bst.chunks) bptrs.push_back(&ch);
    for (const auto& ch : pst.chunks) pptrs.push_back(&ch);
    const size_t nb = bc.v64.size(), np = pc.v64.size();
    rpt::DeviceContext ctx(dev);
    ctx.pipeline_rows = 1ULL << (15 + rng() % 3);
    ctx.flatten_threads = 1 + static_cast<unsigned>(rng() % 8);
    ctx.narrow_keys = rng() % 4 != 0;
    ctx.bits_back = rng() % 3 != 0;
    const int lnb = rpt_oracle_log_num_blocks(nb);
    std::vector<uint64_t> w0(1ULL << lnb, 0), w1(1ULL << lnb, 0);
    const std::vector<uint64_t> vb0 = pack_all(bc.ok0), vb1 = pack_all(bc.ok1);
    rpt_oracle_insert_i64(w0.data(), lnb, bc.v64.data(), nullptr, vb0.data(), nb);
    rpt_oracle_insert_i32(w1.data(), lnb, bc.v32.data(), nullptr, vb1.data(), nb);
    auto f0 = std::make_shared<rpt::PTBloomFilter>(), f1 = std::make_shared<rpt::PTBloomFilter>();
    f0->Initialize(dev, static_cast<uint32_t>(nb));
    f1->Initialize(dev, static_cast<uint32_t>(nb));
    f0->InsertBatch(ctx, bptrs, {0});
    f1->InsertBatch(ctx, bptrs, {1});
    EXPECT(f0->ExportWords() == w0 && f1->ExportWords() == w1, "fuzz %d: pipelined insert words differ", it);
    f0->finalized_ = f1->finalized_ = true;
    // per-row hits of each filter
    std::vector<uint32_t> s0(np), s1(np);
    const std::vector<uint64_t> vp0 = pack_all(pc.ok0), vp1 = pack_all(pc.ok1);
    s0.resize(rpt_oracle_probe_i64(w0.data(), lnb, pc.v64.data(), nullptr, vp0.data(), np, s0.data()));
    s1.resize(rpt_oracle_probe_i32(w1.data(), lnb, pc.v32.data(), nullptr, vp1.data(), np, s1.data()));
    std::vector<uint8_t> h0(np, 0), h1(np, 0);
    for (uint32_t r : s0) h0[r] = 1;
    for (uint32_t r : s1) h1[r] = 1;
    struct Case { std::vector<int> order; };
    const Case cases[] = {{{0}}, {{1}}, {{0, 1}}, {{1, 0}}, {{0, 1, 0}}};
    ctx.stats = {};
    for (const Case& cs : cases) {
      std::vector<rpt::SelectionVector> want(pptrs.size());
      size_t row = 0, total = 0;
      for (size_t k = 0; k < pptrs.size(); k++) {
        for (size_t r = 0; r < pptrs[k]->count; r++, row++) {
          bool pass = true;
          for (int f : cs.order) pass = pass && (f == 0 ? h0[row] : h1[row]);
          if (pass) want[k].push_back(static_cast<uint32_t>(r));
        }
        total += want[k].size();
      }
      std::vector<std::shared_ptr<rpt::PTBloomFilter>> fs;
      std::vector<uint64_t> cols;
      for (int f : cs.order) {
        fs.push_back(f == 0 ? f0 : f1);
        cols.push_back(static_cast<uint64_t>(f));
      }
      rpt::UseBF ub(fs, cols);
      std::vector<rpt::SelectionVector> outs;
      const uint64_t got = ub.ExecuteBatch(ctx, pptrs, outs);
      size_t bad = 0;
      for (size_t k = 0; k < pptrs.size(); k++) bad += outs[k] != want[k];
      EXPECT(bad == 0 && got == total, "fuzz %d (narrow64 %d, stage %llu, workers %u, narrow_keys %d), chain of %zu: %zu chunks differ",
             it, narrow64 ? 1 : 0, (unsigned long long)ctx.pipeline_rows, ctx.flatten_threads, ctx.narrow_keys ? 1 : 0,
             cs.order.size(), bad);
      if (cs.order.size() == 1) {
        std::vector<rpt::SelectionVector> sels;
        fs[0]->LookupSelBatch(ctx, pptrs, sels, {cols[0]});
        size_t bad2 = 0;
        for (size_t k = 0; k < pptrs.size(); k++) bad2 += sels[k] != want[k];
        EXPECT(bad2 == 0, "fuzz %d: LookupSelBatch on column %llu: %zu chunks differ", it, (unsigned long long)cols[0], bad2);
      }
    }
    stages += ctx.stats.stages;
    narrow += ctx.stats.narrow_stages;
    {  // CREATE_BF over the same build chunks: random estimate, flush size, sink threads, flush mode and resize rule
      const uint64_t ests[] = {1000, nb / 8 + 1, nb / 2 + 1, nb, 2 * nb};
      const uint64_t est = ests[rng() % 5];
      const uint64_t flush = 2048 + rng() % 60000;
      const int T = 1 + static_cast<int>(rng() % 4);
      const bool async = rng() % 2;
      const auto rule = rng() % 2 ? rpt::CreateBF::ResizeRule::kReferenceFormula : rpt::CreateBF::ResizeRule::kOnAllocation;
      rpt::CreateBF cb(dev, est, {0, 1}, flush, rule);
      std::vector<std::unique_ptr<rpt::CreateBF::LocalState>> ls;
      for (int t = 0; t < T; t++) {
        ls.push_back(cb.MakeLocalState());
        ls.back()->async_flush = async;
      }
      std::vector<std::thread> th;
      for (int t = 0; t < T; t++)
        th.emplace_back([&, t] {
          for (size_t k = t; k < bst.chunks.size(); k += T) cb.Sink(*ls[t], bst.chunks[k]);
          cb.Combine(*ls[t]);
        });
      for (auto& x : th) x.join();
      cb.Finalize();
      const int lest = rpt_oracle_log_num_blocks(static_cast<uint32_t>(est));
      const bool want_resize = rule == rpt::CreateBF::ResizeRule::kReferenceFormula
                                   ? rpt_oracle_needs_resize(static_cast<uint32_t>(est), nb) > 0
                                   : rpt_oracle_needs_resize_alloc(lest, nb) > 0;
      const int l = want_resize ? lnb : lest;
      std::vector<uint64_t> c0(1ULL << l, 0), c1(1ULL << l, 0);
      rpt_oracle_insert_i64(c0.data(), l, bc.v64.data(), nullptr, vb0.data(), nb);
      rpt_oracle_insert_i32(c1.data(), l, bc.v32.data(), nullptr, vb1.data(), nb);
      EXPECT(cb.Resized(0) == want_resize && cb.Resized(1) == want_resize &&
                 cb.GetBloomFilter(0)->ExportWords() == c0 && cb.GetBloomFilter(1)->ExportWords() == c1,
             "fuzz %d: CREATE_BF (estimate %llu, flush %llu, %d threads, async %d, rule %d): resized %d, words differ",
             it, (unsigned long long)est, (unsigned long long)flush, T, async ? 1 : 0,
             rule == rpt::CreateBF::ResizeRule::kReferenceFormula ? 1 : 0, cb.Resized(0) ? 1 : 0);
      EXPECT(want_resize || cb.SkippedInsertRows() == 0, "fuzz %d: inserts skipped without a resize", it);
      int64_t e[2], mn = 0, mx = 0;
      if (rpt_oracle_minmax_i64(bc.v64.data(), nullptr, vb0.data(), nb, e))
        EXPECT(cb.MinMax(0, mn, mx) && mn == e[0] && mx == e[1], "fuzz %d: CREATE_BF min/max", it);
      create_skipped += cb.SkippedInsertRows() > 0 && cb.SkippedInsertRows() < 2 * nb;
    }
  }
  printf("fuzz: %d batches, %llu pipelined stages, %llu of them narrow, %d builds with skipped inserts after inserted ones\n",
         iters, (unsigned long long)stages, (unsigned long long)narrow, create_skipped);
  EXPECT(stages > 100 && narrow > 10, "the fuzz reached the pipelines (%llu stages, %llu narrow)", (unsigned long long)stages,
         (unsigned long long)narrow);
}

int main() {
  try {
    const int dev = 0;
    fuzz_pipelines(dev);
    narrow_keys(dev);
    pinned_cache(dev);
    pipelined_workers(dev);
    pipelined_chain(dev);
    // ---------------- build -------------------------------------------------------------------
    const size_t nb = 50001;
    Table bt = make_table(nb, 1, 97, 2048);
    ChunkStore bst;
    make_chunks(bt, nb, bst, true);
    // sink batches of >= 5000 rows: several device key segments per sink thread
    rpt::CreateBF create(dev, /*estimated_cardinality=*/1000, {0, 1}, /*sink_flush_rows=*/5000);
    std::vector<std::unique_ptr<rpt::CreateBF::LocalState>> locals;
    for (int t = 0; t < 4; t++) locals.push_back(create.MakeLocalState());
    std::vector<std::thread> ths;
    for (int t = 0; t < 4; t++) {
      ths.emplace_back([&, t] {
        for (size_t k = t; k < bst.chunks.size(); k += 4) create.Sink(*locals[t], bst.chunks[k]);
      });
    }
    for (auto& th : ths) th.join();
    for (auto& l : locals) create.Combine(*l);
    create.Finalize();
    EXPECT(create.MaterializedRows() == nb, "materialized %llu", (unsigned long long)create.MaterializedRows());
    EXPECT(create.Resized(0) && create.Resized(1), "under-estimated filters must be resized");
    // the first flush (>= 5000 rows) already makes the resize certain: no sink-time insert, Finalize rehashes all
    EXPECT(create.SkippedInsertRows() == 2 * nb, "skipped sink inserts %llu", (unsigned long long)create.SkippedInsertRows());
    const int lnb = rpt_oracle_log_num_blocks(nb);
    std::vector<uint64_t> w0(1ULL << lnb, 0), w1(1ULL << lnb, 0);
    {
      std::vector<uint64_t> va = pack(bt.v0, 0, nb), vb = pack(bt.v1, 0, nb);
      rpt_oracle_insert_i64(w0.data(), lnb, bt.c0.data(), nullptr, va.data(), nb);
      rpt_oracle_insert_i32(w1.data(), lnb, bt.c1.data(), nullptr, vb.data(), nb);
    }
    auto f0 = create.GetBloomFilter(0), f1 = create.GetBloomFilter(1);
    EXPECT(f0->LogNumBlocks() == lnb && f0->SizedForRows() == nb, "resized filter sizing");
    EXPECT(f0->ExportWords() == w0, "filter 0 words differ from the oracle");
    EXPECT(f1->ExportWords() == w1, "filter 1 words differ from the oracle");
    EXPECT(f0->finalized_ && f1->finalized_ && !f0->IsEmpty(), "finalized / has data");
    {  // the same build with synchronous sink flushes (LocalState::async_flush = false): the same words
      rpt::CreateBF sync_create(dev, 1000, {0, 1}, 5000);
      std::vector<std::unique_ptr<rpt::CreateBF::LocalState>> ls;
      for (int t = 0; t < 3; t++) {
        ls.push_back(sync_create.MakeLocalState());
        ls.back()->async_flush = false;
      }
      std::vector<std::thread> st;
      for (int t = 0; t < 3; t++)
        st.emplace_back([&, t] {
          for (size_t k = t; k < bst.chunks.size(); k += 3) sync_create.Sink(*ls[t], bst.chunks[k]);
          sync_create.Combine(*ls[t]);
        });
      for (auto& th : st) th.join();
      sync_create.Finalize();
      EXPECT(sync_create.GetBloomFilter(0)->ExportWords() == w0 && sync_create.GetBloomFilter(1)->ExportWords() == w1,
             "synchronous sink flushes: words differ from the oracle");
      EXPECT(ls[0]->flushes >= 3 && ls[0]->materialize_s > 0 && ls[0]->flush_s > 0, "sink stats");
    }
    {  // estimate 20000 (2^12 blocks: resize above 32768 rows): the first flushes insert, the later ones are skipped
      rpt::CreateBF part(dev, 20000, {0, 1}, 5000);
      std::vector<std::unique_ptr<rpt::CreateBF::LocalState>> ls;
      for (int t = 0; t < 4; t++) ls.push_back(part.MakeLocalState());
      std::vector<std::thread> st;
      for (int t = 0; t < 4; t++)
        st.emplace_back([&, t] {
          for (size_t k = t; k < bst.chunks.size(); k += 4) part.Sink(*ls[t], bst.chunks[k]);
          part.Combine(*ls[t]);
        });
      for (auto& th : st) th.join();
      EXPECT(part.GetBloomFilter(0)->LogNumBlocks() == 12, "estimate 20000: 2^%d blocks", part.GetBloomFilter(0)->LogNumBlocks());
      const uint64_t skipped = part.SkippedInsertRows();
      part.Finalize();
      EXPECT(part.Resized(0) && part.Resized(1), "estimate 20000: resized");
      EXPECT(skipped > 0 && skipped < 2 * nb, "estimate 20000: skipped %llu of %llu", (unsigned long long)skipped,
             (unsigned long long)(2 * nb));
      EXPECT(part.GetBloomFilter(0)->ExportWords() == w0 && part.GetBloomFilter(1)->ExportWords() == w1,
             "estimate 20000: words differ from the oracle");
      int64_t mn = 0, mx = 0, e0[2];
      std::vector<uint64_t> va = pack(bt.v0, 0, nb);
      rpt_oracle_minmax_i64(bt.c0.data(), nullptr, va.data(), nb, e0);
      EXPECT(part.MinMax(0, mn, mx) && mn == e0[0] && mx == e0[1], "estimate 20000: min/max");
    }
    {  // a sink state that flushed (making the resize look certain, so later flushes skip their inserts)
       // but is never combined; the combined rows alone do not call for the resize. Finalize must still rehash them.
      rpt::CreateBF lone(dev, 1000, {0}, 5000);
      auto a = lone.MakeLocalState(), b = lone.MakeLocalState();
      for (size_t k = 0; k < 4; k++) lone.Sink(*a, bst.chunks[k]);  // 8192 rows: flushed, resize "certain"
      rpt::DataChunk few = bst.chunks[5];
      few.count = 500;
      lone.Sink(*b, few);
      lone.Combine(*b);  // a is dropped without Combine (its rows never reach the operator's result)
      a.reset();
      EXPECT(lone.SkippedInsertRows() > 0, "the lone state's insert was skipped");
      lone.Finalize();
      const int ll = rpt_oracle_log_num_blocks(1000);
      std::vector<uint64_t> wl(1ULL << ll, 0);
      std::vector<uint64_t> vl = pack(bt.v0, 5 * 2048, 500);
      // chunk 5 is FLAT or DICTIONARY (k % 3 == 2: FLAT): its first 500 rows are rows 10240.. of the table
      rpt_oracle_insert_i64(wl.data(), ll, bt.c0.data() + 5 * 2048, nullptr, vl.data(), 500);
      EXPECT(!lone.Resized(0) && lone.GetBloomFilter(0)->LogNumBlocks() == ll &&
                 lone.GetBloomFilter(0)->ExportWords() == wl,
             "uncombined flushing state: the combined rows' filter differs from the oracle (false negatives)");
    }
    // the rehash from HBM groups NULL-free segments into one insert: a NULL-free build, and one with NULLs in a few
    // segments only (grouped and single segments interleaved)
    for (const int null_every : {0, 70000}) {
      const size_t ng = 150001;
      Table gt = make_table(ng, 5, null_every, 0);
      ChunkStore gst;
      make_chunks(gt, ng, gst, false);
      rpt::CreateBF g(dev, 1000, {0, 1}, 6000);
      std::vector<std::unique_ptr<rpt::CreateBF::LocalState>> ls;
      for (int t = 0; t < 3; t++) ls.push_back(g.MakeLocalState());
      std::vector<std::thread> st;
      for (int t = 0; t < 3; t++)
        st.emplace_back([&, t] {
          for (size_t k = t; k < gst.chunks.size(); k += 3) g.Sink(*ls[t], gst.chunks[k]);
          g.Combine(*ls[t]);
        });
      for (auto& th : st) th.join();
      g.Finalize();
      const int lg = rpt_oracle_log_num_blocks(ng);
      std::vector<uint64_t> g0(1ULL << lg, 0), g1(1ULL << lg, 0);
      std::vector<uint64_t> va = pack(gt.v0, 0, ng), vb = pack(gt.v1, 0, ng);
      rpt_oracle_insert_i64(g0.data(), lg, gt.c0.data(), nullptr, va.data(), ng);
      rpt_oracle_insert_i32(g1.data(), lg, gt.c1.data(), nullptr, vb.data(), ng);
      size_t with_nulls = 0;
      for (const auto& sg : g.DeviceKeys(0).segments()) with_nulls += sg.col.validity != nullptr;
      EXPECT(g.Resized(0) && g.DeviceKeys(0).segments().size() >= 20 && (null_every == 0) == (with_nulls == 0),
             "grouped rehash (NULLs every %d): resized %d, %zu segments, %zu with NULLs", null_every, g.Resized(0) ? 1 : 0,
             g.DeviceKeys(0).segments().size(), with_nulls);
      EXPECT(g.GetBloomFilter(0)->ExportWords() == g0 && g.GetBloomFilter(1)->ExportWords() == g1,
             "grouped rehash (NULLs every %d): words differ from the oracle", null_every);
    }
    // min/max dynamic filter per build column (physical_create_bf.cpp:229-272), NULLs skipped
    {
      std::vector<uint64_t> va = pack(bt.v0, 0, nb), vb = pack(bt.v1, 0, nb);
      int64_t e0[2], e1[2], mn = 0, mx = 0;
      const int h0 = rpt_oracle_minmax_i64(bt.c0.data(), nullptr, va.data(), nb, e0);
      const int h1 = rpt_oracle_minmax_i32(bt.c1.data(), nullptr, vb.data(), nb, e1);
      EXPECT(h0 && create.MinMax(0, mn, mx) && mn == e0[0] && mx == e0[1], "column 0 min/max %lld..%lld vs %lld..%lld",
             (long long)mn, (long long)mx, (long long)e0[0], (long long)e0[1]);
      EXPECT(h1 && create.MinMax(1, mn, mx) && mn == e1[0] && mx == e1[1], "column 1 min/max %lld..%lld vs %lld..%lld",
             (long long)mn, (long long)mx, (long long)e1[0], (long long)e1[1]);
    }

    // ---------------- source: the materialized chunks re-emitted by thread range ---------------
    {
      const size_t cc = create.ChunkCount();
      EXPECT(cc == bst.chunks.size(), "chunk count %zu", cc);
      auto gs = create.GetGlobalSourceState(3);
      const size_t per = (cc + 2) / 3;  // physical_create_bf.cpp:469-485
      EXPECT(gs->chunks_todo.size() == 3 && gs->chunks_todo[0].first == 0 && gs->chunks_todo[0].second == per &&
                 gs->chunks_todo[2].second == cc, "source ranges");
      std::vector<std::vector<rpt::DataChunk>> got(4);
      std::vector<std::thread> src;
      for (int t = 0; t < 4; t++)
        src.emplace_back([&, t] {
          rpt::CreateBF::LocalSourceState ls;
          rpt::DataChunk c;
          while (create.GetData(*gs, ls, c)) got[t].push_back(c);
        });
      for (auto& th : src) th.join();
      size_t empty_threads = 0;
      std::vector<std::pair<int64_t, int64_t>> rows_out, rows_in;  // (c0 or NULL marker, c1 or NULL)
      const int64_t kNull = INT64_MIN;
      for (auto& g : got) {
        empty_threads += g.empty();
        for (const auto& c : g) {
          EXPECT(c.data.size() == 3 && c.data[2].data == nullptr, "payload column shape");
          auto* a = static_cast<const int64_t*>(c.data[0].data);
          auto* b = static_cast<const int32_t*>(c.data[1].data);
          for (size_t r = 0; r < c.count; r++) {
            const bool va = !c.data[0].validity || ((c.data[0].validity[r / 64] >> (r % 64)) & 1);
            const bool vb = !c.data[1].validity || ((c.data[1].validity[r / 64] >> (r % 64)) & 1);
            rows_out.emplace_back(va ? a[r] : kNull, vb ? b[r] : kNull);
          }
        }
      }
      for (size_t i = 0; i < nb; i++) rows_in.emplace_back(bt.v0[i] ? bt.c0[i] : kNull, bt.v1[i] ? bt.c1[i] : kNull);
      std::sort(rows_out.begin(), rows_out.end());
      std::sort(rows_in.begin(), rows_in.end());
      EXPECT(empty_threads == 1, "one of 4 source threads finds no range (%zu)", empty_threads);
      EXPECT(rows_out == rows_in, "the source re-emits exactly the sunk rows (%zu vs %zu)", rows_out.size(), rows_in.size());
    }
    // the resize predicate (physical_create_bf.cpp:383-398) under both rules, sized for 1000 rows:
    // 1024 actual rows fill the allocation at 8 bits/row under either; 2048 resize on the allocation
    // (default) but not by the reference's formula (its 12-bit pricing allocates 16384 bits); 2049 resize
    // under both. Words == the oracle's filter of the size each rule leaves.
    for (const uint64_t rows : {1024ull, 2048ull, 2049ull}) {
      for (const auto rule : {rpt::CreateBF::ResizeRule::kOnAllocation, rpt::CreateBF::ResizeRule::kReferenceFormula}) {
        rpt::CreateBF c3(dev, /*estimated_cardinality=*/1000, {0}, rpt::CreateBF::kDefaultSinkFlushRows, rule);
        auto l3 = c3.MakeLocalState();
        rpt::DataChunk ch = bst.chunks[0];
        size_t done = 0;
        for (size_t k = 0; done < rows; k++) {
          ch = bst.chunks[k];
          ch.count = std::min<size_t>(ch.count, rows - done);
          c3.Sink(*l3, ch);
          done += ch.count;
        }
        c3.Combine(*l3);
        c3.Finalize();
        const bool ref_rule = rule == rpt::CreateBF::ResizeRule::kReferenceFormula;
        const bool want = ref_rule ? rows > 2048 : rows > 1024;
        EXPECT(c3.Resized(0) == want, "rows %llu rule %d: resized %d", (unsigned long long)rows, (int)ref_rule,
               (int)c3.Resized(0));
        const int oracle_says = ref_rule ? rpt_oracle_needs_resize(1000, rows)
                                         : rpt_oracle_needs_resize_alloc(rpt_oracle_log_num_blocks(1000), rows);
        EXPECT(c3.Resized(0) == (oracle_says > 0),
               "rows %llu rule %d: oracle predicate", (unsigned long long)rows, (int)ref_rule);
        const int l = c3.Resized(0) ? rpt_oracle_log_num_blocks(rows) : rpt_oracle_log_num_blocks(1000);
        std::vector<uint64_t> wr(1ULL << l, 0);
        std::vector<uint64_t> va = pack(bt.v0, 0, rows);
        rpt_oracle_insert_i64(wr.data(), l, bt.c0.data(), nullptr, va.data(), rows);
        EXPECT(c3.GetBloomFilter(0)->LogNumBlocks() == l && c3.GetBloomFilter(0)->ExportWords() == wr,
               "rows %llu rule %d: filter words", (unsigned long long)rows, (int)ref_rule);
      }
    }
    // SEQUENCE vectors (DuckDB SEQUENCE_VECTOR: start + row * increment, e.g. range() keys): build two
    // filters from sequence chunks (int64, and int32 wrapping past INT32_MAX as DuckDB's INTEGER sequence),
    // then a USE_BF chain whose second filter sees the sequence sliced by the first's survivors
    {
      const uint64_t rows = 3 * 2048 + 77;
      std::vector<int64_t> s64(rows);
      std::vector<int32_t> s32(rows);
      for (uint64_t r = 0; r < rows; r++) {
        s64[r] = -500000 + 3 * static_cast<int64_t>(r);
        s32[r] = static_cast<int32_t>(static_cast<uint32_t>(INT32_MAX - 5000) + 7u * static_cast<uint32_t>(r));
      }
      rpt::CreateBF cs(dev, /*estimated_cardinality=*/rows, {0, 1});
      auto ls = cs.MakeLocalState();
      for (uint64_t lo = 0; lo < rows; lo += 2048) {
        rpt::DataChunk ch;
        ch.count = std::min<uint64_t>(2048, rows - lo);
        ch.data.resize(2);
        ch.data[0].type = rpt::VectorType::SEQUENCE;
        ch.data[0].key_type = rpt::KeyType::I64;
        ch.data[0].seq_start = s64[lo];
        ch.data[0].seq_increment = 3;
        ch.data[1].type = rpt::VectorType::SEQUENCE;
        ch.data[1].key_type = rpt::KeyType::I32;
        ch.data[1].seq_start = s32[lo];
        ch.data[1].seq_increment = 7;
        cs.Sink(*ls, ch);
      }
      cs.Combine(*ls);
      cs.Finalize();
      const int ls_nb = rpt_oracle_log_num_blocks(rows);
      std::vector<uint64_t> q0(1ULL << ls_nb, 0), q1(1ULL << ls_nb, 0);
      rpt_oracle_insert_i64(q0.data(), ls_nb, s64.data(), nullptr, nullptr, rows);
      rpt_oracle_insert_i32(q1.data(), ls_nb, s32.data(), nullptr, nullptr, rows);
      EXPECT(cs.GetBloomFilter(0)->ExportWords() == q0, "int64 sequence filter differs from the oracle");
      EXPECT(cs.GetBloomFilter(1)->ExportWords() == q1, "int32 sequence filter differs from the oracle");
      // probe: a sequence over a wider range (half the rows hit), filter 0 then filter 1 on the survivors
      const uint64_t np_ = 2000;
      std::vector<int64_t> p64(np_);
      std::vector<int32_t> p32(np_);
      for (uint64_t r = 0; r < np_; r++) {
        p64[r] = -500000 + 3 * 5 * static_cast<int64_t>(r);
        p32[r] = static_cast<int32_t>(static_cast<uint32_t>(INT32_MAX - 5000) + 7u * 2u * static_cast<uint32_t>(r));
      }
      rpt::DataChunk pc;
      pc.count = np_;
      pc.data.resize(2);
      pc.data[0].type = rpt::VectorType::SEQUENCE;
      pc.data[0].key_type = rpt::KeyType::I64;
      pc.data[0].seq_start = p64[0];
      pc.data[0].seq_increment = 15;
      pc.data[1].type = rpt::VectorType::SEQUENCE;
      pc.data[1].key_type = rpt::KeyType::I32;
      pc.data[1].seq_start = p32[0];
      pc.data[1].seq_increment = 14;
      std::vector<uint32_t> o0(np_), o1(np_);
      const uint64_t c0 = rpt_oracle_probe_i64(q0.data(), ls_nb, p64.data(), nullptr, nullptr, np_, o0.data());
      std::vector<int32_t> p32s(c0);
      for (uint64_t r = 0; r < c0; r++) p32s[r] = p32[o0[r]];
      const uint64_t c1 = rpt_oracle_probe_i32(q1.data(), ls_nb, p32s.data(), nullptr, nullptr, c0, o1.data());
      std::vector<uint32_t> want(c1);
      for (uint64_t r = 0; r < c1; r++) want[r] = o0[o1[r]];
      rpt::DeviceContext sctx(dev);
      rpt::UseBF su({cs.GetBloomFilter(0), cs.GetBloomFilter(1)}, {0, 1});
      rpt::SelectionVector got;
      const uint64_t gc = su.Execute(sctx, pc, got);
      EXPECT(gc == c1 && got == want, "sequence USE_BF chain: %llu survivors vs oracle %llu", (unsigned long long)gc,
             (unsigned long long)c1);
      EXPECT(c1 > 0 && c1 < np_, "the sequence probe must keep some rows and drop others (%llu)", (unsigned long long)c1);
    }
    // default sink batching (all inserts at Combine), no resize: same filter as the oracle's
    {
      rpt::CreateBF c2(dev, /*estimated_cardinality=*/nb, {0});
      auto l = c2.MakeLocalState();
      for (const auto& ch : bst.chunks) c2.Sink(*l, ch);
      c2.Combine(*l);
      c2.Finalize();
      EXPECT(!c2.Resized(0) && c2.SkippedInsertRows() == 0, "no resize (and no skipped insert) at the right estimate");
      EXPECT(c2.GetBloomFilter(0)->ExportWords() == w0, "batched-sink filter differs from the oracle");
    }

    // ---------------- probe -------------------------------------------------------------------
    const size_t np = 20000;
    Table pt = make_table(np, 2, 31, 2048);
    for (size_t i = 0; i < np; i += 3) {  // a third of the probe rows hit the build side
      pt.c0[i] = bt.c0[(i * 7) % nb];
      pt.c1[i] = bt.c1[(i * 7) % nb];
    }
    ChunkStore pst;
    make_chunks(pt, np, pst, true);
    rpt::DeviceContext ctx(dev);
    rpt::UseBF use({f0, f1}, {0, 1});
    std::vector<uint32_t> tmp0(np), tmp1(np);
    size_t base = 0, total = 0;
    for (const auto& ch : pst.chunks) {
      rpt::SelectionVector out;
      use.Execute(ctx, ch, out);
      // oracle: AND of the two filters over this chunk's rows
      std::vector<uint64_t> va = pack(pt.v0, base, ch.count), vb = pack(pt.v1, base, ch.count);
      const uint64_t n0 = rpt_oracle_probe_i64(w0.data(), lnb, pt.c0.data() + base, nullptr, va.data(), ch.count, tmp0.data());
      const uint64_t n1 = rpt_oracle_probe_i32(w1.data(), lnb, pt.c1.data() + base, nullptr, vb.data(), ch.count, tmp1.data());
      std::vector<uint32_t> exp;
      for (uint64_t i = 0, j = 0; i < n0; i++) {
        while (j < n1 && tmp1[j] < tmp0[i]) j++;
        if (j < n1 && tmp1[j] == tmp0[i]) exp.push_back(tmp0[i]);
      }
      EXPECT(out == exp, "USE_BF chunk at row %zu: %zu survivors, oracle %zu", base, out.size(), exp.size());
      total += out.size();
      base += ch.count;
    }
    EXPECT(use.rows_in() == np && use.rows_out() == total, "USE_BF counters");
    // The per-chunk Execute above runs the chain as one launch (rpt_bf_probe_chain). One FLAT chunk of all
    // np rows (> RPT_SMALL_PROBE_ROWS) takes the filter-by-filter loop instead, and a never-finalized filter
    // inside the chain is skipped on both paths: both must give the oracle's AND.
    {
      auto nf = std::make_shared<rpt::PTBloomFilter>();
      nf->Initialize(dev, 10);
      rpt::UseBF us({f0, nf, f1}, {0, 0, 1});
      std::vector<uint64_t> va = pack(pt.v0, 0, np), vb = pack(pt.v1, 0, np);
      rpt::DataChunk big;
      big.count = np;
      big.data.resize(2);
      big.data[0].key_type = rpt::KeyType::I64;
      big.data[0].data = pt.c0.data();
      big.data[0].validity = va.data();
      big.data[1].key_type = rpt::KeyType::I32;
      big.data[1].data = pt.c1.data();
      big.data[1].validity = vb.data();
      std::vector<uint32_t> a(np), b(np), exp;
      const uint64_t n0 = rpt_oracle_probe_i64(w0.data(), lnb, pt.c0.data(), nullptr, va.data(), np, a.data());
      const uint64_t n1 = rpt_oracle_probe_i32(w1.data(), lnb, pt.c1.data(), nullptr, vb.data(), np, b.data());
      std::set_intersection(a.begin(), a.begin() + n0, b.begin(), b.begin() + n1, std::back_inserter(exp));
      rpt::SelectionVector out;
      us.Execute(ctx, big, out);
      EXPECT(np > RPT_SMALL_PROBE_ROWS && out == exp, "USE_BF over one %zu-row chunk: %zu survivors, oracle %zu", np,
             out.size(), exp.size());
      size_t base2 = 0;
      for (const auto& ch : pst.chunks) {  // the chained launch with the skipped filter in the middle
        rpt::SelectionVector o2, o1;
        us.Execute(ctx, ch, o2);
        use.Execute(ctx, ch, o1);
        EXPECT(o2 == o1, "skipped filter inside the chain changed chunk at row %zu", base2);
        base2 += ch.count;
      }
    }
    // the same chain over the whole batch at once (survivors stay on the device between filters)
    {
      std::vector<const rpt::DataChunk*> ptrs;
      for (const auto& ch : pst.chunks) ptrs.push_back(&ch);
      rpt::UseBF ub({f0, f1}, {0, 1});
      std::vector<rpt::SelectionVector> outs;
      const uint64_t got = ub.ExecuteBatch(ctx, ptrs, outs);
      EXPECT(got == total && ub.rows_in() == np && ub.rows_out() == total, "batched USE_BF counters %llu",
             (unsigned long long)got);
      for (size_t k = 0; k < ptrs.size(); k++) {
        rpt::SelectionVector one;
        use.Execute(ctx, *ptrs[k], one);
        EXPECT(outs[k] == one, "batched USE_BF differs at chunk %zu", k);
      }
      auto nf = std::make_shared<rpt::PTBloomFilter>();
      nf->Initialize(dev, 10);  // never finalized: skipped
      rpt::UseBF skip({nf}, {0});
      EXPECT(skip.ExecuteBatch(ctx, ptrs, outs) == np && outs[1].size() == ptrs[1]->count, "batched skip");
    }
    // batch lookup == per-chunk lookup
    {
      std::vector<const rpt::DataChunk*> ptrs;
      for (const auto& ch : pst.chunks) ptrs.push_back(&ch);
      std::vector<rpt::SelectionVector> sels;
      f0->LookupSelBatch(ctx, ptrs, sels, {0});
      for (size_t k = 0; k < ptrs.size(); k++) {
        rpt::SelectionVector one;
        f0->LookupSel(ctx, *ptrs[k], one, {0});
        EXPECT(sels[k] == one, "batch lookup differs at chunk %zu", k);
      }
    }
    // pipelined batches: stages of >= 3000 rows (FLAT / CONSTANT / DICTIONARY chunks, NULLs), both key
    // types, lookups == per-chunk lookups and inserts == the oracle's words
    {
      rpt::DeviceContext pctx(dev);
      pctx.pipeline_rows = 3000;
      std::vector<const rpt::DataChunk*> ptrs;
      for (const auto& ch : pst.chunks) ptrs.push_back(&ch);
      for (int c = 0; c < 2; c++) {
        const auto& f = c == 0 ? f0 : f1;
        std::vector<rpt::SelectionVector> sels;
        f->LookupSelBatch(pctx, ptrs, sels, {static_cast<uint64_t>(c)});
        for (size_t k = 0; k < ptrs.size(); k++) {
          rpt::SelectionVector one;
          f->LookupSel(ctx, *ptrs[k], one, {static_cast<uint64_t>(c)});
          EXPECT(sels[k] == one, "pipelined lookup (column %d) differs at chunk %zu", c, k);
        }
      }
      std::vector<const rpt::DataChunk*> bptrs;
      for (const auto& ch : bst.chunks) bptrs.push_back(&ch);
      for (int c = 0; c < 2; c++) {
        rpt::PTBloomFilter fp;
        fp.Initialize(dev, static_cast<uint32_t>(nb));
        fp.InsertBatch(pctx, bptrs, {static_cast<uint64_t>(c)});
        EXPECT(fp.ExportWords() == (c == 0 ? w0 : w1), "pipelined insert (column %d) differs from the oracle", c);
      }
    }
    // ---------------- early exits / skips ---------------------------------------------------
    {
      rpt::CreateBF empty(dev, 100, {0});
      empty.Finalize();
      auto fe = empty.GetBloomFilter(0);
      EXPECT(fe->IsEmpty() && fe->finalized_, "empty build");
      rpt::UseBF u({fe}, {0});
      rpt::SelectionVector out;
      EXPECT(u.Execute(ctx, pst.chunks[0], out) == 0 && out.empty(), "empty filter -> no rows");
      auto nf = std::make_shared<rpt::PTBloomFilter>();
      nf->Initialize(dev, 10);  // never finalized: skipped, all rows pass
      rpt::UseBF u2({nf}, {0});
      EXPECT(u2.Execute(ctx, pst.chunks[0], out) == pst.chunks[0].count, "not-finalized filter is skipped");
      rpt::UseBF u3({f0}, {0}, /*passthrough=*/true);
      EXPECT(u3.Execute(ctx, pst.chunks[0], out) == pst.chunks[0].count, "passthrough");
      bool threw = false;
      try {
        rpt::SelectionVector s2;
        f0->LookupSel(ctx, pst.chunks[0], s2, {});
      } catch (const rpt::GpuError& e) {
        threw = e.status() == RPT_ERR_INVALID_ARGUMENT;
      }
      EXPECT(threw, "an empty key column list is rejected with INVALID_ARGUMENT");
    }
    // ---------------- composite key (HashColumns' CombineHash, bloom_filter.cpp:15-17) --------
    {
      rpt::PTBloomFilter fc;
      fc.Initialize(dev, static_cast<uint32_t>(nb));
      std::vector<const rpt::DataChunk*> ptrs;
      for (const auto& ch : bst.chunks) ptrs.push_back(&ch);
      fc.InsertBatch(ctx, ptrs, {0, 1});
      const int lc = fc.LogNumBlocks();
      std::vector<uint64_t> h(nb), wc(1ULL << lc, 0);
      std::vector<uint64_t> va = pack(bt.v0, 0, nb), vb = pack(bt.v1, 0, nb);
      rpt_oracle_hash_i64(bt.c0.data(), nullptr, va.data(), nb, h.data());
      rpt_oracle_hash_combine_i32(bt.c1.data(), nullptr, vb.data(), nb, h.data());
      rpt_oracle_insert_hashes(wc.data(), lc, h.data(), nb);
      EXPECT(fc.ExportWords() == wc, "composite-key filter words differ from the oracle");
      size_t base = 0;
      std::vector<uint32_t> exp(2048);
      for (const auto& ch : pst.chunks) {
        rpt::SelectionVector out;
        fc.LookupSel(ctx, ch, out, {0, 1});
        std::vector<uint64_t> ph(ch.count);
        std::vector<uint64_t> pa = pack(pt.v0, base, ch.count), pb = pack(pt.v1, base, ch.count);
        rpt_oracle_hash_i64(pt.c0.data() + base, nullptr, pa.data(), ch.count, ph.data());
        rpt_oracle_hash_combine_i32(pt.c1.data() + base, nullptr, pb.data(), ch.count, ph.data());
        const uint64_t ne = rpt_oracle_lookup_sel_hashes(wc.data(), lc, ph.data(), ch.count, exp.data());
        EXPECT(out == std::vector<uint32_t>(exp.begin(), exp.begin() + ne), "composite probe at row %zu", base);
        base += ch.count;
      }
    }
    // ---------------- a 256 MiB filter: batched insert / lookup take the bucketed strategy ----------
    {
      const size_t nbig = 5000000;
      std::vector<int64_t> keys(nbig);
      std::mt19937_64 rng(9);
      for (auto& k : keys) k = static_cast<int64_t>(rng());
      std::vector<rpt::DataChunk> chunks;
      for (size_t lo = 0; lo < nbig; lo += 500000) {
        rpt::DataChunk ch;
        ch.count = std::min<size_t>(500000, nbig - lo);
        rpt::Vector v;
        v.key_type = rpt::KeyType::I64;
        v.data = keys.data() + lo;
        ch.data.push_back(v);
        chunks.push_back(ch);
      }
      std::vector<const rpt::DataChunk*> ptrs;
      for (const auto& c : chunks) ptrs.push_back(&c);
      rpt::PTBloomFilter fb;
      fb.Initialize(dev, 1u << 28);  // 2^28 rows -> 2^25 blocks (256 MiB)
      EXPECT(fb.LogNumBlocks() == 25, "big filter log blocks %d", fb.LogNumBlocks());
      // AUTO routes 256 MiB filters from 32 Mi rows per batch; this batch is pinned to the bucketed path
      rpt_bf_set_insert_strategy(fb.native(), RPT_INSERT_BUCKETED);
      rpt_bf_set_probe_strategy(fb.native(), RPT_PROBE_BUCKETED);
      EXPECT(rpt_bf_insert_strategy_for(fb.native(), nbig) == RPT_INSERT_BUCKETED, "bucketed insert expected");
      fb.InsertBatch(ctx, ptrs, {0});
      std::vector<uint64_t> wb(1ULL << 25, 0);
      rpt_oracle_insert_i64(wb.data(), 25, keys.data(), nullptr, nullptr, nbig);
      EXPECT(fb.ExportWords() == wb, "bucketed insert words differ from the oracle");
      int64_t mn = 0, mx = 0;
      EXPECT(fb.MinMax(mn, mx) && mn == *std::min_element(keys.begin(), keys.end()) &&
                 mx == *std::max_element(keys.begin(), keys.end()), "bucketed insert min/max");
      // probe the same rows plus fresh ones, as one batch (bucketed) -- every build key must pass
      for (size_t i = 0; i < nbig; i += 2) keys[i] = static_cast<int64_t>(rng());
      EXPECT(rpt_bf_probe_strategy_for(fb.native(), nbig) == RPT_PROBE_BUCKETED, "bucketed probe expected");
      std::vector<rpt::SelectionVector> sels;
      fb.LookupSelBatch(ctx, ptrs, sels, {0});
      std::vector<uint32_t> exp(500000);
      for (size_t k = 0; k < chunks.size(); k++) {
        const uint64_t ne = rpt_oracle_probe_i64(wb.data(), 25, keys.data() + k * 500000, nullptr, nullptr,
                                                 chunks[k].count, exp.data());
        EXPECT(sels[k] == std::vector<uint32_t>(exp.begin(), exp.begin() + ne), "bucketed probe chunk %zu", k);
      }
    }
    typed_keys(dev);
  } catch (const std::exception& e) {
    fprintf(stderr, "exception: %s\n", e.what());
    return 2;
  }
  if (g_fail) {
    fprintf(stderr, "%d check(s) failed\n", g_fail);
    return 1;
  }
  printf("ALL OK\n");
  return 0;
}
