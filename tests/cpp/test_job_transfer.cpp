// test_job_transfer.cpp — a JOB-shaped predicate transfer through the C++ operators (include/rpt_host.hpp) on the
// GPU: the closest stand-in for JOB-113 (BASELINE config 4) the image allows. DuckDB is absent,
// so the plan is fixed here; tests/test_gpu_job_transfer.py writes the tables, runs this program and checks what it
// writes against the oracle and a numpy join.
//
// Four tables of INTEGER join keys with NULLs (the JOB shape: a fact table, a dimension, a mid table and a second
// fact table), already reduced by their base predicates:
//   mi(movie_id, info_type_id)   it(id)   t(id)   mc(movie_id)
//   joins: mi.info_type_id = it.id, mi.movie_id = t.id, t.id = mc.movie_id
// The transfer schedule is the one GenerateStageModifications emits for this join tree under the largest_root
// heuristic (reference src/optimizer/rpt_optimizer.cpp:828-995): root mi (largest), level 1 {it, t} sorted by
// cardinality, level 2 {mc}; forward pass leaves -> root, then backward pass root -> leaves:
//   forward   f_mc  = CREATE_BF(mc.movie_id)          -> USE_BF(t.id)
//             f_it  = CREATE_BF(it.id)                -> USE_BF(mi.info_type_id)
//             f_t   = CREATE_BF(t.id)  [t after f_mc] -> USE_BF(mi.movie_id)
//   backward  f_mi_it, f_mi_t = CREATE_BF(mi.info_type_id, mi.movie_id) [mi after f_it, f_t; one operator with
//             two build columns, as BuildStackedBFOperators merges consecutive CREATEs, rpt_optimizer.cpp:1171-1216]
//                                                      -> USE_BF(it.id), USE_BF(t.id)
//             f_t2  = CREATE_BF(t.id)  [t after f_mi_t] -> USE_BF(mc.movie_id)
// Each table flows as DuckDB's pipeline would: scan -> forward USE_BF -> forward CREATE_BF (Sink on several threads,
// Combine, Finalize, then the parallel source re-emits the materialized chunks) -> backward USE_BF -> backward
// CREATE_BF. Every filter is probed inside USE_BF (the GPU mode: no BFTableFilter scan pushdown).
// USE_BF output is the input chunk sliced by the selection vector (DICTIONARY vectors over the input, as
// DataChunk::Slice), fed to the next operator. Every chunk carries the row id (BIGINT payload) through the
// materialization and re-emission, so the survivors can be named.
//
// Files (in the directory argv[1]): inputs <table>_<col>.i32 (int32 keys), <table>_<col>.valid (uint8), est.txt
// ("<filter> <estimated cardinality>" lines); outputs use_<name>.i64 (row ids surviving each USE_BF, any order),
// bf_<name>.u64 (the finalized filter's words) + bf_<name>.txt ("log_num_blocks resized rows").
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <map>
#include <memory>
#include <mutex>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

#include "rpt_host.hpp"

static int g_fail = 0;
#define EXPECT(cond, ...)                                  \
  do {                                                     \
    if (!(cond)) {                                         \
      fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
      fprintf(stderr, __VA_ARGS__);                        \
      fprintf(stderr, "\n");                               \
      g_fail++;                                            \
    }                                                      \
  } while (0)

static std::string g_dir;
constexpr size_t kVector = 2048;  // STANDARD_VECTOR_SIZE

template <typename T>
static std::vector<T> read_file(const std::string& name) {
  std::ifstream f(g_dir + "/" + name, std::ios::binary | std::ios::ate);
  if (!f) throw std::runtime_error("missing input " + name);
  const size_t bytes = static_cast<size_t>(f.tellg());
  std::vector<T> v(bytes / sizeof(T));
  f.seekg(0);
  f.read(reinterpret_cast<char*>(v.data()), static_cast<std::streamsize>(v.size() * sizeof(T)));
  return v;
}

template <typename T>
static void write_file(const std::string& name, const std::vector<T>& v) {
  std::ofstream f(g_dir + "/" + name, std::ios::binary);
  f.write(reinterpret_cast<const char*>(v.data()), static_cast<std::streamsize>(v.size() * sizeof(T)));
}

// A base table as scanned: key columns (INTEGER, with NULLs) + the row id payload (BIGINT), in 2048-row chunks.
// Every third chunk's key columns arrive as DICTIONARY vectors (reversed dictionary), the others FLAT.
struct Table {
  std::string name;
  size_t rows = 0;
  std::vector<std::vector<int32_t>> keys;      // [col][row]
  std::vector<std::vector<uint64_t>> valid;    // [col] ValidityMask words over the whole table (FLAT chunks)
  std::vector<int64_t> row_id;
  // storage of the DICTIONARY chunks
  std::vector<std::vector<int32_t>> dict_keys;
  std::vector<std::vector<uint32_t>> dict_sel;
  std::vector<std::vector<uint64_t>> dict_valid;
  std::vector<std::vector<uint64_t>> flat_valid;
  std::vector<rpt::DataChunk> chunks;
};

static Table load_table(const std::string& name, const std::vector<std::string>& cols) {
  Table t;
  t.name = name;
  for (const auto& c : cols) {
    t.keys.push_back(read_file<int32_t>(name + "_" + c + ".i32"));
    const std::vector<uint8_t> v = read_file<uint8_t>(name + "_" + c + ".valid");
    t.rows = v.size();
    std::vector<uint64_t> w((t.rows + 63) / 64 + 1, 0);
    for (size_t r = 0; r < t.rows; r++)
      if (v[r]) w[r / 64] |= 1ULL << (r % 64);
    t.valid.push_back(std::move(w));
  }
  t.row_id.resize(t.rows);
  for (size_t r = 0; r < t.rows; r++) t.row_id[r] = static_cast<int64_t>(r);
  auto bit = [](const std::vector<uint64_t>& w, size_t r) { return (w[r / 64] >> (r % 64)) & 1; };
  for (size_t lo = 0, k = 0; lo < t.rows; lo += kVector, k++) {
    const size_t cnt = std::min(kVector, t.rows - lo);
    rpt::DataChunk ch;
    ch.count = cnt;
    for (size_t c = 0; c < cols.size(); c++) {
      rpt::Vector v;
      v.key_type = rpt::KeyType::I32;
      if (k % 3 == 2) {
        std::vector<int32_t> dict(cnt);
        std::vector<uint32_t> sel(cnt);
        std::vector<uint64_t> dv((cnt + 63) / 64 + 1, 0);
        for (size_t i = 0; i < cnt; i++) {
          dict[cnt - 1 - i] = t.keys[c][lo + i];
          if (bit(t.valid[c], lo + i)) dv[(cnt - 1 - i) / 64] |= 1ULL << ((cnt - 1 - i) % 64);
          sel[i] = static_cast<uint32_t>(cnt - 1 - i);
        }
        t.dict_keys.push_back(std::move(dict));
        t.dict_sel.push_back(std::move(sel));
        t.dict_valid.push_back(std::move(dv));
        v.type = rpt::VectorType::DICTIONARY;
        v.data = t.dict_keys.back().data();
        v.sel = t.dict_sel.back().data();
        v.dict_size = cnt;
        v.validity = t.dict_valid.back().data();
      } else {
        std::vector<uint64_t> fv((cnt + 63) / 64 + 1, 0);
        for (size_t i = 0; i < cnt; i++)
          if (bit(t.valid[c], lo + i)) fv[i / 64] |= 1ULL << (i % 64);
        t.flat_valid.push_back(std::move(fv));
        v.type = rpt::VectorType::FLAT;
        v.data = t.keys[c].data() + lo;
        v.validity = t.flat_valid.back().data();
      }
      ch.data.push_back(v);
    }
    rpt::Vector id;
    id.key_type = rpt::KeyType::I64;
    id.data = t.row_id.data() + lo;
    ch.data.push_back(id);
    t.chunks.push_back(std::move(ch));
  }
  return t;
}

// DataChunk::Slice(sel, count): every column becomes a DICTIONARY over the input's data (a DICTIONARY input composes
// its selection), the validity stays indexed by the physical index. The slices' selection vectors live in `store`.
static rpt::DataChunk slice(const rpt::DataChunk& in, const rpt::SelectionVector& sel,
                            std::vector<std::unique_ptr<std::vector<uint32_t>>>& store) {
  rpt::DataChunk out;
  out.count = sel.size();
  for (const rpt::Vector& v : in.data) {
    rpt::Vector s = v;
    auto idx = std::make_unique<std::vector<uint32_t>>(sel.size());
    if (v.type == rpt::VectorType::DICTIONARY) {
      for (size_t i = 0; i < sel.size(); i++) (*idx)[i] = v.sel[sel[i]];
    } else {
      for (size_t i = 0; i < sel.size(); i++) (*idx)[i] = sel[i];
      s.dict_size = in.count;
    }
    s.type = rpt::VectorType::DICTIONARY;
    s.sel = idx->data();
    store.push_back(std::move(idx));
    out.data.push_back(s);
  }
  return out;
}

static int64_t row_id_at(const rpt::DataChunk& ch, size_t r) {
  const rpt::Vector& v = ch.data.back();
  const auto* ids = static_cast<const int64_t*>(v.data);
  return v.type == rpt::VectorType::DICTIONARY ? ids[v.sel[r]] : ids[r];
}

// One USE_BF operator over a stream of chunks. batch = false: ExecuteInternal per chunk (the chain in one launch per
// chunk, physical_use_bf.cpp:60-198); true: the caching operator's ExecuteBatch over all chunks (pipelined in stages
// of ctx.pipeline_rows). Returns the sliced chunks; records the survivors' row ids.
struct UseResult {
  std::vector<rpt::DataChunk> chunks;
  std::vector<std::unique_ptr<std::vector<uint32_t>>> store;
  std::vector<int64_t> ids;
};

static void use_bf(int dev, const std::string& name, const std::vector<std::shared_ptr<rpt::PTBloomFilter>>& filters,
                   const std::vector<uint64_t>& cols, const std::vector<rpt::DataChunk>& in, bool batch, UseResult& out,
                   bool passthrough = false) {
  rpt::DeviceContext ctx(dev);
  ctx.pipeline_rows = 1ULL << 16;  // stages of 64 Ki rows: a pipelined chain over several stages
  rpt::UseBF op(filters, cols, passthrough);
  std::vector<rpt::SelectionVector> sels(in.size());
  uint64_t rows_in = 0;
  if (batch) {
    std::vector<const rpt::DataChunk*> ptrs;
    for (const auto& c : in) ptrs.push_back(&c);
    op.ExecuteBatch(ctx, ptrs, sels);
  } else {
    for (size_t k = 0; k < in.size(); k++) op.Execute(ctx, in[k], sels[k]);
  }
  uint64_t kept = 0;
  for (size_t k = 0; k < in.size(); k++) {
    rows_in += in[k].count;
    const auto& s = sels[k];
    bool asc = true;
    for (size_t i = 1; i < s.size(); i++) asc &= s[i] > s[i - 1];
    EXPECT(asc && (s.empty() || s.back() < in[k].count), "%s: chunk %zu sel not ascending / in range", name.c_str(), k);
    if (s.empty()) continue;  // zero survivors: the operator returns no chunk (physical_use_bf.cpp:166-173)
    out.chunks.push_back(slice(in[k], s, out.store));
    for (size_t i = 0; i < s.size(); i++) out.ids.push_back(row_id_at(out.chunks.back(), i));
    kept += s.size();
  }
  EXPECT(passthrough || (op.rows_in() == rows_in && op.rows_out() == kept), "%s: operator counters %llu/%llu vs %llu/%llu", name.c_str(),
         (unsigned long long)op.rows_in(), (unsigned long long)op.rows_out(), (unsigned long long)rows_in,
         (unsigned long long)kept);
  write_file("use_" + name + ".i64", out.ids);
  printf("USE_BF %-10s %8llu -> %8llu rows (%s)\n", name.c_str(), (unsigned long long)rows_in, (unsigned long long)kept,
         batch ? "ExecuteBatch" : "Execute per chunk");
}

// One CREATE_BF operator: Sink on `threads` threads (chunk k to thread k % threads, each with its own local state and
// device context), Combine, Finalize; then the parallel source re-emits the materialized chunks (3 source threads).
static std::vector<rpt::DataChunk> create_bf(rpt::CreateBF& op, const std::vector<std::string>& names,
                                             const std::vector<rpt::DataChunk>& in, int threads) {
  std::vector<std::unique_ptr<rpt::CreateBF::LocalState>> locals;
  for (int t = 0; t < threads; t++) locals.push_back(op.MakeLocalState());
  std::vector<std::thread> ths;
  for (int t = 0; t < threads; t++)
    ths.emplace_back([&, t] {
      for (size_t k = t; k < in.size(); k += threads) op.Sink(*locals[t], in[k]);
    });
  for (auto& th : ths) th.join();
  for (auto& l : locals) op.Combine(*l);
  op.Finalize();
  uint64_t rows = 0;
  for (const auto& c : in) rows += c.count;
  EXPECT(op.MaterializedRows() == rows, "CREATE_BF %s: materialized %llu of %llu", names[0].c_str(),
         (unsigned long long)op.MaterializedRows(), (unsigned long long)rows);
  for (size_t i = 0; i < names.size(); i++) {
    auto f = op.GetBloomFilter(i);
    EXPECT(f->finalized_, "CREATE_BF %s: not finalized", names[i].c_str());
    write_file("bf_" + names[i] + ".u64", f->ExportWords());
    std::ofstream m(g_dir + "/bf_" + names[i] + ".txt");
    m << f->LogNumBlocks() << " " << (op.Resized(i) ? 1 : 0) << " " << rows << "\n";
    printf("CREATE_BF %-8s %8llu rows, 2^%d blocks%s\n", names[i].c_str(), (unsigned long long)rows, f->LogNumBlocks(),
           op.Resized(i) ? " (resized)" : "");
  }
  // the source (physical_create_bf.cpp:441-557): ranges of ceil(chunks / 3) chunks, one per source thread; the
  // re-emitted chunks in range order
  auto gs = op.GetGlobalSourceState(3);
  std::vector<std::vector<rpt::DataChunk>> got(3);
  std::vector<std::thread> src;
  for (int t = 0; t < 3; t++)
    src.emplace_back([&, t] {
      rpt::CreateBF::LocalSourceState ls;
      rpt::DataChunk c;
      while (op.GetData(*gs, ls, c)) got[t].push_back(c);
    });
  for (auto& th : src) th.join();
  std::vector<rpt::DataChunk> out;
  for (auto& g : got)
    for (auto& c : g) out.push_back(c);
  EXPECT(out.size() == op.ChunkCount(), "CREATE_BF %s: source re-emitted %zu of %zu chunks", names[0].c_str(), out.size(),
         op.ChunkCount());
  return out;
}

// The forward CREATE_BF's pushdown in the GPU mode (rpt_device = gpu, filter type 'all', scan targets found):
// SURVEY §8 a10. The BF stays out of the scan and its USE_BF probes on the device; min/max still go to the scan.
static bool forward_passthrough(const rpt::CreateBF& op, size_t col, const char* name) {
  int64_t mn = 0, mx = 0;
  const bool mm = op.MinMax(col, mn, mx);
  const rpt::PushdownPlan p = rpt::PlanPushdown(rpt::Device::kGpu, rpt::FilterType::kAll, /*is_forward_pass=*/true,
                                                /*has_targets=*/true, op.MaterializedRows(),
                                                op.GetBloomFilter(col)->IsEmpty(), mm);
  EXPECT(!p.use_bf_passthrough && p.bf_probed_in_use_bf && !p.push_bf && p.push_minmax == mm && !p.push_always_false,
         "%s: GPU-mode pushdown plan", name);
  const rpt::PushdownPlan c = rpt::PlanPushdown(rpt::Device::kCpu, rpt::FilterType::kAll, true, true,
                                                op.MaterializedRows(), op.GetBloomFilter(col)->IsEmpty(), mm);
  EXPECT(c.use_bf_passthrough && c.push_bf && !c.bf_probed_in_use_bf, "%s: the reference's (CPU) plan", name);
  return p.use_bf_passthrough;
}

int main(int argc, char** argv) {
  if (argc < 2) {
    fprintf(stderr, "usage: test_job_transfer DIR\n");
    return 2;
  }
  g_dir = argv[1];
  try {
    const int dev = 0;
    std::map<std::string, uint64_t> est;
    {
      std::ifstream f(g_dir + "/est.txt");
      std::string k;
      uint64_t v;
      while (f >> k >> v) est[k] = v;
    }
    Table mi = load_table("mi", {"movie_id", "info_type_id"});
    Table it = load_table("it", {"id"});
    Table t = load_table("t", {"id"});
    Table mc = load_table("mc", {"movie_id"});
    // ---- forward pass (leaves -> root) ----
    // level 2: mc -> t
    rpt::CreateBF c_mc(dev, est.at("f_mc"), {0}, /*sink_flush_rows=*/1 << 16);
    const std::vector<rpt::DataChunk> mc_src = create_bf(c_mc, {"f_mc"}, mc.chunks, 4);
    // level 1, smallest first: it -> mi, then t -> mi
    rpt::CreateBF c_it(dev, est.at("f_it"), {0});
    const std::vector<rpt::DataChunk> it_src = create_bf(c_it, {"f_it"}, it.chunks, 2);
    UseResult t_fwd;
    use_bf(dev, "t_fwd", {c_mc.GetBloomFilter(0)}, {0}, t.chunks, /*batch=*/false, t_fwd,
           forward_passthrough(c_mc, 0, "f_mc"));
    rpt::CreateBF c_t(dev, est.at("f_t"), {0}, 1 << 15);  // under-estimated: Finalize resizes + rehashes from HBM
    const std::vector<rpt::DataChunk> t_src = create_bf(c_t, {"f_t"}, t_fwd.chunks, 3);
    // mi (root): its two forward USE_BFs as one filter chain (AND), over the whole scan as a caching operator
    UseResult mi_fwd;
    const bool pt_it = forward_passthrough(c_it, 0, "f_it"), pt_t = forward_passthrough(c_t, 0, "f_t");
    use_bf(dev, "mi_fwd", {c_it.GetBloomFilter(0), c_t.GetBloomFilter(0)}, {1, 0}, mi.chunks, /*batch=*/true, mi_fwd,
           pt_it && pt_t);
    // ---- backward pass (root -> leaves) ----
    // mi's two CREATE_BFs stacked into one operator with two build columns
    rpt::CreateBF c_mi(dev, est.at("f_mi"), {1, 0}, 1 << 17);
    const std::vector<rpt::DataChunk> mi_src = create_bf(c_mi, {"f_mi_it", "f_mi_t"}, mi_fwd.chunks, 4);
    UseResult it_bwd, t_bwd, mc_bwd;
    use_bf(dev, "it_bwd", {c_mi.GetBloomFilter(0)}, {0}, it_src, /*batch=*/false, it_bwd);
    use_bf(dev, "t_bwd", {c_mi.GetBloomFilter(1)}, {0}, t_src, /*batch=*/true, t_bwd);
    rpt::CreateBF c_t2(dev, est.at("f_t2"), {0});
    const std::vector<rpt::DataChunk> t2_src = create_bf(c_t2, {"f_t2"}, t_bwd.chunks, 2);
    use_bf(dev, "mc_bwd", {c_t2.GetBloomFilter(0)}, {0}, mc_src, /*batch=*/true, mc_bwd);
    // the tables the joins read: mi after its forward USE_BFs (re-emitted by its CREATE_BF), it / t / mc after
    // their backward USE_BFs (t re-emitted by its backward CREATE_BF)
    std::vector<int64_t> mi_out, t_out;
    for (const auto& c : mi_src)
      for (size_t r = 0; r < c.count; r++) mi_out.push_back(row_id_at(c, r));
    for (const auto& c : t2_src)
      for (size_t r = 0; r < c.count; r++) t_out.push_back(row_id_at(c, r));
    write_file("final_mi.i64", mi_out);
    write_file("final_it.i64", it_bwd.ids);
    write_file("final_t.i64", t_out);
    write_file("final_mc.i64", mc_bwd.ids);
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
