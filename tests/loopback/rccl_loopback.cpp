// rccl_loopback.cpp — a loopback RCCL for tests (librccl_loopback.so): W ranks as host threads of ONE
// process on ONE device, so the product's multi-GPU OR all-reduce (rpt_bf_allreduce_or)
// runs its real W-rank choreography on a one-GPU box (RCCL itself refuses two ranks on one device).
// Test infrastructure only: handed to the test build of the library (csrc/rpt_gpu_testing.h); the
// product never loads it.
//
// Semantics (the subset rpt_bf_allreduce_or uses, rccl.h signatures):
//   ncclGetUniqueId / ncclCommInitRank   a "world" per id; init blocks until all nranks ranks joined
//   ncclGroupStart / ncclSend / ncclRecv / ncclGroupEnd
//       sends and receives are queued per thread; at the outermost GroupEnd every rank of the world
//       meets (barrier): (1) each send records a ready event on its stream and is posted on the
//       (src, dst) channel, (2) each receive takes the next send of its channel (FIFO, as RCCL pairs
//       p2p operations per peer in issue order), checks the byte count, waits on the sender's ready
//       event and copies device-to-device on the receiver's stream, recording a done event, (3) each
//       sender's stream waits on the done events of its sends (the buffer may be reused after).
//       No host synchronization: every dependency is a stream-event wait.
//   ncclAllReduce   int64/uint64 MIN / MAX / SUM, staged through the host (3 words in the product)
//   failure injection: rpt_loopback_fail_op(rank, k) makes the k-th send/recv call of that rank fail;
//       the failing rank's GroupEnd then aborts the world and every rank's pending GroupEnd fails.
#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <deque>
#include <map>
#include <mutex>
#include <vector>

namespace {

constexpr int kSuccess = 0, kUnhandledCudaError = 1, kInternalError = 3, kInvalidArgument = 4, kInvalidUsage = 5;
constexpr int kInt64 = 4, kUint64 = 5;                 // ncclDataType_t
constexpr int kSum = 0, kMax = 2, kMin = 3;            // ncclRedOp_t
constexpr auto kBarrierTimeout = std::chrono::seconds(120);

struct UniqueId {
  char internal[128];
};

// rccl.h ncclDataType_t: int8, uint8, int32, uint32, int64, uint64, float16, float32, float64, bfloat16
size_t dtype_bytes(int dt) {
  static const size_t bytes[] = {1, 1, 4, 4, 8, 8, 2, 4, 8, 2};
  return dt >= 0 && dt < 10 ? bytes[dt] : 0;
}

struct SendRec {
  const void* buf;
  size_t bytes;
  hipEvent_t ready = nullptr, done = nullptr;
};

struct World {
  int size = 0, joined = 0, live = 0;
  std::mutex mu;
  std::condition_variable cv;
  int arrived = 0;
  uint64_t gen = 0;
  bool aborted = false;
  std::map<std::pair<int, int>, std::deque<SendRec*>> chan;  // (src, dst) -> posted sends
  std::vector<hipEvent_t> retired;                           // destroyed when the world ends
  std::vector<std::vector<int64_t>> ar;                      // all-reduce contributions
  uint64_t groups = 0, bytes_copied = 0;
};

struct Comm {
  World* w;
  int rank, device;
  std::atomic<int> ops{0};
};

struct Op {
  bool send;
  Comm* c;
  void* buf;
  size_t bytes;
  int peer;
  hipStream_t stream;
  SendRec* rec = nullptr;
};

std::mutex g_mu;
std::map<uint64_t, World*> g_worlds;
std::atomic<uint64_t> g_next_id{1};
std::atomic<int> g_fail_rank{-1}, g_fail_op{-1};

thread_local int t_depth = 0;
thread_local bool t_err = false;
thread_local std::vector<Op> t_ops;

// All ranks of w meet; false on abort or timeout (the world is then aborted).
bool barrier(World* w, std::unique_lock<std::mutex>& lk) {
  if (w->aborted) return false;
  const uint64_t g = w->gen;
  if (++w->arrived == w->size) {
    w->arrived = 0;
    w->gen++;
    w->cv.notify_all();
    return true;
  }
  if (!w->cv.wait_for(lk, kBarrierTimeout, [&] { return w->gen != g || w->aborted; })) {
    w->aborted = true;
    w->cv.notify_all();
  }
  return w->gen != g;
}

void abort_world(World* w) {
  w->aborted = true;
  w->cv.notify_all();
}

int fail_injected(Comm* c) {
  const int k = c->ops.fetch_add(1);
  return c->rank == g_fail_rank.load() && k == g_fail_op.load();
}

int enqueue(bool send, const void* buf, size_t count, int dt, int peer, void* comm, hipStream_t stream) {
  Comm* c = static_cast<Comm*>(comm);
  if (!c || peer < 0 || peer >= c->w->size || dtype_bytes(dt) == 0 || (count && !buf)) {
    if (t_depth > 0) t_err = true;
    return kInvalidArgument;
  }
  if (fail_injected(c)) {
    if (t_depth > 0) t_err = true;
    return kInternalError;
  }
  t_ops.push_back(Op{send, c, const_cast<void*>(buf), count * dtype_bytes(dt), peer, stream});
  return kSuccess;
}

int run_group(std::vector<Op>& ops, bool err) {
  if (ops.empty()) return err ? kInternalError : kSuccess;
  World* w = ops[0].c->w;
  const int me = ops[0].c->rank;
  for (const Op& o : ops)
    if (o.c->w != w) return kInvalidUsage;  // one communicator per group in this loopback
  if (hipSetDevice(ops[0].c->device) != hipSuccess) return kUnhandledCudaError;
  std::unique_lock<std::mutex> lk(w->mu);
  if (err) {
    abort_world(w);
    return kInternalError;
  }
  // (1) post the sends
  for (Op& o : ops) {
    if (!o.send) continue;
    o.rec = new SendRec{o.buf, o.bytes};
    if (hipEventCreateWithFlags(&o.rec->ready, hipEventDisableTiming) != hipSuccess ||
        hipEventRecord(o.rec->ready, o.stream) != hipSuccess) {
      abort_world(w);
      return kUnhandledCudaError;
    }
    w->chan[{me, o.peer}].push_back(o.rec);
  }
  if (!barrier(w, lk)) return kInternalError;
  // (2) match the receives in issue order per peer
  int rc = kSuccess;
  for (Op& o : ops) {
    if (o.send) continue;
    auto& q = w->chan[{o.peer, me}];
    if (q.empty() || q.front()->bytes != o.bytes) {
      rc = kInvalidUsage;  // unmatched receive or size mismatch
      abort_world(w);
      break;
    }
    SendRec* r = q.front();
    q.pop_front();
    hipEvent_t done = nullptr;
    if (hipStreamWaitEvent(o.stream, r->ready, 0) != hipSuccess ||
        (o.bytes && hipMemcpyAsync(o.buf, r->buf, o.bytes, hipMemcpyDeviceToDevice, o.stream) != hipSuccess) ||
        hipEventCreateWithFlags(&done, hipEventDisableTiming) != hipSuccess || hipEventRecord(done, o.stream) != hipSuccess) {
      rc = kUnhandledCudaError;
      abort_world(w);
      break;
    }
    r->done = done;
    w->bytes_copied += o.bytes;
  }
  if (!barrier(w, lk)) return rc != kSuccess ? rc : kInternalError;
  // (3) each send's stream waits for its receiver's copy
  for (Op& o : ops) {
    if (!o.send) continue;
    if (!o.rec->done || hipStreamWaitEvent(o.stream, o.rec->done, 0) != hipSuccess) rc = kUnhandledCudaError;
    w->retired.push_back(o.rec->ready);
    if (o.rec->done) w->retired.push_back(o.rec->done);
    delete o.rec;
  }
  if (me == 0) w->groups++;
  if (rc != kSuccess) abort_world(w);
  return rc;
}

}  // namespace

extern "C" {

const char* ncclGetErrorString(int r) {
  switch (r) {
    case kSuccess: return "no error (loopback)";
    case kUnhandledCudaError: return "unhandled HIP error (loopback)";
    case kInternalError: return "internal error (loopback: injected failure or aborted world)";
    case kInvalidArgument: return "invalid argument (loopback)";
    case kInvalidUsage: return "invalid usage (loopback: unmatched or mismatched send/recv)";
    default: return "unknown (loopback)";
  }
}

int ncclGetUniqueId(UniqueId* id) {
  if (!id) return kInvalidArgument;
  std::memset(id->internal, 0, sizeof id->internal);
  const uint64_t v = g_next_id.fetch_add(1);
  std::memcpy(id->internal, "rptloop", 7);
  std::memcpy(id->internal + 8, &v, sizeof v);
  return kSuccess;
}

int ncclCommInitRank(void** comm, int nranks, UniqueId id, int rank) {
  if (!comm || nranks < 1 || rank < 0 || rank >= nranks || std::memcmp(id.internal, "rptloop", 7) != 0)
    return kInvalidArgument;
  uint64_t key = 0;
  std::memcpy(&key, id.internal + 8, sizeof key);
  World* w = nullptr;
  {
    std::lock_guard<std::mutex> g(g_mu);
    World*& slot = g_worlds[key];
    if (!slot) {
      slot = new World();
      slot->size = nranks;
      slot->ar.resize(nranks);
    }
    w = slot;
  }
  if (w->size != nranks) return kInvalidUsage;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return kUnhandledCudaError;
  auto* c = new Comm{w, rank, dev};
  std::unique_lock<std::mutex> lk(w->mu);
  w->joined++;
  w->live++;
  if (!barrier(w, lk)) {  // collective: every rank joins before any returns
    w->live--;
    delete c;
    return kInternalError;
  }
  *comm = c;
  return kSuccess;
}

int ncclCommDestroy(void* comm) {
  Comm* c = static_cast<Comm*>(comm);
  if (!c) return kInvalidArgument;
  World* w = c->w;
  bool last = false;
  {
    std::lock_guard<std::mutex> lk(w->mu);
    last = --w->live == 0;
  }
  if (last) {
    (void)hipSetDevice(c->device);
    (void)hipDeviceSynchronize();  // every retired event has completed
    for (hipEvent_t e : w->retired) (void)hipEventDestroy(e);
    for (auto& kv : w->chan)
      for (SendRec* r : kv.second) {
        if (r->ready) (void)hipEventDestroy(r->ready);
        delete r;
      }
    std::lock_guard<std::mutex> g(g_mu);
    for (auto it = g_worlds.begin(); it != g_worlds.end(); ++it)
      if (it->second == w) {
        g_worlds.erase(it);
        break;
      }
    delete w;
  }
  delete c;
  return kSuccess;
}

int ncclCommCount(void* comm, int* count) {
  if (!comm || !count) return kInvalidArgument;
  *count = static_cast<Comm*>(comm)->w->size;
  return kSuccess;
}

int ncclCommUserRank(void* comm, int* rank) {
  if (!comm || !rank) return kInvalidArgument;
  *rank = static_cast<Comm*>(comm)->rank;
  return kSuccess;
}

int ncclGroupStart() {
  if (t_depth++ == 0) {
    t_ops.clear();
    t_err = false;
  }
  return kSuccess;
}

int ncclGroupEnd() {
  if (t_depth == 0) return kInvalidUsage;
  if (--t_depth > 0) return kSuccess;
  std::vector<Op> ops;
  ops.swap(t_ops);
  const bool err = t_err;
  t_err = false;
  return run_group(ops, err);
}

int ncclSend(const void* buf, size_t count, int dt, int peer, void* comm, hipStream_t stream) {
  if (t_depth > 0) return enqueue(true, buf, count, dt, peer, comm, stream);
  ncclGroupStart();
  const int rc = enqueue(true, buf, count, dt, peer, comm, stream);
  const int rc2 = ncclGroupEnd();
  return rc != kSuccess ? rc : rc2;
}

int ncclRecv(void* buf, size_t count, int dt, int peer, void* comm, hipStream_t stream) {
  if (t_depth > 0) return enqueue(false, buf, count, dt, peer, comm, stream);
  ncclGroupStart();
  const int rc = enqueue(false, buf, count, dt, peer, comm, stream);
  const int rc2 = ncclGroupEnd();
  return rc != kSuccess ? rc : rc2;
}

int ncclAllReduce(const void* sendbuf, void* recvbuf, size_t count, int dt, int op, void* comm, hipStream_t stream) {
  Comm* c = static_cast<Comm*>(comm);
  if (!c || (dt != kInt64 && dt != kUint64) || (op != kMin && op != kMax && op != kSum) || t_depth > 0)
    return kInvalidArgument;
  World* w = c->w;
  if (hipSetDevice(c->device) != hipSuccess) return kUnhandledCudaError;
  std::vector<int64_t> mine(count);
  if (hipStreamSynchronize(stream) != hipSuccess ||
      (count && hipMemcpy(mine.data(), sendbuf, count * 8, hipMemcpyDeviceToHost) != hipSuccess))
    return kUnhandledCudaError;
  auto* out = new std::vector<int64_t>(count);  // alive until the copy below completes
  {
    std::unique_lock<std::mutex> lk(w->mu);
    w->ar[c->rank] = mine;
    if (!barrier(w, lk)) {
      delete out;
      return kInternalError;
    }
    for (size_t i = 0; i < count; i++) {
      int64_t a = w->ar[0][i];
      for (int r = 1; r < w->size; r++) {
        const int64_t b = w->ar[r][i];
        if (op == kSum) a = static_cast<int64_t>(static_cast<uint64_t>(a) + static_cast<uint64_t>(b));
        else if (dt == kInt64) a = op == kMin ? std::min(a, b) : std::max(a, b);
        else a = static_cast<int64_t>(op == kMin ? std::min<uint64_t>(a, b) : std::max<uint64_t>(a, b));
      }
      (*out)[i] = a;
    }
    if (!barrier(w, lk)) {  // every rank has read the contributions before any is overwritten
      delete out;
      return kInternalError;
    }
  }
  int rc = kSuccess;
  if (count && (hipMemcpyAsync(recvbuf, out->data(), count * 8, hipMemcpyHostToDevice, stream) != hipSuccess ||
                hipStreamSynchronize(stream) != hipSuccess))
    rc = kUnhandledCudaError;
  delete out;
  return rc;
}

// ---- test controls ----------------------------------------------------------------------------------
// The k-th send/recv call (0-based, counted per communicator) of rank `rank` fails; (-1, -1) disarms.
void rpt_loopback_fail_op(int rank, int k) {
  g_fail_op.store(k);
  g_fail_rank.store(rank);
}
// Group nesting depth of the calling thread (0 once every group is closed).
int rpt_loopback_group_depth() { return t_depth; }
// Grouped exchanges completed and bytes copied by the world of `comm`.
int rpt_loopback_stats(void* comm, uint64_t* groups, uint64_t* bytes) {
  Comm* c = static_cast<Comm*>(comm);
  if (!c || !groups || !bytes) return kInvalidArgument;
  std::lock_guard<std::mutex> lk(c->w->mu);
  *groups = c->w->groups;
  *bytes = c->w->bytes_copied;
  return kSuccess;
}

}  // extern "C"
