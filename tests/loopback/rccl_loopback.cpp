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
//   ncclCommInitRankConfig   config->blocking == 0 makes a NON-BLOCKING communicator: init, ncclGroupEnd and
//       ncclAllReduce do their work as above but return ncclInProgress, and ncclCommGetAsyncError reports
//       ncclInProgress for two more polls before the call's result (so a caller's polling path runs)
//   ncclCommFinalize   as a non-blocking call (above) on a non-blocking communicator; success at once otherwise
//   ncclCommAbort / ncclCommGetAsyncError   rank-local, as in RCCL: an abort frees that rank's communicator and
//       releases only that rank's blocked streams (below); the asynchronous error is the world's (0 unless a
//       silent peer was set to report)
//   failure injection:
//     rpt_loopback_fail_op(rank, k)   the k-th send/recv call of that rank fails; the failing rank's GroupEnd
//       aborts the world and every rank's pending GroupEnd fails (an error RCCL propagated);
//     rpt_loopback_silent_peer(rank, k, report)   the k-th send/recv call of that rank fails and its group
//       closes WITHOUT telling the world: as a peer that died mid-merge. The other ranks' GroupEnd (and
//       AllReduce) calls then return success, as RCCL's do, and block their streams instead (a host function
//       on the stream that waits until that rank aborts its communicator; 60 s safety bound), so only a
//       bounded wait in the caller ends them. report != 0: ncclCommGetAsyncError reports ncclRemoteError
//       once the peer is gone.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <vector>

namespace {

constexpr int kSuccess = 0, kUnhandledCudaError = 1, kInternalError = 3, kInvalidArgument = 4, kInvalidUsage = 5,
              kRemoteError = 6, kInProgress = 7;
constexpr int kNonblockingPolls = 2;  // ncclCommGetAsyncError answers ncclInProgress this many times first
constexpr int kInt64 = 4, kUint64 = 5;                 // ncclDataType_t
constexpr int kSum = 0, kMax = 2, kMin = 3;            // ncclRedOp_t
constexpr auto kBarrierTimeout = std::chrono::seconds(120);
constexpr auto kBlockedStreamBound = std::chrono::seconds(60);  // safety bound of a silent-peer stream block

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
  bool aborted = false;           // an error propagated to every rank (rpt_loopback_fail_op)
  bool dead = false;              // a silent peer is gone (rpt_loopback_silent_peer): groups never match
  int async_err = kSuccess;       // what ncclCommGetAsyncError reports
  std::vector<bool> rank_aborted;  // ncclCommAbort per rank: releases that rank's blocked streams
  std::map<std::pair<int, int>, std::deque<SendRec*>> chan;  // (src, dst) -> posted sends
  std::vector<hipEvent_t> retired;                           // destroyed when the world ends
  std::vector<std::vector<int64_t>> ar;                      // all-reduce contributions
  uint64_t groups = 0, bytes_copied = 0;
};

struct Comm {
  std::shared_ptr<World> w;
  int rank, device;
  std::atomic<int> ops{0};
  bool nonblocking = false;
  std::atomic<int> polls{0};           // non-blocking: ncclInProgress answers left for the pending call
  std::atomic<int> result{kSuccess};   // non-blocking: the pending call's result
};

// A non-blocking communicator's call has done its work: report ncclInProgress now and `rc` after the polls.
std::atomic<int> g_stuck{0};  // rpt_loopback_stuck: non-blocking calls never leave ncclInProgress
int complete(Comm* c, int rc) {
  if (!c || !c->nonblocking) return rc;
  c->result.store(rc);
  c->polls.store(g_stuck.load() ? (1 << 30) : kNonblockingPolls);
  return kInProgress;
}

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
std::map<uint64_t, std::shared_ptr<World>> g_worlds;
std::atomic<uint64_t> g_next_id{1};
std::atomic<int> g_fail_rank{-1}, g_fail_op{-1};
std::atomic<int> g_silent{0}, g_silent_report{0};  // the armed failure is a silent peer (and reports it)

thread_local int t_depth = 0;
thread_local bool t_err = false;
thread_local std::vector<Op> t_ops;
thread_local Comm* t_err_comm = nullptr;  // the communicator of the group's failed call

// All ranks of w meet; false on abort, timeout (the world is then aborted) or a dead peer (w->dead).
bool barrier(World* w, std::unique_lock<std::mutex>& lk) {
  if (w->aborted || w->dead) return false;
  const uint64_t g = w->gen;
  if (++w->arrived == w->size) {
    w->arrived = 0;
    w->gen++;
    w->cv.notify_all();
    return true;
  }
  if (!w->cv.wait_for(lk, kBarrierTimeout, [&] { return w->gen != g || w->aborted || w->dead; })) {
    w->aborted = true;
    w->cv.notify_all();
  }
  return w->gen != g;
}

// A silent peer's group never completes: block `stream` (as RCCL's kernels would) until rank `rank` aborts
// its communicator, or the safety bound passes.
struct BlockArg {
  std::shared_ptr<World> w;
  int rank;
};
void block_host_fn(void* p) {
  std::unique_ptr<BlockArg> a(static_cast<BlockArg*>(p));
  std::unique_lock<std::mutex> lk(a->w->mu);
  a->w->cv.wait_for(lk, kBlockedStreamBound, [&] { return a->w->rank_aborted[a->rank]; });
}
int block_stream(const std::shared_ptr<World>& w, int rank, hipStream_t stream) {
  auto* a = new BlockArg{w, rank};
  if (hipLaunchHostFunc(stream, block_host_fn, a) != hipSuccess) {
    delete a;
    return kUnhandledCudaError;
  }
  return kSuccess;
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
    if (t_depth > 0) {
      t_err = true;
      t_err_comm = c;
    }
    return kInternalError;
  }
  t_ops.push_back(Op{send, c, const_cast<void*>(buf), count * dtype_bytes(dt), peer, stream});
  return kSuccess;
}

// A group of a world whose silent peer is gone: "succeeds" on the host, every stream of it blocks.
int dead_group(const std::shared_ptr<World>& w, int me, std::vector<Op>& ops) {
  int rc = kSuccess;
  std::vector<hipStream_t> seen;
  for (Op& o : ops) {
    if (std::find(seen.begin(), seen.end(), o.stream) != seen.end()) continue;
    seen.push_back(o.stream);
    if (block_stream(w, me, o.stream) != kSuccess) rc = kUnhandledCudaError;
  }
  return rc;
}

int run_group(std::vector<Op>& ops, bool err, Comm* err_comm) {
  Comm* c0 = !ops.empty() ? ops[0].c : err_comm;
  if (!c0) return err ? kInternalError : kSuccess;
  std::shared_ptr<World> wp = c0->w;
  World* w = wp.get();
  const int me = c0->rank;
  for (const Op& o : ops)
    if (o.c->w != wp) return kInvalidUsage;  // one communicator per group in this loopback
  if (hipSetDevice(c0->device) != hipSuccess) return kUnhandledCudaError;
  std::unique_lock<std::mutex> lk(w->mu);
  if (err) {  // the failing rank's group closes
    if (g_silent.load()) {  // the peer "dies": nobody is told
      w->dead = true;
      if (g_silent_report.load()) w->async_err = kRemoteError;
      w->cv.notify_all();
    } else {
      abort_world(w);
    }
    return kInternalError;
  }
  if (w->dead) {
    lk.unlock();
    return dead_group(wp, me, ops);
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
  if (!barrier(w, lk)) {
    if (!w->dead || w->aborted) return kInternalError;
    lk.unlock();
    return dead_group(wp, me, ops);
  }
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
    case kRemoteError: return "remote error (loopback: a silent peer is gone)";
    case kInProgress: return "in progress (loopback: non-blocking communicator)";
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

static int init_rank(void** comm, int nranks, UniqueId id, int rank, bool nonblocking) {
  if (!comm || nranks < 1 || rank < 0 || rank >= nranks || std::memcmp(id.internal, "rptloop", 7) != 0)
    return kInvalidArgument;
  uint64_t key = 0;
  std::memcpy(&key, id.internal + 8, sizeof key);
  std::shared_ptr<World> w;
  {
    std::lock_guard<std::mutex> g(g_mu);
    std::shared_ptr<World>& slot = g_worlds[key];
    if (!slot) {
      slot = std::make_shared<World>();
      slot->size = nranks;
      slot->ar.resize(nranks);
      slot->rank_aborted.assign(nranks, false);
    }
    w = slot;
  }
  if (w->size != nranks) return kInvalidUsage;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return kUnhandledCudaError;
  auto* c = new Comm{w, rank, dev};
  c->nonblocking = nonblocking;
  std::unique_lock<std::mutex> lk(w->mu);
  w->joined++;
  w->live++;
  if (!barrier(w.get(), lk)) {  // collective: every rank joins before any returns
    w->live--;
    delete c;
    return kInternalError;
  }
  *comm = c;
  return complete(c, kSuccess);
}

// rccl.h ncclConfig_t, as far as read here
struct ConfigHead {
  size_t size;
  unsigned int magic, version;
  int blocking;
};

int ncclCommInitRank(void** comm, int nranks, UniqueId id, int rank) { return init_rank(comm, nranks, id, rank, false); }

int ncclCommInitRankConfig(void** comm, int nranks, UniqueId id, int rank, const ConfigHead* config) {
  return init_rank(comm, nranks, id, rank, config != nullptr && config->blocking == 0);
}

// Frees the communicator; the last one of its world releases the world's events (the World itself lives
// on while a blocked stream's host function still holds it).
static int release_comm(Comm* c, bool abort) {
  std::shared_ptr<World> w = c->w;
  bool last = false;
  {
    std::lock_guard<std::mutex> lk(w->mu);
    if (abort) {
      w->rank_aborted[c->rank] = true;  // this rank's blocked streams resume
      w->cv.notify_all();
    }
    last = --w->live == 0;
  }
  if (last) {
    (void)hipSetDevice(c->device);
    (void)hipDeviceSynchronize();  // every retired event has completed (every rank has aborted or destroyed)
    for (hipEvent_t e : w->retired) (void)hipEventDestroy(e);
    w->retired.clear();
    for (auto& kv : w->chan)
      for (SendRec* r : kv.second) {
        if (r->ready) (void)hipEventDestroy(r->ready);
        delete r;
      }
    w->chan.clear();
    std::lock_guard<std::mutex> g(g_mu);
    for (auto it = g_worlds.begin(); it != g_worlds.end(); ++it)
      if (it->second == w) {
        g_worlds.erase(it);
        break;
      }
  }
  delete c;
  return kSuccess;
}

int ncclCommDestroy(void* comm) {
  Comm* c = static_cast<Comm*>(comm);
  if (!c) return kInvalidArgument;
  return release_comm(c, false);
}

// Finalize before destroy (non-blocking communicators: reports ncclInProgress for two polls, then success,
// or forever under rpt_loopback_stuck). Counted so a test can see that rpt_rccl_comm_destroy finalized one.
static std::atomic<int> g_finalized{0};
int ncclCommFinalize(void* comm) {
  Comm* c = static_cast<Comm*>(comm);
  if (!c) return kInvalidArgument;
  g_finalized.fetch_add(1);
  return complete(c, kSuccess);
}

int rpt_loopback_finalize_count() { return g_finalized.load(); }

// Rank-local, as RCCL's: frees this rank's communicator and releases this rank's blocked streams only.
int ncclCommAbort(void* comm) {
  Comm* c = static_cast<Comm*>(comm);
  if (!c) return kInvalidArgument;
  return release_comm(c, true);
}

int ncclCommGetAsyncError(void* comm, int* async_error) {
  Comm* c = static_cast<Comm*>(comm);
  if (!c || !async_error) return kInvalidArgument;
  if (c->nonblocking && c->polls.load() > 0) {
    c->polls.fetch_sub(1);
    *async_error = kInProgress;
    return kSuccess;
  }
  std::lock_guard<std::mutex> lk(c->w->mu);
  *async_error = c->w->async_err != kSuccess ? c->w->async_err : (c->nonblocking ? c->result.load() : kSuccess);
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
    t_err_comm = nullptr;
  }
  return kSuccess;
}

int ncclGroupEnd() {
  if (t_depth == 0) return kInvalidUsage;
  if (--t_depth > 0) return kSuccess;
  std::vector<Op> ops;
  ops.swap(t_ops);
  const bool err = t_err;
  Comm* err_comm = t_err_comm;
  t_err = false;
  t_err_comm = nullptr;
  Comm* c0 = !ops.empty() ? ops[0].c : err_comm;
  return complete(c0, run_group(ops, err, err_comm));
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

static int all_reduce_impl(const void* sendbuf, void* recvbuf, size_t count, int dt, int op, void* comm, hipStream_t stream) {
  Comm* c = static_cast<Comm*>(comm);
  if (!c || (dt != kInt64 && dt != kUint64) || (op != kMin && op != kMax && op != kSum) || t_depth > 0)
    return kInvalidArgument;
  World* w = c->w.get();
  if (hipSetDevice(c->device) != hipSuccess) return kUnhandledCudaError;
  {
    std::lock_guard<std::mutex> lk(w->mu);
    if (w->dead) return block_stream(c->w, c->rank, stream);  // never completes, as RCCL's would not
  }
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
      if (w->dead && !w->aborted) {
        lk.unlock();
        return block_stream(c->w, c->rank, stream);
      }
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

int ncclAllReduce(const void* sendbuf, void* recvbuf, size_t count, int dt, int op, void* comm, hipStream_t stream) {
  const int rc = all_reduce_impl(sendbuf, recvbuf, count, dt, op, comm, stream);
  return rc == kInvalidArgument ? rc : complete(static_cast<Comm*>(comm), rc);
}

// ---- test controls ----------------------------------------------------------------------------------
// The k-th send/recv call (0-based, counted per communicator) of rank `rank` fails; (-1, -1) disarms.
void rpt_loopback_fail_op(int rank, int k) {
  g_silent.store(0);
  g_silent_report.store(0);
  g_fail_op.store(k);
  g_fail_rank.store(rank);
}
// The k-th send/recv call of rank `rank` fails and that rank goes silent (a peer dying mid-merge: see the
// header); report != 0 makes ncclCommGetAsyncError return ncclRemoteError afterwards. (-1, -1, 0) disarms.
void rpt_loopback_silent_peer(int rank, int k, int report) {
  g_silent.store(rank >= 0 ? 1 : 0);
  g_silent_report.store(report != 0 ? 1 : 0);
  g_fail_op.store(k);
  g_fail_rank.store(rank);
}
// on != 0: every later call on a non-blocking communicator stays ncclInProgress (a call that never completes).
void rpt_loopback_stuck(int on) { g_stuck.store(on != 0); }
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
