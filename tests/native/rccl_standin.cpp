// rccl_standin.cpp -- TEST INFRASTRUCTURE: an in-process stand-in for the twelve
// RCCL entry points libgossip_hip.so calls (nm -u of the library), so that the
// vertex partition's real RCCL path -- exchange_rccl in csrc/partition.hip: the
// count all-gather, the grouped ncclSend / ncclRecv of the boundary entries,
// the unpack, the counters' all-reduce -- runs with P > 1 ranks on a one-GPU
// box.  RCCL itself refuses two ranks on one device ("Duplicate GPU
// detected"), so without this the P > 1 branch would first execute on an
// 8-GPU node.
//
// Model: the P ranks are P threads of one process driving P contexts on one
// device (tests/rccl_standin_driver.py).  A communicator is a rank of a
// "world" named by the unique id.  Calls between ncclGroupStart /
// ncclGroupEnd are recorded and run at the outermost ncclGroupEnd; the k-th
// receive from q matches q's k-th send to this rank inside one group, as in
// RCCL.  Barrier waits time out (ncclSystemError) instead of hanging a test
// when a rank fails.  Two modes (GP_STANDIN_ASYNC in the environment):
//   sync (default)  every call first synchronizes the caller's stream (so the
//                   inputs the engine enqueued are in memory), then runs the
//                   collective with the other ranks' threads and waits for it;
//   async (=1)      nothing is synchronized: like RCCL, a call only enqueues.
//                   The copies run on a side stream of each rank that waits on
//                   an event recorded on the caller's stream at the call, and
//                   the caller's stream waits on the copies' events (outputs
//                   landed, send buffers free) before its next work.  An engine
//                   that wrote an input after the call, or read an output
//                   without ordering on its stream, sees stale data here.
// Fault injection (GP_STANDIN_CORRUPT=rank:k): rank `rank` overwrites the
// first 8 bytes of its k-th non-empty receive (counted from 0 over the
// communicator's life) with ones, after the copy -- the engine's exchange check
// must then fail the round on every rank.
//
// Built by build_lib.build_standin() into _build/libgossip_hip_rccl_standin.so
// together with the engine's own objects; the product library links real RCCL.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <atomic>
#include <chrono>
#include <cstdlib>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <deque>
#include <map>
#include <mutex>
#include <string>
#include <vector>

namespace {

enum OpKind { OP_ALLREDUCE, OP_ALLGATHER, OP_SEND, OP_RECV };

struct Op {
  OpKind kind;
  const void* src;
  void* dst;
  size_t count;   // elements (all-gather: per rank)
  size_t esize;
  int peer;
  hipStream_t stream;
};

struct SendRec {   // the sender's side of a posted send
  char done = 0;                  // the receiver took it
  hipEvent_t copied = nullptr;    // async: recorded on the receiver's side stream after its copy
};
struct Mail {   // a posted send: the receiver copies from src and sets rec->done
  const void* src;
  size_t bytes;
  SendRec* rec;
  hipEvent_t ready;               // async: the sender's stream reached the send
};

struct World {
  int n = 0;
  int joined = 0;
  std::mutex mu;
  std::condition_variable cv;
  uint64_t gen = 0;      // barrier generation
  int arrived = 0;
  bool broken = false;   // a wait timed out: every later wait fails at once
  std::vector<std::vector<Op>*> posted;   // each rank's collectives of the current call
  std::vector<hipEvent_t> ev;             // async: each rank's published event of the current phase
  std::vector<void*> stage;               // async: each rank's staged all-reduce input
  std::map<std::pair<int, int>, std::deque<Mail>> box;   // (from, to) -> sends in posting order
};

std::mutex g_worlds_mu;
std::map<std::string, World*> g_worlds;
std::atomic<uint64_t> g_id_counter{1};

struct RankState {
  int depth = 0;
  std::vector<Op> ops;
};
thread_local RankState t_rank;

}  // namespace

struct ncclComm {
  World* w;
  int rank;
  hipStream_t side = nullptr;   // async mode: the stream the copies run on
  void* stage = nullptr;        // async mode: staged all-reduce input
  size_t stage_bytes = 0;
  long recvs = 0;               // non-empty receives so far (fault injection)
};

namespace {

constexpr int kBarrierTimeoutS = 120;

bool async_mode() {
  static const bool on = [] {
    const char* e = std::getenv("GP_STANDIN_ASYNC");
    return e && e[0] == '1';
  }();
  return on;
}

// GP_STANDIN_CORRUPT=rank:k -> (rank, k); (-1, -1) when unset
std::pair<int, long> corrupt_target() {
  static const std::pair<int, long> t = [] {
    const char* e = std::getenv("GP_STANDIN_CORRUPT");
    int r = -1;
    long k = -1;
    if (e && std::sscanf(e, "%d:%ld", &r, &k) != 2) r = -1, k = -1;
    return std::make_pair(r, k);
  }();
  return t;
}

// after a receive's copy (on stream s): count it, and overwrite it if it is the
// fault-injection target
bool after_recv(ncclComm* comm, void* dst, size_t bytes, hipStream_t s) {
  if (bytes == 0) return true;
  const auto t = corrupt_target();
  const long k = comm->recvs++;
  if (t.first != comm->rank || t.second != k) return true;
  return hipMemsetAsync(dst, 0xFF, std::min<size_t>(bytes, 8), s) == hipSuccess;
}

constexpr int kMaxRanks = 64;
struct Stages { const uint64_t* p[kMaxRanks]; };   // (by value: no pointer table to allocate)
__global__ void k_sum_u64(uint64_t* dst, Stages src, int n, size_t count) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < count; i += (size_t)gridDim.x * blockDim.x) {
    uint64_t t = 0;
    for (int r = 0; r < n; ++r) t += src.p[r][i];
    dst[i] = t;
  }
}

bool barrier(World* w) {
  std::unique_lock<std::mutex> lk(w->mu);
  if (w->broken) return false;
  const uint64_t g = w->gen;
  if (++w->arrived == w->n) {
    w->arrived = 0;
    ++w->gen;
    w->cv.notify_all();
    return true;
  }
  const bool ok = w->cv.wait_for(lk, std::chrono::seconds(kBarrierTimeoutS),
                                 [&] { return w->gen != g || w->broken; });
  if (!ok || w->broken) {
    w->broken = true;
    w->cv.notify_all();
    return false;
  }
  return true;
}

size_t esize_of(ncclDataType_t t) {
  switch (t) {
    case ncclInt8: case ncclUint8: return 1;
    case ncclInt32: case ncclUint32: case ncclFloat32: return 4;
    case ncclInt64: case ncclUint64: case ncclFloat64: return 8;
    default: return 0;
  }
}

// every copy runs on the calling rank's own stream and is waited for: a plain
// hipMemcpy does not order against the engine's non-blocking streams (device-to-
// device and pageable host-to-device copies may return before the data lands),
// so its next kernel could read a receive buffer the copy has not filled yet
bool copy(void* dst, const void* src, size_t bytes, hipStream_t s) {
  if (bytes == 0) return true;
  return hipMemcpyAsync(dst, src, bytes, hipMemcpyDefault, s) == hipSuccess && hipStreamSynchronize(s) == hipSuccess;
}

bool sync_streams(const std::vector<Op>& ops) {
  for (const Op& o : ops)
    if (hipStreamSynchronize(o.stream) != hipSuccess) return false;
  return true;
}

// wait on w->cv for pred, with the stand-in's timeout; false: timed out
template <class Pred>
bool wait_for(World* w, std::unique_lock<std::mutex>& lk, Pred pred) {
  const bool ok = w->cv.wait_for(lk, std::chrono::seconds(kBarrierTimeoutS), [&] { return pred() || w->broken; });
  if (!ok || w->broken) {
    w->broken = true;
    w->cv.notify_all();
    return false;
  }
  return true;
}

// collectives: every rank calls the same sequence; barriers order every
// rank's reads of the inputs before any rank writes its output
ncclResult_t run_collectives(ncclComm* comm, std::vector<Op>& coll) {
  World* w = comm->w;
  const int me = comm->rank;
  {
    std::lock_guard<std::mutex> lk(w->mu);
    w->posted[(size_t)me] = &coll;
  }
  if (!barrier(w)) return ncclSystemError;
  ncclResult_t rc = ncclSuccess;
  for (int r = 0; r < w->n; ++r) {
    const std::vector<Op>& x = *w->posted[(size_t)r];
    if (x.size() != coll.size()) rc = ncclInvalidUsage;
    for (size_t k = 0; k < x.size() && k < coll.size(); ++k)
      if (x[k].kind != coll[k].kind || x[k].count != coll[k].count || x[k].esize != coll[k].esize)
        rc = ncclInvalidUsage;
  }
  for (size_t ci = 0; ci < coll.size(); ++ci) {
    const Op& o = coll[ci];
    std::vector<std::vector<uint8_t>> in((size_t)w->n);
    if (rc == ncclSuccess)
      for (int r = 0; r < w->n; ++r) {
        const Op& x = (*w->posted[(size_t)r])[ci];
        in[(size_t)r].resize(x.count * x.esize);
        if (!copy(in[(size_t)r].data(), x.src, x.count * x.esize, o.stream)) rc = ncclSystemError;
      }
    if (!barrier(w)) return ncclSystemError;
    if (rc == ncclSuccess && o.count) {
      if (o.kind == OP_ALLGATHER) {
        for (int r = 0; r < w->n; ++r)
          if (!copy(static_cast<uint8_t*>(o.dst) + (size_t)r * o.count * o.esize, in[(size_t)r].data(),
                    o.count * o.esize, o.stream))
            rc = ncclSystemError;
      } else {   // all-reduce: sum of u64 (the only reduction the engine asks for)
        std::vector<uint64_t> acc(o.count, 0);
        for (int r = 0; r < w->n; ++r) {
          const uint64_t* x = reinterpret_cast<const uint64_t*>(in[(size_t)r].data());
          for (size_t i = 0; i < o.count; ++i) acc[i] += x[i];
        }
        if (!copy(o.dst, acc.data(), o.count * 8, o.stream)) rc = ncclSystemError;
      }
    }
    if (!barrier(w)) return ncclSystemError;
  }
  {
    std::lock_guard<std::mutex> lk(w->mu);
    w->posted[(size_t)me] = nullptr;
  }
  return rc;
}

// point-to-point: sends are posted to (me, q) mailboxes, the k-th receive from
// q takes q's k-th send to this rank; a rank returns once its own sends were
// copied out (its buffers may be reused right after, as with RCCL's stream
// order).  Ranks without sends or receives in a group do not take part.
ncclResult_t run_p2p(ncclComm* comm, const std::vector<Op>& p2p) {
  World* w = comm->w;
  const int me = comm->rank;
  std::deque<SendRec> recs;   // (stable addresses)
  {
    std::lock_guard<std::mutex> lk(w->mu);
    for (const Op& o : p2p)
      if (o.kind == OP_SEND) {
        recs.emplace_back();
        w->box[{me, o.peer}].push_back(Mail{o.src, o.count * o.esize, &recs.back(), nullptr});
      }
  }
  w->cv.notify_all();
  ncclResult_t rc = ncclSuccess;
  for (const Op& o : p2p) {
    if (o.kind != OP_RECV) continue;
    Mail m{};
    {
      std::unique_lock<std::mutex> lk(w->mu);
      auto& q = w->box[{o.peer, me}];
      if (!wait_for(w, lk, [&] { return !q.empty(); })) return ncclSystemError;
      m = q.front();
      q.pop_front();
    }
    bool ok = m.bytes == o.count * o.esize;
    if (ok && m.bytes) ok = copy(o.dst, m.src, m.bytes, o.stream) && after_recv(comm, o.dst, m.bytes, o.stream) &&
                            hipStreamSynchronize(o.stream) == hipSuccess;
    if (!ok) rc = m.bytes == o.count * o.esize ? ncclSystemError : ncclInvalidUsage;
    {
      std::lock_guard<std::mutex> lk(w->mu);
      m.rec->done = 1;
    }
    w->cv.notify_all();
  }
  {
    std::unique_lock<std::mutex> lk(w->mu);
    if (!wait_for(w, lk, [&] {
          for (const SendRec& r : recs)
            if (!r.done) return false;
          return true;
        }))
      return ncclSystemError;
  }
  return rc;
}

// ---------------------------------------------------------------------------
// async mode: the same rendezvous of the host threads, but every copy is
// enqueued on the rank's side stream behind the events of the streams whose
// data it moves, and the caller's stream waits for the copies' events

hipEvent_t new_event() {
  hipEvent_t e = nullptr;
  if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return nullptr;
  return e;
}

ncclResult_t run_collectives_async(ncclComm* comm, std::vector<Op>& coll, hipEvent_t ready, hipStream_t caller) {
  World* w = comm->w;
  const int me = comm->rank;
  const int n = w->n;
  {
    std::lock_guard<std::mutex> lk(w->mu);
    w->posted[(size_t)me] = &coll;
    w->ev[(size_t)me] = ready;
  }
  if (!barrier(w)) return ncclSystemError;
  ncclResult_t rc = ncclSuccess;
  for (int r = 0; r < n; ++r) {
    const std::vector<Op>& x = *w->posted[(size_t)r];
    if (x.size() != coll.size()) rc = ncclInvalidUsage;
    for (size_t k = 0; k < x.size() && k < coll.size(); ++k)
      if (x[k].kind != coll[k].kind || x[k].count != coll[k].count || x[k].esize != coll[k].esize)
        rc = ncclInvalidUsage;
  }
  std::vector<hipEvent_t> ready_all(w->ev);   // every rank's inputs are complete behind these
  if (!barrier(w)) return ncclSystemError;    // (w->ev is reused below)
  for (int r = 0; r < n && rc == ncclSuccess; ++r)
    if (hipStreamWaitEvent(comm->side, ready_all[(size_t)r], 0) != hipSuccess) rc = ncclSystemError;
  // every all-reduce of the group stages into its own part of the stage buffer
  // (another rank's sum may still read this rank's stage of an earlier op)
  size_t stage_total = 0;
  for (const Op& o : coll)
    if (o.kind == OP_ALLREDUCE) stage_total += o.count * o.esize;
  if (rc == ncclSuccess && comm->stage_bytes < stage_total) {
    if (comm->stage) (void)hipFree(comm->stage);
    comm->stage = nullptr;
    comm->stage_bytes = 0;
    if (hipMalloc(&comm->stage, stage_total) != hipSuccess) rc = ncclSystemError;
    else comm->stage_bytes = stage_total;
  }
  size_t stage_off = 0;
  for (size_t ci = 0; ci < coll.size(); ++ci) {
    const Op& o = coll[ci];
    const size_t bytes = o.count * o.esize;
    if (o.kind == OP_ALLGATHER) {
      for (int r = 0; r < n && rc == ncclSuccess; ++r) {
        const Op& x = (*w->posted[(size_t)r])[ci];
        if (bytes && hipMemcpyAsync(static_cast<uint8_t*>(o.dst) + (size_t)r * bytes, x.src, bytes, hipMemcpyDefault,
                                    comm->side) != hipSuccess)
          rc = ncclSystemError;
      }
      continue;
    }
    // all-reduce (in place allowed): stage every rank's input, then sum the stages
    hipEvent_t staged = new_event();
    uint8_t* my_stage = static_cast<uint8_t*>(comm->stage) + stage_off;
    if (rc == ncclSuccess && bytes && hipMemcpyAsync(my_stage, o.src, bytes, hipMemcpyDefault, comm->side) != hipSuccess)
      rc = ncclSystemError;
    if (!staged || hipEventRecord(staged, comm->side) != hipSuccess) rc = ncclSystemError;
    {
      std::lock_guard<std::mutex> lk(w->mu);
      w->ev[(size_t)me] = staged;
      w->stage[(size_t)me] = comm->stage;
    }
    if (!barrier(w)) return ncclSystemError;
    Stages src{};
    for (int r = 0; r < n; ++r) {   // (the ranks' op sequences match: the same offset on every rank)
      src.p[r] = reinterpret_cast<const uint64_t*>(static_cast<const uint8_t*>(w->stage[(size_t)r]) + stage_off);
      if (rc == ncclSuccess && hipStreamWaitEvent(comm->side, w->ev[(size_t)r], 0) != hipSuccess) rc = ncclSystemError;
    }
    if (rc == ncclSuccess && o.count)
      hipLaunchKernelGGL(k_sum_u64, dim3(std::max<size_t>(1, std::min<size_t>((o.count + 255) / 256, 1024))), dim3(256),
                         0, comm->side, static_cast<uint64_t*>(o.dst), src, n, o.count);
    if (!barrier(w)) return ncclSystemError;   // every rank enqueued its waits on the staged events
    (void)hipEventDestroy(staged);
    stage_off += bytes;
  }
  // the caller's stream waits for every rank's copies (they read this rank's
  // inputs and wrote its outputs)
  hipEvent_t done = new_event();
  if (!done || hipEventRecord(done, comm->side) != hipSuccess) rc = ncclSystemError;
  {
    std::lock_guard<std::mutex> lk(w->mu);
    w->ev[(size_t)me] = done;
  }
  if (!barrier(w)) return ncclSystemError;
  for (int r = 0; r < n; ++r)
    if (hipStreamWaitEvent(caller, w->ev[(size_t)r], 0) != hipSuccess) rc = ncclSystemError;
  if (!barrier(w)) return ncclSystemError;   // every rank enqueued its waits
  (void)hipEventDestroy(done);
  {
    std::lock_guard<std::mutex> lk(w->mu);
    w->posted[(size_t)me] = nullptr;
  }
  return rc;
}

ncclResult_t run_p2p_async(ncclComm* comm, const std::vector<Op>& p2p, hipEvent_t ready, hipStream_t caller) {
  World* w = comm->w;
  const int me = comm->rank;
  std::deque<SendRec> recs;
  {
    std::lock_guard<std::mutex> lk(w->mu);
    for (const Op& o : p2p)
      if (o.kind == OP_SEND) {
        recs.emplace_back();
        w->box[{me, o.peer}].push_back(Mail{o.src, o.count * o.esize, &recs.back(), ready});
      }
  }
  w->cv.notify_all();
  ncclResult_t rc = ncclSuccess;
  // this rank's receive buffers are free once its own stream reached the call
  if (hipStreamWaitEvent(comm->side, ready, 0) != hipSuccess) rc = ncclSystemError;
  for (const Op& o : p2p) {
    if (o.kind != OP_RECV) continue;
    Mail m{};
    {
      std::unique_lock<std::mutex> lk(w->mu);
      auto& q = w->box[{o.peer, me}];
      if (!wait_for(w, lk, [&] { return !q.empty(); })) return ncclSystemError;
      m = q.front();
      q.pop_front();
    }
    bool ok = m.bytes == o.count * o.esize;
    hipEvent_t copied = new_event();
    if (ok && m.bytes) {
      ok = hipStreamWaitEvent(comm->side, m.ready, 0) == hipSuccess &&
           hipMemcpyAsync(o.dst, m.src, m.bytes, hipMemcpyDefault, comm->side) == hipSuccess &&
           after_recv(comm, o.dst, m.bytes, comm->side);
    }
    if (!copied || hipEventRecord(copied, comm->side) != hipSuccess) ok = false;
    if (!ok) rc = m.bytes == o.count * o.esize ? ncclSystemError : ncclInvalidUsage;
    {
      std::lock_guard<std::mutex> lk(w->mu);
      m.rec->copied = copied;
      m.rec->done = 1;
    }
    w->cv.notify_all();
  }
  {
    std::unique_lock<std::mutex> lk(w->mu);
    if (!wait_for(w, lk, [&] {
          for (const SendRec& r : recs)
            if (!r.done) return false;
          return true;
        }))
      return ncclSystemError;
  }
  // the caller's stream waits for its receives and for the copies out of its send buffers
  hipEvent_t recv_done = new_event();
  if (!recv_done || hipEventRecord(recv_done, comm->side) != hipSuccess ||
      hipStreamWaitEvent(caller, recv_done, 0) != hipSuccess)
    rc = ncclSystemError;
  for (SendRec& r : recs)
    if (r.copied && hipStreamWaitEvent(caller, r.copied, 0) != hipSuccess) rc = ncclSystemError;
  for (SendRec& r : recs)
    if (r.copied) (void)hipEventDestroy(r.copied);
  if (recv_done) (void)hipEventDestroy(recv_done);
  return rc;
}

// run this thread's recorded ops (one call, or one outermost group)
ncclResult_t run_group(ncclComm* comm) {
  std::vector<Op> ops;
  ops.swap(t_rank.ops);
  std::vector<Op> coll, p2p;
  for (const Op& o : ops) (o.kind == OP_SEND || o.kind == OP_RECV ? p2p : coll).push_back(o);
  if (async_mode()) {   // (the engine enqueues every op of a group on its one stream)
    const hipStream_t caller = ops.empty() ? nullptr : ops[0].stream;
    for (const Op& o : ops)
      if (o.stream != caller) return ncclInvalidUsage;
    hipEvent_t ready = new_event();
    if (!ready || hipEventRecord(ready, caller) != hipSuccess) return ncclSystemError;
    ncclResult_t rc = ncclSuccess;
    if (!coll.empty()) rc = run_collectives_async(comm, coll, ready, caller);
    if (!p2p.empty()) {
      const ncclResult_t r2 = run_p2p_async(comm, p2p, ready, caller);
      if (rc == ncclSuccess) rc = r2;
    }
    // (every peer enqueued its waits on `ready` before the rendezvous above returned)
    (void)hipEventDestroy(ready);
    return rc;
  }
  if (!sync_streams(ops)) return ncclSystemError;
  ncclResult_t rc = ncclSuccess;
  if (!coll.empty()) rc = run_collectives(comm, coll);
  if (!p2p.empty()) {
    const ncclResult_t r2 = run_p2p(comm, p2p);
    if (rc == ncclSuccess) rc = r2;
  }
  return rc;
}

ncclResult_t record(ncclComm* comm, Op op) {
  if (!comm || !comm->w) return ncclInvalidArgument;
  if (op.esize == 0) return ncclInvalidArgument;
  if ((op.kind == OP_SEND || op.kind == OP_RECV) && (op.peer < 0 || op.peer >= comm->w->n)) return ncclInvalidArgument;
  t_rank.ops.push_back(op);
  if (t_rank.depth > 0) return ncclSuccess;
  return run_group(comm);
}

// the communicator of the ops recorded in this thread's group (one per thread)
thread_local ncclComm* t_comm = nullptr;

}  // namespace

extern "C" {

const char* ncclGetErrorString(ncclResult_t r) {
  switch (r) {
    case ncclSuccess: return "no error (rccl stand-in)";
    case ncclSystemError: return "system error (rccl stand-in: HIP call failed or a rank timed out)";
    case ncclInvalidArgument: return "invalid argument (rccl stand-in)";
    case ncclInvalidUsage: return "invalid usage (rccl stand-in: ranks' calls do not match)";
    default: return "error (rccl stand-in)";
  }
}

ncclResult_t ncclGetUniqueId(ncclUniqueId* id) {
  if (!id) return ncclInvalidArgument;
  std::memset(id, 0, sizeof(*id));
  const std::string s = "rccl-standin-" + std::to_string(g_id_counter.fetch_add(1)) + "-" +
                        std::to_string((unsigned long long)std::chrono::steady_clock::now().time_since_epoch().count());
  std::memcpy(id->internal, s.data(), std::min(s.size(), sizeof(id->internal) - 1));
  return ncclSuccess;
}

ncclResult_t ncclCommInitRank(ncclComm_t* comm, int nranks, ncclUniqueId commId, int rank) {
  if (!comm || nranks < 1 || nranks > kMaxRanks || rank < 0 || rank >= nranks) return ncclInvalidArgument;
  const std::string key(commId.internal, strnlen(commId.internal, sizeof(commId.internal)));
  World* w;
  {
    std::lock_guard<std::mutex> lk(g_worlds_mu);
    auto it = g_worlds.find(key);
    if (it == g_worlds.end()) {
      w = new World();
      w->n = nranks;
      w->posted.assign((size_t)nranks, nullptr);
      w->ev.assign((size_t)nranks, nullptr);
      w->stage.assign((size_t)nranks, nullptr);
      g_worlds[key] = w;
    } else {
      w = it->second;
    }
  }
  if (w->n != nranks) return ncclInvalidUsage;
  {
    std::lock_guard<std::mutex> lk(w->mu);
    ++w->joined;
  }
  if (!barrier(w)) return ncclSystemError;   // like RCCL: returns once every rank joined
  ncclComm* c = new ncclComm{w, rank};
  if (async_mode() && hipStreamCreateWithFlags(&c->side, hipStreamNonBlocking) != hipSuccess) {
    delete c;
    return ncclSystemError;
  }
  *comm = c;
  return ncclSuccess;
}

ncclResult_t ncclCommDestroy(ncclComm_t comm) {
  if (!comm) return ncclSuccess;
  World* w = comm->w;
  bool last = false;
  {
    std::lock_guard<std::mutex> lk(w->mu);
    last = --w->joined == 0;
  }
  if (last) {
    std::lock_guard<std::mutex> lk(g_worlds_mu);
    for (auto it = g_worlds.begin(); it != g_worlds.end(); ++it)
      if (it->second == w) {
        g_worlds.erase(it);
        break;
      }
    delete w;
  }
  if (comm->side) {
    (void)hipStreamSynchronize(comm->side);
    (void)hipStreamDestroy(comm->side);
  }
  if (comm->stage) (void)hipFree(comm->stage);
  delete comm;
  return ncclSuccess;
}

ncclResult_t ncclCommCount(const ncclComm_t comm, int* count) {
  if (!comm || !count) return ncclInvalidArgument;
  *count = comm->w->n;
  return ncclSuccess;
}

ncclResult_t ncclCommUserRank(const ncclComm_t comm, int* rank) {
  if (!comm || !rank) return ncclInvalidArgument;
  *rank = comm->rank;
  return ncclSuccess;
}

ncclResult_t ncclGroupStart() {
  ++t_rank.depth;
  return ncclSuccess;
}

ncclResult_t ncclGroupEnd() {
  if (t_rank.depth <= 0) return ncclInvalidUsage;
  if (--t_rank.depth > 0) return ncclSuccess;
  ncclComm* c = t_comm;
  t_comm = nullptr;
  if (t_rank.ops.empty()) return ncclSuccess;
  return run_group(c);
}

ncclResult_t ncclAllReduce(const void* sendbuff, void* recvbuff, size_t count, ncclDataType_t datatype,
                           ncclRedOp_t op, ncclComm_t comm, hipStream_t stream) {
  if (op != ncclSum || (datatype != ncclUint64 && datatype != ncclInt64)) return ncclInvalidArgument;
  if (t_rank.depth > 0) t_comm = comm;
  return record(comm, Op{OP_ALLREDUCE, sendbuff, recvbuff, count, 8, -1, stream});
}

ncclResult_t ncclAllGather(const void* sendbuff, void* recvbuff, size_t sendcount, ncclDataType_t datatype,
                           ncclComm_t comm, hipStream_t stream) {
  if (t_rank.depth > 0) t_comm = comm;
  return record(comm, Op{OP_ALLGATHER, sendbuff, recvbuff, sendcount, esize_of(datatype), -1, stream});
}

ncclResult_t ncclSend(const void* sendbuff, size_t count, ncclDataType_t datatype, int peer, ncclComm_t comm,
                      hipStream_t stream) {
  if (t_rank.depth > 0) t_comm = comm;
  return record(comm, Op{OP_SEND, sendbuff, nullptr, count, esize_of(datatype), peer, stream});
}

ncclResult_t ncclRecv(void* recvbuff, size_t count, ncclDataType_t datatype, int peer, ncclComm_t comm,
                      hipStream_t stream) {
  if (t_rank.depth > 0) t_comm = comm;
  return record(comm, Op{OP_RECV, nullptr, recvbuff, count, esize_of(datatype), peer, stream});
}

}  // extern "C"
