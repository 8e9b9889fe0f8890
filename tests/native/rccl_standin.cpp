// rccl_standin.cpp -- TEST INFRASTRUCTURE: an in-process stand-in for the ten
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
// "world" named by the unique id.  Every call first synchronizes the caller's
// stream (so the inputs the engine enqueued are in memory), then runs the
// collective synchronously with the other ranks' threads: barriers order the
// reads of every rank's inputs before any rank writes its outputs (in-place
// all-reduce), and point-to-point receives copy straight from the matching
// sender's buffer (the k-th receive from q matches q's k-th send to this rank
// inside one group, as in RCCL).  Calls between ncclGroupStart / ncclGroupEnd
// are recorded and run at the outermost ncclGroupEnd.  Barrier waits time out
// (ncclSystemError) instead of hanging a test when a rank fails.
//
// Built by build_lib.build_standin() into _build/libgossip_hip_rccl_standin.so
// together with the engine's own objects; the product library links real RCCL.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <atomic>
#include <chrono>
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

struct Mail {   // a posted send: the receiver copies from src and sets *done
  const void* src;
  size_t bytes;
  char* done;
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
};

namespace {

constexpr int kBarrierTimeoutS = 120;

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
  std::vector<char> done;
  for (const Op& o : p2p)
    if (o.kind == OP_SEND) done.push_back(0);
  {
    std::lock_guard<std::mutex> lk(w->mu);
    size_t k = 0;
    for (const Op& o : p2p)
      if (o.kind == OP_SEND) {
        w->box[{me, o.peer}].push_back(Mail{o.src, o.count * o.esize, &done[k++]});
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
    if (ok && m.bytes) ok = copy(o.dst, m.src, m.bytes, o.stream);
    if (!ok) rc = m.bytes == o.count * o.esize ? ncclSystemError : ncclInvalidUsage;
    {
      std::lock_guard<std::mutex> lk(w->mu);
      *m.done = 1;
    }
    w->cv.notify_all();
  }
  {
    std::unique_lock<std::mutex> lk(w->mu);
    if (!wait_for(w, lk, [&] {
          for (char d : done)
            if (!d) return false;
          return true;
        }))
      return ncclSystemError;
  }
  return rc;
}

// run this thread's recorded ops (one call, or one outermost group)
ncclResult_t run_group(ncclComm* comm) {
  std::vector<Op> ops;
  ops.swap(t_rank.ops);
  if (!sync_streams(ops)) return ncclSystemError;
  std::vector<Op> coll, p2p;
  for (const Op& o : ops) (o.kind == OP_SEND || o.kind == OP_RECV ? p2p : coll).push_back(o);
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
  if (!comm || nranks < 1 || rank < 0 || rank >= nranks) return ncclInvalidArgument;
  const std::string key(commId.internal, strnlen(commId.internal, sizeof(commId.internal)));
  World* w;
  {
    std::lock_guard<std::mutex> lk(g_worlds_mu);
    auto it = g_worlds.find(key);
    if (it == g_worlds.end()) {
      w = new World();
      w->n = nranks;
      w->posted.assign((size_t)nranks, nullptr);
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
  *comm = new ncclComm{w, rank};
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
  delete comm;
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
