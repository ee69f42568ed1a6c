// Native RCCL communicator: the comm backend SURVEY §5.8 plans (csrc/comm/).
//
// The reference gets its gradient all-reduce from c10d ProcessGroupNCCL inside DDP
// (/root/reference/mingpt/train.py:34, trainer.py:71).  Here the data-parallel engine can own the
// communicator instead:
//  * bootstrap: rank 0 calls ncclGetUniqueId; the 128 bytes travel over the process group's store
//    (parallel/comm.py); every rank calls ncclCommInitRank on its own GPU;
//  * one dedicated comm HIP stream per communicator (highest priority, so a collective is not
//    queued behind compute kernels), fenced against the caller's compute stream by events: the
//    comm stream waits for what the compute stream has enqueued (the bucket's producers), the
//    compute stream later waits on the collective's completion event -- neither side blocks the
//    host, and backward keeps issuing kernels while RCCL moves the bucket over xGMI;
//  * the RCCL entry points come from the library already mapped into the process -- the RCCL
//    torch ships (librccl.so.1, 2.26.6 in this image), never a second copy from /opt/rocm -- by
//    dlopen(RTLD_NOLOAD) + dlsym, so the extension has no link-time RCCL dependency.
#include "comm.h"

#include <dlfcn.h>
#include <rccl/rccl.h>

#include <memory>
#include <mutex>
#include <stdexcept>
#include <unordered_map>
#include <vector>

namespace mg {
namespace comm {
namespace {

struct Fns {
  ncclResult_t (*getUniqueId)(ncclUniqueId*) = nullptr;
  ncclResult_t (*commInitRank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*commDestroy)(ncclComm_t) = nullptr;
  ncclResult_t (*allReduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*reduceScatter)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*allGather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*broadcast)(const void*, void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  const char* (*getErrorString)(ncclResult_t) = nullptr;
  ncclResult_t (*getVersion)(int*) = nullptr;
};
Fns g_fn;
void* g_lib = nullptr;
std::mutex g_mu;

void hip_check(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string("mg::comm: ") + what + ": " + hipGetErrorString(e));
}

void nccl_check(ncclResult_t r, const char* what) {
  if (r != ncclSuccess)
    throw std::runtime_error(std::string("mg::comm: ") + what + ": " +
                             (g_fn.getErrorString ? g_fn.getErrorString(r) : "rccl error"));
}

template <class T>
void sym(T& f, const char* name) {
  f = reinterpret_cast<T>(dlsym(g_lib, name));
  if (!f) throw std::runtime_error(std::string("mg::comm: RCCL symbol missing: ") + name);
}

ncclDataType_t nccl_type(DType d) {
  switch (d) {
    case DType::F32: return ncclFloat32;
    case DType::BF16: return ncclBfloat16;
    case DType::F16: return ncclFloat16;
    case DType::I64: return ncclInt64;
    default: return ncclUint8;
  }
}

struct Comm {
  ncclComm_t comm = nullptr;
  hipStream_t stream = nullptr;
  int device = 0, nranks = 1, rank = 0;
  std::vector<hipEvent_t> free_ev;
  std::unordered_map<int64_t, hipEvent_t> tickets;
  int64_t next_ticket = 1;
  std::mutex mu;

  hipEvent_t event() {
    if (!free_ev.empty()) {
      hipEvent_t e = free_ev.back();
      free_ev.pop_back();
      return e;
    }
    hipEvent_t e;
    hip_check(hipEventCreateWithFlags(&e, hipEventDisableTiming), "hipEventCreate");
    return e;
  }
};

// handle = index + 1; slots are never reused.  Callers hold a shared_ptr copy for the whole call
// (taken under g_mu), so destroy() -- reachable from a Python finaliser on any thread -- can drop
// the slot while a call is inside enqueue()/wait() without freeing the Comm under it: the last
// reference releases it after that call returns.
std::vector<std::shared_ptr<Comm>> g_comms;

std::shared_ptr<Comm> get(int64_t h) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (h <= 0 || h > (int64_t)g_comms.size() || !g_comms[h - 1]) throw std::runtime_error("mg::comm: bad handle");
  return g_comms[h - 1];
}

struct DeviceScope {  // the communicator's device for the duration of a call
  int prev = -1;
  explicit DeviceScope(int d) {
    hip_check(hipGetDevice(&prev), "hipGetDevice");
    if (prev != d) hip_check(hipSetDevice(d), "hipSetDevice");
  }
  ~DeviceScope() {
    int cur = -1;
    if (hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
  }
};

// comm stream after the compute stream's work so far -> collective -> completion ticket
template <class F>
int64_t enqueue(int64_t h, hipStream_t cs, F&& collective, const char* what) {
  const std::shared_ptr<Comm> cp = get(h);
  Comm& c = *cp;
  std::lock_guard<std::mutex> lk(c.mu);
  DeviceScope ds(c.device);
  hipEvent_t before = c.event();
  hip_check(hipEventRecord(before, cs), "hipEventRecord(compute)");
  hip_check(hipStreamWaitEvent(c.stream, before, 0), "hipStreamWaitEvent(comm)");
  c.free_ev.push_back(before);  // the wait captured the record: the event may be re-recorded
  nccl_check(collective(c), what);
  hipEvent_t done = c.event();
  hip_check(hipEventRecord(done, c.stream), "hipEventRecord(comm)");
  const int64_t t = c.next_ticket++;
  c.tickets.emplace(t, done);
  return t;
}

}  // namespace

void load_rccl(const std::string& path) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (g_lib) return;
  // the RCCL torch loaded (soname librccl.so.1); the path only if none is mapped yet
  g_lib = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);
  if (!g_lib && !path.empty()) g_lib = dlopen(path.c_str(), RTLD_NOW);
  if (!g_lib) throw std::runtime_error("mg::comm: no RCCL library loaded (import torch first) and none at '" + path + "'");
  sym(g_fn.getUniqueId, "ncclGetUniqueId");
  sym(g_fn.commInitRank, "ncclCommInitRank");
  sym(g_fn.commDestroy, "ncclCommDestroy");
  sym(g_fn.allReduce, "ncclAllReduce");
  sym(g_fn.reduceScatter, "ncclReduceScatter");
  sym(g_fn.allGather, "ncclAllGather");
  sym(g_fn.broadcast, "ncclBroadcast");
  sym(g_fn.getErrorString, "ncclGetErrorString");
  sym(g_fn.getVersion, "ncclGetVersion");
}

int rccl_version() {
  if (!g_lib) throw std::runtime_error("mg::comm: load_rccl first");
  int v = 0;
  nccl_check(g_fn.getVersion(&v), "ncclGetVersion");
  return v;
}

std::string unique_id() {
  if (!g_lib) throw std::runtime_error("mg::comm: load_rccl first");
  ncclUniqueId id;
  nccl_check(g_fn.getUniqueId(&id), "ncclGetUniqueId");
  return std::string(id.internal, sizeof(id.internal));
}

int64_t create(const std::string& uid, int nranks, int rank, int device) {
  if (!g_lib) throw std::runtime_error("mg::comm: load_rccl first");
  if ((int)uid.size() != kUniqueIdBytes) throw std::runtime_error("mg::comm: unique id must be 128 bytes");
  if (nranks < 1 || rank < 0 || rank >= nranks) throw std::runtime_error("mg::comm: bad rank / world size");
  auto c = std::make_shared<Comm>();
  c->device = device;
  c->nranks = nranks;
  c->rank = rank;
  DeviceScope ds(device);
  int least = 0, greatest = 0;
  hip_check(hipDeviceGetStreamPriorityRange(&least, &greatest), "hipDeviceGetStreamPriorityRange");
  hip_check(hipStreamCreateWithPriority(&c->stream, hipStreamNonBlocking, greatest), "hipStreamCreate");
  ncclUniqueId id;
  std::copy(uid.begin(), uid.end(), id.internal);
  nccl_check(g_fn.commInitRank(&c->comm, nranks, id, rank), "ncclCommInitRank");
  std::lock_guard<std::mutex> lk(g_mu);
  g_comms.push_back(std::move(c));
  return (int64_t)g_comms.size();
}

void destroy(int64_t h) {
  std::shared_ptr<Comm> c;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    if (h <= 0 || h > (int64_t)g_comms.size() || !g_comms[h - 1]) return;
    c = std::move(g_comms[h - 1]);
  }
  std::lock_guard<std::mutex> lk(c->mu);  // a concurrent enqueue()/wait() on another thread finishes first
  DeviceScope ds(c->device);
  (void)hipStreamSynchronize(c->stream);
  if (c->comm) (void)g_fn.commDestroy(c->comm);
  for (auto& kv : c->tickets) (void)hipEventDestroy(kv.second);
  for (auto e : c->free_ev) (void)hipEventDestroy(e);
  c->tickets.clear();
  c->free_ev.clear();
  c->comm = nullptr;
  // the comm stream is NOT destroyed: tensors the caller recorded on it (record_stream, so the
  // caching allocator does not hand their blocks out while a collective may still touch them)
  // make the allocator record events on this stream whenever they are freed -- possibly after
  // the communicator is gone.  One idle stream per communicator for the life of the process.
}

hipStream_t comm_stream(int64_t h) { return get(h)->stream; }
int nranks(int64_t h) { return get(h)->nranks; }
int device(int64_t h) { return get(h)->device; }
int rank(int64_t h) { return get(h)->rank; }

int64_t all_reduce(int64_t h, void* buf, size_t count, DType dt, hipStream_t cs) {
  return enqueue(h, cs, [&](Comm& c) {
    return g_fn.allReduce(buf, buf, count, nccl_type(dt), ncclSum, c.comm, c.stream);
  }, "ncclAllReduce");
}

int64_t reduce_scatter(int64_t h, const void* in, void* out, size_t count_per_rank, DType dt, hipStream_t cs) {
  return enqueue(h, cs, [&](Comm& c) {
    return g_fn.reduceScatter(in, out, count_per_rank, nccl_type(dt), ncclSum, c.comm, c.stream);
  }, "ncclReduceScatter");
}

int64_t all_gather(int64_t h, const void* in, void* out, size_t count_per_rank, DType dt, hipStream_t cs) {
  return enqueue(h, cs, [&](Comm& c) {
    return g_fn.allGather(in, out, count_per_rank, nccl_type(dt), c.comm, c.stream);
  }, "ncclAllGather");
}

int64_t broadcast(int64_t h, void* buf, size_t count, DType dt, int root, hipStream_t cs) {
  return enqueue(h, cs, [&](Comm& c) {
    return g_fn.broadcast(buf, buf, count, nccl_type(dt), root, c.comm, c.stream);
  }, "ncclBroadcast");
}

void wait(int64_t h, int64_t ticket, hipStream_t s) {
  const std::shared_ptr<Comm> cp = get(h);
  Comm& c = *cp;
  std::lock_guard<std::mutex> lk(c.mu);
  auto it = c.tickets.find(ticket);
  if (it == c.tickets.end()) throw std::runtime_error("mg::comm: unknown or already waited ticket");
  DeviceScope ds(c.device);
  hip_check(hipStreamWaitEvent(s, it->second, 0), "hipStreamWaitEvent(compute)");
  c.free_ev.push_back(it->second);
  c.tickets.erase(it);
}

void retire(int64_t h, int64_t ticket) {
  std::shared_ptr<Comm> cp;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    if (h <= 0 || h > (int64_t)g_comms.size() || !g_comms[h - 1]) return;  // destroyed: nothing to release
    cp = g_comms[h - 1];
  }
  std::lock_guard<std::mutex> lk(cp->mu);
  auto it = cp->tickets.find(ticket);
  if (it == cp->tickets.end()) return;
  // nobody will wait on it: the event goes back to the free list (a later re-record of a pending
  // event is fine -- only a stream wait captures a record, and none will for this ticket)
  cp->free_ev.push_back(it->second);
  cp->tickets.erase(it);
}

int query(int64_t h, int64_t ticket) {
  const std::shared_ptr<Comm> cp = get(h);
  std::lock_guard<std::mutex> lk(cp->mu);
  auto it = cp->tickets.find(ticket);
  if (it == cp->tickets.end()) return -1;
  DeviceScope ds(cp->device);
  const hipError_t e = hipEventQuery(it->second);
  if (e == hipSuccess) return 1;
  if (e == hipErrorNotReady) return 0;
  hip_check(e, "hipEventQuery");
  return 0;
}

int pending(int64_t h) {
  const std::shared_ptr<Comm> cp = get(h);
  std::lock_guard<std::mutex> lk(cp->mu);
  return (int)cp->tickets.size();
}

}  // namespace comm
}  // namespace mg
