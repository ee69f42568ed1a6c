// Native RCCL communicator (csrc/comm/rccl_comm.cpp): one communicator per process group, its
// collectives on a dedicated comm HIP stream fenced against the caller's compute stream by events.
//
// Replaces the reference's c10d ProcessGroupNCCL usage for the gradient traffic
// (/root/reference/mingpt/train.py:34 init_process_group("nccl"), trainer.py:71 DDP's bucket
// all-reduce); SURVEY §5.8.  Torch-free (HIP runtime + RCCL C API): the bindings wrap it.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include <string>

namespace mg {
namespace comm {

constexpr int kUniqueIdBytes = 128;  // NCCL_UNIQUE_ID_BYTES

enum class DType : int { F32 = 0, BF16 = 1, F16 = 2, I64 = 3, U8 = 4 };

// Resolves the RCCL entry points from the library already mapped into the process (torch's
// bundled librccl.so.1; `path` is opened only if no such library is loaded).  Throws
// std::runtime_error naming what is missing.
void load_rccl(const std::string& path);
int rccl_version();  // e.g. 22606

// 128 opaque bytes from ncclGetUniqueId (rank 0 creates them, every rank passes them to create()).
std::string unique_id();

// Opaque handle of a communicator; every call below takes it.
int64_t create(const std::string& uid, int nranks, int rank, int device);
void destroy(int64_t h);
hipStream_t comm_stream(int64_t h);
int nranks(int64_t h);
int device(int64_t h);
int rank(int64_t h);

// Collectives.  Each one: the comm stream waits for everything the compute stream `cs` has
// enqueued so far (an event), runs the collective, and records a completion event; the returned
// ticket names that event.  wait(ticket, s) makes stream `s` wait for it (no host block) and
// retires the ticket.  Sums only (the gradient traffic); counts in elements.
int64_t all_reduce(int64_t h, void* buf, size_t count, DType dt, hipStream_t cs);
int64_t reduce_scatter(int64_t h, const void* in, void* out, size_t count_per_rank, DType dt, hipStream_t cs);
int64_t all_gather(int64_t h, const void* in, void* out, size_t count_per_rank, DType dt, hipStream_t cs);
int64_t broadcast(int64_t h, void* buf, size_t count, DType dt, int root, hipStream_t cs);
void wait(int64_t h, int64_t ticket, hipStream_t s);
// release a ticket nobody will wait on (a dropped Work): its event returns to the free list, no
// stream waits; a no-op for unknown tickets or a destroyed communicator
void retire(int64_t h, int64_t ticket);
// 1 if the ticket's collective has completed on the device, 0 if not yet, -1 if the ticket is
// not outstanding (already waited / retired) -- diagnostics (bench.py's hang report)
int query(int64_t h, int64_t ticket);
// outstanding tickets (issued, not yet waited)
int pending(int64_t h);

}  // namespace comm
}  // namespace mg
