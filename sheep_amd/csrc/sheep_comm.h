// Communicators of the multi-GPU path (graph2tree -i -r over RCCL; see sheep_comm.cpp).
// One rank's view of a group of P ranks, one process (or thread) per rank.  Every call is
// collective: all ranks make the same calls in the same order.  Buffers are device memory of
// the rank's device; ops are enqueued on `s` (RCCL) or completed before returning (the thread
// group used to rehearse P ranks on one device).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <memory>

namespace sheep {

struct Comm {
  virtual ~Comm() = default;
  virtual int rank() const = 0;
  virtual int size() const = 0;
  // in place over n elements
  virtual void allreduce_sum_u32(uint32_t* buf, size_t n, hipStream_t s) = 0;
  virtual void allreduce_sum_u64(uint64_t* buf, size_t n, hipStream_t s) = 0;
  virtual void allreduce_max_i64(int64_t* buf, size_t n, hipStream_t s) = 0;
  // recv[r * n + i] = send_r[i]; in place when send == recv + rank * n
  virtual void allgather_u64(const uint64_t* send, uint64_t* recv, size_t n, hipStream_t s) = 0;
  // recv[i] = sum over ranks of send_q[rank * n + i] (send: size * n elements)
  virtual void reduce_scatter_sum_u32(const uint32_t* send, uint32_t* recv, size_t n,
                                      hipStream_t s) = 0;
};

// RCCL (loaded with dlopen on first use: single-GPU callers never load it).  id: 128 bytes.
void rccl_unique_id(uint8_t* id);
std::unique_ptr<Comm> rccl_comm(const uint8_t* id, int n_ranks, int rank);

// P processes through POSIX shared memory (name: "/..."), collectives staged on the host: the
// multi-process rehearsal on a one-GPU box (tests).  Rank 0 creates the region; the others
// attach within 60 s.
std::unique_ptr<Comm> shm_comm(const char* name, int n_ranks, int rank, uint64_t slot_bytes);

// P ranks as P threads of one process on one device: the collectives become device copies
// and a sum / max kernel between barriers.  make_local_group returns the shared state; each
// thread then takes local_comm(group, rank).
struct LocalGroup;
std::shared_ptr<LocalGroup> make_local_group(int n_ranks);
std::unique_ptr<Comm> local_comm(std::shared_ptr<LocalGroup> g, int rank);
// a failed rank releases the others from their barriers (they throw "rank group aborted")
void group_abort(LocalGroup& g);

// kernels (sheep_kernels.hip): dst[i] = op over the P source arrays
void launch_sum_ptrs_u32(uint32_t* dst, const uint32_t* const* srcs, int P, size_t n, hipStream_t s);
void launch_sum_ptrs_u64(uint64_t* dst, const uint64_t* const* srcs, int P, size_t n, hipStream_t s);
void launch_max_ptrs_i64(int64_t* dst, const int64_t* const* srcs, int P, size_t n, hipStream_t s);

}  // namespace sheep
