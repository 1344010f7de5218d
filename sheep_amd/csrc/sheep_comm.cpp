// Communicators of the multi-GPU path: RCCL over xGMI (one process per GPU), and an in-process
// thread group that rehearses P ranks on one device.  The reference's MPI calls these replace:
// MPI_Allreduce MAX / SUM of the degrees (sequence.h:72,78) and the MPI_Reduce of the trees
// (jnode.cpp:241), here an all-gather of each bucket's kept pairs and a sum of pst_weight.
#include <dlfcn.h>
#include <fcntl.h>
#include <pthread.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <thread>

#include <condition_variable>
#include <cstring>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

#include <rccl/rccl.h>

#include "sheep_comm.h"

namespace sheep {

#define HIPC(x)                                                                                \
  do {                                                                                         \
    hipError_t e_ = (x);                                                                       \
    if (e_ != hipSuccess) throw std::runtime_error(std::string(#x) + ": " + hipGetErrorString(e_)); \
  } while (0)

// ---- RCCL, resolved at run time ------------------------------------------------------------
struct RcclApi {
  decltype(&ncclGetUniqueId) get_unique_id = nullptr;
  decltype(&ncclCommInitRank) init_rank = nullptr;
  decltype(&ncclCommDestroy) destroy = nullptr;
  decltype(&ncclAllReduce) all_reduce = nullptr;
  decltype(&ncclAllGather) all_gather = nullptr;
  decltype(&ncclReduceScatter) reduce_scatter = nullptr;
  decltype(&ncclGetErrorString) error_string = nullptr;
};

static const RcclApi& rccl() {
  static RcclApi api;
  static std::once_flag once;
  static std::string err;
  std::call_once(once, [] {
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) {
      err = std::string("cannot load librccl.so.1: ") + dlerror();
      return;
    }
    api.get_unique_id = (decltype(api.get_unique_id))dlsym(h, "ncclGetUniqueId");
    api.init_rank = (decltype(api.init_rank))dlsym(h, "ncclCommInitRank");
    api.destroy = (decltype(api.destroy))dlsym(h, "ncclCommDestroy");
    api.all_reduce = (decltype(api.all_reduce))dlsym(h, "ncclAllReduce");
    api.all_gather = (decltype(api.all_gather))dlsym(h, "ncclAllGather");
    api.reduce_scatter = (decltype(api.reduce_scatter))dlsym(h, "ncclReduceScatter");
    api.error_string = (decltype(api.error_string))dlsym(h, "ncclGetErrorString");
    if (!api.get_unique_id || !api.init_rank || !api.destroy || !api.all_reduce ||
        !api.all_gather || !api.reduce_scatter || !api.error_string)
      err = "librccl.so.1 lacks an entry point";
  });
  if (!err.empty()) throw std::runtime_error(err);
  return api;
}

static void nccl_check(ncclResult_t r, const char* what) {
  if (r != ncclSuccess)
    throw std::runtime_error(std::string(what) + ": " + rccl().error_string(r));
}

void rccl_unique_id(uint8_t* id) {
  ncclUniqueId u;
  nccl_check(rccl().get_unique_id(&u), "ncclGetUniqueId");
  memcpy(id, u.internal, NCCL_UNIQUE_ID_BYTES);
}

struct RcclComm : Comm {
  ncclComm_t comm = nullptr;
  int r = 0, p = 1;
  RcclComm(const uint8_t* id, int n_ranks, int rank) : r(rank), p(n_ranks) {
    ncclUniqueId u;
    memcpy(u.internal, id, NCCL_UNIQUE_ID_BYTES);
    nccl_check(rccl().init_rank(&comm, n_ranks, u, rank), "ncclCommInitRank");
  }
  ~RcclComm() override {
    if (comm) (void)rccl().destroy(comm);
  }
  int rank() const override { return r; }
  int size() const override { return p; }
  void allreduce_sum_u32(uint32_t* buf, size_t n, hipStream_t s) override {
    nccl_check(rccl().all_reduce(buf, buf, n, ncclUint32, ncclSum, comm, s), "ncclAllReduce");
  }
  void allreduce_sum_u64(uint64_t* buf, size_t n, hipStream_t s) override {
    nccl_check(rccl().all_reduce(buf, buf, n, ncclUint64, ncclSum, comm, s), "ncclAllReduce");
  }
  void allreduce_max_i64(int64_t* buf, size_t n, hipStream_t s) override {
    nccl_check(rccl().all_reduce(buf, buf, n, ncclInt64, ncclMax, comm, s), "ncclAllReduce");
  }
  void allgather_u64(const uint64_t* send, uint64_t* recv, size_t n, hipStream_t s) override {
    nccl_check(rccl().all_gather(send, recv, n, ncclUint64, comm, s), "ncclAllGather");
  }
  void reduce_scatter_sum_u32(const uint32_t* send, uint32_t* recv, size_t n, hipStream_t s) override {
    nccl_check(rccl().reduce_scatter(send, recv, n, ncclUint32, ncclSum, comm, s), "ncclReduceScatter");
  }
};

std::unique_ptr<Comm> rccl_comm(const uint8_t* id, int n_ranks, int rank) {
  return std::unique_ptr<Comm>(new RcclComm(id, n_ranks, rank));
}

// ---- P threads on one device ---------------------------------------------------------------
struct LocalGroup {
  int P;
  std::mutex mu;
  std::condition_variable cv;
  int arrived = 0;
  uint64_t generation = 0;
  std::vector<const void*> ptrs;
  void* staging = nullptr;  // device scratch of the reductions (grown by rank 0)
  size_t staging_bytes = 0;
  const void** d_ptrs = nullptr;  // device copy of ptrs
  explicit LocalGroup(int p) : P(p), ptrs(p, nullptr) {}
  ~LocalGroup() {
    if (staging) (void)hipFree(staging);
    if (d_ptrs) (void)hipFree(d_ptrs);
  }
  bool aborted = false;
  void barrier() {
    std::unique_lock<std::mutex> lk(mu);
    if (aborted) throw std::runtime_error("rank group aborted");
    const uint64_t gen = generation;
    if (++arrived == P) {
      arrived = 0;
      ++generation;
      cv.notify_all();
    } else {
      cv.wait(lk, [&] { return generation != gen || aborted; });
      if (aborted) throw std::runtime_error("rank group aborted");
    }
  }
};

void group_abort(LocalGroup& g) {
  std::lock_guard<std::mutex> lk(g.mu);
  g.aborted = true;
  g.cv.notify_all();
}

std::shared_ptr<LocalGroup> make_local_group(int n_ranks) {
  return std::make_shared<LocalGroup>(n_ranks);
}

struct LocalComm : Comm {
  std::shared_ptr<LocalGroup> g;
  int r;
  LocalComm(std::shared_ptr<LocalGroup> grp, int rank) : g(std::move(grp)), r(rank) {}
  int rank() const override { return r; }
  int size() const override { return g->P; }

  // every rank publishes buf; rank 0 reduces all of them into the staging buffer; every rank
  // copies the result back.  The barriers order the device work across the threads (each
  // rank's stream is drained before it arrives).
  template <typename T, typename L>
  void reduce_all(T* buf, size_t n, hipStream_t s, L launch) {
    HIPC(hipStreamSynchronize(s));
    g->ptrs[r] = buf;
    g->barrier();
    if (r == 0) {
      if (g->staging_bytes < n * sizeof(T)) {
        if (g->staging) HIPC(hipFree(g->staging));
        g->staging = nullptr;
        HIPC(hipMalloc(&g->staging, n * sizeof(T)));
        g->staging_bytes = n * sizeof(T);
      }
      if (!g->d_ptrs) HIPC(hipMalloc((void**)&g->d_ptrs, 64 * sizeof(void*)));
      HIPC(hipMemcpyAsync((void*)g->d_ptrs, g->ptrs.data(), g->P * sizeof(void*), hipMemcpyHostToDevice, s));
      launch((T*)g->staging, (const T* const*)g->d_ptrs, g->P, n, s);
      HIPC(hipStreamSynchronize(s));
    }
    g->barrier();
    HIPC(hipMemcpyAsync(buf, g->staging, n * sizeof(T), hipMemcpyDeviceToDevice, s));
    HIPC(hipStreamSynchronize(s));
    g->barrier();
  }
  void allreduce_sum_u32(uint32_t* buf, size_t n, hipStream_t s) override {
    reduce_all(buf, n, s, launch_sum_ptrs_u32);
  }
  void allreduce_sum_u64(uint64_t* buf, size_t n, hipStream_t s) override {
    reduce_all(buf, n, s, launch_sum_ptrs_u64);
  }
  void allreduce_max_i64(int64_t* buf, size_t n, hipStream_t s) override {
    reduce_all(buf, n, s, launch_max_ptrs_i64);
  }
  void allgather_u64(const uint64_t* send, uint64_t* recv, size_t n, hipStream_t s) override {
    HIPC(hipStreamSynchronize(s));
    g->ptrs[r] = send;
    g->barrier();
    for (int q = 0; q < g->P; ++q)
      if (n && (const void*)(recv + (size_t)q * n) != g->ptrs[q])
        HIPC(hipMemcpyAsync(recv + (size_t)q * n, g->ptrs[q], n * 8, hipMemcpyDeviceToDevice, s));
    HIPC(hipStreamSynchronize(s));
    g->barrier();
  }
  // each rank sums its own slice of every rank's buffer (its own device pointer table)
  void reduce_scatter_sum_u32(const uint32_t* send, uint32_t* recv, size_t n, hipStream_t s) override {
    HIPC(hipStreamSynchronize(s));
    g->ptrs[r] = send;
    g->barrier();
    if (!d_mine) HIPC(hipMalloc((void**)&d_mine, 64 * sizeof(void*)));
    std::vector<const uint32_t*> mine(g->P);
    for (int q = 0; q < g->P; ++q) mine[q] = (const uint32_t*)g->ptrs[q] + (size_t)r * n;
    HIPC(hipMemcpyAsync((void*)d_mine, mine.data(), g->P * sizeof(void*), hipMemcpyHostToDevice, s));
    launch_sum_ptrs_u32(recv, (const uint32_t* const*)d_mine, g->P, n, s);
    HIPC(hipStreamSynchronize(s));
    g->barrier();
  }
  const void** d_mine = nullptr;
  ~LocalComm() override {
    if (d_mine) (void)hipFree(d_mine);
  }
};

std::unique_ptr<Comm> local_comm(std::shared_ptr<LocalGroup> g, int rank) {
  return std::unique_ptr<Comm>(new LocalComm(std::move(g), rank));
}

// ---- P processes through host shared memory -------------------------------------------------
// The rehearsal of the multi-process driver where RCCL cannot run (every process on the one GPU
// of a test box): each rank stages its buffer in its slot of a POSIX shared-memory region, a
// process-shared barrier orders the ranks, and each rank combines the slots on the host.
// Synchronous (the stream is drained first), chunked by the slot size.  Tests only: the bytes
// cross PCIe twice.  A group's name must be unique to the group (the tests use uuids): rank 0
// unlinks a crashed run's region of the same name before creating its own, but a rank that
// opened the old one first would attach to it and wait at its barrier.
struct ShmHeader {
  pthread_barrier_t bar;
  std::atomic<uint32_t> ready;
  uint32_t n_ranks;
  uint64_t slot_bytes;
};
static constexpr uint32_t SHM_MAGIC = 0x5ee95ee9u;
static constexpr size_t SHM_HDR = 4096;

struct ShmComm : Comm {
  int r = 0, p = 1;
  std::string name;
  size_t bytes = 0;
  ShmHeader* hdr = nullptr;
  char* slots = nullptr;
  uint64_t slot = 0;
  std::vector<char> tmp;
  ShmComm(const char* nm, int n_ranks, int rank, uint64_t slot_bytes) : r(rank), p(n_ranks), name(nm) {
    slot = slot_bytes;
    bytes = SHM_HDR + (size_t)p * slot;
    int fd = -1;
    if (r == 0) {
      shm_unlink(name.c_str());  // a stale region of a crashed run
      fd = shm_open(name.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600);
      if (fd < 0 || ftruncate(fd, (off_t)bytes) != 0) throw std::runtime_error("shm: create " + name);
    } else {
      const auto t0 = std::chrono::steady_clock::now();
      for (;;) {
        fd = shm_open(name.c_str(), O_RDWR, 0600);
        struct stat st;
        if (fd >= 0 && fstat(fd, &st) == 0 && (size_t)st.st_size >= bytes) break;
        if (fd >= 0) close(fd);
        if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(60))
          throw std::runtime_error("shm: no region " + name);
        std::this_thread::sleep_for(std::chrono::milliseconds(2));
      }
    }
    void* base = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    if (base == MAP_FAILED) throw std::runtime_error("shm: mmap " + name);
    hdr = (ShmHeader*)base;
    slots = (char*)base + SHM_HDR;
    if (r == 0) {
      pthread_barrierattr_t a;
      pthread_barrierattr_init(&a);
      pthread_barrierattr_setpshared(&a, PTHREAD_PROCESS_SHARED);
      pthread_barrier_init(&hdr->bar, &a, (unsigned)p);
      pthread_barrierattr_destroy(&a);
      hdr->n_ranks = (uint32_t)p;
      hdr->slot_bytes = slot;
      hdr->ready.store(SHM_MAGIC, std::memory_order_release);
    } else {
      const auto t0 = std::chrono::steady_clock::now();
      while (hdr->ready.load(std::memory_order_acquire) != SHM_MAGIC) {
        if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(60))
          throw std::runtime_error("shm: region never initialised");
        std::this_thread::sleep_for(std::chrono::milliseconds(1));
      }
      if (hdr->n_ranks != (uint32_t)p || hdr->slot_bytes != slot)
        throw std::runtime_error("shm: ranks disagree on the group");
    }
    barrier();
    if (r == 0) shm_unlink(name.c_str());  // every rank is attached: the name can go
  }
  ~ShmComm() override {
    if (hdr) munmap((void*)hdr, bytes);
  }
  void barrier() { pthread_barrier_wait(&hdr->bar); }
  char* slot_of(int q) const { return slots + (size_t)q * slot; }
  int rank() const override { return r; }
  int size() const override { return p; }

  // out[i] = op over ranks of in_q[i] (in: device, each rank's own); chunked by the slot size
  template <typename T, typename OP>
  void reduce_to(const T* in, T* out, size_t n, hipStream_t s, OP op) {
    const size_t per = slot / sizeof(T);
    tmp.resize(std::min(n, per) * sizeof(T));
    T* acc = (T*)tmp.data();
    HIPC(hipStreamSynchronize(s));
    for (size_t off = 0; off < n; off += per) {
      const size_t c = std::min(per, n - off);
      HIPC(hipMemcpy(slot_of(r), in + off, c * sizeof(T), hipMemcpyDeviceToHost));
      barrier();
      memcpy(acc, slot_of(0), c * sizeof(T));
      for (int q = 1; q < p; ++q) {
        const T* x = (const T*)slot_of(q);
        for (size_t i = 0; i < c; ++i) acc[i] = op(acc[i], x[i]);
      }
      barrier();
      HIPC(hipMemcpy(out + off, acc, c * sizeof(T), hipMemcpyHostToDevice));
    }
  }
  void allreduce_sum_u32(uint32_t* buf, size_t n, hipStream_t s) override {
    reduce_to(buf, buf, n, s, [](uint32_t a, uint32_t b) { return a + b; });
  }
  void allreduce_sum_u64(uint64_t* buf, size_t n, hipStream_t s) override {
    reduce_to(buf, buf, n, s, [](uint64_t a, uint64_t b) { return a + b; });
  }
  void allreduce_max_i64(int64_t* buf, size_t n, hipStream_t s) override {
    reduce_to(buf, buf, n, s, [](int64_t a, int64_t b) { return a > b ? a : b; });
  }
  void allgather_u64(const uint64_t* send, uint64_t* recv, size_t n, hipStream_t s) override {
    const size_t per = slot / 8;
    HIPC(hipStreamSynchronize(s));
    for (size_t off = 0; off < n; off += per) {
      const size_t c = std::min(per, n - off);
      HIPC(hipMemcpy(slot_of(r), send + off, c * 8, hipMemcpyDeviceToHost));
      barrier();
      for (int q = 0; q < p; ++q)
        HIPC(hipMemcpy(recv + (size_t)q * n + off, slot_of(q), c * 8, hipMemcpyHostToDevice));
      barrier();
    }
  }
  void reduce_scatter_sum_u32(const uint32_t* send, uint32_t* recv, size_t n, hipStream_t s) override {
    // rank q's slice is the sum of every rank's send[q n, q n + n): one reduction per slice,
    // each rank keeping its own
    for (int q = 0; q < p; ++q) {
      std::vector<uint32_t> part;
      const size_t per = slot / 4;
      HIPC(hipStreamSynchronize(s));
      for (size_t off = 0; off < n; off += per) {
        const size_t c = std::min(per, n - off);
        HIPC(hipMemcpy(slot_of(r), send + (size_t)q * n + off, c * 4, hipMemcpyDeviceToHost));
        barrier();
        if (q == r) {
          part.assign((const uint32_t*)slot_of(0), (const uint32_t*)slot_of(0) + c);
          for (int u = 1; u < p; ++u) {
            const uint32_t* x = (const uint32_t*)slot_of(u);
            for (size_t i = 0; i < c; ++i) part[i] += x[i];
          }
          HIPC(hipMemcpy(recv + off, part.data(), c * 4, hipMemcpyHostToDevice));
        }
        barrier();
      }
    }
  }
};

std::unique_ptr<Comm> shm_comm(const char* name, int n_ranks, int rank, uint64_t slot_bytes) {
  return std::unique_ptr<Comm>(new ShmComm(name, n_ranks, rank, slot_bytes));
}

}  // namespace sheep
