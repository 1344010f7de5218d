// Streaming baselines on one MI355X (lab, not product): what a record pass can reach.
//   copy8   : out[i] = in[i], one u64 per lane per access, 8 accesses in flight per lane
//   copy16  : the same with 16-B accesses (two records per lane)
//   read8   : sum of in[i] (no stores)
//   gather  : out[i] = in[i] ^ rank[in[i].lo & mask], the rank table `tbl` MB (L2 / MALL / HBM)
// Sizes: N records of 8 B (default 2^30 = 8.6 GB, as RMAT-26).
//   hipcc -O3 --offload-arch=gfx950 -o stream_lab stream_lab.hip && ./stream_lab [log2N]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstdint>

#define CK(x)                                                                 \
  do {                                                                        \
    hipError_t e = (x);                                                       \
    if (e != hipSuccess) {                                                    \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                  \
      exit(1);                                                                \
    }                                                                         \
  } while (0)

template <int U>
__global__ void __launch_bounds__(256) copy8(const uint64_t* __restrict__ in, uint64_t* __restrict__ out, uint64_t n) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride * U) {
    uint64_t v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = i + u * stride < n ? in[i + u * stride] : 0;
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (i + u * stride < n) out[i + u * stride] = v[u];
  }
}

template <int U>
__global__ void __launch_bounds__(256) copy16(const uint4* __restrict__ in, uint4* __restrict__ out, uint64_t n) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride * U) {
    uint4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = i + u * stride < n ? in[i + u * stride] : make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (i + u * stride < n) out[i + u * stride] = v[u];
  }
}

template <int U>
__global__ void __launch_bounds__(256) read8(const uint64_t* __restrict__ in, uint64_t n, uint64_t* sink) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  uint64_t acc = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride * U) {
    uint64_t v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = i + u * stride < n ? in[i + u * stride] : 0;
#pragma unroll
    for (int u = 0; u < U; ++u) acc ^= v[u];
  }
  if (acc == 0x123456789ull) *sink = acc;
}

template <int U>
__global__ void __launch_bounds__(256) gather(const uint64_t* __restrict__ in, uint64_t* __restrict__ out,
                                              uint64_t n, const uint32_t* __restrict__ tbl, uint32_t mask) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride * U) {
    uint64_t v[U];
    uint32_t r[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = i + u * stride < n ? in[i + u * stride] : 0;
#pragma unroll
    for (int u = 0; u < U; ++u) r[u] = tbl[(uint32_t)v[u] & mask];
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (i + u * stride < n) out[i + u * stride] = v[u] ^ ((uint64_t)r[u] << 32);
  }
}

// n random CAS / returning adds / plain loads on a table of (mask + 1) words
template <int OP>
__global__ void __launch_bounds__(256) rnd_atomic(uint32_t* tbl, uint32_t mask, uint64_t n, uint64_t* sink) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  uint32_t acc = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride * 4) {
    uint32_t r[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      uint64_t z = (i + u * stride) * 0x9E3779B97F4A7C15ull;
      z ^= z >> 29;
      const uint32_t k = (uint32_t)z & mask;
      if (OP == 0) r[u] = atomicCAS(&tbl[k], 0xFFFFFFFFu, (uint32_t)i);
      else if (OP == 1) r[u] = atomicAdd(&tbl[k], 1u);
      else if (OP == 2) r[u] = __hip_atomic_load(&tbl[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      else r[u] = tbl[k];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) acc += r[u];
  }
  if (acc == 0x12345678u) *sink = acc;
}

__global__ void fill(uint64_t* p, uint64_t n, uint64_t seed) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t z = (i + seed) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    p[i] = z ^ (z >> 31);
  }
}

template <typename F>
static float timeit(F f, int reps = 5) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  f();
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(a));
  for (int r = 0; r < reps; ++r) f();
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms / reps;
}

int main(int argc, char** argv) {
  const int lg = argc > 1 ? atoi(argv[1]) : 30;
  const uint64_t n = 1ull << lg;
  uint64_t *in, *out, *sink;
  uint32_t* tbl;
  CK(hipMalloc(&in, n * 8));
  CK(hipMalloc(&out, n * 8));
  CK(hipMalloc(&sink, 8));
  CK(hipMalloc(&tbl, 1ull << 30));
  hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, in, n, 1);
  hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, (uint64_t*)tbl, (1ull << 30) / 8, 2);
  CK(hipDeviceSynchronize());
  const double gb = n * 8 / 1e9;
  for (unsigned grid : {1024u, 2048u, 4096u, 8192u}) {
    float t;
    t = timeit([&] { hipLaunchKernelGGL(copy8<8>, dim3(grid), dim3(256), 0, 0, in, out, n); });
    printf("grid %5u copy8   %7.3f ms  %6.0f GB/s (read+write)\n", grid, t, 2e3 * gb / t);
    t = timeit([&] { hipLaunchKernelGGL(copy16<4>, dim3(grid), dim3(256), 0, 0, (const uint4*)in, (uint4*)out, n / 2); });
    printf("grid %5u copy16  %7.3f ms  %6.0f GB/s\n", grid, t, 2e3 * gb / t);
    t = timeit([&] { hipLaunchKernelGGL(read8<8>, dim3(grid), dim3(256), 0, 0, in, n, sink); });
    printf("grid %5u read8   %7.3f ms  %6.0f GB/s (read)\n", grid, t, 1e3 * gb / t);
  }
  for (uint32_t mb : {1u, 4u, 16u, 64u, 256u, 1024u}) {
    const uint32_t mask = (uint32_t)((uint64_t)mb * (1 << 20) / 4 - 1);
    float t = timeit([&] { hipLaunchKernelGGL(gather<8>, dim3(4096), dim3(256), 0, 0, in, out, n, tbl, mask); });
    printf("gather table %4u MB  %7.3f ms  %6.0f GB/s streamed, %6.1f G lookups/s\n", mb, t, 2e3 * gb / t, n / t / 1e6);
  }
  const char* opn[4] = {"cas", "add-ret", "load-agent", "load"};
  for (uint32_t mb : {1u, 16u, 128u, 1024u}) {
    const uint32_t mask = (uint32_t)((uint64_t)mb * (1 << 20) / 4 - 1);
    const uint64_t nops = 1ull << 27;
    for (int op = 0; op < 4; ++op) {
      float t = timeit([&] {
        if (op == 0) hipLaunchKernelGGL(rnd_atomic<0>, dim3(4096), dim3(256), 0, 0, tbl, mask, nops, sink);
        if (op == 1) hipLaunchKernelGGL(rnd_atomic<1>, dim3(4096), dim3(256), 0, 0, tbl, mask, nops, sink);
        if (op == 2) hipLaunchKernelGGL(rnd_atomic<2>, dim3(4096), dim3(256), 0, 0, tbl, mask, nops, sink);
        if (op == 3) hipLaunchKernelGGL(rnd_atomic<3>, dim3(4096), dim3(256), 0, 0, tbl, mask, nops, sink);
      });
      printf("random %-10s table %4u MB  %7.3f ms  %6.2f G ops/s\n", opn[op], mb, t, nops / t / 1e6);
    }
  }
  return 0;
}
