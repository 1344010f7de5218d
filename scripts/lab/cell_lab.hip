// Lab (not product): rank gathers over records in different partitioned orders — one endpoint
// from a 1 MB rank slice (the current two-pass scheme) vs both endpoints from 2D cells.
#include <hip/hip_runtime.h>
#include <stdint.h>

static constexpr uint32_t INV = 0xFFFFFFFFu;

// mode 0: gather rank[y] only -> (x, ry); 1: rank[x] only -> (rx, y); 2: both -> (max, min);
// 3: no gather (the stream alone).
// xcd: tile t is processed by block (t % nxcd) * ... so each XCD walks a contiguous tile range.
template <int IT>
__global__ void __launch_bounds__(1024)
k_cell(const uint2* __restrict__ uv, uint64_t m, const uint32_t* __restrict__ rank,
       uint64_t* __restrict__ out, int mode, int xcd) {
  const uint32_t nb = gridDim.x;
  uint32_t b = blockIdx.x;
  if (xcd) {  // blocks go to XCDs round robin: block b -> XCD b % 8
    const uint32_t per = (nb + 7) / 8;
    b = (b % 8) * per + b / 8;
    if (b >= nb) return;
  }
  const uint64_t base = (uint64_t)b * 1024 * IT;
  uint2 e[IT];
  uint32_t r0[IT], r1[IT];
#pragma unroll
  for (int k = 0; k < IT; ++k) {
    const uint64_t i = base + (uint64_t)k * 1024 + threadIdx.x;
    e[k] = i < m ? uv[i] : make_uint2(0, 0);
  }
#pragma unroll
  for (int k = 0; k < IT; ++k) {
    r0[k] = (mode == 1 || mode == 2) ? rank[e[k].x] : e[k].x;
    r1[k] = (mode == 0 || mode == 2) ? rank[e[k].y] : e[k].y;
  }
#pragma unroll
  for (int k = 0; k < IT; ++k) {
    const uint64_t i = base + (uint64_t)k * 1024 + threadIdx.x;
    if (i >= m) continue;
    uint32_t hi = max(r0[k], r1[k]), lo = min(r0[k], r1[k]);
    out[i] = mode == 2 ? (((uint64_t)hi << 32) | lo) : (((uint64_t)r1[k] << 32) | r0[k]);
  }
}

// Degree by global atomics (no return) in the records' order: deg[x]++ and deg[y]++ (x != y).
template <int IT>
__global__ void __launch_bounds__(1024)
k_deg_atomic(const uint2* __restrict__ uv, uint64_t m, uint32_t* deg, int xcd) {
  const uint32_t nb = gridDim.x;
  uint32_t b = blockIdx.x;
  if (xcd) {
    const uint32_t per = (nb + 7) / 8;
    b = (b % 8) * per + b / 8;
    if (b >= nb) return;
  }
  const uint64_t base = (uint64_t)b * 1024 * IT;
  uint2 e[IT];
#pragma unroll
  for (int k = 0; k < IT; ++k) {
    const uint64_t i = base + (uint64_t)k * 1024 + threadIdx.x;
    e[k] = i < m ? uv[i] : make_uint2(0, 0);
  }
#pragma unroll
  for (int k = 0; k < IT; ++k) {
    const uint64_t i = base + (uint64_t)k * 1024 + threadIdx.x;
    if (i >= m) continue;
    atomicAdd(&deg[e[k].x], 1u);
    if (e[k].x != e[k].y) atomicAdd(&deg[e[k].y], 1u);
  }
}

extern "C" int deg_lab(int xcd, const void* uv, uint64_t m, void* deg, void* stream) {
  const unsigned nb = (unsigned)((m + 8191) / 8192);
  hipLaunchKernelGGL(k_deg_atomic<8>, dim3(nb), dim3(1024), 0, (hipStream_t)stream, (const uint2*)uv, m,
                     (uint32_t*)deg, xcd);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" int cell_lab(int mode, int xcd, const void* uv, uint64_t m, const void* rank, void* out,
                        void* stream) {
  const unsigned nb = (unsigned)((m + 8191) / 8192);
  hipLaunchKernelGGL(k_cell<8>, dim3(nb), dim3(1024), 0, (hipStream_t)stream, (const uint2*)uv, m,
                     (const uint32_t*)rank, (uint64_t*)out, mode, xcd);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
