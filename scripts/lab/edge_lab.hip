// Lab (not product): edge-pass variants for the rank gather.  Built by scripts/lab/Makefile.
#include <hip/hip_runtime.h>
#include <stdint.h>

static constexpr uint32_t INV = 0xFFFFFFFFu;

template <bool NT>
__global__ void k_v(const uint2* __restrict__ uv, uint64_t m, const uint32_t* __restrict__ rank,
                    uint64_t* __restrict__ items, int gather) {
  uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += stride) {
    uint2 e;
    if (NT) {
      uint64_t w = __builtin_nontemporal_load((const uint64_t*)uv + i);
      e.x = (uint32_t)w; e.y = (uint32_t)(w >> 32);
    } else {
      e = uv[i];
    }
    uint32_t hi = INV, lo = INV;
    if (e.x != e.y) {
      uint32_t rx = gather ? rank[e.x] : e.x, ry = gather ? rank[e.y] : e.y;
      lo = min(rx, ry);
      hi = max(rx, ry);
    }
    uint64_t it = ((uint64_t)hi << 32) | lo;
    if (NT) __builtin_nontemporal_store(it, items + i); else items[i] = it;
  }
}

// U edges per thread per iteration (all loads issued before use)
template <int U, bool NT>
__global__ void k_u(const uint2* __restrict__ uv, uint64_t m, const uint32_t* __restrict__ rank,
                    uint64_t* __restrict__ items) {
  uint64_t nthr = (uint64_t)gridDim.x * blockDim.x;
  uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (uint64_t base = 0; base < m; base += nthr * U) {
    uint2 e[U];
    uint32_t rx[U], ry[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      uint64_t i = base + (uint64_t)u * nthr + tid;
      if (i < m) {
        if (NT) { uint64_t w = __builtin_nontemporal_load((const uint64_t*)uv + i); e[u].x = (uint32_t)w; e[u].y = (uint32_t)(w >> 32); }
        else e[u] = uv[i];
      } else { e[u].x = e[u].y = 0; }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) { rx[u] = rank[e[u].x]; ry[u] = rank[e[u].y]; }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      uint64_t i = base + (uint64_t)u * nthr + tid;
      if (i >= m) continue;
      uint32_t hi = INV, lo = INV;
      if (e[u].x != e[u].y) { lo = min(rx[u], ry[u]); hi = max(rx[u], ry[u]); }
      uint64_t it = ((uint64_t)hi << 32) | lo;
      if (NT) __builtin_nontemporal_store(it, items + i); else items[i] = it;
    }
  }
}

// 3-byte packed rank table: rank of id at bytes [3 id, 3 id + 3) of r3 (little endian),
// 0xFFFFFF = INVALID.
__device__ __forceinline__ uint32_t rank3(const uint8_t* r3, uint32_t id) {
  uint64_t a = 3ull * id;
  const uint32_t* w = (const uint32_t*)(r3 + (a & ~3ull));
  uint32_t sh = (uint32_t)(a & 3) * 8;
  uint64_t two = ((uint64_t)w[1] << 32) | w[0];
  uint32_t v = (uint32_t)(two >> sh) & 0xFFFFFFu;
  return v == 0xFFFFFFu ? INV : v;
}

template <bool NT>
__global__ void k_r3(const uint2* __restrict__ uv, uint64_t m, const uint8_t* __restrict__ r3,
                     uint64_t* __restrict__ items) {
  uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += stride) {
    uint2 e;
    if (NT) { uint64_t w = __builtin_nontemporal_load((const uint64_t*)uv + i); e.x = (uint32_t)w; e.y = (uint32_t)(w >> 32); }
    else e = uv[i];
    uint32_t hi = INV, lo = INV;
    if (e.x != e.y) {
      uint32_t rx = rank3(r3, e.x), ry = rank3(r3, e.y);
      lo = min(rx, ry);
      hi = max(rx, ry);
    }
    uint64_t it = ((uint64_t)hi << 32) | lo;
    if (NT) __builtin_nontemporal_store(it, items + i); else items[i] = it;
  }
}

__global__ void k_pack3(const uint32_t* __restrict__ rank, uint64_t n, uint8_t* r3) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    uint32_t r = rank[i];
    if (r == INV) r = 0xFFFFFFu;
    r3[3 * i] = (uint8_t)r; r3[3 * i + 1] = (uint8_t)(r >> 8); r3[3 * i + 2] = (uint8_t)(r >> 16);
  }
}

extern "C" int edge_lab(int variant, const void* uv, uint64_t m, const void* rank, const void* r3,
                        void* items, int grid, int block, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  const uint2* e = (const uint2*)uv;
  const uint32_t* r = (const uint32_t*)rank;
  uint64_t* it = (uint64_t*)items;
  switch (variant) {
    case 0: hipLaunchKernelGGL(k_v<false>, dim3(grid), dim3(block), 0, s, e, m, r, it, 1); break;
    case 1: hipLaunchKernelGGL(k_v<true>, dim3(grid), dim3(block), 0, s, e, m, r, it, 1); break;
    case 2: hipLaunchKernelGGL(k_v<false>, dim3(grid), dim3(block), 0, s, e, m, r, it, 0); break;
    case 3: hipLaunchKernelGGL(k_v<true>, dim3(grid), dim3(block), 0, s, e, m, r, it, 0); break;
    case 4: hipLaunchKernelGGL((k_u<4, false>), dim3(grid), dim3(block), 0, s, e, m, r, it); break;
    case 5: hipLaunchKernelGGL((k_u<4, true>), dim3(grid), dim3(block), 0, s, e, m, r, it); break;
    case 6: hipLaunchKernelGGL(k_r3<false>, dim3(grid), dim3(block), 0, s, e, m, (const uint8_t*)r3, it); break;
    case 7: hipLaunchKernelGGL(k_r3<true>, dim3(grid), dim3(block), 0, s, e, m, (const uint8_t*)r3, it); break;
    case 8: hipLaunchKernelGGL((k_u<8, true>), dim3(grid), dim3(block), 0, s, e, m, r, it); break;
    case 100: hipLaunchKernelGGL(k_pack3, dim3(2048), dim3(256), 0, s, r, m, (uint8_t*)items); break;
    default: return -1;
  }
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

// One-endpoint gather (rank[rec.y]) over records, one tile of 8192 records per block.
// xcd: 0 = tile = blockIdx; 1 = XCD-contiguous tiles (blockIdx % 8 picks the XCD's range).
__global__ void __launch_bounds__(1024) k_gather1(const uint2* __restrict__ uv, uint64_t m,
                                                  const uint32_t* __restrict__ rank,
                                                  uint64_t* __restrict__ out, int xcd, uint32_t ntiles) {
  uint32_t tile = blockIdx.x;
  if (xcd) {
    uint32_t per = (ntiles + 7) / 8;
    tile = (blockIdx.x % 8) * per + blockIdx.x / 8;
    if (tile >= ntiles) return;
  }
  uint64_t base = (uint64_t)tile * 8192 + threadIdx.x;
  uint2 e[8];
  uint32_t r[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) { uint64_t i = base + k * 1024; e[k] = i < m ? uv[i] : make_uint2(0, 0); }
#pragma unroll
  for (int k = 0; k < 8; ++k) r[k] = rank[e[k].y];
#pragma unroll
  for (int k = 0; k < 8; ++k) { uint64_t i = base + k * 1024; if (i < m) out[i] = ((uint64_t)e[k].x << 32) | r[k]; }
}

extern "C" int gather_lab(int xcd, const void* uv, uint64_t m, const void* rank, void* out, void* stream) {
  uint32_t nt = (uint32_t)((m + 8191) / 8192);
  uint32_t grid = xcd ? ((nt + 7) / 8) * 8 : nt;
  hipLaunchKernelGGL(k_gather1, dim3(grid), dim3(1024), 0, (hipStream_t)stream, (const uint2*)uv, m,
                     (const uint32_t*)rank, (uint64_t*)out, xcd, nt);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}
