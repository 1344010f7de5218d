// Partition quality on the GPU: Partition::evaluate(graph) and evaluate(graph, seq)
// (partition.cpp:428-521) — edges cut, communication volume, ECV(hash), ECV(down), ECV(up) and
// their balances — for a k-way vertex partition of the edge records, exactly as the reference
// counts them over LLAMA's undirected adjacency (every record x != y is the two entries
// x -> y and y -> x; a self-loop is one entry x -> x; duplicates are kept).
//
// The reference walks each vertex's adjacency with an unordered_set of parts.  Here a metric's
// per-vertex distinct-part count is a distinct count over (X, part) keys: one key per
// adjacency entry, sorted by part then stably by X (the radix sort orders 32-bit fields), one
// pass counting key changes.
//   ECV(*)   = sum_X (|set_X| - 1)            = distinct keys - vertices with entries
//   Vcom_vol = sum_X (|{part X} ∪ nbr parts| - 1) = distinct keys with part != part(X)
// Balances and edges cut are per-record histograms over the k parts (LDS-privatised).
// All arithmetic is integer; results are bit-exact with the reference's.
// The s_waitcnt immediates below are gfx9 encodings (vmcnt bits [3:0] and [15:14], lgkmcnt
// [11:8]); on another target they would silently mean a different wait.
#if defined(__HIP_DEVICE_COMPILE__) && !defined(__gfx950__)
#error "sheep_amd kernels are written for gfx950 only"
#endif
#include <hip/hip_runtime.h>

#include "sheep_internal.h"

namespace sheep {

static constexpr int EV_BLOCK = 256;
static constexpr uint32_t EV_LDS_PARTS = 2048;  // LDS histograms up to this many parts
static constexpr uint32_t CORMEN_S = 2654435769u;  // floor((sqrt(5)-1)/2 * 2^32), partition.cpp:423

static inline unsigned ev_grid(uint64_t n) {
  uint64_t g = (n + EV_BLOCK - 1) / EV_BLOCK;
  return (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(g, 4096));
}

// ECV metric of an adjacency entry X -> Y: the part that the reference inserts in X's set.
enum { EV_VCOM = 0, EV_HASH = 1, EV_DOWN = 2, EV_UP = 3 };

template <int METRIC>
__device__ __forceinline__ uint64_t ev_key(uint32_t X, uint32_t Y, const int16_t* parts,
                                           const uint32_t* pos) {
  const uint32_t xp = (uint16_t)parts[X], yp = (uint16_t)parts[Y];
  uint32_t v;
  if (METRIC == EV_VCOM) {
    if (xp == yp) return ~0ull;  // X's own part is in its set anyway
    v = yp;
  } else if (METRIC == EV_HASH) {
    v = (X * CORMEN_S) < (Y * CORMEN_S) ? xp : yp;
  } else if (METRIC == EV_DOWN) {
    v = pos[X] < pos[Y] ? xp : yp;
  } else {
    v = pos[X] > pos[Y] ? xp : yp;
  }
  return ((uint64_t)v << 32) | X;  // the radix sort orders the high word: first by part
}

// Workgroup barrier that first drains the wave's LDS operations (see block_sync in
// sheep_kernels.hip: a plain __syncthreads() once lost no-return LDS adds on a loop exit).
__device__ __forceinline__ void ev_block_sync() {
  __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
  __syncthreads();
}

// (part << 32 | X) -> (X << 32 | part) between the two stable sorts; ~0 stays ~0.
__global__ void k_ev_swap(uint64_t* keys, uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t k = keys[i];
    keys[i] = (k << 32) | (k >> 32);
  }
}

// Two keys per record (slot 2e: x -> y, slot 2e + 1: y -> x, or ~0 for a self-loop).
template <int METRIC>
__global__ void k_ev_keys(const uint2* __restrict__ uv, uint64_t m, const int16_t* __restrict__ parts,
                          const uint32_t* __restrict__ pos, uint64_t* __restrict__ keys) {
  for (uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; e < m;
       e += (uint64_t)gridDim.x * blockDim.x) {
    const uint2 r = uv[e];
    keys[2 * e] = ev_key<METRIC>(r.x, r.y, parts, pos);
    keys[2 * e + 1] = r.x != r.y ? ev_key<METRIC>(r.y, r.x, parts, pos) : ~0ull;
  }
}

// The keys of the entries X -> Y with X in [v0, v1) only (a pass of an evaluation whose 2m
// entries exceed one sort), appended in any order at keys[*n_out ...] (wave-aggregated); the
// caller filled keys with ~0 up to the pass's bound.  Distinct keys of different passes differ
// in X, so the passes' distinct counts add up.
template <int METRIC>
__global__ void k_ev_keys_range(const uint2* __restrict__ uv, uint64_t m,
                                const int16_t* __restrict__ parts, const uint32_t* __restrict__ pos,
                                uint32_t v0, uint32_t v1, uint64_t* __restrict__ keys,
                                unsigned long long* n_out) {
  const int lane = threadIdx.x & 63;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t b = (uint64_t)blockIdx.x * blockDim.x; b < m; b += stride) {  // wave-uniform
    const uint64_t e = b + threadIdx.x;
    uint64_t k0 = ~0ull, k1 = ~0ull;
    if (e < m) {
      const uint2 r = uv[e];
      if (r.x >= v0 && r.x < v1) k0 = ev_key<METRIC>(r.x, r.y, parts, pos);
      if (r.x != r.y && r.y >= v0 && r.y < v1) k1 = ev_key<METRIC>(r.y, r.x, parts, pos);
    }
    const uint32_t c = (k0 != ~0ull) + (k1 != ~0ull);
    uint32_t inc = c;
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t v = __shfl_up(inc, o);
      if (lane >= o) inc += v;
    }
    const uint32_t tot = __shfl(inc, 63);
    unsigned long long base = 0;
    if (lane == 63 && tot) base = atomicAdd(n_out, (unsigned long long)tot);
    base = __shfl(base, 63);
    uint64_t at = base + inc - c;
    if (k0 != ~0ull) keys[at++] = k0;
    if (k1 != ~0ull) keys[at] = k1;
  }
}

// Number of distinct keys (~0 excluded) of a sorted array.
__global__ void k_ev_distinct(const uint64_t* __restrict__ keys, uint64_t n,
                              unsigned long long* out) {
  unsigned long long c = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t k = keys[i];
    c += k != ~0ull && (i == 0 || keys[i - 1] != k);
  }
  for (int o = 32; o > 0; o >>= 1) c += __shfl_down(c, o);
  if ((threadIdx.x & 63) == 0 && c) atomicAdd(out, c);
}

// Per record x != y: edges cut (parts differ), ECV(hash) balance (the hash part of the x < y
// entry), ECV(down) balance (part of the lower-position endpoint), ECV(up) balance (part of
// the higher).  Validity: ids < n_ids, parts in [0, k), positions valid.
// hist: 3 * k u64 (hash, down, up); cnt[0] = edges cut, cnt[1] = self-loop records.
__global__ void k_ev_records(const uint2* __restrict__ uv, uint64_t m, uint32_t n_ids,
                             const int16_t* __restrict__ parts, const uint32_t* __restrict__ pos,
                             uint32_t k, unsigned long long* hist, unsigned long long* cnt,
                             uint32_t* err) {
  __shared__ uint32_t lh[3 * EV_LDS_PARTS];
  const bool lds = k <= EV_LDS_PARTS;
  if (lds)
    for (uint32_t i = threadIdx.x; i < 3 * k; i += blockDim.x) lh[i] = 0;
  ev_block_sync();
  unsigned long long cut = 0, self = 0;
  for (uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; e < m;
       e += (uint64_t)gridDim.x * blockDim.x) {
    const uint2 r = uv[e];
    if (r.x >= n_ids || r.y >= n_ids) { atomicOr(err, ERR_RANGE); continue; }
    const int xs = parts[r.x], ys = parts[r.y];
    const uint32_t px = pos[r.x], py = pos[r.y];
    if (xs < 0 || ys < 0 || (uint32_t)xs >= k || (uint32_t)ys >= k || px == INV || py == INV) {
      atomicOr(err, ERR_RANGE);
      continue;
    }
    if (r.x == r.y) { ++self; continue; }
    cut += xs != ys;
    const uint32_t lo = min(r.x, r.y), hi = max(r.x, r.y);
    const uint32_t lop = (uint32_t)parts[lo], hip = (uint32_t)parts[hi];
    const uint32_t hp = (lo * CORMEN_S) < (hi * CORMEN_S) ? lop : hip;
    const uint32_t dp = px < py ? (uint32_t)xs : (uint32_t)ys;
    const uint32_t up = px < py ? (uint32_t)ys : (uint32_t)xs;
    if (lds) {
      atomicAdd(&lh[hp], 1u);
      atomicAdd(&lh[k + dp], 1u);
      atomicAdd(&lh[2 * k + up], 1u);
    } else {
      atomicAdd(&hist[hp], 1ull);
      atomicAdd(&hist[k + dp], 1ull);
      atomicAdd(&hist[2 * k + up], 1ull);
    }
  }
  for (int o = 32; o > 0; o >>= 1) { cut += __shfl_down(cut, o); self += __shfl_down(self, o); }
  if ((threadIdx.x & 63) == 0) {
    if (cut) atomicAdd(&cnt[0], cut);
    if (self) atomicAdd(&cnt[1], self);
  }
  if (lds) {
    ev_block_sync();
    for (uint32_t i = threadIdx.x; i < 3 * k; i += blockDim.x)
      if (lh[i]) atomicAdd(&hist[i], (unsigned long long)lh[i]);
  }
}

// Vertices with adjacency (deg > 0): their count and the vertex balance per part.
__global__ void k_ev_nodes(const uint32_t* __restrict__ deg, uint32_t n_ids,
                           const int16_t* __restrict__ parts, uint32_t k,
                           unsigned long long* vbal, unsigned long long* cnt, uint32_t* err) {
  __shared__ uint32_t lh[EV_LDS_PARTS];
  const bool lds = k <= EV_LDS_PARTS;
  if (lds)
    for (uint32_t i = threadIdx.x; i < k; i += blockDim.x) lh[i] = 0;
  ev_block_sync();
  unsigned long long nodes = 0;
  for (uint32_t v = blockIdx.x * blockDim.x + threadIdx.x; v < n_ids; v += gridDim.x * blockDim.x) {
    if (!deg[v]) continue;
    const int p = parts[v];
    if (p < 0 || (uint32_t)p >= k) { atomicOr(err, ERR_RANGE); continue; }
    ++nodes;
    if (lds) atomicAdd(&lh[p], 1u); else atomicAdd(&vbal[p], 1ull);
  }
  for (int o = 32; o > 0; o >>= 1) nodes += __shfl_down(nodes, o);
  if ((threadIdx.x & 63) == 0 && nodes) atomicAdd(&cnt[2], nodes);
  if (lds) {
    ev_block_sync();
    for (uint32_t i = threadIdx.x; i < k; i += blockDim.x)
      if (lh[i]) atomicAdd(&vbal[i], (unsigned long long)lh[i]);
  }
}

// ws: 4 * k + 8 u64.  keys / keys_b: 2m u64 each.  Returns after enqueueing; the caller reads
// ws (layout in sheep_eval_layout) after a sync.
void launch_evaluate(const uint32_t* uv, uint64_t m, const int16_t* parts, const uint32_t* pos,
                     const uint32_t* deg, uint32_t n_ids, uint32_t k, uint64_t* keys,
                     uint64_t* keys_b, uint32_t* rtmp, unsigned long long* ws, uint32_t* err,
                     hipStream_t s, const std::vector<std::pair<uint32_t, uint64_t>>* passes) {
  unsigned long long* hist = ws;             // [0, 3k): hash, down, up balances
  unsigned long long* vbal = ws + 3 * k;     // [3k, 4k)
  unsigned long long* cnt = ws + 4 * (uint64_t)k;  // cut, self, nodes, vcom, hash, down, up
  (void)hipMemsetAsync(ws, 0, (4 * (size_t)k + 8) * 8, s);
  hipLaunchKernelGGL(k_ev_records, dim3(ev_grid(m)), dim3(EV_BLOCK), 0, s, (const uint2*)uv, m,
                     n_ids, parts, pos, k, hist, cnt, err);
  hipLaunchKernelGGL(k_ev_nodes, dim3(ev_grid(n_ids)), dim3(EV_BLOCK), 0, s, deg, n_ids, parts, k,
                     vbal, cnt, err);
  int idb = 0;
  for (uint32_t v = n_ids ? n_ids - 1 : 0; v; v >>= 1) ++idb;
  // one more bit than the values need in each sort: a ~0 sentinel (missing second entry of a
  // self-loop, a Vcom entry inside X's own part) then sorts after every real key
  if (passes && !passes->empty()) {
    // passes: (first id, keys bound) of consecutive id ranges, the last one ending at n_ids
    unsigned long long* nk = cnt + 7;
    for (int metric = 0; metric < 4; ++metric)
      for (size_t p = 0; p < passes->size(); ++p) {
        const uint32_t v0 = (*passes)[p].first;
        const uint32_t v1 = p + 1 < passes->size() ? (*passes)[p + 1].first : n_ids;
        const uint64_t n = std::max<uint64_t>((*passes)[p].second, 1);
        auto kk = metric == EV_VCOM ? k_ev_keys_range<EV_VCOM>
                : metric == EV_HASH ? k_ev_keys_range<EV_HASH>
                : metric == EV_DOWN ? k_ev_keys_range<EV_DOWN> : k_ev_keys_range<EV_UP>;
        (void)hipMemsetAsync(keys, 0xFF, n * 8, s);
        (void)hipMemsetAsync(nk, 0, 8, s);
        hipLaunchKernelGGL(kk, dim3(ev_grid(m)), dim3(EV_BLOCK), 0, s, (const uint2*)uv, m, parts,
                           pos, v0, v1, keys, nk);
        uint64_t* by_part = radix_sort_u64(keys, keys_b, keys, n, 0, 16, rtmp, s);
        uint64_t* other = by_part == keys ? keys_b : keys;
        hipLaunchKernelGGL(k_ev_swap, dim3(ev_grid(n)), dim3(EV_BLOCK), 0, s, by_part, n);
        const uint64_t* sorted = radix_sort_u64(by_part, other, by_part, n, 0, idb + 1, rtmp, s);
        hipLaunchKernelGGL(k_ev_distinct, dim3(ev_grid(n)), dim3(EV_BLOCK), 0, s, sorted, n,
                           cnt + 3 + metric);
      }
    return;
  }
  const uint64_t n = 2 * m;
  for (int metric = 0; metric < 4; ++metric) {
    auto kk = metric == EV_VCOM ? k_ev_keys<EV_VCOM>
            : metric == EV_HASH ? k_ev_keys<EV_HASH>
            : metric == EV_DOWN ? k_ev_keys<EV_DOWN> : k_ev_keys<EV_UP>;
    hipLaunchKernelGGL(kk, dim3(ev_grid(m)), dim3(EV_BLOCK), 0, s, (const uint2*)uv, m, parts, pos,
                       keys);
    uint64_t* by_part = radix_sort_u64(keys, keys_b, keys, n, 0, 16, rtmp, s);
    uint64_t* other = by_part == keys ? keys_b : keys;
    hipLaunchKernelGGL(k_ev_swap, dim3(ev_grid(n)), dim3(EV_BLOCK), 0, s, by_part, n);
    const uint64_t* sorted = radix_sort_u64(by_part, other, by_part, n, 0, idb + 1, rtmp, s);
    hipLaunchKernelGGL(k_ev_distinct, dim3(ev_grid(n)), dim3(EV_BLOCK), 0, s, sorted, n,
                       cnt + 3 + metric);
  }
}

// ---- graph2tree -p K -o OUT: the records of each part (writePartitionedGraph, partition.cpp:
// 588-630).  The reference walks the graph node by node (X ascending) and writes every edge
// (X, Y) with X < Y to the part of its lower-sequence endpoint, so a part's file lists its
// edges by X, each X's in adjacency order (record order for EdgeGraph); self-loops are skipped.
// Here: key (X, record) sorted stably by X, re-keyed (part, record) and sorted stably by part:
// the records come out grouped by part, each part in the writer's order.
__global__ void k_pe_keys(const uint2* __restrict__ uv, uint64_t m, uint32_t n_ids, uint64_t* items) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m;
       i += (uint64_t)gridDim.x * blockDim.x) {
    const uint2 e = uv[i];
    const uint32_t x = e.x == e.y ? n_ids : min(e.x, e.y);  // n_ids: self-loops sort last
    items[i] = ((uint64_t)x << 32) | (uint32_t)i;
  }
}

__global__ void k_pe_part_keys(const uint64_t* __restrict__ sorted, uint64_t m,
                               const uint2* __restrict__ uv, const int16_t* __restrict__ parts,
                               const uint32_t* __restrict__ pos, uint32_t n_ids, uint32_t n_parts,
                               uint64_t* items, uint32_t* err) {
  for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < m;
       j += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t it = sorted[j];
    const uint32_t i = (uint32_t)it;
    uint32_t p = n_parts;  // self-loops: after every part
    if ((uint32_t)(it >> 32) != n_ids) {
      const uint2 e = uv[i];
      const uint32_t x = min(e.x, e.y), y = max(e.x, e.y);
      if (y >= n_ids) { atomicOr(err, ERR_RANGE); continue; }
      const int16_t q = pos[x] < pos[y] ? parts[x] : parts[y];
      if (q < 0 || (uint32_t)q >= n_parts) atomicOr(err, ERR_RANGE);  // a vertex without a part
      else p = (uint32_t)q;
    }
    items[j] = ((uint64_t)p << 32) | i;
  }
}

// out: the (X, Y) pairs in order; pstart[q] (q <= n_parts) = first position of part q.
__global__ void k_pe_emit(const uint64_t* __restrict__ sorted, uint64_t m, const uint2* __restrict__ uv,
                          uint32_t n_parts, uint2* out, unsigned long long* pstart) {
  for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j <= m;
       j += (uint64_t)gridDim.x * blockDim.x) {
    const int64_t prev = j ? (int64_t)(sorted[j - 1] >> 32) : -1;
    const int64_t cur = j < m ? (int64_t)(sorted[j] >> 32) : (int64_t)n_parts + 1;
    for (int64_t q = prev + 1; q <= cur && q <= (int64_t)n_parts; ++q) pstart[q] = j;
    if (j < m && cur < (int64_t)n_parts) {
      const uint2 e = uv[(uint32_t)sorted[j]];
      out[j] = make_uint2(min(e.x, e.y), max(e.x, e.y));
    }
  }
}

void launch_partition_edges(const uint32_t* uv, uint64_t m, const int16_t* parts, const uint32_t* pos,
                            uint32_t n_ids, uint32_t n_parts, uint64_t* items, uint64_t* items_b,
                            uint32_t* rtmp, uint32_t* out, unsigned long long* pstart, uint32_t* err,
                            hipStream_t s) {
  int xb = 0, pb = 0;
  for (uint32_t v = n_ids; v; v >>= 1) ++xb;    // keys <= n_ids
  for (uint32_t v = n_parts; v; v >>= 1) ++pb;  // keys <= n_parts
  hipLaunchKernelGGL(k_pe_keys, dim3(ev_grid(m)), dim3(EV_BLOCK), 0, s, (const uint2*)uv, m, n_ids,
                     items);
  const uint64_t* by_x = radix_sort_u64(items, items_b, items, m, 0, xb, rtmp, s);
  uint64_t* other = by_x == items ? items_b : items;
  hipLaunchKernelGGL(k_pe_part_keys, dim3(ev_grid(m)), dim3(EV_BLOCK), 0, s, by_x, m,
                     (const uint2*)uv, parts, pos, n_ids, n_parts, other, err);
  const uint64_t* by_part = radix_sort_u64(other, other == items ? items_b : items, other, m, 0, pb,
                                           rtmp, s);
  hipLaunchKernelGGL(k_pe_emit, dim3(ev_grid(m + 1)), dim3(EV_BLOCK), 0, s, by_part, m,
                     (const uint2*)uv, n_parts, (uint2*)out, pstart);
}

}  // namespace sheep
