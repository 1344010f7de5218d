// Synthetic edge streams for the benchmark configs: a Graph500-style Kronecker
// (R-MAT) generator, A/B/C/D = .57/.19/.19/.05, no per-level noise, seeded vertex relabelling.
//
// Everything is integer arithmetic on a counter-based RNG, so the HIP kernel (rmat.hip) and a
// host caller produce bit-identical edges for any slice [e_begin, e_end) of the stream.  That
// is what lets every rank of a multi-GPU run generate its own edge shard in HBM and lets the
// CPU checker regenerate the same input.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define SHEEP_HD __host__ __device__ __forceinline__
#else
#define SHEEP_HD static inline
#endif

namespace sheep_rmat {

SHEEP_HD uint64_t mix64(uint64_t z) {  // splitmix64 finaliser
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// Quadrant thresholds on a u32 draw: [0,TA) -> A, [TA,TB) -> B, [TB,TC) -> C, else D.
static const uint32_t TA = 2448131358u;  // floor(0.57 * 2^32)
static const uint32_t TB = 3264175144u;  // TA + floor(0.19 * 2^32)
static const uint32_t TC = 4080218930u;  // TB + floor(0.19 * 2^32)

// A bijection on [0, 2^scale): odd multiplies and right xor-shifts are each invertible mod 2^s.
SHEEP_HD uint32_t relabel(uint32_t x, int scale, uint64_t seed) {
  const uint64_t mask = (scale >= 32) ? 0xFFFFFFFFull : ((1ull << scale) - 1);
  uint64_t k1 = mix64(seed ^ 0x5EEDull), k2 = mix64(seed ^ 0xB0B0ull);
  uint64_t y = x;
  y = (y * 0x9E3779B1ull + k1) & mask;
  y ^= y >> ((scale + 1) / 2);
  y = (y * (0x85EBCA6Bull | 1ull) + k2) & mask;
  y ^= y >> (scale / 2 + 1);
  y = (y * 0xC2B2AE35ull) & mask;
  return (uint32_t)y;
}

// Edge e of the stream for (scale, seed): writes (tail, head).
SHEEP_HD void edge(uint64_t e, int scale, uint64_t seed, uint32_t* tail, uint32_t* head) {
  uint64_t state = mix64(seed * 0x9E3779B97F4A7C15ull + e);
  uint32_t row = 0, col = 0;
  uint64_t bits = 0;
  for (int l = 0; l < scale; ++l) {
    uint32_t r;
    if ((l & 1) == 0) {
      state += 0x9E3779B97F4A7C15ull;
      bits = mix64(state);
      r = (uint32_t)bits;
    } else {
      r = (uint32_t)(bits >> 32);
    }
    uint32_t rb = (r >= TB) ? 1u : 0u;                        // C or D: row bit
    uint32_t cb = ((r >= TA && r < TB) || r >= TC) ? 1u : 0u;  // B or D: column bit
    row |= rb << l;
    col |= cb << l;
  }
  *tail = relabel(row, scale, seed);
  *head = relabel(col, scale, seed);
}

}  // namespace sheep_rmat
