// Synthetic power-law edge streams for the LiveJournal-shape and twitter-shape configs
// (BASELINE.json configs C3 and C5): a Chung-Lu style stream where each endpoint is
// drawn independently with P(i) proportional to (i + i0)^-beta, beta = 1 / (gamma - 1), and the
// vertex ids are then relabelled by a seeded bijection of [0, n).
//
// The draw is integer-only so that the HIP kernel and a host caller give bit-identical edges
// for any slice of the stream (as rmat.h): the index space is cut into levels
// [2^L - 1, 2^(L+1) - 1) (level 0 = vertex 0), a first u32 picks the level against cumulative
// thresholds, a second the vertex uniformly inside it — a step approximation of the power law
// with exact geometric weights.  Only the threshold table is computed in floating point, on the
// host, once (powerlaw_table); the table is then plain data for both sides.
#pragma once
#include <math.h>
#include <stdint.h>

#include "rmat.h"

namespace sheep_pl {

static const int MAX_LEVELS = 33;

struct Table {
  uint32_t n = 0;         // vertices
  int levels = 0;         // level L covers [2^L - 1, min(2^(L+1) - 1, n))
  int sbits = 0;          // 2^sbits >= n: relabelling by cycle-walking a bijection of 2^sbits
  uint64_t thr[MAX_LEVELS] = {};  // cumulative, scaled to 2^32 (thr[levels-1] == 2^32)
};

// Host only: the level weights sum (i + i0)^-beta over each level exactly (levels are short
// near the head) or by the integral of the continuous density (long levels).
static inline Table powerlaw_table(uint32_t n, double gamma, double i0) {
  Table t;
  t.n = n;
  while ((1ull << t.sbits) < n) ++t.sbits;
  if (n == 0) return t;
  const double beta = 1.0 / (gamma - 1.0);
  double w[MAX_LEVELS] = {}, total = 0;
  int L = 0;
  for (; L < MAX_LEVELS; ++L) {
    uint64_t lo = (1ull << L) - 1, hi = (2ull << L) - 1;
    if (lo >= n) break;
    if (hi > n) hi = n;
    double s = 0;
    if (hi - lo <= 4096) {
      for (uint64_t i = lo; i < hi; ++i) s += pow((double)i + i0, -beta);
    } else {  // integral of (x + i0)^-beta over [lo - 0.5, hi - 0.5]
      double a = (double)lo - 0.5 + i0, b = (double)hi - 0.5 + i0;
      s = (fabs(beta - 1.0) < 1e-12) ? log(b / a) : (pow(b, 1 - beta) - pow(a, 1 - beta)) / (1 - beta);
    }
    w[L] = s;
    total += s;
  }
  t.levels = L;
  double cum = 0;
  for (int l = 0; l < L; ++l) {
    cum += w[l];
    t.thr[l] = (uint64_t)floor(cum / total * 4294967296.0);
  }
  t.thr[L - 1] = 1ull << 32;
  return t;
}

SHEEP_HD uint32_t draw(const Table& t, uint64_t bits) {
  const uint32_t r = (uint32_t)bits;
  int L = 0;
  while (L + 1 < t.levels && (uint64_t)r >= t.thr[L]) ++L;
  const uint64_t lo = (1ull << L) - 1;
  uint64_t hi = (2ull << L) - 1;
  if (hi > t.n) hi = t.n;
  const uint64_t off = ((bits >> 32) * (hi - lo)) >> 32;
  return (uint32_t)(lo + off);
}

// The seeded bijection of [0, n): rmat's bijection of [0, 2^sbits), walked until it lands
// inside [0, n) (it permutes a superset, so every cycle returns into [0, n)).
SHEEP_HD uint32_t relabel(const Table& t, uint32_t x, uint64_t seed) {
  if (t.sbits == 0) return x;
  uint32_t y = sheep_rmat::relabel(x, t.sbits, seed);
  while (y >= t.n) y = sheep_rmat::relabel(y, t.sbits, seed);
  return y;
}

// Edge e of the stream for (table, seed): writes (tail, head).
SHEEP_HD void edge(const Table& t, uint64_t e, uint64_t seed, uint32_t* tail, uint32_t* head) {
  uint64_t s = sheep_rmat::mix64(seed * 0xD1B54A32D192ED03ull + e);
  uint64_t b1 = sheep_rmat::mix64(s + 0x9E3779B97F4A7C15ull);
  uint64_t b2 = sheep_rmat::mix64(s + 2 * 0x9E3779B97F4A7C15ull);
  *tail = relabel(t, draw(t, b1), seed);
  *head = relabel(t, draw(t, b2), seed);
}

}  // namespace sheep_pl
