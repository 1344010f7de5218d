// The C-ABI (include/sheep_amd.h) over the HIP kernels in sheep_kernels.hip.
//
// Error model: every entry point catches everything, stores the text in a thread-local string
// and returns a negative errno.  Device scratch is owned per device by a Ctx and grows on
// demand; the hot path allocates nothing after its first call at a given size.
#include <errno.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <cmath>
#include <memory>
#include <chrono>
#include <mutex>
#include <thread>
#include <stdexcept>
#include <string>
#include <tuple>
#include <vector>

#include "../../include/sheep_amd.h"
#include "sheep_comm.h"
#include "sheep_internal.h"

namespace sheep {

static thread_local std::string g_last_error;
void set_last_error(const char* msg) { g_last_error = msg; }
static thread_local int g_device = -1;
static Ctx g_ctx[64];
static std::mutex g_mu;

// ---- options (sheep_internal.h Knobs): SHEEP_<NAME> once, then sheep_set_option ----------
struct KnobDef {
  const char* name;
  int Knobs::*field;
};
static const KnobDef kKnobs[] = {
    {"degree", &Knobs::degree},           {"edge_part", &Knobs::edge_part},
    {"part_overlap", &Knobs::part_overlap},
    {"kb_buckets", &Knobs::kb_buckets},   {"kb_rankb", &Knobs::kb_rankb},
    {"kb_pipe", &Knobs::kb_pipe},         {"tree_stats", &Knobs::tree_stats},
    {"bin_direct", &Knobs::bin_direct},   {"bin_slack", &Knobs::bin_slack},
    {"kb_gsum", &Knobs::kb_gsum},         {"eval_pass", &Knobs::eval_pass},
    {"ls_split", &Knobs::ls_split},       {"ls_seq", &Knobs::ls_seq},
    {"kb_merge", &Knobs::kb_merge},       {"ff_groups", &Knobs::ff_groups},
    {"kb_rlink", &Knobs::kb_rlink},
    {"kb_fresh_lo", &Knobs::kb_fresh_lo}, {"kb_fresh_hi", &Knobs::kb_fresh_hi},
};

static Knobs g_knobs;
// the fused front pass's tile groups (Knobs::ff_groups), clamped to 1..8
static uint32_t ff_groups();
static std::once_flag g_knobs_once;

static void load_knobs_from_env() {
  for (const KnobDef& d : kKnobs) {
    std::string env = "SHEEP_";
    for (const char* q = d.name; *q; ++q) env += (char)toupper(*q);
    const char* v = getenv(env.c_str());
    if (!v) continue;
    if (d.field == &Knobs::degree)  // "atomic" / "bucketed" (or the number)
      g_knobs.degree = !strcmp(v, "atomic") ? 1 : !strcmp(v, "bucketed") ? 2 : atoi(v);
    else
      g_knobs.*d.field = atoi(v);
  }
}

Knobs& knobs() {
  std::call_once(g_knobs_once, load_knobs_from_env);
  return g_knobs;
}

static uint32_t ff_groups() { return (uint32_t)std::max(1, std::min(8, knobs().ff_groups)); }

struct HipError : std::runtime_error {
  using std::runtime_error::runtime_error;
};
struct ApiError : std::runtime_error {
  int code;
  ApiError(int c, const std::string& s) : std::runtime_error(s), code(c) {}
};

#define HIP_CHECK(x)                                                                          \
  do {                                                                                        \
    hipError_t e_ = (x);                                                                      \
    if (e_ != hipSuccess)                                                                     \
      throw HipError(std::string(#x) + ": " + hipGetErrorString(e_));                         \
  } while (0)

// SHEEP_SCRATCH_LOG=1: every allocation's name, address and size on stderr (diagnostics: where
// the big buffers land, DESIGN.md §9 "run-to-run spread").
static bool scratch_log() {
  static const bool on = getenv("SHEEP_SCRATCH_LOG") && atoi(getenv("SHEEP_SCRATCH_LOG")) != 0;
  return on;
}

static void scratch_alloc(void** p, size_t bytes, const char* name) {
  HIP_CHECK(hipMalloc(p, bytes));
  if (scratch_log())
    fprintf(stderr, "scratch %s %p %zu (2MB-aligned %d)\n", name, *p, bytes,
            (int)(((uintptr_t)*p & ((2u << 20) - 1)) == 0));
}

void* Scratch::get(const char* name, size_t bytes) {
  if (bytes == 0) bytes = 4;
  for (auto& s : slots) {
    if (s.first == name) {
      if (s.second.bytes >= bytes) return s.second.p;
      HIP_CHECK(hipFree(s.second.p));
      s.second.p = nullptr;
      s.second.bytes = 0;
      scratch_alloc(&s.second.p, bytes, name);
      s.second.bytes = bytes;
      return s.second.p;
    }
  }
  Slot sl;
  scratch_alloc(&sl.p, bytes, name);
  sl.bytes = bytes;
  slots.emplace_back(name, sl);
  return sl.p;
}

size_t Scratch::bytes_of(const char* name) const {
  for (auto& s : slots)
    if (s.first == name) return s.second.bytes;
  return 0;
}

void Scratch::release() {
  for (auto& s : slots)
    if (s.second.p) (void)hipFree(s.second.p);
  slots.clear();
}

// Streams, events and pinned words of a context (a device's, or a rehearsal rank thread's).
static void ctx_setup(Ctx& c, int device) {
  {
    HIP_CHECK(hipStreamCreateWithFlags(&c.stream, hipStreamNonBlocking));
    HIP_CHECK(hipStreamCreateWithFlags(&c.side, hipStreamNonBlocking));
    for (auto& e : c.kb_ev) HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    for (auto& e : c.part_ev) HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    HIP_CHECK(hipEventCreateWithFlags(&c.bins_ev, hipEventDisableTiming));
    HIP_CHECK(hipHostMalloc((void**)&c.h_bstart, 513 * 8, hipHostMallocDefault));
    HIP_CHECK(hipMalloc(&c.d_err, 16));
    HIP_CHECK(hipMemset(c.d_err, 0, 16));
    HIP_CHECK(hipHostMalloc(&c.h_pinned, 64, hipHostMallocDefault));
    c.device = device;
  }
}

static void ctx_teardown(Ctx& c) {
  c.scratch.release();
  (void)hipStreamDestroy(c.stream);
  (void)hipStreamDestroy(c.side);
  for (auto& e : c.kb_ev) (void)hipEventDestroy(e);
  for (auto& e : c.part_ev) (void)hipEventDestroy(e);
  (void)hipEventDestroy(c.bins_ev);
  for (hipEvent_t e : c.ev_pool) (void)hipEventDestroy(e);
  c.ev_pool.clear();
  (void)hipHostFree(c.h_bstart);
  if (c.h_chunks) (void)hipHostFree(c.h_chunks);
  (void)hipFree(c.d_err);
  (void)hipHostFree(c.h_pinned);
}

static Ctx& init_ctx(int device) {
  if (device < 0 || device >= 64) throw ApiError(-EINVAL, "device index out of range");
  std::lock_guard<std::mutex> lk(g_mu);
  Ctx& c = g_ctx[device];
  (void)knobs();  // the environment is read once, here
  HIP_CHECK(hipSetDevice(device));
  if (c.device < 0) ctx_setup(c, device);
  g_device = device;
  return c;
}

Ctx& ctx() {
  if (g_device < 0) {
    int d = 0;
    HIP_CHECK(hipGetDevice(&d));
    return init_ctx(d);
  }
  HIP_CHECK(hipSetDevice(g_device));
  return g_ctx[g_device];
}

// Device-pointer calls run on the caller's stream; NULL is HIP's default (null) stream, as
// for any HIP API (torch's default stream handle is 0).  Host-pointer calls use c.stream.
static hipStream_t pick(Ctx& c, void* stream) {
  (void)c;
  return (hipStream_t)stream;
}

// Phase timing with HIP events on the working stream.  The events come from the context's
// pool and go back to it (creating and destroying ~120 events per graph2tree call cost about
// 0.4 ms of host time, the destruction after the GPU had finished).
struct Timer {
  hipStream_t s;
  std::vector<hipEvent_t>* pool;
  std::vector<std::pair<const char*, hipEvent_t>> ev;
  std::mutex* mu;
  explicit Timer(hipStream_t st) : s(st), pool(&ctx().ev_pool), mu(&ctx().ev_mu) { mark("start"); }
  hipEvent_t take() {
    std::lock_guard<std::mutex> lk(*mu);
    if (pool->empty()) {
      hipEvent_t e;
      HIP_CHECK(hipEventCreate(&e));
      return e;
    }
    hipEvent_t e = pool->back();
    pool->pop_back();
    return e;
  }
  // host-side durations (ms), reported after the device phases
  std::vector<std::pair<const char*, double>> host;
  void host_ms(const char* name, double ms) { host.emplace_back(name, ms); }
  void mark(const char* name) {
    hipEvent_t e = take();
    HIP_CHECK(hipEventRecord(e, s));
    ev.emplace_back(name, e);
  }
  // Kernel spans on any stream (events right before and after one launch), summed per name
  // in finish(): "<name>" = total ms, "<name>#" = launches.
  std::vector<std::tuple<const char*, hipEvent_t, hipEvent_t>> spans;
  size_t span_begin(const char* name, hipStream_t st) {
    hipEvent_t a = take(), b = take();
    HIP_CHECK(hipEventRecord(a, st));
    spans.emplace_back(name, a, b);
    return spans.size() - 1;
  }
  void span_end(size_t i, hipStream_t st) { HIP_CHECK(hipEventRecord(std::get<2>(spans[i]), st)); }
  void finish(Ctx& c) {  // after the stream has been synchronised
    c.timings.clear();
    c.span_names.clear();
    for (size_t i = 1; i < ev.size(); ++i) {
      float ms = 0;
      (void)hipEventElapsedTime(&ms, ev[i - 1].second, ev[i].second);
      c.timings.emplace_back(ev[i].first, (double)ms);
    }
    std::vector<std::pair<const char*, std::pair<double, double>>> sums;
    for (auto& sp : spans) {
      float ms = 0;
      (void)hipEventElapsedTime(&ms, std::get<1>(sp), std::get<2>(sp));
      size_t j = 0;
      while (j < sums.size() && strcmp(sums[j].first, std::get<0>(sp))) ++j;
      if (j == sums.size()) sums.push_back({std::get<0>(sp), {0.0, 0.0}});
      sums[j].second.first += ms;
      sums[j].second.second += 1;
    }
    for (auto& x : sums) {
      c.timings.emplace_back(x.first, x.second.first);
      c.span_names.push_back(std::string(x.first) + "#");
      c.timings.emplace_back(c.span_names.back().c_str(), x.second.second);
    }
    for (auto& x : host) c.timings.push_back(x);
  }
  ~Timer() {  // (a recorded event may be re-recorded: the pool holds them for the next call)
    std::lock_guard<std::mutex> lk(*mu);
    for (auto& e : ev) pool->push_back(e.second);
    for (auto& sp : spans) {
      pool->push_back(std::get<1>(sp));
      pool->push_back(std::get<2>(sp));
    }
  }
};

// The walk guards' fault bits (sheep_kernels.hip FAULT_*).
static const char* fault_text(uint32_t f) {
  return (f & 1) ? "forest not heap-ordered"
         : (f & 4) ? "kept pairs past their buffer"
                   : "union-find cycle";
}

// Read and clear the device error word (synchronises s).
static void check_err(Ctx& c, hipStream_t s) {
  HIP_CHECK(hipMemcpyAsync(c.h_pinned, c.d_err, 4, hipMemcpyDeviceToHost, s));
  uint32_t* fw = fault_word();  // the device's walk guard (sheep_kernels.hip)
  if (fw) HIP_CHECK(hipMemcpyAsync(c.h_pinned + 12, fw, 4, hipMemcpyDeviceToHost, s));
  HIP_CHECK(hipStreamSynchronize(s));
  uint32_t e = c.h_pinned[0];
  if (fw && c.h_pinned[12]) {
    const uint32_t f = c.h_pinned[12];
    HIP_CHECK(hipMemsetAsync(fw, 0, 4, s));
    HIP_CHECK(hipStreamSynchronize(s));
    throw ApiError(-EIO, std::string("device walk guard tripped (") + fault_text(f) +
                             "): corrupt intermediate data");
  }
  if (e) {
    HIP_CHECK(hipMemsetAsync(c.d_err, 0, 4, s));
    HIP_CHECK(hipStreamSynchronize(s));
    if (e & ERR_DUP_SEQ) throw ApiError(-EINVAL, "sequence repeats a vertex id");
    if (e & ERR_RANGE) throw ApiError(-ERANGE, "vertex id out of range of the sequence/id space");
  }
}

// check_err for a group: every rank's error word and walk guard, MAX-reduced over the ranks, so
// that a fault on one rank (whose corrupt forest the parent sum hands to all) fails the call on
// every rank, after the same collectives.  Synchronises s.
static void check_err_group(Ctx& c, Comm& comm, hipStream_t s) {
  uint32_t* fw = fault_word();
  HIP_CHECK(hipMemcpyAsync(c.h_pinned, c.d_err, 4, hipMemcpyDeviceToHost, s));
  c.h_pinned[12] = 0;
  if (fw) HIP_CHECK(hipMemcpyAsync(c.h_pinned + 12, fw, 4, hipMemcpyDeviceToHost, s));
  HIP_CHECK(hipStreamSynchronize(s));
  int64_t h = ((int64_t)c.h_pinned[12] << 32) | c.h_pinned[0];
  if (comm.size() > 1) {
    int64_t* d = (int64_t*)c.scratch.get("mt_err", 8);
    HIP_CHECK(hipMemcpyAsync(d, &h, 8, hipMemcpyHostToDevice, s));
    comm.allreduce_max_i64(d, 1, s);
    HIP_CHECK(hipMemcpyAsync(&h, d, 8, hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipStreamSynchronize(s));
  }
  if (h == 0) return;
  HIP_CHECK(hipMemsetAsync(c.d_err, 0, 4, s));
  if (fw) HIP_CHECK(hipMemsetAsync(fw, 0, 4, s));
  HIP_CHECK(hipStreamSynchronize(s));
  const uint32_t f = (uint32_t)(h >> 32), e = (uint32_t)h;
  if (f)
    throw ApiError(-EIO, std::string("device walk guard tripped on a rank (") + fault_text(f) +
                             "): corrupt intermediate data");
  if (e & ERR_DUP_SEQ) throw ApiError(-EINVAL, "sequence repeats a vertex id");
  throw ApiError(-ERANGE, "vertex id out of range of the sequence/id space");
}

// Counters, tile offsets and kept-pair positions of the tree build are u32 (records), and the
// degree pass's endpoint offsets are u32 (2 per record): reject inputs beyond them.
static void require_records(uint64_t m, const char* what) {
  if (m >= (1ull << 32))
    throw ApiError(-EINVAL, std::string(what) + ": at most 2^32 - 1 records (u32 offsets)");
}
static void require_endpoints(uint64_t m, const char* what) {
  if (2 * m >= (1ull << 32))
    throw ApiError(-EINVAL, std::string(what) + ": at most 2^31 - 1 records (u32 endpoint offsets)");
}

static inline int bits_for(uint64_t v) {  // number of significant bits
  int b = 0;
  while (v) { ++b; v >>= 1; }
  return b;
}

// The device copy of host records: a registered range's, else one upload into "h_uv".
static uint32_t* upload_records(Ctx& c, const uint32_t* edges_uv, uint64_t m, hipStream_t s) {
  for (const Ctx::Registered& r : c.registered)
    if (r.host == edges_uv && r.m == m) return r.dev;
  uint32_t* uv = (uint32_t*)c.scratch.get("h_uv", std::max<uint64_t>(8 * m, 8));
  if (m) HIP_CHECK(hipMemcpyAsync(uv, edges_uv, 8 * m, hipMemcpyHostToDevice, s));
  return uv;
}

// ---- device-level building blocks ---------------------------------------------------------

// Degree: LDS-bucketed histogram for large inputs, global atomics for small ones.
// Returns true when the bucketed path also counted the rank-gather partition's y digits into
// the "part_ws" scratch (yhist).
static bool degree_dev(Ctx& c, const uint32_t* d_uv, uint64_t m, uint32_t n_ids, int mode,
                       uint32_t* d_deg, uint32_t* d_selfc, hipStream_t s, bool want_yhist = false,
                       hipEvent_t counted = nullptr, uint32_t* stats = nullptr) {
  const int kd = knobs().degree;
  bool bucketed = kd == 0 ? m >= (1ull << 18) : kd == 2;
  if (!bucketed || n_ids == 0) {
    launch_degree(d_uv, m, n_ids, mode, d_deg, d_selfc, c.d_err, s);
    if (stats) launch_deg_stats(d_deg, n_ids, stats, s);
    return false;
  }
  if (2 * m >= (1ull << 32) && fh_tmp_words(m, n_ids) > 1) {
    // beyond the endpoint array's u32 offsets: the fused pass, whose offsets count records
    // (it also writes the records grouped by y bucket, into scratch here)
    require_records(m, "degree");
    uint32_t* tmp = (uint32_t*)c.scratch.get("degb_tmp", fh_tmp_words(m, n_ids) * 4);
    uint64_t* recs = (uint64_t*)c.scratch.get("e_items", m * 8);
    uint32_t* pws = (uint32_t*)c.scratch.get("part_ws", PART_WS_WORDS * 4);
    uint32_t* st = stats ? stats : (uint32_t*)c.scratch.get("stats", 16);
    launch_fh_front(d_uv, m, n_ids, mode, d_deg, d_selfc, c.d_err, tmp, recs, pws, st, s);
    if (counted) HIP_CHECK(hipEventRecord(counted, s));
    return false;
  }
  // (ids beyond 2^26: launch_degree_bucketed takes the global-atomic pass, no offsets)
  if (degb_tmp_words(m, n_ids, nullptr, nullptr) > 1) require_endpoints(m, "degree");
  uint32_t* tmp = (uint32_t*)c.scratch.get("degb_tmp", degb_tmp_words(m, n_ids, nullptr, nullptr) * 4);
  uint32_t* yhist = want_yhist ? (uint32_t*)c.scratch.get("part_ws", PART_WS_WORDS * 4) : nullptr;
  return launch_degree_bucketed(d_uv, m, n_ids, mode, d_deg, d_selfc, c.d_err, tmp, s, yhist,
                                counted, stats);
}

// Optional degree information for pst without per-edge atomics (launch_pst_from_degree).
struct DegInfo {
  const uint32_t* seq = nullptr;    // jnid -> vid
  const uint32_t* deg = nullptr;    // degrees of THESE records
  const uint32_t* selfc = nullptr;  // self-loop records per vid
  int mode = SHEEP_DEGREE_LLAMA;
  bool yhist_ready = false;         // degree_dev counted the partition's y digits (part_ws)
  const uint32_t* nsd = nullptr;    // rank-ordered deg - w * selfc (nullable, see sequence_dev)
  bool part_first_done = false;     // the first partition pass was launched on c.side into
                                    // e_items; c.part_ev[1] marks its end
  uint64_t mid_slots = 0;           // ... of which e_items holds this many (0: m)
  bool mid_caps = false;            // ... into capacity regions (launch_part_first_caps): its
                                    // overflow word is c.d_err[3]
  bool mid_p6 = false;              // ... packed by the fused front pass (launch_front_fused)
  bool ids_checked = false;         // an id >= n_rank fails the call anyway (the degree pass's
                                    // ERR_RANGE): the partition passes may pack (part_p6_ok)
};

// Rank gathers in partitioned order (launch_part_gather) for large inputs.
static bool use_part(uint64_t m) {
  const int ep = knobs().edge_part;
  return ep < 0 ? m >= (1ull << 22) : ep != 0;
}

// stats_ready: the degree pass already wrote max degree / zero-degree count to "stats".
// nsd (nullable, n_ids words): rank-ordered non-self-loop degrees (k_unpack_seq) for these
// same records' selfc / mode.
// stats_host: ... and they are already in c.h_pinned[0..1] (read back with another word).
static uint32_t sequence_dev(Ctx& c, const uint32_t* d_deg, uint32_t n_ids, uint32_t* d_seq,
                             uint32_t* d_rank, hipStream_t s, bool stats_ready = false,
                             uint32_t* nsd = nullptr, const uint32_t* selfc = nullptr,
                             int mode = 0, bool stats_host = false) {
  if (n_ids == 0) return 0;
  uint32_t* stats = (uint32_t*)c.scratch.get("stats", 16);
  if (!stats_ready) launch_deg_stats(d_deg, n_ids, stats, s);
  if (!stats_host) {
    HIP_CHECK(hipMemcpyAsync(c.h_pinned, stats, 12, hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipStreamSynchronize(s));
  }
  // max degree, zero-degree ids, ids of degree >= seqc_threshold() (the radix-sorted tail)
  const uint32_t maxdeg = c.h_pinned[0], zeros = c.h_pinned[1], n_big = c.h_pinned[2];
  uint32_t n_seq = n_ids - zeros;
  if (n_seq == 0) {
    if (d_rank) launch_fill(d_rank, INV, n_ids, s);
    return 0;
  }
  // counting sort by degree classes; radix sort only for the ids of degree >= 1024
  uint32_t* qtmp = (uint32_t*)c.scratch.get("seqc_tmp", seqc_tmp_words(n_ids) * 4);
  uint64_t* big = (uint64_t*)c.scratch.get("seq_items", (size_t)n_seq * 8);
  const uint32_t* sc = nsd ? selfc : nullptr;  // the self-loop records off nsd in place
  const uint32_t* first = launch_seqc_place(d_deg, n_ids, d_seq, d_rank, nsd, big, qtmp, s, sc, mode);
  (void)first;  // (its first position is n_seq - n_big: no readback)
  if (maxdeg >= seqc_threshold()) {
    if (n_big == 0 || n_big > n_seq) throw ApiError(-EIO, "sequence: degree stats disagree");
    const uint32_t base = n_seq - n_big;
    uint64_t* big_b = (uint64_t*)c.scratch.get("seq_items_b", (size_t)n_big * 8);
    uint32_t* tmp = (uint32_t*)c.scratch.get("rsort_tmp", rsort_tmp_words(n_big) * 4);
    uint64_t* sorted = radix_sort_u64(big, big_b, big, n_big, 0, bits_for(maxdeg), tmp, s);
    launch_unpack_seq(sorted, 0, n_big, d_seq, d_rank, s, nsd, sc, mode, base);
  }
  return n_seq;
}

// Liu's elimination tree from items sorted by hi down to groups of 2^lo_bit ranks (m items,
// INVALID his last): the kb bucket loop.  parent: n_seq words, INVALID
// filled; jump: n_seq zeroed words; spare: m free u64 (kept pairs); hcnt: nullable hi counts.
// Bucket boundaries (rank, first record) of a kb loop, ending with (n_seq, m_valid).
using Buckets = std::vector<std::pair<uint32_t, uint64_t>>;

// kb bucket counts: each bucket costs a fixed ~60-100 us of launches and small kernels, while
// too few buckets leave the zipper long in-bucket walks (profiles/r01/kb_bucket_sweep.txt).
// kmax = 40 (below ~40 a bucket's in-bucket walks grow long, above it the fixed per-bucket
// cost dominates).  With the device-picked anchor (launch_kb_pick), tree phase at K_e = K_r =
// 32/36/40/44/48: RMAT-26 25.5/20.4/19.8/22.5/20.6 ms, twitter shape (32/40/48) 29.1/29.6/30.4
// ms, RMAT-25 (40/48) 12.3/13.8 ms (profiles/r02/lab/lab_kpick.jsonl); the lockstep loop's
// apply at P = 8, K = 40/48/56/64: 18.8/18.7/19.2/20.5 ms (round 1).
// Edge-quantile cuts: 2/5 as many (at least 8): with the rank cuts at 40 and the device-picked
// anchor, K_e = 8/12/16/24/32/40 -> RMAT-26 tree 19.2/19.0/18.9/19.1/19.4/19.7 ms, twitter shape
// (12/16/24/40) 28.4/28.3/29.1/29.4 ms, RMAT-25 (16/40) 11.6/12.5 ms (lab_kcuts.jsonl).
// n_seq = 0 leaves out the dense-graph rule below: it was tuned on the one-GPU loop only, and
// the lockstep loop's bucket placement has its own measurements (ls_plan).
static void kb_counts(uint64_t m, uint32_t* K_e, uint32_t* K_r, uint32_t kmax = 40,
                      uint32_t n_seq = 0) {
  const uint32_t K_auto = (uint32_t)std::min<uint64_t>(kmax, std::max<uint64_t>(8, m >> 23));
  *K_e = knobs().kb_buckets > 0 ? (uint32_t)knobs().kb_buckets : std::max<uint32_t>(8, K_auto * 2 / 5);
  *K_r = knobs().kb_rankb > 0 ? (uint32_t)knobs().kb_rankb : K_auto;
  // Dense graphs (mean degree >= 40) of 1.5 x 2^25 .. 1.5 x 2^27 records: 12 rank cuts
  // (instead of 8 .. 23).  Step ms, default -> 12 (profiles/r05/ah_dense_cuts/): R-MAT-22 seeds
  // 22 / 1 / 2 / 5 / 9 4.10 / 4.15 / 4.43 / 4.18 / 4.10 -> 3.93 / 3.98 / 4.07 / 4.03 / 3.89 (its
  // percolation bucket's zipper: 10.3 M -> 1.0 M steps), R-MAT-23 seeds 23 / 7 6.77 / 6.65 ->
  // 6.32 / 6.60.  Either side the same cuts are mixed (R-MAT-21 +0.09 ms; R-MAT-24 seeds 24 / 3
  // -0.59 / +1.16 ms), and the LJ shape (mean degree 28) loses 0.2-2.5 ms at any other count.
  if (n_seq && m >= (3ull << 24) && m < (3ull << 26) && 2 * m >= 40ull * n_seq &&
      knobs().kb_rankb <= 0 && knobs().kb_buckets <= 0)
    *K_r = 12;
}

// Directly binned records (launch_edge_bin): the buckets' .second are bin indices, bucket k's
// records are the filled parts of bins [bk[k].second, bk[k+1].second).
struct SegPlan {
  KbSegs dev{};                       // device start / cursor / capacity-end arrays
  std::vector<unsigned long long> cstart;  // host: capacity start of each bin, then the end
};

// Giant sweeps (launch_gb_sweep): after which buckets' applies the giant bitmap is completed
// from the union-find.  The giant swallows small components bucket after bucket, and their
// ranks miss the bitmap until a refresh meets them as the lo end of a kept pair: 102 M of the
// 179 M pairs the RMAT-26 maps keep resolve to the giant in the refresh
// (profiles/r05/f_sweep/refresh.jsonl).  A sweep costs a pass over the applied ranks (a find for
// each clear bit), so it runs once the giant exists — after the bucket before the last one
// mapped fresh (the mean degree below it crosses 1/2, fresh[]) — and then whenever the records
// since the last sweep reach SWEEP_ALPHA x n_seq.  Tree ms at alpha 1.5 / 2.5 / 4 against none:
// RMAT-26 14.16 / 13.95 / 14.00 vs 15.00, twitter shape 20.26 / 20.59 / 20.64 vs 21.43, RMAT-22
// 2.35 / 2.36 / 2.44 vs 2.63, RMAT-24 5.83 / 5.88 / 5.83 vs 6.22, LJ shape within noise
// (profiles/r05/h_sweep_alpha/).  recs(k): the records of bucket k.
static constexpr double SWEEP_ALPHA = 2.0;
template <typename Recs>
static std::vector<char> sweep_plan(const std::vector<std::pair<uint32_t, uint64_t>>& bk,
                                    Recs recs, const std::vector<char>& fresh, uint32_t n_seq) {
  const size_t nbk = bk.size() - 1;
  std::vector<char> sweep(nbk + 1, 0);
  size_t kf = 0;
  for (size_t k = 1; k < nbk && k < fresh.size(); ++k)
    if (fresh[k]) kf = k;
  if (kf == 0) return sweep;
  sweep[kf - 1] = 1;
  double acc = 0;
  for (size_t k = kf; k + 1 < nbk; ++k) {
    acc += (double)recs(k);
    if (acc >= SWEEP_ALPHA * n_seq) {
      sweep[k] = 1;
      acc = 0;
    }
  }
  return sweep;
}

// The buckets after which the mean degree 2E/B of the graph below the bucket's end crosses 1/2
// to 1 (the giant's birth, estimated from the records): fresh[k + 1] = 1 for each (see
// tree_from_sorted's fresh anchors).
template <typename Recs>
static std::vector<char> birth_window(const std::vector<std::pair<uint32_t, uint64_t>>& bk,
                                      Recs recs) {
  const size_t nbk = bk.size() - 1;
  std::vector<char> fresh(nbk + 1, 0);
  double E = 0;
  for (size_t k = 0; k + 1 < nbk; ++k) {
    E += (double)recs(k);
    const double B = (double)bk[k + 1].first, d = B > 0 ? 2.0 * E / B : 0.0;
    if (d >= knobs().kb_fresh_lo / 100.0) fresh[k + 1] = 1;
    if (d >= knobs().kb_fresh_hi / 100.0) break;
  }
  return fresh;
}

static void tree_from_sorted(Ctx& c, const uint64_t* sorted, uint64_t* spare, uint64_t m,
                             uint32_t n_seq, int lo_bit, uint32_t* d_parent, uint32_t* jump,
                             uint32_t* hcnt, bool stats, unsigned long long* ws, hipStream_t s,
                             Timer* tm, const Buckets* given = nullptr,
                             const uint32_t* bins = nullptr, uint32_t nb = 0,
                             const SegPlan* seg = nullptr) {
  uint32_t K_e, K_r;
  kb_counts(m, &K_e, &K_r, 40, n_seq);
  uint32_t K = K_e + K_r;
  // parent and hint interleaved (pj[2v], pj[2v + 1]): a zipper step loads one line; the parents
  // go to d_parent after the loop
  uint32_t* const d_out = d_parent;
  uint32_t* pj = (uint32_t*)c.scratch.get("kb_pj", (size_t)n_seq * 8);
  launch_pj_init(pj, n_seq, s);
  d_parent = pj;
  jump = pj + 1;
  uint32_t* uf = (uint32_t*)c.scratch.get("kb_uf", (size_t)n_seq * 4);
  uint32_t* label = (uint32_t*)c.scratch.get("kb_label", (size_t)n_seq * 4);
  uint32_t* linked = (uint32_t*)c.scratch.get("kb_linked", (size_t)n_seq * 4);
  uint32_t* counters = (uint32_t*)c.scratch.get("kb_counters", 2 * 64);
  const size_t bm_words = (size_t)n_seq / 32 + 2, spq_words = (size_t)n_seq / 32 + 64;
  uint32_t* bitmaps = (uint32_t*)c.scratch.get("kb_bitmap", 2 * bm_words * 4);
  uint32_t* spqs = (uint32_t*)c.scratch.get("kb_spq", 2 * spq_words * 4);
  // giant bitmap (k_kb_map) and the two slots of its reference vertex (INV: none yet)
  uint32_t* gbits = (uint32_t*)c.scratch.get("kb_gbits", bm_words * 4);
  uint32_t* gx = (uint32_t*)c.scratch.get("kb_gx", 2 * 4);
  // the giant summary the next map reads (written after each rebase)
  uint32_t* gsum = (uint32_t*)c.scratch.get("kb_gsum", ((size_t)n_seq / 2048 + 2) * 4);
  // the giant's anchor of each map, picked on the device (two slots by bucket parity)
  uint32_t* anc = (uint32_t*)c.scratch.get("kb_anchor", 2 * 4);
  (void)hipMemsetAsync(anc, 0xFF, 2 * 4, s);
  (void)hipMemsetAsync(counters, 0, 2 * 64, s);
  (void)hipMemsetAsync(bitmaps, 0, 2 * bm_words * 4, s);
  (void)hipMemsetAsync(gx, 0xFF, 2 * 4, s);
  unsigned long long* bounds =
      (unsigned long long*)c.scratch.get("kb_bounds", (size_t)(K + 1) * 16);
  launch_iota(uf, n_seq, s);
  launch_iota(label, n_seq, s);
  (void)hipMemsetAsync(ws, 0, 64 * 2, s);
  Buckets bk;
  uint64_t m_valid = 0;
  if (given) {
    bk = *given;
    m_valid = bk.back().second;
  } else {
    launch_kb_bounds(sorted, m, K_e, K_r, n_seq, lo_bit, bounds, s);
    std::vector<unsigned long long> hb(2 * (K + 1));
    HIP_CHECK(hipMemcpyAsync(hb.data(), bounds, hb.size() * 8, hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipStreamSynchronize(s));
    m_valid = hb[2 * K + 1];
    // distinct rank boundaries; bucket k = ranks [B_k, B_{k+1}), edges [e_k, e_{k+1})
    std::vector<std::pair<uint32_t, uint64_t>> cand;
    for (uint32_t k = 0; k < K; ++k) cand.emplace_back((uint32_t)hb[2 * k], hb[2 * k + 1]);
    std::sort(cand.begin(), cand.end());
    for (auto& cb : cand)
      if (cb.first < n_seq && (bk.empty() || cb.first > bk.back().first)) bk.push_back(cb);
    if (bk.empty() || bk[0].first != 0) bk.insert(bk.begin(), {0u, 0ull});
    bk.emplace_back(n_seq, m_valid);
  }
  if (tm) tm->mark("kb_bounds");
  const auto host_t0 = std::chrono::steady_clock::now();
  const size_t nbk = bk.size() - 1;
  // The sort's free ping-pong buffer (m items) holds the kept (b, g) pairs of a bucket.
  // Pipelined (default): bucket k+1 is mapped on the side stream while bucket k is applied
  // on s, with kept pairs, marks and counters double-buffered by bucket parity — each needs
  // half of the buffer.  The map of bucket k+1 anchors the giant at the last rank of bucket
  // k-1 (launch_kb_map).
  // records of bucket k (at most: the capacity of its bins when directly binned)
  auto recs = [&](size_t k) -> uint64_t {
    return seg ? seg->cstart[bk[k + 1].second] - seg->cstart[bk[k].second]
               : bk[k + 1].second - bk[k].second;
  };
  uint64_t max_e = 0;
  for (size_t k = 0; k < nbk; ++k) max_e = std::max<uint64_t>(max_e, recs(k));
  const bool per_bucket = knobs().tree_stats == 2;
  const bool pipe = knobs().kb_pipe && !per_bucket && 2 * max_e <= m;
  uint64_t* kept[2] = {spare, pipe ? spare + m / 2 : spare};
  auto par = [&](size_t k) { return pipe ? (int)(k & 1) : 0; };
  // Fresh anchors around the giant's birth.  A pipelined map anchors on the state before the
  // previous bucket's apply, so the bucket after the one where the giant forms is mapped
  // against a component that is not the giant yet, and its zipper walks the new giant's chains
  // without the spine rules (RMAT-26 seed 5: tree 19.7 ms, 14.8 with a fresh anchor).  Where
  // that happens is estimated from the records: the mean degree 2E/B of the graph on the ranks
  // below a bucket's end crossing 1/2 to 1.  Each bucket after such a bucket is mapped after the
  // previous apply (anchored on it), not beside it.  Tree ms, default -> fresh: RMAT-26 seed 26
  // 14.8 -> 15.0, seed 5 19.7 -> 15.1, RMAT-25 seed 9 11.5 -> 9.6, RMAT-24 7.1 -> 6.2, RMAT-22
  // 3.07 -> 2.64, twitter shape 21.8 -> 21.1 (profiles/r04/ak_fresh_anchor/).
  std::vector<char> fresh = pipe ? birth_window(bk, recs) : std::vector<char>(nbk + 1, 0);
  std::vector<char> sweep = sweep_plan(bk, recs, fresh, n_seq);
  auto anchor_of = [&](size_t k) -> uint32_t {
    size_t a = pipe && !fresh[k] ? k - std::min<size_t>(k, 1) : k;  // bucket whose start - 1 anchors
    return (a >= 1 && bk[a].first > 0) ? bk[a].first - 1 : INV;
  };
  // The giant bitmap's reference vertex lives in slot j & 1 for map j: the rebase before map
  // j reads slot (j-1) & 1 and writes slot j & 1, at a point where neither stream touches the
  // union-find (map j-1 and apply j-1 complete); an apply uses the slot most recently written
  // on its stream.
  // the summary costs a launch per bucket: it pays on large inputs only (RMAT-26 tree 18.5 ->
  // 16.7 ms; RMAT-22 3.25 -> 3.45 ms)
  if (!(knobs().kb_gsum > 0 || (knobs().kb_gsum < 0 && m >= (1ull << 27)))) gsum = nullptr;
  // the map leaves its union-find misses to the apply's refresh kernel
  hipStream_t sa = s;  // the applies and the rebases between them
  auto rebase = [&](size_t j) {  // the anchor of map j, then the bitmap's rebase on it
    const uint32_t a = anchor_of(j);
    launch_kb_pick(uf, a == INV ? 0u : a + 1, anc + ((j - 1) & 1), anc + (j & 1), gbits, n_seq,
                   gx + ((j - 1) & 1), gx + (j & 1), sa);
    if (gsum) launch_gb_sum(gbits, n_seq, gsum, sa);
  };
  auto map_k = [&](size_t k, hipStream_t st) {
    int p = par(k);
    size_t sp = tm ? tm->span_begin("kb_map", st) : 0;
    KbSegs sg{};
    if (seg) {
      sg = seg->dev;
      sg.i0 = (uint32_t)bk[k].second;
      sg.i1 = (uint32_t)bk[k + 1].second;
    }
    launch_kb_map(sorted, seg ? seg->cstart[bk[k].second] : bk[k].second,
                  seg ? seg->cstart[bk[k + 1].second] : bk[k + 1].second, bk[k].first,
                  anchor_of(k), uf, label, kept[p], pipe ? m / 2 : m, bitmaps + p * bm_words,
                  counters + p * 16,
                  lo_bit, hcnt, stats, ws, bins, nb, gbits, gbits ? gx + (k & 1) : nullptr, 1,
                  st, seg ? &sg : nullptr, anc ? anc + (k & 1) : nullptr, k >= 1 ? gsum : nullptr);
    if (tm) tm->span_end(sp, st);
  };
  // anc_next: the union keeps the root of the next map's anchor on top, so that the map running
  // beside it sees the giant's root unchanged.  When map k+1 is fresh (fresh[k+1]), the apply runs
  // before rebase(k+1), so that slot still holds the anchor picked for map k-1: nothing maps
  // beside this union then, and keeping that (after the birth: the giant's) root on top is
  // harmless (ADVICE r04 noted the stale slot).
  auto apply_k = [&](size_t k, size_t slot, hipStream_t st) {
    int p = par(k);
    launch_kb_apply(recs(k) > 0, bk[k].first, bk[k + 1].first, anchor_of(k),
                    uf, label, d_parent, jump, kept[p], linked, bitmaps + p * bm_words,
                    spqs + p * spq_words, counters + p * 16, true, stats,
                    ws, gbits, gbits ? gx + (slot & 1) : nullptr, st, anc ? anc + (k & 1) : nullptr,
                    anc ? anc + ((k + 1) & 1) : nullptr);
  };
  if (pipe) {
    // map k+1 runs on the side stream while bucket k is applied; the rebase for map k+1 sits
    // on s after map k has finished (and after apply k-1), so map k+1 waits for it
    hipStream_t s2 = c.side;
    hipEvent_t* ev_map = c.kb_ev;
    hipEvent_t* ev_reb = c.kb_ev + 2;
    HIP_CHECK(hipEventRecord(c.kb_ev[4], s));
    HIP_CHECK(hipStreamWaitEvent(s2, c.kb_ev[4], 0));
    if (sa != s) HIP_CHECK(hipStreamWaitEvent(sa, c.kb_ev[4], 0));
    map_k(0, s2);
    HIP_CHECK(hipEventRecord(ev_map[0], s2));
    size_t slot = 0;
    for (size_t k = 0; k < nbk; ++k) {
      HIP_CHECK(hipStreamWaitEvent(sa, ev_map[k & 1], 0));
      // side: map k+1 on the maps' stream beside apply k; else (a fresh map, after apply k)
      // on the applies' stream itself, which runs it right after the apply anyway — two
      // cross-stream event hops fewer (~20 us each on the GPU timeline, round 6)
      auto next = [&](bool side) {
        rebase(k + 1);
        slot = k + 1;
        if (!side) {
          map_k(k + 1, sa);
          HIP_CHECK(hipEventRecord(ev_map[(k + 1) & 1], sa));
          return;
        }
        HIP_CHECK(hipEventRecord(ev_reb[k & 1], sa));
        HIP_CHECK(hipStreamWaitEvent(s2, ev_reb[k & 1], 0));
        map_k(k + 1, s2);
        HIP_CHECK(hipEventRecord(ev_map[(k + 1) & 1], s2));
      };
      if (k + 1 < nbk && !fresh[k + 1]) next(true);
      apply_k(k, slot, sa);
      if (sweep[k]) launch_gb_sweep(uf, gbits, bk[k + 1].first, gx + (slot & 1), sa);
      if (k + 1 < nbk && fresh[k + 1]) next(false);
    }
    if (sa != s) {  // s resumes after the last apply
      HIP_CHECK(hipEventRecord(c.kb_ev[4], sa));
      HIP_CHECK(hipStreamWaitEvent(s, c.kb_ev[4], 0));
    }
    if (tm)  // the host's time to enqueue the loop (the device's is the tree_insert phase)
      tm->host_ms("kb_loop_host", std::chrono::duration<double, std::milli>(
                                      std::chrono::steady_clock::now() - host_t0).count());
  } else {
    for (size_t k = 0; k < nbk; ++k) {
      if (per_bucket) (void)hipMemsetAsync(ws, 0, 128, s);
      if (k >= 1) rebase(k);
      map_k(k, s);
      apply_k(k, k, s);
      if (per_bucket) {
        unsigned long long h[16];
        HIP_CHECK(hipMemcpyAsync(h, ws, 128, hipMemcpyDeviceToHost, s));
        HIP_CHECK(hipStreamSynchronize(s));
        fprintf(stderr, "bucket %zu ranks [%u,%u) edges %llu kept %llu inbucket_lo %llu finds %llu zip %llu steps %llu cas %llu fail %llu maxsteps %llu zroot %llu zone %llu\n",
                k, bk[k].first, bk[k + 1].first, h[0], h[5], h[6], h[7], h[8], h[9], h[10], h[11], h[12], h[13], h[14]);
      }
    }
  }
  launch_pj_parents(pj, n_seq, d_out, s);
}

// ---- hi bins (the one-pass grouping of the edge items, see sheep_kernels.hip) -------------
// Bin bounds from the 256-rank chunk degree sums: the records with hi in chunk c are estimated
// as dsum(c) * (D_c + dsum(c)/2) / total, D_c the degree mass of the chunks below.  A bin
// closes at 1/320 of the estimated records, or when 32K ranks wide (the kb map's LDS window)
// unless it holds almost nothing; at most 511 bins, then the INVALID bin (bound n_seq).
// est (nullable): the estimated records of each bin but the last (the INVALID bin).
static std::vector<uint32_t> make_bins(const std::vector<uint64_t>& dsum, uint32_t n_seq,
                                       std::vector<double>* est = nullptr) {
  const size_t nch = dsum.size();
  std::vector<double> w(nch);
  double tot = 0, D = 0, W = 0;
  for (uint64_t d : dsum) tot += (double)d;
  for (size_t c = 0; c < nch; ++c) {
    w[c] = tot > 0 ? (double)dsum[c] * (D + 0.5 * (double)dsum[c]) / tot : 0.0;
    D += (double)dsum[c];
    W += w[c];
  }
  std::vector<uint32_t> b;
  // the estimate of bins [b[i], b[i+1]) (chunk-aligned bounds, the last one n_seq)
  auto estimate = [&](const std::vector<uint32_t>& bb) {
    if (!est) return;
    est->assign(bb.size() - 1, 0.0);
    for (size_t i = 0; i + 1 < bb.size(); ++i)
      for (size_t c = bb[i] / 256; c < std::min<size_t>(nch, ((size_t)bb[i + 1] + 255) / 256); ++c)
        (*est)[i] += w[c];
  };
  // No estimated records (every record a self-loop, or no degrees): one bin holds them all.
  if (!(tot > 0) || !(W > 0) || nch < 2) {
    std::vector<uint32_t> one = {0u, n_seq};
    if (est) est->assign(1, (double)W);
    return one;
  }
  double wmax = W / 320, wide = W / 50000;
  for (int attempt = 0; attempt < 32; ++attempt) {
    b.assign(1, 0u);
    double acc = 0;
    for (size_t c = 0; c + 1 < nch; ++c) {
      acc += w[c];
      const uint64_t end = (uint64_t)(c + 1) * 256, width = end - b.back();
      if (acc >= wmax || (width >= 32768 && acc >= wide)) {
        b.push_back((uint32_t)end);
        acc = 0;
      }
    }
    if (b.size() + 1 <= 512) break;
    wide *= 2;
    wmax *= 1.25;
  }
  // Hard cap (the bin digit, the LDS tables of the scatter and the bin-start buffers hold 512
  // entries): keep every s-th bound.  Any bounds give the same tree; only the work shifts.
  if (b.size() + 1 > 512) {
    const size_t st = (b.size() + 510) / 511;
    std::vector<uint32_t> c;
    for (size_t i = 0; i < b.size(); i += st) c.push_back(b[i]);
    b.swap(c);
  }
  b.push_back(n_seq);
  if (b.size() > 512) throw ApiError(-EIO, "make_bins: more than 512 hi bins");
  estimate(b);
  return b;
}

// Buckets as unions of bins: K_e cuts at edge quantiles (exact bin counts) and K_r at rank
// quantiles, each snapped to a bin bound.  bin_start: nb + 1 record offsets.
// The cuts as bin indices (sorted, distinct, in (0, nb - 1)).
static std::vector<uint32_t> bucket_cuts(const std::vector<uint32_t>& bounds,
                                         const std::vector<unsigned long long>& bin_start,
                                         uint64_t m, uint32_t n_seq, uint32_t kmax = 40,
                                         int merge = -1 /* kb_merge; -1: the option */,
                                         bool one_gpu = true /* kb_counts' dense-graph rule */) {
  const uint32_t nb = (uint32_t)bounds.size();
  if (merge < 0) merge = knobs().kb_merge;
  const uint64_t m_valid = bin_start[nb - 1];
  uint32_t K_e, K_r;
  kb_counts(m, &K_e, &K_r, kmax, one_gpu ? n_seq : 0);
  std::vector<uint32_t> cuts;
  for (uint32_t k = 1; k < K_e; ++k) {
    const uint64_t target = m_valid * k / K_e;
    uint32_t i = (uint32_t)(std::lower_bound(bin_start.begin(), bin_start.begin() + (nb - 1),
                                             (unsigned long long)target) - bin_start.begin());
    if (i > 0 && i < nb - 1) cuts.push_back(i);
  }
  for (uint32_t j = 1; j < K_r; ++j) {
    const uint32_t r = (uint32_t)((uint64_t)n_seq * j / K_r);
    uint32_t i = (uint32_t)(std::upper_bound(bounds.begin(), bounds.begin() + (nb - 1), r) -
                            bounds.begin()) - 1;
    if (i > 0 && i < nb - 1) cuts.push_back(i);
  }
  std::sort(cuts.begin(), cuts.end());
  cuts.erase(std::unique(cuts.begin(), cuts.end()), cuts.end());
  if (merge > 0) {  // drop a cut while the buckets either side hold few records
    const uint64_t thr = m_valid * (uint64_t)merge / 10000;
    std::vector<uint32_t> kept;
    uint32_t prev = 0;
    for (size_t i = 0; i < cuts.size(); ++i) {
      const uint32_t next = i + 1 < cuts.size() ? cuts[i + 1] : nb - 1;
      if (bin_start[next] - bin_start[prev] > thr) {
        kept.push_back(cuts[i]);
        prev = cuts[i];
      }
    }
    cuts.swap(kept);
  }
  return cuts;
}

static Buckets buckets_from_bins(const std::vector<uint32_t>& bounds,
                                 const std::vector<unsigned long long>& bin_start, uint64_t m,
                                 uint32_t n_seq) {
  const uint32_t nb = (uint32_t)bounds.size();
  Buckets bk;
  bk.emplace_back(0u, 0ull);
  for (uint32_t i : bucket_cuts(bounds, bin_start, m, n_seq))
    bk.emplace_back(bounds[i], (uint64_t)bin_start[i]);
  bk.emplace_back(n_seq, (uint64_t)bin_start[nb - 1]);
  return bk;
}

// allow_direct: the hi bins may be filled directly by the edge pass (launch_edge_bin); false
// after a bin outgrew its estimate (the records are then grouped by the scatter).
static void build_tree_dev(Ctx& c, const uint32_t* d_uv, uint64_t m, const uint32_t* d_rank,
                           uint32_t n_rank, uint32_t n_seq, uint32_t* d_parent, uint32_t* d_pst,
                           hipStream_t s, Timer* tm, const DegInfo* di = nullptr,
                           bool allow_direct = true) {
  require_records(m, "tree build");
  if (n_seq == 0) return;
  launch_fill(d_parent, INV, n_seq, s);
  launch_fill(d_pst, 0, n_seq, s);
  uint32_t* jump = nullptr;  // (the kb loop keeps its hints beside the parents)
  if (m == 0) return;
  uint64_t* items = (uint64_t*)c.scratch.get("e_items", m * 8);
  uint64_t* items_b = (uint64_t*)c.scratch.get("e_items_b", m * 8);
  uint32_t* tmp = (uint32_t*)c.scratch.get("rsort_tmp", rsort_tmp_words(m) * 4);
  if (tm) tm->mark("tree_init");
  const bool stats = knobs().tree_stats != 0;
  // Sort keys: hi's bits [lo_bit, top + 1) — bit `top` puts INVALID his after every rank.
  // kb needs hi order only down to groups of 2^lo_bit ranks (bucket ranges; the run lengths
  // that pst needs are counted per group inside k_kb_map): 18 bits = 2 passes.
  int top = bits_for(n_seq);
  int lo_bit = std::max(0, top + 1 - 18);
  // pst from degrees (di) needs the run length of every hi: counted by k_kb_map.  Otherwise
  // pst_weight[lo] += 1 per record in the edge pass.
  bool pst_count = di != nullptr;
  // Large inputs: rank gathers in partitioned order (launch_part_gather), via items_b/items.
  bool part = use_part(m);
  const uint32_t* src = d_uv;
  // Hi bins (one scatter pass) when the degrees are at hand; else the two-pass radix sort.
  const bool use_bins = pst_count && m >= (1ull << 20) && n_seq > 256;
  // The bins come from the chunk degree sums (seq order): they are summed and copied to the
  // host BEFORE the second partition pass is enqueued, so the host cuts the bins while the GPU
  // runs that pass instead of idling for the round trip.
  const size_t nch = ((size_t)n_seq + 255) / 256;
  if (use_bins) {
    uint64_t* cds = (uint64_t*)c.scratch.get("chunk_deg", nch * 8);
    launch_chunk_degsum(di->seq, di->deg, n_seq, cds, s, di->nsd);
    if (c.h_chunks_n < nch) {
      if (c.h_chunks) HIP_CHECK(hipHostFree(c.h_chunks));
      c.h_chunks = nullptr;
      c.h_chunks_n = 0;
      HIP_CHECK(hipHostMalloc((void**)&c.h_chunks, nch * 8, hipHostMallocDefault));
      c.h_chunks_n = nch;
    }
    HIP_CHECK(hipMemcpyAsync(c.h_chunks, cds, nch * 8, hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipEventRecord(c.bins_ev, s));
  }
  const bool direct = use_bins && allow_direct && knobs().bin_direct;
  // the second pass's records packed to 6 bytes: only the direct edge pass reads them
  const bool pre6 = part && direct && di && di->ids_checked && part_p6_ok(n_rank);
  uint32_t* pws = part ? (uint32_t*)c.scratch.get("part_ws", PART_WS_WORDS * 4) : nullptr;
  if (part) {
    if (di && di->part_first_done) {  // pass 1 ran on c.side, beside the sequence sort
      HIP_CHECK(hipStreamWaitEvent(s, c.part_ev[1], 0));
      launch_part_second(items, m, d_rank, n_rank, items_b, pws, s, pre6, di->mid_slots,
                         di->mid_caps, di->mid_p6, ff_groups());
    } else {
      launch_part_gather(d_uv, m, d_rank, n_rank, items, items_b, pws, s, di && di->yhist_ready,
                         pre6);
    }
    src = (const uint32_t*)items_b;
    if (tm) tm->mark("partition");
  }
  if (!direct && part && di && di->part_first_done && di->mid_caps) {
    // The first pass wrote capacity regions (launch_front_fused / launch_part_first_caps) whose
    // overflow word the direct branch reads with the bins' own; without direct binning (n_seq
    // <= 256, or bin_direct 0) it is read here: an overflowed region lost records, so the
    // partition is run again from the records.
    HIP_CHECK(hipMemcpyAsync(c.h_pinned + 10, c.d_err + 3, 4, hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipStreamSynchronize(s));
    if (c.h_pinned[10]) {
      DegInfo d2 = *di;
      d2.part_first_done = false;
      d2.mid_caps = false;
      d2.mid_p6 = false;
      d2.mid_slots = 0;
      d2.yhist_ready = false;
      build_tree_dev(c, d_uv, m, d_rank, n_rank, n_seq, d_parent, d_pst, s, tm, &d2, allow_direct);
      return;
    }
  }
  const uint64_t* sorted;
  uint64_t* spare;
  Buckets given;
  const uint32_t* dbins = nullptr;
  uint32_t nbins = 0;
  SegPlan plan;
  uint32_t* ovf = c.d_err + 1;  // a directly binned bin outgrew its capacity
  if (direct) {
    // Each bin gets a capacity region sized by its estimated records (+ slack); the edge pass
    // fills them directly, and the buckets are cut on the estimate (any cuts are exact).
    HIP_CHECK(hipEventSynchronize(c.bins_ev));
    std::vector<uint64_t> hd(c.h_chunks, c.h_chunks + nch);
    std::vector<double> est;
    std::vector<uint32_t> bounds = make_bins(hd, n_seq, &est);
    nbins = (uint32_t)bounds.size();
    uint32_t* db = (uint32_t*)c.scratch.get("hi_bins", 512 * 4);
    HIP_CHECK(hipMemcpyAsync(db, bounds.data(), nbins * 4, hipMemcpyHostToDevice, s));
    dbins = db;
    const double slack = 1.0 + knobs().bin_slack / 1000.0;
    plan.cstart.assign(nbins, 0ull);
    std::vector<unsigned long long> h(3 * 512, 0ull);  // start | cursor | capacity end
    for (uint32_t i = 0; i + 1 < nbins; ++i) {
      // a bin never holds more than m items (and the map keeps segment lengths in u32)
      const uint64_t cap = std::min<uint64_t>((uint64_t)std::ceil(est[i] * slack) + 8192, m);
      plan.cstart[i + 1] = plan.cstart[i] + cap;
      h[i] = h[512 + i] = plan.cstart[i];
      h[1024 + i] = plan.cstart[i + 1];
    }
    unsigned long long* dseg = (unsigned long long*)c.scratch.get("bin_segs", h.size() * 8);
    HIP_CHECK(hipMemcpyAsync(dseg, h.data(), h.size() * 8, hipMemcpyHostToDevice, s));
    HIP_CHECK(hipMemsetAsync(ovf, 0, 4, s));
    uint64_t* binned = (uint64_t*)c.scratch.get(
        "e_binned", std::max<uint64_t>(plan.cstart[nbins - 1], 1) * 8);
    launch_edge_bin(src, part, m, d_rank, n_rank, c.d_err, db, nbins, dseg + 512, dseg + 1024,
                    binned, ovf, s, pre6 ? pws : nullptr);
    if (tm) tm->mark("edge_pass");
    // One readback before the kb loop is enqueued (the host then enqueues while the GPU runs
    // the first buckets): a bin that outgrew its estimate holds a hole where its dropped runs
    // were reserved, so the records are grouped again through the scatter.
    // (with ovf the first partition pass's overflow word, c.d_err[3]: capacity regions)
    HIP_CHECK(hipMemcpyAsync(c.h_pinned + 8, ovf, 12, hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipStreamSynchronize(s));
    if (c.h_pinned[8] || (di && di->mid_caps && c.h_pinned[10])) {
      DegInfo d2 = *di;
      d2.part_first_done = false;  // k_part's passes are run again from d_uv (unpacked)
      d2.mid_caps = false;
      d2.mid_p6 = false;
      d2.mid_slots = 0;
      d2.yhist_ready = false;      // the first partition consumed the y-digit counts
      build_tree_dev(c, d_uv, m, d_rank, n_rank, n_seq, d_parent, d_pst, s, tm, &d2, false);
      return;
    }
    plan.dev = {dseg, dseg + 512, dseg + 1024, 0u, 0u};
    given.emplace_back(0u, 0ull);
    for (uint32_t i : bucket_cuts(bounds, plan.cstart, m, n_seq)) given.emplace_back(bounds[i], i);
    given.emplace_back(n_seq, (uint64_t)(nbins - 1));
    sorted = binned;
    spare = items;  // free: held k_part's mid records (src is items_b or d_uv)
  } else if (use_bins) {
    HIP_CHECK(hipEventSynchronize(c.bins_ev));
    std::vector<uint64_t> hd(c.h_chunks, c.h_chunks + nch);
    std::vector<uint32_t> bounds = make_bins(hd, n_seq);
    nbins = (uint32_t)bounds.size();
    uint32_t* db = (uint32_t*)c.scratch.get("hi_bins", 512 * 4);
    HIP_CHECK(hipMemcpyAsync(db, bounds.data(), nbins * 4, hipMemcpyHostToDevice, s));
    dbins = db;
    uint16_t* digits = (uint16_t*)c.scratch.get("item_bins", m * 2);
    unsigned long long* dstart = (unsigned long long*)c.scratch.get("bin_start", 513 * 8);
    // the bin starts reach the host before the scatter runs: the buckets are cut meanwhile
    uint64_t* out = group_by_bins(src, part, m, d_rank, n_rank, c.d_err, db, nbins, items, items_b,
                                  tmp, digits, dstart, s, c.h_bstart, c.bins_ev);
    if (tm) tm->mark("edge_pass");
    HIP_CHECK(hipEventSynchronize(c.bins_ev));
    std::vector<unsigned long long> hs(c.h_bstart, c.h_bstart + nbins + 1);
    given = buckets_from_bins(bounds, hs, m, n_seq);
    sorted = out;
    spare = out == items ? items_b : items;
  } else {
    launch_edge_pass_tiles(src, m, d_rank, n_rank, pst_count ? nullptr : d_pst, items, c.d_err,
                           lo_bit, rsort_first_width(top + 1 - lo_bit), tmp, s, part);
    if (tm) tm->mark("edge_pass");
    sorted = radix_sort_u64(items, items_b, items, m, lo_bit, top + 1, tmp, s, true);
    spare = (sorted == items) ? items_b : items;  // free ping-pong buffer
  }
  if (tm) tm->mark("bucket_sort");
  uint32_t* hcnt = nullptr;
  if (pst_count) {
    hcnt = (uint32_t*)c.scratch.get("hi_count", (size_t)n_seq * 4);
    launch_fill(hcnt, 0, n_seq, s);
  }
  unsigned long long* ws = (unsigned long long*)c.scratch.get("tree_ws", 64 * 2);
  tree_from_sorted(c, sorted, spare, m, n_seq, lo_bit, d_parent, jump, hcnt, stats, ws, s, tm,
                   use_bins ? &given : nullptr, dbins, nbins, direct ? &plan : nullptr);
  if (tm) tm->mark("tree_insert");
  if (pst_count) {
    launch_pst_from_count(di->seq, n_seq, di->deg, di->selfc, di->mode, hcnt, d_pst, s, di->nsd);
    if (tm) tm->mark("pst");
  }
  if (stats) {
    unsigned long long h[16];
    HIP_CHECK(hipMemcpyAsync(h, ws, 128, hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipStreamSynchronize(s));
    fprintf(stderr, "tree_stats algo=kb edges=%llu kept=%llu map_finds=%llu zip_edges=%llu steps=%llu cas=%llu casfail=%llu maxsteps=%llu\n",
            h[0], h[5], h[7], h[8], h[9], h[10], h[11], h[12]);
  }
}

// etree of the union of T forests over the same n ranks (the multi-GPU reduce): their edges
// (v, parent_t[v]) as items, sorted by parent, through the kb loop.
static void merge_forests_dev(Ctx& c, const uint32_t* d_parents, uint32_t T, uint32_t n,
                              uint32_t* d_parent, hipStream_t s, Timer* tm) {
  require_records((uint64_t)T * n, "forest merge");
  if (n == 0) return;
  launch_fill(d_parent, INV, n, s);
  uint32_t* jump = nullptr;  // (the kb loop keeps its hints beside the parents)
  const uint64_t m = (uint64_t)T * n;
  if (m == 0) return;
  uint64_t* items = (uint64_t*)c.scratch.get("e_items", m * 8);
  uint64_t* items_b = (uint64_t*)c.scratch.get("e_items_b", m * 8);
  uint32_t* tmp = (uint32_t*)c.scratch.get("rsort_tmp", rsort_tmp_words(m) * 4);
  for (uint32_t t = 0; t < T; ++t) launch_forest_items(d_parents + (size_t)t * n, n, items + (size_t)t * n, s);
  if (tm) tm->mark("forest_items");
  const int top = bits_for(n);
  const int lo_bit = std::max(0, top + 1 - 18);
  const uint64_t* sorted = radix_sort_u64(items, items_b, items, m, lo_bit, top + 1, tmp, s, false);
  uint64_t* spare = (sorted == items) ? items_b : items;
  if (tm) tm->mark("bucket_sort");
  unsigned long long* ws = (unsigned long long*)c.scratch.get("tree_ws", 64 * 2);
  tree_from_sorted(c, sorted, spare, m, n, lo_bit, d_parent, jump, nullptr, false, ws, s, tm);
  if (tm) tm->mark("tree_insert");
}

// ---- lockstep: the kb loop of ONE tree run by P ranks, each over its own edge shard --------
// Every rank holds the same union-find, labels and forest.  Per bucket each rank maps only its
// own records (the map is the part that scales with m), the kept pairs and giant marks of all
// ranks are all-gathered by the caller (RCCL), and every rank applies the same union — the
// zipper's result is the unique etree whatever the order, so the replicas stay identical.
// Bins and buckets come from GLOBAL degrees and GLOBAL bin counts, hence agree on all ranks.
struct Lockstep {
  // Buffers: the device's scratch (kept across calls, like every other entry point) for the
  // first live session; a private one for further concurrent sessions on the same device (the
  // one-GPU simulation of P ranks).
  Ctx* ctx = nullptr;
  Scratch own;
  Scratch* scp = nullptr;
  uint64_t m = 0;
  uint32_t n_seq = 0;
  std::vector<uint32_t> bounds;                // hi bins (global)
  std::vector<unsigned long long> local_start;  // this shard's bin offsets, nb + 1
  Buckets bk;                                   // (rank, local record offset)
  std::vector<uint64_t> global_e;               // records per bucket over all ranks
  uint32_t ms = 0;                              // mark slots (u64) per rank per bucket
  // Pipelined: the caller may map (and exchange) bucket k+1 while bucket k is applied, as the
  // one-GPU loop does (tree_from_sorted): counters, marks and spine queues are double-buffered
  // by bucket parity, the map of bucket k anchors the giant at the last rank of bucket k-2, and
  // the apply refreshes the kept starts first.  Exact for any interleaving of the two.
  static constexpr bool pipe = true;
  size_t bm_words = 0, spq_words = 0;
  uint32_t *bins = nullptr, *uf = nullptr, *label = nullptr, *linked = nullptr,
           *counters = nullptr, *bitmap = nullptr, *spq = nullptr, *parent = nullptr,
           *jump = nullptr, *hcnt = nullptr;
  const uint64_t* sorted = nullptr;
  unsigned long long* ws = nullptr;
  uint32_t* h_pinned = nullptr;
  size_t kept_bytes = 0;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> map_ev, apply_ev;
  // the giant's anchor of each map, picked on the device by the apply of the bucket before
  // (launch_kb_pick; identical on every rank: the replicas are identical), two slots by parity
  uint32_t* anc = nullptr;
  hipEvent_t pick_ev[2] = {nullptr, nullptr};
  // direct binning (launch_edge_bin): the buckets' .second are bin indices and bin i's items
  // lie at [cstart[i], fill); dseg: start | cursor | capacity end, 512 u64 each
  bool direct = false;
  std::vector<unsigned long long> cstart;
  unsigned long long* dseg = nullptr;
  // giant bitmap of this rank's maps (set bits are exact, so ranks may differ in them: they
  // only spare finds) and the two slots of its reference vertex; rebased by the pick
  uint32_t* gbits = nullptr;
  uint32_t* gx = nullptr;
  uint32_t* gsum = nullptr;  // the giant summary of the next map (launch_gb_sum, after the pick)
  std::vector<char> sweep;   // giant sweeps after these buckets' applies (sweep_plan)
  // The maps leave their union-find misses to the apply's refresh (as the one-GPU loop does)
  // only for a one-rank group: with P ranks the refresh would repeat on every rank the finds
  // that the maps split P ways.
  bool defer = false;
  // per-bucket apply spans ("kb_apply": the one-GPU rehearsal's per-rank apply time); the
  // multi-GPU driver times only the maps
  bool time_apply = true;
  // the exchange buffers were sized for the whole loop before it started (multi_tree): the
  // applies never grow them, so nothing inside the loop synchronises
  bool presized = false;
  // Split apply (P > 1 ranks, launch_ls_fold_union_label / launch_ls_zip): bucket k's spine and
  // zipper run only on its owner rank (k mod P), on zs, from copies of the bucket's refreshed
  // pairs and marks (two slots, by owned-bucket parity); every rank applies the union-find part.
  // parent[] then holds this rank's buckets' forest edges only: the ranks' forests are disjoint
  // and are summed by the caller.
  bool split = false;
  uint32_t rank = 0, P = 1, nzip = 0;
  hipStream_t zs = nullptr;
  uint64_t* zkept[2] = {nullptr, nullptr};
  uint32_t *zbm[2] = {nullptr, nullptr}, *zn[2] = {nullptr, nullptr}, *zspq = nullptr;
  hipEvent_t zready[2] = {nullptr, nullptr}, zdone[2] = {nullptr, nullptr};
  bool zused[2] = {false, false};
  size_t zkept_bytes[2] = {0, 0};
  std::vector<std::pair<hipEvent_t, hipEvent_t>> zip_ev;
  ~Lockstep() {
    if (zs) (void)hipStreamSynchronize(zs);
    for (auto& e : zready)
      if (e) (void)hipEventDestroy(e);
    for (auto& e : zdone)
      if (e) (void)hipEventDestroy(e);
    for (auto& e : zip_ev) { (void)hipEventDestroy(e.first); (void)hipEventDestroy(e.second); }
    if (zs) (void)hipStreamDestroy(zs);
    for (auto& e : pick_ev)
      if (e) (void)hipEventDestroy(e);
    for (auto& e : map_ev) { (void)hipEventDestroy(e.first); (void)hipEventDestroy(e.second); }
    for (auto& e : apply_ev) { (void)hipEventDestroy(e.first); (void)hipEventDestroy(e.second); }
    if (h_pinned) (void)hipHostFree(h_pinned);
    own.release();
    if (ctx) ctx->ls_live--;
  }
  uint32_t anchor(size_t k) const {
    const size_t a = pipe ? k - std::min<size_t>(k, 1) : k;
    return (a >= 1 && bk[a].first > 0) ? bk[a].first - 1 : INV;
  }
  uint32_t* cnt_of(size_t k) const { return counters + (pipe ? (k & 1) * 16 : 0); }
  uint32_t* bm_of(size_t k) const { return bitmap + (pipe ? (k & 1) * bm_words : 0); }
  uint32_t* spq_of(size_t k) const { return spq + (pipe ? (k & 1) * spq_words : 0); }
  std::pair<hipEvent_t, hipEvent_t> span(std::vector<std::pair<hipEvent_t, hipEvent_t>>& v,
                                         hipStream_t s) {
    hipEvent_t a, b;
    HIP_CHECK(hipEventCreate(&a));
    HIP_CHECK(hipEventCreate(&b));
    HIP_CHECK(hipEventRecord(a, s));
    v.emplace_back(a, b);
    return v.back();
  }
};

// part_done (nullable): the first partition pass of the rank gathers was launched by the caller
// into "ls_items" (with "part_ws" holding its cursors) and completes at this event.
// nsd (nullable): the global degrees in sequence order, read instead of d_deg[d_seq[r]].
// mid_caps: the first pass wrote capacity regions of mid_slots records (launch_front_fused,
// packed: mid_p6) whose overflow word is d_err[3]; an overflow sends this rank's partition
// back to the unpacked records (as build_tree_dev does).
static void ls_begin(Lockstep& L, const uint32_t* d_uv, uint64_t m, const uint32_t* d_rank,
                     uint32_t n_rank, const uint32_t* d_seq, uint32_t n_seq,
                     const uint32_t* d_deg, uint64_t* counts_out, uint32_t* nb_out,
                     uint32_t* d_err, hipStream_t s, hipEvent_t part_done = nullptr,
                     const uint32_t* nsd = nullptr, bool ids_checked = false,
                     uint64_t mid_slots = 0, bool mid_caps = false, bool mid_p6 = false) {
  require_records(m, "lockstep");
  Scratch& sc = *L.scp;
  L.m = m;
  L.n_seq = n_seq;
  HIP_CHECK(hipHostMalloc(&L.h_pinned, 64, hipHostMallocDefault));
  const size_t n = std::max<uint32_t>(n_seq, 1);
  L.parent = (uint32_t*)sc.get("ls_parent", n * 8);
  L.jump = L.parent + 1;
  L.hcnt = (uint32_t*)sc.get("ls_hcnt", n * 4);
  L.uf = (uint32_t*)sc.get("ls_uf", n * 4);
  L.label = (uint32_t*)sc.get("ls_label", n * 4);
  L.linked = (uint32_t*)sc.get("ls_linked", n * 4);
  L.counters = (uint32_t*)sc.get("ls_counters", 2 * 64);
  const size_t bm_words = n / 32 + 2, spq_words = n / 32 + 64;
  L.bm_words = bm_words;
  L.spq_words = spq_words;
  L.bitmap = (uint32_t*)sc.get("ls_bitmap", 2 * bm_words * 4);
  L.spq = (uint32_t*)sc.get("ls_spq", 2 * spq_words * 4);
  L.ws = (unsigned long long*)sc.get("ls_ws", 128);
  L.anc = (uint32_t*)sc.get("ls_anchor", 2 * 4);
  HIP_CHECK(hipMemsetAsync(L.anc, 0xFF, 2 * 4, s));
  for (auto& e : L.pick_ev) HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  L.gbits = (uint32_t*)sc.get("ls_gbits", bm_words * 4);
  L.gx = (uint32_t*)sc.get("ls_gx", 2 * 4);
  HIP_CHECK(hipMemsetAsync(L.gbits, 0, bm_words * 4, s));
  HIP_CHECK(hipMemsetAsync(L.gx, 0xFF, 2 * 4, s));
  // this rank's maps walk m records: the summary rule of tree_from_sorted
  if (knobs().kb_gsum > 0 || (knobs().kb_gsum < 0 && m >= (1ull << 27)))
    L.gsum = (uint32_t*)sc.get("ls_gsum", ((size_t)n_seq / 2048 + 2) * 4);
  launch_pj_init(L.parent, (uint32_t)n, s);
  launch_fill(L.hcnt, 0, n, s);
  launch_iota(L.uf, n, s);
  launch_iota(L.label, n, s);
  HIP_CHECK(hipMemsetAsync(L.counters, 0, 2 * 64, s));
  HIP_CHECK(hipMemsetAsync(L.bitmap, 0, 2 * bm_words * 4, s));
  HIP_CHECK(hipMemsetAsync(L.ws, 0, 128, s));
  if (n_seq == 0) {
    L.bounds.assign(1, 0u);
    L.local_start.assign(2, 0ull);
    L.local_start[1] = m;
    *nb_out = 1;
    counts_out[0] = m;
    return;
  }
  // hi bins from the global degrees (identical on every rank): the chunk sums go to pinned host
  // memory, and the host cuts the bins while the second partition pass (which needs no bins)
  // runs
  Ctx& c = *L.ctx;
  const size_t nch = ((size_t)n_seq + 255) / 256;
  uint64_t* cds = (uint64_t*)sc.get("ls_chunk_deg", nch * 8);
  launch_chunk_degsum(d_seq, d_deg, n_seq, cds, s, nsd);
  if (c.h_chunks_n < nch) {
    if (c.h_chunks) HIP_CHECK(hipHostFree(c.h_chunks));
    c.h_chunks = nullptr;
    c.h_chunks_n = 0;
    HIP_CHECK(hipHostMalloc((void**)&c.h_chunks, nch * 8, hipHostMallocDefault));
    c.h_chunks_n = nch;
  }
  HIP_CHECK(hipMemcpyAsync(c.h_chunks, cds, nch * 8, hipMemcpyDeviceToHost, s));
  HIP_CHECK(hipEventRecord(c.bins_ev, s));
  // this shard's records -> items (hi, lo) grouped by bin
  const uint64_t mm = std::max<uint64_t>(m, 1);
  uint64_t* items = (uint64_t*)sc.get("ls_items", mm * 8);
  uint64_t* items_b = (uint64_t*)sc.get("ls_items_b", mm * 8);
  uint32_t* tmp = (uint32_t*)sc.get("ls_rsort_tmp", rsort_tmp_words(mm) * 4);
  uint16_t* digits = (uint16_t*)sc.get("ls_item_bins", mm * 2);
  const uint32_t* src = d_uv;
  const bool part = use_part(m);
  // the second pass's records packed to 6 bytes for the direct edge pass (ids_checked: an id
  // >= n_rank fails the caller anyway)
  const bool pre6 = part && knobs().bin_direct && m > 0 && n_seq > 0 && ids_checked &&
                    part_p6_ok(n_rank);
  uint32_t* pws = nullptr;
  if (part) {
    if (part_done) {  // pass 1 ran beside the degree all-reduce and the sequence
      pws = (uint32_t*)sc.get("part_ws", PART_WS_WORDS * 4);
      HIP_CHECK(hipStreamWaitEvent(s, part_done, 0));
      launch_part_second(items, m, d_rank, n_rank, items_b, pws, s, pre6, mid_slots, mid_caps,
                         mid_p6, ff_groups());
    } else {
      mid_caps = false;
      pws = (uint32_t*)sc.get("ls_part_ws", PART_WS_WORDS * 4);
      launch_part_gather(d_uv, m, d_rank, n_rank, items, items_b, pws, s, false, pre6);
    }
    src = (const uint32_t*)items_b;
  }
  HIP_CHECK(hipEventSynchronize(c.bins_ev));
  std::vector<uint64_t> hd(c.h_chunks, c.h_chunks + nch);
  std::vector<double> est;
  L.bounds = make_bins(hd, n_seq, &est);
  const uint32_t nb = (uint32_t)L.bounds.size();
  L.bins = (uint32_t*)sc.get("ls_bins", 512 * 4);
  HIP_CHECK(hipMemcpyAsync(L.bins, L.bounds.data(), nb * 4, hipMemcpyHostToDevice, s));
  mid_caps = mid_caps && part && part_done;
  bool part_ovf = false, part_checked = false;
  // Direct binning, as the one-GPU path: this shard's share of each bin's estimate (the bins
  // and estimates are global) sizes its capacity; a bin that outgrows it sends this rank
  // through the scatter below (ranks may differ in that: only per-bin counts are exchanged).
  if (knobs().bin_direct && m > 0) {
    double W = 0;
    for (double e : est) W += e;
    const double share = W > 0 ? std::min(1.0, (double)m / W) : 1.0;
    const double slack = 1.0 + knobs().bin_slack / 1000.0;
    L.cstart.assign(nb, 0ull);
    std::vector<unsigned long long> h(3 * 512, 0ull);
    for (uint32_t i = 0; i + 1 < nb; ++i) {
      const uint64_t cap = std::min<uint64_t>((uint64_t)std::ceil(est[i] * share * slack) + 8192, m);
      L.cstart[i + 1] = L.cstart[i] + cap;
      h[i] = h[512 + i] = L.cstart[i];
      h[1024 + i] = L.cstart[i + 1];
    }
    L.dseg = (unsigned long long*)sc.get("ls_bin_segs", h.size() * 8);
    HIP_CHECK(hipMemcpyAsync(L.dseg, h.data(), h.size() * 8, hipMemcpyHostToDevice, s));
    uint32_t* ovf = (uint32_t*)sc.get("ls_ovf", 4);
    HIP_CHECK(hipMemsetAsync(ovf, 0, 4, s));
    uint64_t* binned = (uint64_t*)sc.get("ls_binned", std::max<uint64_t>(L.cstart[nb - 1], 1) * 8);
    launch_edge_bin(src, part, m, d_rank, n_rank, d_err, L.bins, nb, L.dseg + 512, L.dseg + 1024,
                    binned, ovf, s, pre6 ? pws : nullptr);
    std::vector<unsigned long long> cur(nb);
    HIP_CHECK(hipMemcpyAsync(cur.data(), L.dseg + 512, nb * 8, hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipMemcpyAsync(L.h_pinned, ovf, 4, hipMemcpyDeviceToHost, s));
    L.h_pinned[1] = 0;
    if (mid_caps) HIP_CHECK(hipMemcpyAsync(L.h_pinned + 1, d_err + 3, 4, hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipStreamSynchronize(s));
    part_checked = true;
    part_ovf = mid_caps && L.h_pinned[1] != 0;
    if (L.h_pinned[0] == 0 && !part_ovf) {
      L.direct = true;
      L.sorted = binned;
      for (uint32_t i = 0; i + 1 < nb; ++i) counts_out[i] = cur[i] - L.cstart[i];
      counts_out[nb - 1] = 0;  // INVALID his are not stored (no bucket reads them)
      *nb_out = nb;
      return;
    }
  }
  if (mid_caps && !part_checked) {  // (no direct binning: the regions' overflow word alone)
    HIP_CHECK(hipMemcpyAsync(L.h_pinned + 1, d_err + 3, 4, hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipStreamSynchronize(s));
    part_ovf = L.h_pinned[1] != 0;
  }
  // A bin overflowed (the scatter path reads unpacked records), or a capacity region of the
  // first pass did (its records are incomplete): partition again from the records.
  if (pre6 || part_ovf) {
    uint32_t* pws2 = (uint32_t*)sc.get("ls_part_ws", PART_WS_WORDS * 4);
    launch_part_gather(d_uv, m, d_rank, n_rank, items, items_b, pws2, s, false, false);
  }
  unsigned long long* dstart = (unsigned long long*)sc.get("ls_bin_start", 513 * 8);
  L.sorted = group_by_bins(src, part, m, d_rank, n_rank, d_err, L.bins, nb, items, items_b, tmp,
                           digits, dstart, s);
  if (m) {
    L.local_start.resize(nb + 1);
    HIP_CHECK(hipMemcpyAsync(L.local_start.data(), dstart, (nb + 1) * 8, hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipStreamSynchronize(s));
  } else {
    L.local_start.assign(nb + 1, 0ull);
  }
  for (uint32_t i = 0; i < nb; ++i) counts_out[i] = L.local_start[i + 1] - L.local_start[i];
  *nb_out = nb;
}

// The split apply for rank `rank` of P (P > 1; after ls_begin).  Its own buffers are taken from
// the session's scratch; kept_hint: the largest P * cap the loop will apply (0: grown on demand).
static void ls_plan_sweeps(Lockstep& L);

static void ls_set_split(Lockstep& L, uint32_t rank, uint32_t P, uint64_t kept_hint) {
  if (P < 2 || rank >= P) throw ApiError(-EINVAL, "lockstep split: rank out of range or P < 2");
  Scratch& sc = *L.scp;
  L.split = true;
  L.rank = rank;
  L.P = P;
  HIP_CHECK(hipStreamCreateWithFlags(&L.zs, hipStreamNonBlocking));
  for (int z = 0; z < 2; ++z) {
    L.zbm[z] = (uint32_t*)sc.get(z ? "ls_zbm1" : "ls_zbm0", L.bm_words * 4);
    L.zn[z] = (uint32_t*)sc.get(z ? "ls_zn1" : "ls_zn0", 16);
    if (kept_hint) {
      L.zkept_bytes[z] = kept_hint * 8;
      L.zkept[z] = (uint64_t*)sc.get(z ? "ls_zkept1" : "ls_zkept0", L.zkept_bytes[z]);
    }
    HIP_CHECK(hipEventCreateWithFlags(&L.zready[z], hipEventDisableTiming));
    HIP_CHECK(hipEventCreateWithFlags(&L.zdone[z], hipEventDisableTiming));
  }
  L.zspq = (uint32_t*)sc.get("ls_zspq", L.spq_words * 4);
  ls_plan_sweeps(L);  // (the spacing depends on P; a no-op before ls_plan)
}

// Giant sweeps as the one-GPU loop's (sweep_plan), the birth from the global records per bucket,
// the spacing from this rank's share of them: a sweep costs every rank a pass over the ranks,
// and spares only the finds of its own maps (its bitmap is its own; the maps resolve their
// misses with finds, so the exchanged pairs do not change).  At P = 8 with the one-GPU spacing:
// maps 2.4 -> 1.8 ms per rank, applies 3.5-4.2 -> 4.4-5.0 ms (profiles/r05/i_sim/).
static void ls_plan_sweeps(Lockstep& L) {
  if (L.bk.size() < 2) { L.sweep.clear(); return; }
  auto grecs = [&](size_t k) { return L.global_e[k]; };
  auto mine = [&](size_t k) { return L.global_e[k] / std::max<uint32_t>(L.P, 1); };
  L.sweep = sweep_plan(L.bk, mine, birth_window(L.bk, grecs), L.n_seq);
}

static void ls_plan(Lockstep& L, const uint64_t* global_counts, uint32_t* nbk_out,
                    uint32_t* ms_out) {
  const uint32_t nb = (uint32_t)L.bounds.size();
  std::vector<unsigned long long> gstart(nb + 1, 0ull);
  for (uint32_t i = 0; i < nb; ++i) gstart[i + 1] = gstart[i] + global_counts[i];
  L.bk.clear();
  L.global_e.clear();
  L.ms = 0;
  if (L.n_seq == 0) {
    *nbk_out = 0;
    *ms_out = 0;
    return;
  }
  // the lockstep loop merges at 0.2 %: at the one-GPU loop's 0.35 % the giant of RMAT-26 forms
  // where the P = 8 simulation's tree critical path goes 6.7 -> 16.4 ms
  std::vector<uint32_t> cuts = bucket_cuts(L.bounds, gstart, gstart[nb], L.n_seq, 40,
                                           knobs().kb_merge > 0 ? 20 : 0, /*one_gpu=*/false);
  std::vector<uint32_t> bi;  // bin index at each bucket start, then nb - 1 (the INVALID bin)
  bi.push_back(0);
  for (uint32_t i : cuts) bi.push_back(i);
  bi.push_back(nb - 1);
  for (size_t k = 0; k < bi.size(); ++k) {
    const uint32_t r = k + 1 < bi.size() ? L.bounds[bi[k]] : L.n_seq;
    L.bk.emplace_back(r, L.direct ? (uint64_t)bi[k] : (uint64_t)L.local_start[bi[k]]);
  }
  for (size_t k = 0; k + 1 < bi.size(); ++k) {
    L.global_e.push_back(gstart[bi[k + 1]] - gstart[bi[k]]);
    const uint32_t B0 = L.bk[k].first, B1 = L.bk[k + 1].first;
    if (B1 > B0) L.ms = std::max<uint32_t>(L.ms, (((B1 - 1) >> 5) - (B0 >> 5) + 2) / 2);
  }
  *nbk_out = (uint32_t)L.global_e.size();
  *ms_out = L.ms;
  ls_plan_sweeps(L);
}

// d_count (nullable, device int64) receives the count without a host round trip;
// n_kept_out (nullable) receives it on the host (synchronises).
static void ls_map(Lockstep& L, uint32_t k, uint64_t* d_send, long long* d_count,
                   uint32_t* n_kept_out, hipStream_t s) {
  if (k >= L.global_e.size()) throw ApiError(-EINVAL, "lockstep: bucket index out of range");
  const uint32_t B0 = L.bk[k].first;
  // the anchor of this map was picked by the apply of bucket k-1 (on the apply's stream)
  if (L.anc && k >= 1) HIP_CHECK(hipStreamWaitEvent(s, L.pick_ev[k & 1], 0));
  auto ev = L.span(L.map_ev, s);
  KbSegs sg{};
  if (L.direct)
    sg = {L.dseg, L.dseg + 512, L.dseg + 1024, (uint32_t)L.bk[k].second,
          (uint32_t)L.bk[k + 1].second};
  // d_send holds ms mark words, then at least min(span, m) pair slots — the caller's contract:
  // multi_tree sizes it by the largest bucket span over the ranks, the Python mirror
  // (sheep_amd/dist.py) by this shard's records.  The map keeps at most one pair per record
  // of the bucket, which is at most both, so kept_cap (the kept-pair guard, FAULT bit 4)
  // bounds the writes by the buffer in either case (the span alone can exceed the
  // Python buffer, since directly binned spans include the bins' slack).
  const uint64_t e0 = L.direct ? L.cstart[L.bk[k].second] : L.bk[k].second;
  const uint64_t e1 = L.direct ? L.cstart[L.bk[k + 1].second] : L.bk[k + 1].second;
  const uint64_t kcap = std::min<uint64_t>(e1 - e0, std::max<uint64_t>(L.m, 1));
  launch_kb_map(L.sorted, e0, e1, B0, L.anchor(k),
                L.uf, L.label, d_send + L.ms, kcap, L.bm_of(k), L.cnt_of(k), 0, L.hcnt,
                false, L.ws,
                L.bins, (uint32_t)L.bounds.size(), L.gbits, L.gbits ? L.gx + (k & 1) : nullptr,
                L.split ? 2 : (int)L.defer, s, L.direct ? &sg : nullptr,
                L.anc ? L.anc + (k & 1) : nullptr,
                k >= 1 ? L.gsum : nullptr);
  HIP_CHECK(hipEventRecord(ev.second, s));
  if (d_count) launch_ls_count(L.cnt_of(k) + 3, d_count, s);
  if (n_kept_out) {
    HIP_CHECK(hipMemcpyAsync(L.h_pinned, L.cnt_of(k) + 3, 4, hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipStreamSynchronize(s));
    *n_kept_out = L.h_pinned[0];
  }
}

static void ls_words(const Lockstep& L, uint32_t k, uint32_t* w0, uint32_t* w1) {
  const uint32_t B0 = L.bk[k].first, B1 = L.bk[k + 1].first;
  *w0 = B0 >> 5;
  *w1 = B1 > B0 ? (B1 - 1) >> 5 : B0 >> 5;
}

static void ls_pack(Lockstep& L, uint32_t k, uint64_t* d_send, uint32_t cap, hipStream_t s) {
  if (k >= L.global_e.size()) throw ApiError(-EINVAL, "lockstep: bucket index out of range");
  uint32_t w0, w1;
  ls_words(L, k, &w0, &w1);
  launch_ls_pack(L.bm_of(k), w0, w1, L.ms, d_send, L.cnt_of(k) + 3, cap, s);
}

// solo (a group of one, nothing exchanged): d_recv is the map's own output buffer of bucket k
// (its kept pairs at d_recv + S, their count and the marks where the map left them), applied
// in place; cap is ignored.
static void ls_apply(Lockstep& L, uint32_t k, const uint64_t* d_recv, uint32_t P, uint32_t cap,
                     hipStream_t s, bool solo = false) {
  if (k >= L.global_e.size()) throw ApiError(-EINVAL, "lockstep: bucket index out of range");
  const uint32_t B0 = L.bk[k].first, B1 = L.bk[k + 1].first;
  uint32_t w0, w1;
  ls_words(L, k, &w0, &w1);
  const size_t need = std::max<uint64_t>((uint64_t)P * cap, 1) * 8;  // the unpacked pairs
  uint64_t* kept = nullptr;  // where the replicated apply reads the pairs (not split)
  if (solo) {
    kept = (uint64_t*)d_recv + L.ms;
  } else if (!L.split) {
    // a larger kept buffer replaces one that earlier applies (on s) may still read: drain s
    // first.  multi_tree sizes it before its loop, so this only happens through the sheep_ls_*
    // calls (their caller gives no bound)
    if (L.kept_bytes == 0) L.kept_bytes = L.scp->bytes_of("ls_kept_all");
    if (need > L.kept_bytes) {
      if (L.presized) throw ApiError(-EIO, "lockstep: kept pairs beyond the pre-sized buffer");
      HIP_CHECK(hipStreamSynchronize(s));
      L.kept_bytes = std::max(need, L.kept_bytes * 5 / 4);
    }
    kept = (uint64_t*)L.scp->get("ls_kept_all", L.kept_bytes);
  }
  // the anchor of map k+1 first: the union-find is as bucket k-1 left it (the caller applies
  // in order on one stream and has waited for map k), and map k+1 waits for this pick
  size_t gslot = k;  // the bitmap slot most recently written on this stream
  if (L.anc && k + 1 < L.global_e.size()) {
    const uint32_t a = L.anchor(k + 1);
    launch_kb_pick(L.uf, a == INV ? 0u : a + 1, L.anc + (k & 1), L.anc + ((k + 1) & 1), L.gbits,
                   L.n_seq, L.gbits ? L.gx + (k & 1) : nullptr,
                   L.gbits ? L.gx + ((k + 1) & 1) : nullptr, s);
    // map k+1 reads the summary; the next one is written by apply k+1, after map k+1 is done
    if (L.gsum) launch_gb_sum(L.gbits, L.n_seq, L.gsum, s);
    HIP_CHECK(hipEventRecord(L.pick_ev[(k + 1) & 1], s));
    gslot = k + 1;
  }
  std::pair<hipEvent_t, hipEvent_t> ev{nullptr, nullptr};
  if (L.time_apply) ev = L.span(L.apply_ev, s);
  if (L.split) {
    // Every rank: the marks (OR over ranks), the fold, the union of the pairs read straight
    // from d_recv (their starts need no refresh for that), the labels.  The bucket's owner
    // first unpacks the pairs into its slot and refreshes them there (the zipper needs the
    // pre-bucket roots, against the union-find as bucket k-1 left it), then hands them to zs.
    const bool ne = L.global_e[k] > 0;
    const uint32_t* gx = L.gbits ? L.gx + (gslot & 1) : nullptr;
    const uint32_t* anc_k = L.anc ? L.anc + (k & 1) : nullptr;
    if (ne && k % L.P == L.rank) {
      const int z = L.nzip++ & 1;
      if (L.zused[z]) HIP_CHECK(hipStreamWaitEvent(s, L.zdone[z], 0));  // the slot's last zipper
      if (need > L.zkept_bytes[z]) {  // (pre-sized by multi_tree: only via sheep_ls_*)
        if (L.presized) throw ApiError(-EIO, "lockstep: kept pairs beyond the pre-sized buffer");
        // the slot's last readers: the zipper on zs (waited for above) and the unpack on s
        HIP_CHECK(hipStreamSynchronize(s));
        HIP_CHECK(hipStreamSynchronize(L.zs));
        L.zkept_bytes[z] = std::max(need, L.zkept_bytes[z] * 5 / 4);
        L.zkept[z] = (uint64_t*)L.scp->get(z ? "ls_zkept1" : "ls_zkept0", L.zkept_bytes[z]);
      }
      launch_ls_unpack(d_recv, P, L.ms, cap, L.bm_of(k), w0, w1, L.zkept[z], L.zn[z], s);
      HIP_CHECK(hipMemcpyAsync(L.zbm[z] + w0, L.bm_of(k) + w0, (size_t)(w1 - w0 + 1) * 4,
                               hipMemcpyDeviceToDevice, s));
      launch_kb_refresh(L.zkept[z], L.zn[z], L.uf, L.label, L.zbm[z], B0, L.anchor(k), L.gbits, gx,
                        anc_k, s);
      launch_ls_gslot(L.uf, L.label, L.anchor(k), anc_k, L.zn[z] + 2, s);
      HIP_CHECK(hipEventRecord(L.zready[z], s));
      HIP_CHECK(hipStreamWaitEvent(L.zs, L.zready[z], 0));
      auto zev = L.span(L.zip_ev, L.zs);
      launch_ls_zip(L.zkept[z], L.zn[z], L.zbm[z], L.zspq, B0, B1, L.anchor(k) != INV, L.parent,
                    L.jump, L.zs);
      HIP_CHECK(hipEventRecord(zev.second, L.zs));
      HIP_CHECK(hipEventRecord(L.zdone[z], L.zs));
      L.zused[z] = true;
    } else {
      launch_ls_unpack(d_recv, P, L.ms, cap, L.bm_of(k), w0, w1, nullptr, nullptr, s);
    }
    launch_ls_fold_union_label(ne, B0, B1, L.anchor(k), L.uf, L.label, d_recv, P, L.ms, cap,
                               L.bm_of(k), L.cnt_of(k), L.gbits, gx, s, anc_k,
                               L.anc ? L.anc + ((k + 1) & 1) : nullptr);
  } else {
    if (!solo) launch_ls_unpack(d_recv, P, L.ms, cap, L.bm_of(k), w0, w1, kept, L.cnt_of(k) + 3, s);
    launch_kb_apply(L.global_e[k] > 0, B0, B1, L.anchor(k), L.uf, L.label, L.parent, L.jump, kept,
                    L.linked, L.bm_of(k), L.spq_of(k), L.cnt_of(k), L.pipe, false, L.ws, L.gbits,
                    L.gbits ? L.gx + (gslot & 1) : nullptr, s, L.anc ? L.anc + (k & 1) : nullptr,
                    L.anc ? L.anc + ((k + 1) & 1) : nullptr);
  }
  // (after the apply, before the next pick on this stream: nothing may move the bitmap's vertex
  // beside a sweep; the map of bucket k + 1 runs beside it)
  if (k < L.sweep.size() && L.sweep[k] && L.gbits)
    launch_gb_sweep(L.uf, L.gbits, B1, L.gx + (gslot & 1), s);
  if (ev.second) HIP_CHECK(hipEventRecord(ev.second, s));
}

// The session's kernel-span sums (after its work has completed) -> c.timings.
static void ls_timings(Ctx& c, Lockstep& L);

// sync = false: only enqueued (the caller synchronises, then calls ls_timings).
// d_pst nullable: pst already computed (multi_tree does it beside the last applies).
static void ls_finish(Ctx& c, Lockstep& L, const uint32_t* d_seq, const uint32_t* d_deg,
                      const uint32_t* d_selfc, int mode, uint32_t* d_parent, uint32_t* d_pst,
                      hipStream_t s, bool sync = true) {
  for (int z = 0; z < 2; ++z)  // split: this rank's zippers
    if (L.zused[z]) HIP_CHECK(hipStreamWaitEvent(s, L.zdone[z], 0));
  if (L.n_seq) {
    if (d_pst) launch_pst_from_count(d_seq, L.n_seq, d_deg, d_selfc, mode, L.hcnt, d_pst, s);
    launch_pj_parents(L.parent, L.n_seq, d_parent, s);
  }
  if (!sync) return;
  HIP_CHECK(hipStreamSynchronize(s));
  ls_timings(c, L);
}

static void ls_timings(Ctx& c, Lockstep& L) {
  c.timings.clear();
  c.span_names.clear();
  auto sum = [&](const char* name, std::vector<std::pair<hipEvent_t, hipEvent_t>>& v) {
    if (v.empty()) return;
    double t = 0;
    for (auto& e : v) {
      float ms = 0;
      (void)hipEventElapsedTime(&ms, e.first, e.second);
      t += ms;
    }
    c.timings.emplace_back(name, t);
    const std::string nm(name);
    c.timings.emplace_back(nm == "kb_map" ? "kb_map#" : nm == "kb_zip" ? "kb_zip#" : "kb_apply#",
                           (double)v.size());
  };
  sum("kb_map", L.map_ev);
  sum("kb_apply", L.apply_ev);
  if (L.split) sum("kb_zip", L.zip_ev);
}

// ---- the degree sequence of P ranks, sharded (mpiSequence, sequence.h:65-93) ---------------
// Instead of every rank sorting all ids after an all-reduce of the degrees: the degrees are
// reduce-scattered (rank r gets the global degrees of ids [r c, (r + 1) c)), each rank sorts
// only its ids (stable, by degree), the ranks' histograms over degree values are all-gathered,
// and each rank computes the global position of its ids from them (launch_seq_rank; ids of
// different ranks never interleave within a degree).  One all-gather of the rank slices gives
// every rank the whole rank map, from which it scatters seq.  Returns n_seq; rank: n_pad
// words (>= n_ids; INVALID for degree 0); *nsd_out: the global degrees in sequence order (for
// the bins' estimate).  The same result as all-reduce + sequence_dev.
static uint32_t sequence_sharded(Ctx& c, Comm& comm, const uint32_t* deg_local, uint32_t n_ids,
                                 uint32_t* d_seq, uint32_t** rank_out, const uint32_t** nsd_out,
                                 hipStream_t s) {
  Scratch& sc = c.scratch;
  const uint32_t P = (uint32_t)comm.size(), r = (uint32_t)comm.rank();
  uint64_t cw = ((uint64_t)n_ids + P - 1) / P;
  cw += cw & 1;  // even: the all-gathers move u64 words
  const uint64_t n_pad = cw * P;
  if (n_pad >= (1ull << 32)) throw ApiError(-EINVAL, "sharded sequence: id space too large");
  const uint32_t cs = (uint32_t)cw;
  uint32_t* send = (uint32_t*)sc.get("sq_send", n_pad * 4);
  HIP_CHECK(hipMemcpyAsync(send, deg_local, (size_t)n_ids * 4, hipMemcpyDeviceToDevice, s));
  if (n_pad > n_ids) HIP_CHECK(hipMemsetAsync(send + n_ids, 0, (size_t)(n_pad - n_ids) * 4, s));
  uint32_t* dsl = (uint32_t*)sc.get("sq_slice", (size_t)cs * 4);
  comm.reduce_scatter_sum_u32(send, dsl, cs, s);
  uint32_t* stats = (uint32_t*)sc.get("sq_stats", 16);
  launch_deg_stats(dsl, cs, stats, s);
  long long* st64 = (long long*)sc.get("sq_st64", 32);
  launch_seq_stats64(stats, cs, st64, s);
  HIP_CHECK(hipMemcpyAsync(st64 + 2, st64 + 1, 8, hipMemcpyDeviceToDevice, s));
  comm.allreduce_max_i64((int64_t*)st64, 1, s);           // [0] max degree over all ranks
  comm.allreduce_sum_u64((uint64_t*)st64 + 2, 1, s);     // [2] ids of degree > 0 over all ranks
  long long h[3];
  HIP_CHECK(hipMemcpyAsync(h, st64, 24, hipMemcpyDeviceToHost, s));
  HIP_CHECK(hipStreamSynchronize(s));
  const uint32_t maxdeg = (uint32_t)h[0], n_loc = (uint32_t)h[1];
  const uint32_t n_seq = (uint32_t)h[2];
  uint32_t* rank = (uint32_t*)sc.get("mt_rank", n_pad * 4);
  *rank_out = rank;
  *nsd_out = nullptr;
  launch_fill(rank + (size_t)r * cs, INV, cs, s);
  if (n_seq == 0) {
    comm.allgather_u64((const uint64_t*)(rank + (size_t)r * cs), (uint64_t*)rank, cs / 2, s);
    return 0;
  }
  // The histograms over degree values are all-gathered: P x (max degree + 1) words.  When that
  // is more than the degree slices themselves (a hub of high degree; or max degree 2^32 - 1,
  // where max degree + 1 wraps), all-gather the slices instead and sort every id on every rank
  // (maxdeg is the same on every rank here, so every rank takes the same branch).
  if ((uint64_t)maxdeg + 1 > (uint64_t)cs) {
    uint32_t* dall = (uint32_t*)sc.get("sq_deg_all", n_pad * 4);
    comm.allgather_u64((const uint64_t*)dsl, (uint64_t*)dall, cs / 2, s);
    uint32_t* nsd = (uint32_t*)sc.get("sq_nsd", (size_t)n_seq * 4);
    const uint32_t n2 = sequence_dev(c, dall, n_ids, d_seq, rank, s, false, nsd);
    if (n2 != n_seq) throw ApiError(-EIO, "sharded sequence: id counts disagree");
    // rank holds n_pad words, INVALID past the id space (as the sharded path's fill + gather)
    if (n_pad > n_ids) launch_fill(rank + n_ids, INV, n_pad - n_ids, s);
    *nsd_out = nsd;
    return n_seq;
  }
  const uint32_t D = maxdeg + 1, Dp = D + (D & 1);
  // this rank's ids of degree > 0, sorted stably by degree (local ids: global - r c)
  const int passes = (bits_for(maxdeg) + 7) / 8;
  uint64_t* items = (uint64_t*)sc.get("seq_items", (size_t)cs * 8);
  uint64_t* items_b = (uint64_t*)sc.get("seq_items_b", (size_t)cs * 8);
  uint32_t* tmp = (uint32_t*)sc.get("rsort_tmp", rsort_tmp_words(cs) * 4);
  uint32_t* ptmp = (uint32_t*)sc.get("seq_pack_tmp", pack_nz_tmp_words(cs) * 4);
  launch_pack_nonzero(dsl, cs, items, ptmp, s);
  const uint64_t* sorted = n_loc ? radix_sort_u64(items, items_b, items, n_loc, 0, 8 * passes, tmp, s)
                                 : items;
  uint32_t* H = (uint32_t*)sc.get("sq_hist", (size_t)Dp * 4);
  uint32_t* lst = (uint32_t*)sc.get("sq_lst", (size_t)D * 4);
  HIP_CHECK(hipMemsetAsync(H, 0, (size_t)Dp * 4, s));
  launch_seq_runs(sorted, n_loc, lst, H, s);
  uint32_t* hall = (uint32_t*)sc.get("sq_hall", (size_t)P * Dp * 4);
  comm.allgather_u64((const uint64_t*)H, (uint64_t*)hall, Dp / 2, s);
  uint32_t* tot = (uint32_t*)sc.get("sq_tot", (size_t)D * 4);
  uint32_t* pre = (uint32_t*)sc.get("sq_pre", (size_t)D * 4);
  uint32_t* S = (uint32_t*)sc.get("sq_S", (size_t)D * 4);
  uint32_t* stmp = (uint32_t*)sc.get("sq_scan_tmp", scan_tmp_words(D) * 4);
  launch_seq_base(hall, P, r, D, Dp, tot, pre, s);
  launch_scan_exclusive(tot, S, D, stmp, s);
  launch_seq_rank(sorted, n_loc, S, pre, lst, rank + (size_t)r * cs, s);
  comm.allgather_u64((const uint64_t*)(rank + (size_t)r * cs), (uint64_t*)rank, cs / 2, s);
  launch_seq_from_rank(rank, n_ids, d_seq, s);
  uint32_t* nsd = (uint32_t*)sc.get("sq_nsd", (size_t)n_seq * 4);
  launch_deg_of_rank(S, D, n_seq, nsd, s);
  *nsd_out = nsd;
  return n_seq;
}

// ---- graph2tree -i -r on one rank (the multi-GPU driver) ------------------------------------
// This rank's shard -> its degrees, summed over the ranks (mpiSequence's MPI_Allreduce,
// sequence.h:72-78) -> the identical seq / rank on every rank -> the lockstep tree over all
// shards (every rank maps its own records per bucket; the kept pairs and marks of all ranks are
// all-gathered and applied by every rank) -> pst_weight summed (the merge adds the partial
// trees' pst, jnode.cpp:174-201).  Every rank ends with seq, parent and pst.  seq_given: d_seq
// already holds n_seq ids (sheep_build_tree_multi); else it is computed (n_ids entries).
static uint32_t multi_tree(Ctx& c, Comm& comm, const uint32_t* d_uv, uint64_t m, uint32_t n_ids,
                           int mode, uint32_t* d_seq, bool seq_given, uint32_t n_seq_given,
                           uint32_t* d_parent, uint32_t* d_pst, hipStream_t s, Timer* tm) {
  require_records(m, "multi tree");
  const size_t n = std::max<uint32_t>(n_ids, 1);
  uint32_t* deg_local = (uint32_t*)c.scratch.get("mt_deg_local", n * 4);
  uint32_t* selfc = (uint32_t*)c.scratch.get("mt_selfc", n * 4);
  uint32_t* deg = (uint32_t*)c.scratch.get("mt_deg", n * 4);
  uint32_t* rank = (uint32_t*)c.scratch.get("mt_rank", n * 4);
  // The front half of this rank's shard, as graph2tree_dev's: from 2^25 records ONE read of the
  // shard gives its degrees and the first partition pass of the rank gathers, packed into
  // sampled capacity regions (launch_front_fused; part_overlap 4).  Else the first pass, which
  // needs no ranks, runs on the side stream beside the degree pass, the degree collectives and
  // the sequence.
  const int ov = knobs().part_overlap;
  const bool ffused = ov == 4 && m >= (1ull << 25) && use_part(m) && knobs().bin_direct &&
                      knobs().degree != 1 && part_p6_ok(n_ids) && front_fused_ok(m, n_ids) &&
                      degs_tmp_words(m, n_ids) > 1;
  const uint64_t mid_slots = ffused ? front_fused_slots(m, n_ids, ff_groups()) : m;
  const bool overlap = !ffused && ov != 0 && m > 0 && use_part(m);
  hipEvent_t part_done = nullptr;
  if (ffused) {
    uint32_t* ovf_deg = c.d_err + 2;
    HIP_CHECK(hipMemsetAsync(ovf_deg, 0, 8, s));  // both overflow words ([3]: the partition's)
    uint32_t* tmp = (uint32_t*)c.scratch.get("degs_tmp", degs_tmp_words(m, n_ids) * 4);
    uint32_t* pws = (uint32_t*)c.scratch.get("part_ws", PART_WS_WORDS * 4);
    // (at least m u64: ls_begin takes the same buffer at that size and must not regrow it)
    uint64_t* mid = (uint64_t*)c.scratch.get("ls_items", std::max<uint64_t>(m, mid_slots) * 8);
    uint32_t* stats = (uint32_t*)c.scratch.get("stats", 16);
    launch_front_fused(d_uv, m, n_ids, mode, deg_local, selfc, c.d_err, tmp, pws, mid, mid_slots,
                       stats, ovf_deg, c.d_err + 3, s, nullptr, nullptr, ff_groups());
    HIP_CHECK(hipEventRecord(c.part_ev[1], s));
    part_done = c.part_ev[1];
    // this shard's degrees are complete unless a region outgrew its capacity — an x bucket, or
    // a y digit, whose ids the histogram counts from the packed records (a local decision: the
    // exact pass has no collectives)
    HIP_CHECK(hipMemcpyAsync(c.h_pinned + 4, ovf_deg, 8, hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipStreamSynchronize(s));
    if (tm) tm->mark("front_fused");
    if (c.h_pinned[4] || c.h_pinned[5]) {
      degree_dev(c, d_uv, m, n_ids, mode, deg_local, selfc, s);
      if (tm) tm->mark("degree_exact");
    }
  }
  if (overlap) HIP_CHECK(hipEventRecord(c.part_ev[0], s));  // in case degree_dev records none
  const bool yh = ffused ? false
                         : degree_dev(c, d_uv, m, n_ids, mode, deg_local, selfc, s, overlap,
                                      overlap ? c.part_ev[0] : nullptr);
  if (overlap) {
    uint64_t* mid = (uint64_t*)c.scratch.get("ls_items", m * 8);
    uint32_t* pws = (uint32_t*)c.scratch.get("part_ws", PART_WS_WORDS * 4);
    HIP_CHECK(hipStreamWaitEvent(c.side, c.part_ev[0], 0));
    launch_part_first(d_uv, m, n_ids, mid, pws, c.side, yh);
    HIP_CHECK(hipEventRecord(c.part_ev[1], c.side));
    part_done = c.part_ev[1];
  }
  uint32_t n_seq = n_seq_given;
  const uint32_t* nsd = nullptr;  // sharded: the global degrees in sequence order
  if (!seq_given && comm.size() > 1 && knobs().ls_seq) {
    if (tm) tm->mark("degree");
    n_seq = sequence_sharded(c, comm, deg_local, n_ids, d_seq, &rank, &nsd, s);
  } else {
    if (n_ids) HIP_CHECK(hipMemcpyAsync(deg, deg_local, (size_t)n_ids * 4, hipMemcpyDeviceToDevice, s));
    comm.allreduce_sum_u32(deg, n_ids, s);
    if (tm) tm->mark("degree");
    if (!seq_given) {
      n_seq = sequence_dev(c, deg, n_ids, d_seq, rank, s);
    } else {
      launch_fill(rank, INV, n_ids, s);
      launch_rank_scatter(d_seq, n_seq, rank, c.d_err, s);
    }
  }
  // a range error of any rank's degree pass fails every rank here, after the same collectives
  // (a rank throwing alone would leave the others waiting in the next one)
  check_err_group(c, comm, s);
  if (tm) tm->mark("sequence");
  // the lockstep session keeps its buffers in this context's scratch
  Lockstep L;
  L.ctx = &c;
  L.scp = &c.scratch;
  L.defer = comm.size() == 1;
  L.time_apply = false;
  c.ls_live++;
  std::vector<uint64_t> counts(513, 0);
  uint32_t nb = 0;
  ls_begin(L, d_uv, m, rank, n_ids, d_seq, n_seq, deg, counts.data(), &nb, c.d_err, s, part_done,
           nsd, true, mid_slots, ffused, ffused);
  if (part_done) HIP_CHECK(hipStreamWaitEvent(s, part_done, 0));  // also when no tree is built
  check_err_group(c, comm, s);
  uint64_t* dcounts = (uint64_t*)c.scratch.get("mt_counts", 513 * 8);
  HIP_CHECK(hipMemcpyAsync(dcounts, counts.data(), (size_t)nb * 8, hipMemcpyHostToDevice, s));
  comm.allreduce_sum_u64(dcounts, nb, s);
  HIP_CHECK(hipMemcpyAsync(counts.data(), dcounts, (size_t)nb * 8, hipMemcpyDeviceToHost, s));
  HIP_CHECK(hipStreamSynchronize(s));
  uint32_t nbk = 0, S = 0;
  ls_plan(L, counts.data(), &nbk, &S);
  // The exchange buffers, sized once: a rank keeps at most one pair per record of the bucket,
  // so the MAX over ranks and buckets of a rank's records in one bucket bounds every all-gather
  // width (no allocation inside the loop).
  uint64_t max_recs = 0;
  for (uint32_t k = 0; k < nbk; ++k) {
    const uint64_t a = L.direct ? L.cstart[L.bk[k].second] : L.bk[k].second;
    const uint64_t b = L.direct ? L.cstart[L.bk[k + 1].second] : L.bk[k + 1].second;
    max_recs = std::max<uint64_t>(max_recs, b - a);
  }
  int64_t* d_max = (int64_t*)c.scratch.get("mt_max", 8);
  HIP_CHECK(hipMemcpyAsync(d_max, &max_recs, 8, hipMemcpyHostToDevice, s));
  comm.allreduce_max_i64(d_max, 1, s);
  HIP_CHECK(hipMemcpyAsync(&max_recs, d_max, 8, hipMemcpyDeviceToHost, s));
  HIP_CHECK(hipStreamSynchronize(s));
  if (tm) tm->mark("binned");
  // The bucket loop, pipelined: bucket k+1 is mapped and exchanged on the side stream while
  // bucket k is applied on s.  The host waits once per bucket, for the MAX over the ranks of
  // the kept counts (the all-gather's size).
  const int P = comm.size();
  hipStream_t s2 = c.side;
  const uint64_t cap_send = (uint64_t)S + std::max<uint64_t>(max_recs, 1);
  uint64_t* send = (uint64_t*)c.scratch.get("mt_send", cap_send * 8);
  uint64_t* recv[2] = {(uint64_t*)c.scratch.get("mt_recv0", (uint64_t)P * cap_send * 8),
                       (uint64_t*)c.scratch.get("mt_recv1", (uint64_t)P * cap_send * 8)};
  L.kept_bytes = 0;
  if (P > 1 && knobs().ls_split && n_seq)
    ls_set_split(L, (uint32_t)comm.rank(), (uint32_t)P, (uint64_t)P * cap_send);
  if (!L.split && P > 1)  // ls_apply's unpacked pairs, sized once
    (void)L.scp->get("ls_kept_all", (uint64_t)P * cap_send * 8);
  L.presized = true;
  int64_t* d_cnt = (int64_t*)c.scratch.get("mt_cnt", 8);
  uint32_t caps[2] = {0, 0};
  hipEvent_t* exchanged = c.kb_ev;
  hipEvent_t* applied = c.kb_ev + 2;
  // A group of one exchanges nothing: each map writes into recv[k & 1] (its kept pairs are
  // then where the apply reads them) and no count travels to the host.
  const bool solo = P == 1 && !L.split;
  auto produce = [&](uint32_t k) {
    const int p = k & 1;
    if (solo) {
      ls_map(L, k, recv[p], nullptr, nullptr, s2);
      HIP_CHECK(hipEventRecord(exchanged[p], s2));
      return;
    }
    ls_map(L, k, send, (long long*)d_cnt, nullptr, s2);
    comm.allreduce_max_i64(d_cnt, 1, s2);
    HIP_CHECK(hipMemcpyAsync(c.h_pinned, d_cnt, 8, hipMemcpyDeviceToHost, s2));
    HIP_CHECK(hipStreamSynchronize(s2));
    const uint32_t cap = (uint32_t)*(const int64_t*)c.h_pinned;
    const uint64_t width = (uint64_t)S + cap;
    if (width > cap_send) throw ApiError(-EIO, "lockstep: kept pairs exceed the bucket's records");
    ls_pack(L, k, send, cap, s2);
    comm.allgather_u64(send, recv[p], width, s2);
    HIP_CHECK(hipEventRecord(exchanged[p], s2));
    caps[p] = cap;
  };
  HIP_CHECK(hipEventRecord(c.kb_ev[4], s));  // s2 starts after everything before the loop
  HIP_CHECK(hipStreamWaitEvent(s2, c.kb_ev[4], 0));
  if (nbk) {
    produce(0);
    for (uint32_t k = 0; k < nbk; ++k) {
      HIP_CHECK(hipStreamWaitEvent(s, exchanged[k & 1], 0));
      ls_apply(L, k, recv[k & 1], (uint32_t)P, caps[k & 1], s, solo);
      HIP_CHECK(hipEventRecord(applied[k & 1], s));
      if (k + 1 < nbk) {
        if (k >= 1) HIP_CHECK(hipStreamWaitEvent(s2, applied[(k + 1) & 1], 0));
        produce(k + 1);
      }
    }
  }
  // pst needs only the maps' hi counts: it is computed and summed over the ranks on the map
  // stream, beside the last applies and zippers; the parent sum then waits for it (one
  // collective at a time on the communicator, in the same order on every rank)
  if (n_seq) {
    launch_pst_from_count(d_seq, n_seq, deg_local, selfc, mode, L.hcnt, d_pst, s2);
    if (P > 1) comm.allreduce_sum_u32(d_pst, n_seq, s2);
  }
  HIP_CHECK(hipEventRecord(c.kb_ev[4], s2));
  if (tm) tm->mark("tree");
  ls_finish(c, L, d_seq, deg_local, selfc, mode, d_parent, nullptr, s, false);
  HIP_CHECK(hipStreamWaitEvent(s, c.kb_ev[4], 0));
  if (L.split) {  // the owners' forests are disjoint: sum parent + 1 (INVALID + 1 = 0)
    launch_add_u32(d_parent, n_seq, 1u, s);
    comm.allreduce_sum_u32(d_parent, n_seq, s);
    launch_add_u32(d_parent, n_seq, INV, s);
  }
  if (tm) tm->mark("pst");
  HIP_CHECK(hipStreamSynchronize(s));
  ls_timings(c, L);
  // a walk guard or range error raised inside the bucket loop (maps, applies, zippers)
  check_err_group(c, comm, s);
  return n_seq;
}

}  // namespace sheep

using namespace sheep;

#define API_BEGIN try {
#define API_END                                                                               \
  }                                                                                           \
  catch (const ApiError& e) {                                                                 \
    g_last_error = e.what();                                                                  \
    return e.code;                                                                            \
  }                                                                                           \
  catch (const HipError& e) {                                                                 \
    g_last_error = e.what();                                                                  \
    return -EIO;                                                                              \
  }                                                                                           \
  catch (const std::bad_alloc&) {                                                             \
    g_last_error = "out of memory";                                                           \
    return -ENOMEM;                                                                           \
  }                                                                                           \
  catch (const std::exception& e) {                                                           \
    g_last_error = e.what();                                                                  \
    return -EIO;                                                                              \
  }                                                                                           \
  return SHEEP_OK;

static void require_aligned(const void* p, const char* what) {
  if (((uintptr_t)p) & 7u) throw ApiError(-EINVAL, std::string(what) + " must be 8-byte aligned");
}

extern "C" {

int sheep_abi_version(void) { return (1 << 16) | 0; }

const char* sheep_last_error(void) { return g_last_error.c_str(); }

int sheep_gpu_init(int device) {
  API_BEGIN
  init_ctx(device);
  g_last_error.clear();
  API_END
}

int sheep_release(void) {
  API_BEGIN
  Ctx& c = ctx();
  if (c.ls_live > 0) throw ApiError(-EBUSY, "sheep_release: a lockstep session is live");
  HIP_CHECK(hipStreamSynchronize(c.stream));
  c.scratch.release();
  API_END
}

int sheep_set_option(const char* name, long long value) {
  API_BEGIN
  if (!name) throw ApiError(-EINVAL, "null option name");
  Knobs& k = knobs();
  for (const KnobDef& d : kKnobs)
    if (!strcmp(d.name, name)) {
      k.*d.field = (int)value;
      return SHEEP_OK;
    }
  throw ApiError(-EINVAL, std::string("unknown option ") + name);
  API_END
}

int sheep_get_option(const char* name, long long* value) {
  API_BEGIN
  if (!name || !value) throw ApiError(-EINVAL, "null argument");
  Knobs& k = knobs();
  for (const KnobDef& d : kKnobs)
    if (!strcmp(d.name, name)) {
      *value = k.*d.field;
      return SHEEP_OK;
    }
  throw ApiError(-EINVAL, std::string("unknown option ") + name);
  API_END
}

int sheep_last_timings(const char** names, double* ms, int cap) {
  Ctx& c = g_ctx[g_device < 0 ? 0 : g_device];
  int n = std::min<int>(cap, (int)c.timings.size());
  for (int i = 0; i < n; ++i) {
    names[i] = c.timings[i].first;
    ms[i] = c.timings[i].second;
  }
  return n;
}

// ---- device-pointer API -------------------------------------------------------------------

int sheep_degree_dev(const uint32_t* d_uv, uint64_t m, uint32_t n_ids, int degree_mode,
                     uint32_t* d_deg, void* stream) {
  API_BEGIN
  Ctx& c = ctx();
  require_aligned(d_uv, "d_uv");
  if (degree_mode != SHEEP_DEGREE_LLAMA && degree_mode != SHEEP_DEGREE_FILE)
    throw ApiError(-EINVAL, "degree_mode");
  degree_dev(c, d_uv, m, n_ids, degree_mode, d_deg, nullptr, pick(c, stream));
  API_END
}

int sheep_degree_ex_dev(const uint32_t* d_uv, uint64_t m, uint32_t n_ids, int degree_mode,
                        uint32_t* d_deg, uint32_t* d_selfc, void* stream) {
  API_BEGIN
  Ctx& c = ctx();
  require_aligned(d_uv, "d_uv");
  if (degree_mode != SHEEP_DEGREE_LLAMA && degree_mode != SHEEP_DEGREE_FILE)
    throw ApiError(-EINVAL, "degree_mode");
  degree_dev(c, d_uv, m, n_ids, degree_mode, d_deg, d_selfc, pick(c, stream));
  API_END
}

int sheep_build_tree_deg_dev(const uint32_t* d_uv, uint64_t m, const uint32_t* d_rank,
                             uint32_t n_rank, const uint32_t* d_seq, uint32_t n_seq,
                             const uint32_t* d_deg, const uint32_t* d_selfc, int degree_mode,
                             uint32_t* d_parent, uint32_t* d_pst, void* stream) {
  API_BEGIN
  Ctx& c = ctx();
  require_aligned(d_uv, "d_uv");
  hipStream_t s = pick(c, stream);
  Timer tm(s);
  DegInfo di;
  di.seq = d_seq;
  di.deg = d_deg;
  di.selfc = d_selfc;
  di.mode = degree_mode;
  build_tree_dev(c, d_uv, m, d_rank, n_rank, n_seq, d_parent, d_pst, s, &tm, &di);
  check_err(c, s);
  tm.finish(c);
  API_END
}

int sheep_merge_forests_dev(const uint32_t* d_parents, uint32_t n_trees, uint32_t n,
                            uint32_t* d_parent_out, void* stream) {
  API_BEGIN
  Ctx& c = ctx();
  hipStream_t s = pick(c, stream);
  Timer tm(s);
  merge_forests_dev(c, d_parents, n_trees, n, d_parent_out, s, &tm);
  check_err(c, s);
  tm.finish(c);
  API_END
}

int sheep_sequence_dev(const uint32_t* d_deg, uint32_t n_ids, uint32_t* d_seq, uint32_t* d_rank,
                       uint32_t* n_seq_out, void* stream) {
  API_BEGIN
  Ctx& c = ctx();
  hipStream_t s = pick(c, stream);
  uint32_t n = sequence_dev(c, d_deg, n_ids, d_seq, d_rank, s);
  check_err(c, s);
  if (n_seq_out) *n_seq_out = n;
  API_END
}

int sheep_build_tree_dev(const uint32_t* d_uv, uint64_t m, const uint32_t* d_rank, uint32_t n_rank,
                         uint32_t n_seq, uint32_t* d_parent, uint32_t* d_pst, void* stream) {
  API_BEGIN
  Ctx& c = ctx();
  require_aligned(d_uv, "d_uv");
  hipStream_t s = pick(c, stream);
  Timer tm(s);
  build_tree_dev(c, d_uv, m, d_rank, n_rank, n_seq, d_parent, d_pst, s, &tm);
  check_err(c, s);
  tm.finish(c);
  API_END
}

int sheep_merge_trees_dev(uint32_t* d_parent_a, uint32_t* d_pst_a, const uint32_t* d_parent_b,
                          const uint32_t* d_pst_b, uint32_t n, void* stream) {
  API_BEGIN
  Ctx& c = ctx();
  hipStream_t s = pick(c, stream);
  uint32_t* jump = (uint32_t*)c.scratch.get("merge_jump", (size_t)n * 4);
  launch_merge(d_parent_a, d_pst_a, d_parent_b, d_pst_b, n, jump, s);
  API_END
}

int sheep_graph2tree_dev(const uint32_t* d_uv, uint64_t m, uint32_t n_ids, int degree_mode,
                         uint32_t* d_seq, uint32_t* d_parent, uint32_t* d_pst,
                         uint32_t* n_seq_out, void* stream) {
  API_BEGIN
  Ctx& c = ctx();
  require_aligned(d_uv, "d_uv");
  hipStream_t s = pick(c, stream);
  Timer tm(s);
  uint32_t* deg = (uint32_t*)c.scratch.get("deg", (size_t)n_ids * 4);
  uint32_t* selfc = (uint32_t*)c.scratch.get("selfc", (size_t)n_ids * 4);
  uint32_t* rank = (uint32_t*)c.scratch.get("rank", (size_t)n_ids * 4);
  // The first partition pass of the rank gathers needs no ranks, only the y-digit counts of
  // the degree pass's first kernel: it runs on the side stream beside the rest of the degree
  // pass and the sequence sort (SHEEP_PART_OVERLAP=0: in line, after them; =1: after the
  // whole degree pass).
  int ov = knobs().part_overlap;
  uint32_t* stats = (uint32_t*)c.scratch.get("stats", 16);
  // Fused (ov 3, and always past 2^31 records, where the endpoint offsets of the unfused
  // degree pass end): the degree pass itself writes the records grouped by y bucket
  // (launch_fh_front), so the first partition pass and its read are gone.  Not the default:
  // it moves fewer bytes but in shorter runs, and measured no faster.
  bool fused = false;
  if ((ov == 3 || 2 * m >= (1ull << 32)) && use_part(m) && knobs().degree != 1 &&
      fh_tmp_words(m, n_ids) > 1) {
    require_records(m, "degree");  // its offsets count records, not endpoints
    uint32_t* tmp = (uint32_t*)c.scratch.get("degb_tmp", fh_tmp_words(m, n_ids) * 4);
    uint64_t* mid = (uint64_t*)c.scratch.get("e_items", m * 8);
    uint32_t* pws = (uint32_t*)c.scratch.get("part_ws", PART_WS_WORDS * 4);
    fused = launch_fh_front(d_uv, m, n_ids, degree_mode, deg, selfc, c.d_err, tmp, mid, pws,
                            stats, s, [](void* t, const char* n) { ((Timer*)t)->mark(n); }, &tm);
  }
  // Fused sampled (ov 4): ONE read of the records for the degrees and the first partition pass
  // (launch_front_fused; packed first-pass records in sampled capacity regions).
  const bool ffused = !fused && ov == 4 && use_part(m) && knobs().bin_direct &&
                      part_p6_ok(n_ids) && m >= (1ull << 25) && knobs().degree != 1 &&
                      front_fused_ok(m, n_ids) && degs_tmp_words(m, n_ids) > 1;
  if (ffused) fused = true;
  if (ov == 4 && !ffused) ov = 2;  // (below 2^25 records, or ids it cannot take: beside)
  const bool overlap = !fused && ov != 0 && m > 0 && use_part(m);
  // Sampled capacities (from 2^25 records, the bucketed degree path, the first pass beside
  // it): no counting read of the records — the degree scatter and the first partition pass
  // write into capacity regions sized from a 1/256 sample (launch_degree_sampled).  A region
  // that overflows sends the degrees (here, before the sequence reads them) or the partition
  // (after the edge pass, with the hi bins' overflow) through the exact pass.
  const bool sampled = overlap && knobs().bin_direct && part_p6_ok(n_ids) && ov == 2 &&
                       m >= (1ull << 25) && 2 * m < (1ull << 32) && knobs().degree != 1 &&
                       degs_tmp_words(m, n_ids) > 1;
  // records the mid buffer holds (capacity regions: their largest possible sum)
  const uint64_t mid_slots = ffused    ? front_fused_slots(m, n_ids, ff_groups())
                             : sampled ? (fs_room(m, 1024) + 7) & ~7ull
                                       : m;
  uint32_t* ovf_deg = c.d_err + 2;
  uint32_t* ovf_part = c.d_err + 3;
  if (overlap) HIP_CHECK(hipEventRecord(c.part_ev[0], s));  // in case degree_dev records none
  bool yh = false;
  bool stats_host = false;  // the degree stats already read back (sequence_dev skips its readback)
  if (ffused) {
    HIP_CHECK(hipMemsetAsync(ovf_deg, 0, 8, s));  // both overflow words
    uint32_t* tmp = (uint32_t*)c.scratch.get("degs_tmp", degs_tmp_words(m, n_ids) * 4);
    uint32_t* pws = (uint32_t*)c.scratch.get("part_ws", PART_WS_WORDS * 4);
    uint64_t* mid = (uint64_t*)c.scratch.get("e_items", std::max<uint64_t>(m, mid_slots) * 8);
    launch_front_fused(d_uv, m, n_ids, degree_mode, deg, selfc, c.d_err, tmp, pws, mid, mid_slots,
                       stats, ovf_deg, ovf_part, s,
                       [](void* t, const char* n) { ((Timer*)t)->mark(n); }, &tm, ff_groups());
    tm.mark("degree_hist");
    HIP_CHECK(hipEventRecord(c.part_ev[1], s));
    // One readback: the error word and both overflow words (d_err[0..3]) with the degree stats.
    // The degrees are complete unless a region outgrew its capacity: an x bucket, or a y digit
    // (the histogram counts y's ids from the packed records, which then lost the run's tail);
    // an id out of range leaves the pass's record array short, which is reported here, before
    // anything reads it (the check_err the sequence would otherwise need).
    HIP_CHECK(hipMemcpyAsync(c.h_pinned + 4, c.d_err, 16, hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipMemcpyAsync(c.h_pinned, stats, 12, hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipStreamSynchronize(s));
    if (c.h_pinned[4] & ERR_RANGE) check_err(c, s);  // (throws -ERANGE, resetting the word)
    stats_host = true;
    if (c.h_pinned[6] || c.h_pinned[7]) {
      degree_dev(c, d_uv, m, n_ids, degree_mode, deg, selfc, s, false, nullptr, stats);
      tm.mark("degree_exact");
      stats_host = false;  // (the exact pass rewrote them)
    }
  } else if (sampled) {
    HIP_CHECK(hipMemsetAsync(ovf_deg, 0, 8, s));  // both overflow words
    uint32_t* tmp = (uint32_t*)c.scratch.get("degs_tmp", degs_tmp_words(m, n_ids) * 4);
    uint32_t* pws = (uint32_t*)c.scratch.get("part_ws", PART_WS_WORDS * 4);
    launch_degree_sampled(d_uv, m, n_ids, degree_mode, deg, selfc, c.d_err, tmp, pws, mid_slots,
                          stats, ovf_deg, s, c.part_ev[0]);
  } else if (!fused) {
    yh = degree_dev(c, d_uv, m, n_ids, degree_mode, deg, selfc, s, true,
                    overlap && ov == 2 ? c.part_ev[0] : nullptr, stats);
  }
  if (!ffused) tm.mark(fused ? "degree_hist" : "degree");
  if (fused && !ffused) HIP_CHECK(hipEventRecord(c.part_ev[1], s));
  if (sampled) {
    // (at least m u64: the tree build takes the same buffer at that size and must not regrow it)
    uint64_t* mid = (uint64_t*)c.scratch.get("e_items", std::max<uint64_t>(m, mid_slots) * 8);
    uint32_t* pws = (uint32_t*)c.scratch.get("part_ws", PART_WS_WORDS * 4);
    HIP_CHECK(hipStreamWaitEvent(c.side, c.part_ev[0], 0));
    const size_t sp = tm.span_begin("part_first", c.side);  // k_part<0>, live-timed for bench
    launch_part_first_caps(d_uv, m, n_ids, mid, mid_slots, pws, ovf_part, c.side);
    tm.span_end(sp, c.side);
    HIP_CHECK(hipEventRecord(c.part_ev[1], c.side));
    // the degrees are complete and valid unless a bucket outgrew its region (the stream syncs
    // here once; sequence_dev would wait for the degree pass anyway)
    HIP_CHECK(hipMemcpyAsync(c.h_pinned + 4, ovf_deg, 4, hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipStreamSynchronize(s));
    if (c.h_pinned[4]) {
      degree_dev(c, d_uv, m, n_ids, degree_mode, deg, selfc, s, false, nullptr, stats);
      tm.mark("degree_exact");
    }
  } else if (overlap) {
    uint64_t* mid = (uint64_t*)c.scratch.get("e_items", m * 8);
    uint32_t* pws = (uint32_t*)c.scratch.get("part_ws", PART_WS_WORDS * 4);
    if (ov != 2) HIP_CHECK(hipEventRecord(c.part_ev[0], s));
    HIP_CHECK(hipStreamWaitEvent(c.side, c.part_ev[0], 0));
    const size_t sp = tm.span_begin("part_first", c.side);  // k_part<0>, live-timed for bench
    launch_part_first(d_uv, m, n_ids, mid, pws, c.side, yh);
    tm.span_end(sp, c.side);
    HIP_CHECK(hipEventRecord(c.part_ev[1], c.side));
  }
  uint32_t* nsd = (uint32_t*)c.scratch.get("nsd", (size_t)std::max<uint32_t>(n_ids, 1) * 4);
  uint32_t n_seq = sequence_dev(c, deg, n_ids, d_seq, rank, s, true, nsd, selfc, degree_mode,
                                stats_host);
  // an id out of range leaves the fused pass's record array short: report it before the
  // partition passes read the array (the stream is idle here: sequence_dev synchronised it;
  // the sampled fused pass read its error word above, unless the exact degree pass ran since)
  if (fused && !stats_host) check_err(c, s);
  tm.mark("sequence");
  DegInfo di;
  di.nsd = nsd;
  di.part_first_done = overlap || fused;
  di.mid_slots = mid_slots;
  di.mid_caps = sampled || ffused;
  di.mid_p6 = ffused;
  di.ids_checked = true;
  di.yhist_ready = yh;
  di.seq = d_seq;
  di.deg = deg;
  di.selfc = selfc;
  di.mode = degree_mode;
  build_tree_dev(c, d_uv, m, rank, n_ids, n_seq, d_parent, d_pst, s, &tm, &di);
  if (overlap) HIP_CHECK(hipStreamWaitEvent(s, c.part_ev[1], 0));  // also when no tree was built
  check_err(c, s);
  tm.finish(c);
  if (n_seq_out) *n_seq_out = n_seq;
  API_END
}

static void evaluate_dev(Ctx& c, const uint32_t* d_uv, uint64_t m, const int16_t* d_parts,
                         const uint32_t* d_rank, uint32_t n_ids, uint32_t n_parts, uint64_t* out,
                         hipStream_t s) {
  if (n_parts == 0 || n_parts > 32768) throw ApiError(-EINVAL, "n_parts must be in [1, 32768]");
  uint32_t* deg = (uint32_t*)c.scratch.get("deg", (size_t)std::max<uint32_t>(n_ids, 1) * 4);
  launch_degree(d_uv, m, n_ids, SHEEP_DEGREE_LLAMA, deg, nullptr, c.d_err, s);
  // Each metric sorts one key per adjacency entry (2m of them, less the self-loops' second).
  // Beyond 2^eval_pass entries the ids are cut into ranges whose entries (their LLAMA degrees)
  // fit a pass, and each pass sorts only the entries of its range.
  const int ep = std::min(31, std::max(10, knobs().eval_pass));
  std::vector<std::pair<uint32_t, uint64_t>> passes;
  uint64_t n_keys = 2 * m;
  if (2 * m > (1ull << ep)) {
    check_err(c, s);  // an id out of range would leave the degrees short
    std::vector<uint32_t> hdeg(n_ids);
    if (n_ids) HIP_CHECK(hipMemcpyAsync(hdeg.data(), deg, (size_t)n_ids * 4, hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipStreamSynchronize(s));
    const uint64_t cap = 1ull << ep;
    uint64_t run = 0;
    n_keys = 0;
    passes.emplace_back(0u, 0ull);
    for (uint32_t v = 0; v < n_ids; ++v) {
      if (hdeg[v] > cap) throw ApiError(-EINVAL, "evaluate: one vertex has more adjacency entries than a pass");
      if (run + hdeg[v] > cap) {
        passes.back().second = run;
        n_keys = std::max(n_keys, run);
        passes.emplace_back(v, 0ull);
        run = 0;
      }
      run += hdeg[v];
    }
    passes.back().second = run;
    n_keys = std::max(n_keys, run);
  }
  uint64_t* keys = (uint64_t*)c.scratch.get("e_items", std::max<uint64_t>(n_keys, 1) * 8);
  uint64_t* keys_b = (uint64_t*)c.scratch.get("e_items_b", std::max<uint64_t>(n_keys, 1) * 8);
  uint32_t* rtmp = (uint32_t*)c.scratch.get("rsort_tmp", rsort_tmp_words(std::max<uint64_t>(n_keys, 1)) * 4);
  const size_t wsn = 4 * (size_t)n_parts + 8;
  unsigned long long* ws = (unsigned long long*)c.scratch.get("eval_ws", wsn * 8);
  launch_evaluate(d_uv, m, d_parts, d_rank, deg, n_ids, n_parts, keys, keys_b, rtmp, ws, c.d_err, s,
                  &passes);
  std::vector<unsigned long long> h(wsn);
  HIP_CHECK(hipMemcpyAsync(h.data(), ws, wsn * 8, hipMemcpyDeviceToHost, s));
  check_err(c, s);  // synchronises; -ERANGE for an id, part or position out of range
  const unsigned long long* cnt = h.data() + 4 * (size_t)n_parts;
  auto mx = [&](size_t off) {
    unsigned long long v = 0;
    for (uint32_t i = 0; i < n_parts; ++i) v = std::max(v, h[off + i]);
    return (uint64_t)v;
  };
  const uint64_t nodes = cnt[2];
  out[0] = cnt[0];
  out[1] = cnt[3];
  out[2] = mx(3 * (size_t)n_parts);
  out[3] = cnt[4] - nodes;
  out[4] = mx(0);
  out[5] = cnt[5] - nodes;
  out[6] = mx(n_parts);
  out[7] = cnt[6] - nodes;
  out[8] = mx(2 * (size_t)n_parts);
  out[9] = (2 * m - cnt[1]) / 2;
  out[10] = nodes;
}

int sheep_evaluate_dev(const uint32_t* d_uv, uint64_t m, const int16_t* d_parts,
                       const uint32_t* d_rank, uint32_t n_ids, uint32_t n_parts, uint64_t* out,
                       void* stream) {
  API_BEGIN
  Ctx& c = ctx();
  require_aligned(d_uv, "d_uv");
  evaluate_dev(c, d_uv, m, d_parts, d_rank, n_ids, n_parts, out, pick(c, stream));
  API_END
}

static void partition_edges_dev(Ctx& c, const uint32_t* d_uv, uint64_t m, const int16_t* d_parts,
                                const uint32_t* d_rank, uint32_t n_ids, uint32_t n_parts,
                                uint32_t* d_out, uint64_t* part_start, hipStream_t s) {
  require_records(m, "partition edges");
  if (n_parts == 0 || n_parts > 32768) throw ApiError(-EINVAL, "n_parts must be in [1, 32768]");
  const uint64_t mm = std::max<uint64_t>(m, 1);
  uint64_t* items = (uint64_t*)c.scratch.get("e_items", mm * 8);
  uint64_t* items_b = (uint64_t*)c.scratch.get("e_items_b", mm * 8);
  uint32_t* rtmp = (uint32_t*)c.scratch.get("rsort_tmp", rsort_tmp_words(mm) * 4);
  unsigned long long* dstart = (unsigned long long*)c.scratch.get("pe_start", ((size_t)n_parts + 1) * 8);
  launch_partition_edges(d_uv, m, d_parts, d_rank, n_ids, n_parts, items, items_b, rtmp, d_out,
                         dstart, c.d_err, s);
  HIP_CHECK(hipMemcpyAsync(part_start, dstart, ((size_t)n_parts + 1) * 8, hipMemcpyDeviceToHost, s));
  check_err(c, s);  // synchronises; -ERANGE for an id outside the sequence or a vertex without part
}

// ---- records resident in HBM ---------------------------------------------------------------

int sheep_records_register(const uint32_t* uv, uint64_t m) {
  API_BEGIN
  Ctx& c = ctx();
  if (!uv) throw ApiError(-EINVAL, "null records");
  for (const Ctx::Registered& r : c.registered)
    if (r.host == uv) throw ApiError(-EBUSY, "records already registered");
  uint32_t* dev = nullptr;
  HIP_CHECK(hipMalloc(&dev, std::max<uint64_t>(8 * m, 8)));
  if (m) HIP_CHECK(hipMemcpy(dev, uv, 8 * m, hipMemcpyHostToDevice));
  c.registered.push_back({uv, m, dev});
  API_END
}

int sheep_records_release(const uint32_t* uv) {
  API_BEGIN
  Ctx& c = ctx();
  for (size_t i = 0; i < c.registered.size(); ++i)
    if (c.registered[i].host == uv) {
      HIP_CHECK(hipStreamSynchronize(c.stream));
      (void)hipFree(c.registered[i].dev);
      c.registered.erase(c.registered.begin() + i);
      return SHEEP_OK;
    }
  throw ApiError(-ENOENT, "records not registered");
  API_END
}

// XS1 records of a .dat file: every complete record (LLAMA's load), or the contiguous range of
// part/num_parts (1-based, graph2tree -l, graph_wrapper.h:48-49).  Returns the open file.
static FILE* open_dat(const char* path, uint64_t part, uint64_t num_parts, uint64_t* lo,
                      uint64_t* hi) {
  if (!path) throw ApiError(-EINVAL, "null path");
  FILE* f = fopen(path, "rb");
  if (!f) throw ApiError(-ENOENT, std::string("cannot open ") + path);
  if (fseeko(f, 0, SEEK_END) != 0) { fclose(f); throw ApiError(-EIO, "seek"); }
  const uint64_t R = (uint64_t)ftello(f) / 12;
  *lo = 0;
  *hi = R;
  if (num_parts) {
    if (part < 1 || part > num_parts) { fclose(f); throw ApiError(-EINVAL, "part must be in [1, num_parts]"); }
    *lo = R * (part - 1) / num_parts;
    *hi = R * part / num_parts;
  }
  return f;
}

// Streams records [lo, lo + m) to dev (2m u32) through two pinned staging buffers: the file read
// of chunk i+1 overlaps the upload and the weight-stripping kernel of chunk i; host (nullable)
// receives the pairs too.  Returns max id + 1.  Synchronises s.
static uint32_t ingest_dat(Ctx& c, FILE* f, uint64_t lo, uint64_t m, uint32_t* dev, uint32_t* host,
                           hipStream_t s) {
  constexpr uint64_t CH = 1ull << 22;  // records per chunk (48 MB)
  uint32_t* pin[2] = {nullptr, nullptr};
  uint32_t* raw[2] = {nullptr, nullptr};
  hipEvent_t done[2] = {nullptr, nullptr};
  auto cleanup = [&] {
    (void)hipStreamSynchronize(s);
    for (int i = 0; i < 2; ++i) {
      if (pin[i]) (void)hipHostFree(pin[i]);
      if (raw[i]) (void)hipFree(raw[i]);
      if (done[i]) (void)hipEventDestroy(done[i]);
    }
  };
  uint32_t mx = 0;
  try {
    for (int i = 0; i < 2; ++i) {
      HIP_CHECK(hipHostMalloc((void**)&pin[i], CH * 12, hipHostMallocDefault));
      HIP_CHECK(hipMalloc(&raw[i], CH * 12));
      HIP_CHECK(hipEventCreateWithFlags(&done[i], hipEventDisableTiming));
    }
    uint32_t* dmax = (uint32_t*)c.scratch.get("ingest_max", 4);
    HIP_CHECK(hipMemsetAsync(dmax, 0, 4, s));
    if (fseeko(f, (off_t)(lo * 12), SEEK_SET) != 0) throw ApiError(-EIO, "seek");
    for (uint64_t b = 0, k = 0; b < m; b += CH, ++k) {
      const int i = (int)(k & 1);
      const uint64_t n = std::min(CH, m - b);
      if (k >= 2) HIP_CHECK(hipEventSynchronize(done[i]));  // chunk k-2's upload is done
      if (fread(pin[i], 12, n, f) != n) throw ApiError(-EIO, "short read");
      HIP_CHECK(hipMemcpyAsync(raw[i], pin[i], n * 12, hipMemcpyHostToDevice, s));
      launch_strip_xs1(raw[i], n, dev + 2 * b, dmax, s);
      HIP_CHECK(hipEventRecord(done[i], s));
      if (host)
        for (uint64_t j = 0; j < n; ++j) {
          host[2 * (b + j)] = pin[i][3 * j];
          host[2 * (b + j) + 1] = pin[i][3 * j + 1];
        }
    }
    HIP_CHECK(hipMemcpyAsync(c.h_pinned, dmax, 4, hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipStreamSynchronize(s));
    mx = c.h_pinned[0];
    if (mx == INV)  // max id + 1 does not fit u32: a record names INVALID (or 0xFFFFFFFE)
      throw ApiError(-ERANGE, "a record's vertex id is 0xFFFFFFFE or 0xFFFFFFFF (u32 id space)");
  } catch (...) {
    cleanup();
    throw;
  }
  cleanup();
  return mx;
}

int sheep_records_load_dat(const char* path, uint64_t part, uint64_t num_parts, uint32_t* uv_out,
                           uint64_t cap, uint64_t* m_out, uint32_t* max_id_out) {
  API_BEGIN
  Ctx& c = ctx();
  uint64_t lo, hi;
  std::unique_ptr<FILE, int (*)(FILE*)> f(open_dat(path, part, num_parts, &lo, &hi), fclose);
  const uint64_t m = hi - lo;
  if (m_out) *m_out = m;
  if (!uv_out) return SHEEP_OK;  // size query
  if (cap < m) throw ApiError(-ERANGE, "uv_out holds fewer records than the range");
  for (const Ctx::Registered& r : c.registered)
    if (r.host == uv_out) throw ApiError(-EBUSY, "records already registered");
  uint32_t* dev = nullptr;
  HIP_CHECK(hipMalloc(&dev, std::max<uint64_t>(8 * m, 8)));
  try {
    const uint32_t mx = ingest_dat(c, f.get(), lo, m, dev, uv_out, c.stream);
    if (max_id_out) *max_id_out = mx;
  } catch (...) {
    (void)hipFree(dev);
    throw;
  }
  c.registered.push_back({uv_out, m, dev});
  API_END
}

int sheep_read_dat_dev(const char* path, uint64_t part, uint64_t num_parts, uint32_t* d_uv,
                       uint64_t cap, uint64_t* m_out, uint32_t* max_id_out, void* stream) {
  API_BEGIN
  Ctx& c = ctx();
  uint64_t lo, hi;
  std::unique_ptr<FILE, int (*)(FILE*)> f(open_dat(path, part, num_parts, &lo, &hi), fclose);
  const uint64_t m = hi - lo;
  if (m_out) *m_out = m;
  if (!d_uv) return SHEEP_OK;  // size query
  if (cap < m) throw ApiError(-ERANGE, "d_uv holds fewer records than the range");
  const uint32_t mx = ingest_dat(c, f.get(), lo, m, d_uv, nullptr, pick(c, stream));
  if (max_id_out) *max_id_out = mx;
  API_END
}

int sheep_partition_edges_dev(const uint32_t* d_uv, uint64_t m, const int16_t* d_parts,
                              const uint32_t* d_rank, uint32_t n_ids, uint32_t n_parts,
                              uint32_t* d_out, uint64_t* part_start, void* stream) {
  API_BEGIN
  Ctx& c = ctx();
  require_aligned(d_uv, "d_uv");
  partition_edges_dev(c, d_uv, m, d_parts, d_rank, n_ids, n_parts, d_out, part_start, pick(c, stream));
  API_END
}

int sheep_partition_edges(const uint32_t* edges_uv, uint64_t m, const int16_t* parts,
                          uint32_t n_parts_vid, const uint32_t* seq, uint32_t n_seq, uint32_t n_parts,
                          uint32_t* out_uv, uint64_t* part_start) {
  API_BEGIN
  Ctx& c = ctx();
  hipStream_t s = c.stream;
  uint64_t top = n_parts_vid;  // 64-bit: an id 0xFFFFFFFF would wrap max id + 1 to 0
  for (uint64_t i = 0; i < 2 * m; ++i) top = std::max<uint64_t>(top, (uint64_t)edges_uv[i] + 1);
  for (uint32_t i = 0; i < n_seq; ++i) top = std::max<uint64_t>(top, (uint64_t)seq[i] + 1);
  if (top > 0xFFFFFFFEull) throw ApiError(-ERANGE, "partition_edges: vertex id 0xFFFFFFFF (INVALID)");
  const uint32_t n_ids = (uint32_t)top;
  uint32_t* uv = upload_records(c, edges_uv, m, s);
  int16_t* dparts = (int16_t*)c.scratch.get("h_parts", (size_t)std::max<uint32_t>(n_ids, 1) * 2);
  HIP_CHECK(hipMemsetAsync(dparts, 0xFF, (size_t)n_ids * 2, s));
  if (n_parts_vid)
    HIP_CHECK(hipMemcpyAsync(dparts, parts, (size_t)n_parts_vid * 2, hipMemcpyHostToDevice, s));
  uint32_t* dseq = (uint32_t*)c.scratch.get("h_seq", (size_t)std::max<uint32_t>(n_seq, 1) * 4);
  if (n_seq) HIP_CHECK(hipMemcpyAsync(dseq, seq, (size_t)n_seq * 4, hipMemcpyHostToDevice, s));
  uint32_t* rank = (uint32_t*)c.scratch.get("rank", (size_t)std::max<uint32_t>(n_ids, 1) * 4);
  launch_fill(rank, INV, n_ids, s);
  launch_rank_scatter(dseq, n_seq, rank, c.d_err, s);
  uint32_t* out = (uint32_t*)c.scratch.get("pe_out", std::max<uint64_t>(8 * m, 8));
  partition_edges_dev(c, uv, m, dparts, rank, n_ids, n_parts, out, part_start, s);
  const uint64_t kept = part_start[n_parts];
  if (kept) HIP_CHECK(hipMemcpyAsync(out_uv, out, 8 * kept, hipMemcpyDeviceToHost, s));
  HIP_CHECK(hipStreamSynchronize(s));
  API_END
}

int sheep_rmat_dev(uint32_t* d_uv, int scale, uint64_t seed, uint64_t e_begin, uint64_t e_end,
                   void* stream) {
  API_BEGIN
  Ctx& c = ctx();
  require_aligned(d_uv, "d_uv");
  if (scale < 1 || scale > 32) throw ApiError(-EINVAL, "scale must be in [1, 32]");
  launch_rmat(d_uv, scale, seed, e_begin, e_end, pick(c, stream));
  API_END
}

int sheep_powerlaw_dev(uint32_t* d_uv, uint32_t n, double gamma, double i0, uint64_t seed,
                       uint64_t e_begin, uint64_t e_end, void* stream) {
  API_BEGIN
  Ctx& c = ctx();
  require_aligned(d_uv, "d_uv");
  if (n == 0 || !(gamma > 1.0) || !(i0 >= 0.0)) throw ApiError(-EINVAL, "powerlaw: n > 0, gamma > 1, i0 >= 0");
  launch_powerlaw(d_uv, n, gamma, i0, seed, e_begin, e_end, pick(c, stream));
  API_END
}

// ---- lockstep multi-GPU tree build ---------------------------------------------------------

int sheep_ls_begin(const uint32_t* d_uv, uint64_t m, const uint32_t* d_rank, uint32_t n_rank,
                   const uint32_t* d_seq, uint32_t n_seq, const uint32_t* d_deg,
                   uint64_t* bin_counts_out, uint32_t* n_bins_out, void** handle_out,
                   void* stream) {
  API_BEGIN
  Ctx& c = ctx();
  require_aligned(d_uv, "d_uv");
  if (!bin_counts_out || !n_bins_out || !handle_out) throw ApiError(-EINVAL, "null output");
  *handle_out = nullptr;
  hipStream_t s = pick(c, stream);
  Lockstep* L = new Lockstep();
  L->ctx = &c;
  L->scp = c.ls_live++ == 0 ? &c.scratch : &L->own;
  try {
    ls_begin(*L, d_uv, m, d_rank, n_rank, d_seq, n_seq, d_deg, bin_counts_out, n_bins_out,
             c.d_err, s);
    check_err(c, s);
  } catch (...) {
    delete L;
    throw;
  }
  *handle_out = L;
  API_END
}

int sheep_ls_plan(void* handle, const uint64_t* global_bin_counts, uint32_t* n_buckets_out,
                  uint32_t* mark_slots_out) {
  API_BEGIN
  if (!handle || !global_bin_counts) throw ApiError(-EINVAL, "null argument");
  ls_plan(*(Lockstep*)handle, global_bin_counts, n_buckets_out, mark_slots_out);
  API_END
}

int sheep_ls_split(void* handle, uint32_t rank, uint32_t n_ranks) {
  API_BEGIN
  if (!handle) throw ApiError(-EINVAL, "null handle");
  Lockstep& L = *(Lockstep*)handle;
  if (L.split || !L.map_ev.empty()) throw ApiError(-EINVAL, "lockstep split: set once, before the first map");
  if (L.n_seq) ls_set_split(L, rank, n_ranks, 0);
  API_END
}

int sheep_ls_map(void* handle, uint32_t k, uint64_t* d_send, int64_t* d_count,
                 uint32_t* n_kept_out, void* stream) {
  API_BEGIN
  Ctx& c = ctx();
  if (!handle) throw ApiError(-EINVAL, "null handle");
  ls_map(*(Lockstep*)handle, k, d_send, (long long*)d_count, n_kept_out, pick(c, stream));
  API_END
}

int sheep_ls_pack(void* handle, uint32_t k, uint64_t* d_send, uint32_t cap, void* stream) {
  API_BEGIN
  Ctx& c = ctx();
  if (!handle) throw ApiError(-EINVAL, "null handle");
  ls_pack(*(Lockstep*)handle, k, d_send, cap, pick(c, stream));
  API_END
}

int sheep_ls_apply(void* handle, uint32_t k, const uint64_t* d_recv, uint32_t n_ranks,
                   uint32_t cap, void* stream) {
  API_BEGIN
  Ctx& c = ctx();
  if (!handle || n_ranks == 0) throw ApiError(-EINVAL, "null handle or no ranks");
  ls_apply(*(Lockstep*)handle, k, d_recv, n_ranks, cap, pick(c, stream));
  API_END
}

int sheep_ls_finish(void* handle, const uint32_t* d_seq, const uint32_t* d_deg,
                    const uint32_t* d_selfc, int degree_mode, uint32_t* d_parent, uint32_t* d_pst,
                    void* stream) {
  API_BEGIN
  Ctx& c = ctx();
  if (!handle) throw ApiError(-EINVAL, "null handle");
  if (degree_mode != SHEEP_DEGREE_LLAMA && degree_mode != SHEEP_DEGREE_FILE)
    throw ApiError(-EINVAL, "degree_mode");
  hipStream_t s = pick(c, stream);
  ls_finish(c, *(Lockstep*)handle, d_seq, d_deg, d_selfc, degree_mode, d_parent, d_pst, s);
  check_err(c, s);
  API_END
}

int sheep_ls_free(void* handle) {
  API_BEGIN
  delete (Lockstep*)handle;
  API_END
}

// ---- multi-GPU: communicator + graph2tree -i -r ---------------------------------------------

int sheep_comm_unique_id(uint8_t* id_out) {
  API_BEGIN
  if (!id_out) throw ApiError(-EINVAL, "null id");
  rccl_unique_id(id_out);
  API_END
}

int sheep_comm_init(const uint8_t* id, int n_ranks, int rank) {
  API_BEGIN
  if (!id || n_ranks < 1 || rank < 0 || rank >= n_ranks) throw ApiError(-EINVAL, "comm: id, n_ranks, rank");
  Ctx& c = ctx();
  if (c.comm) throw ApiError(-EBUSY, "comm: this device already has a communicator");
  c.comm = rccl_comm(id, n_ranks, rank).release();
  API_END
}

int sheep_comm_init_host(const char* name, int n_ranks, int rank) {
  API_BEGIN
  if (!name || name[0] != '/' || n_ranks < 1 || rank < 0 || rank >= n_ranks)
    throw ApiError(-EINVAL, "comm: name (\"/...\"), n_ranks, rank");
  Ctx& c = ctx();
  if (c.comm) throw ApiError(-EBUSY, "comm: this device already has a communicator");
  c.comm = shm_comm(name, n_ranks, rank, 16ull << 20).release();
  API_END
}

int sheep_comm_free(void) {
  API_BEGIN
  Ctx& c = ctx();
  delete c.comm;
  c.comm = nullptr;
  API_END
}

int sheep_comm_info(int* rank, int* n_ranks) {
  API_BEGIN
  Ctx& c = ctx();
  if (!c.comm) throw ApiError(-ENOENT, "comm: no communicator (sheep_comm_init)");
  if (rank) *rank = c.comm->rank();
  if (n_ranks) *n_ranks = c.comm->size();
  API_END
}

static Comm& need_comm(Ctx& c) {
  if (!c.comm) throw ApiError(-ENOENT, "no communicator: call sheep_comm_init on every rank first");
  return *c.comm;
}

// Timings of a multi-rank build: the phase marks, then the lockstep loop's kernel sums.
static void multi_timings(Ctx& c, Timer& tm) {
  std::vector<std::pair<const char*, double>> kb = c.timings;  // ls_finish's (static names)
  tm.finish(c);
  for (auto& x : kb) c.timings.push_back(x);
}

int sheep_graph2tree_multi_dev(const uint32_t* d_uv, uint64_t m, uint32_t n_ids, int degree_mode,
                               uint32_t* d_seq, uint32_t* d_parent, uint32_t* d_pst,
                               uint32_t* n_seq_out, void* stream) {
  API_BEGIN
  Ctx& c = ctx();
  require_aligned(d_uv, "d_uv");
  if (degree_mode != SHEEP_DEGREE_LLAMA && degree_mode != SHEEP_DEGREE_FILE)
    throw ApiError(-EINVAL, "degree_mode");
  hipStream_t s = pick(c, stream);
  Timer tm(s);
  uint32_t n = multi_tree(c, need_comm(c), d_uv, m, n_ids, degree_mode, d_seq, false, 0, d_parent,
                          d_pst, s, &tm);
  multi_timings(c, tm);
  if (n_seq_out) *n_seq_out = n;
  API_END
}

int sheep_mpi_sequence(const uint32_t* edges_uv, uint64_t m, uint32_t n_ids, int degree_mode,
                       uint32_t* seq_out, uint32_t seq_cap, uint32_t* n_seq_out) {
  API_BEGIN
  Ctx& c = ctx();
  Comm& comm = need_comm(c);
  hipStream_t s = c.stream;
  if (degree_mode != SHEEP_DEGREE_LLAMA && degree_mode != SHEEP_DEGREE_FILE)
    throw ApiError(-EINVAL, "degree_mode");
  // MPI_Allreduce MAX of the id spaces (sequence.h:72), then SUM of the degrees (:78).  The
  // smallest seq_cap of all ranks travels with it (as -cap under MAX), so that a sequence longer
  // than some rank's buffer fails on EVERY rank after the same collectives (n_seq is the same
  // everywhere): no rank leaves the others waiting in a later collective.
  uint64_t top = n_ids;  // 64-bit: an id 0xFFFFFFFF would wrap max id + 1 to 0
  for (uint64_t i = 0; i < 2 * m; ++i) top = std::max<uint64_t>(top, (uint64_t)edges_uv[i] + 1);
  int64_t* d_n = (int64_t*)c.scratch.get("mt_cnt", 16);
  int64_t hn[2] = {(int64_t)top, -(int64_t)seq_cap};
  HIP_CHECK(hipMemcpyAsync(d_n, hn, 16, hipMemcpyHostToDevice, s));
  comm.allreduce_max_i64(d_n, 2, s);
  HIP_CHECK(hipMemcpyAsync(hn, d_n, 16, hipMemcpyDeviceToHost, s));
  HIP_CHECK(hipStreamSynchronize(s));
  if (hn[0] > (int64_t)0xFFFFFFFEll)  // as the other entry points: n_ids must stay below INVALID
    throw ApiError(-ERANGE, "mpi_sequence: vertex id >= 0xFFFFFFFE in the records");
  n_ids = (uint32_t)hn[0];
  const uint64_t min_cap = (uint64_t)(-hn[1]);
  uint32_t* uv = upload_records(c, edges_uv, m, s);
  const size_t n = std::max<uint32_t>(n_ids, 1);
  uint32_t* deg = (uint32_t*)c.scratch.get("deg", n * 4);
  uint32_t* rank = (uint32_t*)c.scratch.get("rank", n * 4);
  uint32_t* seq = (uint32_t*)c.scratch.get("h_seq", n * 4);
  degree_dev(c, uv, m, n_ids, degree_mode, deg, nullptr, s);
  check_err(c, s);
  comm.allreduce_sum_u32(deg, n_ids, s);
  uint32_t n_seq = sequence_dev(c, deg, n_ids, seq, rank, s);
  if (n_seq_out) *n_seq_out = n_seq;
  if (n_seq > min_cap)  // on every rank at once (see above); the caller grows seq_out and retries
    throw ApiError(-ERANGE, "mpi_sequence: a rank's seq_out holds fewer ids than the sequence");
  if (n_seq) HIP_CHECK(hipMemcpyAsync(seq_out, seq, (size_t)n_seq * 4, hipMemcpyDeviceToHost, s));
  check_err(c, s);
  API_END
}

int sheep_build_tree_multi(const uint32_t* edges_uv, uint64_t m, const uint32_t* seq, uint32_t n_seq,
                           uint32_t* parent_out, uint32_t* pst_out) {
  API_BEGIN
  Ctx& c = ctx();
  Comm& comm = need_comm(c);
  hipStream_t s = c.stream;
  if (n_seq == 0) return SHEEP_OK;
  // the index size of JTree (jtree.h:113): max(seq) + 1, the same on every rank
  const uint32_t n_rank = *std::max_element(seq, seq + n_seq) + 1;
  uint32_t* uv = upload_records(c, edges_uv, m, s);
  uint32_t* dseq = (uint32_t*)c.scratch.get("h_seq", (size_t)n_seq * 4);
  HIP_CHECK(hipMemcpyAsync(dseq, seq, (size_t)n_seq * 4, hipMemcpyHostToDevice, s));
  uint32_t* parent = (uint32_t*)c.scratch.get("h_parent", (size_t)n_seq * 4);
  uint32_t* pst = (uint32_t*)c.scratch.get("h_pst", (size_t)n_seq * 4);
  Timer tm(s);
  multi_tree(c, comm, uv, m, n_rank, SHEEP_DEGREE_LLAMA, dseq, true, n_seq, parent, pst, s, &tm);
  multi_timings(c, tm);
  HIP_CHECK(hipMemcpyAsync(parent_out, parent, (size_t)n_seq * 4, hipMemcpyDeviceToHost, s));
  HIP_CHECK(hipMemcpyAsync(pst_out, pst, (size_t)n_seq * 4, hipMemcpyDeviceToHost, s));
  HIP_CHECK(hipStreamSynchronize(s));
  API_END
}

int sheep_mpi_merge(uint32_t* parent, uint32_t* pst, uint32_t n) {
  API_BEGIN
  Ctx& c = ctx();
  Comm& comm = need_comm(c);
  hipStream_t s = c.stream;
  if (n == 0) return SHEEP_OK;
  const int P = comm.size();
  // MPI_Reduce with the merge op (jnode.cpp:213-250): every rank's forest is gathered (as u64
  // words, two parents each) and their union's elimination tree is built once; pst is summed.
  const size_t words = ((size_t)n + 1) / 2;
  uint64_t* mine = (uint64_t*)c.scratch.get("mm_mine", words * 8);
  uint64_t* all = (uint64_t*)c.scratch.get("mm_all", (size_t)P * words * 8);
  uint32_t* dpst = (uint32_t*)c.scratch.get("mm_pst", (size_t)n * 4);
  uint32_t* out = (uint32_t*)c.scratch.get("mm_out", (size_t)n * 4);
  HIP_CHECK(hipMemsetAsync(mine, 0xFF, words * 8, s));
  HIP_CHECK(hipMemcpyAsync(mine, parent, (size_t)n * 4, hipMemcpyHostToDevice, s));
  HIP_CHECK(hipMemcpyAsync(dpst, pst, (size_t)n * 4, hipMemcpyHostToDevice, s));
  comm.allgather_u64(mine, all, words, s);
  comm.allreduce_sum_u32(dpst, n, s);
  uint32_t* stack = (uint32_t*)c.scratch.get("mm_stack", (size_t)P * n * 4);
  for (int r = 0; r < P; ++r)
    HIP_CHECK(hipMemcpyAsync(stack + (size_t)r * n, (const uint32_t*)(all + (size_t)r * words),
                             (size_t)n * 4, hipMemcpyDeviceToDevice, s));
  Timer tm(s);
  merge_forests_dev(c, stack, (uint32_t)P, n, out, s, &tm);
  check_err(c, s);
  tm.finish(c);
  HIP_CHECK(hipMemcpyAsync(parent, out, (size_t)n * 4, hipMemcpyDeviceToHost, s));
  HIP_CHECK(hipMemcpyAsync(pst, dpst, (size_t)n * 4, hipMemcpyDeviceToHost, s));
  HIP_CHECK(hipStreamSynchronize(s));
  API_END
}

int sheep_graph2tree_multi_local(const uint32_t* const* d_uv, const uint64_t* m, uint32_t n_ranks,
                                 uint32_t n_ids, int degree_mode, uint32_t* d_seq,
                                 uint32_t* d_parent, uint32_t* d_pst, uint32_t* n_seq_out) {
  API_BEGIN
  if (!d_uv || !m || n_ranks == 0 || n_ranks > 64) throw ApiError(-EINVAL, "multi_local: 1..64 shards");
  if (degree_mode != SHEEP_DEGREE_LLAMA && degree_mode != SHEEP_DEGREE_FILE)
    throw ApiError(-EINVAL, "degree_mode");
  Ctx& c0 = ctx();
  const int dev = c0.device;
  HIP_CHECK(hipDeviceSynchronize());
  auto group = make_local_group((int)n_ranks);
  const size_t n = std::max<uint32_t>(n_ids, 1);
  std::vector<uint32_t*> outs(3 * n_ranks, nullptr);  // ranks > 0: their own seq/parent/pst
  std::vector<uint32_t> nseq(n_ranks, 0);
  std::vector<std::string> errs(n_ranks);
  std::vector<int> codes(n_ranks, 0);
  outs[0] = d_seq;
  outs[1] = d_parent;
  outs[2] = d_pst;
  for (uint32_t r = 1; r < n_ranks; ++r)
    for (int j = 0; j < 3; ++j) HIP_CHECK(hipMalloc(&outs[3 * r + j], n * 4));
  std::vector<std::thread> th;
  for (uint32_t r = 0; r < n_ranks; ++r)
    th.emplace_back([&, r] {
      Ctx c;
      try {
        HIP_CHECK(hipSetDevice(dev));
        ctx_setup(c, dev);
        std::unique_ptr<Comm> comm = local_comm(group, (int)r);
        nseq[r] = multi_tree(c, *comm, d_uv[r], m[r], n_ids, degree_mode, outs[3 * r], false, 0,
                             outs[3 * r + 1], outs[3 * r + 2], c.stream, nullptr);
      } catch (const ApiError& e) {
        errs[r] = e.what();
        codes[r] = e.code;
        group_abort(*group);
      } catch (const std::exception& e) {
        errs[r] = e.what();
        codes[r] = -EIO;
        group_abort(*group);
      }
      if (c.device >= 0) ctx_teardown(c);
    });
  for (auto& t : th) t.join();
  int code = 0;
  std::string msg;
  for (uint32_t r = 0; r < n_ranks && !code; ++r)
    if (codes[r] && errs[r] != "rank group aborted") { code = codes[r]; msg = errs[r]; }
  for (uint32_t r = 0; r < n_ranks && !code; ++r)
    if (codes[r]) { code = codes[r]; msg = errs[r]; }
  // every replica must be the same tree (the etree is unique)
  if (!code)
    for (uint32_t r = 1; r < n_ranks && !code; ++r) {
      if (nseq[r] != nseq[0]) { code = -EIO; msg = "multi_local: ranks disagree on n_seq"; break; }
      for (int j = 0; j < 3 && !code; ++j) {
        std::vector<uint32_t> a(nseq[0]), b(nseq[0]);
        HIP_CHECK(hipMemcpy(a.data(), outs[j], (size_t)nseq[0] * 4, hipMemcpyDeviceToHost));
        HIP_CHECK(hipMemcpy(b.data(), outs[3 * r + j], (size_t)nseq[0] * 4, hipMemcpyDeviceToHost));
        if (a != b) { code = -EIO; msg = "multi_local: rank replicas diverged"; }
      }
    }
  for (uint32_t r = 1; r < n_ranks; ++r)
    for (int j = 0; j < 3; ++j) (void)hipFree(outs[3 * r + j]);
  if (code) throw ApiError(code, msg);
  if (n_seq_out) *n_seq_out = nseq[0];
  API_END
}

// ---- host-pointer API ----------------------------------------------------------------------

int sheep_degree_seq(const uint32_t* edges_uv, uint64_t m, uint32_t n_ids, int degree_mode,
                     uint32_t* seq_out, uint32_t* n_seq_out, uint32_t* rank_out) {
  API_BEGIN
  Ctx& c = ctx();
  hipStream_t s = c.stream;
  if (degree_mode != SHEEP_DEGREE_LLAMA && degree_mode != SHEEP_DEGREE_FILE)
    throw ApiError(-EINVAL, "degree_mode");
  if (n_ids == 0) {
    uint64_t top = 0;  // 64-bit: an id 0xFFFFFFFF would wrap max id + 1 to 0
    for (uint64_t i = 0; i < 2 * m; ++i) top = std::max<uint64_t>(top, (uint64_t)edges_uv[i] + 1);
    if (top > 0xFFFFFFFEull) throw ApiError(-ERANGE, "degree_seq: vertex id 0xFFFFFFFF (INVALID)");
    n_ids = (uint32_t)top;
  }
  uint32_t* uv = upload_records(c, edges_uv, m, s);
  uint32_t* deg = (uint32_t*)c.scratch.get("deg", (size_t)n_ids * 4);
  uint32_t* rank = (uint32_t*)c.scratch.get("rank", (size_t)n_ids * 4);
  uint32_t* seq = (uint32_t*)c.scratch.get("h_seq", (size_t)n_ids * 4);
  degree_dev(c, uv, m, n_ids, degree_mode, deg, nullptr, s);
  check_err(c, s);
  uint32_t n_seq = sequence_dev(c, deg, n_ids, seq, rank, s);
  if (n_seq) HIP_CHECK(hipMemcpyAsync(seq_out, seq, (size_t)n_seq * 4, hipMemcpyDeviceToHost, s));
  if (rank_out && n_ids)
    HIP_CHECK(hipMemcpyAsync(rank_out, rank, (size_t)n_ids * 4, hipMemcpyDeviceToHost, s));
  check_err(c, s);
  if (n_seq_out) *n_seq_out = n_seq;
  API_END
}

int sheep_evaluate(const uint32_t* edges_uv, uint64_t m, const int16_t* parts, uint32_t n_parts_vid,
                   const uint32_t* seq, uint32_t n_seq, uint32_t n_parts, uint64_t* out) {
  API_BEGIN
  Ctx& c = ctx();
  hipStream_t s = c.stream;
  uint64_t top = n_parts_vid;  // 64-bit: an id 0xFFFFFFFF would wrap max id + 1 to 0
  for (uint64_t i = 0; i < 2 * m; ++i) top = std::max<uint64_t>(top, (uint64_t)edges_uv[i] + 1);
  for (uint32_t i = 0; i < n_seq; ++i) top = std::max<uint64_t>(top, (uint64_t)seq[i] + 1);
  if (top > 0xFFFFFFFEull) throw ApiError(-ERANGE, "evaluate: vertex id 0xFFFFFFFF (INVALID)");
  const uint32_t n_ids = (uint32_t)top;
  uint32_t* uv = upload_records(c, edges_uv, m, s);
  int16_t* dparts = (int16_t*)c.scratch.get("h_parts", (size_t)std::max<uint32_t>(n_ids, 1) * 2);
  HIP_CHECK(hipMemsetAsync(dparts, 0xFF, (size_t)n_ids * 2, s));  // INVALID_PART = -1
  if (n_parts_vid)
    HIP_CHECK(hipMemcpyAsync(dparts, parts, (size_t)n_parts_vid * 2, hipMemcpyHostToDevice, s));
  uint32_t* dseq = (uint32_t*)c.scratch.get("h_seq", (size_t)std::max<uint32_t>(n_seq, 1) * 4);
  if (n_seq) HIP_CHECK(hipMemcpyAsync(dseq, seq, (size_t)n_seq * 4, hipMemcpyHostToDevice, s));
  uint32_t* rank = (uint32_t*)c.scratch.get("rank", (size_t)std::max<uint32_t>(n_ids, 1) * 4);
  launch_fill(rank, INV, n_ids, s);
  launch_rank_scatter(dseq, n_seq, rank, c.d_err, s);
  check_err(c, s);
  evaluate_dev(c, uv, m, dparts, rank, n_ids, n_parts, out, s);
  API_END
}

int sheep_build_tree(const uint32_t* edges_uv, uint64_t m, const uint32_t* seq, uint32_t n_seq,
                     uint32_t* parent_out, uint32_t* pst_out) {
  API_BEGIN
  Ctx& c = ctx();
  hipStream_t s = c.stream;
  if (n_seq == 0) return SHEEP_OK;
  uint32_t n_rank = *std::max_element(seq, seq + n_seq) + 1;  // reference index size, jtree.h:113
  uint32_t* uv = upload_records(c, edges_uv, m, s);
  uint32_t* dseq = (uint32_t*)c.scratch.get("h_seq", (size_t)n_seq * 4);
  HIP_CHECK(hipMemcpyAsync(dseq, seq, (size_t)n_seq * 4, hipMemcpyHostToDevice, s));
  uint32_t* rank = (uint32_t*)c.scratch.get("rank", (size_t)n_rank * 4);
  launch_fill(rank, INV, n_rank, s);
  launch_rank_scatter(dseq, n_seq, rank, c.d_err, s);
  check_err(c, s);
  uint32_t* parent = (uint32_t*)c.scratch.get("h_parent", (size_t)n_seq * 4);
  uint32_t* pst = (uint32_t*)c.scratch.get("h_pst", (size_t)n_seq * 4);
  Timer tm(s);
  build_tree_dev(c, uv, m, rank, n_rank, n_seq, parent, pst, s, &tm);
  check_err(c, s);
  tm.finish(c);
  HIP_CHECK(hipMemcpyAsync(parent_out, parent, (size_t)n_seq * 4, hipMemcpyDeviceToHost, s));
  HIP_CHECK(hipMemcpyAsync(pst_out, pst, (size_t)n_seq * 4, hipMemcpyDeviceToHost, s));
  HIP_CHECK(hipStreamSynchronize(s));
  API_END
}

int sheep_merge_trees(const uint32_t* parent_a, const uint32_t* pst_a, const uint32_t* parent_b,
                      const uint32_t* pst_b, uint32_t n, uint32_t* parent_out, uint32_t* pst_out) {
  API_BEGIN
  Ctx& c = ctx();
  hipStream_t s = c.stream;
  if (n == 0) return SHEEP_OK;
  size_t b = (size_t)n * 4;
  uint32_t* pa = (uint32_t*)c.scratch.get("m_pa", b);
  uint32_t* sa = (uint32_t*)c.scratch.get("m_sa", b);
  uint32_t* pb = (uint32_t*)c.scratch.get("m_pb", b);
  uint32_t* sb = (uint32_t*)c.scratch.get("m_sb", b);
  HIP_CHECK(hipMemcpyAsync(pa, parent_a, b, hipMemcpyHostToDevice, s));
  HIP_CHECK(hipMemcpyAsync(sa, pst_a, b, hipMemcpyHostToDevice, s));
  HIP_CHECK(hipMemcpyAsync(pb, parent_b, b, hipMemcpyHostToDevice, s));
  HIP_CHECK(hipMemcpyAsync(sb, pst_b, b, hipMemcpyHostToDevice, s));
  uint32_t* jump = (uint32_t*)c.scratch.get("merge_jump", b);
  launch_merge(pa, sa, pb, sb, n, jump, s);
  HIP_CHECK(hipMemcpyAsync(parent_out, pa, b, hipMemcpyDeviceToHost, s));
  HIP_CHECK(hipMemcpyAsync(pst_out, sa, b, hipMemcpyDeviceToHost, s));
  check_err(c, s);
  API_END
}

}  // extern "C"
