// Internal declarations shared by the HIP kernels (sheep_kernels.hip) and the C-ABI
// (sheep_capi.cpp).  Not part of the public ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <deque>
#include <mutex>
#include <string>
#include <vector>

namespace sheep {

constexpr uint32_t INV = 0xFFFFFFFFu;

// Bits of the device error word (OR-ed by kernels, read by the host after a sync).
constexpr uint32_t ERR_RANGE = 1u;      // an id >= n_ids, or index.at(nbr) out of range
constexpr uint32_t ERR_DUP_SEQ = 2u;    // an id repeated in seq

// The current device's walk-guard word (sheep_kernels.hip): non-zero after a zipper or
// union-find walk met corrupt data and stopped; check_err reports it as -EIO and clears it.
uint32_t* fault_word();

// Growable device scratch.  One instance per device; slots are named so that the hot path
// reuses its buffers across calls (allocation only happens on the first / a larger call).
struct Scratch {
  struct Slot { void* p = nullptr; size_t bytes = 0; };
  std::vector<std::pair<std::string, Slot>> slots;
  void* get(const char* name, size_t bytes);  // throws std::runtime_error on hipMalloc failure
  size_t bytes_of(const char* name) const;    // current size of a slot (0: none)
  void release();
};

// Tuning options.  Every setting gives the same results (the etree is unique); they move work
// between kernels.  Read from SHEEP_<NAME> environment variables once, when the library first
// initialises a device, and changeable afterwards through sheep_set_option (include/
// sheep_amd.h) — never re-read per call.
struct Knobs {
  int degree = 0;        // SHEEP_DEGREE: 0 auto (bucketed from 2^18 records), 1 atomic, 2 bucketed
  int edge_part = -1;    // SHEEP_EDGE_PART: partitioned rank gathers; -1 auto (m >= 2^22), 0, 1
  int part_overlap = 4;  // SHEEP_PART_OVERLAP: one read for the degrees and the first partition
                         //   pass into sampled regions (4, graph2tree_dev from 2^25 records;
                         //   else 2), the first pass beside the degree pass (2), after it (1),
                         //   in line (0), fused into a counted degree scatter (3; taken anyway
                         //   from 2^31 records)
  int kb_buckets = 0;    // SHEEP_KB_BUCKETS: kb buckets cut at edge quantiles (0 = auto)
  int kb_rankb = 0;      // SHEEP_KB_RANKB: kb buckets cut at rank quantiles (0 = auto)
  int kb_pipe = 1;       // SHEEP_KB_PIPE: map of bucket k+1 beside the apply of bucket k
  int tree_stats = 0;    // SHEEP_TREE_STATS: 1 totals, 2 per bucket (stderr; diagnostics)
  int bin_direct = 1;    // SHEEP_BIN_DIRECT: the edge pass fills the hi bins directly (no scatter)
  int bin_slack = 50;    // SHEEP_BIN_SLACK: bin capacity = estimate x (1 + slack / 1000) + 8192
  int kb_gsum = -1;      // SHEEP_KB_GSUM: the map tests 64-rank "all in the giant" blocks in LDS
                         //   first; -1 auto (from 2^27 records), 0, 1
  int ls_seq = 1;        // SHEEP_LS_SEQ: with P > 1 ranks each sorts the ids of its 1/P of the id
                         //   space (degrees reduce-scattered; 0: all-reduced, every rank sorts all)
  int ls_split = 1;      // SHEEP_LS_SPLIT: with P > 1 ranks each bucket's zipper runs on one owner
                         //   rank (0: every rank applies every bucket's zipper)
  int kb_merge = 35;     // SHEEP_KB_MERGE: merge adjacent kb buckets while together they hold at
                         //   most kb_merge / 10000 of the records (0: off;
                         //   the lockstep loop: 20 unless off)
  int kb_fresh_lo = 50;  // SHEEP_KB_FRESH_LO / _HI: the kb loop's birth window, in hundredths of
  int kb_fresh_hi = 100; //   the mean degree 2E/B below a bucket's end (tree_from_sorted)
  int ff_groups = 1;     // SHEEP_FF_GROUPS: tile groups of the fused front pass (1..8): group g's
                         //   tiles write their own subregion of every region, so a subregion's
                         //   runs come from one XCD's blocks and merge in its L2 (round 6)
  int kb_rlink = 1;      // SHEEP_KB_RLINK: the refresh makes the zipper's first step of pairs from
                         //   pre-bucket roots (CAS INVALID -> b), leaving the rest to the zipper
  int eval_pass = 31;    // SHEEP_EVAL_PASS: at most 2^eval_pass adjacency entries sorted per pass
                         //   of the partition evaluation (more: passes over id ranges)
};
Knobs& knobs();  // the process-wide options (sheep_capi.cpp)

struct Ctx {
  int device = -1;
  hipStream_t stream = nullptr;
  hipStream_t side = nullptr;     // second stream of the pipelined kb loop (the maps)
  hipEvent_t kb_ev[5] = {};       // kb loop: [0,1] map done, [2,3] apply done (by parity), [4] start
  hipEvent_t part_ev[2] = {};     // graph2tree: [0] degree done, [1] first partition pass done
  hipEvent_t bins_ev = nullptr;   // the chunk degree sums reached the pinned host buffer
  uint64_t* h_chunks = nullptr;   // pinned host buffer for them (grown on demand)
  unsigned long long* h_bstart = nullptr;  // pinned: the 513 bin starts of the scatter
  size_t h_chunks_n = 0;
  Scratch scratch;
  uint32_t* d_err = nullptr;     // device error word
  uint32_t* h_pinned = nullptr;  // pinned host words for small readbacks
  std::vector<std::pair<const char*, double>> timings;
  std::deque<std::string> span_names;  // storage for the "<name>#" timing labels
  std::vector<hipEvent_t> ev_pool;     // timing events of finished calls (Timer), reused
  std::mutex ev_mu;                    // guards ev_pool (the rest of a context is one caller's at
                                       // a time: include/sheep_amd.h "Threads")
  int ls_live = 0;                     // live lockstep sessions (sheep_ls_*) on this device
  struct Comm* comm = nullptr;         // this rank's communicator (sheep_comm_init), if any
  // host record ranges declared immutable (sheep_records_register / sheep_records_load_dat)
  // and their device copies: host-pointer calls on them upload nothing
  struct Registered { const uint32_t* host; uint64_t m; uint32_t* dev; };
  std::vector<Registered> registered;
};

Ctx& ctx();  // this thread's context for the current device (sheep_gpu_init)

// ---- launchers (sheep_kernels.hip); all enqueue on `s` -------------------------------------
void launch_degree(const uint32_t* uv, uint64_t m, uint32_t n_ids, int file_mode, uint32_t* deg,
                   uint32_t* selfc, uint32_t* err, hipStream_t s);
// pst = nsdeg - run length of r in the hi-sorted items (start/end: n_seq scratch words each)
void launch_pst_from_degree(const uint64_t* sorted, uint64_t m, const uint32_t* seq, uint32_t n_seq,
                            const uint32_t* deg, const uint32_t* selfc, int file_mode,
                            uint32_t* start, uint32_t* end, uint32_t* pst, hipStream_t s);
// Bucketed LDS degree histogram for large m (same result as launch_degree); selfc nullable.
size_t degb_tmp_words(uint64_t m, uint32_t n_ids, int* SH_out, uint32_t* NB_out);
// yhist (nullable, 1024 words): also counts the y digits of launch_part_gather's first pass
// (n_rank = n_ids), so that pass needs no counting read; returns true when it did.
bool launch_degree_bucketed(const uint32_t* uv, uint64_t m, uint32_t n_ids, int file_mode,
                            uint32_t* deg, uint32_t* selfc, uint32_t* err, uint32_t* tmp,
                            hipStream_t s, uint32_t* yhist = nullptr,
                            hipEvent_t counted = nullptr /* recorded once yhist is complete */,
                            uint32_t* stats = nullptr /* [0] max degree, [1] zero-degree ids */);
// Fused front half (graph2tree_dev): degrees (deg, selfc, stats as launch_degree_bucketed)
// and the records (x, y) grouped by y bucket into recs (m u64), the x digits of
// launch_part_second counted into part_ws (spread, xh_ix) — what launch_part_first produced.  tmp:
// fh_tmp_words (1: not applicable, n_ids beyond 2^26).  False when not applicable.
size_t fh_tmp_words(uint64_t m, uint32_t n_ids);
bool launch_fh_front(const uint32_t* uv, uint64_t m, uint32_t n_ids, int file_mode, uint32_t* deg,
                     uint32_t* selfc, uint32_t* err, uint32_t* tmp, uint64_t* recs,
                     uint32_t* part_ws, uint32_t* stats, hipStream_t s,
                     void (*mark)(void*, const char*) = nullptr /* phase marks (timing) */,
                     void* mark_arg = nullptr);
void launch_deg_stats(const uint32_t* deg, uint32_t n, uint32_t* stats /*[0]=max,[1]=zeros*/,
                      hipStream_t s);
// Exclusive scan of n u32 (n < 2^32); tmp needs scan_tmp_words(n) u32.
size_t scan_tmp_words(uint64_t n);
void launch_scan_exclusive(const uint32_t* in, uint32_t* out, uint64_t n, uint32_t* tmp,
                           hipStream_t s);
size_t rsort_tmp_words(uint64_t n);
int rsort_first_width(int bits);
uint64_t* radix_sort_u64(const uint64_t* in, uint64_t* a, uint64_t* b, uint64_t n, int bit_lo,
                         int bit_hi, uint32_t* tmp, hipStream_t s, bool counted0 = false);
void launch_pack_deg(const uint32_t* deg, uint32_t n, uint64_t* items, hipStream_t s);
// (deg << 32 | id) of the ids with deg > 0 only, in id order; tmp: pack_nz_tmp_words(n) u32.
size_t pack_nz_tmp_words(uint32_t n);
void launch_pack_nonzero(const uint32_t* deg, uint32_t n, uint64_t* items, uint32_t* tmp,
                         hipStream_t s);
void launch_unpack_seq(const uint64_t* items, uint32_t zeros, uint32_t n_seq, uint32_t* seq,
                       uint32_t* rank, hipStream_t s, uint32_t* nsd = nullptr,
                       const uint32_t* selfc = nullptr, int file_mode = 0,
                       uint32_t base = 0 /* first sequence position written */);
// Counting-sort sequence (k_seqc_*): seq/rank/nsd of every id of degree 1 .. seqc_threshold()-1,
// rank INVALID for degree 0; the ids of higher degree go to big as (deg << 32 | id) in id order,
// to be sorted and unpacked from the position the returned device word (u64) holds.
size_t seqc_tmp_words(uint32_t n);
uint32_t seqc_threshold();
// selfc (nullable): nsd = deg - w * selfc (w = 2 in FILE mode), as launch_nsd_selfloops.
uint32_t* launch_seqc_place(const uint32_t* deg, uint32_t n, uint32_t* seq, uint32_t* rank,
                            uint32_t* nsd, uint64_t* big, uint32_t* tmp, hipStream_t s,
                            const uint32_t* selfc, int file_mode);
// nsd[rank[v]] -= w * selfc[v] (w = 2 in FILE mode): the self-loop part of launch_unpack_seq's nsd.
void launch_nsd_selfloops(const uint32_t* selfc, uint32_t n_ids, const uint32_t* rank,
                          int file_mode, uint32_t* nsd, hipStream_t s);
void launch_fill(uint32_t* p, uint32_t value, uint64_t n, hipStream_t s);
void launch_rank_scatter(const uint32_t* seq, uint32_t n_seq, uint32_t* rank, uint32_t* err,
                         hipStream_t s);
void launch_edge_pass(const uint32_t* uv, uint64_t m, const uint32_t* rank, uint32_t n_rank,
                      uint32_t* pst /* nullable: no pst */, uint64_t* items, uint32_t* err,
                      hipStream_t s);
// edge pass + the first radix pass's tile histograms (sort bits from `shift`, DB wide)
void launch_edge_pass_tiles(const uint32_t* uv, uint64_t m, const uint32_t* rank, uint32_t n_rank,
                            uint32_t* pst, uint64_t* items, uint32_t* err, int shift, int DB,
                            uint32_t* tmp, hipStream_t s, bool pre = false);
// Hi bins (one-pass grouping, see sheep_kernels.hip): chunk degree sums (256 ranks per chunk),
// the edge pass counting bins (no pst; nb <= 512 bounds, bounds[0] = 0, bounds[nb-1] = n_seq
// so that INVALID his fall in the last bin), and the scatter by bin (bin_start: nb+1 u64).
void launch_chunk_degsum(const uint32_t* seq, const uint32_t* deg, uint32_t n_seq, uint64_t* out,
                         hipStream_t s, const uint32_t* nsd = nullptr);
// digits: m u16 scratch (each item's bin, written by the edge pass, read by the scatter)
void launch_edge_pass_bins(const uint32_t* uv, uint64_t m, const uint32_t* rank, uint32_t n_rank,
                           uint64_t* items, uint32_t* err, const uint32_t* bins, uint32_t nb,
                           uint32_t* tmp, uint16_t* digits, hipStream_t s, bool pre);
void bin_sort_u64(const uint64_t* in, uint64_t* out, uint64_t n, const uint32_t* bins, uint32_t nb,
                  uint32_t* tmp, unsigned long long* bin_start, const uint16_t* digits,
                  hipStream_t s,
                  unsigned long long* h_start = nullptr /* pinned: bin_start, before the scatter */,
                  hipEvent_t started = nullptr /* recorded once h_start is written */);
// Records (uv, or k_part's pre records) -> items (hi << 32 | lo) grouped by hi bin: the edge
// pass (items, each item's bin into digits (m u16), tile bin counts), then the scatter.
// Returns the buffer holding the result (items_b; items is then free); uv may be items_b.
// bin_start, h_start, started: as bin_sort_u64.
uint64_t* group_by_bins(const uint32_t* uv, bool pre, uint64_t m, const uint32_t* rank,
                        uint32_t n_rank, uint32_t* err, const uint32_t* bins, uint32_t nb,
                        uint64_t* items, uint64_t* items_b, uint32_t* tmp, uint16_t* digits,
                        unsigned long long* bin_start, hipStream_t s,
                        unsigned long long* h_start = nullptr, hipEvent_t started = nullptr);
// Partitioned rank gathers: uv (x, y) -> pre (x, rank[y] | sentinel) in x-digit order (mid:
// m u64 scratch, ws: PART_WS_WORDS u32 scratch); then launch_edge_pass_tiles(pre, ..., pre = true).
// ws: y / x digit counts, the first pass's u64 cursors, the u32 region starts of both passes'
// outputs, the second pass's cursors, the first pass's capacity region ends (sheep_kernels.hip).
// The fused front pass's region cursors (k_front_fused: one device-scope atomic per region and
// tile, ~134 M a call at RMAT-26, performed at the memory side) are spread over memory: cursor
// q sits at u64 index fs_cix(q) = (q / 8) * SHEEP_FS_CLS + q % 8, eight to a 64-B line and
// consecutive lines SHEEP_FS_CLS u64 apart (8: contiguous).
#ifndef SHEEP_FS_CLS
#define SHEEP_FS_CLS 64
#endif
constexpr uint32_t FS_CLS = SHEEP_FS_CLS;
__host__ __device__ inline uint32_t fs_cix(uint32_t q) { return (q >> 3) * FS_CLS + (q & 7u); }
constexpr size_t fs_cur_words(uint32_t n) { return 2 * (size_t)((n + 7) / 8) * FS_CLS; }
// (+ the fused front pass's subregion tables: 8192 u64 starts + 2, cursors (spread), ends, u32
// tile map)
// The second partition pass's x-digit counts (256 u32, added to by every tile of the first pass
// or the fused pass) are spread the same way: digit i at xh_ix(i) = (i / 16) * XH_CLS + i % 16.
constexpr uint32_t XH_CLS = 128;
__host__ __device__ inline uint32_t xh_ix(uint32_t i) { return (i >> 4) * XH_CLS + (i & 15u); }
constexpr size_t XH_WORDS = (256 / 16) * XH_CLS;
constexpr size_t PART_WS_WORDS = 1280 + 2 * 1024 + 1025 + 257 + 2 * 256 + 2 * 1024 +
                                 2 * (8192 + 2) + fs_cur_words(8192) + 2 * 8192 + 8192 + 1 +
                                 1 + XH_WORDS;
// p6: the second pass's records are packed to 6 bytes (sheep_kernels.hip "packed 6-byte
// records"; only where part_p6_ok(n_rank) and an id >= n_rank fails the call).
bool part_p6_ok(uint32_t n_rank);
void launch_part_gather(const uint32_t* uv, uint64_t m, const uint32_t* rank, uint32_t n_rank,
                        uint64_t* mid, uint64_t* pre, uint32_t* ws, hipStream_t s,
                        bool yhist_ready = false, bool p6 = false);
// The two passes of launch_part_gather separately (the first needs no ranks, so it can run
// while the sequence is sorted): uv -> mid (y-digit order), then mid -> pre (x-digit order).
void launch_part_first(const uint32_t* uv, uint64_t m, uint32_t n_rank, uint64_t* mid,
                       uint32_t* ws, hipStream_t s, bool yhist_ready);
// out6: pre is written packed; caps: mid holds launch_part_first_caps's regions (mid_slots);
// in6 (with caps): ... launch_front_fused's packed ones.
// (in6: the tiles follow the fused pass's subregions, G per y digit: launch_front_fused's G.)
void launch_part_second(const uint64_t* mid, uint64_t m, const uint32_t* rank, uint32_t n_rank,
                        uint64_t* pre, uint32_t* ws, hipStream_t s, bool out6 = false,
                        uint64_t mid_slots = 0, bool caps = false, bool in6 = false,
                        uint32_t G = 1);
// Sampled capacities (sheep_kernels.hip, "sampled capacities"): the degree pass without a
// counting read — a 1/256 sample sizes each bucket's and each y digit's capacity region; the
// y regions go to part_ws for launch_part_first_caps (mid_slots records; the event caps_done
// marks them written).  *ovf is set when a run outgrew its region: the degrees
// are then invalid and the caller runs the exact pass.  False when not applicable.
size_t degs_tmp_words(uint64_t m, uint32_t n_ids);
// The most slots the sampled capacity regions of `items` items over n_regions can take (the
// first pass's packed records: fs_room(m, 1024) slots of 6 bytes).
uint64_t fs_room(uint64_t items, uint32_t n_regions);
bool launch_degree_sampled(const uint32_t* uv, uint64_t m, uint32_t n_ids, int file_mode,
                           uint32_t* deg, uint32_t* selfc, uint32_t* err, uint32_t* tmp,
                           uint32_t* part_ws, uint64_t mid_slots, uint32_t* stats, uint32_t* ovf,
                           hipStream_t s, hipEvent_t caps_done);
// The fused front pass (sheep_kernels.hip k_front_fused): degrees and the first partition from
// ONE read of the records, into sampled capacity regions (mid_slots, a multiple of 8, packed
// records in mid).  *ovf_x: the degrees need the exact pass; *ovf_y: the partition must be
// redone from uv, and the degrees too (the histogram counts y's ids from the packed records).  False when not applicable (front_fused_ok).
// G (option ff_groups, 1..8): tile groups, each writing its own subregion of every region
// (sheep_kernels.hip k_front_fused); front_fused_slots: the mid_slots these regions need.
bool front_fused_ok(uint64_t m, uint32_t n_ids);
uint64_t front_fused_slots(uint64_t m, uint32_t n_ids, uint32_t G);
bool launch_front_fused(const uint32_t* uv, uint64_t m, uint32_t n_ids, int file_mode,
                        uint32_t* deg, uint32_t* selfc, uint32_t* err, uint32_t* tmp,
                        uint32_t* part_ws, uint64_t* mid, uint64_t mid_slots, uint32_t* stats,
                        uint32_t* ovf_x, uint32_t* ovf_y, hipStream_t s,
                        void (*mark)(void*, const char*) = nullptr, void* mark_arg = nullptr,
                        uint32_t G = 1);
void launch_part_first_caps(const uint32_t* uv, uint64_t m, uint32_t n_rank, uint64_t* mid,
                            uint64_t mid_slots, uint32_t* ws, uint32_t* ovf, hipStream_t s);
void launch_pst_from_count(const uint32_t* seq, uint32_t n_seq, const uint32_t* deg,
                           const uint32_t* selfc, int file_mode, const uint32_t* cnt, uint32_t* pst,
                           hipStream_t s,
                           const uint32_t* nsd = nullptr);
void launch_kb_bounds(const uint64_t* items, uint64_t n, uint32_t K_e, uint32_t K_r,
                      uint32_t n_seq, int gshift, unsigned long long* out, hipStream_t s);
// The records of a kb bucket when they were binned directly (launch_edge_bin): bins [i0, i1),
// bin i's items at [start[i], min(cur[i], cap[i])) (device arrays).
struct KbSegs {
  const unsigned long long* start;
  const unsigned long long* cur;
  const unsigned long long* cap;
  uint32_t i0, i1;
};
// Direct binning (sheep_kernels.hip): records (uv, or k_part's pre records) -> items grouped by
// hi bin, each bin in its capacity region [cursor[b] at entry, cap_end[b]); cursor[b] ends at
// the bin's fill.  *ovf is set (and the run dropped) when a bin overflows its capacity.
// part_ws (non-null only with pre): the records are launch_part_second's packed output, whose
// x-digit regions part_ws holds.
void launch_edge_bin(const uint32_t* uv, bool pre, uint64_t m, const uint32_t* rank,
                     uint32_t n_rank, uint32_t* err, const uint32_t* bins, uint32_t nb,
                     unsigned long long* cursor, const unsigned long long* cap_end, uint64_t* out,
                     uint32_t* ovf, hipStream_t s, const uint32_t* part_ws = nullptr);
// One kb bucket in two halves (sheep_kernels.hip): the map (records -> kept pairs + giant marks
// + hi counts) and the apply (spine, zipper, union-find fold, labels).  counters: this
// bucket parity's 4 words; anchor: see launch_kb_map.
// kept_cap: the u64 slots kept holds (a reservation past it raises the fault word, -EIO).
void launch_kb_map(const uint64_t* items, uint64_t e_begin, uint64_t e_end, uint32_t B0,
                   uint32_t anchor, uint32_t* uf, const uint32_t* label, uint64_t* kept,
                   uint64_t kept_cap, uint32_t* bitmap, uint32_t* counters, int gshift,
                   uint32_t* cnt /* nullable: hi run lengths */, bool stats,
                   unsigned long long* st, const uint32_t* bins /* nullable: hi bins */,
                   uint32_t nb, uint32_t* gbits /* nullable: giant bitmap */,
                   const uint32_t* gx /* its reference-vertex slot (nullable: no bitmap) */,
                   int defer /* 1: misses kept as (b, a) for launch_kb_apply's refresh;
                                2: as (b, root of a) (split lockstep); 0: as (b, label) */,
                   hipStream_t s, const KbSegs* segs = nullptr,
                   const uint32_t* anc = nullptr /* device-picked anchor (launch_kb_pick) */,
                   const uint32_t* gsum = nullptr /* giant summary (launch_gb_sum) */);
// Giant summary for the next map (nothing writing gbits): bit q = ranks [64q, 64q + 64) all set
// in gbits; (n_seq / 2048 + 1) words.
void launch_gb_sum(const uint32_t* gbits, uint32_t n_seq, uint32_t* gsum, hipStream_t s);
// Giant sweep (sheep_kernels.hip k_gb_sweep): the giant bits of every rank v < B0lim in the
// component of *gx, with nothing that may move *gx running beside it.
void launch_gb_sweep(uint32_t* uf, uint32_t* gbits, uint32_t B0lim, const uint32_t* gx,
                     hipStream_t s);
// The giant's anchor for the next map, picked on the device among ranks [0, B0lim) (the
// component holding most of an even sample; see sheep_kernels.hip), written to *anc_out (INV
// when B0lim = 0); gbits (nullable): the bitmap is then rebased on it (launch_gb_rebase).
void launch_kb_pick(const uint32_t* uf, uint32_t B0lim, const uint32_t* anc_prev, uint32_t* anc_out,
                    uint32_t* gbits, uint32_t n_seq, const uint32_t* gx_rd, uint32_t* gx_wr,
                    hipStream_t s);
// Before a map (nothing else touching the union-find): keep the giant bitmap's reference
// vertex (*gx_rd) if it is in the anchor's component, else move it to the anchor and clear
// the bitmap (n_seq / 32 + 2 words); the result goes to *gx_wr.
void launch_gb_rebase(uint32_t* gbits, uint32_t n_seq, const uint32_t* uf, uint32_t anchor,
                      const uint32_t* gx_rd, uint32_t* gx_wr, hipStream_t s);
// refresh: re-resolve the kept starts against the current union-find first (pipelined loop).
// gbits / gx: the giant bitmap and the slot written by the latest rebase on this stream.
void launch_kb_apply(bool nonempty, uint32_t B0, uint32_t B1, uint32_t anchor, uint32_t* uf,
                     uint32_t* label, uint32_t* parent, uint32_t* jump, uint64_t* kept,
                     uint32_t* linked, uint32_t* bitmap, uint32_t* spq, uint32_t* counters,
                     bool refresh, bool stats, unsigned long long* st, uint32_t* gbits,
                     const uint32_t* gx, hipStream_t s,
                     const uint32_t* anc = nullptr /* this bucket's device anchor */,
                     const uint32_t* anc_next = nullptr /* the next map's: its root is kept */);
// Lockstep exchange of one bucket (sheep_ls_*): pack this rank's mark words [w0, w1] (ms u64
// slots) and kept pairs (padded to cap) for an all-gather; unpack P such blocks into the
// bitmap (OR) and a contiguous kept array, setting *n_kept = P * cap (kept and n_kept
// nullable: the marks only).
void launch_ls_pack(const uint32_t* bitmap, uint32_t w0, uint32_t w1, uint32_t ms, uint64_t* send,
                    const uint32_t* n_kept /* device */, uint32_t cap, hipStream_t s);
void launch_ls_count(const uint32_t* n_kept, long long* out, hipStream_t s);
void launch_ls_unpack(const uint64_t* recv, uint32_t P, uint32_t ms, uint32_t cap, uint32_t* bitmap,
                      uint32_t w0, uint32_t w1, uint64_t* kept, uint32_t* n_kept, hipStream_t s);
// Split lockstep apply (P > 1; see sheep_kernels.hip): the refresh alone; G of the bucket's
// giant into *gslot; every rank's union-find part (fold, union of the kept pairs, labels;
// counters reset); the owner's spine + zipper over its copies (zn: n_kept, n_spine, G).
void launch_kb_refresh(uint64_t* kept, const uint32_t* n_kept, uint32_t* uf, const uint32_t* label,
                       uint32_t* bitmap, uint32_t B0, uint32_t anchor, uint32_t* gbits,
                       const uint32_t* gx, const uint32_t* anc, hipStream_t s);
void launch_ls_gslot(const uint32_t* uf, const uint32_t* label, uint32_t anchor, const uint32_t* anc,
                     uint32_t* gslot, hipStream_t s);
void launch_ls_fold_union_label(bool nonempty, uint32_t B0, uint32_t B1, uint32_t anchor,
                                uint32_t* uf, uint32_t* label, const uint64_t* recv, uint32_t P,
                                uint32_t ms, uint32_t cap, uint32_t* bitmap, uint32_t* counters,
                                uint32_t* gbits, const uint32_t* gx, hipStream_t s,
                                const uint32_t* anc, const uint32_t* anc_next);
void launch_ls_zip(const uint64_t* zkept, uint32_t* zn, const uint32_t* zbm, uint32_t* zspq,
                   uint32_t B0, uint32_t B1, bool has_anchor, uint32_t* parent, uint32_t* jump,
                   hipStream_t s);
void launch_add_u32(uint32_t* p, uint64_t n, uint32_t d, hipStream_t s);  // p[i] += d (wraps)
// Sharded degree sequence (P > 1, sheep_capi.cpp sequence_sharded; see sheep_kernels.hip).
void launch_seq_runs(const uint64_t* sorted, uint32_t n, uint32_t* lst, uint32_t* H, hipStream_t s);
void launch_seq_base(const uint32_t* hall, uint32_t P, uint32_t r, uint32_t D, uint32_t Dp,
                     uint32_t* tot, uint32_t* pre, hipStream_t s);
void launch_seq_rank(const uint64_t* sorted, uint32_t n, const uint32_t* S, const uint32_t* pre,
                     const uint32_t* lst, uint32_t* rank_slice, hipStream_t s);
void launch_seq_from_rank(const uint32_t* rank, uint32_t n_ids, uint32_t* seq, hipStream_t s);
void launch_deg_of_rank(const uint32_t* S, uint32_t D, uint32_t n_seq, uint32_t* out, hipStream_t s);
void launch_seq_stats64(const uint32_t* stats, uint32_t c, long long* out, hipStream_t s);
void launch_iota(uint32_t* p, uint32_t n, hipStream_t s);
void launch_forest_items(const uint32_t* parent, uint32_t n, uint64_t* items, hipStream_t s);
// The kb loop's parents and hints, interleaved (pj[2v] = parent, pj[2v + 1] = hint; 2n words):
// (INVALID, 0) for every rank; the parents out to parent[0, n).
void launch_pj_init(uint32_t* pj, uint32_t n, hipStream_t s);

void launch_pj_parents(const uint32_t* pj, uint32_t n, uint32_t* parent, hipStream_t s);
// Partition quality (sheep_eval.hip).  ws: 4k + 8 u64: [0,3k) hash/down/up balances, [3k,4k)
// vertex balance, then cut, self-loop records, nodes, and the distinct keys of vcom, hash,
// down, up.  keys/keys_b: 2m u64; rtmp: rsort_tmp_words(2m) u32; deg: LLAMA degrees.
// passes (nullable / empty: one pass over the 2m entries): (first id, keys bound) of
// consecutive id ranges; each pass sorts only the entries X -> Y with X in its range (keys /
// keys_b then need the largest bound, not 2m).  ws[4k + 7] is the passes' append counter.
void launch_evaluate(const uint32_t* uv, uint64_t m, const int16_t* parts, const uint32_t* pos,
                     const uint32_t* deg, uint32_t n_ids, uint32_t k, uint64_t* keys,
                     uint64_t* keys_b, uint32_t* rtmp, unsigned long long* ws, uint32_t* err,
                     hipStream_t s,
                     const std::vector<std::pair<uint32_t, uint64_t>>* passes = nullptr);
// graph2tree -p K -o OUT (sheep_eval.hip): the non-self-loop records as (min, max) pairs,
// grouped by the part of their lower-sequence endpoint, each part in (min, record) order.
// items / items_b: m u64; rtmp: rsort_tmp_words(m); out: 2m u32; pstart: n_parts + 1 u64.
void launch_partition_edges(const uint32_t* uv, uint64_t m, const int16_t* parts, const uint32_t* pos,
                            uint32_t n_ids, uint32_t n_parts, uint64_t* items, uint64_t* items_b,
                            uint32_t* rtmp, uint32_t* out, unsigned long long* pstart, uint32_t* err,
                            hipStream_t s);
// XS1 records {u32 tail, u32 head, f32 weight} -> (tail, head) pairs; max id + 1 into *max_id.
void launch_strip_xs1(const uint32_t* raw, uint64_t n, uint32_t* uv, uint32_t* max_id, hipStream_t s);
void launch_merge(uint32_t* parent_a, uint32_t* pst_a, const uint32_t* parent_b,
                  const uint32_t* pst_b, uint32_t n, uint32_t* jump, hipStream_t s);
void launch_rmat(uint32_t* uv, int scale, uint64_t seed, uint64_t e_begin, uint64_t e_end,
                 hipStream_t s);
void launch_powerlaw(uint32_t* uv, uint32_t n, double gamma, double i0, uint64_t seed,
                     uint64_t e_begin, uint64_t e_end, hipStream_t s);

}  // namespace sheep
