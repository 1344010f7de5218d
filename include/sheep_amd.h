/* sheep_amd.h — the C-ABI of the MI355X build of Sheep's tree-construction hot path.
 *
 * Drop-in boundary.  The reference has no FFI: its boundary is the header-only C++
 * API in lib/ (sequence.h, jtree.h, jnode.h), consumed by the graph2tree / degree_sequence /
 * merge_trees binaries.  Each entry point below replaces one reference interface; the C++
 * host layer in sheep_amd/lib/ keeps the reference's C++ signatures and calls these.
 *
 * ABI rules:
 *   - every call returns 0 (SHEEP_OK) or a negative errno-style code; no exception crosses the
 *     ABI; sheep_last_error() gives the text of the calling thread's last failure;
 *   - the caller owns every buffer; the library owns its device scratch (grown on demand,
 *     released by sheep_release());
 *   - host-pointer calls are synchronous; *_dev calls take device pointers and a HIP stream
 *     (hipStream_t passed as void*; NULL = HIP's default stream, as everywhere in HIP) and
 *     return when the work is ENQUEUED, except where documented as synchronising;
 *   - calls are not re-entrant per device.  Threads: a device's context (its scratch, streams
 *     and pinned words) serves one caller at a time — two host threads driving the same device
 *     at once must serialise their calls themselves (the timing-event pool alone is locked);
 *     the n_ranks rehearsal entry points below give each rank thread a context of its own.
 *
 * Types follow lib/defs.h:76-82: ids, jnids and weights are uint32, INVALID = 0xFFFFFFFF.
 * An edge stream is m records of (tail, head) as 2*m uint32 (the XS1 weight is dropped).
 *
 * Size limits: every call takes m < 2^32 records (record offsets and counters are u32; larger
 * inputs return -EINVAL: shard them with -l n/k + merge, or the multi-GPU entry points).  The
 * degree pass counts endpoints with record offsets beyond 2^31 records (the fused pass of
 * graph2tree); the partition evaluation sorts at most 2^31 adjacency entries per pass and
 * beyond that walks id ranges, so only a single vertex with more than 2^31 entries is refused.
 */
#ifndef SHEEP_AMD_H
#define SHEEP_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SHEEP_OK 0
#define SHEEP_INVALID 0xFFFFFFFFu

/* Degree conventions.
 * LLAMA: what graph2tree sees (graph_wrapper.h:87-89): a self-loop counts once.
 * FILE:  degree_sequence's streaming count (sequence.h:101-107): a self-loop counts twice. */
#define SHEEP_DEGREE_LLAMA 0
#define SHEEP_DEGREE_FILE 1

/* ---- device / library ------------------------------------------------------------------- */

/* Select the HIP device for this thread's calls and create the library stream + scratch.
 * Replaces the process/device setup around MPI_Init in graph2tree.cpp:134-157.  It takes the
 * device INDEX, not SURVEY §8b's draft n_devices: one process (MPI rank) drives one GPU, so
 * a rank names its own device (LOCAL_RANK); the multi-GPU calls below take the rank count. */
int sheep_gpu_init(int device);

/* ---- records resident in HBM (the graph LLAMA keeps in RAM, graph_wrapper.h:43-63) --------
 * sheep_records_register: the host records [uv, uv + 2m) are immutable until
 * sheep_records_release(uv); the library keeps ONE device copy, and every host-pointer call
 * given exactly (uv, m) uses it instead of uploading the records again.
 * sheep_records_load_dat: reads the XS1 records of a .dat file (all of them, or the contiguous
 * range of part/num_parts, 1-based, as graph2tree -l; the weight dropped) through pinned
 * staging buffers straight into a registered device copy, filling uv_out (cap records) on the
 * host meanwhile; uv_out NULL: *m_out only (size query).  *max_id_out = max id + 1 of the
 * range.  Release with sheep_records_release(uv_out). */
int sheep_records_register(const uint32_t* uv, uint64_t m);
int sheep_records_release(const uint32_t* uv);
int sheep_records_load_dat(const char* path, uint64_t part, uint64_t num_parts, uint32_t* uv_out,
                           uint64_t cap, uint64_t* m_out, uint32_t* max_id_out);
/* The same ingest into caller device memory d_uv (cap records; NULL: size query only).
 * Synchronises the stream. */
int sheep_read_dat_dev(const char* path, uint64_t part, uint64_t num_parts, uint32_t* d_uv,
                       uint64_t cap, uint64_t* m_out, uint32_t* max_id_out, void* stream);

/* Free all device scratch held by the library on the current device. */
int sheep_release(void);

/* Text of the last error on this thread ("" if none). */
const char* sheep_last_error(void);

/* ABI version: (major << 16) | minor. */
int sheep_abi_version(void);

/* Tuning options (sheep_amd/csrc/sheep_internal.h, struct Knobs): they move work between
 * kernels and never change a result.  Their defaults come from SHEEP_<NAME> environment
 * variables, read ONCE when the library first initialises a device; afterwards only these
 * calls change them (process-wide).  Names: degree, edge_part, part_overlap, kb_buckets,
 * kb_rankb, kb_merge, kb_pipe, tree_stats, bin_direct, bin_slack, kb_gsum, eval_pass,
 * ls_split, ls_seq.
 * -EINVAL for an unknown name. */
int sheep_set_option(const char* name, long long value);
int sheep_get_option(const char* name, long long* value);

/* ---- host-pointer API (synchronous; what the reference's lib/ would bind) --------------- */

/* Degree sequence: the ids with degree>0 ordered by (degree asc, id asc).
 * Replaces degreeSequence (sequence.h:52-63) [LLAMA mode] and fileSequence_template
 * (sequence.h:95-122) [FILE mode].  n_ids: every id in edges_uv must be < n_ids; pass 0 to
 * take max id + 1.  seq_out must hold n_ids entries; *n_seq_out receives the length.
 * rank_out (nullable, n_ids entries) receives jnid = position in seq, or INVALID. */
int sheep_degree_seq(const uint32_t* edges_uv, uint64_t m, uint32_t n_ids, int degree_mode,
                     uint32_t* seq_out, uint32_t* n_seq_out, uint32_t* rank_out);

/* Elimination tree of the edge stream under seq: JNode{parent, pst_weight} per jnid.
 * Replaces JTree(graph, seq[, file], Options()) (jtree.h:111-136 -> insertSequence
 * jtree.cpp:112-145 -> insert jtree.cpp:65-110).  parent_out/pst_out hold n_seq entries.
 * Errors: -EINVAL if seq repeats an id (the reference asserts, jtree.h:166);
 *         -ERANGE if an edge joins a seq vertex to an id > max(seq) (index.at throws,
 *         jtree.cpp:75).
 * No n_ids argument (SURVEY §8b's draft had one): the reference sizes its rank index by
 * max(seq) + 1 (jtree.h:113-122), and that bound, not the id space, decides which records are
 * ignored and which raise index.at's out_of_range; a separate n_ids could only disagree with
 * it.  The device entry points below take n_ids because there the caller owns the rank map. */
int sheep_build_tree(const uint32_t* edges_uv, uint64_t m, const uint32_t* seq, uint32_t n_seq,
                     uint32_t* parent_out, uint32_t* pst_out);

/* Associative tree union: etree(A ∪ B), pst summed (u32, wraps).
 * Replaces JNodeTable::merge (jnode.cpp:174-201) as called by merge_trees.cpp:85-88 and by
 * mpi_merge_reduction (jnode.cpp:203-211).  Both trees must come from the same seq. */
int sheep_merge_trees(const uint32_t* parent_a, const uint32_t* pst_a, const uint32_t* parent_b,
                      const uint32_t* pst_b, uint32_t n, uint32_t* parent_out, uint32_t* pst_out);

/* ---- device-pointer API (the hot path; all pointers are device memory) ------------------ */

/* deg[v] = degree of v over the m records (written, not accumulated); ids >= n_ids are an
 * error (-ERANGE, reported by the next synchronising call).  Replaces the per-rank degree
 * vector of mpiSequence (sequence.h:75-77). */
int sheep_degree_dev(const uint32_t* d_uv, uint64_t m, uint32_t n_ids, int degree_mode,
                     uint32_t* d_deg, void* stream);

/* As sheep_degree_dev, and d_selfc (nullable, n_ids entries) receives the number of
 * self-loop records at each id — what sheep_build_tree_deg_dev needs to derive pst_weight
 * from degrees instead of one atomic per record. */
int sheep_degree_ex_dev(const uint32_t* d_uv, uint64_t m, uint32_t n_ids, int degree_mode,
                        uint32_t* d_deg, uint32_t* d_selfc, void* stream);

/* seq/rank from a degree vector (after an all-reduce for sharded input: sequence.h:78-91).
 * d_seq and d_rank hold n_ids entries.  Synchronises the stream; *n_seq_out is set. */
int sheep_sequence_dev(const uint32_t* d_deg, uint32_t n_ids, uint32_t* d_seq, uint32_t* d_rank,
                       uint32_t* n_seq_out, void* stream);

/* Partial or full elimination tree of the m records under the rank map d_rank (n_ids
 * entries, INVALID for ids outside seq).  d_parent/d_pst hold n_seq entries.  Synchronises
 * the stream (the tree builder sizes its passes on the host). */
int sheep_build_tree_dev(const uint32_t* d_uv, uint64_t m, const uint32_t* d_rank, uint32_t n_ids,
                         uint32_t n_seq, uint32_t* d_parent, uint32_t* d_pst, void* stream);

/* sheep_build_tree_dev with the degrees of THESE m records (d_deg, d_selfc from
 * sheep_degree_ex_dev, in degree_mode) and d_seq (n_seq entries): pst_weight is derived as
 * (non-self-loop degree) - (PREORDER records), with no per-record atomics.  For an edge shard,
 * pass the shard's own (pre-all-reduce) degrees.  Synchronises the stream. */
int sheep_build_tree_deg_dev(const uint32_t* d_uv, uint64_t m, const uint32_t* d_rank,
                             uint32_t n_rank, const uint32_t* d_seq, uint32_t n_seq,
                             const uint32_t* d_deg, const uint32_t* d_selfc, int degree_mode,
                             uint32_t* d_parent, uint32_t* d_pst, void* stream);

/* In-place merge: (parent_a, pst_a) <- etree(A ∪ B).  Enqueue only. */
int sheep_merge_trees_dev(uint32_t* d_parent_a, uint32_t* d_pst_a, const uint32_t* d_parent_b,
                          const uint32_t* d_pst_b, uint32_t n, void* stream);

/* d_parent_out <- etree of the union of n_trees forests over the same n ranks, given as
 * n_trees consecutive parent arrays in d_parents (n_trees * n words; INVALID = root).  The
 * parent half of an n_trees-way merge (jnode.cpp:174-201 applied pairwise, mpi_merge
 * jnode.cpp:213-250) done in one build: the edges (v, parent_t[v]) of every tree sorted by
 * parent and inserted as in graph2tree; pst_weight of a merge is the plain sum.  Synchronises. */
int sheep_merge_forests_dev(const uint32_t* d_parents, uint32_t n_trees, uint32_t n,
                            uint32_t* d_parent_out, void* stream);

/* ---- lockstep multi-GPU tree build (graph2tree -i -r, graph2tree.cpp:134-200) -----------
 * The elimination tree of the union of P edge shards, one shard per rank, without partial
 * trees: every rank keeps the SAME union-find and forest and walks the same rank buckets; per
 * bucket it maps only its own records (sheep_ls_map), the caller all-gathers the packed
 * contributions (sheep_ls_pack) of all ranks over RCCL, and every rank applies the union
 * (sheep_ls_apply).  Replaces the per-rank JTree + mpi_merge (jnode.cpp:213-250) reduce; the
 * result equals the serial tree (the etree is unique).  Call sequence per rank:
 *   sheep_ls_begin   this shard's records -> hi-binned items; bin bounds come from the GLOBAL
 *                    degrees d_deg (after the degree all-reduce), so they agree on every rank;
 *                    bin_counts_out (host, >= 512 words) receives this shard's records per bin
 *                    and *n_bins_out their number.  Synchronises.  *handle_out owns the state.
 *   sheep_ls_plan    with the bin counts summed over ranks: *n_buckets_out buckets and the
 *                    mark slots S of a contribution (host only).
 *   per bucket k:    sheep_ls_map(k, d_send) maps into d_send (>= S + m u64); this rank's
 *                    kept-pair count goes to d_count (device int64, nullable; enqueue only)
 *                    and/or *n_kept_out (host, nullable; synchronises); cap = max over ranks;
 *                    sheep_ls_pack(k, d_send, cap) lays out S + cap u64 (d_send must hold
 *                    them: cap may exceed this shard's m);
 *                    [all-gather of d_send[0, S + cap) from every rank into d_recv];
 *                    sheep_ls_apply(k, d_recv, P, cap).
 *                    Order: sheep_ls_map(k + 1) is called after sheep_ls_apply(k) has been
 *                    called (it may run while that apply runs): the apply of bucket k picks
 *                    the giant's anchor of map k + 1 on the device, and the map waits for it.
 *   sheep_ls_finish  d_parent (n_seq, identical on every rank) and d_pst (n_seq) of THIS
 *                    shard's records from its own degrees d_deg / d_selfc (sum over ranks =
 *                    the tree's pst_weight).  Synchronises.
 *   sheep_ls_free    releases the state.
 * Split apply (optional, P >= 2; sheep_ls_split(handle, rank, P) once, before the first map):
 * the spine and zipper of bucket k run only on rank k mod P; every rank still applies the
 * union-find part, so the maps stay exact.  sheep_ls_finish then gives in d_parent only the
 * forest edges of this rank's buckets (INVALID elsewhere); the ranks' forests are disjoint, so
 * the caller's sum over ranks of (d_parent + 1) (u32, wrapping) is the tree's parent + 1. */
int sheep_ls_split(void* handle, uint32_t rank, uint32_t n_ranks);
int sheep_ls_begin(const uint32_t* d_uv, uint64_t m, const uint32_t* d_rank, uint32_t n_rank,
                   const uint32_t* d_seq, uint32_t n_seq, const uint32_t* d_deg,
                   uint64_t* bin_counts_out, uint32_t* n_bins_out, void** handle_out,
                   void* stream);
int sheep_ls_plan(void* handle, const uint64_t* global_bin_counts, uint32_t* n_buckets_out,
                  uint32_t* mark_slots_out);
int sheep_ls_map(void* handle, uint32_t k, uint64_t* d_send, int64_t* d_count,
                 uint32_t* n_kept_out, void* stream);
int sheep_ls_pack(void* handle, uint32_t k, uint64_t* d_send, uint32_t cap, void* stream);
int sheep_ls_apply(void* handle, uint32_t k, const uint64_t* d_recv, uint32_t n_ranks,
                   uint32_t cap, void* stream);
int sheep_ls_finish(void* handle, const uint32_t* d_seq, const uint32_t* d_deg,
                    const uint32_t* d_selfc, int degree_mode, uint32_t* d_parent, uint32_t* d_pst,
                    void* stream);
int sheep_ls_free(void* handle);

/* ---- multi-GPU graph2tree -i -r over RCCL (graph2tree.cpp:134-201) ------------------------
 * One process per GPU.  The communicator replaces MPI_Init / MPI_COMM_WORLD
 * (graph2tree.cpp:134-143): rank 0 makes an id, the caller hands its 128 bytes to every rank
 * (a file, a socket, torch.distributed: the library does not care), and every rank joins with
 * sheep_comm_init on its current device.  The collective calls below must then be made by
 * every rank, in the same order; a failing rank leaves the others waiting, as with MPI. */
#define SHEEP_COMM_ID_BYTES 128
int sheep_comm_unique_id(uint8_t* id_out);
int sheep_comm_init(const uint8_t* id, int n_ranks, int rank);
/* The same group through host shared memory instead of RCCL (name: a POSIX shm name "/..."
 * that every rank passes; rank 0 creates it): the collectives are staged on the host, so P
 * processes can share one GPU.  For rehearsing the multi-process driver where RCCL cannot run
 * (it refuses two ranks on one device); not a transport for real runs. */
int sheep_comm_init_host(const char* name, int n_ranks, int rank);
int sheep_comm_free(void);
int sheep_comm_info(int* rank, int* n_ranks);

/* mpiSequence (sequence.h:65-93): this rank's records (host), the id spaces MAX-reduced
 * (:72), the degrees SUM-reduced (:78), then the same degree sequence on every rank.  seq_out
 * holds seq_cap ids; -ERANGE (with *n_seq_out set) if the sequence is longer. */
int sheep_mpi_sequence(const uint32_t* edges_uv, uint64_t m, uint32_t n_ids, int degree_mode,
                       uint32_t* seq_out, uint32_t seq_cap, uint32_t* n_seq_out);

/* JTree over this rank's records + JNodeTable::mpi_merge (jtree.h:111-136, jnode.cpp:213-250):
 * the elimination tree of the UNION of every rank's records under seq (the same seq on every
 * rank, e.g. from sheep_mpi_sequence).  Every rank receives the whole tree (parent) and the
 * summed pst_weight (n_seq entries each); rank 0's is what graph2tree -r saves. */
int sheep_build_tree_multi(const uint32_t* edges_uv, uint64_t m, const uint32_t* seq,
                           uint32_t n_seq, uint32_t* parent_out, uint32_t* pst_out);

/* JNodeTable::mpi_merge (jnode.cpp:213-250), in place on host arrays: the partial trees of all
 * ranks (the same n jnodes, the same seq) -> etree of their union on every rank, pst summed. */
int sheep_mpi_merge(uint32_t* parent, uint32_t* pst, uint32_t n);

/* The whole graph2tree -i -r on device memory: this rank's m records (d_uv), ids < n_ids (the
 * global id space, the same on every rank) -> seq (n_ids entries), parent and pst (n_ids
 * entries, n_seq used) on every rank.  No partial trees: the ranks walk one bucketed tree
 * build together, each mapping its own records and applying the kept pairs of all
 * (DESIGN.md §6).  Synchronises the stream. */
int sheep_graph2tree_multi_dev(const uint32_t* d_uv, uint64_t m, uint32_t n_ids, int degree_mode,
                               uint32_t* d_seq, uint32_t* d_parent, uint32_t* d_pst,
                               uint32_t* n_seq_out, void* stream);

/* The same driver for n_ranks shards held by ONE process on the current device, one thread
 * per rank, the collectives done as device copies (the one-device rehearsal of the P-GPU path;
 * tests).  Rank 0's seq/parent/pst are returned; -EIO if any rank's replica differs. */
int sheep_graph2tree_multi_local(const uint32_t* const* d_uv, const uint64_t* m, uint32_t n_ranks,
                                 uint32_t n_ids, int degree_mode, uint32_t* d_seq,
                                 uint32_t* d_parent, uint32_t* d_pst, uint32_t* n_seq_out);

/* Partition quality of a k-way vertex partition (Partition::evaluate(graph) and
 * evaluate(graph, seq), partition.cpp:428-521) over the m edge records in HBM, counted on
 * LLAMA's undirected adjacency as the reference does.  d_parts: n_ids int16 parts (every id
 * with an edge needs one in [0, n_parts)); d_rank: n_ids positions in seq (sheep_sequence_dev).
 * out (host, 11 words): edges cut, Vcom vol, vertex balance (max), ECV(hash), its balance,
 * ECV(down), its balance, ECV(up), its balance, edges (adjacency entries / 2), nodes.
 * Synchronises.  -ERANGE: an id, part or position out of range; -EINVAL: n_parts outside
 * [1, 32768] or 2m >= 2^32. */
int sheep_evaluate_dev(const uint32_t* d_uv, uint64_t m, const int16_t* d_parts,
                       const uint32_t* d_rank, uint32_t n_ids, uint32_t n_parts, uint64_t* out,
                       void* stream);

/* Host-pointer sheep_evaluate_dev, as Partition::evaluate(graph, seq) calls it: parts are
 * n_parts_vid int16 per vertex id (ids beyond it have no part), seq the n_seq ids in sequence
 * order.  Uploads, evaluates, synchronises. */
int sheep_evaluate(const uint32_t* edges_uv, uint64_t m, const int16_t* parts, uint32_t n_parts_vid,
                   const uint32_t* seq, uint32_t n_seq, uint32_t n_parts, uint64_t* out);

/* graph2tree -p K -o OUT's edge output (Partition::writePartitionedGraph, partition.cpp:588-630)
 * on the GPU: every record (X, Y), X < Y after ordering its endpoints, self-loops skipped,
 * assigned to the part of its lower-sequence endpoint; d_out (2m u32) receives the (X, Y)
 * pairs grouped by part, each part in the host writer's order (X ascending, then record
 * order); part_start (host, n_parts + 1) the first pair of each part (part_start[n_parts] = the
 * number written).  d_parts / d_rank: n_ids int16 parts and positions in seq.  Synchronises.
 * -ERANGE: an id outside the sequence, or an endpoint without a part in [0, n_parts). */
int sheep_partition_edges_dev(const uint32_t* d_uv, uint64_t m, const int16_t* d_parts,
                              const uint32_t* d_rank, uint32_t n_ids, uint32_t n_parts,
                              uint32_t* d_out, uint64_t* part_start, void* stream);
/* The same from host arrays (parts: n_parts_vid int16 per id, seq: n_seq ids), out_uv: 2m u32. */
int sheep_partition_edges(const uint32_t* edges_uv, uint64_t m, const int16_t* parts,
                          uint32_t n_parts_vid, const uint32_t* seq, uint32_t n_seq, uint32_t n_parts,
                          uint32_t* out_uv, uint64_t* part_start);

/* The whole single-device hot path: degree -> sequence -> tree (graph2tree's Sorted+Mapped).
 * d_seq holds n_ids entries, d_parent/d_pst hold n_ids entries (n_seq used).  Synchronises. */
int sheep_graph2tree_dev(const uint32_t* d_uv, uint64_t m, uint32_t n_ids, int degree_mode,
                         uint32_t* d_seq, uint32_t* d_parent, uint32_t* d_pst,
                         uint32_t* n_seq_out, void* stream);

/* Synthetic R-MAT records [e_begin, e_end) of the stream (scale, seed) into d_uv
 * (2*(e_end-e_begin) u32).  Bit-identical to sheep_amd/csrc/rmat.h on the host.  Enqueue only. */
int sheep_rmat_dev(uint32_t* d_uv, int scale, uint64_t seed, uint64_t e_begin, uint64_t e_end,
                   void* stream);

/* Power-law (Chung-Lu style) synthetic records [e_begin, e_end) for the LiveJournal- and
 * twitter-shape configs: endpoints drawn with P(i) ~ (i + i0)^(-1/(gamma-1)) over n ids, then
 * relabelled by a seeded bijection.  Bit-identical to sheep_amd/csrc/powerlaw.h on the host.
 * Enqueue only. */
int sheep_powerlaw_dev(uint32_t* d_uv, uint32_t n, double gamma, double i0, uint64_t seed,
                       uint64_t e_begin, uint64_t e_end, void* stream);

/* ---- host-side partition (the reference keeps it on the host) ---------------------------- */

/* Partition(seq, jnodes, k, balance, false, true, false) (partition.cpp:50-67 ->
 * forwardPartition :86-157, pst weights) for each k of ks[0..n_k) in turn on ONE table, as
 * partition_tree does (partition_tree.cpp:130-146): the kids lists that one k sorts in place
 * are the starting order of the next.  parent/pst: the n_seq jnodes; seq: the n_seq ids;
 * parts_out: n_k * n_vid int16, vid-indexed (-1 = INVALID_PART for ids not in seq), n_vid >=
 * max(seq) + 1; created_out (nullable): n_k part counts ("Actually created").  Host only. */
int sheep_partition(const uint32_t* parent, const uint32_t* pst, uint32_t n_seq,
                    const uint32_t* seq, const int32_t* ks, uint32_t n_k, double balance,
                    int16_t* parts_out, uint32_t n_vid, uint32_t* created_out);

/* Kernel timing of the last synchronising call (ms per named phase), for bench/profiling.
 * Fills up to cap (name, ms) pairs; returns the count. */
int sheep_last_timings(const char** names, double* ms, int cap);

#ifdef __cplusplus
}
#endif
#endif /* SHEEP_AMD_H */
