// =====================================================================================
// sheep_oracle — CPU restatement of the Sheep hot path.  TEST INFRASTRUCTURE ONLY.
//
// This file is the parity CHECKER for the MI355X build.  Only tests/, __graft_entry__.smoke()
// and bench.py's cpu_baseline leg may load it.  The product library (libsheep_amd.so) never
// links, loads or calls it; the product fails loudly when its HIP code object is missing.
//
// It restates, from a reading of the reference sources (arpang/sheep, /root/reference), the
// semantics of every function on the hot path.  Each function cites the file:line it follows.
// It is a clean-room restatement, not a copy: the reference cannot be compiled here (it needs
// MPI and the un-vendored LLAMA library, see DESIGN.md "Oracle"), so the oracle is pinned by
// the reference's own published fixtures (data/hep-th.dat with data/quality/hep.degree.raw and
// data/quality/hep.cost) and a hand-checked known-answer graph (tests/golden/).
//
// Written in C++ (g++) rather than C for one reason: Partition::forwardPartition orders kids
// with libstdc++'s unstable std::sort (partition.cpp:104-106); bit-exact partition parity needs
// the same std::sort called on the same ranges in the same order.
// =====================================================================================
#include <algorithm>
#include <chrono>
#include <cerrno>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <numeric>
#include <unordered_set>
#include <thread>
#include <vector>

#include "../sheep_amd/csrc/rmat.h"  // the build's synthetic-input definition (not reference code)
#include "../sheep_amd/csrc/powerlaw.h"  // likewise, the power-law configs

typedef uint32_t vid_t;   // defs.h:76
typedef uint32_t jnid_t;  // jnode.h:42
typedef int16_t part_t;   // partition.h:43
static const uint32_t INVALID = 0xFFFFFFFFu;  // defs.h:82, jnode.h:43
static const part_t INVALID_PART = -1;        // partition.h:44

extern "C" {

// ----------------------------------------------------------------------------------------
// Edge-file readers.
// ----------------------------------------------------------------------------------------

// XS1 records are {u32 tail, u32 head, f32 weight} (readerwriter.h:36-40).
// LLAMA's .dat loader (graph2tree's path, graph_wrapper.h:43-63) takes every complete record;
// the published Σpst of com-lj/orkut/amazon equals their edge counts, so it does NOT repeat
// the last record.  Returns the record count; fills uv (2 u32 per record) if given.
uint64_t orc_read_dat(const char* path, uint32_t* uv, uint64_t cap) {
  FILE* f = fopen(path, "rb");
  if (!f) return (uint64_t)-1;
  uint32_t rec[3];
  uint64_t n = 0;
  while (fread(rec, 12, 1, f) == 1) {
    if (uv && n < cap) { uv[2 * n] = rec[0]; uv[2 * n + 1] = rec[1]; }
    ++n;
  }
  fclose(f);
  return n;
}

// XS1Reader::read (readerwriter.h:50-58) checks eof() BEFORE read(): after the last record the
// next read fails, sets eof, and still returns true with the stale buffer.  So the FILE-mode
// stream (fileSequence_template, sequence.h:95-122) sees the last record twice.  For an empty
// file the reference returns an uninitialised buffer; we return no records (documented).
uint64_t orc_read_dat_xs1reader(const char* path, uint32_t* uv, uint64_t cap) {
  uint64_t n = orc_read_dat(path, uv, cap);
  if (n == (uint64_t)-1 || n == 0) return n;
  if (uv && n < cap) { uv[2 * n] = uv[2 * (n - 1)]; uv[2 * n + 1] = uv[2 * (n - 1) + 1]; }
  return n + 1;
}

// SNAPReader::read (readerwriter.h:84-89): `stream >> X` then `stream >> Y`; stops at the first
// token that does not parse as an unsigned (e.g. a '#' comment line ends the stream).
uint64_t orc_read_net(const char* path, uint32_t* uv, uint64_t cap) {
  std::ifstream s(path);
  if (!s) return (uint64_t)-1;
  uint64_t n = 0;
  uint32_t x, y;
  while (true) {
    bool ok = (bool)(s >> x);
    ok &= (bool)(s >> y);
    if (!ok) break;
    if (uv && n < cap) { uv[2 * n] = x; uv[2 * n + 1] = y; }
    ++n;
  }
  return n;
}

// ----------------------------------------------------------------------------------------
// Degrees and the degree sequence.
// ----------------------------------------------------------------------------------------

// mode 0 = LLAMA (graph_wrapper.h:87-89, undirected-double CSR, a self-loop stored once);
// mode 1 = FILE  (sequence.h:101-107, degree[X]++ and degree[Y]++, so a self-loop counts 2).
// deg must hold n_ids zeroed-or-not entries; it is overwritten.  Returns max id + 1 seen
// (0 for no records), or -ERANGE as (uint32)-1 if an id >= n_ids.
int64_t orc_degree(const uint32_t* uv, uint64_t m, int mode, uint32_t* deg, uint32_t n_ids) {
  std::fill(deg, deg + n_ids, 0u);
  int64_t top = 0;
  for (uint64_t e = 0; e < m; ++e) {
    uint32_t t = uv[2 * e], h = uv[2 * e + 1];
    if (t >= n_ids || h >= n_ids) return -ERANGE;
    top = std::max<int64_t>(top, (int64_t)std::max(t, h) + 1);
    deg[t] += 1;
    if (mode == 1 || t != h) deg[h] += 1;
  }
  return top;
}

// degreeSequence / mpiSequence / fileSequence_template (sequence.h:52-63, :65-93, :95-122):
// the ids with deg>0, ordered by (deg ascending, id ascending).  Returns n_seq.
uint32_t orc_sequence(const uint32_t* deg, uint32_t n_ids, uint32_t* seq_out) {
  uint32_t n = 0;
  for (uint32_t v = 0; v < n_ids; ++v)
    if (deg[v] != 0) seq_out[n++] = v;
  std::sort(seq_out, seq_out + n, [deg](uint32_t a, uint32_t b) {
    return deg[a] != deg[b] ? deg[a] < deg[b] : a < b;
  });
  return n;
}

// ----------------------------------------------------------------------------------------
// The tree: JNodeTable + FastUnionFind + JTree::insert.
// ----------------------------------------------------------------------------------------

// FastUnionFind (unionfind.h:39-103): union by rank, path compression, and the set ROOT's
// parent slot holds the set's label (the current elimination-tree root = max jnid in the set).
struct UF {
  std::vector<uint32_t> par;
  std::vector<uint8_t> rank;
  explicit UF(uint32_t n) : par(n), rank(n, 0) { std::iota(par.begin(), par.end(), 0u); }
  uint32_t find_root(uint32_t e) {  // unionfind.h:46-63
    uint32_t it = e;
    while (rank[it] < rank[par[it]]) it = par[it];
    uint32_t root = it;
    it = e;
    while (it != root) { uint32_t nx = par[it]; par[it] = root; it = nx; }
    return root;
  }
  uint32_t unify(uint32_t lesser, uint32_t greater) {  // unionfind.h:82-102
    uint32_t gr = find_root(greater), lr = find_root(lesser);
    uint32_t old_label = par[lr];
    if (lr != gr) {
      if (rank[lr] > rank[gr]) { par[lr] = greater; par[gr] = lr; }
      else { par[lr] = gr; if (rank[lr] == rank[gr]) rank[gr] += 1; }
    }
    return old_label;
  }
};

// JNodeTable::adopt (jnode.h:158-162).
static inline void adopt(UF& uf, uint32_t* parent, uint32_t kid, uint32_t id) {
  uint32_t label = uf.unify(kid, id);
  if (label != id) parent[label] = id;
}

// Undirected-double CSR as LLAMA presents it to JTree (graph_wrapper.h:43-63, 128-158):
// record (t,h) adds t->h, and h->t only when t != h; neighbour order = record order.
struct CSR {
  std::vector<uint64_t> off;
  std::vector<uint32_t> adj;
};
static CSR build_csr(const uint32_t* uv, uint64_t m, uint32_t n_ids) {
  CSR g;
  g.off.assign((size_t)n_ids + 1, 0);
  for (uint64_t e = 0; e < m; ++e) {
    uint32_t t = uv[2 * e], h = uv[2 * e + 1];
    g.off[t + 1]++;
    if (t != h) g.off[h + 1]++;
  }
  for (uint32_t v = 0; v < n_ids; ++v) g.off[v + 1] += g.off[v];
  g.adj.resize(g.off[n_ids]);
  std::vector<uint64_t> pos(g.off.begin(), g.off.end() - 1);
  for (uint64_t e = 0; e < m; ++e) {
    uint32_t t = uv[2 * e], h = uv[2 * e + 1];
    g.adj[pos[t]++] = h;
    if (t != h) g.adj[pos[h]++] = t;
  }
  return g;
}

// JTree(graph, seq) with default Options (jtree.h:111-122, 88-90: make_pad=true) runs the
// parameterised insertSequence (jtree.cpp:112-145; opts.isDefault() is false because
// width_limit defaults to (size_t)-1, jtree.h:89 vs :96) whose per-vertex body is
// insert(graph, X, opts) (jtree.cpp:65-110) with make_kids/pst/jxn off:
//   current = newJNode()                       (parent=INVALID, pst=0; jnode.h:107-111)
//   for nbr in adj(X): nbr_id = index.at(nbr)   (std::out_of_range if nbr > max(seq))
//     nbr_id valid  -> adopt(nbr_id, current)   (PREORDER edge)
//     else nbr != X -> ++pst_weight(current)    (POSTORDER edge)
//   index[X] = current                          (assert: X not already inserted, jtree.h:165-168)
// Returns 0, -ERANGE (index.at throw), -EINVAL (duplicate id in seq: the assert).
int orc_build_tree(const uint32_t* uv, uint64_t m, const uint32_t* seq, uint32_t n_seq,
                   uint32_t* parent, uint32_t* pst) {
  if (n_seq == 0) return 0;
  uint32_t max_seq = *std::max_element(seq, seq + n_seq);
  uint32_t n_ids = max_seq + 1;
  for (uint64_t e = 0; e < 2 * m; ++e) n_ids = std::max(n_ids, uv[e] + 1);
  CSR g = build_csr(uv, m, n_ids);
  std::vector<uint32_t> index((size_t)max_seq + 1, INVALID);
  UF uf(n_seq);
  for (uint32_t cur = 0; cur < n_seq; ++cur) {
    uint32_t X = seq[cur];
    parent[cur] = INVALID;
    pst[cur] = 0;
    for (uint64_t k = g.off[X]; k < g.off[X + 1]; ++k) {
      uint32_t nbr = g.adj[k];
      if (nbr > max_seq) return -ERANGE;
      uint32_t nid = index[nbr];
      if (nid != INVALID) adopt(uf, parent, nid, cur);
      else if (nbr != X) ++pst[cur];
    }
    if (index[X] != INVALID) return -EINVAL;
    index[X] = cur;
  }
  return 0;
}

// JNodeTable::makeKids (jnode.h:190-204): kids listed in ascending jnid order.
struct Kids {
  std::vector<uint64_t> off;
  std::vector<uint32_t> ids;
};
static Kids make_kids(const uint32_t* parent, uint32_t n) {
  Kids k;
  k.off.assign((size_t)n + 1, 0);
  for (uint32_t v = 0; v < n; ++v)
    if (parent[v] != INVALID) k.off[parent[v] + 1]++;
  for (uint32_t v = 0; v < n; ++v) k.off[v + 1] += k.off[v];
  k.ids.resize(k.off[n]);
  std::vector<uint64_t> pos(k.off.begin(), k.off.end() - 1);
  for (uint32_t v = 0; v < n; ++v)
    if (parent[v] != INVALID) k.ids[pos[parent[v]]++] = v;
  return k;
}

// JNodeTable::merge (jnode.cpp:174-201) with make_kids=false: for current in ascending order,
// adopt every kid of current in lhs, then in rhs, summing pst (u32, wraps).  Both inputs are
// tables loaded from .tre files, so their kids come from makeKids (jnode.cpp:101, 104-110).
int orc_merge(const uint32_t* pa, const uint32_t* sa, const uint32_t* pb, const uint32_t* sb,
              uint32_t n, uint32_t* parent, uint32_t* pst) {
  Kids ka = make_kids(pa, n), kb = make_kids(pb, n);
  UF uf(n);
  for (uint32_t cur = 0; cur < n; ++cur) {
    parent[cur] = INVALID;
    pst[cur] = 0;
    for (uint64_t i = ka.off[cur]; i < ka.off[cur + 1]; ++i) adopt(uf, parent, ka.ids[i], cur);
    pst[cur] += sa[cur];
    for (uint64_t i = kb.off[cur]; i < kb.off[cur + 1]; ++i) adopt(uf, parent, kb.ids[i], cur);
    pst[cur] += sb[cur];
  }
  return 0;
}

// JNodeTable::Facts (jnode.cpp:256-290).  width(id) = 1 + pst_weight (jnode.h:258-260, no jxn).
// out = {width, roots, vheight, eheight, verts, edges, halo, core, fill}; halo/core INVALID->2^32-1.
void orc_facts(const uint32_t* parent, const uint32_t* pst, uint32_t n, uint64_t* out) {
  std::vector<uint64_t> vh(n, 0), eh(n, 0);
  uint64_t verts = 0, edges = 0, width = 0, fill = 0, vheight = 0, eheight = 0, roots = 0;
  uint32_t halo = INVALID, core = INVALID;
  for (uint32_t id = 0; id < n; ++id) {
    uint64_t w = 1 + (uint64_t)pst[id];
    verts++;
    edges += pst[id];
    width = std::max(width, w);
    fill += w - pst[id] - 1;
    vh[id]++;
    eh[id] += pst[id];
    uint32_t p = parent[id];
    if (p != INVALID) {
      vh[p] = std::max(vh[p], vh[id]);
      eh[p] = std::max(eh[p], eh[id]);
    } else {
      vheight = std::max(vheight, vh[id]);
      eheight = std::max(eheight, eh[id]);
      roots++;
    }
    if (halo == INVALID && w > 3) halo = id;
    if (core == INVALID && w >= width) core = id;
  }
  out[0] = width; out[1] = roots; out[2] = vheight; out[3] = eheight; out[4] = verts;
  out[5] = edges; out[6] = halo; out[7] = core; out[8] = fill;
}

// ----------------------------------------------------------------------------------------
// Partition (forwardPartition) and evaluation.
// ----------------------------------------------------------------------------------------

// A tree loaded for partitioning (partition_tree.cpp:105, JNodeTable(file) -> makeKids).  The
// kids lists are sorted IN PLACE by forwardPartition and stay sorted for the next k of the
// same partition_tree run (partition_tree.cpp:130-146), so the handle carries them.
struct PartTree {
  std::vector<uint32_t> parent, pst;
  Kids kids;
};

void* orc_parttree_new(const uint32_t* parent, const uint32_t* pst, uint32_t n) {
  PartTree* t = new PartTree;
  t->parent.assign(parent, parent + n);
  t->pst.assign(pst, pst + n);
  t->kids = make_kids(parent, n);
  return t;
}
void orc_parttree_free(void* h) { delete (PartTree*)h; }

// Partition::Partition + forwardPartition (partition.cpp:50-67, 86-157), pst weighting
// (partition_tree.cpp:95-96: with no -x/-d/-u flag, pst_weight=true), balance factor b.
// parts_vid (size n_vid = max(seq)+1) receives vid-indexed parts (INVALID_PART for ids not
// in seq).  Returns the number of bins opened.
int orc_partition(void* h, const uint32_t* seq, uint32_t n_seq, int k, double balance,
                  int16_t* parts_vid, uint32_t n_vid) {
  PartTree& t = *(PartTree*)h;
  uint32_t n = (uint32_t)t.parent.size();
  std::vector<part_t> parts(n, INVALID_PART);
  size_t total = 0;
  for (uint32_t id = 0; id < n; ++id) total += t.pst[id];
  size_t max_component = (size_t)((total / (part_t)k) * balance);
  std::vector<size_t> part_size;
  std::vector<size_t> below(n, 0);
  for (uint32_t id = 0; id < n; ++id) {
    below[id] += t.pst[id];
    if (below[id] > max_component) {
      uint32_t* kb = t.kids.ids.data() + t.kids.off[id];
      uint32_t* ke = t.kids.ids.data() + t.kids.off[id + 1];
      std::sort(kb, ke, [&below](uint32_t l, uint32_t r) { return below.at(l) > below.at(r); });
      do {
        for (uint32_t* it = kb; below[id] > max_component && it != ke; ++it) {
          uint32_t kid = *it;
          if (parts[kid] != INVALID_PART) continue;
          for (part_t cp = 0; cp != (part_t)part_size.size(); ++cp) {
            if (part_size[cp] + below[kid] <= max_component) {
              below[id] -= below[kid];
              part_size[cp] += below[kid];
              parts[kid] = cp;
              break;
            }
          }
        }
        if (below[id] > max_component) part_size.push_back(0);
      } while (below[id] > max_component);
    }
    if (t.parent[id] != INVALID) below[t.parent[id]] += below[id];
  }
  for (uint32_t id = n - 1; id != (uint32_t)-1; --id) {
    if (parts[id] == INVALID_PART && t.parent[id] != INVALID) parts[id] = parts[t.parent[id]];
    while (parts[id] == INVALID_PART) {
      for (part_t cp = (part_t)part_size.size() - 1; cp != -1; --cp) {
        if (part_size[cp] + below[id] <= max_component) {
          part_size[cp] += below[id];
          parts[id] = cp;
          break;
        }
      }
      if (parts[id] == INVALID_PART) part_size.push_back(0);
    }
  }
  // jnid-indexed -> vid-indexed (partition.cpp:63-66).
  std::fill(parts_vid, parts_vid + n_vid, INVALID_PART);
  for (uint32_t i = 0; i < n_seq; ++i) parts_vid[seq[i]] = parts[i];
  return (int)part_size.size();
}

static inline uint32_t cormen_hash(uint32_t k) {  // partition.cpp:420-424
  double A = 0.5 * (sqrt(5) - 1);
  uint32_t s = (uint32_t)floor(A * pow(2, 32));
  return k * s;
}

// Partition::evaluate(graph) + evaluate(graph, seq) (partition.cpp:428-473, 475-521) over the
// LLAMA adjacency.  out (u64[16]) = {edges_cut, vcom_vol, max_vertex_bal, ecv_hash,
// max_hash_bal, ecv_down, max_down_bal, ecv_up, max_up_bal, getEdges, getNodes}.
// Returns 0, or -EINVAL when a vertex of the graph has no part (the reference asserts).
int orc_evaluate(const uint32_t* uv, uint64_t m, const int16_t* parts_vid, uint32_t n_vid,
                 const uint32_t* seq, uint32_t n_seq, uint64_t* out) {
  uint32_t n_ids = 0;
  for (uint64_t e = 0; e < 2 * m; ++e) n_ids = std::max(n_ids, uv[e] + 1);
  CSR g = build_csr(uv, m, n_ids);
  part_t maxp = *std::max_element(parts_vid, parts_vid + n_vid);
  std::vector<uint64_t> vbal(maxp + 1, 0), hbal(maxp + 1, 0), dbal(maxp + 1, 0), ubal(maxp + 1, 0);
  std::vector<uint32_t> pos(n_vid, INVALID);
  for (uint32_t i = 0; i < n_seq; ++i) pos[seq[i]] = i;
  uint64_t cut = 0, vcom = 0, ecvh = 0, ecvd = 0, ecvu = 0, nodes = 0;
  for (uint32_t X = 0; X < n_ids; ++X) {
    if (g.off[X + 1] == g.off[X]) continue;
    nodes++;
    if (X >= n_vid || parts_vid[X] == INVALID_PART) return -EINVAL;
    part_t xp = parts_vid[X];
    uint32_t xpos = pos[X];
    vbal[xp] += 1;
    std::unordered_set<part_t> vs = {xp}, hs, ds, us;
    for (uint64_t k = g.off[X]; k < g.off[X + 1]; ++k) {
      uint32_t Y = g.adj[k];
      if (Y >= n_vid || parts_vid[Y] == INVALID_PART) return -EINVAL;
      part_t yp = parts_vid[Y];
      uint32_t ypos = pos[Y];
      if (X < Y && xp != yp) ++cut;
      vs.insert(yp);
      part_t hp = cormen_hash(X) < cormen_hash(Y) ? xp : yp;
      hs.insert(hp);
      if (X < Y) hbal[hp] += 1;
      ds.insert(xpos < ypos ? xp : yp);
      us.insert(xpos > ypos ? xp : yp);
      if (xpos < ypos) dbal[xp] += 1;
      if (xpos > ypos) ubal[xp] += 1;
    }
    vcom += vs.size() - 1;
    ecvh += hs.size() - 1;
    ecvd += ds.size() - 1;
    ecvu += us.size() - 1;
  }
  out[0] = cut; out[1] = vcom; out[2] = *std::max_element(vbal.begin(), vbal.end());
  out[3] = ecvh; out[4] = *std::max_element(hbal.begin(), hbal.end());
  out[5] = ecvd; out[6] = *std::max_element(dbal.begin(), dbal.end());
  out[7] = ecvu; out[8] = *std::max_element(ubal.begin(), ubal.end());
  out[9] = g.adj.size() / 2; out[10] = nodes;
  return 0;
}

// CPU baseline timing (bench.py cpu_baseline leg): the reference's timed window is
// "Sorted in" + "Mapped in" (graph2tree.cpp:169-193) with the graph already loaded into
// LLAMA's CSR (load excluded).  So: build the CSR untimed, then time (a) degrees from the CSR
// + the (deg, id) sort (degreeSequence, sequence.h:52-63) and (b) the JTree map
// (jtree.cpp:112-145 with FastUnionFind).  Single thread.  out = {sort_s, map_s, n_seq}.
int orc_time_graph2tree(const uint32_t* uv, uint64_t m, uint32_t n_ids, double* out) {
  CSR g = build_csr(uv, m, n_ids);
  auto t0 = std::chrono::steady_clock::now();
  std::vector<uint32_t> seq;
  seq.reserve(n_ids);
  for (uint32_t v = 0; v < n_ids; ++v)
    if (g.off[v + 1] != g.off[v]) seq.push_back(v);
  std::sort(seq.begin(), seq.end(), [&g](uint32_t a, uint32_t b) {
    uint64_t da = g.off[a + 1] - g.off[a], db = g.off[b + 1] - g.off[b];
    return da != db ? da < db : a < b;
  });
  auto t1 = std::chrono::steady_clock::now();
  uint32_t n = (uint32_t)seq.size();
  std::vector<uint32_t> index(n_ids, INVALID), parent(n), pst(n);
  UF uf(n);
  for (uint32_t cur = 0; cur < n; ++cur) {
    uint32_t X = seq[cur];
    parent[cur] = INVALID;
    pst[cur] = 0;
    for (uint64_t k = g.off[X]; k < g.off[X + 1]; ++k) {
      uint32_t nid = index[g.adj[k]];
      if (nid != INVALID) adopt(uf, parent.data(), nid, cur);
      else if (g.adj[k] != X) ++pst[cur];
    }
    index[X] = cur;
  }
  auto t2 = std::chrono::steady_clock::now();
  out[0] = std::chrono::duration<double>(t1 - t0).count();
  out[1] = std::chrono::duration<double>(t2 - t1).count();
  out[2] = n;
  volatile uint32_t sink = parent.empty() ? 0 : parent[n / 2];
  (void)sink;
  return 0;
}

// The `mpirun -n T graph2tree -ir` analogue (graph2tree.cpp:134-200) on T threads, the
// reference's multi-core CPU path, for bench.py's cpu_baseline: T contiguous record shards
// (-l i/T, graph_wrapper.h:48-49), each loaded as its own CSR (untimed, as LLAMA's load);
// timed: "Sorted" = shard degrees + their sum (mpiSequence's MPI_Allreduce, sequence.h:65-93)
// + the (deg, id) sort; "Mapped" = each shard's JTree on its thread (jtree.cpp:112-145);
// "Reduced" = the partial trees merged pairwise in log2(T) rounds, the pairs of a round on
// parallel threads (mpi_merge's reduce tree, jnode.cpp:203-250).  Checks that the result is
// the serial tree's.  out = {sort_s, map_s, reduce_s, n_seq, ok}.
int orc_time_graph2tree_ir(const uint32_t* uv, uint64_t m, uint32_t n_ids, int T, double* out) {
  if (T < 1) T = 1;
  std::vector<CSR> g(T);
  {
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t)
      th.emplace_back([&, t] {
        uint64_t lo = m * t / T, hi = m * (t + 1) / T;
        g[t] = build_csr(uv + 2 * lo, hi - lo, n_ids);
      });
    for (auto& x : th) x.join();
  }
  auto t0 = std::chrono::steady_clock::now();
  // Sorted: degrees of every shard, summed by id range on the T threads, then the sort
  std::vector<uint32_t> deg(n_ids, 0);
  {
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t)
      th.emplace_back([&, t] {
        uint64_t lo = (uint64_t)n_ids * t / T, hi = (uint64_t)n_ids * (t + 1) / T;
        for (int s = 0; s < T; ++s)
          for (uint64_t v = lo; v < hi; ++v) deg[v] += (uint32_t)(g[s].off[v + 1] - g[s].off[v]);
      });
    for (auto& x : th) x.join();
  }
  std::vector<uint32_t> seq;
  seq.reserve(n_ids);
  for (uint32_t v = 0; v < n_ids; ++v)
    if (deg[v]) seq.push_back(v);
  auto less = [&deg](uint32_t a, uint32_t b) { return deg[a] != deg[b] ? deg[a] < deg[b] : a < b; };
  {  // T sorted runs, then pairwise merges (what __gnu_parallel::sort does with T threads)
    std::vector<size_t> cut(T + 1);
    for (int t = 0; t <= T; ++t) cut[t] = seq.size() * t / T;
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t)
      th.emplace_back([&, t] { std::sort(seq.begin() + cut[t], seq.begin() + cut[t + 1], less); });
    for (auto& x : th) x.join();
    for (int w = 1; w < T; w *= 2) {
      std::vector<std::thread> mt;
      for (int t = 0; t + w < T; t += 2 * w)
        mt.emplace_back([&, t, w] {
          size_t e = cut[std::min(T, t + 2 * w)];
          std::inplace_merge(seq.begin() + cut[t], seq.begin() + cut[t + w], seq.begin() + e, less);
        });
      for (auto& x : mt) x.join();
    }
  }
  auto t1 = std::chrono::steady_clock::now();
  const uint32_t n = (uint32_t)seq.size();
  std::vector<std::vector<uint32_t>> par(T, std::vector<uint32_t>(n)), ps(T, std::vector<uint32_t>(n));
  {
    std::vector<uint32_t> index(n_ids, INVALID);
    for (uint32_t i = 0; i < n; ++i) index[seq[i]] = i;
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t)
      th.emplace_back([&, t] {
        UF uf(n);
        uint32_t* parent = par[t].data();
        uint32_t* pst = ps[t].data();
        const CSR& c = g[t];
        for (uint32_t cur = 0; cur < n; ++cur) {
          uint32_t X = seq[cur];
          parent[cur] = INVALID;
          pst[cur] = 0;
          for (uint64_t k = c.off[X]; k < c.off[X + 1]; ++k) {
            uint32_t nb = c.adj[k], nid = index[nb];
            if (nid < cur) adopt(uf, parent, nid, cur);
            else if (nid != cur) ++pst[cur];
          }
        }
      });
    for (auto& x : th) x.join();
  }
  auto t2 = std::chrono::steady_clock::now();
  for (int w = 1; w < T; w *= 2) {
    std::vector<std::thread> th;
    for (int t = 0; t + w < T; t += 2 * w)
      th.emplace_back([&, t, w] {
        std::vector<uint32_t> p(n), q(n);
        orc_merge(par[t].data(), ps[t].data(), par[t + w].data(), ps[t + w].data(), n, p.data(), q.data());
        par[t].swap(p);
        ps[t].swap(q);
      });
    for (auto& x : th) x.join();
  }
  auto t3 = std::chrono::steady_clock::now();
  std::vector<uint32_t> sp(n), ss(n);
  int ok = orc_build_tree(uv, m, seq.data(), n, sp.data(), ss.data()) == 0 && sp == par[0] && ss == ps[0];
  out[0] = std::chrono::duration<double>(t1 - t0).count();
  out[1] = std::chrono::duration<double>(t2 - t1).count();
  out[2] = std::chrono::duration<double>(t3 - t2).count();
  out[3] = n;
  out[4] = ok;
  return 0;
}

// Synthetic R-MAT edges [e_begin, e_end) of the stream (scale, seed); see rmat.h.  Used by the
// tests to regenerate on the host exactly what the GPU generator wrote into HBM.
void orc_powerlaw(uint32_t n, double gamma, double i0, uint64_t seed, uint64_t e_begin,
                  uint64_t e_end, uint32_t* uv) {
  const sheep_pl::Table t = sheep_pl::powerlaw_table(n, gamma, i0);
  for (uint64_t e = e_begin; e < e_end; ++e)
    sheep_pl::edge(t, e, seed, &uv[2 * (e - e_begin)], &uv[2 * (e - e_begin) + 1]);
}

void orc_rmat(int scale, uint64_t seed, uint64_t e_begin, uint64_t e_end, uint32_t* uv) {
  for (uint64_t e = e_begin; e < e_end; ++e)
    sheep_rmat::edge(e, scale, seed, &uv[2 * (e - e_begin)], &uv[2 * (e - e_begin) + 1]);
}

}  // extern "C"
