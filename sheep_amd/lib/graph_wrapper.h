// The graph as graph2tree sees it (reference: lib/graph_wrapper.h:36-163, LLAMAGraph).
//
// LLAMA is not part of this build: the graph is the edge stream itself, held as u32 (tail,
// head) pairs (what the GPU consumes), with a lazily built undirected-double CSR for the
// host-side iterators (partition evaluation / partitioned output).  Semantics kept:
//   - .dat loads every complete record (no XS1Reader tail duplication), .net via SNAPReader;
//   - undirected double: record (t,h) is adjacency t->h and h->t, a self-loop is stored once;
//   - duplicates are kept (no DDUP_GRAPH);
//   - partial load part/num_parts (1-based part, graph2tree -l) takes the contiguous record
//     range [R*(p-1)/k, R*p/k) while ids span the whole file (getMaxVid = max id + 1);
//   - getEdges() = adjacency entries / 2 (graph_wrapper.h:79-81).
#pragma once
#include <algorithm>
#include <cstring>
#include <stdexcept>
#include <vector>

#include "defs.h"
#include "readerwriter.h"
#include "sheep_call.h"

class EdgeGraph {
  std::vector<uint32_t> uv_;  // 2 * m
  vid_t max_vid_ = 0;         // max id + 1 over the whole file (over the part, loaded to_device)
  mutable const uint32_t* reg_ = nullptr;  // uv_ registered with the library (one device copy)
  mutable std::vector<uint64_t> off_;
  mutable std::vector<uint32_t> adj_;
  mutable size_t num_nodes_ = 0;

  void build_csr() const {
    if (!off_.empty() || max_vid_ == 0) return;
    size_t m = records();
    off_.assign((size_t)max_vid_ + 1, 0);
    for (size_t e = 0; e < m; ++e) {
      off_[uv_[2 * e] + 1]++;
      if (uv_[2 * e] != uv_[2 * e + 1]) off_[uv_[2 * e + 1] + 1]++;
    }
    for (vid_t v = 0; v < max_vid_; ++v) off_[v + 1] += off_[v];
    adj_.resize(off_[max_vid_]);
    std::vector<uint64_t> pos(off_.begin(), off_.end() - 1);
    for (size_t e = 0; e < m; ++e) {
      uint32_t t = uv_[2 * e], h = uv_[2 * e + 1];
      adj_[pos[t]++] = h;
      if (t != h) adj_[pos[h]++] = t;
    }
    num_nodes_ = 0;
    for (vid_t v = 0; v < max_vid_; ++v) num_nodes_ += off_[v + 1] != off_[v];
  }

 public:
  EdgeGraph() = default;
  EdgeGraph(EdgeGraph const&) = delete;
  EdgeGraph& operator=(EdgeGraph const&) = delete;
  EdgeGraph(EdgeGraph&& o) noexcept { *this = std::move(o); }
  ~EdgeGraph() {
    if (reg_) (void)sheep_records_release(reg_);
  }

  // to_device: a .dat file goes straight to HBM through pinned staging (sheep_records_load_dat)
  // and stays there for every GPU call on this graph; the host copy is filled on the way.
  EdgeGraph(char const* filename, size_t part, size_t num_parts, bool to_device) {
    if (!to_device || !is_dat(filename)) {
      *this = EdgeGraph(filename, part, num_parts);
      if (to_device) this->to_device();
      return;
    }
    uint64_t m = 0;
    uint32_t mx = 0;
    sheep_check(sheep_records_load_dat(filename, part, num_parts, nullptr, 0, &m, nullptr), "load");
    uv_.resize(2 * std::max<uint64_t>(m, 1));
    sheep_check(sheep_records_load_dat(filename, part, num_parts, uv_.data(), m, &m, &mx), "load");
    uv_.resize(2 * m);
    reg_ = uv_.data();
    max_vid_ = mx;
  }
  EdgeGraph& operator=(EdgeGraph&& o) noexcept {
    if (this != &o) {
      if (reg_) (void)sheep_records_release(reg_);
      uv_ = std::move(o.uv_);
      max_vid_ = o.max_vid_;
      off_ = std::move(o.off_);
      adj_ = std::move(o.adj_);
      num_nodes_ = o.num_nodes_;
      reg_ = o.reg_;
      o.reg_ = nullptr;
    }
    return *this;
  }

  // Keep one device copy of the records for the GPU calls that follow (idempotent).
  void to_device() const {
    if (reg_ || uv_.empty()) return;
    sheep_check(sheep_records_register(uv_.data(), records()), "records");
    reg_ = uv_.data();
  }

  EdgeGraph(char const* filename, size_t part = 0, size_t num_parts = 0) {
    std::vector<uint32_t> all;
    if (is_dat(filename)) {
      FILE* f = fopen(filename, "rb");
      if (!f) throw std::runtime_error(std::string("cannot open ") + filename);
      xs1 r;
      while (fread(&r, sizeof(xs1), 1, f) == 1) {
        all.push_back(r.tail);
        all.push_back(r.head);
      }
      fclose(f);
    } else {
      SNAPReader rd(filename);
      vid_t X, Y;
      while (rd.read(X, Y)) {
        all.push_back(X);
        all.push_back(Y);
      }
    }
    for (uint32_t x : all) max_vid_ = std::max<vid_t>(max_vid_, x + 1);
    size_t R = all.size() / 2, lo = 0, hi = R;
    if (num_parts) {
      lo = R * (part - 1) / num_parts;
      hi = R * part / num_parts;
    }
    uv_.assign(all.begin() + 2 * lo, all.begin() + 2 * hi);
  }
  EdgeGraph(std::vector<uint32_t> uv, vid_t max_vid) : uv_(std::move(uv)), max_vid_(max_vid) {}

  // the GPU view
  const uint32_t* records_data() const { return uv_.data(); }
  size_t records() const { return uv_.size() / 2; }

  vid_t getMaxVid() const { return max_vid_; }
  size_t getNodes() const { build_csr(); return num_nodes_; }
  size_t getEdges() const { build_csr(); return adj_.size() / 2; }
  bool isNode(vid_t X) const { build_csr(); return X < max_vid_ && off_[X + 1] != off_[X]; }
  size_t getDeg(vid_t X) const { build_csr(); return X < max_vid_ ? off_[X + 1] - off_[X] : 0; }

  class NodeItr {
    const EdgeGraph* g_;
    vid_t n_;
    void skip() { while (n_ != g_->max_vid_ && g_->off_[n_ + 1] == g_->off_[n_]) ++n_; }

   public:
    explicit NodeItr(const EdgeGraph* g) : g_(g), n_(0) { skip(); }
    vid_t operator*() const { return n_; }
    vid_t operator++() { ++n_; skip(); return n_; }
    bool isEnd() const { return n_ == g_->max_vid_; }
  };
  NodeItr getNodeItr() const { build_csr(); return NodeItr(this); }

  class EdgeItr {
    const uint32_t* p_;
    const uint32_t* e_;

   public:
    EdgeItr(const uint32_t* p, const uint32_t* e) : p_(p), e_(e) {}
    vid_t operator*() const { return *p_; }
    vid_t operator++() { ++p_; return p_ < e_ ? *p_ : INVALID_VID; }
    bool isEnd() const { return p_ == e_; }
  };
  EdgeItr getEdgeItr(vid_t X) const {
    build_csr();
    if (X >= max_vid_) return EdgeItr(nullptr, nullptr);
    return EdgeItr(adj_.data() + off_[X], adj_.data() + off_[X + 1]);
  }
};
typedef EdgeGraph GraphWrapper;
