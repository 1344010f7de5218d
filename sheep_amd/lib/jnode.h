// The tree (reference: lib/jnode.h:45-298, lib/jnode.cpp).  JNode = {jnid_t parent,
// esize_t pst_weight}; INVALID parent = root.  Construction (JTree) and merge run on the GPU
// through the C-ABI.  .tre = u32 end_id, then max_id JNodes.
// Storage, as the reference's (jnode.h:52-53, jnode.cpp:42-110): ALLOCATED (heap) or MAPPED —
// the nodes live in a MAP_SHARED mapping of the .tre file itself, so a tree larger than RAM is
// paged by the kernel (the reference's out-of-core mode, README:112-121).  The open
// constructor maps the file (jnode.cpp:76-102); JNodeTable(file, max_jnids) creates and maps a
// new one (jnode.cpp:52-74); a mapped table writes end_id into the header when it is destroyed
// (jnode.cpp:153-161).
#pragma once
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cstdio>
#include <fstream>
#include <stdexcept>
#include <utility>
#include <vector>

#include "defs.h"
#include "sheep_call.h"

class JNodeTable {
 public:
  struct JNode {
    jnid_t parent;
    esize_t pst_weight;
  };

 private:
  std::vector<JNode> heap_;     // ALLOCATED storage
  char* map_ = nullptr;         // MAPPED storage: header word, then the nodes
  size_t map_bytes_ = 0;
  JNode* nodes_ = nullptr;
  jnid_t end_id_ = 0;
  size_t max_id_ = 0;
  std::vector<uint64_t> kid_off_;  // makeKids (jnode.h:190-204): ascending jnid order
  std::vector<jnid_t> kid_ids_;

  void map_file(int fd, size_t bytes) {
    void* p = bytes ? mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0) : nullptr;
    close(fd);
    if (p == MAP_FAILED) throw std::bad_alloc();
    map_ = (char*)p;
    map_bytes_ = bytes;
    nodes_ = map_ ? (JNode*)(map_ + sizeof(jnid_t)) : nullptr;
  }
  void unmap() {
    if (map_) {
      *(jnid_t*)map_ = end_id_;
      munmap(map_, map_bytes_);
    }
    map_ = nullptr;
    map_bytes_ = 0;
  }
  void take(JNodeTable& o) {
    heap_ = std::move(o.heap_);
    map_ = o.map_;
    map_bytes_ = o.map_bytes_;
    nodes_ = map_ ? (JNode*)(map_ + sizeof(jnid_t)) : heap_.data();
    end_id_ = o.end_id_;
    max_id_ = o.max_id_;
    kid_off_ = std::move(o.kid_off_);
    kid_ids_ = std::move(o.kid_ids_);
    o.map_ = nullptr;
    o.map_bytes_ = 0;
    o.nodes_ = nullptr;
    o.end_id_ = 0;
    o.max_id_ = 0;
  }

 public:
  JNodeTable() = default;
  explicit JNodeTable(jnid_t max_jnids)
      : heap_(max_jnids, JNode{INVALID_JNID, 0}), nodes_(heap_.data()), end_id_(max_jnids),
        max_id_(max_jnids) {}
  JNodeTable(std::vector<jnid_t> const& parent, std::vector<esize_t> const& pst) {
    heap_.resize(parent.size());
    for (size_t i = 0; i < parent.size(); ++i) heap_[i] = JNode{parent[i], pst[i]};
    nodes_ = heap_.data();
    end_id_ = (jnid_t)parent.size();
    max_id_ = parent.size();
  }
  // Mapped constructor (jnode.cpp:52-74): a new .tre of max_jnids nodes, all roots, mapped.
  JNodeTable(char const* filename, jnid_t max_jnids) {
    int fd = open(filename, O_RDWR | O_CREAT | O_TRUNC, 0666);
    if (fd == -1) throw std::bad_alloc();
    const size_t bytes = sizeof(jnid_t) + sizeof(JNode) * (size_t)max_jnids;
    if (posix_fallocate(fd, 0, (off_t)bytes) != 0) {
      close(fd);
      throw std::bad_alloc();
    }
    map_file(fd, bytes);
    max_id_ = max_jnids;
    end_id_ = max_jnids;
    for (size_t i = 0; i < max_id_; ++i) nodes_[i] = JNode{INVALID_JNID, 0};
  }
  // Open constructor (jnode.cpp:76-102): the file mapped in place; max_id from its size,
  // end_id from its header, then makeKids.
  explicit JNodeTable(char const* filename) {
    int fd = open(filename, O_RDWR);
    if (fd == -1) throw std::bad_alloc();
    struct stat st;
    if (fstat(fd, &st) == -1 || (size_t)st.st_size < sizeof(jnid_t)) {
      close(fd);
      throw std::bad_alloc();
    }
    max_id_ = ((size_t)st.st_size - sizeof(jnid_t)) / sizeof(JNode);
    map_file(fd, sizeof(jnid_t) + sizeof(JNode) * max_id_);
    end_id_ = *(const jnid_t*)map_;
    if (end_id_ > max_id_) throw std::bad_alloc();
    makeKids();
  }
  JNodeTable(JNodeTable&& o) noexcept { take(o); }
  JNodeTable& operator=(JNodeTable&& o) noexcept {
    if (this != &o) {
      unmap();
      take(o);
    }
    return *this;
  }
  JNodeTable(JNodeTable const&) = delete;
  JNodeTable& operator=(JNodeTable const&) = delete;
  ~JNodeTable() { unmap(); }

  bool mapped() const { return map_ != nullptr; }
  // A mapped table's contents <- (parent, pst) (sizes must match; end_id = their size).
  void assign(std::vector<jnid_t> const& parent, std::vector<esize_t> const& pst) {
    if (!map_) {
      *this = JNodeTable(parent, pst);
      return;
    }
    if (parent.size() > max_id_) throw std::invalid_argument("JNodeTable: more nodes than mapped");
    for (size_t i = 0; i < parent.size(); ++i) nodes_[i] = JNode{parent[i], pst[i]};
    end_id_ = (jnid_t)parent.size();
    kid_off_.clear();
    kid_ids_.clear();
  }

  jnid_t size() const { return end_id_; }
  jnid_t& parent(jnid_t id) { return nodes_[id].parent; }
  jnid_t parent(jnid_t id) const { return nodes_[id].parent; }
  esize_t& pst_weight(jnid_t id) { return nodes_[id].pst_weight; }
  esize_t pst_weight(jnid_t id) const { return nodes_[id].pst_weight; }
  size_t width(jnid_t id) const { return 1 + (size_t)nodes_[id].pst_weight; }  // jnode.h:258-260

  std::vector<jnid_t> parents() const {
    std::vector<jnid_t> p(end_id_);
    for (jnid_t i = 0; i < end_id_; ++i) p[i] = nodes_[i].parent;
    return p;
  }
  std::vector<esize_t> psts() const {
    std::vector<esize_t> w(end_id_);
    for (jnid_t i = 0; i < end_id_; ++i) w[i] = nodes_[i].pst_weight;
    return w;
  }

  // save (jnode.cpp:164-168)
  void save(char const* filename) const {
    std::ofstream s(filename, std::ios::binary | std::ios::trunc);
    s.write((const char*)&end_id_, sizeof(jnid_t));
    s.write((const char*)nodes_, max_id_ * sizeof(JNode));
  }

  // merge (jnode.cpp:174-201) on the GPU: *this <- etree(lhs ∪ rhs), pst summed.
  void merge(JNodeTable const& lhs, JNodeTable const& rhs) {
    if (lhs.size() != rhs.size()) throw std::invalid_argument("merge: tables of different size");
    jnid_t n = lhs.size();
    std::vector<jnid_t> pa = lhs.parents(), pb = rhs.parents(), po(n);
    std::vector<esize_t> sa = lhs.psts(), sb = rhs.psts(), so(n);
    if (n) sheep_check(sheep_merge_trees(pa.data(), sa.data(), pb.data(), sb.data(), n, po.data(), so.data()), "merge");
    assign(po, so);  // a mapped table stays mapped
  }

  // mpi_merge (jnode.cpp:213-250): every rank's partial tree (same seq) -> the tree of the union
  // of their graphs, on every rank (the reference leaves it on rank 0), pst summed.
  void mpi_merge() {
    std::vector<jnid_t> p = parents();
    std::vector<esize_t> w = psts();
    if (!p.empty()) sheep_check(sheep_mpi_merge(p.data(), w.data(), (uint32_t)p.size()), "mpi_merge");
    assign(p, w);
  }

  void makeKids() {
    kid_off_.assign((size_t)end_id_ + 1, 0);
    for (jnid_t id = 0; id < end_id_; ++id)
      if (parent(id) != INVALID_JNID) kid_off_.at(parent(id) + 1)++;
    for (jnid_t id = 0; id < end_id_; ++id) kid_off_[id + 1] += kid_off_[id];
    kid_ids_.resize(kid_off_[end_id_]);
    std::vector<uint64_t> pos(kid_off_.begin(), kid_off_.end() - 1);
    for (jnid_t id = 0; id < end_id_; ++id)
      if (parent(id) != INVALID_JNID) kid_ids_[pos[parent(id)]++] = id;
  }
  bool hasKids() const { return kid_off_.size() == (size_t)end_id_ + 1; }
  jnid_t* kids_begin(jnid_t id) { return kid_ids_.data() + kid_off_[id]; }
  jnid_t* kids_end(jnid_t id) { return kid_ids_.data() + kid_off_[id + 1]; }

  // Facts (jnode.cpp:256-290; print jnode.h:285-291)
  struct Facts {
    size_t vert_cnt = 0, edge_cnt = 0, width = 0, fill = 0, vert_height = 0, edge_height = 0,
           root_cnt = 0;
    jnid_t halo_id = INVALID_JNID, core_id = INVALID_JNID;
    explicit Facts(JNodeTable const& jn) {
      std::vector<unsigned long long> vh(jn.size(), 0), eh(jn.size(), 0);
      for (jnid_t id = 0; id != jn.size(); ++id) {
        jnid_t p = jn.parent(id);
        vert_cnt++;
        edge_cnt += jn.pst_weight(id);
        width = std::max(width, jn.width(id));
        fill += jn.width(id) - jn.pst_weight(id) - 1;
        vh[id]++;
        eh[id] += jn.pst_weight(id);
        if (p != INVALID_JNID) {
          vh.at(p) = std::max(vh[p], vh[id]);
          eh.at(p) = std::max(eh[p], eh[id]);
        } else {
          vert_height = std::max<size_t>(vert_height, vh[id]);
          edge_height = std::max<size_t>(edge_height, eh[id]);
          root_cnt++;
        }
        if (halo_id == INVALID_JNID && jn.width(id) > 3) halo_id = id;
        if (core_id == INVALID_JNID && jn.width(id) >= width) core_id = id;
      }
    }
    void print() const {
      printf("TREEFAQS: width:%zu\troots:%zu\n", width, root_cnt);
      printf("\tvheight:%zu\teheight:%zu\n", vert_height, edge_height);
      printf("\tverts:%zu\tedges:%zu\n", vert_cnt, edge_cnt);
      printf("\thalo:%zu\tcore:%zu\n", (size_t)halo_id, (size_t)core_id);
      printf("\tfill:%zu\n", fill);
    }
  };
  Facts getFacts() const { return Facts(*this); }

  void print(jnid_t id) const {  // jnode.h:264-267 (pre_weight is always 0 without USE_PRE_WEIGHT)
    printf("%6zu:w%6zu:pre%6zu:pst        ->[%4zu]\n", width(id), (size_t)0,
           (size_t)pst_weight(id), (size_t)parent(id));
  }
};
