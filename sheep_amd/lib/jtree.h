// JTree (reference: lib/jtree.h:39-188): vid -> jnid index plus the elimination tree of the
// graph under seq.  The tree is built on the GPU (sheep_build_tree); the chordal-extension
// options (-k/-e/-j/-m/-w/-x) are out of scope of this build and rejected.
#pragma once
#include <algorithm>
#include <stdexcept>
#include <vector>

#include "defs.h"
#include "graph_wrapper.h"
#include "jnode.h"
#include "sheep_call.h"

class JTree {
  std::vector<jnid_t> index;  // vid -> jnid (jtree.h:44)

 public:
  JNodeTable jnodes;

  struct Options {  // jtree.h:71-108; only the default path is built here
    bool verbose = false;
    bool make_pad = true;
    bool make_kids = false, make_pst = false, make_jxn = false;
    size_t memory_limit = 1 * GIGA, width_limit = (size_t)-1;
    bool find_max_width = false, do_rooting = false;
    size_t rooting_limit = 0;
    bool isSupported() const {
      return make_pad && !make_kids && !make_pst && !make_jxn && width_limit == (size_t)-1 &&
             !find_max_width && !do_rooting && rooting_limit == 0;
    }
  };

  template <typename GraphType>
  JTree(GraphType const& graph, std::vector<vid_t> const& seq, Options opts = Options()) {
    build(graph, seq, opts);
  }
  // built into a mapped .tre (jtree.h:125-137: the table is the file, jnode.cpp:52-74)
  template <typename GraphType>
  JTree(GraphType const& graph, std::vector<vid_t> const& seq, char const* filename,
        Options opts = Options())
      : jnodes(filename, (jnid_t)seq.size()) {
    build(graph, seq, opts);
  }
  // graph2tree -i -r in one collective step (ranks of a joined ProcessGroup, comm.h): the tree
  // of the union of every rank's partial graph under the shared seq, on every rank — the
  // result of JTree(partial graph) + jnodes.mpi_merge() without the partial trees.
  struct Collective {};
  template <typename GraphType>
  JTree(GraphType const& graph, std::vector<vid_t> const& seq, Collective, Options opts = Options()) {
    if (!opts.isSupported())
      throw std::invalid_argument("JTree: chordal-extension options are not built on MI355X");
    make_index(seq);
    graph.to_device();
    std::vector<jnid_t> parent(seq.size());
    std::vector<esize_t> pst(seq.size());
    if (!seq.empty())
      sheep_check(sheep_build_tree_multi(graph.records_data(), graph.records(), seq.data(),
                                         (uint32_t)seq.size(), parent.data(), pst.data()),
                  "JTree (collective)");
    jnodes.assign(parent, pst);
  }

  // open constructor (jtree.h:138-143): the .tre mapped in place
  JTree(std::vector<vid_t> const& seq, char const* filename) : jnodes(filename) { make_index(seq); }

  jnid_t vid2jnid(vid_t X) const { return X < index.size() ? index[X] : INVALID_JNID; }
  size_t size() const { return jnodes.size(); }

  std::vector<vid_t> get_sequence() const {
    std::vector<vid_t> seq(size());
    for (vid_t X = 0; X != index.size(); ++X)
      if (index[X] != INVALID_JNID) seq.at(index[X]) = X;
    return seq;
  }

  void print() const {
    std::vector<vid_t> s = get_sequence();
    for (jnid_t id = 0; id != size(); ++id) {
      printf("%4zu:%-8zu", (size_t)id, (size_t)s.at(id));
      jnodes.print(id);
    }
  }

  // Validity as jtree.cpp:238-300 intends: heap order, and for every edge the higher endpoint
  // is an ancestor of the lower one (the reference's check reads index.at(X) where it meant
  // index.at(nbr); this one checks the intended property).  O(m * height): a debug option.
  template <typename GraphType>
  bool isValid(GraphType const& graph, std::vector<vid_t> const& seq, Options = Options()) const {
    for (jnid_t id = 0; id < size(); ++id)
      if (jnodes.parent(id) != INVALID_JNID && jnodes.parent(id) <= id) return false;
    for (vid_t X : seq) {
      if (!graph.isNode(X)) continue;
      jnid_t cur = vid2jnid(X);
      for (auto e = graph.getEdgeItr(X); !e.isEnd(); ++e) {
        jnid_t nb = vid2jnid(*e);
        if (nb == INVALID_JNID || nb >= cur) continue;
        while (nb != INVALID_JNID && nb < cur) nb = jnodes.parent(nb);
        if (nb != cur) return false;
      }
    }
    return true;
  }

 private:
  void make_index(std::vector<vid_t> const& seq) {
    if (seq.empty()) return;
    index.assign(*std::max_element(seq.begin(), seq.end()) + 1, INVALID_JNID);
    for (jnid_t id = 0; id != seq.size(); ++id) index[seq[id]] = id;
  }

  template <typename GraphType>
  void build(GraphType const& graph, std::vector<vid_t> const& seq, Options opts) {
    if (!opts.isSupported())
      throw std::invalid_argument("JTree: chordal-extension options are not built on MI355X");
    make_index(seq);
    graph.to_device();
    std::vector<jnid_t> parent(seq.size());
    std::vector<esize_t> pst(seq.size());
    if (!seq.empty())
      sheep_check(sheep_build_tree(graph.records_data(), graph.records(), seq.data(),
                                   (uint32_t)seq.size(), parent.data(), pst.data()),
                  "JTree");
    jnodes.assign(parent, pst);
  }
};
