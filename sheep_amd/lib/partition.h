// Tree partitioning and its evaluation (reference: lib/partition.h, lib/partition.cpp).
// Host C++, as in the reference.  Built: forwardPartition (the paper's method, FFD bin
// packing, partition.cpp:86-157), print, evaluate(graph) / evaluate(graph, seq)
// (partition.cpp:428-521), writePartitionedGraph (partition.cpp:588-681).  The experimental
// partitioners (backward/depth/height/naive/random/fennel) are out of scope of this build.
//
// Parity note: forwardPartition orders kids with the unstable std::sort (partition.cpp:104)
// IN PLACE on the table's kids lists, and partition_tree reuses one table for every k, so the
// same libstdc++ std::sort is called here on the same ranges in the same order.
#pragma once
#include <algorithm>
#include <atomic>
#include <charconv>
#include <cassert>
#include <string>
#include <thread>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <memory>
#include <unordered_set>
#include <vector>

#include "defs.h"
#include "graph_wrapper.h"
#include "jnode.h"
#include "sheep_call.h"
#include "readerwriter.h"

class Partition {
 public:
  std::vector<part_t> parts;
  part_t num_parts = 0;

  Partition() = default;

  // partition.cpp:50-67 (pre_weight is always 0 without USE_PRE_WEIGHT, defs.h:62)
  Partition(std::vector<jnid_t> const& seq, JNodeTable& jnodes, part_t np, double balance_factor = 1.03,
            bool vtx_weight = false, bool pst_weight = true, bool pre_weight = false)
      : parts(jnodes.size(), INVALID_PART), num_parts(np) {
    (void)pre_weight;
    if (!jnodes.hasKids()) jnodes.makeKids();
    size_t total_weight = 0;
    for (jnid_t id = 0; id != jnodes.size(); ++id) total_weight += weight(jnodes, id, vtx_weight, pst_weight);
    size_t max_component = (total_weight / num_parts) * balance_factor;
    forwardPartition(jnodes, max_component, vtx_weight, pst_weight);
    std::vector<part_t> tmp(*std::max_element(seq.cbegin(), seq.cend()) + 1, INVALID_PART);
    for (size_t i = 0; i != seq.size(); ++i) tmp.at(seq.at(i)) = parts.at(i);
    parts = std::move(tmp);
  }

  static size_t weight(JNodeTable const& jn, jnid_t id, bool vtx, bool pst) {  // partition.cpp:38-48
    return (vtx ? 1 : 0) + (pst ? (size_t)jn.pst_weight(id) : 0);
  }

  void forwardPartition(JNodeTable& jnodes, size_t const max_component, bool vtx, bool pst) {
    std::vector<size_t> part_size;
    std::vector<size_t> below(jnodes.size(), 0);
    for (jnid_t id = 0; id != jnodes.size(); ++id) {
      below.at(id) += weight(jnodes, id, vtx, pst);
      if (below.at(id) > max_component) {
        std::sort(jnodes.kids_begin(id), jnodes.kids_end(id),
                  [&below](jnid_t const l, jnid_t const r) { return below.at(l) > below.at(r); });
        do {
          for (jnid_t* it = jnodes.kids_begin(id); below.at(id) > max_component && it != jnodes.kids_end(id); ++it) {
            jnid_t const kid = *it;
            if (parts.at(kid) != INVALID_PART) continue;
            for (part_t cp = 0; cp != (part_t)part_size.size(); ++cp) {
              if (part_size.at(cp) + below.at(kid) <= max_component) {
                below.at(id) -= below.at(kid);
                part_size.at(cp) += below.at(kid);
                parts.at(kid) = cp;
                break;
              }
            }
          }
          if (below.at(id) > max_component) part_size.push_back(0);
        } while (below.at(id) > max_component);
      }
      if (jnodes.parent(id) != INVALID_JNID) below.at(jnodes.parent(id)) += below.at(id);
    }
    for (jnid_t id = jnodes.size() - 1; id != (jnid_t)-1; --id) {
      if (parts.at(id) == INVALID_PART && jnodes.parent(id) != INVALID_JNID) parts.at(id) = parts.at(jnodes.parent(id));
      while (parts.at(id) == INVALID_PART) {
        for (part_t cp = part_size.size() - 1; cp != -1; --cp) {
          if (part_size.at(cp) + below.at(id) <= max_component) {
            part_size.at(cp) += below.at(id);
            parts.at(id) = cp;
            break;
          }
        }
        if (parts.at(id) == INVALID_PART) part_size.push_back(0);
      }
    }
  }

  void print() const {  // partition.h:135-143
    part_t max_part = *std::max_element(parts.cbegin(), parts.cend()) + 1;
    size_t first = std::count(parts.cbegin(), parts.cend(), 0);
    size_t second = std::count(parts.cbegin(), parts.cend(), 1);
    printf("Actually created %d partitions.\n", max_part);
    printf("First two partition sizes: %zu and %zu\n", first, second);
  }

  static uint32_t cormen_hash(vid_t k) {  // partition.cpp:420-424
    double A = 0.5 * (sqrt(5) - 1);
    uint32_t s = floor(A * pow(2, 32));
    return k * s;
  }

  template <typename GraphType>
  void evaluate(GraphType const& graph) const {  // partition.cpp:428-473
    size_t edges_cut = 0, Vcom_vol = 0, ECV_hash = 0;
    part_t max_part = *std::max_element(parts.cbegin(), parts.cend());
    std::vector<size_t> vertex_balance(max_part + 1, 0), hash_balance(max_part + 1, 0);
    for (auto n = graph.getNodeItr(); !n.isEnd(); ++n) {
      vid_t const X = *n;
      part_t const Xp = parts.at(X);
      vertex_balance.at(Xp) += 1;
      std::unordered_set<part_t> vset = {Xp}, hset = {};
      for (auto e = graph.getEdgeItr(X); !e.isEnd(); ++e) {
        vid_t const Y = *e;
        part_t const Yp = parts.at(Y);
        if (X < Y && Xp != Yp) ++edges_cut;
        vset.insert(Yp);
        part_t hp = cormen_hash(X) < cormen_hash(Y) ? Xp : Yp;
        hset.insert(hp);
        if (X < Y) hash_balance.at(hp) += 1;
      }
      Vcom_vol += vset.size() - 1;
      ECV_hash += hset.size() - 1;
    }
    size_t mvb = *std::max_element(vertex_balance.cbegin(), vertex_balance.cend());
    size_t mhb = *std::max_element(hash_balance.cbegin(), hash_balance.cend());
    printf("edges cut: %zu (%f%%)\n", edges_cut, (double)edges_cut / graph.getEdges());
    printf("Vcom. vol: %zu (%f%%)\n", Vcom_vol, (double)Vcom_vol / graph.getEdges());
    printf("  balance: %zu (%f%%)\n", mvb, (double)mvb / (graph.getNodes() / num_parts));
    printf("ECV(hash): %zu (%f%%)\n", ECV_hash, (double)ECV_hash / graph.getEdges());
    printf("  balance: %zu (%f%%)\n", mhb, (double)mhb / (graph.getEdges() / num_parts));
  }

  template <typename GraphType>
  void evaluate(GraphType const& graph, std::vector<vid_t> const& seq) const {  // :475-521
    evaluate(graph);
    std::vector<jnid_t> pos(*std::max_element(seq.cbegin(), seq.cend()) + 1, INVALID_JNID);
    for (jnid_t i = 0; i != seq.size(); ++i) pos[seq[i]] = i;
    size_t ECV_down = 0, ECV_up = 0;
    part_t max_part = *std::max_element(parts.cbegin(), parts.cend()) + 1;
    std::vector<size_t> down_balance(max_part, 0), up_balance(max_part, 0);
    for (auto n = graph.getNodeItr(); !n.isEnd(); ++n) {
      vid_t const X = *n;
      jnid_t const Xpos = pos.at(X);
      part_t const Xp = parts.at(X);
      std::unordered_set<part_t> dset = {}, uset = {};
      for (auto e = graph.getEdgeItr(X); !e.isEnd(); ++e) {
        vid_t const Y = *e;
        jnid_t const Ypos = pos.at(Y);
        part_t const Yp = parts.at(Y);
        dset.insert((Xpos < Ypos) ? Xp : Yp);
        uset.insert((Xpos > Ypos) ? Xp : Yp);
        if (Xpos < Ypos) down_balance.at(Xp) += 1;
        if (Xpos > Ypos) up_balance.at(Xp) += 1;
      }
      ECV_down += dset.size() - 1;
      ECV_up += uset.size() - 1;
    }
    size_t mdb = *std::max_element(down_balance.cbegin(), down_balance.cend());
    size_t mub = *std::max_element(up_balance.cbegin(), up_balance.cend());
    printf("ECV(down): %zu (%f%%)\n", ECV_down, (double)ECV_down / graph.getEdges());
    printf("  balance: %zu (%f%%)\n", mdb, (double)mdb / (graph.getEdges() / num_parts));
    printf("ECV(up)  : %zu (%f%%)\n", ECV_up, (double)ECV_up / graph.getEdges());
    printf("  balance: %zu (%f%%)\n", mub, (double)mub / (graph.getEdges() / num_parts));
  }

  // evaluate(graph) + evaluate(graph, seq) in one call on the GPU (sheep_evaluate, the MI355X
  // path for big graphs): the same numbers and the same printed lines as the two host loops
  // above, which walk an unordered_set per vertex.  partition_tree -G selects it.
  template <typename GraphType>
  void evaluate_gpu(GraphType const& graph, std::vector<vid_t> const& seq) const {
    uint64_t o[11];
    graph.to_device();
    part_t max_part = *std::max_element(parts.cbegin(), parts.cend());
    sheep_check(sheep_evaluate(graph.records_data(), graph.records(), parts.data(),
                               (uint32_t)parts.size(), seq.data(), (uint32_t)seq.size(),
                               (uint32_t)max_part + 1, o),
                "Partition::evaluate");
    const double E = (double)graph.getEdges();
    printf("edges cut: %zu (%f%%)\n", (size_t)o[0], (double)o[0] / E);
    printf("Vcom. vol: %zu (%f%%)\n", (size_t)o[1], (double)o[1] / E);
    printf("  balance: %zu (%f%%)\n", (size_t)o[2], (double)o[2] / (graph.getNodes() / num_parts));
    printf("ECV(hash): %zu (%f%%)\n", (size_t)o[3], (double)o[3] / E);
    printf("  balance: %zu (%f%%)\n", (size_t)o[4], (double)o[4] / (graph.getEdges() / num_parts));
    printf("ECV(down): %zu (%f%%)\n", (size_t)o[5], (double)o[5] / E);
    printf("  balance: %zu (%f%%)\n", (size_t)o[6], (double)o[6] / (graph.getEdges() / num_parts));
    printf("ECV(up)  : %zu (%f%%)\n", (size_t)o[7], (double)o[7] / E);
    printf("  balance: %zu (%f%%)\n", (size_t)o[8], (double)o[8] / (graph.getEdges() / num_parts));
  }

  // writePartitionedGraph (partition.cpp:588-630): edge (X,Y), X<Y, goes to the part of the
  // lower-sequence endpoint; one "%s%04d" file per part.  The records are grouped by part on
  // the GPU (sheep_partition_edges: X ascending, then record order, as the node-by-node walk
  // below writes them) and the part files are formatted and written by parallel host threads.
  void writePartitionedGraph(EdgeGraph const& graph, std::vector<vid_t> const& seq,
                             char const* prefix) const {
    part_t const max_part = *std::max_element(parts.cbegin(), parts.cend());
    assert(max_part < 10000);
    const uint32_t np = (uint32_t)max_part + 1;
    graph.to_device();
    std::vector<uint32_t> out(2 * std::max<size_t>(graph.records(), 1));
    std::vector<uint64_t> start(np + 1);
    sheep_check(sheep_partition_edges(graph.records_data(), graph.records(), parts.data(),
                                      (uint32_t)parts.size(), seq.data(), (uint32_t)seq.size(), np,
                                      out.data(), start.data()),
                "writePartitionedGraph");
    std::vector<char> name(strlen(prefix) + 16);
    std::vector<std::string> names(np);
    for (uint32_t p = 0; p < np; ++p) {
      snprintf(name.data(), name.size(), "%s%04d", prefix, (int)p);
      names[p] = name.data();
    }
    std::atomic<uint32_t> next(0);
    std::atomic<bool> failed(false);
    auto work = [&] {
      std::vector<char> buf;
      for (uint32_t p; (p = next++) < np;) {
        const uint64_t b = start[p], e = start[p + 1];
        buf.resize((e - b) * 22 + 1);
        char* w = buf.data();
        for (uint64_t i = b; i < e; ++i) {
          w = std::to_chars(w, w + 11, out[2 * i]).ptr;
          *w++ = ' ';
          w = std::to_chars(w, w + 11, out[2 * i + 1]).ptr;
          *w++ = '\n';
        }
        FILE* f = fopen(names[p].c_str(), "wb");
        if (!f || fwrite(buf.data(), 1, w - buf.data(), f) != (size_t)(w - buf.data())) failed = true;
        if (f) fclose(f);
      }
    };
    const unsigned nt = std::max(1u, std::min<unsigned>(np, std::thread::hardware_concurrency()));
    std::vector<std::thread> th;
    for (unsigned i = 0; i < nt; ++i) th.emplace_back(work);
    for (auto& t : th) t.join();
    if (failed) throw std::runtime_error(std::string("cannot write the part files ") + prefix + "*");
  }

  // The node-by-node walk of the reference (any GraphType with the LLAMA iterators).
  template <typename GraphType, typename WriterType = SNAPWriter>
  void writePartitionedGraph_walk(GraphType const& graph, std::vector<vid_t> const& seq,
                                  char const* prefix) const {
    std::vector<jnid_t> pos(*std::max_element(seq.cbegin(), seq.cend()) + 1, INVALID_JNID);
    for (jnid_t i = 0; i != seq.size(); ++i) pos[seq[i]] = i;
    auto w = open_writers<WriterType>(prefix);
    for (auto n = graph.getNodeItr(); !n.isEnd(); ++n) {
      vid_t const X = *n;
      for (auto e = graph.getEdgeItr(X); !e.isEnd(); ++e) {
        vid_t const Y = *e;
        if (X >= Y) continue;
        part_t p = pos.at(X) < pos.at(Y) ? parts.at(X) : parts.at(Y);
        w.at(p)->write(X, Y);
      }
    }
  }

  // file variant (partition.cpp:632-681): streams the records through the reader.
  template <typename ReaderType, typename WriterType = SNAPWriter>
  void writePartitionedGraph_template(char const* input, std::vector<vid_t> const& seq,
                                      char const* prefix) const {
    std::vector<jnid_t> pos(*std::max_element(seq.cbegin(), seq.cend()) + 1, INVALID_JNID);
    for (jnid_t i = 0; i != seq.size(); ++i) pos[seq[i]] = i;
    auto w = open_writers<WriterType>(prefix);
    vid_t X, Y;
    ReaderType reader(input);
    while (reader.read(X, Y)) {
      part_t p = pos.at(X) < pos.at(Y) ? parts.at(X) : parts.at(Y);
      w.at(p)->write(X, Y);
    }
  }
  template <typename WriterType = SNAPWriter>
  void writePartitionedGraph(char const* input, std::vector<vid_t> const& seq, char const* prefix) const {
    if (is_dat(input)) writePartitionedGraph_template<XS1Reader, WriterType>(input, seq, prefix);
    else writePartitionedGraph_template<SNAPReader, WriterType>(input, seq, prefix);
  }

 private:
  template <typename WriterType>
  std::vector<std::unique_ptr<WriterType>> open_writers(char const* prefix) const {
    part_t const max_part = *std::max_element(parts.cbegin(), parts.cend());
    assert(max_part < 10000);
    std::vector<std::unique_ptr<WriterType>> w;
    std::vector<char> name(strlen(prefix) + 16);
    for (part_t p = 0; p != max_part + 1; ++p) {
      snprintf(name.data(), name.size(), "%s%04d", prefix, p);
      w.emplace_back(new WriterType(name.data()));
    }
    return w;
  }
};
