// Vertex sequences (reference: lib/sequence.h:43-184).  The degree count and the
// (degree asc, id asc) sort run on the GPU through sheep_degree_seq.
#pragma once
#include <fstream>
#include <vector>

#include "defs.h"
#include "graph_wrapper.h"
#include "readerwriter.h"
#include "sheep_call.h"

// defaultSequence (sequence.h:43-50): non-isolated ids in id order.
template <typename GraphType>
std::vector<vid_t> defaultSequence(GraphType const& graph) {
  std::vector<vid_t> seq;
  seq.reserve(graph.getNodes());
  for (auto it = graph.getNodeItr(); !it.isEnd(); ++it) seq.push_back(*it);
  return seq;
}

inline std::vector<vid_t> edgeSequence(const uint32_t* uv, size_t m, vid_t n_ids, int mode) {
  std::vector<vid_t> seq(n_ids ? n_ids : 1);
  uint32_t n_seq = 0;
  if (m) sheep_check(sheep_degree_seq(uv, m, n_ids, mode, seq.data(), &n_seq, nullptr), "degree sequence");
  seq.resize(n_seq);
  return seq;
}

// degreeSequence (sequence.h:52-63): LLAMA degrees (a self-loop counts once).
template <typename GraphType>
std::vector<vid_t> degreeSequence(GraphType const& graph) {
  graph.to_device();
  return edgeSequence(graph.records_data(), graph.records(), graph.getMaxVid(), SHEEP_DEGREE_LLAMA);
}

// mpiSequence (sequence.h:65-93): this rank's partial graph; the id spaces MAX-reduced and the
// degrees SUM-reduced over the ranks (RCCL; a ProcessGroup from comm.h must be joined), so
// every rank gets the same sequence.  getMaxVid() is this rank's share only (its records), and
// the global sequence can be longer: then EVERY rank gets -ERANGE with the global length
// (sheep_mpi_sequence compares with the smallest buffer of all ranks), and all retry together.
template <typename GraphType>
std::vector<vid_t> mpiSequence(GraphType const& graph) {
  graph.to_device();
  std::vector<vid_t> seq(std::max<vid_t>(graph.getMaxVid(), 1));
  uint32_t n_seq = 0;
  int rc = sheep_mpi_sequence(graph.records_data(), graph.records(), graph.getMaxVid(),
                              SHEEP_DEGREE_LLAMA, seq.data(), (uint32_t)seq.size(), &n_seq);
  if (rc == -ERANGE && n_seq > 0) {  // on every rank, also those whose buffer was large enough
    seq.resize(std::max<size_t>(seq.size(), n_seq));
    rc = sheep_mpi_sequence(graph.records_data(), graph.records(), graph.getMaxVid(),
                            SHEEP_DEGREE_LLAMA, seq.data(), (uint32_t)seq.size(), &n_seq);
  }
  sheep_check(rc, "mpiSequence");
  seq.resize(n_seq);
  return seq;
}

// fileSequence (sequence.h:95-128): FILE degrees (degree[X]++, degree[Y]++) over the reader
// stream, including XS1Reader's repeated last record.
template <typename ReaderType>
std::vector<vid_t> fileSequence_template(char const* filename) {
  ReaderType reader(filename);
  std::vector<uint32_t> uv;
  vid_t X, Y, top = 0;
  while (reader.read(X, Y)) {
    uv.push_back(X);
    uv.push_back(Y);
    top = std::max(top, std::max(X, Y) + 1);
  }
  return edgeSequence(uv.data(), uv.size() / 2, top, SHEEP_DEGREE_FILE);
}

inline std::vector<vid_t> fileSequence(char const* filename) {
  return is_dat(filename) ? fileSequence_template<XS1Reader>(filename)
                          : fileSequence_template<SNAPReader>(filename);
}

// Text format, one decimal id per line (USE_BIN_SEQUENCE off, sequence.h:153-184).
inline void writeSequence(std::vector<vid_t> const& seq, char const* filename) {
  std::ofstream s(filename, std::ios::trunc);
  for (vid_t X : seq) s << X << '\n';
}

inline std::vector<vid_t> readSequence(char const* filename) {
  std::vector<vid_t> seq;
  std::ifstream s(filename);
  vid_t X;
  while (s >> X) seq.push_back(X);
  return seq;
}
