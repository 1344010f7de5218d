// graph2tree — MI355X build of the reference CLI (graph2tree.cpp:44-243): same flags and the
// same "Loaded graph in / Sorted in / Mapped in / Reduced in" timer lines.  The degree sort
// and the tree build run on the GPU.  -i / -r run one process per GPU (the MPI ranks of the
// reference): launch with torchrun --no-python or mpirun, see sheep_amd/lib/comm.h.
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "comm.h"
#include "graph_wrapper.h"
#include "jtree.h"
#include "partition.h"
#include "sequence.h"

using clk = std::chrono::steady_clock;
static double secs(clk::duration d) { return std::chrono::duration_cast<std::chrono::milliseconds>(d).count() / 1000.0; }

int main(int argc, char* argv[]) {
  bool use_mpi_sort = false, use_mpi_reduce = false;
  size_t part = 0, num_parts = 0, partitions = 0;
  const char* sequence_filename = "";
  const char* output_filename = "";
  JTree::Options jopts;
  bool do_faqs = false, do_print = false, do_validate = false;
  opterr = 0;
  int opt;
  while ((opt = getopt(argc, argv, "irl:p:s:o:vkejm:w:xfdtc")) != -1) {
    switch (opt) {
      case 'i': use_mpi_sort = !use_mpi_sort; break;
      case 'r': use_mpi_reduce = !use_mpi_reduce; break;
      case 'l': {
        char* a = strtok(optarg, "/");
        char* b = strtok(nullptr, "/");
        if (!a || !b) { printf("Option -l requires part/num_parts.\n"); return 1; }
        part = atoll(a);
        num_parts = atoll(b);
        break;
      }
      case 'p': partitions = atoll(optarg); break;
      case 's': sequence_filename = optarg; break;
      case 'o': output_filename = optarg; break;
      case 'v': jopts.verbose = !jopts.verbose; break;
      case 'k': jopts.make_kids = !jopts.make_kids; break;
      case 'e': jopts.make_pst = !jopts.make_pst; break;
      case 'j': jopts.make_jxn = !jopts.make_jxn; break;
      case 'm': jopts.memory_limit = atoll(optarg) * MEGA; break;
      case 'w': jopts.width_limit = atoll(optarg); break;
      case 'x': jopts.find_max_width = !jopts.find_max_width; break;
      case 'f': do_faqs = !do_faqs; break;
      case 'd': break;
      case 't': do_print = !do_print; break;
      case 'c': do_validate = !do_validate; break;
      case '?':
        if (optopt == 's' || optopt == 'o') printf("Option -%c requires a string.\n", optopt);
        else if (optopt == 'm' || optopt == 'w') printf("Option -%c requires a long long.\n", optopt);
        else printf("Unknown option character '\\x%x'.\n", optopt);
        return 1;
      default: abort();
    }
  }
  if (optind >= argc) {
    printf("USAGE: graph2tree input_graph [options ...]\n");
    return 1;
  }
  if (!jopts.isSupported()) {
    printf("ERROR: the chordal-extension options -k -e -j -w -x are not built in this version.\n");
    return 1;
  }
  const char* graph_filename = argv[optind];
  auto t0 = clk::now();
  std::string tmp_name;
  ProcessGroup pg;
  try {
    if (use_mpi_sort || use_mpi_reduce) {  // graph2tree.cpp:134-157
      pg.init();
      part = pg.rank + 1;
      num_parts = pg.size;
      char buf[4096];
      if (!use_mpi_reduce && strcmp(output_filename, "") != 0) {
        snprintf(buf, sizeof buf, "%s%02dr0.tre", output_filename, pg.rank);
        tmp_name = buf;
        output_filename = tmp_name.c_str();
      } else if (use_mpi_reduce && partitions != 0 && strcmp(output_filename, "") != 0) {
        snprintf(buf, sizeof buf, "%s-w%04d-p", output_filename, pg.rank);
        tmp_name = buf;
        output_filename = tmp_name.c_str();
      }
    }
  } catch (const std::exception& e) {
    fprintf(stderr, "graph2tree: %s\n", e.what());
    return 2;
  }
  bool const is_leader = ((use_mpi_sort || use_mpi_reduce) && part == 1) ||
                         (!(use_mpi_sort || use_mpi_reduce) && strcmp(sequence_filename, "") == 0);
  try {
    if (jopts.verbose) printf("Loading %s...\n", graph_filename);
    GraphWrapper graph(graph_filename, part, num_parts, true);  // records straight to HBM
    if (jopts.verbose) printf("Nodes:%zu Edges:%zu\n", graph.getNodes(), graph.getEdges());
    auto t_load = clk::now();
    if (is_leader) printf("Loaded graph in: %f seconds\n", secs(t_load - t0));

    std::vector<vid_t> seq = use_mpi_sort ? mpiSequence(graph)
                             : strcmp(sequence_filename, "") != 0 ? readSequence(sequence_filename)
                                                                  : degreeSequence(graph);
    if (use_mpi_sort && part == 1 && strcmp(sequence_filename, "") != 0) writeSequence(seq, sequence_filename);
    auto t_sort = clk::now();
    if (is_leader && (use_mpi_sort || strcmp(sequence_filename, "") == 0))
      printf("Sorted in: %f seconds\n", secs(t_sort - t_load));

    // -i -r: the ranks build ONE tree together (no partial trees, no reduce step of its own);
    // -r alone: partial trees, then mpi_merge, as the reference does
    bool const collective = use_mpi_sort && use_mpi_reduce;
    bool to_file = !use_mpi_reduce && strcmp(output_filename, "") != 0 && partitions == 0;
    JTree tree = collective ? JTree(graph, seq, JTree::Collective(), jopts)
                 : to_file  ? JTree(graph, seq, output_filename, jopts)
                            : JTree(graph, seq, jopts);
    auto t_map = clk::now();
    if (is_leader) printf("Mapped in: %f seconds\n", secs(t_map - t_sort));

    if (use_mpi_reduce) {  // jnode.cpp:213-250
      if (!collective) tree.jnodes.mpi_merge();
      auto t_red = clk::now();
      if (is_leader) printf("Reduced in: %f seconds\n", secs(t_red - t_map));
    }
    if (partitions != 0) {
      // every rank holds the whole tree, so each computes the same Partition (the reference
      // partitions on rank 0 and broadcasts it, partition.cpp:69-79) and writes its own records
      tree.jnodes.makeKids();
      Partition p(seq, tree.jnodes, (part_t)partitions);
      if (strcmp(output_filename, "") != 0) p.writePartitionedGraph(graph, seq, output_filename);
      else if (is_leader) p.print();
    } else if (use_mpi_reduce && part == 1 && strcmp(output_filename, "") != 0) {
      tree.jnodes.save(output_filename);
    }
    if (jopts.verbose) printf("Built in: %f seconds\n", secs(clk::now() - t0));
    if (do_faqs) tree.jnodes.getFacts().print();
    if (do_print) tree.print();
    if (do_validate) printf(tree.isValid(graph, seq, jopts) ? "Tree is valid.\n" : "ERROR: Tree is not valid.\n");
    if (jopts.verbose) printf("Finished in: %f seconds\n", secs(clk::now() - t0));
  } catch (const std::exception& e) {
    fprintf(stderr, "graph2tree: %s\n", e.what());
    return 2;
  }
  return 0;
}
