// partition_tree — reference partition_tree.cpp:40-170: forwardPartition of a .tre for each k,
// then evaluate against the graph (-g) or write partitioned edge files (-g -o).
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "graph_wrapper.h"
#include "jnode.h"
#include "partition.h"
#include "sequence.h"

using clk = std::chrono::steady_clock;
static double secs(clk::duration d) { return std::chrono::duration_cast<std::chrono::milliseconds>(d).count() / 1000.0; }

int main(int argc, char* argv[]) {
  bool verbose = true, do_faqs = false, gpu_eval = false;
  double balance_factor = 1.03;
  bool vtx_weight = false, pst_weight = false, pre_weight = false;
  const char* graph_filename = "";
  const char* output_filename = "";
  opterr = 0;
  int opt;
  // -G (not in the reference): evaluate on the GPU (sheep_evaluate), same output lines
  while ((opt = getopt(argc, argv, "vfb:xdug:o:G")) != -1) {
    switch (opt) {
      case 'v': verbose = !verbose; break;
      case 'f': do_faqs = !do_faqs; break;
      case 'b': balance_factor = atof(optarg); break;
      case 'x': vtx_weight = true; break;
      case 'd': pst_weight = true; break;
      case 'u': pre_weight = true; break;
      case 'g': graph_filename = optarg; break;
      case 'o': output_filename = optarg; break;
      case 'G': gpu_eval = true; break;
      case '?':
        if (optopt == 'b') printf("Option -%c requires a double.\n", optopt);
        else if (optopt == 'g' || optopt == 'o') printf("Option -%c requires a string.\n", optopt);
        else printf("Unknown option character '\\x%x'.\n", optopt);
        return 1;
      default: abort();
    }
  }
  if (!(vtx_weight || pst_weight || pre_weight)) pst_weight = true;
  if (optind + 2 >= argc) {
    printf("USAGE: partition_tree [options] input_sequence input_tree parts [parts...]\n");
    return 1;
  }
  auto t0 = clk::now();
  try {
    JNodeTable jnodes(argv[optind + 1]);
    if (verbose) printf("Loaded tree in: %f seconds\n", secs(clk::now() - t0));
    if (do_faqs) jnodes.getFacts().print();
    if (strcmp(graph_filename, "") == 0) {
      std::vector<vid_t> seq = readSequence(argv[optind]);
      for (int i = optind + 2; i != argc; ++i) {
        short const np = atoi(argv[optind + 2]);  // the reference reads argv[optind+2] here
        Partition p(seq, jnodes, np, balance_factor, vtx_weight, pst_weight, pre_weight);
        p.print();
      }
    } else if (strcmp(output_filename, "") == 0) {
      GraphWrapper graph(graph_filename);
      std::vector<vid_t> seq = strcmp(argv[optind], "-") == 0 ? degreeSequence(graph) : readSequence(argv[optind]);
      for (int i = optind + 2; i != argc; ++i) {
        short const np = atoi(argv[i]);
        auto ps = clk::now();
        Partition p(seq, jnodes, np, balance_factor, vtx_weight, pst_weight, pre_weight);
        if (verbose) printf("Partitioning took: %f seconds\n", secs(clk::now() - ps));
        p.print();
        if (gpu_eval) p.evaluate_gpu(graph, seq);
        else p.evaluate(graph, seq);
      }
    } else {
      std::vector<vid_t> seq = strcmp(argv[optind], "-") == 0 ? fileSequence(graph_filename) : readSequence(argv[optind]);
      short const np = atoi(argv[optind + 2]);
      auto ps = clk::now();
      Partition p(seq, jnodes, np, balance_factor, vtx_weight, pst_weight, pre_weight);
      if (verbose) printf("Partitioning took: %f seconds\n", secs(clk::now() - ps));
      p.print();
      p.writePartitionedGraph(graph_filename, seq, output_filename);
    }
  } catch (const std::exception& e) {
    fprintf(stderr, "partition_tree: %s\n", e.what());
    return 2;
  }
  if (verbose) printf("Finished in: %f seconds\n", secs(clk::now() - t0));
  return 0;
}
