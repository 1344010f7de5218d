// merge_trees — reference merge_trees.cpp:37-100: etree(A ∪ B) of two .tre files (GPU merge).
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstring>

#include "jnode.h"

int main(int argc, char* argv[]) {
  const char* output_filename = "";
  bool verbose = false, make_kids = false, do_faqs = false;
  opterr = 0;
  int opt;
  while ((opt = getopt(argc, argv, "o:vkf")) != -1) {
    switch (opt) {
      case 'o': output_filename = optarg; break;
      case 'v': verbose = !verbose; break;
      case 'k': make_kids = !make_kids; break;
      case 'f': do_faqs = !do_faqs; break;
      case '?':
        if (optopt == 'o') printf("Option -%c requires a string.\n", optopt);
        else printf("Unknown option character '\\x%x'.\n", optopt);
        return 1;
      default: abort();
    }
  }
  if (optind + 1 >= argc) {
    printf("USAGE: merge_trees [options ...] first.tree second.tree\n");
    return 1;
  }
  (void)make_kids;  // pre_weight bookkeeping only (USE_PRE_WEIGHT off): no effect on the result
  auto t0 = std::chrono::steady_clock::now();
  try {
    JNodeTable lhs(argv[optind]), rhs(argv[optind + 1]);
    auto t1 = std::chrono::steady_clock::now();
    if (verbose) printf("Loaded in: %lums\n", (unsigned long)std::chrono::duration_cast<std::chrono::milliseconds>(t1 - t0).count());
    JNodeTable out;
    out.merge(lhs, rhs);
    if (strcmp(output_filename, "") != 0) out.save(output_filename);
    auto t2 = std::chrono::steady_clock::now();
    if (verbose) printf("Built in: %lums\n", (unsigned long)std::chrono::duration_cast<std::chrono::milliseconds>(t2 - t1).count());
    if (do_faqs) out.getFacts().print();
  } catch (const std::exception& e) {
    fprintf(stderr, "merge_trees: %s\n", e.what());
    return 2;
  }
  return 0;
}
