// degree_sequence — reference degree_sequence.cpp:35-51: FILE-mode degree sequence of a graph
// file (GPU sort), written as text.
#include <chrono>
#include <cstdio>

#include "sequence.h"

int main(int argc, char* argv[]) {
  if (argc != 3) {
    printf("USAGE: degree_sequence graph_file output_file");
    return 1;
  }
  auto t0 = std::chrono::steady_clock::now();
  try {
    std::vector<vid_t> seq = fileSequence(argv[1]);
    writeSequence(seq, argv[2]);
  } catch (const std::exception& e) {
    fprintf(stderr, "degree_sequence: %s\n", e.what());
    return 2;
  }
  auto ms = std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::steady_clock::now() - t0);
  printf("Sorted in: %lums\n", (unsigned long)ms.count());
  return 0;
}
