// The process group of graph2tree -i / -r (graph2tree.cpp:134-157: MPI_Init, MPI_Comm_rank,
// MPI_Comm_size).  This build has no MPI: one process per GPU is started by any launcher that
// exports the usual rank variables, and the RCCL id travels through a file, the way the
// reference's scripts hand results between workers (write a .tmp, then rename it).
//   torchrun --no-python --nproc-per-node N graph2tree G -ir ...   (RANK, WORLD_SIZE, LOCAL_RANK)
//   mpirun -n N graph2tree G -ir ...          (OMPI_COMM_WORLD_RANK / _SIZE / _LOCAL_RANK)
// SHEEP_COMM_DIR (default /tmp) holds the id file.  Its name joins every job-identifying variable
// the launcher set (SHEEP_COMM_KEY, TORCHELASTIC_RUN_ID, MASTER_ADDR, MASTER_PORT,
// OMPI_MCA_ess_base_jobid): a plain torchrun has run id "none", and MASTER_ADDR:MASTER_PORT is
// what keeps two jobs on one host apart.  Rank 0 removes a file left under that name before it
// writes the new one and on every error path; the other ranks ignore a file written more than
// kStaleSec before they started (a crashed run's).
#pragma once
#include <sys/stat.h>
#include <unistd.h>

#include <ctime>

#include <cctype>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <stdexcept>
#include <string>
#include <thread>

#include "sheep_call.h"

struct ProcessGroup {
  int rank = 0, size = 1, local_rank = 0;
  bool joined = false;

  static int env_int(const char* a, const char* b, int dflt) {
    const char* v = getenv(a);
    if (!v) v = getenv(b);
    return v ? atoi(v) : dflt;
  }

  // Reads the launcher's variables; with more than one rank, selects the GPU (LOCAL_RANK) and
  // joins the RCCL communicator.  One rank: nothing to join (MPI with one process).
  void init() {
    rank = env_int("RANK", "OMPI_COMM_WORLD_RANK", 0);
    size = env_int("WORLD_SIZE", "OMPI_COMM_WORLD_SIZE", 1);
    local_rank = env_int("LOCAL_RANK", "OMPI_COMM_WORLD_LOCAL_RANK", 0);
    if (size < 1 || rank < 0 || rank >= size) throw std::invalid_argument("bad RANK / WORLD_SIZE");
    sheep_check(sheep_gpu_init(local_rank), "gpu init");
    if (size == 1) {
      uint8_t id[SHEEP_COMM_ID_BYTES];
      sheep_check(sheep_comm_unique_id(id), "comm id");
      sheep_check(sheep_comm_init(id, 1, 0), "comm init");
      joined = true;
      return;
    }
    const std::string path = id_path();
    uint8_t id[SHEEP_COMM_ID_BYTES];
    if (rank == 0) {
      unlink(path.c_str());  // a crashed run's id must not be read by this job's ranks
      const std::string tmp = path + ".tmp";
      try {
        sheep_check(sheep_comm_unique_id(id), "comm id");
        FILE* f = fopen(tmp.c_str(), "wb");
        if (!f || fwrite(id, 1, sizeof id, f) != sizeof id || fclose(f) != 0)
          throw std::runtime_error("cannot write " + tmp);
        if (rename(tmp.c_str(), path.c_str()) != 0) throw std::runtime_error("cannot rename " + tmp);
        sheep_check(sheep_comm_init(id, size, rank), "comm init");  // collective
      } catch (...) {
        unlink(tmp.c_str());
        unlink(path.c_str());
        throw;
      }
      unlink(path.c_str());
    } else {
      const time_t started = time(nullptr);
      auto until = std::chrono::steady_clock::now() + std::chrono::seconds(120);
      for (;;) {
        struct stat st;
        FILE* f = fopen(path.c_str(), "rb");
        if (f) {
          const bool fresh = fstat(fileno(f), &st) == 0 && st.st_mtime + kStaleSec >= started;
          size_t got = fread(id, 1, sizeof id, f);
          fclose(f);
          if (fresh && got == sizeof id) break;
        }
        if (std::chrono::steady_clock::now() > until)
          throw std::runtime_error("rank " + std::to_string(rank) + ": no communicator id at " + path);
        std::this_thread::sleep_for(std::chrono::milliseconds(20));
      }
      sheep_check(sheep_comm_init(id, size, rank), "comm init");  // collective: all ranks joined
    }
    joined = true;
  }

  ~ProcessGroup() {
    if (joined) (void)sheep_comm_free();
  }

 private:
  static constexpr long kStaleSec = 60;  // ranks start within a minute of each other

  static std::string id_path() {
    const char* dir = getenv("SHEEP_COMM_DIR");
    std::string key;
    for (const char* k : {"SHEEP_COMM_KEY", "TORCHELASTIC_RUN_ID", "MASTER_ADDR", "MASTER_PORT",
                          "OMPI_MCA_ess_base_jobid"})
      if (const char* v = getenv(k)) {
        if (!key.empty()) key += '-';
        for (const char* p = v; *p; ++p)  // a file name: keep [A-Za-z0-9._]
          key += (isalnum((unsigned char)*p) || *p == '.' || *p == '_') ? *p : '_';
      }
    if (key.empty()) key = "default";
    return std::string(dir ? dir : "/tmp") + "/sheep-comm-" + key + ".id";
  }
};
