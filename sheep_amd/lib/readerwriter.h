// Edge-file readers/writers (reference: lib/readerwriter.h:36-102), same stream semantics.
//   .dat = XS1 records {u32 tail, u32 head, f32 weight}, little-endian, 12 B each.
//   .net = whitespace-separated unsigned pairs (SNAP text).
#pragma once
#include <cstdio>
#include <fstream>
#include <string>

#include "defs.h"

struct xs1 {
  unsigned tail;
  unsigned head;
  float weight;
};

// XS1Reader::read tests eof() before read() (readerwriter.h:50-58): after the last record the
// next read fails and still yields the previous record once more.  degree_sequence's FILE-mode
// degrees depend on this, so the stream is reproduced exactly (empty file: no records).
class XS1Reader {
  FILE* f_;
  xs1 buf_;
  bool have_ = false, eof_ = false;

 public:
  explicit XS1Reader(char const* filename) : f_(fopen(filename, "rb")) {}
  ~XS1Reader() {
    if (f_) fclose(f_);
  }
  bool read(vid_t& X, vid_t& Y) {
    if (!f_ || eof_) return false;
    xs1 r;
    if (fread(&r, sizeof(xs1), 1, f_) == 1) {
      buf_ = r;
      have_ = true;
    } else {
      eof_ = true;
      if (!have_) return false;
    }
    X = buf_.tail;
    Y = buf_.head;
    return true;
  }
};

class XS1Writer {
  FILE* f_;

 public:
  explicit XS1Writer(char const* filename) : f_(fopen(filename, "wb")) {}
  ~XS1Writer() {
    if (f_) fclose(f_);
  }
  void write(vid_t X, vid_t Y) {
    xs1 r{X, Y, 1.0f};
    fwrite(&r, sizeof(xs1), 1, f_);
  }
};

// SNAPReader::read (readerwriter.h:84-89): stops at the first token that is not an unsigned.
class SNAPReader {
  std::ifstream s_;

 public:
  explicit SNAPReader(char const* filename) : s_(filename) {}
  bool read(vid_t& X, vid_t& Y) {
    bool ok = (bool)(s_ >> X);
    ok &= (bool)(s_ >> Y);
    return ok;
  }
};

class SNAPWriter {
  std::ofstream s_;

 public:
  explicit SNAPWriter(char const* filename) : s_(filename, std::ios::trunc) {}
  void write(vid_t X, vid_t Y) { s_ << X << ' ' << Y << '\n'; }
};

inline bool is_dat(char const* filename) {
  std::string f(filename);
  return f.size() >= 4 && f.compare(f.size() - 4, 4, ".dat") == 0;
}
