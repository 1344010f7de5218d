// C-ABI error -> C++ exception, as the reference's lib/ throws: allocation and
// device failures -> std::bad_alloc / std::runtime_error, index.at() range -> std::out_of_range.
#pragma once
#include <cerrno>
#include <new>
#include <stdexcept>
#include <string>

#include "../../include/sheep_amd.h"

inline void sheep_check(int rc, const char* what) {
  if (rc == SHEEP_OK) return;
  std::string msg = std::string(what) + ": " + sheep_last_error();
  if (rc == -ENOMEM) throw std::bad_alloc();
  if (rc == -ERANGE) throw std::out_of_range(msg);
  if (rc == -EINVAL) throw std::invalid_argument(msg);
  throw std::runtime_error(msg);
}
