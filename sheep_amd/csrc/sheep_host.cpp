// Host-side entry points of the C-ABI: the parts of Sheep's path that the reference keeps on
// the host and that ctypes callers (tests, bench.py, a Python port of partition_tree) need
// without writing C++.  They run the product's own lib/ headers (sheep_amd/lib/), not the
// checker.
#include <errno.h>

#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/sheep_amd.h"
#include "../lib/jnode.h"
#include "../lib/partition.h"

namespace sheep {
void set_last_error(const char* msg);  // sheep_capi.cpp
}

extern "C" int sheep_partition(const uint32_t* parent, const uint32_t* pst, uint32_t n_seq,
                               const uint32_t* seq, const int32_t* ks, uint32_t n_k,
                               double balance, int16_t* parts_out, uint32_t n_vid,
                               uint32_t* created_out) {
  try {
    if (n_seq == 0 || !parent || !pst || !seq || !ks || !parts_out)
      throw std::invalid_argument("sheep_partition: empty tree or null argument");
    std::vector<vid_t> s(seq, seq + n_seq);
    uint32_t max_vid = 0;
    for (vid_t v : s) max_vid = v > max_vid ? v : max_vid;
    if (n_vid < max_vid + 1) throw std::out_of_range("sheep_partition: n_vid < max(seq) + 1");
    for (uint32_t i = 0; i < n_k; ++i)
      if (ks[i] < 1 || ks[i] > 32767) throw std::invalid_argument("sheep_partition: k outside [1, 32767]");
    // One table for every k: forwardPartition sorts its kids lists in place, and the next k
    // starts from that order (partition_tree.cpp:130-146 reuses its JNodeTable).
    JNodeTable jn(std::vector<jnid_t>(parent, parent + n_seq), std::vector<esize_t>(pst, pst + n_seq));
    size_t total = 0, wmax = 0;
    for (uint32_t i = 0; i < n_seq; ++i) {
      total += pst[i];
      wmax = pst[i] > wmax ? pst[i] : wmax;
    }
    for (uint32_t i = 0; i < n_k; ++i) {
      // A vertex heavier than a part never fits: forwardPartition would open empty parts
      // forever (the reference loops until bad_alloc).  Refuse it up front.
      const size_t max_component = (size_t)((total / (part_t)ks[i]) * balance);
      if (wmax > max_component)
        throw std::invalid_argument("sheep_partition: a vertex's pst weight exceeds total/k*balance");
      Partition p(s, jn, (part_t)ks[i], balance, false, true, false);
      int16_t* out = parts_out + (size_t)i * n_vid;
      for (uint32_t v = 0; v < n_vid; ++v) out[v] = v < p.parts.size() ? p.parts[v] : INVALID_PART;
      if (created_out) {
        part_t mx = INVALID_PART;
        for (part_t q : p.parts) mx = q > mx ? q : mx;
        created_out[i] = (uint32_t)(mx + 1);
      }
    }
  } catch (const std::bad_alloc&) {
    sheep::set_last_error("out of memory");
    return -ENOMEM;
  } catch (const std::out_of_range& e) {
    sheep::set_last_error(e.what());
    return -ERANGE;
  } catch (const std::invalid_argument& e) {
    sheep::set_last_error(e.what());
    return -EINVAL;
  } catch (const std::exception& e) {
    sheep::set_last_error(e.what());
    return -EIO;
  }
  return SHEEP_OK;
}
