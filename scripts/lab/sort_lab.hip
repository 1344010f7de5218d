// Lab (not product): rocPRIM/hipCUB radix sort of packed u64 items as a speed reference.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <stdint.h>

extern "C" int sort_lab(void* keys_in, void* keys_out, uint64_t n, int begin_bit, int end_bit,
                        void* tmp, size_t* tmp_bytes, void* stream) {
  size_t tb = *tmp_bytes;
  hipError_t e = hipcub::DeviceRadixSort::SortKeys(tmp, tb, (const uint64_t*)keys_in,
                                                   (uint64_t*)keys_out, (int)n, begin_bit, end_bit,
                                                   (hipStream_t)stream);
  *tmp_bytes = tb;
  return e == hipSuccess ? 0 : -1;
}
