// sort.hip — read ordering for the chain2aln launch: a stable LSD radix sort
// of (key, read index) pairs with rocPRIM (kept in its own translation unit:
// the header is heavy and the kernels do not need it).
#include <cstring>

#include <rocprim/device/device_radix_sort.hpp>

#include "engine.h"

namespace bwagpu {

hipError_t sort_reads(void* temp, size_t& temp_bytes, const uint32_t* keys_in, uint32_t* keys_out,
                      const int32_t* vals_in, int32_t* vals_out, int n, hipStream_t st) {
  // keys use 18 bits: [variant:2 | 0xffff - cost:16]
  return rocprim::radix_sort_pairs(temp, temp_bytes, keys_in, keys_out, vals_in, vals_out, (unsigned)n, 0, 18, st);
}

}  // namespace bwagpu
