// le_sort.hip -- device radix sort (stable, key-value) and exclusive scan used by
// the marker binning.  rocPRIM's onesweep radix sort is the device sort; kept in
// its own translation unit so the heavy templates compile once.
#include <hip/hip_runtime.h>

#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>

#include "le_internal.h"

namespace ibtk_le {

hipError_t launch_sort(void* temp, size_t& temp_bytes, const unsigned* kin, unsigned* kout, const int* vin,
                       int* vout, int n, int end_bit, hipStream_t s) {
    return rocprim::radix_sort_pairs(temp, temp_bytes, kin, kout, vin, vout, (size_t)n, 0u, (unsigned)end_bit, s,
                                     false);
}

hipError_t launch_scan(void* temp, size_t& temp_bytes, const int* in, int* out, int n, hipStream_t s) {
    return rocprim::exclusive_scan(temp, temp_bytes, in, out, 0, (size_t)n, rocprim::plus<int>(), s, false);
}

}  // namespace ibtk_le
