// le_sort.hip -- device radix sort (stable, key-value) and exclusive scan used by
// the marker binning.  rocPRIM's onesweep radix sort is the device sort; kept in
// its own translation unit so the heavy templates compile once.
#include <hip/hip_runtime.h>

#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>
#include <rocprim/iterator/reverse_iterator.hpp>

#include "le_internal.h"

// Onesweep with IBTK_LE_SORT_BITS key bits per pass (0: rocPRIM's tuned gfx950
// config, 8 bits per pass).  The cfg4 keys are 25 bits: 9 bits per pass sorts
// them in 3 passes instead of 4, measured 1.0 ms faster per binning (2.9 ->
// 1.9 ms).  10 and 11 bits measured slower (larger digit histograms); 12 and
// more do not fit the histogram kernel's LDS.
#ifndef IBTK_LE_SORT_BITS
#define IBTK_LE_SORT_BITS 9
#endif
#ifndef IBTK_LE_SORT_BLOCK
#define IBTK_LE_SORT_BLOCK 1024
#endif
#ifndef IBTK_LE_SORT_IPT
#define IBTK_LE_SORT_IPT 8
#endif

namespace ibtk_le {

#if IBTK_LE_SORT_BITS
using SortConfig = rocprim::radix_sort_config<
    rocprim::default_config, rocprim::default_config,
    rocprim::radix_sort_onesweep_config<rocprim::kernel_config<IBTK_LE_SORT_BLOCK, IBTK_LE_SORT_IPT>,
                                        rocprim::kernel_config<IBTK_LE_SORT_BLOCK, IBTK_LE_SORT_IPT>,
                                        IBTK_LE_SORT_BITS, rocprim::block_radix_rank_algorithm::match>>;
#else
using SortConfig = rocprim::default_config;
#endif

hipError_t launch_sort(void* temp, size_t& temp_bytes, const unsigned* kin, unsigned* kout, const int* vin,
                       int* vout, int n, int end_bit, hipStream_t s) {
    return rocprim::radix_sort_pairs<SortConfig>(temp, temp_bytes, kin, kout, vin, vout, (size_t)n, 0u, (unsigned)end_bit, s,
                                     false);
}

hipError_t launch_scan(void* temp, size_t& temp_bytes, const int* in, int* out, int n, hipStream_t s) {
    return rocprim::exclusive_scan(temp, temp_bytes, in, out, 0, (size_t)n, rocprim::plus<int>(), s, false);
}

// out[i] = min(in[i..n-1]): the bucket starts from the first entry of every
// non-empty bucket (an empty bucket starts where the next non-empty one does)
hipError_t launch_suffix_min(void* temp, size_t& temp_bytes, const int* in, int* out, int n, hipStream_t s) {
    return rocprim::inclusive_scan(temp, temp_bytes, rocprim::make_reverse_iterator(in + n),
                                   rocprim::make_reverse_iterator(out + n), (size_t)n, rocprim::minimum<int>(), s, false);
}

}  // namespace ibtk_le
