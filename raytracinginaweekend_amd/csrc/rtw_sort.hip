// rtw_sort.hip -- device radix sort used by the render scheduler (tile order by measured cost).
// Kept out of rtw_device.hip: hipcub instantiates many kernels, and none of this is arithmetic
// the parity contract covers (it only reorders work).
#include <hip/hip_runtime.h>

#include <hipcub/device/device_radix_sort.hpp>

#include "rtw_common.h"

namespace rtw {

hipError_t sort_pairs_desc(const uint32_t* keys_in, uint32_t* keys_out, const uint32_t* vals_in, uint32_t* vals_out,
                           int n, void* tmp, size_t* tmp_bytes, hipStream_t stream) {
    return hipcub::DeviceRadixSort::SortPairsDescending(tmp, *tmp_bytes, keys_in, keys_out, vals_in, vals_out, n, 0, 32,
                                                        stream);
}

}  // namespace rtw
