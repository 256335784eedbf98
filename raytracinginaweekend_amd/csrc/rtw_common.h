// rtw_common.h -- shared host-side helpers of librtw.so (error reporting).
#pragma once

#include <cstddef>
#include <cstdint>
#include <string>

#include <hip/hip_runtime_api.h>

#include "../../include/rtw.h"
#include "../../include/rtw_scalar.h"

// The scene RNG handle (TRng = Xoroshiro128PlusPlus, common.rs:1).
struct rtw_rng {
    rtw_xoro s;
};

namespace rtw {

// Thread-local last error (returned by rtw_last_error()).
void set_error(const std::string& msg);
int fail(int code, const std::string& msg);
const char* last_error();

// Descending key sort carrying values (hipcub radix sort, rtw_sort.hip).  With tmp == nullptr
// only sets *tmp_bytes.
hipError_t sort_pairs_desc(const uint32_t* keys_in, uint32_t* keys_out, const uint32_t* vals_in, uint32_t* vals_out,
                           int n, void* tmp, size_t* tmp_bytes, hipStream_t stream);

}  // namespace rtw
