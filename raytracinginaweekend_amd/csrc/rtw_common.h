// rtw_common.h -- shared host-side helpers of librtw.so (error reporting).
#pragma once

#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

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

// The render kernel's surface-area-heuristic tree over n leaf boxes (lo/hi: 3 floats per leaf),
// children encoded as in rtw_bvh_node (>= 0 node, < 0 leaf -1 - index).  *depth = nodes on the
// longest root-to-leaf path (rtw_sah.cpp).
int sah_build(const float* lo, const float* hi, int32_t n, std::vector<rtw_bvh_node>& nodes, int32_t* root, int* depth);
// The same with spatial splits (rtw_sah.cpp): tri = 9 floats per leaf (vertices; x = NaN: not a
// triangle, cut as a box), leaf_km = {k, m} per leaf (k < 0: never hits), at most budget x n extra
// references.  Node boxes are the unions of the references' clipped boxes below (rounded outward);
// km = 2 floats per node, the maxima of the leaf constants below.
int sah_build_split(const float* lo, const float* hi, const float* tri, const float* leaf_km, int32_t n, double budget,
                    std::vector<rtw_bvh_node>& nodes, std::vector<float>& km, int32_t* root, int* depth,
                    int depth_cap = 0);

}  // namespace rtw
