// rtw_common.h -- shared host-side helpers of librtw.so (error reporting).
#pragma once

#include <string>

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

}  // namespace rtw
