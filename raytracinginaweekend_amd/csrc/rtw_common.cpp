// rtw_common.cpp -- error reporting shared by every C entry point of librtw.so.
#include "rtw_common.h"

namespace rtw {

namespace {
thread_local std::string g_last_error;
}

void set_error(const std::string& msg) { g_last_error = msg; }

int fail(int code, const std::string& msg) {
    g_last_error = msg;
    return code;
}

const char* last_error() { return g_last_error.c_str(); }

}  // namespace rtw

extern "C" RTW_API const char* rtw_last_error(void) { return rtw::last_error(); }
extern "C" RTW_API int rtw_version(void) { return RTW_ABI_VERSION; }
