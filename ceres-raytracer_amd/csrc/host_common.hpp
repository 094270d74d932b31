// host_common.hpp -- error reporting shared by the C-ABI translation units.
#pragma once
#include <cstdarg>
#include <cstdio>

namespace ceres {

// Per-thread message behind ceres_last_error(); defined in render_hip.hip.
char* error_buffer();
constexpr int kErrorBufferSize = 512;

inline int set_error(int code, const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    std::vsnprintf(error_buffer(), kErrorBufferSize, fmt, ap);
    va_end(ap);
    return code;
}

}  // namespace ceres
