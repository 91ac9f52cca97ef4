// errors.hpp — thread-local last-error message shared by every C entry point (mpccbf_last_error).
#pragma once

#include <string>

namespace mpccbf {
// Records msg as the calling thread's last error and returns code (for `return set_error(...)`).
int set_error(int code, const std::string& msg);
}  // namespace mpccbf
