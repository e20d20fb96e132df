// errors.cpp — thread-local text of the last failure (grt_last_error, include/grt_api.h).
#include <string>

#include "host_internal.h"

namespace grt_host {
static thread_local std::string g_last_error;
void set_error(const std::string& msg) { g_last_error = msg; }
}  // namespace grt_host

extern "C" const char* grt_last_error(void) { return grt_host::g_last_error.c_str(); }
