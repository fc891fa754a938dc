// bdpt_err.h — the thread-local message behind bdpt_last_error() (defined in bdpt_hip.hip).
#pragma once

#include <string>

namespace bdpt {
extern thread_local std::string g_err;
}  // namespace bdpt
