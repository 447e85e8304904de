// dn_internal.hpp — shared declarations of the native library (not part of the C-ABI).
#pragma once

#include "dn_shamir.h"

namespace dn {
// Record a thread-local error message and return `code` (printf-style).
int set_error(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
}  // namespace dn
