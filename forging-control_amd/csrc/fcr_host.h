// fcr_host.h — host-side helpers shared by the C-ABI translation units (fcr_abi.hip, fcr_rows.hip).
#pragma once
#include <hip/hip_runtime.h>

#include "fcr.h"

namespace fcr {

// Record a message in the thread-local last-error buffer (fcr_last_error) and return `code`.
int fail(int code, const char *fmt, ...) __attribute__((format(printf, 2, 3)));

// FCR_OK, or FCR_EHIP with the launch error of the kernel just enqueued.
int launch_check(const char *what);

}  // namespace fcr
