// jr_error.h — the C-ABI error convention (host-only, no HIP): every entry
// point returns a jr_status; the message of the last failure on the calling
// thread is returned by jr_last_error().  Used by the HIP sources through
// jr_common.h and by the host-only sources (TFRecord / Example parsing)
// directly, so those build without HIP (the AddressSanitizer build).
#pragma once
#include <string>

#include "../../include/jr.h"

#define JR_API extern "C" __attribute__((visibility("default")))

namespace jr {
void set_error(const std::string& msg);
int fail(int status, const std::string& msg);
}  // namespace jr
