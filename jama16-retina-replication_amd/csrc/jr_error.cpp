// jr_error.cpp — thread-local last-error text behind jr_last_error().
#include "jr_error.h"

namespace jr {

static thread_local std::string g_last_error;

void set_error(const std::string& msg) { g_last_error = msg; }

int fail(int status, const std::string& msg) {
  g_last_error = msg;
  return status;
}

}  // namespace jr

JR_API const char* jr_last_error(void) { return jr::g_last_error.c_str(); }
