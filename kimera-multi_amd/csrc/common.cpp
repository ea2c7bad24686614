// common.cpp — error state and version entry points of the C ABI.
#include "common.h"

namespace kmx {
static thread_local std::string g_err;
void set_error(const std::string& msg) { g_err = msg; }
int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}
}  // namespace kmx

extern "C" const char* kmx_last_error(void) { return kmx::g_err.c_str(); }
extern "C" int kmx_abi_version(void) { return KMX_ABI_VERSION; }
extern "C" int kmx_device_count(int* out) {
  if (!out) return kmx::fail(KMX_EINVAL, "null out");
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  *out = (e == hipSuccess) ? n : 0;
  return KMX_OK;
}
