// common.h — internal helpers shared by the dpgo and LCD halves of libkmx.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdio>
#include <string>

#include "kmx_abi.h"

namespace kmx {
void set_error(const std::string& msg);
int fail(int code, const std::string& msg);
}  // namespace kmx

#define KMX_HIP(call)                                                        \
  do {                                                                       \
    hipError_t _e = (call);                                                  \
    if (_e != hipSuccess)                                                    \
      return kmx::fail(KMX_EHIP, std::string(#call) + ": " +                 \
                                     hipGetErrorString(_e));                 \
  } while (0)

#define KMX_CHECK(cond, code, msg)                  \
  do {                                              \
    if (!(cond)) return kmx::fail((code), (msg));   \
  } while (0)

// Exceptions never cross the ABI.
#define KMX_GUARD_BEGIN try {
#define KMX_GUARD_END                                                   \
  }                                                                     \
  catch (const std::bad_alloc&) {                                       \
    return kmx::fail(KMX_ENOMEM, "host allocation failed");             \
  }                                                                     \
  catch (const std::exception& ex) {                                    \
    return kmx::fail(KMX_EINVAL, ex.what());                            \
  }
