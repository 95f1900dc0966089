// api_common.h -- error plumbing shared by the C-ABI translation units.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>

#include "../../include/amr.h"

namespace amr {
int fail(int code, const std::string& msg);   // sets amr_last_error(), returns code
int64_t dtype_size(int dtype);                // bytes per sample, 0 = unknown
// device + stream a *_device call on `plan` runs on (plan NULL: current device, null stream)
int plan_stream(amr_psk_plan* plan, int* dev, hipStream_t* st);
}  // namespace amr

#define HIP_TRY(expr)                                                                              \
  do {                                                                                             \
    hipError_t e_ = (expr);                                                                        \
    if (e_ != hipSuccess)                                                                          \
      return ::amr::fail(e_ == hipErrorOutOfMemory ? AMR_E_NOMEM : AMR_E_HIP,                      \
                         std::string(#expr) + ": " + hipGetErrorString(e_));                      \
  } while (0)
