// Error handling shared by the engine and the C ABI.
#pragma once
#include <hip/hip_runtime.h>

#include <stdexcept>
#include <string>

#include "pocket_tts.h"

namespace ptts {

struct Error : std::runtime_error {
  int code;
  Error(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

#define PTTS_HIP(expr)                                                                              \
  do {                                                                                              \
    hipError_t e_ = (expr);                                                                         \
    if (e_ != hipSuccess)                                                                           \
      throw ::ptts::Error(PTTS_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(e_) + " (" + \
                                            __FILE__ + ":" + std::to_string(__LINE__) + ")");       \
  } while (0)

#define PTTS_REQUIRE(cond, msg)                                         \
  do {                                                                  \
    if (!(cond)) throw ::ptts::Error(PTTS_ERR_INVALID, std::string(msg)); \
  } while (0)

// model-config check (config.cpp): throws Error(PTTS_ERR_INVALID) naming the first key that
// differs from the compiled b6369a24 dimensions; a null or empty path is accepted
void check_model_config(const char* path);

}  // namespace ptts
