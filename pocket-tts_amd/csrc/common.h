// Error handling shared by the engine and the C ABI.
#pragma once
#include <hip/hip_runtime.h>

#include <stdexcept>
#include <cstdlib>
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

// Measurement and tuning knobs of the tools/ scripts (PTTS_OVR tile overrides, per-op caps,
// probes): read only by a -DPTTS_PROBES build (make -C pocket-tts_amd probes); the product
// library ignores the environment.
inline const char* probe_env(const char* name) {
#ifdef PTTS_PROBES
  return std::getenv(name);
#else
  (void)name;
  return nullptr;
#endif
}

// model-config check (config.cpp): throws Error(PTTS_ERR_INVALID) naming the first key that
// differs from the compiled b6369a24 dimensions; a null or empty path is accepted
void check_model_config(const char* path);

}  // namespace ptts
