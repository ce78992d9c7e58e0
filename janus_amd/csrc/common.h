// Shared helpers for the janus HIP library (gfx950 / CDNA4 only).
//
// Error model: every extern "C" entry point returns int (0 = OK) and never lets a
// C++ exception cross the ABI; the message is kept per thread and read back with
// janus_last_error().
#pragma once

#include <hip/hip_runtime.h>
#include <hip/hip_fp16.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <stdexcept>

namespace janus {

void set_error(const std::string& msg);

// Kernel-geometry A/B switches (JANUS_* environment variables) are read only by builds made
// with -DJANUS_AB_KNOBS (the A/B libraries the tools build beside the product); the product
// library takes no tuning from the environment and always runs the measured defaults.
inline const char* ab_env(const char* name) {
#ifdef JANUS_AB_KNOBS
  return std::getenv(name);
#else
  (void)name;
  return nullptr;
#endif
}

// CUs a stream may dispatch to: the popcount of its CU mask (hipExtStreamGetCUMask; all
// CUs for an unmasked stream). Cached per stream handle. Persistent / per-CU grids size
// themselves with it, so a kernel on a half-GPU partition runs one round, not two.
int stream_cu_count(hipStream_t s);

struct Error : std::runtime_error {
  using std::runtime_error::runtime_error;
};

#define JANUS_HIP(expr)                                                          \
  do {                                                                           \
    hipError_t e_ = (expr);                                                      \
    if (e_ != hipSuccess)                                                        \
      throw ::janus::Error(std::string(#expr) + ": " + hipGetErrorString(e_) +   \
                           " (" + __FILE__ + ":" + std::to_string(__LINE__) + ")"); \
  } while (0)

#define JANUS_CHECK(cond, msg)                                                   \
  do {                                                                           \
    if (!(cond)) throw ::janus::Error(std::string(msg));                         \
  } while (0)

// Wrap an entry-point body: map exceptions to status codes.
template <class F>
inline int guarded(F&& f) {
  try {
    f();
    return 0;
  } catch (const std::exception& e) {
    set_error(e.what());
    return 1;
  } catch (...) {
    set_error("unknown C++ exception");
    return 1;
  }
}

// Launch check after <<<>>> (launch config errors surface here, not faults).
#define JANUS_LAUNCH_CHECK() JANUS_HIP(hipGetLastError())

constexpr int kWave = 64;  // CDNA wavefront width (never 32)

__host__ __device__ inline int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

}  // namespace janus
