// Grow-only device buffers and a named fp32 parameter store (host orchestration).
#pragma once
#include <map>
#include <string>
#include <vector>
#include "common.h"

namespace janus {

struct DevMem {
  void* p = nullptr;
  size_t n = 0;
  DevMem() = default;
  DevMem(const DevMem&) = delete;
  DevMem& operator=(const DevMem&) = delete;
  DevMem(DevMem&& o) noexcept : p(o.p), n(o.n) { o.p = nullptr; o.n = 0; }
  ~DevMem() {
    if (p) (void)hipFree(p);
  }
  // (Re)allocate to at least `bytes`; hipFree synchronises the device first.
  void ensure(size_t bytes) {
    if (bytes <= n) return;
    if (p) JANUS_HIP(hipFree(p));
    p = nullptr;
    n = 0;
    JANUS_HIP(hipMalloc(&p, bytes < 256 ? 256 : bytes));
    n = bytes;
  }
  template <class T> T* as() const { return static_cast<T*>(p); }
};

// fp32 parameters uploaded by name (PyTorch / HF checkpoint naming).
struct ParamStore {
  std::map<std::string, DevMem> f32;
  std::map<std::string, int64_t> numel;
  void set(const std::string& name, const float* host, int64_t count) {
    DevMem& m = f32[name];
    m.ensure(sizeof(float) * count);
    JANUS_HIP(hipMemcpy(m.p, host, sizeof(float) * count, hipMemcpyHostToDevice));
    numel[name] = count;
  }
  bool has(const std::string& name) const { return f32.count(name) != 0; }
  const float* get(const std::string& name, int64_t expect) const {
    auto it = f32.find(name);
    JANUS_CHECK(it != f32.end(), "missing parameter '" + name + "'");
    JANUS_CHECK(expect < 0 || numel.at(name) == expect,
                "parameter '" + name + "' has " + std::to_string(numel.at(name)) +
                    " elements, expected " + std::to_string(expect));
    return it->second.as<float>();
  }
};

}  // namespace janus
