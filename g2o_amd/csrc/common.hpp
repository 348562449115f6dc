// Shared host helpers for libg2o_hip: HIP error handling and device buffers.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <stdexcept>
#include <string>
#include <vector>

namespace g2ohip {

struct DeviceError : std::runtime_error {
  using std::runtime_error::runtime_error;
};

#define HIP_CHECK(expr)                                                                                  \
  do {                                                                                                   \
    hipError_t _e = (expr);                                                                              \
    if (_e != hipSuccess)                                                                                \
      throw ::g2ohip::DeviceError(std::string(#expr) + " failed: " + hipGetErrorString(_e) + " @" +     \
                                  __FILE__ + ":" + std::to_string(__LINE__));                           \
  } while (0)

#define KERNEL_CHECK() HIP_CHECK(hipGetLastError())

// RAII device buffer (hipMalloc'd, never host-mapped).
template <typename T>
class DevBuf {
 public:
  DevBuf() = default;
  explicit DevBuf(size_t n) { resize(n); }
  ~DevBuf() { release(); }
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
  DevBuf(DevBuf&& o) noexcept : p_(o.p_), n_(o.n_) { o.p_ = nullptr; o.n_ = 0; }
  DevBuf& operator=(DevBuf&& o) noexcept {
    if (this != &o) { release(); p_ = o.p_; n_ = o.n_; o.p_ = nullptr; o.n_ = 0; }
    return *this;
  }
  void resize(size_t n) {
    if (n == n_) return;
    release();
    if (n) HIP_CHECK(hipMalloc(&p_, n * sizeof(T)));
    n_ = n;
  }
  void release() {
    if (p_) (void)hipFree(p_);
    p_ = nullptr;
    n_ = 0;
  }
  T* get() const { return p_; }
  size_t size() const { return n_; }
  size_t bytes() const { return n_ * sizeof(T); }
  // structure-time upload: completes before returning (the host source may be a temporary)
  void upload(const T* h, size_t n, hipStream_t s) {
    resize(n);
    if (n) {
      HIP_CHECK(hipMemcpyAsync(p_, h, n * sizeof(T), hipMemcpyHostToDevice, s));
      HIP_CHECK(hipStreamSynchronize(s));
    }
  }
  void upload(const std::vector<T>& v, hipStream_t s) { upload(v.data(), v.size(), s); }
  void download(T* h, size_t n, hipStream_t s) const {
    if (n) HIP_CHECK(hipMemcpyAsync(h, p_, n * sizeof(T), hipMemcpyDeviceToHost, s));
  }
  void zero(hipStream_t s) {
    if (n_) HIP_CHECK(hipMemsetAsync(p_, 0, n_ * sizeof(T), s));
  }

 private:
  T* p_ = nullptr;
  size_t n_ = 0;
};

inline unsigned grid_for(size_t n, unsigned block) { return (unsigned)((n + block - 1) / block); }

}  // namespace g2ohip
