// Small HIP helpers shared by the native kernels (gfx950 / wave64 only).
#pragma once
#include <hip/hip_runtime.h>

#include <stdexcept>
#include <string>

#define SML_HIP_CHECK(expr)                                                                 \
  do {                                                                                      \
    hipError_t _e = (expr);                                                                 \
    if (_e != hipSuccess)                                                                   \
      throw std::runtime_error(std::string("HIP error: ") + hipGetErrorString(_e) + " at " + \
                               __FILE__ + ":" + std::to_string(__LINE__) + " (" #expr ")"); \
  } while (0)

namespace sml {

constexpr int kWave = 64;

// Caching device allocator shared by every engine buffer of the process (dev_pool.cpp).
void* DevPoolAlloc(size_t bytes, size_t* granted);
void DevPoolFree(void* p, size_t granted);
void DevPoolTrim();
struct DevPoolStats {
  size_t cached_bytes, live_bytes;
  int64_t hits, misses;
};
DevPoolStats DevPoolGetStats();

template <class T>
struct DevBuf {
  T* p = nullptr;
  size_t n = 0;
  size_t granted = 0;
  DevBuf() = default;
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
  ~DevBuf() { release(); }
  void alloc(size_t count) {
    if (count <= n && p) return;
    release();
    if (count) p = static_cast<T*>(DevPoolAlloc(sizeof(T) * count, &granted));
    n = count;
  }
  void release() {
    if (p) DevPoolFree(p, granted);
    p = nullptr;
    n = 0;
    granted = 0;
  }
  T* get() const { return p; }
};

#if defined(__HIPCC__)
__device__ __forceinline__ int ceil_div_i(int a, int b) { return (a + b - 1) / b; }

// inclusive wave64 scan (double)
__device__ __forceinline__ double wave_incl_scan(double v, int lane) {
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    double o = __shfl_up(v, off, 64);
    if (lane >= off) v += o;
  }
  return v;
}
#endif  // __HIPCC__

}  // namespace sml
