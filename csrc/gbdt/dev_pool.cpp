// Process-wide caching allocator for device memory (the GBDT engine's DevBuf).
//
// A fit allocates ~2.5 GB of device buffers for an 11M-row dataset (bins, scores,
// gradients, row permutations, histogram slabs) and frees them at the end;
// hipMalloc / hipFree of buffers that size cost milliseconds each and hipFree
// synchronises the device. An executor that fits repeatedly (Spark tasks,
// hyper-parameter search, numBatches, the benchmark) reuses the same sizes, so
// freed blocks are cached per device and handed back to the next request of a
// similar size. Reuse is safe across streams because Free() first waits for
// the device to go idle - the same ordering hipFree gives - and frees only
// happen when a dataset or booster is destroyed.
//
// SML_DEV_POOL_MB caps the cached (not live) bytes (default 32768); 0 turns
// caching off. An allocation that fails with out-of-memory trims the cache and
// retries once.
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <map>
#include <mutex>
#include <stdexcept>
#include <string>
#include <unordered_map>

#include "hip_common.h"

namespace sml {
namespace {

struct Pool {
  std::mutex mu;
  std::unordered_map<int, std::multimap<size_t, void*>> free_blocks;  // device -> size -> block
  size_t cached = 0;
  size_t live = 0;
  int64_t hits = 0, misses = 0;
  size_t cap = 0;
  bool cap_read = false;

  size_t Cap() {
    if (!cap_read) {
      cap_read = true;
      const char* e = std::getenv("SML_DEV_POOL_MB");
      cap = static_cast<size_t>(e ? std::atoll(e) : 32768) << 20;
    }
    return cap;
  }
  void TrimLocked(int dev) {
    auto it = free_blocks.find(dev);
    if (it == free_blocks.end()) return;
    int cur = -1;
    (void)hipGetDevice(&cur);
    if (cur != dev) (void)hipSetDevice(dev);
    for (auto& kv : it->second) {
      (void)hipFree(kv.second);
      cached -= kv.first;
    }
    it->second.clear();
    if (cur != dev && cur >= 0) (void)hipSetDevice(cur);
  }
};

Pool& P() {
  static Pool* p = new Pool();  // never destroyed: blocks may be freed during interpreter teardown
  return *p;
}

size_t RoundUp(size_t b) {
  constexpr size_t kSmall = 64 << 10, kLarge = 2 << 20;
  if (b <= kSmall) return kSmall;
  if (b < (32u << 20)) return (b + kSmall - 1) / kSmall * kSmall;
  return (b + kLarge - 1) / kLarge * kLarge;
}

}  // namespace

void* DevPoolAlloc(size_t bytes, size_t* granted) {
  if (bytes == 0) { *granted = 0; return nullptr; }
  int dev = 0;
  SML_HIP_CHECK(hipGetDevice(&dev));
  const size_t want = RoundUp(bytes);
  Pool& p = P();
  {
    std::lock_guard<std::mutex> lk(p.mu);
    auto& fl = p.free_blocks[dev];
    auto it = fl.lower_bound(want);
    // best fit, but never hand out a block more than 1/8 larger than asked (keeps big blocks for big asks)
    if (it != fl.end() && it->first <= want + want / 8) {
      void* ptr = it->second;
      *granted = it->first;
      p.cached -= it->first;
      p.live += it->first;
      fl.erase(it);
      ++p.hits;
      return ptr;
    }
    ++p.misses;
  }
  void* ptr = nullptr;
  hipError_t e = hipMalloc(&ptr, want);
  if (e == hipErrorOutOfMemory || e == hipErrorMemoryAllocation) {
    (void)hipGetLastError();
    std::lock_guard<std::mutex> lk(p.mu);
    (void)hipDeviceSynchronize();
    p.TrimLocked(dev);
    e = hipMalloc(&ptr, want);
  }
  if (e != hipSuccess)
    throw std::runtime_error(std::string("HIP error: ") + hipGetErrorString(e) + " (hipMalloc of " +
                             std::to_string(want) + " bytes)");
  std::lock_guard<std::mutex> lk(p.mu);
  p.live += want;
  *granted = want;
  return ptr;
}

void DevPoolFree(void* ptr, size_t granted) {
  if (!ptr) return;
  Pool& p = P();
  int dev = 0;
  if (hipPointerAttribute_t a; hipPointerGetAttributes(&a, ptr) == hipSuccess) dev = a.device;
  else (void)hipGetLastError();
  // work still queued on any stream may read this block: wait, as hipFree would
  (void)hipDeviceSynchronize();
  std::lock_guard<std::mutex> lk(p.mu);
  p.live -= granted;
  if (p.cached + granted > p.Cap()) {
    (void)hipFree(ptr);
    return;
  }
  p.free_blocks[dev].emplace(granted, ptr);
  p.cached += granted;
}

void DevPoolTrim() {
  Pool& p = P();
  (void)hipDeviceSynchronize();
  std::lock_guard<std::mutex> lk(p.mu);
  for (auto& kv : p.free_blocks) p.TrimLocked(kv.first);
}

DevPoolStats DevPoolGetStats() {
  Pool& p = P();
  std::lock_guard<std::mutex> lk(p.mu);
  return DevPoolStats{p.cached, p.live, p.hits, p.misses};
}

}  // namespace sml
