// Process-wide cache of large host blocks for the per-row vectors of a Dataset (labels, weights, initial
// scores).
//
// An 11M-row fit allocates a fresh 44 MB label vector, zero-fills it, copies the labels over it and returns it
// to the OS at the end of the fit: ~11.9k first-touch page faults on the way in and an munmap on the way out,
// measured at ~4 ms of dataset creation and ~4 ms of dataset teardown per bench step (profiles/r6, pass 15).
// Fits in one process (Spark tasks, hyper-parameter search, the benchmark) ask for the same sizes again, so
// blocks of >= 1 MiB are kept here (best fit, at most 1/8 larger than asked) and handed back already
// faulted in. SML_HOST_POOL_MB caps the cached bytes (default 4096; 0 turns caching off).
//
// PooledVector<T> is a std::vector with this allocator whose value-less construction leaves elements
// default-initialised (no zero fill): a caller that resizes and then overwrites every element pays one pass
// over the memory instead of two.
#pragma once
#include <cstddef>
#include <cstdlib>
#include <map>
#include <mutex>
#include <new>
#include <utility>
#include <vector>

namespace sml {

class HostBlockPool {
 public:
  static constexpr size_t kMinBytes = size_t(1) << 20;

  static HostBlockPool& Get() {
    static HostBlockPool* p = new HostBlockPool();  // never destroyed: vectors may die during teardown
    return *p;
  }
  void* Alloc(size_t bytes) {
    {
      std::lock_guard<std::mutex> lk(mu_);
      auto it = free_.lower_bound(bytes);
      if (it != free_.end() && it->first <= bytes + bytes / 8) {
        // the block keeps its own size: Free() is told the requested size, so record the grant
        void* p = it->second;
        granted_[p] = it->first;
        cached_ -= it->first;
        free_.erase(it);
        return p;
      }
    }
    void* p = std::malloc(bytes);
    if (!p) throw std::bad_alloc();
    std::lock_guard<std::mutex> lk(mu_);
    granted_[p] = bytes;
    return p;
  }
  void Free(void* p) {
    if (!p) return;
    std::unique_lock<std::mutex> lk(mu_);
    auto g = granted_.find(p);
    const size_t size = g == granted_.end() ? 0 : g->second;
    if (g != granted_.end()) granted_.erase(g);
    if (size == 0 || cached_ + size > Cap()) {
      lk.unlock();
      std::free(p);
      return;
    }
    free_.emplace(size, p);
    cached_ += size;
  }
  size_t cached_bytes() {
    std::lock_guard<std::mutex> lk(mu_);
    return cached_;
  }

 private:
  size_t Cap() {
    if (!cap_read_) {
      cap_read_ = true;
      const char* e = std::getenv("SML_HOST_POOL_MB");
      cap_ = static_cast<size_t>(e ? std::atoll(e) : 4096) << 20;
    }
    return cap_;
  }
  std::mutex mu_;
  std::multimap<size_t, void*> free_;
  std::map<void*, size_t> granted_;
  size_t cached_ = 0, cap_ = 0;
  bool cap_read_ = false;
};

template <class T>
struct PooledAllocator {
  using value_type = T;
  PooledAllocator() noexcept = default;
  template <class U>
  PooledAllocator(const PooledAllocator<U>&) noexcept {}
  T* allocate(size_t n) {
    const size_t bytes = n * sizeof(T);
    if (bytes >= HostBlockPool::kMinBytes) return static_cast<T*>(HostBlockPool::Get().Alloc(bytes));
    return static_cast<T*>(::operator new(bytes));
  }
  void deallocate(T* p, size_t n) noexcept {
    if (n * sizeof(T) >= HostBlockPool::kMinBytes) HostBlockPool::Get().Free(p);
    else ::operator delete(p);
  }
  // value-less construction default-initialises (no zero fill for arithmetic T)
  template <class U>
  void construct(U* p) noexcept(noexcept(::new (static_cast<void*>(p)) U)) {
    ::new (static_cast<void*>(p)) U;
  }
  template <class U, class... Args>
  void construct(U* p, Args&&... args) {
    ::new (static_cast<void*>(p)) U(std::forward<Args>(args)...);
  }
  template <class U>
  bool operator==(const PooledAllocator<U>&) const noexcept { return true; }
  template <class U>
  bool operator!=(const PooledAllocator<U>&) const noexcept { return false; }
};

template <class T>
using PooledVector = std::vector<T, PooledAllocator<T>>;

}  // namespace sml
