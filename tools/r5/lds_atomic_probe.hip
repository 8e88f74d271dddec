// LDS atomic throughput probe (round 5): wave-wide ds_add_u64 / ds_add_u32 / ds_add_f32 rates on one
// 1024-thread block per CU, conflict-free addresses (lane-consecutive words, as the histogram kernels' rotated
// layout) and random-bin addresses (one 256-bin row per lane group, as a real feature). Prints lane-atomics
// per clock per CU (clock from the kernel's shader-clock delta).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { std::printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

constexpr int kThr = 1024, kIters = 512;

template <int kMode, bool kRand>
__global__ __launch_bounds__(kThr) void probe(unsigned long long* out, long long* clk) {
  __shared__ unsigned long long sh[16384];  // 128 KB
  const int tid = threadIdx.x;
  for (int i = tid; i < 16384; i += kThr) sh[i] = 0;
  __syncthreads();
  const long long t0 = static_cast<long long>(__builtin_amdgcn_s_memtime());
  uint32_t x = 2463534242u ^ (tid * 2654435761u) ^ blockIdx.x;
#pragma unroll 8
  for (int it = 0; it < kIters; ++it) {
    int w;
    if constexpr (kRand) {
      x ^= x << 13; x ^= x >> 17; x ^= x << 5;
      w = ((x & 255) * 32 + (tid & 31)) & 8191;  // bin-major with 32 lane columns (the rotated layout's spread)
    } else {
      w = (tid + it * kThr) & 8191;
    }
    if constexpr (kMode == 0) atomicAdd(&sh[w], 3ull);
    else if constexpr (kMode == 1) atomicAdd(reinterpret_cast<unsigned*>(sh) + w, 3u);
    else atomicAdd(reinterpret_cast<float*>(sh) + w, 1.0f);
  }
  __syncthreads();
  const long long t1 = static_cast<long long>(__builtin_amdgcn_s_memtime());
  if (tid == 0) clk[blockIdx.x] = t1 - t0;
  unsigned long long acc = 0;
  for (int i = tid; i < 16384; i += kThr) acc += sh[i];
  if (acc == 0x12345) out[blockIdx.x] = acc;  // keeps the adds live
}

template <int kMode, bool kRand>
int run(const char* name, int blocks, unsigned long long* out, long long* clk) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  hipLaunchKernelGGL((probe<kMode, kRand>), dim3(blocks), dim3(kThr), 0, 0, out, clk);
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(a));
  hipLaunchKernelGGL((probe<kMode, kRand>), dim3(blocks), dim3(kThr), 0, 0, out, clk);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  std::vector<long long> c(blocks);
  CK(hipMemcpy(c.data(), clk, sizeof(long long) * blocks, hipMemcpyDeviceToHost));
  double mc = 0;
  for (long long v : c) mc += static_cast<double>(v);
  mc /= blocks;
  const double lanes = static_cast<double>(kThr) * kIters;  // lane-atomics per block
  std::printf("%-28s %8.1f us  %6.2f lane-atomics/clock/CU  (%.0f clocks per block, %.2f Glane-atomics/s total)\n",
              name, ms * 1e3, lanes / mc, mc, lanes * blocks / (ms * 1e-3) / 1e9);
  CK(hipEventDestroy(a)); CK(hipEventDestroy(b));
  return 0;
}

int main() {
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  unsigned long long* out; long long* clk;
  CK(hipMalloc(&out, sizeof(unsigned long long) * cus));
  CK(hipMalloc(&clk, sizeof(long long) * cus));
  std::printf("CUs %d, one %d-thread block per CU, %d atomics per thread\n", cus, kThr, kIters);
  if (run<0, false>("ds_add_u64 conflict-free", cus, out, clk)) return 1;
  if (run<1, false>("ds_add_u32 conflict-free", cus, out, clk)) return 1;
  if (run<2, false>("ds_add_f32 conflict-free", cus, out, clk)) return 1;
  if (run<0, true>("ds_add_u64 random bins", cus, out, clk)) return 1;
  if (run<1, true>("ds_add_u32 random bins", cus, out, clk)) return 1;
  CK(hipFree(out)); CK(hipFree(clk));
  return 0;
}
