// Direct NHWC grouped / depthwise convolution (module _nn): the convs the implicit-GEMM kernels do not
// fit - depthwise (one input channel per group) and narrow groups, where a 64-wide MFMA tile along N or
// K would be mostly padding. One thread per (output pixel, output channel): consecutive threads take
// consecutive output channels of one pixel, so for depthwise layers (channel g reads input channel g)
// the input taps are read as contiguous channel runs; weights [Cout][R][S][Cg] stay in L1/L2. fp32
// accumulation, bias / ReLU / residual epilogue as the fused conv (relu 1 before the add, 2 after).
#include <hip/hip_runtime.h>

#include <cstdint>

#include "nn_ops.h"

namespace smlnn {
namespace {

template <class T>
__global__ __launch_bounds__(256) void group_conv_kernel(GroupConvArgs a) {
  const T* __restrict__ x = static_cast<const T*>(a.x);
  const T* __restrict__ w = static_cast<const T*>(a.w);
  const T* __restrict__ res = static_cast<const T*>(a.res);
  T* __restrict__ y = static_cast<T*>(a.y);
  const int Cg = a.C / a.groups, Ng = a.Cout / a.groups;
  const int64_t total = static_cast<int64_t>(a.B) * a.OH * a.OW * a.Cout;
  for (int64_t idx = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; idx < total;
       idx += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const int co = static_cast<int>(idx % a.Cout);
    const int64_t m = idx / a.Cout;
    const int ow = static_cast<int>(m % a.OW);
    const int64_t t = m / a.OW;
    const int oh = static_cast<int>(t % a.OH);
    const int b = static_cast<int>(t / a.OH);
    const int g = co / Ng;
    const int ih0 = oh * a.stride_h - a.pad_h, iw0 = ow * a.stride_w - a.pad_w;
    const T* wr = w + static_cast<int64_t>(co) * a.R * a.S * Cg;
    float acc = 0.f;
    for (int r = 0; r < a.R; ++r) {
      const int ih = ih0 + r * a.dil_h;
      if (ih < 0 || ih >= a.H) continue;
      for (int s = 0; s < a.S; ++s) {
        const int iw = iw0 + s * a.dil_w;
        if (iw < 0 || iw >= a.W) continue;
        const T* xp = x + ((static_cast<int64_t>(b) * a.H + ih) * a.W + iw) * a.C + g * Cg;
        const T* wp = wr + (r * a.S + s) * Cg;
        for (int c = 0; c < Cg; ++c) acc += static_cast<float>(xp[c]) * static_cast<float>(wp[c]);
      }
    }
    if (a.bias) acc += a.bias[co];
    if (a.relu == 1 || (a.relu == 2 && !res)) acc = fmaxf(acc, 0.f);
    if (res) {
      acc = static_cast<float>(static_cast<T>(acc)) + static_cast<float>(res[idx]);  // the unfused graph rounds first
      if (a.relu == 2) acc = fmaxf(acc, 0.f);
    }
    y[idx] = static_cast<T>(acc);
  }
}

}  // namespace

int GroupConv(const GroupConvArgs& a, int dtype, void* stream) {
  if (a.groups <= 0 || a.C % a.groups != 0 || a.Cout % a.groups != 0 || a.OH <= 0 || a.OW <= 0 || a.B <= 0) return -1;
  const int64_t total = static_cast<int64_t>(a.B) * a.OH * a.OW * a.Cout;
  const int grid = static_cast<int>(std::min<int64_t>((total + 255) / 256, 1 << 16));
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (dtype == 0) hipLaunchKernelGGL(group_conv_kernel<float>, dim3(grid), dim3(256), 0, st, a);
  else if (dtype == 1) hipLaunchKernelGGL(group_conv_kernel<_Float16>, dim3(grid), dim3(256), 0, st, a);
  else if (dtype == 2) hipLaunchKernelGGL(group_conv_kernel<__bf16>, dim3(grid), dim3(256), 0, st, a);
  else return -1;
  return hipGetLastError() == hipSuccess ? 0 : -3;
}

}  // namespace smlnn
