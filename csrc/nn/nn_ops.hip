// Fused epilogue / post-processing kernels for the ONNX executor on gfx950.
//
// The executor runs convolutions/GEMMs through the library path and fuses
// everything elementwise that follows them into one pass over the activation
// (SURVEY §2.4 K15): y = act(x * scale[c] + shift[c] + residual), and the
// pre-activation ResNet pattern "sum = a + b; out = relu(bn(sum))" with both
// results written in the same pass. Tensors are channels-last (NHWC) or NCHW;
// 8 elements per thread (one 16-B load for fp16/bf16, two for fp32), the
// channel vector of 8 consecutive NHWC elements is loaded once per thread.
#include <hip/hip_bf16.h>
#include <hip/hip_fp16.h>
#include <hip/hip_runtime.h>
#include <type_traits>

#include <algorithm>
#include <cstdint>
#include <stdexcept>
#include <string>

#include "nn_ops.h"

#define NN_HIP_CHECK(e)                                                                                \
  do {                                                                                                 \
    hipError_t _e = (e);                                                                               \
    if (_e != hipSuccess) throw std::runtime_error(std::string("HIP error: ") + hipGetErrorString(_e)); \
  } while (0)

namespace smlnn {
namespace {

constexpr int kThreads = 256;
constexpr int kVec = 8;

template <typename T> __device__ __forceinline__ float ld(const T* p, int64_t i);
template <> __device__ __forceinline__ float ld<float>(const float* p, int64_t i) { return p[i]; }
template <> __device__ __forceinline__ float ld<__half>(const __half* p, int64_t i) { return __half2float(p[i]); }
template <> __device__ __forceinline__ float ld<__hip_bfloat16>(const __hip_bfloat16* p, int64_t i) {
  return __bfloat162float(p[i]);
}
template <typename T> __device__ __forceinline__ T cv(float v);
template <> __device__ __forceinline__ float cv<float>(float v) { return v; }
template <> __device__ __forceinline__ __half cv<__half>(float v) { return __float2half(v); }
template <> __device__ __forceinline__ __hip_bfloat16 cv<__hip_bfloat16>(float v) { return __float2bfloat16(v); }

template <typename T>
struct alignas(16) Vec8 {
  T v[kVec];
};

__device__ __forceinline__ float act_fn(float x, int act, float alpha) {
  if (act == 1) return fmaxf(x, 0.f);
  if (act == 2) return x > 0.f ? x : alpha * x;          // leaky relu
  if (act == 3) return 1.f / (1.f + __expf(-x));        // sigmoid
  if (act == 4) return fminf(fmaxf(x, 0.f), alpha);     // clip(0, alpha) (relu6 when alpha = 6)
  return x;
}

// channel of element i
__device__ __forceinline__ int chan(int64_t i, int C, int HW, int nhwc) {
  return nhwc ? static_cast<int>(i % C) : static_cast<int>((i / HW) % C);
}

template <typename T>
__global__ __launch_bounds__(kThreads) void affine_act_kernel(const T* __restrict__ x, int64_t n, int C, int HW,
                                                              int nhwc, const float* __restrict__ scale,
                                                              const float* __restrict__ shift,
                                                              const T* __restrict__ res, int act, float alpha,
                                                              T* __restrict__ y) {
  const int64_t base = (static_cast<int64_t>(blockIdx.x) * kThreads + threadIdx.x) * kVec;
  if (base >= n) return;
  const bool full = base + kVec <= n && (!nhwc || C % kVec == 0) && (nhwc || HW % kVec == 0);
  if (full) {
    Vec8<T> a = *reinterpret_cast<const Vec8<T>*>(x + base);
    Vec8<T> r;
    if (res) r = *reinterpret_cast<const Vec8<T>*>(res + base);
    Vec8<T> o;
    const int c0 = chan(base, C, HW, nhwc);
#pragma unroll
    for (int j = 0; j < kVec; ++j) {
      const int c = nhwc ? c0 + j : c0;
      float v = ld<T>(a.v, j);
      if (scale) v *= scale[c];
      if (shift) v += shift[c];
      if (res) v += ld<T>(r.v, j);
      o.v[j] = cv<T>(act_fn(v, act, alpha));
    }
    *reinterpret_cast<Vec8<T>*>(y + base) = o;
  } else {
    for (int64_t i = base; i < n && i < base + kVec; ++i) {
      const int c = chan(i, C, HW, nhwc);
      float v = ld<T>(x, i);
      if (scale) v *= scale[c];
      if (shift) v += shift[c];
      if (res) v += ld<T>(res, i);
      y[i] = cv<T>(act_fn(v, act, alpha));
    }
  }
}

template <typename T>
__global__ __launch_bounds__(kThreads) void add_affine_act_kernel(const T* __restrict__ a, const T* __restrict__ b,
                                                                  int64_t n, int C, int HW, int nhwc,
                                                                  const float* __restrict__ scale,
                                                                  const float* __restrict__ shift, int act,
                                                                  T* __restrict__ sum_out, T* __restrict__ act_out) {
  const int64_t base = (static_cast<int64_t>(blockIdx.x) * kThreads + threadIdx.x) * kVec;
  if (base >= n) return;
  const bool full = base + kVec <= n && (!nhwc || C % kVec == 0) && (nhwc || HW % kVec == 0);
  if (full) {
    Vec8<T> va = *reinterpret_cast<const Vec8<T>*>(a + base);
    Vec8<T> vb = *reinterpret_cast<const Vec8<T>*>(b + base);
    Vec8<T> s, o;
    const int c0 = chan(base, C, HW, nhwc);
#pragma unroll
    for (int j = 0; j < kVec; ++j) {
      const int c = nhwc ? c0 + j : c0;
      const T sv = cv<T>(ld<T>(va.v, j) + ld<T>(vb.v, j));
      s.v[j] = sv;
      o.v[j] = cv<T>(act_fn(ld<T>(&sv, 0) * scale[c] + shift[c], act, 0.f));
    }
    *reinterpret_cast<Vec8<T>*>(sum_out + base) = s;
    *reinterpret_cast<Vec8<T>*>(act_out + base) = o;
  } else {
    for (int64_t i = base; i < n && i < base + kVec; ++i) {
      const int c = chan(i, C, HW, nhwc);
      const T sv = cv<T>(ld<T>(a, i) + ld<T>(b, i));
      sum_out[i] = sv;
      act_out[i] = cv<T>(act_fn(ld<T>(&sv, 0) * scale[c] + shift[c], act, 0.f));
    }
  }
}

// K16: global average pool over HW of an NHWC tensor -> [N, C] in the input dtype (fp32 accumulation, one
// rounding); one thread per (n, c), lanes of a wave on consecutive channels (coalesced rows). The output is
// the [N, C, 1, 1] tensor the classifier head reads, so no dtype-conversion pass follows it.
template <typename T>
__global__ __launch_bounds__(kThreads) void gap_nhwc_kernel(const T* __restrict__ x, int N, int HW, int C,
                                                            T* __restrict__ out) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * kThreads + threadIdx.x;
  if (i >= static_cast<int64_t>(N) * C) return;
  const int n = static_cast<int>(i / C), c = static_cast<int>(i % C);
  const T* p = x + static_cast<int64_t>(n) * HW * C + c;
  float s = 0.f;
  for (int k = 0; k < HW; ++k) s += ld<T>(p, static_cast<int64_t>(k) * C);
  out[i] = cv<T>(s / HW);
}

// K16: max pool over an NHWC tensor (kh x kw window, stride, symmetric pads, no dilation; padded cells
// never win, as ONNX pads max pools with -inf). One thread per (output pixel, 8 channels): 16-B loads
// of consecutive channels for fp16 / bf16. C % 8 == 0 (the host checks).
// Optional epilogue y = relu?(max + shift[c]): the producing conv's bias + ReLU moved past the pool
// (x -> round(x + b), ReLU are monotone, so max commutes with them exactly) - a quarter of the writes.
// KH / KW > 0: a compile-time window (the 3x3 image-stem pool): every tap's load is issued before the first max
// (row / column clamped into the image, out-of-range taps masked), instead of one load latency per tap of the
// runtime loop.
template <typename T, int KH = 0, int KW = 0>
__global__ __launch_bounds__(kThreads) void maxpool_nhwc_kernel(const T* __restrict__ x, int N, int H, int W, int C,
                                                                int kh, int kw, int sh, int sw, int ph, int pw,
                                                                int OH, int OW, const float* __restrict__ shift,
                                                                int relu, T* __restrict__ y) {
  const int cv8 = C / kVec;
  const int64_t total = static_cast<int64_t>(N) * OH * OW * cv8;
  for (int64_t t = static_cast<int64_t>(blockIdx.x) * kThreads + threadIdx.x; t < total;
       t += static_cast<int64_t>(gridDim.x) * kThreads) {
    const int cg = static_cast<int>(t % cv8);
    int64_t r = t / cv8;
    const int ow = static_cast<int>(r % OW); r /= OW;
    const int oh = static_cast<int>(r % OH);
    const int n = static_cast<int>(r / OH);
    float m[kVec];
#pragma unroll
    for (int j = 0; j < kVec; ++j) m[j] = -INFINITY;
    const int h0 = oh * sh - ph, w0 = ow * sw - pw;
    if constexpr (KH > 0 && KW > 0) {
      Vec8<T> v[KH][KW];
#pragma unroll
      for (int i = 0; i < KH; ++i)
#pragma unroll
        for (int k = 0; k < KW; ++k) {
          const int hh = min(max(h0 + i, 0), H - 1), ww = min(max(w0 + k, 0), W - 1);
          v[i][k] = *reinterpret_cast<const Vec8<T>*>(x + ((static_cast<int64_t>(n) * H + hh) * W + ww) * C + cg * kVec);
        }
#pragma unroll
      for (int i = 0; i < KH; ++i)
#pragma unroll
        for (int k = 0; k < KW; ++k) {
          if (h0 + i < 0 || h0 + i >= H || w0 + k < 0 || w0 + k >= W) continue;
#pragma unroll
          for (int j = 0; j < kVec; ++j) m[j] = fmaxf(m[j], ld<T>(v[i][k].v, j));
        }
    }
    for (int i = 0; i < (KH > 0 ? 0 : kh); ++i) {
      const int hh = h0 + i;
      if (hh < 0 || hh >= H) continue;
      for (int k = 0; k < kw; ++k) {
        const int ww = w0 + k;
        if (ww < 0 || ww >= W) continue;
        const Vec8<T> v = *reinterpret_cast<const Vec8<T>*>(x + ((static_cast<int64_t>(n) * H + hh) * W + ww) * C +
                                                           cg * kVec);
#pragma unroll
        for (int j = 0; j < kVec; ++j) m[j] = fmaxf(m[j], ld<T>(v.v, j));
      }
    }
    if (shift) {
#pragma unroll
      for (int j = 0; j < kVec; ++j) m[j] += shift[cg * kVec + j];
    }
    if (relu) {
#pragma unroll
      for (int j = 0; j < kVec; ++j) m[j] = fmaxf(m[j], 0.f);
    }
    Vec8<T> o;
#pragma unroll
    for (int j = 0; j < kVec; ++j) o.v[j] = cv<T>(m[j]);
    *reinterpret_cast<Vec8<T>*>(y + ((static_cast<int64_t>(n) * OH + oh) * OW + ow) * C + cg * kVec) = o;
  }
}

// row softmax / argmax, one wave per row (fp32)
__global__ __launch_bounds__(kThreads) void softmax_rows_kernel(const float* __restrict__ x, int rows, int cols,
                                                                float* __restrict__ y, int64_t* __restrict__ amax) {
  const int lane = threadIdx.x & 63;
  const int r = blockIdx.x * (kThreads / 64) + (threadIdx.x >> 6);
  if (r >= rows) return;
  const float* p = x + static_cast<int64_t>(r) * cols;
  float m = -INFINITY;
  int mi = 0x7fffffff;
  for (int j = lane; j < cols; j += 64) {
    const float v = p[j];
    if (v > m || (v == m && j < mi)) { m = v; mi = j; }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const float om = __shfl_xor(m, off, 64);
    const int oi = __shfl_xor(mi, off, 64);
    if (om > m || (om == m && oi < mi)) { m = om; mi = oi; }
  }
  if (amax && lane == 0) amax[r] = mi;
  if (!y) return;
  float s = 0.f;
  for (int j = lane; j < cols; j += 64) s += __expf(p[j] - m);
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
  const float inv = 1.f / s;
  for (int j = lane; j < cols; j += 64) y[static_cast<int64_t>(r) * cols + j] = __expf(p[j] - m) * inv;
}

int Blocks(int64_t n, int per_thread) {
  const int64_t t = (n + per_thread - 1) / per_thread;
  return static_cast<int>((t + kThreads - 1) / kThreads);
}

}  // namespace

void MaxPoolNhwc(const void* x, int N, int H, int W, int C, int kh, int kw, int sh, int sw, int ph, int pw, int OH,
                 int OW, int dtype, void* y, void* stream, const float* shift, int relu) {
  if (C % kVec != 0) throw std::runtime_error("maxpool_nhwc: channels must be a multiple of 8");
  const int64_t total = static_cast<int64_t>(N) * OH * OW * (C / kVec);
  if (total <= 0) return;
  auto s = static_cast<hipStream_t>(stream);
  const int g = static_cast<int>(std::min<int64_t>((total + kThreads - 1) / kThreads, 1 << 20));
  auto launch = [&](auto tag, auto win) {
    using TT = decltype(tag);
    constexpr int K = decltype(win)::value;
    hipLaunchKernelGGL((maxpool_nhwc_kernel<TT, K, K>), dim3(g), dim3(kThreads), 0, s, static_cast<const TT*>(x), N, H,
                       W, C, kh, kw, sh, sw, ph, pw, OH, OW, shift, relu, static_cast<TT*>(y));
  };
  const bool k3 = kh == 3 && kw == 3;
  if (dtype == 1) {
    if (k3) launch(__half{}, std::integral_constant<int, 3>{});
    else launch(__half{}, std::integral_constant<int, 0>{});
  } else if (dtype == 2) {
    if (k3) launch(__hip_bfloat16{}, std::integral_constant<int, 3>{});
    else launch(__hip_bfloat16{}, std::integral_constant<int, 0>{});
  } else {
    if (k3) launch(float{}, std::integral_constant<int, 3>{});
    else launch(float{}, std::integral_constant<int, 0>{});
  }
  NN_HIP_CHECK(hipGetLastError());
}

bool NnGpuAvailable() {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) { (void)hipGetLastError(); return false; }
  return n > 0;
}

void AffineAct(const void* x, int64_t n, int C, int HW, int nhwc, const float* scale, const float* shift,
               const void* res, int act, float alpha, int dtype, void* y, void* stream) {
  if (n <= 0) return;
  auto s = static_cast<hipStream_t>(stream);
  const int g = Blocks(n, kVec);
  if (dtype == 1)
    hipLaunchKernelGGL(affine_act_kernel<__half>, dim3(g), dim3(kThreads), 0, s, static_cast<const __half*>(x), n, C,
                       HW, nhwc, scale, shift, static_cast<const __half*>(res), act, alpha, static_cast<__half*>(y));
  else if (dtype == 2)
    hipLaunchKernelGGL(affine_act_kernel<__hip_bfloat16>, dim3(g), dim3(kThreads), 0, s,
                       static_cast<const __hip_bfloat16*>(x), n, C, HW, nhwc, scale, shift,
                       static_cast<const __hip_bfloat16*>(res), act, alpha, static_cast<__hip_bfloat16*>(y));
  else
    hipLaunchKernelGGL(affine_act_kernel<float>, dim3(g), dim3(kThreads), 0, s, static_cast<const float*>(x), n, C, HW,
                       nhwc, scale, shift, static_cast<const float*>(res), act, alpha, static_cast<float*>(y));
  NN_HIP_CHECK(hipGetLastError());
}

void AddAffineAct(const void* a, const void* b, int64_t n, int C, int HW, int nhwc, const float* scale,
                  const float* shift, int act, int dtype, void* sum_out, void* act_out, void* stream) {
  if (n <= 0) return;
  auto s = static_cast<hipStream_t>(stream);
  const int g = Blocks(n, kVec);
  if (dtype == 1)
    hipLaunchKernelGGL(add_affine_act_kernel<__half>, dim3(g), dim3(kThreads), 0, s, static_cast<const __half*>(a),
                       static_cast<const __half*>(b), n, C, HW, nhwc, scale, shift, act, static_cast<__half*>(sum_out),
                       static_cast<__half*>(act_out));
  else if (dtype == 2)
    hipLaunchKernelGGL(add_affine_act_kernel<__hip_bfloat16>, dim3(g), dim3(kThreads), 0, s,
                       static_cast<const __hip_bfloat16*>(a), static_cast<const __hip_bfloat16*>(b), n, C, HW, nhwc,
                       scale, shift, act, static_cast<__hip_bfloat16*>(sum_out),
                       static_cast<__hip_bfloat16*>(act_out));
  else
    hipLaunchKernelGGL(add_affine_act_kernel<float>, dim3(g), dim3(kThreads), 0, s, static_cast<const float*>(a),
                       static_cast<const float*>(b), n, C, HW, nhwc, scale, shift, act, static_cast<float*>(sum_out),
                       static_cast<float*>(act_out));
  NN_HIP_CHECK(hipGetLastError());
}

void GapNhwc(const void* x, int N, int HW, int C, int dtype, void* out, void* stream) {
  const int64_t n = static_cast<int64_t>(N) * C;
  if (n <= 0) return;
  auto s = static_cast<hipStream_t>(stream);
  const int g = Blocks(n, 1);
  if (dtype == 1)
    hipLaunchKernelGGL(gap_nhwc_kernel<__half>, dim3(g), dim3(kThreads), 0, s, static_cast<const __half*>(x), N, HW, C,
                       static_cast<__half*>(out));
  else if (dtype == 2)
    hipLaunchKernelGGL(gap_nhwc_kernel<__hip_bfloat16>, dim3(g), dim3(kThreads), 0, s,
                       static_cast<const __hip_bfloat16*>(x), N, HW, C, static_cast<__hip_bfloat16*>(out));
  else
    hipLaunchKernelGGL(gap_nhwc_kernel<float>, dim3(g), dim3(kThreads), 0, s, static_cast<const float*>(x), N, HW, C,
                       static_cast<float*>(out));
  NN_HIP_CHECK(hipGetLastError());
}

void SoftmaxRows(const float* x, int rows, int cols, float* y, int64_t* amax, void* stream) {
  if (rows <= 0) return;
  const int g = (rows + kThreads / 64 - 1) / (kThreads / 64);
  hipLaunchKernelGGL(softmax_rows_kernel, dim3(g), dim3(kThreads), 0, static_cast<hipStream_t>(stream), x, rows, cols,
                     y, amax);
  NN_HIP_CHECK(hipGetLastError());
}

}  // namespace smlnn
