// K19/K20 image kernels for gfx950. One thread per output pixel; a wave covers
// 64 consecutive pixels of a row, so the (per-channel CHW) stores are
// coalesced and the bilinear source taps of neighbouring lanes share cache
// lines. All arithmetic is the shared fixed-point code of image_ops.h, so the
// device results are bit-identical to the host path.
#include <hip/hip_bf16.h>
#include <hip/hip_fp16.h>
#include <hip/hip_runtime.h>

#include <stdexcept>
#include <string>

#include "image_cpu.h"

#define IMG_HIP_CHECK(e)                                                                               \
  do {                                                                                                 \
    hipError_t _e = (e);                                                                               \
    if (_e != hipSuccess) throw std::runtime_error(std::string("HIP error: ") + hipGetErrorString(_e)); \
  } while (0)

namespace smlimg {
namespace {

constexpr int kThreads = 256;

template <typename T>
__device__ __forceinline__ T cast_out(float v);
template <>
__device__ __forceinline__ float cast_out<float>(float v) { return v; }
template <>
__device__ __forceinline__ __half cast_out<__half>(float v) { return __float2half(v); }
template <>
__device__ __forceinline__ __hip_bfloat16 cast_out<__hip_bfloat16>(float v) { return __float2bfloat16(v); }

template <typename T>
__global__ __launch_bounds__(kThreads) void preprocess_kernel(const uint8_t* __restrict__ src,
                                                              const int64_t* __restrict__ offsets,
                                                              const int32_t* __restrict__ dims, PrepParams p,
                                                              T* __restrict__ out) {
  const int b = blockIdx.y;
  const int npx = p.out_h * p.out_w;
  const int i = blockIdx.x * kThreads + threadIdx.x;
  if (i >= npx) return;
  const int y = i / p.out_w, x = i - y * p.out_w;
  const int h = dims[3 * b], w = dims[3 * b + 1], c = dims[3 * b + 2];
  const uint8_t* img = src + offsets[b];
  const int ry = y + p.crop_y, rx = x + p.crop_x;
  int y0 = ry, y1 = ry, wy = 0, x0 = rx, x1 = rx, wx = 0;
  const bool rs = p.resize_h > 0;
  if (rs) {
    LinearTap(ry, h, static_cast<double>(h) / p.resize_h, &y0, &y1, &wy);
    LinearTap(rx, w, static_cast<double>(w) / p.resize_w, &x0, &x1, &wx);
  }
  for (int k = 0; k < p.cout; ++k) {
    const int s = p.chan_map[k] < c ? p.chan_map[k] : c - 1;
    const uint8_t v = rs ? ResizePixel(img, h, w, c, s, y0, y1, wy, x0, x1, wx) : img[(ry * w + rx) * c + s];
    const float o = static_cast<float>((static_cast<double>(v) * p.scale - p.mean[k]) / p.stdv[k]);
    const size_t dst = p.nhwc ? (static_cast<size_t>(b) * npx + i) * p.cout + k
                              : (static_cast<size_t>(b) * p.cout + k) * npx + i;
    out[dst] = cast_out<T>(o);
  }
}

__global__ __launch_bounds__(kThreads) void resize_kernel(const uint8_t* __restrict__ src, int sh, int sw, int c,
                                                          uint8_t* __restrict__ dst, int dh, int dw) {
  const int b = blockIdx.y;
  const int i = blockIdx.x * kThreads + threadIdx.x;
  if (i >= dh * dw) return;
  const int y = i / dw, x = i - y * dw;
  int y0, y1, wy, x0, x1, wx;
  LinearTap(y, sh, static_cast<double>(sh) / dh, &y0, &y1, &wy);
  LinearTap(x, sw, static_cast<double>(sw) / dw, &x0, &x1, &wx);
  const uint8_t* img = src + static_cast<size_t>(b) * sh * sw * c;
  uint8_t* o = dst + (static_cast<size_t>(b) * dh * dw + i) * c;
  for (int ch = 0; ch < c; ++ch) o[ch] = ResizePixel(img, sh, sw, c, ch, y0, y1, wy, x0, x1, wx);
}

__global__ __launch_bounds__(kThreads) void box_blur_kernel(const uint8_t* __restrict__ src, int h, int w, int c,
                                                            uint8_t* __restrict__ dst, int kw, int kh) {
  const int b = blockIdx.y;
  const int i = blockIdx.x * kThreads + threadIdx.x;
  if (i >= h * w) return;
  const int y = i / w, x = i - y * w;
  const uint8_t* img = src + static_cast<size_t>(b) * h * w * c;
  const double scale = 1.0 / (static_cast<double>(kw) * kh);
  for (int ch = 0; ch < c; ++ch) {
    int s = 0;
    for (int j = 0; j < kh; ++j) {
      const int yy = Reflect101(y + j - kh / 2, h);
      for (int t = 0; t < kw; ++t) s += img[(yy * w + Reflect101(x + t - kw / 2, w)) * c + ch];
    }
    dst[(static_cast<size_t>(b) * h * w + i) * c + ch] = SatRound(s * scale);
  }
}

struct Taps {
  double k[32];
};

__global__ __launch_bounds__(kThreads) void column_filter_kernel(const uint8_t* __restrict__ src, int h, int w, int c,
                                                                 uint8_t* __restrict__ dst, Taps taps, int n) {
  const int b = blockIdx.y;
  const int i = blockIdx.x * kThreads + threadIdx.x;
  if (i >= h * w) return;
  const int y = i / w, x = i - y * w;
  const uint8_t* img = src + static_cast<size_t>(b) * h * w * c;
  for (int ch = 0; ch < c; ++ch) {
    double s = 0;
    for (int j = 0; j < n; ++j) s += taps.k[j] * img[(Reflect101(y + j - n / 2, h) * w + x) * c + ch];
    dst[(static_cast<size_t>(b) * h * w + i) * c + ch] = SatRound(s);
  }
}

__global__ void threshold_kernel(const uint8_t* __restrict__ src, int64_t n, uint8_t* __restrict__ dst, double thr,
                                 double maxval, int type) {
  for (int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; i < n;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x)
    dst[i] = ThresholdPx(src[i], thr, maxval, type);
}

__global__ __launch_bounds__(kThreads) void flip_kernel(const uint8_t* __restrict__ src, int h, int w, int c,
                                                        uint8_t* __restrict__ dst, int code) {
  const int b = blockIdx.y;
  const int i = blockIdx.x * kThreads + threadIdx.x;
  if (i >= h * w) return;
  const int y = i / w, x = i - y * w;
  const int sy = (code == 0 || code < 0) ? h - 1 - y : y;   // 0: up-down, 1: left-right, -1: both
  const int sx = (code > 0 || code < 0) ? w - 1 - x : x;
  const size_t base = static_cast<size_t>(b) * h * w;
  for (int ch = 0; ch < c; ++ch) dst[(base + i) * c + ch] = src[(base + sy * w + sx) * c + ch];
}

__global__ void cvt_kernel(const uint8_t* __restrict__ src, int64_t npx, int cin, int cout, int code,
                           uint8_t* __restrict__ dst) {
  for (int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; i < npx;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const uint8_t* s = src + i * cin;
    uint8_t* d = dst + i * cout;
    switch (code) {
      case 0: d[0] = s[0]; d[1] = s[1]; d[2] = s[2]; d[3] = 255; break;
      case 2: d[0] = s[2]; d[1] = s[1]; d[2] = s[0]; d[3] = 255; break;
      case 1: d[0] = s[0]; d[1] = s[1]; d[2] = s[2]; break;
      case 3: case 4: d[0] = s[2]; d[1] = s[1]; d[2] = s[0]; break;
      case 5: d[0] = s[2]; d[1] = s[1]; d[2] = s[0]; d[3] = s[3]; break;
      case 6: case 10: d[0] = Luma(s[0], s[1], s[2]); break;
      case 7: case 11: d[0] = Luma(s[2], s[1], s[0]); break;
      case 8: d[0] = d[1] = d[2] = s[0]; break;
      case 9: d[0] = d[1] = d[2] = s[0]; d[3] = 255; break;
    }
  }
}

int Grid1D(int64_t n) {
  int64_t g = (n + kThreads - 1) / kThreads;
  return static_cast<int>(g < 1 ? 1 : (g > 65535 ? 65535 : g));
}

}  // namespace

bool ImageGpuAvailable() {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) { (void)hipGetLastError(); return false; }
  return n > 0;
}

void PreprocessBatchDevice(const uint8_t* src, const int64_t* offsets, const int32_t* dims, int B,
                           const PrepParams& p, void* out, void* stream) {
  if (B <= 0) return;
  if (p.cout < 1 || p.cout > 4) throw std::invalid_argument("preprocess: 1..4 output channels");
  dim3 grid((p.out_h * p.out_w + kThreads - 1) / kThreads, B);
  auto s = static_cast<hipStream_t>(stream);
  if (p.out_dtype == 1)
    hipLaunchKernelGGL(preprocess_kernel<__half>, grid, dim3(kThreads), 0, s, src, offsets, dims, p,
                       static_cast<__half*>(out));
  else if (p.out_dtype == 2)
    hipLaunchKernelGGL(preprocess_kernel<__hip_bfloat16>, grid, dim3(kThreads), 0, s, src, offsets, dims, p,
                       static_cast<__hip_bfloat16*>(out));
  else
    hipLaunchKernelGGL(preprocess_kernel<float>, grid, dim3(kThreads), 0, s, src, offsets, dims, p,
                       static_cast<float*>(out));
  IMG_HIP_CHECK(hipGetLastError());
}

void ResizeBatchDevice(const uint8_t* src, int B, int sh, int sw, int c, uint8_t* dst, int dh, int dw, void* stream) {
  dim3 grid((dh * dw + kThreads - 1) / kThreads, B);
  hipLaunchKernelGGL(resize_kernel, grid, dim3(kThreads), 0, static_cast<hipStream_t>(stream), src, sh, sw, c, dst, dh,
                     dw);
  IMG_HIP_CHECK(hipGetLastError());
}

void BoxBlurBatchDevice(const uint8_t* src, int B, int h, int w, int c, uint8_t* dst, int kw, int kh, void* stream) {
  dim3 grid((h * w + kThreads - 1) / kThreads, B);
  hipLaunchKernelGGL(box_blur_kernel, grid, dim3(kThreads), 0, static_cast<hipStream_t>(stream), src, h, w, c, dst, kw,
                     kh);
  IMG_HIP_CHECK(hipGetLastError());
}

void ColumnFilterBatchDevice(const uint8_t* src, int B, int h, int w, int c, uint8_t* dst, const double* k_host, int n,
                             void* stream) {
  if (n > 32) throw std::invalid_argument("column filter: kernel longer than 32 taps");
  Taps t{};
  for (int i = 0; i < n; ++i) t.k[i] = k_host[i];
  dim3 grid((h * w + kThreads - 1) / kThreads, B);
  hipLaunchKernelGGL(column_filter_kernel, grid, dim3(kThreads), 0, static_cast<hipStream_t>(stream), src, h, w, c,
                     dst, t, n);
  IMG_HIP_CHECK(hipGetLastError());
}

void ThresholdDevice(const uint8_t* src, int64_t n, uint8_t* dst, double thr, double maxval, int type, void* stream) {
  hipLaunchKernelGGL(threshold_kernel, dim3(Grid1D(n)), dim3(kThreads), 0, static_cast<hipStream_t>(stream), src, n,
                     dst, thr, maxval, type);
  IMG_HIP_CHECK(hipGetLastError());
}

void FlipBatchDevice(const uint8_t* src, int B, int h, int w, int c, uint8_t* dst, int code, void* stream) {
  dim3 grid((h * w + kThreads - 1) / kThreads, B);
  hipLaunchKernelGGL(flip_kernel, grid, dim3(kThreads), 0, static_cast<hipStream_t>(stream), src, h, w, c, dst, code);
  IMG_HIP_CHECK(hipGetLastError());
}

void CvtColorDevice(const uint8_t* src, int64_t npx, int cin, int code, uint8_t* dst, void* stream) {
  const int cout = CvtChannelsOut(code, cin);
  hipLaunchKernelGGL(cvt_kernel, dim3(Grid1D(npx)), dim3(kThreads), 0, static_cast<hipStream_t>(stream), src, npx, cin,
                     cout, code, dst);
  IMG_HIP_CHECK(hipGetLastError());
}

}  // namespace smlimg
