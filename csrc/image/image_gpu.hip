// K19/K20 image kernels for gfx950. One thread per output pixel; a wave covers
// 64 consecutive pixels of a row, so the (per-channel CHW) stores are
// coalesced and the bilinear source taps of neighbouring lanes share cache
// lines. All arithmetic is the shared fixed-point code of image_ops.h, so the
// device results are bit-identical to the host path.
#include <hip/hip_bf16.h>
#include <hip/hip_fp16.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <stdexcept>
#include <string>
#include <vector>

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

// K19. Per-image resize taps (LinearTap on the host: y taps then x taps, int4 {s0, s1, w1, 0}) and the
// per-channel output LUT (the host's (v * scale - mean) / std in fp64, rounded to float, for all 256 byte
// values) replace the fp64 coordinate math and the fp64 division of every pixel: one bilinear in integers
// and one LDS lookup per output value, bit-identical to ToTensorHost.
template <typename T>
__global__ __launch_bounds__(kThreads) void preprocess_kernel(const uint8_t* __restrict__ src,
                                                              const int64_t* __restrict__ offsets,
                                                              const int32_t* __restrict__ dims, PrepParams p,
                                                              const int4* __restrict__ taps,
                                                              const float* __restrict__ lut, T* __restrict__ out) {
  __shared__ float s_lut[4 * 256];
  for (int i = threadIdx.x; i < p.cout * 256; i += kThreads) s_lut[i] = lut[i];
  __syncthreads();
  const int b = blockIdx.y;
  const int npx = p.out_h * p.out_w;
  const int i = blockIdx.x * kThreads + threadIdx.x;
  if (i >= npx) return;
  const int y = i / p.out_w, x = i - y * p.out_w;
  const int w = dims[3 * b + 1], c = dims[3 * b + 2];
  const uint8_t* img = src + offsets[b];
  const int ry = y + p.crop_y, rx = x + p.crop_x;
  const bool rs = p.resize_h > 0;
  int4 ty = make_int4(ry, ry, 0, 0), tx = make_int4(rx, rx, 0, 0);
  if (rs) {
    const int4* tb = taps + (p.taps_uniform ? size_t(0) : static_cast<size_t>(b) * (p.resize_h + p.resize_w));
    ty = tb[ry];
    tx = tb[p.resize_h + rx];
  }
  for (int k = 0; k < p.cout; ++k) {
    const int sc = p.chan_map[k] < c ? p.chan_map[k] : c - 1;
    const uint8_t v = rs ? ResizePixel(img, 0, w, c, sc, ty.x, ty.y, ty.z, tx.x, tx.y, tx.z) : img[(ry * w + rx) * c + sc];
    const size_t dst = p.nhwc ? (static_cast<size_t>(b) * npx + i) * p.cout + k
                              : (static_cast<size_t>(b) * p.cout + k) * npx + i;
    out[dst] = cast_out<T>(s_lut[k * 256 + v]);
  }
}

// ---- K20: stage kernels on a uniform batch of HWC uint8 images. Row-parallel: grid.y = (image, output row),
// each thread produces 4 consecutive bytes of the output row and stores them as one dword (byte stores only
// at an unaligned row tail), channel counts are template constants (no per-byte division), and every index /
// weight table (resize taps, BORDER_REFLECT_101 indices) is computed once on the host by the host kernels' own
// code, so no fp64 coordinate math runs per pixel and the results stay bit-identical to the host path.
__device__ __forceinline__ void StoreQuad(uint8_t* o, uint32_t v, int nbytes) {
  if (nbytes == 4 && (reinterpret_cast<uintptr_t>(o) & 3u) == 0) {
    *reinterpret_cast<uint32_t*>(o) = v;
  } else {
    for (int j = 0; j < nbytes; ++j) o[j] = static_cast<uint8_t>(v >> (8 * j));
  }
}

template <int C>
__global__ __launch_bounds__(kThreads) void resize_rows_kernel(const uint8_t* __restrict__ src, int sh, int sw,
                                                               uint8_t* __restrict__ dst, int dh, int dw,
                                                               const int4* __restrict__ ytap,
                                                               const int4* __restrict__ xtap) {
  const int row = blockIdx.y, b = row / dh, y = row - b * dh;
  const int rb = dw * C;
  const int q = (blockIdx.x * kThreads + threadIdx.x) * 4;
  if (q >= rb) return;
  const int4 ty = ytap[y];
  const uint8_t* img = src + static_cast<size_t>(b) * sh * sw * C;
  uint32_t v = 0;
  const int nb = min(4, rb - q);
  for (int j = 0; j < nb; ++j) {
    const int xb = q + j, x = xb / C, ch = xb - x * C;
    const int4 tx = xtap[x];
    v |= static_cast<uint32_t>(ResizePixel(img, sh, sw, C, ch, ty.x, ty.y, ty.z, tx.x, tx.y, tx.z)) << (8 * j);
  }
  StoreQuad(dst + static_cast<size_t>(row) * rb + q, v, nb);
}

// crop (and flip) as row copies: output row y of image b reads source row sy, bytes from byte offset x0 of
// the row (flip: mirrored pixels, channels kept in order)
template <int C>
__global__ __launch_bounds__(kThreads) void crop_flip_rows_kernel(const uint8_t* __restrict__ src, int sh, int sw,
                                                                  uint8_t* __restrict__ dst, int dh, int dw, int cy,
                                                                  int cx, int flip) {
  const int row = blockIdx.y, b = row / dh, y = row - b * dh;
  const int rb = dw * C;
  const int q = (blockIdx.x * kThreads + threadIdx.x) * 4;
  if (q >= rb) return;
  const int sy = (flip == 0 || flip == 2) ? (dh - 1 - y) + cy : y + cy;  // 0 / 2 (= both): up-down
  const uint8_t* r = src + (static_cast<size_t>(b) * sh + sy) * sw * C;
  uint32_t v = 0;
  const int nb = min(4, rb - q);
  for (int j = 0; j < nb; ++j) {
    const int xb = q + j, x = xb / C, ch = xb - x * C;
    const int sx = (flip == 1 || flip == 2) ? (dw - 1 - x) + cx : x + cx;
    v |= static_cast<uint32_t>(r[sx * C + ch]) << (8 * j);
  }
  StoreQuad(dst + static_cast<size_t>(row) * rb + q, v, nb);
}

// Separable box filter, exact: the horizontal pass writes int32 row sums of kw reflected taps, the vertical
// pass adds kh of them - the same integer as the host's kw x kh double loop - and rounds s * (1 / (kw kh)).
// O(kw + kh) loads per pixel instead of O(kw kh).
__global__ __launch_bounds__(kThreads) void box_h_kernel(const uint8_t* __restrict__ src, int h, int w, int c,
                                                         int32_t* __restrict__ tmp, int kw,
                                                         const int32_t* __restrict__ xr) {
  const int row = blockIdx.y;
  const int rb = w * c;
  const int xb = blockIdx.x * kThreads + threadIdx.x;
  if (xb >= rb) return;
  const int x = xb / c, ch = xb - x * c;
  const uint8_t* r = src + static_cast<size_t>(row) * rb;
  const int32_t* t = xr + static_cast<size_t>(x) * kw;
  int32_t s = 0;
  for (int i = 0; i < kw; ++i) s += r[t[i] * c + ch];
  tmp[static_cast<size_t>(row) * rb + xb] = s;
}

__global__ __launch_bounds__(kThreads) void box_v_kernel(const int32_t* __restrict__ tmp, int h, int w, int c,
                                                         uint8_t* __restrict__ dst, int kh,
                                                         const int32_t* __restrict__ yr, double scale) {
  const int row = blockIdx.y, b = row / h, y = row - b * h;
  const int rb = w * c;
  const int q = (blockIdx.x * kThreads + threadIdx.x) * 4;
  if (q >= rb) return;
  const int32_t* base = tmp + static_cast<size_t>(b) * h * rb;
  const int32_t* t = yr + static_cast<size_t>(y) * kh;
  const int nb = min(4, rb - q);
  int64_t s[4] = {0, 0, 0, 0};
  for (int j = 0; j < kh; ++j) {
    const int32_t* r = base + static_cast<size_t>(t[j]) * rb + q;
    for (int k = 0; k < nb; ++k) s[k] += r[k];
  }
  uint32_t v = 0;
  for (int k = 0; k < nb; ++k) v |= static_cast<uint32_t>(SatRound(static_cast<double>(s[k]) * scale)) << (8 * k);
  StoreQuad(dst + static_cast<size_t>(row) * rb + q, v, nb);
}

// vertical (column) filter with fp64 taps, as ColumnFilterHost: the same products and sums in the same order,
// with explicit round-to-nearest operations so the compiler cannot contract them into FMAs the host never does
__global__ __launch_bounds__(kThreads) void column_rows_kernel(const uint8_t* __restrict__ src, int h, int w, int c,
                                                               uint8_t* __restrict__ dst, const double* __restrict__ k,
                                                               int n, const int32_t* __restrict__ yr) {
  const int row = blockIdx.y, b = row / h, y = row - b * h;
  const int rb = w * c;
  const int q = (blockIdx.x * kThreads + threadIdx.x) * 4;
  if (q >= rb) return;
  const uint8_t* base = src + static_cast<size_t>(b) * h * rb;
  const int32_t* t = yr + static_cast<size_t>(y) * n;
  const int nb = min(4, rb - q);
  double s[4] = {0, 0, 0, 0};
  for (int j = 0; j < n; ++j) {
    const uint8_t* r = base + static_cast<size_t>(t[j]) * rb + q;
    const double kj = k[j];
    for (int e = 0; e < nb; ++e) s[e] = __dadd_rn(s[e], __dmul_rn(kj, static_cast<double>(r[e])));
  }
  uint32_t v = 0;
  for (int e = 0; e < nb; ++e) v |= static_cast<uint32_t>(SatRound(s[e])) << (8 * e);
  StoreQuad(dst + static_cast<size_t>(row) * rb + q, v, nb);
}

// byte -> byte through a 256-entry table (threshold: ThresholdPx of every byte value, on the host), 4 bytes per
// thread with dword loads / stores
__global__ __launch_bounds__(kThreads) void lut_kernel(const uint8_t* __restrict__ src, int64_t n,
                                                       uint8_t* __restrict__ dst, const uint8_t* __restrict__ lut) {
  __shared__ uint8_t s_lut[256];
  if (threadIdx.x < 256) s_lut[threadIdx.x] = lut[threadIdx.x];
  __syncthreads();
  const int64_t nq = n / 4;
  for (int64_t i = blockIdx.x * static_cast<int64_t>(kThreads) + threadIdx.x; i < nq;
       i += static_cast<int64_t>(gridDim.x) * kThreads) {
    const uint32_t v = reinterpret_cast<const uint32_t*>(src)[i];
    uint32_t o = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) o |= static_cast<uint32_t>(s_lut[(v >> (8 * j)) & 255u]) << (8 * j);
    reinterpret_cast<uint32_t*>(dst)[i] = o;
  }
  if (blockIdx.x == 0 && threadIdx.x < n - nq * 4) dst[nq * 4 + threadIdx.x] = s_lut[src[nq * 4 + threadIdx.x]];
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

// Small per-call tables (taps, reflect indices, LUTs) go to a stream-ordered device allocation freed on the
// same stream; the host source vectors are pageable, so the copy is staged before hipMemcpyAsync returns.
template <class T>
T* UploadTable(const std::vector<T>& v, hipStream_t s) {
  void* d = nullptr;
  IMG_HIP_CHECK(hipMallocAsync(&d, std::max<size_t>(16, v.size() * sizeof(T)), s));
  if (!v.empty()) IMG_HIP_CHECK(hipMemcpyAsync(d, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice, s));
  return static_cast<T*>(d);
}

std::vector<int4> AxisTaps(int dst_len, int src_len) {
  std::vector<int4> t(dst_len);
  const double inv = static_cast<double>(src_len) / dst_len;
  for (int d = 0; d < dst_len; ++d) {
    int s0, s1, w1;
    LinearTap(d, src_len, inv, &s0, &s1, &w1);
    t[d] = make_int4(s0, s1, w1, 0);
  }
  return t;
}

std::vector<int32_t> ReflectTable(int len, int k) {
  std::vector<int32_t> t(static_cast<size_t>(len) * k);
  for (int i = 0; i < len; ++i)
    for (int j = 0; j < k; ++j) t[static_cast<size_t>(i) * k + j] = Reflect101(i + j - k / 2, len);
  return t;
}

int RowBlocks(int row_bytes) { return (row_bytes / 4 + kThreads) / kThreads; }

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
  auto s = static_cast<hipStream_t>(stream);
  // output value of byte v in channel k: the host's ToTensorHost expression, once per (k, v)
  std::vector<float> lut(static_cast<size_t>(p.cout) * 256);
  for (int k = 0; k < p.cout; ++k)
    for (int v = 0; v < 256; ++v)
      lut[k * 256 + v] = static_cast<float>((static_cast<double>(v) * p.scale - p.mean[k]) / p.stdv[k]);
  std::vector<int4> taps;
  PrepParams q = p;
  if (p.resize_h > 0) {
    if (!p.host_dims) throw std::invalid_argument("preprocess: resize needs the images' host dims");
    // one set of taps when every image has the same size (a 256-image batch's per-image tables were 2 MB of
    // pageable upload, which waited for the batch's own H2D before returning: r6 pass 19)
    bool uniform = true;
    for (int b = 1; b < B && uniform; ++b)
      uniform = p.host_dims[3 * b] == p.host_dims[0] && p.host_dims[3 * b + 1] == p.host_dims[1];
    q.taps_uniform = uniform ? 1 : 0;
    const int nb = uniform ? 1 : B;
    taps.reserve(static_cast<size_t>(nb) * (p.resize_h + p.resize_w));
    for (int b = 0; b < nb; ++b) {
      const auto ty = AxisTaps(p.resize_h, p.host_dims[3 * b]), tx = AxisTaps(p.resize_w, p.host_dims[3 * b + 1]);
      taps.insert(taps.end(), ty.begin(), ty.end());
      taps.insert(taps.end(), tx.begin(), tx.end());
    }
  }
  float* d_lut = UploadTable(lut, s);
  int4* d_taps = UploadTable(taps, s);
  dim3 grid((p.out_h * p.out_w + kThreads - 1) / kThreads, B);
  if (p.out_dtype == 1)
    hipLaunchKernelGGL(preprocess_kernel<__half>, grid, dim3(kThreads), 0, s, src, offsets, dims, q, d_taps, d_lut,
                       static_cast<__half*>(out));
  else if (p.out_dtype == 2)
    hipLaunchKernelGGL(preprocess_kernel<__hip_bfloat16>, grid, dim3(kThreads), 0, s, src, offsets, dims, q, d_taps,
                       d_lut, static_cast<__hip_bfloat16*>(out));
  else
    hipLaunchKernelGGL(preprocess_kernel<float>, grid, dim3(kThreads), 0, s, src, offsets, dims, q, d_taps, d_lut,
                       static_cast<float*>(out));
  IMG_HIP_CHECK(hipGetLastError());
  IMG_HIP_CHECK(hipFreeAsync(d_lut, s));
  IMG_HIP_CHECK(hipFreeAsync(d_taps, s));
}

void ResizeBatchDevice(const uint8_t* src, int B, int sh, int sw, int c, uint8_t* dst, int dh, int dw, void* stream) {
  if (B <= 0) return;
  auto s = static_cast<hipStream_t>(stream);
  int4* ty = UploadTable(AxisTaps(dh, sh), s);
  int4* tx = UploadTable(AxisTaps(dw, sw), s);
  dim3 grid(RowBlocks(dw * c), B * dh);
  switch (c) {
    case 1: hipLaunchKernelGGL(resize_rows_kernel<1>, grid, dim3(kThreads), 0, s, src, sh, sw, dst, dh, dw, ty, tx); break;
    case 3: hipLaunchKernelGGL(resize_rows_kernel<3>, grid, dim3(kThreads), 0, s, src, sh, sw, dst, dh, dw, ty, tx); break;
    case 4: hipLaunchKernelGGL(resize_rows_kernel<4>, grid, dim3(kThreads), 0, s, src, sh, sw, dst, dh, dw, ty, tx); break;
    default: throw std::invalid_argument("resize: 1, 3 or 4 channels");
  }
  IMG_HIP_CHECK(hipGetLastError());
  IMG_HIP_CHECK(hipFreeAsync(ty, s));
  IMG_HIP_CHECK(hipFreeAsync(tx, s));
}

void CropFlipBatchDevice(const uint8_t* src, int B, int sh, int sw, int c, uint8_t* dst, int dh, int dw, int cy, int cx,
                         int flip, void* stream) {
  if (B <= 0) return;
  if (cy < 0 || cx < 0 || cy + dh > sh || cx + dw > sw) throw std::invalid_argument("crop rectangle outside the image");
  auto s = static_cast<hipStream_t>(stream);
  dim3 grid(RowBlocks(dw * c), B * dh);
  switch (c) {
    case 1: hipLaunchKernelGGL(crop_flip_rows_kernel<1>, grid, dim3(kThreads), 0, s, src, sh, sw, dst, dh, dw, cy, cx, flip); break;
    case 3: hipLaunchKernelGGL(crop_flip_rows_kernel<3>, grid, dim3(kThreads), 0, s, src, sh, sw, dst, dh, dw, cy, cx, flip); break;
    case 4: hipLaunchKernelGGL(crop_flip_rows_kernel<4>, grid, dim3(kThreads), 0, s, src, sh, sw, dst, dh, dw, cy, cx, flip); break;
    default: throw std::invalid_argument("crop / flip: 1, 3 or 4 channels");
  }
  IMG_HIP_CHECK(hipGetLastError());
}

void BoxBlurBatchDevice(const uint8_t* src, int B, int h, int w, int c, uint8_t* dst, int kw, int kh, void* stream) {
  if (B <= 0) return;
  if (kw < 1 || kh < 1) throw std::invalid_argument("blur: kernel size must be positive");
  auto s = static_cast<hipStream_t>(stream);
  int32_t* xr = UploadTable(ReflectTable(w, kw), s);
  int32_t* yr = UploadTable(ReflectTable(h, kh), s);
  int32_t* tmp = nullptr;
  IMG_HIP_CHECK(hipMallocAsync(reinterpret_cast<void**>(&tmp), sizeof(int32_t) * static_cast<size_t>(B) * h * w * c, s));
  hipLaunchKernelGGL(box_h_kernel, dim3((w * c + kThreads - 1) / kThreads, B * h), dim3(kThreads), 0, s, src, h, w, c,
                     tmp, kw, xr);
  IMG_HIP_CHECK(hipGetLastError());
  hipLaunchKernelGGL(box_v_kernel, dim3(RowBlocks(w * c), B * h), dim3(kThreads), 0, s, tmp, h, w, c, dst, kh, yr,
                     1.0 / (static_cast<double>(kw) * kh));
  IMG_HIP_CHECK(hipGetLastError());
  IMG_HIP_CHECK(hipFreeAsync(tmp, s));
  IMG_HIP_CHECK(hipFreeAsync(xr, s));
  IMG_HIP_CHECK(hipFreeAsync(yr, s));
}

void ColumnFilterBatchDevice(const uint8_t* src, int B, int h, int w, int c, uint8_t* dst, const double* k_host, int n,
                             void* stream) {
  if (B <= 0) return;
  if (n < 1) throw std::invalid_argument("column filter: empty kernel");
  auto s = static_cast<hipStream_t>(stream);
  double* k = UploadTable(std::vector<double>(k_host, k_host + n), s);
  int32_t* yr = UploadTable(ReflectTable(h, n), s);
  hipLaunchKernelGGL(column_rows_kernel, dim3(RowBlocks(w * c), B * h), dim3(kThreads), 0, s, src, h, w, c, dst, k, n,
                     yr);
  IMG_HIP_CHECK(hipGetLastError());
  IMG_HIP_CHECK(hipFreeAsync(k, s));
  IMG_HIP_CHECK(hipFreeAsync(yr, s));
}

void ThresholdDevice(const uint8_t* src, int64_t n, uint8_t* dst, double thr, double maxval, int type, void* stream) {
  if (n <= 0) return;
  auto s = static_cast<hipStream_t>(stream);
  std::vector<uint8_t> lut(256);
  for (int v = 0; v < 256; ++v) lut[v] = ThresholdPx(static_cast<uint8_t>(v), thr, maxval, type);
  uint8_t* d = UploadTable(lut, s);
  if ((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst)) & 3u)
    throw std::invalid_argument("threshold: device buffers must be 4-byte aligned");
  hipLaunchKernelGGL(lut_kernel, dim3(Grid1D(std::max<int64_t>(1, n / 4))), dim3(kThreads), 0, s, src, n, dst, d);
  IMG_HIP_CHECK(hipGetLastError());
  IMG_HIP_CHECK(hipFreeAsync(d, s));
}

void FlipBatchDevice(const uint8_t* src, int B, int h, int w, int c, uint8_t* dst, int code, void* stream) {
  // OpenCV flipCode: 0 up-down, > 0 left-right, < 0 both
  CropFlipBatchDevice(src, B, h, w, c, dst, h, w, 0, 0, code == 0 ? 0 : (code > 0 ? 1 : 2), stream);
}

void CvtColorDevice(const uint8_t* src, int64_t npx, int cin, int code, uint8_t* dst, void* stream) {
  const int cout = CvtChannelsOut(code, cin);
  hipLaunchKernelGGL(cvt_kernel, dim3(Grid1D(npx)), dim3(kThreads), 0, static_cast<hipStream_t>(stream), src, npx, cin,
                     cout, code, dst);
  IMG_HIP_CHECK(hipGetLastError());
}

}  // namespace smlimg
