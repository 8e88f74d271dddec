// Host + device entry points of the image component (module _image).
#pragma once
#include <cstdint>
#include <vector>

#include "image_ops.h"

namespace smlimg {

// ---- host (OpenMP)
void ResizeHost(const uint8_t* src, int sh, int sw, int c, uint8_t* dst, int dh, int dw);
void BoxBlurHost(const uint8_t* src, int h, int w, int c, uint8_t* dst, int kw, int kh);
void ColumnFilterHost(const uint8_t* src, int h, int w, int c, uint8_t* dst, const double* k, int n);
void ThresholdHost(const uint8_t* src, int64_t n, uint8_t* dst, double thr, double maxval, int type);
std::vector<double> GaussianKernel(int n, double sigma);
int CvtChannelsOut(int code, int cin);
void CvtColorHost(const uint8_t* src, int64_t npx, int cin, int code, uint8_t* dst);
void ToTensorHost(const uint8_t* src, int h, int w, int c, const int* chan_map, int cout, double scale,
                  const double* mean, const double* stdv, float* dst);

// ---- device (HIP). Pointers are device pointers; `stream` is a hipStream_t.
struct PrepParams {
  int out_h, out_w;       // tensor spatial size
  int resize_h, resize_w; // 0 = no resize
  int crop_y, crop_x;     // crop window origin inside the (resized) image
  int cout;               // output channels
  int chan_map[4];        // output channel k <- source channel chan_map[k]
  double scale;
  double mean[4], stdv[4];
  int out_dtype;          // 0 f32, 1 f16, 2 bf16
  int nhwc;               // 0 = NCHW (ONNX layout), 1 = NHWC
  const int32_t* host_dims = nullptr;  // HOST copy of dims (the resize taps are built per image on the host)
  int taps_uniform = 0;   // device path: every image has the same (h, w), one set of resize taps for the batch
};

// K19: batched decode-free preprocess. Images are packed HWC uint8 at
// src + offsets[b] with dims[3b..3b+2] = (h, w, c). One launch resizes (OpenCV
// INTER_LINEAR fixed point), crops, reorders channels and normalizes every
// image into out[b] (B x cout x out_h x out_w, or NHWC).
void PreprocessBatchDevice(const uint8_t* src, const int64_t* offsets, const int32_t* dims, int B,
                           const PrepParams& p, void* out, void* stream);

// K20: per-stage kernels on a uniform batch (B, h, w, c) of HWC uint8 images.
void ResizeBatchDevice(const uint8_t* src, int B, int sh, int sw, int c, uint8_t* dst, int dh, int dw, void* stream);
void BoxBlurBatchDevice(const uint8_t* src, int B, int h, int w, int c, uint8_t* dst, int kw, int kh, void* stream);
void ColumnFilterBatchDevice(const uint8_t* src, int B, int h, int w, int c, uint8_t* dst, const double* k_host, int n,
                             void* stream);
void ThresholdDevice(const uint8_t* src, int64_t n, uint8_t* dst, double thr, double maxval, int type, void* stream);
void FlipBatchDevice(const uint8_t* src, int B, int h, int w, int c, uint8_t* dst, int code, void* stream);
// crop window (cy, cx, dh x dw) of every image, optionally flipped (0 up-down, 1 left-right, 2 both, -1 none)
void CropFlipBatchDevice(const uint8_t* src, int B, int sh, int sw, int c, uint8_t* dst, int dh, int dw, int cy, int cx,
                         int flip, void* stream);
void CvtColorDevice(const uint8_t* src, int64_t npx, int cin, int code, uint8_t* dst, void* stream);
bool ImageGpuAvailable();

}  // namespace smlimg
