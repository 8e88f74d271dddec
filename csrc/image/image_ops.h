// Image kernels shared by the host (OpenMP) and device (HIP) paths.
//
// Semantics follow the OpenCV calls the reference makes for its image stages
// (opencv/.../ImageTransformer.scala:68-283): INTER_LINEAR resize with
// OpenCV's 11-bit fixed-point coefficients, cvtColor's 14-bit fixed-point
// luma, box blur / column-Gaussian filtering with BORDER_REFLECT_101, and
// threshold types 0-4. Tensorization is (x * scale - mean) / std in CHW
// (ImageTransformer.scala:379-415). Images are HWC uint8, channel order as
// stored (BGR / BGRA / gray).
#pragma once
#include <cmath>
#include <cstdint>

#if defined(__HIPCC__)
#define SML_IHD __host__ __device__ __forceinline__
#else
#define SML_IHD inline
#endif

namespace smlimg {

constexpr int kCoefBits = 11;                 // INTER_RESIZE_COEF_BITS
constexpr int kCoefScale = 1 << kCoefBits;    // 2048

// Source coordinate + fixed-point weight of output index d along one axis
// (half-pixel centres, clamped at the borders the way OpenCV does).
SML_IHD void LinearTap(int d, int src_len, double inv_scale, int* s0, int* s1, int* w1) {
  double fx = (d + 0.5) * inv_scale - 0.5;
  int sx = static_cast<int>(floor(fx));
  double u = fx - sx;
  if (sx < 0) { sx = 0; u = 0.0; }
  if (sx >= src_len - 1) { sx = src_len - 1; u = 0.0; }
  int wi = static_cast<int>(u * kCoefScale + (u >= 0 ? 0.5 : -0.5));
  *s0 = sx;
  *s1 = sx + 1 < src_len ? sx + 1 : sx;
  *w1 = wi;
}

// One resized channel value at (oy, ox): horizontal taps, then vertical, with
// OpenCV's rounding (22 fractional bits total).
SML_IHD uint8_t ResizePixel(const uint8_t* src, int sh, int sw, int c, int ch, int y0, int y1, int wy, int x0, int x1,
                            int wx) {
  const int ax0 = kCoefScale - wx, ay0 = kCoefScale - wy;
  const int r0 = src[(y0 * sw + x0) * c + ch] * ax0 + src[(y0 * sw + x1) * c + ch] * wx;
  const int r1 = src[(y1 * sw + x0) * c + ch] * ax0 + src[(y1 * sw + x1) * c + ch] * wx;
  int v = (r0 * ay0 + r1 * wy + (1 << (2 * kCoefBits - 1))) >> (2 * kCoefBits);
  return static_cast<uint8_t>(v < 0 ? 0 : (v > 255 ? 255 : v));
}

// cvtColor luma: Y = (B*1868 + G*9617 + R*4899 + 2^13) >> 14
SML_IHD uint8_t Luma(int b, int g, int r) {
  return static_cast<uint8_t>((b * 1868 + g * 9617 + r * 4899 + (1 << 13)) >> 14);
}

// BORDER_REFLECT_101 index
SML_IHD int Reflect101(int i, int n) {
  if (n == 1) return 0;
  while (i < 0 || i >= n) {
    if (i < 0) i = -i;
    if (i >= n) i = 2 * n - 2 - i;
  }
  return i;
}

// round half to even (cvRound), then saturate to uint8
SML_IHD uint8_t SatRound(double v) {
  double r = nearbyint(v);
  return static_cast<uint8_t>(r < 0 ? 0 : (r > 255 ? 255 : r));
}

SML_IHD uint8_t ThresholdPx(uint8_t x, double thr, double maxval, int type) {
  const double v = x;
  const uint8_t mx = SatRound(maxval);
  // OpenCV compares against floor(thresh) for 8-bit images
  const int t = static_cast<int>(floor(thr));
  switch (type & 7) {
    case 0: return v > t ? mx : 0;                 // THRESH_BINARY
    case 1: return v > t ? 0 : mx;                 // THRESH_BINARY_INV
    case 2: return v > t ? static_cast<uint8_t>(t < 0 ? 0 : (t > 255 ? 255 : t)) : x;  // THRESH_TRUNC
    case 3: return v > t ? x : 0;                  // THRESH_TOZERO
    case 4: return v > t ? 0 : x;                  // THRESH_TOZERO_INV
    default: return x;
  }
}

}  // namespace smlimg
