// Host (OpenMP) implementations of the image stages; bit-identical to the
// device kernels in image_gpu.hip (both use image_ops.h).
#include "image_cpu.h"

#include <algorithm>
#include <cmath>
#include <stdexcept>
#include <vector>

namespace smlimg {

void ResizeHost(const uint8_t* src, int sh, int sw, int c, uint8_t* dst, int dh, int dw) {
  if (sh <= 0 || sw <= 0 || dh <= 0 || dw <= 0) throw std::invalid_argument("resize: empty image");
  std::vector<int> x0(dw), x1(dw), wx(dw);
  const double ix = static_cast<double>(sw) / dw, iy = static_cast<double>(sh) / dh;
  for (int x = 0; x < dw; ++x) LinearTap(x, sw, ix, &x0[x], &x1[x], &wx[x]);
#pragma omp parallel for schedule(static) if (static_cast<int64_t>(dh) * dw > 65536)
  for (int y = 0; y < dh; ++y) {
    int y0, y1, wy;
    LinearTap(y, sh, iy, &y0, &y1, &wy);
    for (int x = 0; x < dw; ++x)
      for (int ch = 0; ch < c; ++ch)
        dst[(static_cast<int64_t>(y) * dw + x) * c + ch] = ResizePixel(src, sh, sw, c, ch, y0, y1, wy, x0[x], x1[x], wx[x]);
  }
}

void BoxBlurHost(const uint8_t* src, int h, int w, int c, uint8_t* dst, int kw, int kh) {
  const int ax = kw / 2, ay = kh / 2;
  const double scale = 1.0 / (static_cast<double>(kw) * kh);
#pragma omp parallel for schedule(static) if (static_cast<int64_t>(h) * w > 65536)
  for (int y = 0; y < h; ++y)
    for (int x = 0; x < w; ++x)
      for (int ch = 0; ch < c; ++ch) {
        int64_t s = 0;
        for (int j = 0; j < kh; ++j) {
          const int yy = Reflect101(y + j - ay, h);
          for (int i = 0; i < kw; ++i) s += src[(static_cast<int64_t>(yy) * w + Reflect101(x + i - ax, w)) * c + ch];
        }
        dst[(static_cast<int64_t>(y) * w + x) * c + ch] = SatRound(s * scale);
      }
}

void ColumnFilterHost(const uint8_t* src, int h, int w, int c, uint8_t* dst, const double* k, int n) {
  const int ay = n / 2;
#pragma omp parallel for schedule(static) if (static_cast<int64_t>(h) * w > 65536)
  for (int y = 0; y < h; ++y)
    for (int x = 0; x < w; ++x)
      for (int ch = 0; ch < c; ++ch) {
        double s = 0;
        for (int j = 0; j < n; ++j) s += k[j] * src[(static_cast<int64_t>(Reflect101(y + j - ay, h)) * w + x) * c + ch];
        dst[(static_cast<int64_t>(y) * w + x) * c + ch] = SatRound(s);
      }
}

void ThresholdHost(const uint8_t* src, int64_t n, uint8_t* dst, double thr, double maxval, int type) {
#pragma omp parallel for schedule(static) if (n > 262144)
  for (int64_t i = 0; i < n; ++i) dst[i] = ThresholdPx(src[i], thr, maxval, type);
}

std::vector<double> GaussianKernel(int n, double sigma) {
  static const double k1[] = {1.0};
  static const double k3[] = {0.25, 0.5, 0.25};
  static const double k5[] = {0.0625, 0.25, 0.375, 0.25, 0.0625};
  static const double k7[] = {0.03125, 0.109375, 0.21875, 0.28125, 0.21875, 0.109375, 0.03125};
  if (n <= 0 || n % 2 == 0) throw std::invalid_argument("gaussian kernel size must be odd and positive");
  if (sigma <= 0 && n <= 7) {
    const double* t = n == 1 ? k1 : (n == 3 ? k3 : (n == 5 ? k5 : k7));
    return std::vector<double>(t, t + n);
  }
  const double s = sigma > 0 ? sigma : ((n - 1) * 0.5 - 1) * 0.3 + 0.8;
  const double s2 = -0.5 / (s * s);
  std::vector<double> k(n);
  double sum = 0;
  for (int i = 0; i < n; ++i) {
    const double x = i - (n - 1) * 0.5;
    k[i] = std::exp(s2 * x * x);
    sum += k[i];
  }
  for (auto& v : k) v /= sum;
  return k;
}

// cvtColor codes used by the reference's ColorFormat stage (OpenCV enum values)
int CvtChannelsOut(int code, int cin) {
  // the source channels each conversion reads (a 3-channel image given to BGRA2RGBA would read past
  // every pixel into the next one, and past the buffer at the last)
  const int need = (code == 1 || code == 3 || code == 5) ? 4 : ((code == 8 || code == 9) ? 1 : 3);
  if (code >= 0 && code <= 11 && (cin < need || cin > 4))
    throw std::invalid_argument("color conversion code " + std::to_string(code) + " needs a " + std::to_string(need) +
                                "-channel source, got " + std::to_string(cin));
  switch (code) {
    case 0: case 2: return 4;                 // BGR2BGRA / BGR2RGBA
    case 1: case 3: return 3;                 // BGRA2BGR / BGRA2RGB
    case 4: return 3;                         // BGR2RGB
    case 5: return 4;                         // BGRA2RGBA
    case 6: case 7: case 10: case 11: return 1;  // *2GRAY
    case 8: return 3;                         // GRAY2BGR
    case 9: return 4;                         // GRAY2BGRA
    default: throw std::invalid_argument("unsupported color conversion code " + std::to_string(code));
  }
}

void CvtColorHost(const uint8_t* src, int64_t npx, int cin, int code, uint8_t* dst) {
  const int cout = CvtChannelsOut(code, cin);
#pragma omp parallel for schedule(static) if (npx > 65536)
  for (int64_t i = 0; i < npx; ++i) {
    const uint8_t* s = src + i * cin;
    uint8_t* d = dst + i * cout;
    switch (code) {
      case 0: d[0] = s[0]; d[1] = s[1]; d[2] = s[2]; d[3] = 255; break;
      case 2: d[0] = s[2]; d[1] = s[1]; d[2] = s[0]; d[3] = 255; break;
      case 1: d[0] = s[0]; d[1] = s[1]; d[2] = s[2]; break;
      case 3: d[0] = s[2]; d[1] = s[1]; d[2] = s[0]; break;
      case 4: d[0] = s[2]; d[1] = s[1]; d[2] = s[0]; break;
      case 5: d[0] = s[2]; d[1] = s[1]; d[2] = s[0]; d[3] = s[3]; break;
      case 6: case 10: d[0] = Luma(s[0], s[1], s[2]); break;   // BGR(A)2GRAY
      case 7: case 11: d[0] = Luma(s[2], s[1], s[0]); break;   // RGB(A)2GRAY
      case 8: d[0] = d[1] = d[2] = s[0]; break;
      case 9: d[0] = d[1] = d[2] = s[0]; d[3] = 255; break;
    }
  }
}

void ToTensorHost(const uint8_t* src, int h, int w, int c, const int* chan_map, int cout, double scale,
                  const double* mean, const double* stdv, float* dst) {
#pragma omp parallel for schedule(static) if (static_cast<int64_t>(h) * w > 65536)
  for (int y = 0; y < h; ++y)
    for (int x = 0; x < w; ++x)
      for (int k = 0; k < cout; ++k) {
        const int sc = chan_map[k] < c ? chan_map[k] : c - 1;
        const double v = src[(static_cast<int64_t>(y) * w + x) * c + sc];
        dst[(static_cast<int64_t>(k) * h + y) * w + x] = static_cast<float>((v * scale - mean[k]) / stdv[k]);
      }
}

}  // namespace smlimg
