// Native host test of the image kernels (image_ops.cpp) for the ASan + UBSan build: resize up / down /
// to and from 1-pixel sizes, box blur and column filters with kernels larger than the image (the
// BORDER_REFLECT_101 walk), thresholds, every colour conversion and the tensorizer, on odd shapes with
// 1, 3 and 4 channels. Exit code != 0 on any mismatch.
#include <cmath>
#include <cstdio>
#include <random>
#include <stdexcept>
#include <vector>

#include "image_cpu.h"

using namespace smlimg;

static int failures = 0;
#define CHECK(c)                                                                   \
  do {                                                                             \
    if (!(c)) {                                                                    \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c);    \
      ++failures;                                                                  \
    }                                                                              \
  } while (0)

static std::vector<uint8_t> img(int h, int w, int c, std::mt19937& rng) {
  std::vector<uint8_t> v(static_cast<size_t>(h) * w * c);
  for (auto& x : v) x = static_cast<uint8_t>(rng() & 255);
  return v;
}

int main() {
  std::mt19937 rng(1);
  const int shapes[][2] = {{1, 1}, {1, 9}, {9, 1}, {2, 3}, {7, 13}, {31, 17}, {64, 48}};
  for (const auto& sh : shapes) {
    for (int c : {1, 3, 4}) {
      const int h = sh[0], w = sh[1];
      auto src = img(h, w, c, rng);
      // identity resize reproduces the image
      std::vector<uint8_t> same(src.size());
      ResizeHost(src.data(), h, w, c, same.data(), h, w);
      CHECK(same == src);
      for (const auto& d : shapes) {
        std::vector<uint8_t> dst(static_cast<size_t>(d[0]) * d[1] * c);
        ResizeHost(src.data(), h, w, c, dst.data(), d[0], d[1]);
      }
      // a constant image stays constant under resize / blur / normalised filters
      std::vector<uint8_t> flat(src.size(), 77), out(src.size());
      ResizeHost(flat.data(), h, w, c, out.data(), h, w);
      CHECK(out == flat);
      for (int k : {1, 3, 5, 2 * std::max(h, w) + 1}) {
        BoxBlurHost(flat.data(), h, w, c, out.data(), k, k);
        CHECK(out == flat);
        BoxBlurHost(src.data(), h, w, c, out.data(), k, std::max(1, k - 2));
        const auto g = GaussianKernel(k, 0.0);
        ColumnFilterHost(flat.data(), h, w, c, out.data(), g.data(), k);
        CHECK(out == flat);
        ColumnFilterHost(src.data(), h, w, c, out.data(), g.data(), k);
      }
      for (int type = 0; type <= 4; ++type) {
        ThresholdHost(src.data(), static_cast<int64_t>(src.size()), out.data(), 127.5, 200, type);
        for (size_t i = 0; i < src.size(); ++i) {
          if (type == 0) CHECK(out[i] == (src[i] > 127 ? 200 : 0));
          if (type == 3) CHECK(out[i] == (src[i] > 127 ? src[i] : 0));
        }
      }
      const int64_t npx = static_cast<int64_t>(h) * w;
      for (int code = 0; code <= 11; ++code) {
        const int need = (code == 1 || code == 3 || code == 5) ? 4 : ((code == 8 || code == 9) ? 1 : 3);
        int co = 0;
        try {
          co = CvtChannelsOut(code, c);
        } catch (const std::invalid_argument&) {
          CHECK(c < need);  // refused only when the source has too few channels
          continue;
        }
        CHECK(c >= need);
        std::vector<uint8_t> cv(static_cast<size_t>(npx) * co);
        CvtColorHost(src.data(), npx, c, code, cv.data());
      }
      const int map[4] = {2, 1, 0, 3};
      const double mean[4] = {0.485, 0.456, 0.406, 0.5}, stdv[4] = {0.229, 0.224, 0.225, 0.25};
      const int cout = std::min(c, 3);
      std::vector<float> t(static_cast<size_t>(cout) * npx);
      ToTensorHost(src.data(), h, w, c, map, cout, 1.0 / 255, mean, stdv, t.data());
      for (float v : t) CHECK(std::isfinite(v));
    }
  }
  int rejected = 0;
  try { std::vector<uint8_t> d(4); uint8_t s = 0; ResizeHost(&s, 0, 1, 1, d.data(), 2, 2); } catch (const std::exception&) { ++rejected; }
  try { CvtChannelsOut(99, 3); } catch (const std::exception&) { ++rejected; }
  CHECK(rejected == 2);
  if (failures) {
    std::fprintf(stderr, "%d failures\n", failures);
    return 1;
  }
  std::printf("all native image host tests passed\n");
  return 0;
}
