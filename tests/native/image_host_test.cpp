// Native host test of the image kernels (image_ops.cpp) for the ASan + UBSan build: resize up / down /
// to and from 1-pixel sizes, box blur and column filters with kernels larger than the image (the
// BORDER_REFLECT_101 walk), thresholds, every colour conversion and the tensorizer, on odd shapes with
// 1, 3 and 4 channels; the baseline JPEG decoder (jpeg_decode.cpp) on two embedded files (4:2:0 colour with
// restart markers, gray) against PIL's pixel sums, then on thousands of mutated / truncated copies, which
// must be rejected or decoded without any out-of-bounds access. Exit code != 0 on any mismatch.
#include <cmath>
#include <cstdio>
#include <algorithm>
#include <random>
#include <string>
#include <stdexcept>
#include <vector>

#include "image_cpu.h"
#include "jpeg_decode.h"

using namespace smlimg;

// written by PIL (quality 80 4:2:0 with DRI = 2 MCUs; quality 70 gray), 23x19
static const uint8_t kColor420[] = {255,216,255,224,0,16,74,70,73,70,0,1,1,0,0,1,0,1,0,0,255,219,0,67,0,6,4,5,6,5,4,6,6,5,6,7,7,6,8,10,16,10,10,9,9,10,20,14,15,12,16,23,20,24,24,23,20,22,22,26,29,37,31,26,27,35,28,22,22,32,44,32,35,38,39,41,42,41,25,31,45,48,45,40,48,37,40,41,40,255,219,0,67,1,7,7,7,10,8,10,19,10,10,19,40,26,22,26,40,40,40,40,40,40,40,40,40,40,40,40,40,40,40,40,40,40,40,40,40,40,40,40,40,40,40,40,40,40,40,40,40,40,40,40,40,40,40,40,40,40,40,40,40,40,40,40,40,40,255,192,0,17,8,0,19,0,23,3,1,34,0,2,17,1,3,17,1,255,196,0,31,0,0,1,5,1,1,1,1,1,1,0,0,0,0,0,0,0,0,1,2,3,4,5,6,7,8,9,10,11,255,196,0,181,16,0,2,1,3,3,2,4,3,5,5,4,4,0,0,1,125,1,2,3,0,4,17,5,18,33,49,65,6,19,81,97,7,34,113,20,50,129,145,161,8,35,66,177,193,21,82,209,240,36,51,98,114,130,9,10,22,23,24,25,26,37,38,39,40,41,42,52,53,54,55,56,57,58,67,68,69,70,71,72,73,74,83,84,85,86,87,88,89,90,99,100,101,102,103,104,105,106,115,116,117,118,119,120,121,122,131,132,133,134,135,136,137,138,146,147,148,149,150,151,152,153,154,162,163,164,165,166,167,168,169,170,178,179,180,181,182,183,184,185,186,194,195,196,197,198,199,200,201,202,210,211,212,213,214,215,216,217,218,225,226,227,228,229,230,231,232,233,234,241,242,243,244,245,246,247,248,249,250,255,196,0,31,1,0,3,1,1,1,1,1,1,1,1,1,0,0,0,0,0,0,1,2,3,4,5,6,7,8,9,10,11,255,196,0,181,17,0,2,1,2,4,4,3,4,7,5,4,4,0,1,2,119,0,1,2,3,17,4,5,33,49,6,18,65,81,7,97,113,19,34,50,129,8,20,66,145,161,177,193,9,35,51,82,240,21,98,114,209,10,22,36,52,225,37,241,23,24,25,26,38,39,40,41,42,53,54,55,56,57,58,67,68,69,70,71,72,73,74,83,84,85,86,87,88,89,90,99,100,101,102,103,104,105,106,115,116,117,118,119,120,121,122,130,131,132,133,134,135,136,137,138,146,147,148,149,150,151,152,153,154,162,163,164,165,166,167,168,169,170,178,179,180,181,182,183,184,185,186,194,195,196,197,198,199,200,201,202,210,211,212,213,214,215,216,217,218,226,227,228,229,230,231,232,233,234,242,243,244,245,246,247,248,249,250,255,221,0,4,0,2,255,218,0,12,3,1,0,2,17,3,17,0,63,0,241,59,79,14,204,160,180,74,92,6,194,236,95,188,120,29,115,245,39,28,254,64,87,79,162,232,108,64,221,20,102,66,27,25,5,112,120,228,31,192,156,255,0,60,215,89,167,248,116,161,49,237,69,59,87,59,48,73,3,57,3,190,222,64,207,111,198,186,93,47,65,111,51,230,95,37,126,249,12,9,203,100,224,103,166,115,146,84,245,235,208,98,184,233,226,122,92,230,201,120,131,187,254,191,174,199,45,166,232,121,82,206,21,79,80,195,25,207,112,14,49,140,238,234,123,14,58,81,94,171,167,248,124,176,49,186,55,64,170,161,120,29,79,205,128,51,211,142,71,81,69,116,202,164,103,173,209,250,118,31,136,33,24,37,57,114,159,255,208,235,44,108,224,89,10,42,109,85,219,128,24,142,216,254,92,87,71,167,70,131,77,51,4,65,41,132,57,96,160,114,91,159,228,63,42,40,175,159,161,38,235,164,222,151,253,15,206,178,57,55,54,159,116,117,122,76,17,45,143,152,171,135,83,193,7,234,63,144,20,81,69,122,144,138,215,67,239,105,206,92,171,83,255,217};
static const uint8_t kGray[] = {255,216,255,224,0,16,74,70,73,70,0,1,1,0,0,1,0,1,0,0,255,219,0,67,0,10,7,7,8,7,6,10,8,8,8,11,10,10,11,14,24,16,14,13,13,14,29,21,22,17,24,35,31,37,36,34,31,34,33,38,43,55,47,38,41,52,41,33,34,48,65,49,52,57,59,62,62,62,37,46,68,73,67,60,72,55,61,62,59,255,192,0,11,8,0,19,0,23,1,1,17,0,255,196,0,31,0,0,1,5,1,1,1,1,1,1,0,0,0,0,0,0,0,0,1,2,3,4,5,6,7,8,9,10,11,255,196,0,181,16,0,2,1,3,3,2,4,3,5,5,4,4,0,0,1,125,1,2,3,0,4,17,5,18,33,49,65,6,19,81,97,7,34,113,20,50,129,145,161,8,35,66,177,193,21,82,209,240,36,51,98,114,130,9,10,22,23,24,25,26,37,38,39,40,41,42,52,53,54,55,56,57,58,67,68,69,70,71,72,73,74,83,84,85,86,87,88,89,90,99,100,101,102,103,104,105,106,115,116,117,118,119,120,121,122,131,132,133,134,135,136,137,138,146,147,148,149,150,151,152,153,154,162,163,164,165,166,167,168,169,170,178,179,180,181,182,183,184,185,186,194,195,196,197,198,199,200,201,202,210,211,212,213,214,215,216,217,218,225,226,227,228,229,230,231,232,233,234,241,242,243,244,245,246,247,248,249,250,255,218,0,8,1,1,0,0,63,0,243,232,116,121,7,40,165,128,110,54,142,167,129,215,243,38,181,236,52,182,35,152,212,177,7,28,17,207,29,15,224,121,254,117,179,107,165,228,18,216,30,132,117,250,103,30,185,234,105,214,218,62,211,179,106,142,6,118,242,72,25,200,29,241,200,173,107,61,40,239,228,121,99,239,16,70,114,115,235,245,207,21,181,109,164,22,202,50,158,128,0,7,3,175,94,149,5,189,188,65,202,133,192,24,198,9,173,91,84,95,177,153,66,168,115,30,236,129,142,73,231,249,10,218,179,137,5,182,240,184,96,122,254,99,250,10,255,217};

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
  // ---- JPEG decoder
  {
    struct Case { const uint8_t* d; size_t n; int c; long long sum; };
    const Case cases[] = {{kColor420, sizeof(kColor420), 3, 149201}, {kGray, sizeof(kGray), 1, 51390}};
    for (const auto& cs : cases) {
      JpegInfo info = JpegProbe(cs.d, cs.n);
      CHECK(info.supported && info.width == 23 && info.height == 19 && info.channels == cs.c);
      std::vector<uint8_t> out(static_cast<size_t>(23) * 19 * cs.c);
      std::string why;
      CHECK(JpegDecode(cs.d, cs.n, out.data(), out.size(), &why));
      long long sum = 0;
      for (uint8_t v : out) sum += v;
      CHECK(sum == cs.sum);
      CHECK(!JpegDecode(cs.d, cs.n, out.data(), out.size() - 1, &why));  // too-small buffer refused
      // mutations: byte flips, truncation, random garbage runs
      std::vector<uint8_t> buf;
      for (int it = 0; it < 3000; ++it) {
        buf.assign(cs.d, cs.d + cs.n);
        const int kind = it % 3;
        if (kind == 0) {
          for (int k = 0; k < 1 + static_cast<int>(rng() % 4); ++k) buf[rng() % buf.size()] = static_cast<uint8_t>(rng());
        } else if (kind == 1) {
          buf.resize(rng() % buf.size());
        } else {
          const size_t at = rng() % buf.size();
          for (size_t k = at; k < std::min(buf.size(), at + 1 + rng() % 32); ++k) buf[k] = static_cast<uint8_t>(rng());
        }
        JpegInfo mi = JpegProbe(buf.data(), buf.size());
        if (!mi.supported) continue;
        std::vector<uint8_t> o(static_cast<size_t>(mi.width) * mi.height * mi.channels);
        JpegDecode(buf.data(), buf.size(), o.data(), o.size(), &why);
      }
    }
    // truncated SOS segments at the very end of the input (segment length 2 = no component count, and a
    // count whose component list runs past the segment): refused without reading past the buffer (ASan)
    {
      size_t sos = 0;
      for (size_t i = 0; i + 1 < sizeof(kColor420); ++i)
        if (kColor420[i] == 0xFF && kColor420[i + 1] == 0xDA) { sos = i; break; }
      CHECK(sos > 0);
      for (int seglen : {2, 3, 4}) {
        std::vector<uint8_t> t(kColor420, kColor420 + sos + 2);
        t.push_back(0);
        t.push_back(static_cast<uint8_t>(seglen));
        if (seglen >= 3) t.push_back(3);  // 3 components named, none or one listed
        if (seglen >= 4) t.push_back(1);
        t.shrink_to_fit();
        std::string why;
        std::vector<uint8_t> o(23 * 19 * 3);
        CHECK(!JpegDecode(t.data(), t.size(), o.data(), o.size(), &why));
      }
    }
    // threaded batch: both files twice, plus an invalid entry
    std::vector<const uint8_t*> ptrs = {kColor420, kGray, kColor420, kGray, kGray};
    std::vector<size_t> lens = {sizeof(kColor420), sizeof(kGray), sizeof(kColor420), sizeof(kGray), 10};
    std::vector<int64_t> sizes = {23 * 19 * 3, 23 * 19, 23 * 19 * 3, 23 * 19, 23 * 19};
    std::vector<int64_t> offs(5, 0);
    for (int i = 1; i < 5; ++i) offs[i] = offs[i - 1] + sizes[i - 1];
    std::vector<uint8_t> all(static_cast<size_t>(offs[4] + sizes[4]));
    std::vector<uint8_t> ok(5);
    JpegDecodeBatch(ptrs, lens, all.data(), offs, sizes, ok.data(), 3);
    CHECK(ok[0] && ok[1] && ok[2] && ok[3] && !ok[4]);
    CHECK(std::equal(all.begin(), all.begin() + sizes[0], all.begin() + offs[2]));
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
