// Native baseline JPEG decoder for the image pipeline (the decode half of K19 in SURVEY §2.4: the
// reference decodes with OpenCV on its executors, ImageTransformer.scala:312-330 / ImageInjections).
//
// Scope: baseline / extended-Huffman sequential JPEG (SOF0 / SOF1), 8-bit samples, 1 component (gray) or
// 3 components (YCbCr -> RGB) in one interleaved scan, any sampling factors up to 2x2, restart intervals.
// Arithmetic IDCT, upsampling and colour conversion follow libjpeg's defaults (ISLOW integer IDCT, "fancy"
// triangle-filter chroma upsampling, fixed-point YCbCr tables), so the pixels match the decoder behind
// PIL / OpenCV. Anything else (progressive, multi-scan, arithmetic coding, 12-bit, CMYK, Adobe RGB) is
// reported as unsupported and the caller falls back to PIL for that image.
//
// Decoding runs on a pool of native threads with no Python involvement, straight into the caller's
// (pinned) buffer, so a batch of JPEGs decodes at core count x single-core speed.
#pragma once
#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

namespace smlimg {

struct JpegInfo {
  int width = 0, height = 0, channels = 0;  // channels: 1 (gray) or 3 (RGB output)
  bool supported = false;
  std::string why;  // reason when unsupported / invalid
};

// Parse the headers only (dimensions and whether this decoder handles the file).
JpegInfo JpegProbe(const uint8_t* data, size_t len);

// Decode into out (height * width * channels bytes, row-major, RGB or gray). Returns false with `why` set on
// any unsupported or corrupt input (out is then unspecified).
bool JpegDecode(const uint8_t* data, size_t len, uint8_t* out, size_t out_len, std::string* why);

// Batch: image i of (ptrs[i], lens[i]) decodes to out + offsets[i] (sized by a previous probe); ok[i] = 1 on
// success. `threads` native threads share the batch.
void JpegDecodeBatch(const std::vector<const uint8_t*>& ptrs, const std::vector<size_t>& lens, uint8_t* out,
                     const std::vector<int64_t>& offsets, const std::vector<int64_t>& sizes, uint8_t* ok,
                     int threads);

}  // namespace smlimg
