// Baseline JPEG decoder (see jpeg_decode.h). Written from the JPEG specification (ITU-T T.81 Annex F
// Huffman decoding, A.3.3 IDCT) with libjpeg's default arithmetic for the parts the standard leaves open
// (ISLOW integer IDCT constants, triangle-filter chroma upsampling, 16-bit fixed-point YCbCr tables), so
// the output matches the decoder PIL and OpenCV use.
#include "jpeg_decode.h"

#include <algorithm>
#include <atomic>
#include <climits>
#include <cstring>
#include <thread>

namespace smlimg {
namespace {

// natural (row-major) index of the k-th coefficient in zigzag order
constexpr uint8_t kNatural[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,
                                  12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28,
                                  35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
                                  58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

constexpr int kFastBits = 9;
constexpr int kMaxDim = 1 << 15;

struct Huff {
  uint16_t fast[1 << kFastBits];  // (length << 8) | symbol; 0 = longer than kFastBits
  int32_t maxcode[18];
  int32_t valptr[17];
  int32_t mincode[17];
  uint8_t vals[256];
  // AC fast path: (value << 16) | (run << 8) | (code length + magnitude bits) for codes whose symbol and
  // magnitude bits both fit in kFastBits; 0 = take the slow path
  int32_t ac_fast[1 << kFastBits];
  bool present = false;
};

bool BuildHuff(Huff* h, const uint8_t* counts, const uint8_t* vals, int nvals) {
  std::memset(h->fast, 0, sizeof(h->fast));
  std::memcpy(h->vals, vals, static_cast<size_t>(nvals));
  int code = 0, k = 0;
  for (int len = 1; len <= 16; ++len) {
    h->valptr[len] = k;
    h->mincode[len] = code;
    const int n = counts[len - 1];
    if (k + n > nvals) return false;
    for (int i = 0; i < n; ++i, ++k, ++code) {
      if (len <= kFastBits) {
        const int shift = kFastBits - len;
        for (int s = 0; s < (1 << shift); ++s) h->fast[(code << shift) | s] = static_cast<uint16_t>((len << 8) | vals[k]);
      }
    }
    h->maxcode[len] = n ? code - 1 : -1;
    if (code > (1 << len)) return false;  // over-subscribed code
    code <<= 1;
  }
  h->maxcode[17] = INT_MAX;
  for (int i = 0; i < (1 << kFastBits); ++i) {
    h->ac_fast[i] = 0;
    const uint16_t f = h->fast[i];
    if (!f) continue;
    const int len = f >> 8, rs = f & 255, run = rs >> 4, mag = rs & 15;
    if (mag == 0 || len + mag > kFastBits) continue;
    int v = (i >> (kFastBits - len - mag)) & ((1 << mag) - 1);
    if (v < (1 << (mag - 1))) v -= (1 << mag) - 1;
    h->ac_fast[i] = static_cast<int32_t>((static_cast<uint32_t>(v) << 16) | (run << 8) | (len + mag));
  }
  h->present = true;
  return true;
}

struct Bits {
  const uint8_t* p;
  const uint8_t* end;
  uint64_t buf = 0;
  int n = 0;
  bool marker = false;  // a marker (not a stuffed 0xFF00) was reached: zeros are fed from here on
  int pad = 0;          // zero bits fed past the end of the entropy-coded segment

  void Fill() {
    while (n <= 56) {
      uint32_t b = 0;
      if (!marker && p < end) {
        b = *p++;
        if (b == 0xFF) {
          const uint8_t nx = p < end ? *p : 0xD9;
          if (nx == 0x00) {
            ++p;  // stuffed byte
          } else {
            marker = true;
            --p;  // leave the marker for the restart handler
            b = 0;
          }
        }
      } else {
        pad += 8;
      }
      buf |= static_cast<uint64_t>(b) << (56 - n);
      n += 8;
    }
  }
  int Get(int k) {
    if (k == 0) return 0;
    if (n < k) Fill();
    const int v = static_cast<int>(buf >> (64 - k));
    buf <<= k;
    n -= k;
    return v;
  }
  int Decode(const Huff& h) {
    if (n < 16) Fill();
    const uint16_t f = h.fast[buf >> (64 - kFastBits)];
    if (f) {
      const int len = f >> 8;
      buf <<= len;
      n -= len;
      return f & 255;
    }
    for (int len = kFastBits + 1; len <= 16; ++len) {
      const int code = static_cast<int>(buf >> (64 - len));
      if (code <= h.maxcode[len]) {
        buf <<= len;
        n -= len;
        const int idx = h.valptr[len] + code - h.mincode[len];
        return idx >= 0 && idx < 256 ? h.vals[idx] : -1;
      }
    }
    return -1;
  }
  // more bits were consumed than the segment holds (the fed zeros still buffered are not consumed)
  bool Overrun() const { return pad > n; }
  static int Extend(int v, int s) { return s == 0 ? 0 : (v < (1 << (s - 1)) ? v - (1 << s) + 1 : v); }
  // restart marker: drop the partial byte, step over RSTn
  bool Restart() {
    buf = 0;
    n = 0;
    pad = 0;
    if (marker && p + 1 < end && p[0] == 0xFF && p[1] >= 0xD0 && p[1] <= 0xD7) {
      p += 2;
      marker = false;
      return true;
    }
    // tolerate a missing marker by scanning for the next RSTn
    while (p + 1 < end && !(p[0] == 0xFF && p[1] >= 0xD0 && p[1] <= 0xD7)) ++p;
    if (p + 1 < end) {
      p += 2;
      marker = false;
      return true;
    }
    return false;
  }
};

// ---------------------------------------------------------------- ISLOW IDCT (libjpeg jidctint)
constexpr int kConstBits = 13, kPass1Bits = 2;
constexpr int32_t F0298 = 2446, F0390 = 3196, F0541 = 4433, F0765 = 6270, F0899 = 7373, F1175 = 9633,
                  F1501 = 12299, F1847 = 15137, F1961 = 16069, F2053 = 16819, F2562 = 20995, F3072 = 25172;

template <class T>
inline int32_t Descale(T x, int n) { return static_cast<int32_t>((x + (T(1) << (n - 1))) >> n); }
inline uint8_t Clamp8(int v) { return static_cast<uint8_t>(v < 0 ? 0 : (v > 255 ? 255 : v)); }

// coef: dequantized coefficients in natural order; out: 8x8 samples, row stride `stride`.
// T = int32_t is libjpeg's own 32-bit arithmetic, exact for blocks whose dequantized coefficients stay in the
// range 8-bit sample data can produce (|c| < 2^12, checked by the caller); anything larger (corrupt data) runs
// with T = int64_t so no intermediate overflows.
template <class T>
void Idct8x8(const int32_t* coef, uint8_t* out, int stride) {
  int32_t ws[64];
  for (int c = 0; c < 8; ++c) {
    const int32_t* in = coef + c;
    int32_t* w = ws + c;
    if (!in[8] && !in[16] && !in[24] && !in[32] && !in[40] && !in[48] && !in[56]) {
      const int32_t dc = in[0] * (1 << kPass1Bits);
      for (int r = 0; r < 8; ++r) w[8 * r] = dc;
      continue;
    }
    T z2 = in[16], z3 = in[48];
    T z1 = (z2 + z3) * F0541;
    T tmp2 = z1 + z3 * -F1847, tmp3 = z1 + z2 * F0765;
    z2 = in[0];
    z3 = in[32];
    T tmp0 = (z2 + z3) * (1 << kConstBits), tmp1 = (z2 - z3) * (1 << kConstBits);
    const T t10 = tmp0 + tmp3, t13 = tmp0 - tmp3, t11 = tmp1 + tmp2, t12 = tmp1 - tmp2;
    tmp0 = in[56]; tmp1 = in[40]; tmp2 = in[24]; tmp3 = in[8];
    z1 = tmp0 + tmp3; z2 = tmp1 + tmp2; z3 = tmp0 + tmp2;
    T z4 = tmp1 + tmp3;
    const T z5 = (z3 + z4) * F1175;
    tmp0 *= F0298; tmp1 *= F2053; tmp2 *= F3072; tmp3 *= F1501;
    z1 *= -F0899; z2 *= -F2562; z3 *= -F1961; z4 *= -F0390;
    z3 += z5; z4 += z5;
    tmp0 += z1 + z3; tmp1 += z2 + z4; tmp2 += z2 + z3; tmp3 += z1 + z4;
    const int sh = kConstBits - kPass1Bits;
    w[0] = Descale(t10 + tmp3, sh); w[56] = Descale(t10 - tmp3, sh);
    w[8] = Descale(t11 + tmp2, sh); w[48] = Descale(t11 - tmp2, sh);
    w[16] = Descale(t12 + tmp1, sh); w[40] = Descale(t12 - tmp1, sh);
    w[24] = Descale(t13 + tmp0, sh); w[32] = Descale(t13 - tmp0, sh);
  }
  for (int r = 0; r < 8; ++r) {
    const int32_t* w = ws + 8 * r;
    uint8_t* o = out + r * stride;
    if (!w[1] && !w[2] && !w[3] && !w[4] && !w[5] && !w[6] && !w[7]) {
      const uint8_t v = Clamp8(Descale(w[0], kPass1Bits + 3) + 128);
      for (int c = 0; c < 8; ++c) o[c] = v;
      continue;
    }
    T z2 = w[2], z3 = w[6];
    T z1 = (z2 + z3) * F0541;
    T tmp2 = z1 + z3 * -F1847, tmp3 = z1 + z2 * F0765;
    T tmp0 = (static_cast<T>(w[0]) + w[4]) * (1 << kConstBits);
    T tmp1 = (static_cast<T>(w[0]) - w[4]) * (1 << kConstBits);
    const T t10 = tmp0 + tmp3, t13 = tmp0 - tmp3, t11 = tmp1 + tmp2, t12 = tmp1 - tmp2;
    tmp0 = w[7]; tmp1 = w[5]; tmp2 = w[3]; tmp3 = w[1];
    z1 = tmp0 + tmp3; z2 = tmp1 + tmp2; z3 = tmp0 + tmp2;
    T z4 = tmp1 + tmp3;
    const T z5 = (z3 + z4) * F1175;
    tmp0 *= F0298; tmp1 *= F2053; tmp2 *= F3072; tmp3 *= F1501;
    z1 *= -F0899; z2 *= -F2562; z3 *= -F1961; z4 *= -F0390;
    z3 += z5; z4 += z5;
    tmp0 += z1 + z3; tmp1 += z2 + z4; tmp2 += z2 + z3; tmp3 += z1 + z4;
    const int sh = kConstBits + kPass1Bits + 3;
    o[0] = Clamp8(Descale(t10 + tmp3, sh) + 128); o[7] = Clamp8(Descale(t10 - tmp3, sh) + 128);
    o[1] = Clamp8(Descale(t11 + tmp2, sh) + 128); o[6] = Clamp8(Descale(t11 - tmp2, sh) + 128);
    o[2] = Clamp8(Descale(t12 + tmp1, sh) + 128); o[5] = Clamp8(Descale(t12 - tmp1, sh) + 128);
    o[3] = Clamp8(Descale(t13 + tmp0, sh) + 128); o[4] = Clamp8(Descale(t13 - tmp0, sh) + 128);
  }
}

// ---------------------------------------------------------------- header + scan
struct Comp {
  int id = 0, h = 1, v = 1, tq = 0, td = 0, ta = 0;
  int bw = 0, bh = 0;  // plane size in blocks
  int dw = 0, dh = 0;  // downsampled (real) size in samples
  std::vector<uint8_t> plane;
  int pred = 0;
};

struct Jpeg {
  int width = 0, height = 0, ncomp = 0, restart = 0;
  bool baseline = false, adobe_rgb = false, sos = false;
  uint16_t qt[4][64];
  bool qt_present[4] = {};
  Huff dc[4], ac[4];
  Comp comp[3];
  int scan_comp[3] = {0, 1, 2}, scan_n = 0;
  const uint8_t* scan_begin = nullptr;
  std::string why;
};

inline int Be16(const uint8_t* p) { return (p[0] << 8) | p[1]; }

// parse up to the first SOS (headers only); scan_begin points at the entropy-coded data
bool ParseHeaders(const uint8_t* d, size_t len, Jpeg* j) {
  const uint8_t* p = d;
  const uint8_t* end = d + len;
  if (len < 4 || p[0] != 0xFF || p[1] != 0xD8) { j->why = "not a JPEG (no SOI)"; return false; }
  p += 2;
  while (p < end) {
    while (p < end && *p != 0xFF) ++p;  // tolerate garbage between segments
    while (p < end && *p == 0xFF) ++p;  // fill bytes
    if (p >= end) break;
    const uint8_t m = *p++;
    if (m == 0xD8 || (m >= 0xD0 && m <= 0xD7) || m == 0x01) continue;
    if (m == 0xD9) break;
    if (p + 2 > end) { j->why = "truncated segment"; return false; }
    const int seg = Be16(p);
    if (seg < 2 || p + seg > end) { j->why = "truncated segment"; return false; }
    const uint8_t* s = p + 2;
    const uint8_t* se = p + seg;
    switch (m) {
      case 0xDB:  // DQT
        while (s < se) {
          const int pq = *s >> 4, tq = *s & 15;
          ++s;
          if (tq > 3 || s + (pq ? 128 : 64) > se) { j->why = "bad DQT"; return false; }
          for (int k = 0; k < 64; ++k) j->qt[tq][k] = pq ? static_cast<uint16_t>(Be16(s + 2 * k)) : s[k];
          s += pq ? 128 : 64;
          j->qt_present[tq] = true;
        }
        break;
      case 0xC0: case 0xC1: {  // SOF0 / SOF1
        if (se - s < 6) { j->why = "bad SOF"; return false; }
        if (s[0] != 8) { j->why = "only 8-bit samples"; return false; }
        j->height = Be16(s + 1);
        j->width = Be16(s + 3);
        j->ncomp = s[5];
        if (j->ncomp != 1 && j->ncomp != 3) { j->why = "only gray or YCbCr"; return false; }
        if (se - s < 6 + 3 * j->ncomp) { j->why = "bad SOF"; return false; }
        for (int c = 0; c < j->ncomp; ++c) {
          Comp& k = j->comp[c];
          k.id = s[6 + 3 * c];
          k.h = s[7 + 3 * c] >> 4;
          k.v = s[7 + 3 * c] & 15;
          k.tq = s[8 + 3 * c] & 3;
          if (k.h < 1 || k.h > 2 || k.v < 1 || k.v > 2) { j->why = "sampling factor"; return false; }
        }
        j->baseline = true;
        break;
      }
      case 0xC2: case 0xC3: case 0xC5: case 0xC6: case 0xC7: case 0xC9: case 0xCA: case 0xCB: case 0xCD:
      case 0xCE: case 0xCF:
        j->why = "progressive / lossless / arithmetic JPEG";
        return false;
      case 0xC4:  // DHT
        while (s < se) {
          const int tc = *s >> 4, th = *s & 15;
          ++s;
          if (tc > 1 || th > 3 || s + 16 > se) { j->why = "bad DHT"; return false; }
          int nv = 0;
          for (int i = 0; i < 16; ++i) nv += s[i];
          if (nv > 256 || s + 16 + nv > se) { j->why = "bad DHT"; return false; }
          if (!BuildHuff(tc ? &j->ac[th] : &j->dc[th], s, s + 16, nv)) { j->why = "bad Huffman table"; return false; }
          s += 16 + nv;
        }
        break;
      case 0xDD:
        if (se - s < 2) { j->why = "bad DRI"; return false; }
        j->restart = Be16(s);
        break;
      case 0xEE:  // Adobe: transform 0 = RGB / CMYK stored as is
        if (se - s >= 12 && std::memcmp(s, "Adobe", 5) == 0 && s[11] == 0 && j->ncomp == 3) j->adobe_rgb = true;
        break;
      case 0xDA: {  // SOS
        if (!j->baseline) { j->why = "SOS before SOF"; return false; }
        if (se - s < 1) { j->why = "bad SOS"; return false; }
        const int ns = s[0];
        if (ns != j->ncomp) { j->why = "multi-scan JPEG"; return false; }
        if (se - s < 1 + 2 * ns) { j->why = "bad SOS"; return false; }
        for (int i = 0; i < ns; ++i) {
          const int cid = s[1 + 2 * i];
          int c = 0;
          while (c < j->ncomp && j->comp[c].id != cid) ++c;
          if (c == j->ncomp) { j->why = "scan names an unknown component"; return false; }
          j->scan_comp[i] = c;
          j->comp[c].td = s[2 + 2 * i] >> 4;
          j->comp[c].ta = s[2 + 2 * i] & 15;
          if (j->comp[c].td > 3 || j->comp[c].ta > 3) { j->why = "bad table id"; return false; }
        }
        j->scan_n = ns;
        j->scan_begin = se;
        j->sos = true;
        return true;
      }
      default:
        break;
    }
    p = se;
  }
  j->why = "no scan";
  return false;
}

bool Validate(Jpeg* j) {
  if (j->width <= 0 || j->height <= 0 || j->width > kMaxDim || j->height > kMaxDim) { j->why = "bad dimensions"; return false; }
  if (j->adobe_rgb) { j->why = "Adobe RGB-coded JPEG"; return false; }
  for (int c = 0; c < j->ncomp; ++c) {
    const Comp& k = j->comp[c];
    if (!j->qt_present[k.tq] || !j->dc[k.td].present || !j->ac[k.ta].present) { j->why = "missing table"; return false; }
  }
  if (j->ncomp == 3) {
    // luma at the maximum sampling, chroma at 1x1 (4:4:4, 4:2:2, 4:2:0, 4:4:0)
    if (j->comp[1].h != 1 || j->comp[1].v != 1 || j->comp[2].h != 1 || j->comp[2].v != 1) {
      j->why = "chroma sampling";
      return false;
    }
  }
  return true;
}

bool DecodeScan(const uint8_t* end, Jpeg* j) {
  int hmax = 1, vmax = 1;
  for (int c = 0; c < j->ncomp; ++c) { hmax = std::max(hmax, j->comp[c].h); vmax = std::max(vmax, j->comp[c].v); }
  const bool single = j->ncomp == 1;
  const int mcuw = single ? 8 : 8 * hmax, mcuh = single ? 8 : 8 * vmax;
  const int mcux = (j->width + mcuw - 1) / mcuw, mcuy = (j->height + mcuh - 1) / mcuh;
  for (int c = 0; c < j->ncomp; ++c) {
    Comp& k = j->comp[c];
    const int hs = single ? 1 : k.h, vs = single ? 1 : k.v;
    k.bw = mcux * hs;
    k.bh = mcuy * vs;
    k.dw = (j->width * k.h + hmax - 1) / hmax;
    k.dh = (j->height * k.v + vmax - 1) / vmax;
    if (single) { k.dw = j->width; k.dh = j->height; }
    k.plane.assign(static_cast<size_t>(k.bw) * 8 * k.bh * 8, 0);
    k.pred = 0;
  }
  Bits bits{j->scan_begin, end};
  int32_t coef[64];
  int mcus_left = j->restart;
  const int total = mcux * mcuy;
  for (int m = 0; m < total; ++m) {
    if (j->restart && mcus_left == 0) {
      if (!bits.Restart()) return false;
      for (int c = 0; c < j->ncomp; ++c) j->comp[c].pred = 0;
      mcus_left = j->restart;
    }
    const int mx = m % mcux, my = m / mcux;
    for (int si = 0; si < j->scan_n; ++si) {
      Comp& k = j->comp[j->scan_comp[si]];
      const int hs = single ? 1 : k.h, vs = single ? 1 : k.v;
      const uint16_t* q = j->qt[k.tq];
      for (int by = 0; by < vs; ++by)
        for (int bx = 0; bx < hs; ++bx) {
          std::memset(coef, 0, sizeof(coef));
          const int t = bits.Decode(j->dc[k.td]);
          if (t < 0 || t > 11) return false;
          k.pred = static_cast<int32_t>(static_cast<uint32_t>(k.pred) + static_cast<uint32_t>(Bits::Extend(bits.Get(t), t)));
          coef[0] = static_cast<int16_t>(k.pred) * q[0];  // libjpeg keeps coefficients as 16-bit JCOEF
          int last = 0;
          int32_t amax = coef[0] < 0 ? -coef[0] : coef[0];
          const Huff& ac = j->ac[k.ta];
          for (int kk = 1; kk < 64;) {
            if (bits.n < 16) bits.Fill();
            const int32_t fa = ac.ac_fast[bits.buf >> (64 - kFastBits)];
            if (fa) {
              kk += (fa >> 8) & 255;
              if (kk > 63) return false;
              const int tl = fa & 255;
              bits.buf <<= tl;
              bits.n -= tl;
              const int32_t cv = (fa >> 16) * q[kk];
            amax |= cv < 0 ? -cv : cv;
            coef[kNatural[kk]] = cv;
              last = kk++;
              continue;
            }
            const int rs = bits.Decode(ac);
            if (rs < 0) return false;
            const int r = rs >> 4, s = rs & 15;
            if (s == 0) {
              if (r != 15) break;  // EOB
              kk += 16;
              continue;
            }
            kk += r;
            if (kk > 63) return false;
            const int32_t cv = Bits::Extend(bits.Get(s), s) * q[kk];
            amax |= cv < 0 ? -cv : cv;
            coef[kNatural[kk]] = cv;
            last = kk++;
          }
          const int bcol = mx * hs + bx, brow = my * vs + by;
          uint8_t* dst = k.plane.data() + static_cast<size_t>(brow) * 8 * k.bw * 8 + bcol * 8;
          if (last == 0) {  // DC only: both IDCT passes reduce to one constant
            const uint8_t v = Clamp8(Descale(static_cast<int64_t>(coef[0]) * (1 << kPass1Bits), kPass1Bits + 3) + 128);
            for (int r = 0; r < 8; ++r) std::memset(dst + r * k.bw * 8, v, 8);
          } else if (amax < 4096) {
            Idct8x8<int32_t>(coef, dst, k.bw * 8);
          } else {
            Idct8x8<int64_t>(coef, dst, k.bw * 8);
          }
        }
    }
    if (bits.Overrun()) return false;
    --mcus_left;
  }
  return true;
}

// chroma plane (dw x dh real samples, row stride `stride`) upsampled by (fh, fv) into full-res row `y`
// (libjpeg's fancy upsampling for 2x1, 2x2, 1x2; replication otherwise)
void UpsampleRow(const Comp& k, int fh, int fv, int y, int width, uint8_t* out) {
  const int stride = k.bw * 8;
  const uint8_t* plane = k.plane.data();
  auto row = [&](int r) { return plane + static_cast<size_t>(std::min(std::max(r, 0), k.dh - 1)) * stride; };
  if (fh == 1 && fv == 1) {
    std::memcpy(out, row(y), static_cast<size_t>(width));
    return;
  }
  if (fh == 2 && fv == 1) {
    const uint8_t* in = row(y);
    const int dw = k.dw;
    uint8_t tmp[2 * kMaxDim + 4];
    uint8_t* o = tmp;
    if (dw == 1) { o[0] = o[1] = in[0]; }
    else {
      int v = in[0];
      *o++ = static_cast<uint8_t>(v);
      *o++ = static_cast<uint8_t>((v * 3 + in[1] + 2) >> 2);
      for (int c = 1; c < dw - 1; ++c) {
        v = in[c] * 3;
        *o++ = static_cast<uint8_t>((v + in[c - 1] + 1) >> 2);
        *o++ = static_cast<uint8_t>((v + in[c + 1] + 2) >> 2);
      }
      v = in[dw - 1];
      *o++ = static_cast<uint8_t>((v * 3 + in[dw - 2] + 1) >> 2);
      *o++ = static_cast<uint8_t>(v);
    }
    std::memcpy(out, tmp, static_cast<size_t>(width));
    return;
  }
  if (fv == 2) {
    const int r0 = y >> 1;
    const bool upper = (y & 1) == 0;
    const uint8_t* in0 = row(r0);
    const uint8_t* in1 = row(upper ? r0 - 1 : r0 + 1);
    const int dw = k.dw;
    if (fh == 2) {
      uint8_t tmp[2 * kMaxDim + 4];
      uint8_t* o = tmp;
      if (dw == 1) {
        const int s = in0[0] * 3 + in1[0];
        o[0] = static_cast<uint8_t>((s * 4 + 8) >> 4);
        o[1] = static_cast<uint8_t>((s * 4 + 7) >> 4);
      } else {
        int thiss = in0[0] * 3 + in1[0], nexts = in0[1] * 3 + in1[1], lasts;
        *o++ = static_cast<uint8_t>((thiss * 4 + 8) >> 4);
        *o++ = static_cast<uint8_t>((thiss * 3 + nexts + 7) >> 4);
        lasts = thiss;
        thiss = nexts;
        for (int c = 2; c < dw; ++c) {
          nexts = in0[c] * 3 + in1[c];
          *o++ = static_cast<uint8_t>((thiss * 3 + lasts + 8) >> 4);
          *o++ = static_cast<uint8_t>((thiss * 3 + nexts + 7) >> 4);
          lasts = thiss;
          thiss = nexts;
        }
        *o++ = static_cast<uint8_t>((thiss * 3 + lasts + 8) >> 4);
        *o++ = static_cast<uint8_t>((thiss * 4 + 7) >> 4);
      }
      std::memcpy(out, tmp, static_cast<size_t>(width));
    } else {  // h1v2
      const int bias = upper ? 1 : 2;
      for (int c = 0; c < width; ++c) out[c] = static_cast<uint8_t>((in0[c] * 3 + in1[c] + bias) >> 2);
    }
    return;
  }
  // other ratios: replication
  const uint8_t* in = row(y / fv);
  for (int c = 0; c < width; ++c) out[c] = in[c / fh];
}

struct YccTables {
  int cr_r[256], cb_b[256], cr_g[256], cb_g[256];
  uint8_t range[1024];
  YccTables() {
    for (int i = 0; i < 1024; ++i) range[i] = Clamp8(i - 384);
    constexpr int kScale = 16;
    auto fix = [](double x) { return static_cast<int>(x * (1 << kScale) + 0.5); };
    for (int i = 0; i < 256; ++i) {
      const int x = i - 128;
      cr_r[i] = (fix(1.40200) * x + (1 << (kScale - 1))) >> kScale;
      cb_b[i] = (fix(1.77200) * x + (1 << (kScale - 1))) >> kScale;
      cr_g[i] = -fix(0.71414) * x;
      cb_g[i] = -fix(0.34414) * x + (1 << (kScale - 1));
    }
  }
};
const YccTables& Ycc() {
  static const YccTables t;
  return t;
}

bool Emit(const Jpeg& j, uint8_t* out) {
  const int W = j.width, H = j.height;
  if (j.ncomp == 1) {
    const Comp& k = j.comp[0];
    for (int y = 0; y < H; ++y) std::memcpy(out + static_cast<size_t>(y) * W, k.plane.data() + static_cast<size_t>(y) * k.bw * 8, W);
    return true;
  }
  int hmax = 1, vmax = 1;
  for (int c = 0; c < 3; ++c) { hmax = std::max(hmax, j.comp[c].h); vmax = std::max(vmax, j.comp[c].v); }
  const YccTables& T = Ycc();
  std::vector<uint8_t> cb(W), cr(W);
  const Comp &Y = j.comp[0], &Cb = j.comp[1], &Cr = j.comp[2];
  for (int y = 0; y < H; ++y) {
    const uint8_t* yr = Y.plane.data() + static_cast<size_t>(y) * Y.bw * 8;
    UpsampleRow(Cb, hmax / Cb.h, vmax / Cb.v, y, W, cb.data());
    UpsampleRow(Cr, hmax / Cr.h, vmax / Cr.v, y, W, cr.data());
    uint8_t* o = out + static_cast<size_t>(y) * W * 3;
    const uint8_t* lim = T.range + 384;  // branchless clamp: lim[v] for v in [-384, 640)
    for (int x = 0; x < W; ++x) {
      const int yy = yr[x], b = cb[x], r = cr[x];
      o[3 * x] = lim[yy + T.cr_r[r]];
      o[3 * x + 1] = lim[yy + ((T.cb_g[b] + T.cr_g[r]) >> 16)];
      o[3 * x + 2] = lim[yy + T.cb_b[b]];
    }
  }
  return true;
}

}  // namespace

JpegInfo JpegProbe(const uint8_t* data, size_t len) {
  JpegInfo info;
  Jpeg j;
  if (!ParseHeaders(data, len, &j)) { info.why = j.why; return info; }
  info.width = j.width;
  info.height = j.height;
  info.channels = j.ncomp == 1 ? 1 : 3;
  info.supported = Validate(&j);
  info.why = j.why;
  return info;
}

bool JpegDecode(const uint8_t* data, size_t len, uint8_t* out, size_t out_len, std::string* why) {
  Jpeg j;
  if (!ParseHeaders(data, len, &j) || !Validate(&j)) { if (why) *why = j.why; return false; }
  const size_t need = static_cast<size_t>(j.width) * j.height * (j.ncomp == 1 ? 1 : 3);
  if (out_len < need) { if (why) *why = "output buffer too small"; return false; }
  if (!DecodeScan(data + len, &j)) { if (why) *why = "corrupt or truncated entropy-coded data"; return false; }
  return Emit(j, out);
}

void JpegDecodeBatch(const std::vector<const uint8_t*>& ptrs, const std::vector<size_t>& lens, uint8_t* out,
                     const std::vector<int64_t>& offsets, const std::vector<int64_t>& sizes, uint8_t* ok,
                     int threads) {
  const int64_t n = static_cast<int64_t>(ptrs.size());
  std::atomic<int64_t> next{0};
  auto work = [&]() {
    for (int64_t i = next.fetch_add(1); i < n; i = next.fetch_add(1)) {
      ok[i] = 0;
      if (offsets[i] < 0 || sizes[i] <= 0) continue;
      std::string why;
      ok[i] = JpegDecode(ptrs[i], lens[i], out + offsets[i], static_cast<size_t>(sizes[i]), &why) ? 1 : 0;
    }
  };
  threads = std::max(1, std::min<int>(threads, static_cast<int>(n)));
  std::vector<std::thread> pool;
  for (int t = 1; t < threads; ++t) pool.emplace_back(work);
  work();
  for (auto& t : pool) t.join();
}

}  // namespace smlimg
