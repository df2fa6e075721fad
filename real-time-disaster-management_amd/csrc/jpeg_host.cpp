// JPEG frame ingest, host half: marker parsing and the Huffman entropy decode of baseline
// (SOF0 / SOF1) 8-bit JPEGs into dequantisation-ready coefficient blocks.
//
// Replaces the decode inside cv2.imread (victim_localization/yolov3/utils/datasets.py:97,
// disaster_detection/aider-predict.py:57).  cv2 (and Pillow) decode with libjpeg-turbo's
// defaults; its pipeline is jdhuff.c (entropy decode, sequential by nature: every code's
// length depends on the previous one) -> jidctint.c (islow IDCT) -> jdsample.c (fancy
// upsampling) -> jdcolor.c (YCbCr -> RGB).  The split here follows the data: the bit-serial
// first stage stays on the host (this file), everything per block / per pixel runs on the
// device (jpeg.hip).  Restated from ITU-T T.81 (Annex C canonical Huffman codes, F.2.2
// decode procedure, Annex B marker syntax) and libjpeg's conventions where the standard
// leaves room: a marker or the end of data inside the entropy-coded segment reads as zero
// bits, the AC run index past 63 clamps to 63 (jpeg_natural_order's guard entries), the DC
// predictor is an int that the JCOEF store truncates.
#include <algorithm>
#include <cstring>
#include <vector>

#include "common.h"

namespace rtdm {
namespace {

// zig-zag index -> natural (row-major) index, plus libjpeg's 16 guard entries for corrupt runs
const int kNatural[64 + 16] = {
    0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,  12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13,
    6,  7,  14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51, 58, 59, 52, 45, 38, 31,
    39, 46, 53, 60, 61, 54, 47, 55, 62, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63};

constexpr int kLook = 9;  // lookahead bits of the fast Huffman table

struct Huff {
  bool ok = false;
  uint8_t vals[256] = {};
  int32_t maxcode[18] = {};  // largest code of each length (-1: none); [17] sentinel
  int32_t valoff[17] = {};   // vals index of a code = code + valoff[len]
  int16_t look[1 << kLook];  // (len << 8) | symbol for codes of <= kLook bits, else -1
};

void build_huff(Huff& h, const uint8_t* counts, const uint8_t* vals, int nvals) {
  std::memcpy(h.vals, vals, nvals);
  for (int i = 0; i < (1 << kLook); ++i) h.look[i] = -1;
  int code = 0, k = 0;
  for (int len = 1; len <= 16; ++len) {
    const int n = counts[len - 1];
    if (n) {
      h.valoff[len] = k - code;
      for (int i = 0; i < n; ++i, ++k, ++code) {
        if (len <= kLook) {
          const int base = code << (kLook - len);
          for (int j = 0; j < (1 << (kLook - len)); ++j) h.look[base + j] = (int16_t)((len << 8) | vals[k]);
        }
      }
      h.maxcode[len] = code - 1;
    } else {
      h.maxcode[len] = -1;
    }
    RTDM_REQUIRE(code <= (1 << len), RTDM_E_INVALID, "jpeg: bad Huffman table");
    code <<= 1;
  }
  h.maxcode[17] = 0x7fffffff;
  h.ok = true;
}

struct Comp {
  int id = 0, h = 1, v = 1, tq = 0, td = 0, ta = 0;
  int bw = 0, bh = 0;     // coefficient block grid (MCU-padded)
  int cbw = 0, cbh = 0;   // blocks covering the component's own samples (non-interleaved scans)
  int64_t off = 0;        // first block in the coefficient buffer
};

struct Jpeg {
  int w = 0, h = 0, nc = 0, hmax = 1, vmax = 1, mcux = 0, mcuy = 0;
  int precision = 8;
  bool sof = false, unsupported = false;
  Comp c[4];
  uint16_t q[4][64] = {};  // natural order
  bool qok[4] = {};
  Huff dc[4], ac[4];
  int ri = 0;
  int64_t nblocks = 0;
};

struct Reader {
  const uint8_t* p;
  const uint8_t* end;
  uint8_t u8() {
    RTDM_REQUIRE(p < end, RTDM_E_INVALID, "jpeg: truncated header");
    return *p++;
  }
  int u16() {
    const int a = u8();
    return (a << 8) | u8();
  }
};

// Bit reader over the entropy-coded segment: FF 00 is a data FF; any other FF xx is a
// marker, after which (and past the end of the data) the reader supplies zero bits.
struct Bits {
  const uint8_t* p;
  const uint8_t* end;
  uint64_t acc = 0;
  int n = 0;
  bool marker = false;
  void fill() {
    while (n <= 56) {
      uint32_t b = 0;
      if (!marker && p < end) {
        b = *p;
        if (b == 0xFF) {
          const uint32_t b2 = p + 1 < end ? p[1] : 0xD9;
          if (b2 == 0) {
            p += 2;
          } else {
            marker = true;
            b = 0;
          }
        } else {
          ++p;
        }
      }
      acc |= (uint64_t)b << (56 - n);
      n += 8;
    }
  }
  int get(int k) {
    if (k == 0) return 0;
    if (n < k) fill();
    const int v = (int)(acc >> (64 - k));
    acc <<= k;
    n -= k;
    return v;
  }
  int decode(const Huff& h) {
    if (n < 16) fill();
    const int e = h.look[acc >> (64 - kLook)];
    if (e >= 0) {
      const int len = e >> 8;
      acc <<= len;
      n -= len;
      return e & 255;
    }
    int len = kLook + 1;
    int code = (int)(acc >> (64 - len));
    while (len <= 16 && code > h.maxcode[len]) {
      ++len;
      code = (int)(acc >> (64 - len));
    }
    if (len > 16) {  // corrupt data: libjpeg warns and returns symbol 0
      acc <<= 16;
      n -= 16;
      return 0;
    }
    acc <<= len;
    n -= len;
    return h.vals[code + h.valoff[len]];
  }
  // restart marker (libjpeg process_restart): drop the bits left of the partial byte, then
  // step over the next RSTn (the reader stops at a marker, so normally it is right here)
  void restart() {
    acc = 0;
    n = 0;
    while (p + 1 < end && !(p[0] == 0xFF && p[1] >= 0xD0 && p[1] <= 0xD7)) ++p;
    if (p + 1 < end) p += 2;
    marker = false;
  }
};

inline int extend(int v, int s) { return v < (1 << (s - 1)) ? v + (int)((~0u) << s) + 1 : v; }

void parse_sof(Jpeg& j, Reader& r, int marker) {
  const int len = r.u16();
  (void)len;
  j.precision = r.u8();
  j.h = r.u16();
  j.w = r.u16();
  j.nc = r.u8();
  RTDM_REQUIRE(j.nc == 1 || j.nc == 3, RTDM_E_UNSUPPORTED, "jpeg: only 1- or 3-component images");
  RTDM_REQUIRE(j.w > 0 && j.h > 0, RTDM_E_UNSUPPORTED, "jpeg: zero size (DNL) not supported");
  for (int i = 0; i < j.nc; ++i) {
    j.c[i].id = r.u8();
    const int hv = r.u8();
    j.c[i].h = hv >> 4;
    j.c[i].v = hv & 15;
    j.c[i].tq = r.u8() & 3;
    RTDM_REQUIRE(j.c[i].h >= 1 && j.c[i].h <= 4 && j.c[i].v >= 1 && j.c[i].v <= 4, RTDM_E_INVALID,
                 "jpeg: bad sampling factor");
  }
  if (marker != 0xC0 && marker != 0xC1) j.unsupported = true;  // progressive / lossless / arithmetic
  if (j.precision != 8) j.unsupported = true;
  if (j.nc == 1) j.c[0].h = j.c[0].v = 1;  // a single-component image's MCU is one block
  j.hmax = j.vmax = 1;
  for (int i = 0; i < j.nc; ++i) {
    j.hmax = std::max(j.hmax, j.c[i].h);
    j.vmax = std::max(j.vmax, j.c[i].v);
  }
  j.mcux = (j.w + 8 * j.hmax - 1) / (8 * j.hmax);
  j.mcuy = (j.h + 8 * j.vmax - 1) / (8 * j.vmax);
  int64_t off = 0;
  for (int i = 0; i < j.nc; ++i) {
    Comp& c = j.c[i];
    c.bw = j.mcux * c.h;
    c.bh = j.mcuy * c.v;
    const int sw = (int)(((int64_t)j.w * c.h + j.hmax - 1) / j.hmax), sh = (int)(((int64_t)j.h * c.v + j.vmax - 1) / j.vmax);
    c.cbw = (sw + 7) / 8;
    c.cbh = (sh + 7) / 8;
    c.off = off;
    off += (int64_t)c.bw * c.bh;
  }
  j.nblocks = off;
  j.sof = true;
}

void parse_dqt(Jpeg& j, Reader& r) {
  const int len = r.u16();
  const uint8_t* stop = r.p + len - 2;
  while (r.p < stop) {
    const int pq = r.u8();
    const int t = pq & 3;
    for (int k = 0; k < 64; ++k) j.q[t][kNatural[k]] = (uint16_t)((pq >> 4) ? r.u16() : r.u8());
    j.qok[t] = true;
  }
}

void parse_dht(Jpeg& j, Reader& r) {
  const int len = r.u16();
  const uint8_t* stop = r.p + len - 2;
  while (r.p < stop) {
    const int tc = r.u8();
    uint8_t counts[16];
    int nv = 0;
    for (int i = 0; i < 16; ++i) nv += counts[i] = r.u8();
    RTDM_REQUIRE(nv <= 256, RTDM_E_INVALID, "jpeg: bad Huffman table");
    uint8_t vals[256];
    for (int i = 0; i < nv; ++i) vals[i] = r.u8();
    build_huff((tc >> 4) ? j.ac[tc & 3] : j.dc[tc & 3], counts, vals, nv);
  }
}

// One scan's entropy-coded segment (T.81 F.2.2, libjpeg jdhuff.c decode_mcu) into coef.
const uint8_t* decode_scan(Jpeg& j, const int* sc, int ns, const uint8_t* p, const uint8_t* end, int16_t* coef) {
  Bits b{p, end};
  int pred[4] = {0, 0, 0, 0};
  const bool inter = ns > 1;
  const int64_t mcus = inter ? (int64_t)j.mcux * j.mcuy : (int64_t)j.c[sc[0]].cbw * j.c[sc[0]].cbh;
  const int cols = inter ? j.mcux : j.c[sc[0]].cbw;
  for (int k = 0; k < ns; ++k)
    RTDM_REQUIRE(j.dc[j.c[sc[k]].td].ok && j.ac[j.c[sc[k]].ta].ok, RTDM_E_INVALID, "jpeg: missing Huffman table");
  auto block = [&](int ci, int by, int bx) {
    const Comp& c = j.c[ci];
    int16_t* blk = coef + (c.off + (int64_t)by * c.bw + bx) * 64;
    std::memset(blk, 0, 64 * sizeof(int16_t));
    const Huff& hd = j.dc[c.td];
    const Huff& ha = j.ac[c.ta];
    const int t = b.decode(hd);
    if (t) pred[ci] += extend(b.get(t), t);
    blk[0] = (int16_t)pred[ci];
    for (int k = 1; k < 64; ++k) {
      const int rs = b.decode(ha);
      const int r = rs >> 4, s = rs & 15;
      if (s) {
        k += r;
        blk[kNatural[k]] = (int16_t)extend(b.get(s), s);
      } else {
        if (r != 15) break;
        k += 15;
      }
    }
  };
  int todo = j.ri;
  for (int64_t m = 0; m < mcus; ++m) {
    if (j.ri) {
      if (todo == 0) {
        b.restart();
        for (int k = 0; k < 4; ++k) pred[k] = 0;
        todo = j.ri;
      }
      --todo;
    }
    const int my = (int)(m / cols), mx = (int)(m - (int64_t)my * cols);
    if (inter) {
      for (int k = 0; k < ns; ++k) {
        const Comp& c = j.c[sc[k]];
        for (int v = 0; v < c.v; ++v)
          for (int h = 0; h < c.h; ++h) block(sc[k], my * c.v + v, mx * c.h + h);
      }
    } else {
      block(sc[0], my, mx);
    }
  }
  // continue after the segment: the next marker that is not RSTn
  const uint8_t* q = b.p;
  while (q + 1 < end && !(q[0] == 0xFF && q[1] != 0 && !(q[1] >= 0xD0 && q[1] <= 0xD7))) ++q;
  return q;
}

// Walk the markers; with coef != nullptr decode every scan.  Returns the parsed header.
Jpeg walk(const uint8_t* data, int64_t len, int16_t* coef, int64_t nblocks) {
  RTDM_REQUIRE(data && len >= 4, RTDM_E_INVALID, "jpeg: no data");
  RTDM_REQUIRE(data[0] == 0xFF && data[1] == 0xD8, RTDM_E_INVALID, "jpeg: missing SOI");
  Jpeg j;
  Reader r{data + 2, data + len};
  bool scanned = false;
  while (r.p < r.end) {
    // next marker (fill bytes FF FF ... allowed)
    if (*r.p != 0xFF) {
      ++r.p;
      continue;
    }
    while (r.p < r.end && *r.p == 0xFF) ++r.p;
    if (r.p >= r.end) break;
    const int m = *r.p++;
    if (m == 0xD9) break;                      // EOI
    if (m == 0x01 || (m >= 0xD0 && m <= 0xD7)) continue;  // TEM / stray RSTn
    if (m >= 0xC0 && m <= 0xCF && m != 0xC4 && m != 0xC8 && m != 0xCC) {
      parse_sof(j, r, m);
      if (!coef) return j;  // geometry is all the caller asked for
      RTDM_REQUIRE(!j.unsupported, RTDM_E_UNSUPPORTED,
                   "jpeg: only baseline / extended sequential 8-bit Huffman JPEGs (SOF0 / SOF1) are decoded on the device");
      RTDM_REQUIRE(nblocks >= j.nblocks, RTDM_E_CAPACITY, "jpeg: coefficient buffer too small");
      std::memset(coef, 0, (size_t)j.nblocks * 64 * sizeof(int16_t));
    } else if (m == 0xC4) {
      parse_dht(j, r);
    } else if (m == 0xDB) {
      parse_dqt(j, r);
    } else if (m == 0xDD) {
      r.u16();
      j.ri = r.u16();
    } else if (m == 0xDA) {
      RTDM_REQUIRE(j.sof, RTDM_E_INVALID, "jpeg: SOS before SOF");
      r.u16();
      const int ns = r.u8();
      RTDM_REQUIRE(ns >= 1 && ns <= j.nc, RTDM_E_INVALID, "jpeg: bad scan");
      int sc[4];
      for (int k = 0; k < ns; ++k) {
        const int id = r.u8(), t = r.u8();
        int ci = -1;
        for (int i = 0; i < j.nc; ++i)
          if (j.c[i].id == id) ci = i;
        RTDM_REQUIRE(ci >= 0, RTDM_E_INVALID, "jpeg: scan names an unknown component");
        j.c[ci].td = t >> 4;
        j.c[ci].ta = t & 3;
        sc[k] = ci;
      }
      const int ss = r.u8(), se = r.u8(), a = r.u8();
      RTDM_REQUIRE(ss == 0 && se == 63 && a == 0, RTDM_E_UNSUPPORTED, "jpeg: not a sequential scan");
      r.p = decode_scan(j, sc, ns, r.p, r.end, coef);
      scanned = true;
    } else {  // APPn, COM, DNL, ...: skip
      const int l = r.u16();
      RTDM_REQUIRE(l >= 2 && r.p + l - 2 <= r.end, RTDM_E_INVALID, "jpeg: truncated marker segment");
      r.p += l - 2;
    }
  }
  RTDM_REQUIRE(j.sof, RTDM_E_INVALID, "jpeg: no frame header");
  RTDM_REQUIRE(scanned, RTDM_E_INVALID, "jpeg: no scan");
  return j;
}

void fill_info(const Jpeg& j, rtdm_jpeg_info* info) {
  std::memset(info, 0, sizeof(*info));
  info->width = j.w;
  info->height = j.h;
  info->ncomp = j.nc;
  for (int i = 0; i < j.nc; ++i) {
    info->h[i] = j.c[i].h;
    info->v[i] = j.c[i].v;
    info->bw[i] = j.c[i].bw;
    info->bh[i] = j.c[i].bh;
    info->coef_off[i] = j.c[i].off;
  }
  info->nblocks = j.nblocks;
  info->supported = j.unsupported ? 0 : 1;
}

}  // namespace
}  // namespace rtdm

using namespace rtdm;

extern "C" {

rtdm_status rtdm_jpeg_info_get(const uint8_t* data, int64_t len, rtdm_jpeg_info* info) {
  return guard([&] {
    RTDM_REQUIRE(info, RTDM_E_INVALID, "jpeg_info_get: NULL info");
    fill_info(walk(data, len, nullptr, 0), info);
  });
}

rtdm_status rtdm_jpeg_entropy_decode(const uint8_t* data, int64_t len, int16_t* coef, int64_t nblocks, uint16_t* qt,
                                     rtdm_jpeg_info* info) {
  return guard([&] {
    RTDM_REQUIRE(coef && qt, RTDM_E_INVALID, "jpeg_entropy_decode: NULL buffer");
    const Jpeg j = walk(data, len, coef, nblocks);
    for (int i = 0; i < j.nc; ++i) {
      RTDM_REQUIRE(j.qok[j.c[i].tq], RTDM_E_INVALID, "jpeg: missing quantisation table");
      std::memcpy(qt + 64 * i, j.q[j.c[i].tq], 64 * sizeof(uint16_t));
    }
    if (info) fill_info(j, info);
  });
}

}  // extern "C"
