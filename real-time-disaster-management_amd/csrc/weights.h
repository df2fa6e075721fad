// Host-side weight packing into one device blob.
#pragma once

#include <cmath>
#include <cstring>
#include <map>

#include "common.h"

namespace rtdm {

// Output-channel padding of packed GEMM weights (matches the tile widths of
// launch_conv: 16 / 32 / 64, then multiples of 128).
inline int cout_pad_for(int cout) {
  if (cout <= 16) return 16;
  if (cout <= 32) return 32;
  if (cout <= 64) return 64;
  return (int)round_up(cout, 128);
}

// Host staging of everything that goes to the device once at create time.
struct Blob {
  std::vector<uint8_t> host;
  size_t add(const void* p, size_t bytes) {
    const size_t off = (size_t)round_up((int64_t)host.size(), 256);
    host.resize(off + bytes);
    if (p) std::memcpy(host.data() + off, p, bytes);
    return off;
  }
  size_t add_f32(const std::vector<float>& v) { return add(v.data(), v.size() * sizeof(float)); }
};

// Packed conv weights + epilogue vectors, as offsets into a Blob.
struct PackedConv {
  int cout = 0, cin = 0, ks = 1, kpad = 0, cout_pad = 0;
  bool mfma = false;      // fp16 MFMA layout (else fp32 for the VALU kernel)
  size_t w_off = 0;       // [cout_pad][kpad]
  size_t b_off = SIZE_MAX, s_off = SIZE_MAX, t_off = SIZE_MAX;  // bias / post scale / post shift
  size_t stem_off = SIZE_MAX;  // MFMA stem copy (Cin=3, 3x3)
};

// Cin=3 3x3 stem weights for conv_stem3: fp16 [cout_pad16][64].  K index
// k = 8*G + j: G < 6 -> kh = G >> 1, kw = 2*(G & 1) + (j >> 2), c = j & 3 (zero
// when kw == 3 or c == 3); G = 6, 7 zero.  Matches the kernel's LDS image of
// 4-channel pixels read as 2-pixel x 4-channel groups.
inline size_t pack_stem(Blob& blob, const float* w, int cout, const double* oscale) {
  const int cp = (int)round_up(cout, 16);
  std::vector<_Float16> h((size_t)cp * 64, (_Float16)0.f);
  for (int o = 0; o < cout; ++o)
    for (int G = 0; G < 6; ++G)
      for (int j = 0; j < 8; ++j) {
        const int kh = G >> 1, kw = 2 * (G & 1) + (j >> 2), c = j & 3;
        if (kw >= 3 || c >= 3) continue;
        double v = w[(((size_t)o * 3 + c) * 3 + kh) * 3 + kw];
        if (oscale) v *= oscale[o];
        h[(size_t)o * 64 + 8 * G + j] = (_Float16)(float)v;
      }
  return blob.add(h.data(), h.size() * sizeof(_Float16));
}

// w: OIHW fp32 [cout][cin][ks][ks]; oscale: optional per-out-channel multiplier
// (folded BN).  K index = (kh*ks + kw)*cin + c so each tap is a contiguous NHWC
// channel slice.
inline PackedConv pack_conv(Blob& blob, const float* w, int cout, int cin, int ks, const double* oscale, bool mfma,
                            int cout_pad = 0) {
  PackedConv p;
  p.cout = cout;
  p.cin = cin;
  p.ks = ks;
  p.mfma = mfma;
  p.kpad = (int)round_up((int64_t)ks * ks * cin, 64);
  p.cout_pad = cout_pad > 0 ? cout_pad : cout_pad_for(cout);
  const size_t nel = (size_t)p.cout_pad * p.kpad;
  if (mfma) {
    std::vector<_Float16> h(nel, (_Float16)0.f);
    for (int o = 0; o < cout; ++o)
      for (int c = 0; c < cin; ++c)
        for (int kh = 0; kh < ks; ++kh)
          for (int kw = 0; kw < ks; ++kw) {
            double v = w[(((size_t)o * cin + c) * ks + kh) * ks + kw];
            if (oscale) v *= oscale[o];
            h[(size_t)o * p.kpad + (kh * ks + kw) * cin + c] = (_Float16)(float)v;
          }
    p.w_off = blob.add(h.data(), nel * sizeof(_Float16));
  } else {
    std::vector<float> f(nel, 0.f);
    for (int o = 0; o < cout; ++o)
      for (int c = 0; c < cin; ++c)
        for (int kh = 0; kh < ks; ++kh)
          for (int kw = 0; kw < ks; ++kw) {
            double v = w[(((size_t)o * cin + c) * ks + kh) * ks + kw];
            if (oscale) v *= oscale[o];
            f[(size_t)o * p.kpad + (kh * ks + kw) * cin + c] = (float)v;
          }
    p.w_off = blob.add_f32(f);
  }
  return p;
}

// Device-resident blob; pointers = base + offset.
struct DevBlob {
  DevBuf buf;
  void upload(const Blob& b) {
    buf.alloc(b.host.size());
    RTDM_HIP(hipMemcpy(buf.p, b.host.data(), b.host.size(), hipMemcpyHostToDevice));
  }
  template <class T>
  T* at(size_t off) const {
    return off == SIZE_MAX ? nullptr : reinterpret_cast<T*>(static_cast<char*>(buf.p) + off);
  }
};

}  // namespace rtdm
