// JPEG frame ingest, device half: dequantisation + islow IDCT per 8x8 block, then fancy
// upsampling + YCbCr -> RGB per pixel, on the coefficient blocks jpeg_host.cpp decoded on the host.
//
// Bit-exact with libjpeg-turbo's default decompression (what cv2.imread,
// victim_localization/yolov3/utils/datasets.py:97 / disaster_detection/aider-predict.py:57,
// and Pillow return): JDCT_ISLOW (jidctint.c: CONST_BITS 13, PASS1_BITS 2, the
// post-IDCT range-limit table indexed & 1023), do_fancy_upsampling (jdsample.c
// h2v2_fancy_upsample / h2v1_fancy_upsample, triangle filters with the 8 / 7 and 1 / 2
// rounding biases, the first / last column special cases and edge-replicated context rows;
// plain replication when the downsampled width is <= 2), and jdcolor.c ycc_rgb_convert
// (16-bit fixed point, FIX(x) = x * 65536 + 0.5).  Restated from the published algorithms;
// the oracle (oracle/jpeg.py) restates them again in numpy and both are pinned against
// Pillow's decode of the reference's bundled JPEGs.
//
// Work: per block 2 x 8 one-dimensional 8-point IDCTs in int32 (the SIMD islow's arithmetic
// width; the C code's JLONG gives the same values for any coefficient a baseline stream can
// carry); the kernels are bandwidth-trivial (1.5 bytes per output pixel in, 3 out).
#include "common.h"

namespace rtdm {

struct JpegPlanes {
  int ncomp, w, h;
  int bw[3], bh[3];   // block grids
  int64_t off[3];     // first block of each component in the coefficient buffer
  int64_t poff[3];    // byte offset of each component's sample plane (pitch bw * 8)
  int h_samp[3], v_samp[3], hmax, vmax;
};

namespace {

constexpr int kCB = 13, kP1 = 2;  // CONST_BITS, PASS1_BITS
constexpr int F0_298 = 2446, F0_390 = 3196, F0_541 = 4433, F0_765 = 6270, F0_899 = 7373, F1_175 = 9633,
              F1_501 = 12299, F1_847 = 15137, F1_961 = 16069, F2_053 = 16819, F2_562 = 20995, F3_072 = 25172;

__device__ __forceinline__ int descale(int x, int n) { return (x + (1 << (n - 1))) >> n; }

// the post-IDCT range limit: table[x & 1023] of jdmaster.c prepare_range_limit_table
__device__ __forceinline__ uint8_t idct_limit(int x) {
  const int v = x & 1023;
  return (uint8_t)(v < 128 ? v + 128 : v < 512 ? 255 : v < 896 ? 0 : v - 896);
}

// one 8-point islow IDCT (even part from z0 z2 z4 z6, odd from z1 z3 z5 z7): the eight
// outputs before descaling, in output order 0..7
__device__ __forceinline__ void idct8(int z0, int z1, int z2, int z3, int z4, int z5, int z6, int z7, int (&o)[8],
                                      bool pass1) {
  // even part
  int z_1 = (z2 + z6) * F0_541;
  const int tmp2 = z_1 + z6 * (-F1_847);
  const int tmp3 = z_1 + z2 * F0_765;
  const int t0 = (z0 + z4) * (1 << kCB);
  const int t1 = (z0 - z4) * (1 << kCB);
  const int tmp10 = t0 + tmp3, tmp13 = t0 - tmp3, tmp11 = t1 + tmp2, tmp12 = t1 - tmp2;
  // odd part: tmp0..3 = z7, z5, z3, z1
  int a0 = z7, a1 = z5, a2 = z3, a3 = z1;
  int q1 = a0 + a3, q2 = a1 + a2, q3 = a0 + a2, q4 = a1 + a3;
  const int z5_ = (q3 + q4) * F1_175;
  a0 *= F0_298;
  a1 *= F2_053;
  a2 *= F3_072;
  a3 *= F1_501;
  q1 *= -F0_899;
  q2 *= -F2_562;
  q3 *= -F1_961;
  q4 *= -F0_390;
  q3 += z5_;
  q4 += z5_;
  a0 += q1 + q3;
  a1 += q2 + q4;
  a2 += q2 + q3;
  a3 += q1 + q4;
  const int n = pass1 ? kCB - kP1 : kCB + kP1 + 3;
  o[0] = descale(tmp10 + a3, n);
  o[7] = descale(tmp10 - a3, n);
  o[1] = descale(tmp11 + a2, n);
  o[6] = descale(tmp11 - a2, n);
  o[2] = descale(tmp12 + a1, n);
  o[5] = descale(tmp12 - a1, n);
  o[3] = descale(tmp13 + a0, n);
  o[4] = descale(tmp13 - a0, n);
}

// one thread per 8x8 block: DEQUANTIZE -> columns (pass 1) -> rows (pass 2) -> range limit
__global__ __launch_bounds__(256) void jpeg_idct_kernel(const int16_t* __restrict__ coef,
                                                        const uint16_t* __restrict__ qt, JpegPlanes p,
                                                        int64_t nblocks, uint8_t* __restrict__ planes) {
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= nblocks) return;
  const int c = (p.ncomp > 2 && b >= p.off[2]) ? 2 : (p.ncomp > 1 && b >= p.off[1]) ? 1 : 0;
  const int64_t lb = b - p.off[c];
  const int by = (int)(lb / p.bw[c]), bx = (int)(lb - (int64_t)by * p.bw[c]);
  int x[64];
  {
    const int4* src = (const int4*)(coef + b * 64);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int4 v = src[k];
      const int w4[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        x[8 * k + 2 * e] = (int)(int16_t)(w4[e] & 0xffff);
        x[8 * k + 2 * e + 1] = (int)(int16_t)((uint32_t)w4[e] >> 16);
      }
    }
  }
  const uint16_t* q = qt + 64 * c;
#pragma unroll
  for (int k = 0; k < 64; ++k) x[k] *= (int)q[k];
  int ws[64];
#pragma unroll
  for (int col = 0; col < 8; ++col) {
    int o[8];
    idct8(x[col], x[8 + col], x[16 + col], x[24 + col], x[32 + col], x[40 + col], x[48 + col], x[56 + col], o, true);
#pragma unroll
    for (int r = 0; r < 8; ++r) ws[8 * r + col] = o[r];
  }
  const int pitch = p.bw[c] * 8;
  uint8_t* dst = planes + p.poff[c] + ((int64_t)by * 8) * pitch + bx * 8;
#pragma unroll
  for (int r = 0; r < 8; ++r) {
    int o[8];
    const int* w = ws + 8 * r;
    idct8(w[0], w[1], w[2], w[3], w[4], w[5], w[6], w[7], o, false);
    uint32_t lo = 0, hi = 0;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      lo |= (uint32_t)idct_limit(o[e]) << (8 * e);
      hi |= (uint32_t)idct_limit(o[4 + e]) << (8 * e);
    }
    *(uint2*)(dst + (int64_t)r * pitch) = make_uint2(lo, hi);
  }
}

// fancy-upsampled chroma sample (x, y) of plane pl (downsampled size cw x ch, pitch)
template <int HF, int VF>
__device__ __forceinline__ int chroma(const uint8_t* __restrict__ pl, int pitch, int cw, int ch, int x, int y) {
  if constexpr (HF == 1 && VF == 1) {
    return pl[(int64_t)y * pitch + x];
  } else if constexpr (VF == 1) {  // h2v1_fancy_upsample
    const uint8_t* row = pl + (int64_t)y * pitch;
    const int cx = x >> 1;
    if (cw <= 2) return row[cx];  // h2v1_upsample (box) for tiny widths
    const int in = row[cx];
    if ((x & 1) == 0) return cx == 0 ? in : (in * 3 + row[cx - 1] + 1) >> 2;
    return cx == cw - 1 ? in : (in * 3 + row[cx + 1] + 2) >> 2;
  } else {  // h2v2_fancy_upsample
    const int cy = y >> 1, cx = x >> 1;
    if (cw <= 2) return pl[(int64_t)cy * pitch + cx];  // h2v2_upsample (box)
    const int ny = (y & 1) ? (cy + 1 < ch ? cy + 1 : ch - 1) : (cy > 0 ? cy - 1 : 0);
    const uint8_t* r0 = pl + (int64_t)cy * pitch;
    const uint8_t* r1 = pl + (int64_t)ny * pitch;
    const int th = r0[cx] * 3 + r1[cx];
    if ((x & 1) == 0) return cx == 0 ? (th * 4 + 8) >> 4 : (th * 3 + (r0[cx - 1] * 3 + r1[cx - 1]) + 8) >> 4;
    return cx == cw - 1 ? (th * 4 + 7) >> 4 : (th * 3 + (r0[cx + 1] * 3 + r1[cx + 1]) + 7) >> 4;
  }
}

__device__ __forceinline__ uint8_t clamp255(int v) { return (uint8_t)(v < 0 ? 0 : v > 255 ? 255 : v); }

// one thread per output pixel: Y + upsampled Cb / Cr -> RGB (jdcolor.c ycc_rgb_convert)
template <int HF, int VF>
__global__ __launch_bounds__(256) void jpeg_color_kernel(const uint8_t* __restrict__ planes, JpegPlanes p, int bgr,
                                                         uint8_t* __restrict__ rgb, int64_t pitch_out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)p.w * p.h) return;
  const int y = (int)(i / p.w), x = (int)(i - (int64_t)y * p.w);
  const int py = p.bw[0] * 8;
  const int yv = planes[p.poff[0] + (int64_t)y * py + x];
  uint8_t* o = rgb + (int64_t)y * pitch_out + 3 * x;
  if (p.ncomp == 1) {  // grayscale: the three channels of cv2.imread's BGR image
    o[0] = o[1] = o[2] = (uint8_t)yv;
    return;
  }
  const int cw = (p.w * p.h_samp[1] + p.hmax - 1) / p.hmax, ch = (p.h * p.v_samp[1] + p.vmax - 1) / p.vmax;
  const int pc = p.bw[1] * 8;
  const int cb = chroma<HF, VF>(planes + p.poff[1], pc, cw, ch, x, y) - 128;
  const int cr = chroma<HF, VF>(planes + p.poff[2], p.bw[2] * 8, cw, ch, x, y) - 128;
  const int r = yv + ((91881 * cr + 32768) >> 16);
  const int g = yv + ((-22554 * cb + 32768 - 46802 * cr) >> 16);
  const int bb = yv + ((116130 * cb + 32768) >> 16);
  o[bgr ? 2 : 0] = clamp255(r);
  o[1] = clamp255(g);
  o[bgr ? 0 : 2] = clamp255(bb);
}

JpegPlanes planes_of(const rtdm_jpeg_info& in, int64_t* bytes) {
  JpegPlanes p{};
  p.ncomp = in.ncomp;
  p.w = in.width;
  p.h = in.height;
  p.hmax = p.vmax = 1;
  int64_t o = 0;
  for (int c = 0; c < in.ncomp; ++c) {
    p.bw[c] = in.bw[c];
    p.bh[c] = in.bh[c];
    p.off[c] = in.coef_off[c];
    p.h_samp[c] = in.h[c];
    p.v_samp[c] = in.v[c];
    p.hmax = std::max(p.hmax, in.h[c]);
    p.vmax = std::max(p.vmax, in.v[c]);
    p.poff[c] = o;
    o += (int64_t)in.bw[c] * 8 * in.bh[c] * 8;
  }
  if (bytes) *bytes = o;
  return p;
}

}  // namespace
}  // namespace rtdm

using namespace rtdm;

extern "C" {

int64_t rtdm_jpeg_workspace_bytes(const rtdm_jpeg_info* info) {
  if (!info) return 0;
  int64_t b = 0;
  planes_of(*info, &b);
  return b;
}

rtdm_status rtdm_jpeg_reconstruct(const int16_t* coef, const uint16_t* qt, const rtdm_jpeg_info* info, uint8_t* planes,
                                  int64_t planes_bytes, uint8_t* rgb, int64_t pitch, int bgr, void* stream) {
  return guard([&] {
    RTDM_REQUIRE(coef && qt && info && planes && rgb, RTDM_E_INVALID, "jpeg_reconstruct: NULL pointer");
    RTDM_REQUIRE(info->supported, RTDM_E_UNSUPPORTED, "jpeg_reconstruct: unsupported JPEG");
    RTDM_REQUIRE(info->ncomp == 1 || info->ncomp == 3, RTDM_E_UNSUPPORTED, "jpeg_reconstruct: 1 or 3 components");
    RTDM_REQUIRE(info->width > 0 && info->height > 0 && pitch >= 3ll * info->width, RTDM_E_INVALID,
                 "jpeg_reconstruct: bad geometry");
    int64_t need = 0;
    const JpegPlanes p = planes_of(*info, &need);
    RTDM_REQUIRE(planes_bytes >= need, RTDM_E_CAPACITY, "jpeg_reconstruct: workspace too small");
    for (int c = 0; c < info->ncomp; ++c)
      RTDM_REQUIRE(info->bw[c] > 0 && info->bh[c] > 0 && info->bw[c] * 8 >= (info->width * info->h[c] + p.hmax - 1) / p.hmax &&
                       info->bh[c] * 8 >= (info->height * info->v[c] + p.vmax - 1) / p.vmax,
                   RTDM_E_INVALID, "jpeg_reconstruct: block grid smaller than the image");
    int hf = 1, vf = 1;
    if (info->ncomp == 3) {
      RTDM_REQUIRE(info->h[1] == 1 && info->v[1] == 1 && info->h[2] == 1 && info->v[2] == 1, RTDM_E_UNSUPPORTED,
                   "jpeg_reconstruct: chroma sampling factors must be 1");
      hf = info->h[0];
      vf = info->v[0];
      RTDM_REQUIRE((hf == 1 && vf == 1) || (hf == 2 && vf == 1) || (hf == 2 && vf == 2), RTDM_E_UNSUPPORTED,
                   "jpeg_reconstruct: only 4:4:4, 4:2:2 (h2v1) and 4:2:0 (h2v2) sampling");
    }
    hipStream_t s = (hipStream_t)stream;
    const int64_t nb = info->nblocks;
    RTDM_REQUIRE(nb > 0 && nb < (1ll << 31), RTDM_E_INVALID, "jpeg_reconstruct: bad block count");
    hipLaunchKernelGGL(jpeg_idct_kernel, dim3((unsigned)((nb + 255) / 256)), dim3(256), 0, s, coef, qt, p, nb, planes);
    RTDM_HIP(hipGetLastError());
    const int64_t px = (int64_t)info->width * info->height;
    const dim3 g((unsigned)((px + 255) / 256));
    if (hf == 2 && vf == 2)
      hipLaunchKernelGGL((jpeg_color_kernel<2, 2>), g, dim3(256), 0, s, planes, p, bgr, rgb, pitch);
    else if (hf == 2)
      hipLaunchKernelGGL((jpeg_color_kernel<2, 1>), g, dim3(256), 0, s, planes, p, bgr, rgb, pitch);
    else
      hipLaunchKernelGGL((jpeg_color_kernel<1, 1>), g, dim3(256), 0, s, planes, p, bgr, rgb, pitch);
    RTDM_HIP(hipGetLastError());
  });
}

}  // extern "C"
