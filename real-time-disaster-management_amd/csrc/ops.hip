// Non-GEMM kernels of the hot path (gfx950): ACFF dilated depthwise branches,
// max pooling, upsample / route copies, the classifier tail, the CLI
// pre-processing (Pillow 8-bit antialiased bilinear resize + crop + normalize),
// the stand-alone YOLO decode, and per-image greedy NMS.
#include "common.h"

#include <cmath>

namespace rtdm {

template <typename T>
__device__ __forceinline__ float ldf(const T* p) {
  return (float)(*p);
}

// ------------------------------------------------------------------ ACFF dw --
// The three depthwise branches of ACFF (acff.py:25-30): 3x3 dilation 1/2/3,
// padding 0/1/2, +bias each, concatenated along channels (acff.py:46) into an
// NHWC [n, h-2, w-2, 3c] buffer: channel b*c + ch holds branch b.  All three
// windows are centred on input pixel (oy+1, ox+1) with radius 1/2/3; only the
// dilated branches ever read zero padding.  Only the top-left lim_h x lim_w
// outputs are produced (the rest is dropped by the following floor maxpool).
template <typename T>
__global__ __launch_bounds__(256) void dw3_acff_kernel(const T* __restrict__ in, int in_cs, int in_co, int n, int h,
                                                       int w, int c, int lim_h, int lim_w,
                                                       const float* __restrict__ wts, const float* __restrict__ bias,
                                                       T* __restrict__ out) {
  const int oh = h - 2, ow = w - 2;
  const int64_t total = (int64_t)n * lim_h * lim_w * c;
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const int ch = (int)(idx % c);
    int64_t p = idx / c;
    const int ox = (int)(p % lim_w);
    p /= lim_w;
    const int oy = (int)(p % lim_h);
    const int b = (int)(p / lim_h);
    const T* src = in + (size_t)b * h * w * in_cs + in_co + ch;
    T* dst = out + (((size_t)b * oh + oy) * ow + ox) * (3 * c) + ch;
#pragma unroll
    for (int br = 0; br < 3; ++br) {
      const int d = br + 1;
      const float* wk = wts + ((size_t)br * c + ch) * 9;
      float acc = 0.f;
#pragma unroll
      for (int kh = 0; kh < 3; ++kh) {
        const int iy = oy + 1 + (kh - 1) * d;
        if ((unsigned)iy >= (unsigned)h) continue;
#pragma unroll
        for (int kw = 0; kw < 3; ++kw) {
          const int ix = ox + 1 + (kw - 1) * d;
          if ((unsigned)ix >= (unsigned)w) continue;
          acc = fmaf(wk[kh * 3 + kw], ldf(src + ((size_t)iy * w + ix) * in_cs), acc);
        }
      }
      dst[br * c] = (T)(acc + bias[br * c + ch]);
    }
  }
}

static inline int grid_for(int64_t total, int block) {
  int64_t g = (total + block - 1) / block;
  if (g > 2048 * 4) g = 2048 * 4;
  if (g < 1) g = 1;
  return (int)g;
}

// Vector form: one thread per (output pixel, 8 fp16 / 4 fp32 channels): 27
// 16-byte loads (3 branches x 9 taps) instead of 27 scalar loads per channel.
template <typename T, int VEC>
__global__ __launch_bounds__(256) void dw3_acff_vec_kernel(const T* __restrict__ in, int in_cs, int in_co, int n,
                                                           int h, int w, int c, int lim_h, int lim_w,
                                                           const float* __restrict__ wts,
                                                           const float* __restrict__ bias, T* __restrict__ out) {
  typedef T tv __attribute__((ext_vector_type(VEC)));
  const int oh = h - 2, ow = w - 2;
  const int cg = c / VEC;
  const int64_t total = (int64_t)n * lim_h * lim_w * cg;
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const int g = (int)(idx % cg);
    int64_t p = idx / cg;
    const int ox = (int)(p % lim_w);
    p /= lim_w;
    const int oy = (int)(p % lim_h);
    const int b = (int)(p / lim_h);
    const int ch0 = g * VEC;
    const T* src = in + (size_t)b * h * w * in_cs + in_co + ch0;
    T* dst = out + (((size_t)b * oh + oy) * ow + ox) * (3 * c) + ch0;
#pragma unroll
    for (int br = 0; br < 3; ++br) {
      const int d = br + 1;
      float acc[VEC];
#pragma unroll
      for (int j = 0; j < VEC; ++j) acc[j] = bias[br * c + ch0 + j];
#pragma unroll
      for (int kh = 0; kh < 3; ++kh) {
        const int iy = oy + 1 + (kh - 1) * d;
        if ((unsigned)iy >= (unsigned)h) continue;
#pragma unroll
        for (int kw = 0; kw < 3; ++kw) {
          const int ix = ox + 1 + (kw - 1) * d;
          if ((unsigned)ix >= (unsigned)w) continue;
          const tv x = *(const tv*)(src + ((size_t)iy * w + ix) * in_cs);
#pragma unroll
          for (int j = 0; j < VEC; ++j)
            acc[j] = fmaf(wts[((size_t)br * c + ch0 + j) * 9 + kh * 3 + kw], (float)x[j], acc[j]);
        }
      }
      tv o;
#pragma unroll
      for (int j = 0; j < VEC; ++j) o[j] = (T)acc[j];
      *(tv*)(dst + br * c) = o;
    }
  }
}

void launch_dw3_acff(const void* in, int in_cs, int in_co, int n, int h, int w, int c, int lim_h, int lim_w,
                     const float* wts, const float* bias, void* out, int dtype, hipStream_t s) {
  const int64_t total = (int64_t)n * lim_h * lim_w * c;
  if (total <= 0) return;
  const int vec = dtype == RTDM_F16 ? 8 : 4;
  if (c % vec == 0 && in_cs % vec == 0 && in_co % vec == 0) {
    const int gv = grid_for(total / vec, 256);
    if (dtype == RTDM_F16)
      hipLaunchKernelGGL((dw3_acff_vec_kernel<_Float16, 8>), dim3(gv), dim3(256), 0, s, (const _Float16*)in, in_cs,
                         in_co, n, h, w, c, lim_h, lim_w, wts, bias, (_Float16*)out);
    else
      hipLaunchKernelGGL((dw3_acff_vec_kernel<float, 4>), dim3(gv), dim3(256), 0, s, (const float*)in, in_cs, in_co,
                         n, h, w, c, lim_h, lim_w, wts, bias, (float*)out);
    RTDM_HIP(hipGetLastError());
    return;
  }
  const int g = grid_for(total, 256);
  if (dtype == RTDM_F16)
    hipLaunchKernelGGL(dw3_acff_kernel<_Float16>, dim3(g), dim3(256), 0, s, (const _Float16*)in, in_cs, in_co, n, h,
                       w, c, lim_h, lim_w, wts, bias, (_Float16*)out);
  else
    hipLaunchKernelGGL(dw3_acff_kernel<float>, dim3(g), dim3(256), 0, s, (const float*)in, in_cs, in_co, n, h, w, c,
                       lim_h, lim_w, wts, bias, (float*)out);
  RTDM_HIP(hipGetLastError());
}

// YOLO-ACFF depthwise stage, additive (models.py:296-302: conv1(x) + conv2(x) + conv3(x)):
// the three dilated 3x3 depthwise branches d1p0 / d2p1 / d3p2 of channel c, all centred
// on input (oy+1, ox+1), summed with their biases in fp32 and stored ONCE as a C-channel
// map (rounded once in the fp16 path), which the 1x1 fusion conv then reads with its
// original [F][C] weights (the classifier's ACFF, acff.py:46, concatenates instead:
// dw3_acff_*kernel above).  The 27 tap weights [27][C] and the summed bias [C] sit in
// LDS for the whole grid-stride loop; a thread owns VEC channels of one pixel (16-byte
// loads of the NHWC input; the 27 shifted reads of neighbouring pixels hit L1/L2).
template <typename T, int VEC>
__global__ __launch_bounds__(256) void dw3_sum_kernel(const T* __restrict__ in, int in_cs, int in_co, int n, int h,
                                                      int w, int c, const float* __restrict__ wts,
                                                      const float* __restrict__ bsum, T* __restrict__ out) {
  typedef T tv __attribute__((ext_vector_type(VEC)));
  typedef float fv __attribute__((ext_vector_type(VEC)));
  extern __shared__ float s_dw[];  // [27][c] taps (branch-major), then [c] bias sums
  for (int i = threadIdx.x; i < 28 * c; i += blockDim.x) s_dw[i] = i < 27 * c ? wts[i] : bsum[i - 27 * c];
  __syncthreads();
  const int oh = h - 2, ow = w - 2;
  const int cg = c / VEC;
  const int64_t total = (int64_t)n * oh * ow * cg;
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const int g = (int)(idx % cg);
    int64_t p = idx / cg;
    const int ox = (int)(p % ow);
    p /= ow;
    const int oy = (int)(p % oh);
    const int b = (int)(p / oh);
    const int ch0 = g * VEC;
    const T* src = in + (size_t)b * h * w * in_cs + in_co + ch0;
    fv acc;
#pragma unroll
    for (int j = 0; j < VEC; ++j) acc[j] = s_dw[27 * c + ch0 + j];
#pragma unroll
    for (int br = 0; br < 3; ++br) {
      const int d = br + 1;
#pragma unroll
      for (int kh = 0; kh < 3; ++kh) {
        const int iy = oy + 1 + (kh - 1) * d;
        if ((unsigned)iy >= (unsigned)h) continue;
#pragma unroll
        for (int kw = 0; kw < 3; ++kw) {
          const int ix = ox + 1 + (kw - 1) * d;
          if ((unsigned)ix >= (unsigned)w) continue;
          const tv x = *(const tv*)(src + ((size_t)iy * w + ix) * in_cs);
          const float* wp = s_dw + (br * 9 + kh * 3 + kw) * c + ch0;
#pragma unroll
          for (int j = 0; j < VEC; ++j) acc[j] = fmaf(wp[j], (float)x[j], acc[j]);
        }
      }
    }
    tv o;
#pragma unroll
    for (int j = 0; j < VEC; ++j) o[j] = (T)acc[j];
    *(tv*)(out + (((size_t)b * oh + oy) * ow + ox) * c + ch0) = o;
  }
}

// LDS-tiled fp16 form of dw3_sum_kernel for C % 64 == 0: a block stages an 8 x 32 output
// tile's input window (14 x 38 pixels: radius 3 around the tap centre; row stride 39 so
// vertically adjacent pixels fall in opposite LDS bank halves) of one 64-channel slice
// into LDS once (70 KB, zero outside the image = the branches' zero padding).  Each thread
// owns 8 neighbouring output pixels of one row x 8 channels and walks, per (branch, kernel
// row), the 8 + 2d input pixels that row segment reads: each is read from LDS and
// converted to fp32 ONCE and feeds its up to 3 taps (kw) in registers (the per-tap form
// converted every operand for every tap: 1.5 VALU per MAC, here ~1).  Same sum order per
// output as dw3_sum_kernel (bias, branch, kh, kw): bit-identical.
constexpr int kDwTH = 8, kDwTW = 32, kDwCS = 64, kDwIWS = kDwTW + 7;
template <int D>
__device__ __forceinline__ void dw3_row(const uint4* __restrict__ s_row, const float* __restrict__ wp,
                                        float (&acc)[8][8]) {
  // s_row: this thread's channel group at the segment's first input pixel (x0 + 3 - D)
  float w[3][8];
#pragma unroll
  for (int kw = 0; kw < 3; ++kw)
#pragma unroll
    for (int j = 0; j < 8; ++j) w[kw][j] = wp[kw * kDwCS + j];
#pragma unroll
  for (int i = 0; i < 8 + 2 * D; ++i) {
    const uint4 raw = s_row[i * (kDwCS / 8)];
    const uint32_t u[4] = {raw.x, raw.y, raw.z, raw.w};
    float x[8];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      x[2 * j] = (float)__builtin_bit_cast(_Float16, (uint16_t)(u[j] & 0xffffu));
      x[2 * j + 1] = (float)__builtin_bit_cast(_Float16, (uint16_t)(u[j] >> 16));
    }
#pragma unroll
    for (int kw = 0; kw < 3; ++kw) {
      const int p = i - kw * D;  // output pixel this input pixel feeds through tap kw
      if (p >= 0 && p < 8) {
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[p][j] = fmaf(w[kw][j], x[j], acc[p][j]);
      }
    }
  }
}

__global__ __launch_bounds__(256, 2) void dw3_sum_tile_kernel(const _Float16* __restrict__ in, int in_cs, int in_co,
                                                           int n, int h, int w, int c, const float* __restrict__ wts,
                                                           const float* __restrict__ bsum,
                                                           _Float16* __restrict__ out) {
  typedef _Float16 h8t __attribute__((ext_vector_type(8)));
  constexpr int IH = kDwTH + 6, IW = kDwTW + 6, G = kDwCS / 8;
  __shared__ uint4 s_in[(IH * kDwIWS * G + 63) / 64 * 64];  // whole 64-vector DMA rows
  __shared__ float s_w[28 * kDwCS];
  const int oh = h - 2, ow = w - 2;
  const int tx = (ow + kDwTW - 1) / kDwTW, ty = (oh + kDwTH - 1) / kDwTH, tc = c / kDwCS;
  int bid = blockIdx.x;
  const int ci = bid % tc;
  bid /= tc;
  const int xi = bid % tx;
  bid /= tx;
  const int yi = bid % ty;
  const int b = bid / ty;
  const int c0 = ci * kDwCS, oy0 = yi * kDwTH, ox0 = xi * kDwTW;
  for (int i = threadIdx.x; i < 28 * kDwCS; i += 256) {
    const int t = i / kDwCS, j = i - t * kDwCS;
    s_w[i] = t < 27 ? wts[t * c + c0 + j] : bsum[c0 + j];
  }
  // input window -> LDS by LDS-DMA (buffer_load ... lds): every 16-byte vector of the
  // window in flight at once (a register-staged loop waited on each load in turn); a lane
  // whose pixel lies outside the image (or in the stride's pad column) loads from an
  // out-of-range offset, which returns zeros
  {
    typedef __attribute__((address_space(3))) void* lds_p;
    const _Float16* src = in + (size_t)b * h * w * in_cs + in_co + c0;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)src, 0, (int)((((int64_t)h * w - 1) * in_cs + kDwCS) * 2), 0x00020000);
    constexpr int NV = IH * kDwIWS * G;  // 16-byte vectors of the LDS image
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
    for (int k = wid; k * 64 < NV; k += 4) {
      const int e = k * 64 + lane;
      const int g = e & 7, px = e >> 3;
      const int ry = px / kDwIWS, rx = px - ry * kDwIWS;
      const int gy = oy0 - 2 + ry, gx = ox0 - 2 + rx;
      const bool ok = e < NV && rx < IW && (unsigned)gy < (unsigned)h && (unsigned)gx < (unsigned)w;
      const int vo = ok ? ((gy * w + gx) * in_cs + g * 8) * 2 : (int)0x80000000;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_p)(s_in + k * 64), 16, vo, 0, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  // thread -> (channel group g, output row y, 8-pixel segment): lanes 8 apart take
  // adjacent rows (opposite bank halves), 4 segments per row
  const int g = threadIdx.x & 7, q = threadIdx.x >> 3;
  const int y = q & 7, x0 = (q >> 3) * 8;
  float acc[8][8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float bj = s_w[27 * kDwCS + g * 8 + j];
#pragma unroll
    for (int p = 0; p < 8; ++p) acc[p][j] = bj;
  }
  // (branch, kernel row) in the reference's order; kw inside dw3_row
#pragma unroll 1
  for (int kh = 0; kh < 3; ++kh)
    dw3_row<1>(s_in + ((y + 3 + (kh - 1)) * kDwIWS + x0 + 2) * G + g, s_w + (0 * 9 + kh * 3) * kDwCS + g * 8, acc);
#pragma unroll 1
  for (int kh = 0; kh < 3; ++kh)
    dw3_row<2>(s_in + ((y + 3 + (kh - 1) * 2) * kDwIWS + x0 + 1) * G + g, s_w + (1 * 9 + kh * 3) * kDwCS + g * 8, acc);
#pragma unroll 1
  for (int kh = 0; kh < 3; ++kh)
    dw3_row<3>(s_in + ((y + 3 + (kh - 1) * 3) * kDwIWS + x0) * G + g, s_w + (2 * 9 + kh * 3) * kDwCS + g * 8, acc);
  const int oy = oy0 + y;
  if (oy >= oh) return;
#pragma unroll
  for (int p = 0; p < 8; ++p) {
    const int ox = ox0 + x0 + p;
    if (ox >= ow) break;
    h8t o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = (_Float16)acc[p][j];
    *(h8t*)(out + (((size_t)b * oh + oy) * ow + ox) * c + c0 + g * 8) = o;
  }
}

bool dw3_sum_tile_ok(int c, int in_cs, int in_co, int dtype) {
  return tune().dw3_tile && dtype == RTDM_F16 && c % kDwCS == 0 && in_cs % 8 == 0 && in_co % 8 == 0;
}

bool dw3_sum_vec_ok(int c, int in_cs, int in_co, int dtype) {
  const int vec = dtype == RTDM_F16 ? 8 : 4;
  return c % vec == 0 && in_cs % vec == 0 && in_co % vec == 0;
}

void launch_dw3_sum(const void* in, int in_cs, int in_co, int n, int h, int w, int c, const float* wts,
                    const float* bsum, void* out, int dtype, hipStream_t s) {
  const int64_t total = (int64_t)n * (h - 2) * (w - 2) * c;
  if (total <= 0) return;
  const size_t lds = (size_t)28 * c * sizeof(float);
  RTDM_REQUIRE(lds <= 160 * 1024, RTDM_E_UNSUPPORTED, "acff: too many channels for the LDS tap table");
  if (dw3_sum_tile_ok(c, in_cs, in_co, dtype)) {
    const int64_t blocks = (int64_t)n * ((h - 2 + kDwTH - 1) / kDwTH) * ((w - 2 + kDwTW - 1) / kDwTW) * (c / kDwCS);
    RTDM_REQUIRE(blocks < (1ll << 31), RTDM_E_CAPACITY, "acff: grid too large");
    hipLaunchKernelGGL(dw3_sum_tile_kernel, dim3((unsigned)blocks), dim3(256), 0, s, (const _Float16*)in, in_cs, in_co,
                       n, h, w, c, wts, bsum, (_Float16*)out);
    RTDM_HIP(hipGetLastError());
    return;
  }
  const bool vec = dw3_sum_vec_ok(c, in_cs, in_co, dtype);
  const int g = grid_for(vec ? total / (dtype == RTDM_F16 ? 8 : 4) : total, 256);
  if (dtype == RTDM_F16) {
    if (vec)
      hipLaunchKernelGGL((dw3_sum_kernel<_Float16, 8>), dim3(g), dim3(256), lds, s, (const _Float16*)in, in_cs, in_co,
                         n, h, w, c, wts, bsum, (_Float16*)out);
    else
      hipLaunchKernelGGL((dw3_sum_kernel<_Float16, 1>), dim3(g), dim3(256), lds, s, (const _Float16*)in, in_cs, in_co,
                         n, h, w, c, wts, bsum, (_Float16*)out);
  } else {
    if (vec)
      hipLaunchKernelGGL((dw3_sum_kernel<float, 4>), dim3(g), dim3(256), lds, s, (const float*)in, in_cs, in_co, n, h,
                         w, c, wts, bsum, (float*)out);
    else
      hipLaunchKernelGGL((dw3_sum_kernel<float, 1>), dim3(g), dim3(256), lds, s, (const float*)in, in_cs, in_co, n, h,
                         w, c, wts, bsum, (float*)out);
  }
  RTDM_HIP(hipGetLastError());
}

// ----------------------------------------------------------------- maxpool --
// nn.MaxPool2d(k, s, padding=pad) (implicit -inf padding), or, for the
// Darknet size-2/stride-1 case, ZeroPad2d((0,1,0,1)) + MaxPool2d(2,1)
// (models.py:57-64): padded cells read as 0.
template <typename T>
__global__ __launch_bounds__(256) void maxpool_kernel(const T* __restrict__ in, int in_cs, int in_co, int n, int h,
                                                      int w, int c, int k, int stride, int pad, int zero_rb,
                                                      T* __restrict__ out, int out_cs, int out_co, int oh, int ow) {
  const int64_t total = (int64_t)n * oh * ow * c;
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const int ch = (int)(idx % c);
    int64_t p = idx / c;
    const int ox = (int)(p % ow);
    p /= ow;
    const int oy = (int)(p % oh);
    const int b = (int)(p / oh);
    float m = -INFINITY;
    const int y0 = oy * stride - pad, x0 = ox * stride - pad;
    for (int dy = 0; dy < k; ++dy) {
      const int iy = y0 + dy;
      for (int dx = 0; dx < k; ++dx) {
        const int ix = x0 + dx;
        float v;
        if ((unsigned)iy < (unsigned)h && (unsigned)ix < (unsigned)w)
          v = ldf(in + (((size_t)b * h + iy) * w + ix) * in_cs + in_co + ch);
        else if (zero_rb)
          v = 0.f;
        else
          continue;
        m = fmaxf(m, v);
      }
    }
    out[(((size_t)b * oh + oy) * ow + ox) * out_cs + out_co + ch] = (T)m;
  }
}

template <typename T, int VEC>
// 32-bit item index (total < 2^31, checked at launch; unsigned loop cursor) split by multiply-shift divisions:
// the 64-bit div / mod chain per item cost more than the item's memory traffic.
__global__ __launch_bounds__(256) void maxpool_vec_kernel(const T* __restrict__ in, int in_cs, int in_co, int n,
                                                          int h, int w, int c, int k, int stride, int pad,
                                                          int zero_rb, T* __restrict__ out, int out_cs, int out_co,
                                                          int oh, int ow, FastDiv fcg, FastDiv fow, FastDiv foh) {
  typedef T tv __attribute__((ext_vector_type(VEC)));
  const int cg = c / VEC;
  const int total = n * oh * ow * cg;
  // unsigned cursor: total < 2^31 and the stride < 2^31, so idx + stride < 2^32 never wraps
  // (a signed idx + stride could overflow for total within a grid's span of 2^31)
  for (unsigned uidx = blockIdx.x * blockDim.x + threadIdx.x; uidx < (unsigned)total; uidx += gridDim.x * blockDim.x) {
    const int idx = (int)uidx;
    int p = fdiv(idx, fcg);
    const int g = idx - p * cg;
    const int q = fdiv(p, fow);
    const int ox = p - q * ow;
    const int b = fdiv(q, foh);
    const int oy = q - b * oh;
    float m[VEC];
#pragma unroll
    for (int j = 0; j < VEC; ++j) m[j] = -INFINITY;
    const int y0 = oy * stride - pad, x0 = ox * stride - pad;
    for (int dy = 0; dy < k; ++dy) {
      const int iy = y0 + dy;
      for (int dx = 0; dx < k; ++dx) {
        const int ix = x0 + dx;
        if ((unsigned)iy < (unsigned)h && (unsigned)ix < (unsigned)w) {
          const tv v = *(const tv*)(in + (((size_t)b * h + iy) * w + ix) * in_cs + in_co + g * VEC);
#pragma unroll
          for (int j = 0; j < VEC; ++j) m[j] = fmaxf(m[j], (float)v[j]);
        } else if (zero_rb) {
#pragma unroll
          for (int j = 0; j < VEC; ++j) m[j] = fmaxf(m[j], 0.f);
        }
      }
    }
    tv o;
#pragma unroll
    for (int j = 0; j < VEC; ++j) o[j] = (T)m[j];
    *(tv*)(out + (((size_t)b * oh + oy) * ow + ox) * out_cs + out_co + g * VEC) = o;
  }
}

// Stride-1 "same" max pools with K >= 5 (the SPP block of yolov3-spp: 5 / 9 / 13,
// models.py:57-64 with padding (K-1)/2, i.e. -inf outside the map): one thread per (image,
// column, 8-channel group, band of R output rows) computes the R + K - 1 horizontal K-maxima
// its band needs once (K loads each) and takes each output as the max of K of them: ~(R + K
// - 1) K / R loads per output instead of K^2 (13: 32.5 instead of 169).  max is exact and
// takes the same window, so the values are the generic kernel's (in fp16, as stored).
// ZRB: Darknet's size-2 stride-1 pool (ZeroPad2d((0,1,0,1)) + MaxPool2d(2,1), models.py:57-64):
// the window starts at the output pixel and taps past the right / bottom edge are zeros.
template <int K, int R, bool ZRB = false>
__global__ __launch_bounds__(256) void maxpool_s1_sep_kernel(const _Float16* __restrict__ in, int in_cs, int in_co, int n,
                                                             int h, int w, int c, _Float16* __restrict__ out, int out_cs,
                                                             int out_co) {
  typedef _Float16 h8v_ __attribute__((ext_vector_type(8)));
  constexpr int P = ZRB ? 0 : K / 2, NR = R + K - 1;
  const _Float16 pad_v = ZRB ? (_Float16)0.f : (_Float16)-INFINITY;  // value of a tap off the map
  const int cg = c >> 3, bands = (h + R - 1) / R;
  const int total = n * bands * w * cg;
  for (unsigned uidx = blockIdx.x * blockDim.x + threadIdx.x; uidx < (unsigned)total; uidx += gridDim.x * blockDim.x) {
    int idx = (int)uidx;
    const int g = idx % cg;
    idx /= cg;
    const int x = idx % w;
    idx /= w;
    const int band = idx % bands, b = idx / bands;
    const int y0 = band * R;
    const _Float16* base = in + (size_t)b * h * w * in_cs + in_co + g * 8;
    h8v_ hm[NR];
#pragma unroll
    for (int r = 0; r < NR; ++r) {
      const int iy = y0 - P + r;
      h8v_ m;
#pragma unroll
      for (int j = 0; j < 8; ++j) m[j] = pad_v;
      if ((unsigned)iy < (unsigned)h) {  // (a row off the map is pad_v throughout)
#pragma unroll
        for (int j = 0; j < 8; ++j) m[j] = (_Float16)-INFINITY;
#pragma unroll
        for (int dx = 0; dx < K; ++dx) {
          const int ix = x - P + dx;
          if ((unsigned)ix < (unsigned)w) {
            const h8v_ v = *(const h8v_*)(base + ((size_t)iy * w + ix) * in_cs);
#pragma unroll
            for (int j = 0; j < 8; ++j) m[j] = m[j] > v[j] ? m[j] : v[j];
          } else if (ZRB) {
#pragma unroll
            for (int j = 0; j < 8; ++j) m[j] = m[j] > pad_v ? m[j] : pad_v;
          }
        }
      }
      hm[r] = m;
    }
#pragma unroll
    for (int o = 0; o < R; ++o) {
      const int oy = y0 + o;
      if (oy >= h) break;
      h8v_ m = hm[o];
#pragma unroll
      for (int r = 1; r < K; ++r)
#pragma unroll
        for (int j = 0; j < 8; ++j) m[j] = m[j] > hm[o + r][j] ? m[j] : hm[o + r][j];
      *(h8v_*)(out + (((size_t)b * h + oy) * w + x) * out_cs + out_co + g * 8) = m;
    }
  }
}

void launch_maxpool(const void* in, View iv, int n, int h, int w, int c, int k, int stride, int pad, int zero_rb,
                    View ov, int oh, int ow, int dtype, hipStream_t s) {
  (void)in;
  const int64_t total = (int64_t)n * oh * ow * c;
  if (total <= 0) return;
  const bool spp = !zero_rb && (k == 5 || k == 9 || k == 13) && pad == k / 2;
  const bool zrb2 = zero_rb && k == 2 && pad == 0;
  if (dtype == RTDM_F16 && tune().pool_sep && stride == 1 && (spp || zrb2) && oh == h && ow == w && c % 8 == 0 &&
      ((iv.cs | iv.co | ov.cs | ov.co) % 8) == 0 && (int64_t)n * ((h + 7) / 8) * w * (c / 8) < (1ll << 31)) {
    constexpr int R = 8;
    const int gv = grid_for((int64_t)n * ((h + R - 1) / R) * w * (c / 8), 256);
    const _Float16* ip = (const _Float16*)iv.ptr;
    _Float16* op = (_Float16*)ov.ptr;
    if (zrb2)
      hipLaunchKernelGGL((maxpool_s1_sep_kernel<2, R, true>), dim3(gv), dim3(256), 0, s, ip, iv.cs, iv.co, n, h, w, c, op, ov.cs, ov.co);
    else if (k == 5)
      hipLaunchKernelGGL((maxpool_s1_sep_kernel<5, R>), dim3(gv), dim3(256), 0, s, ip, iv.cs, iv.co, n, h, w, c, op, ov.cs, ov.co);
    else if (k == 9)
      hipLaunchKernelGGL((maxpool_s1_sep_kernel<9, R>), dim3(gv), dim3(256), 0, s, ip, iv.cs, iv.co, n, h, w, c, op, ov.cs, ov.co);
    else
      hipLaunchKernelGGL((maxpool_s1_sep_kernel<13, R>), dim3(gv), dim3(256), 0, s, ip, iv.cs, iv.co, n, h, w, c, op, ov.cs, ov.co);
    RTDM_HIP(hipGetLastError());
    return;
  }
  const int vec = dtype == RTDM_F16 ? 8 : 4;
  if (c % vec == 0 && ((iv.cs | iv.co | ov.cs | ov.co) % vec) == 0 && total / vec < (1ll << 31)) {
    const int gv = grid_for(total / vec, 256);
    const FastDiv fcg = make_fastdiv(c / vec), fow = make_fastdiv(ow), foh = make_fastdiv(oh);
    if (dtype == RTDM_F16)
      hipLaunchKernelGGL((maxpool_vec_kernel<_Float16, 8>), dim3(gv), dim3(256), 0, s, (const _Float16*)iv.ptr, iv.cs,
                         iv.co, n, h, w, c, k, stride, pad, zero_rb, (_Float16*)ov.ptr, ov.cs, ov.co, oh, ow, fcg, fow,
                         foh);
    else
      hipLaunchKernelGGL((maxpool_vec_kernel<float, 4>), dim3(gv), dim3(256), 0, s, (const float*)iv.ptr, iv.cs, iv.co,
                         n, h, w, c, k, stride, pad, zero_rb, (float*)ov.ptr, ov.cs, ov.co, oh, ow, fcg, fow, foh);
    RTDM_HIP(hipGetLastError());
    return;
  }
  const int g = grid_for(total, 256);
  if (dtype == RTDM_F16)
    hipLaunchKernelGGL(maxpool_kernel<_Float16>, dim3(g), dim3(256), 0, s, (const _Float16*)iv.ptr, iv.cs, iv.co, n,
                       h, w, c, k, stride, pad, zero_rb, (_Float16*)ov.ptr, ov.cs, ov.co, oh, ow);
  else
    hipLaunchKernelGGL(maxpool_kernel<float>, dim3(g), dim3(256), 0, s, (const float*)iv.ptr, iv.cs, iv.co, n, h, w,
                       c, k, stride, pad, zero_rb, (float*)ov.ptr, ov.cs, ov.co, oh, ow);
  RTDM_HIP(hipGetLastError());
}

// ----------------------------------------------------- upsample / route copy --
template <typename T>
__global__ __launch_bounds__(256) void upsample_kernel(const T* __restrict__ in, int in_cs, int in_co, int n, int h,
                                                       int w, int c, int f, T* __restrict__ out, int out_cs,
                                                       int out_co) {
  const int oh = h * f, ow = w * f;
  const int64_t total = (int64_t)n * oh * ow * c;
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const int ch = (int)(idx % c);
    int64_t p = idx / c;
    const int ox = (int)(p % ow);
    p /= ow;
    const int oy = (int)(p % oh);
    const int b = (int)(p / oh);
    out[(((size_t)b * oh + oy) * ow + ox) * out_cs + out_co + ch] =
        in[(((size_t)b * h + oy / f) * w + ox / f) * in_cs + in_co + ch];
  }
}

void launch_upsample(View iv, int n, int h, int w, int c, int f, View ov, int dtype, hipStream_t s) {
  const int64_t total = (int64_t)n * h * f * w * f * c;
  if (total <= 0) return;
  const int g = grid_for(total, 256);
  if (dtype == RTDM_F16)
    hipLaunchKernelGGL(upsample_kernel<_Float16>, dim3(g), dim3(256), 0, s, (const _Float16*)iv.ptr, iv.cs, iv.co, n,
                       h, w, c, f, (_Float16*)ov.ptr, ov.cs, ov.co);
  else
    hipLaunchKernelGGL(upsample_kernel<float>, dim3(g), dim3(256), 0, s, (const float*)iv.ptr, iv.cs, iv.co, n, h, w,
                       c, f, (float*)ov.ptr, ov.cs, ov.co);
  RTDM_HIP(hipGetLastError());
}

// Unfused [shortcut] (weightedFeatureFusion.forward, models.py:135-155): out has the current
// map's c channels; the first cb of them get the residual added (cb = min(c, residual
// channels): dc > 0 adds into x[:, :ac], dc < 0 reads only a[:, :nc]); the rest are copied.
template <typename T>
__global__ __launch_bounds__(256) void add_kernel(const T* __restrict__ a, int a_cs, int a_co, const T* __restrict__ b,
                                                  int b_cs, int b_co, int64_t pix, int c, int cb, T* __restrict__ out,
                                                  int o_cs, int o_co) {
  const int64_t total = pix * c;
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const int ch = (int)(idx % c);
    const int64_t p = idx / c;
    const T x = a[p * a_cs + a_co + ch];
    out[p * o_cs + o_co + ch] = ch < cb ? (T)((float)x + (float)b[p * b_cs + b_co + ch]) : x;
  }
}

void launch_add(View a, View b, int n, int h, int w, int c, int cb, View ov, int dtype, hipStream_t s) {
  const int64_t pix = (int64_t)n * h * w;
  if (pix * c <= 0) return;
  const int g = grid_for(pix * c, 256);
  if (dtype == RTDM_F16)
    hipLaunchKernelGGL(add_kernel<_Float16>, dim3(g), dim3(256), 0, s, (const _Float16*)a.ptr, a.cs, a.co,
                       (const _Float16*)b.ptr, b.cs, b.co, pix, c, cb, (_Float16*)ov.ptr, ov.cs, ov.co);
  else
    hipLaunchKernelGGL(add_kernel<float>, dim3(g), dim3(256), 0, s, (const float*)a.ptr, a.cs, a.co,
                       (const float*)b.ptr, b.cs, b.co, pix, c, cb, (float*)ov.ptr, ov.cs, ov.co);
  RTDM_HIP(hipGetLastError());
}

// Route resize of YOLO-ACFF (models.py:364-375 -> F.interpolate nearest, given size):
// PyTorch's nearest source index, scale = in / out in fp32.
template <typename T>
__global__ __launch_bounds__(256) void resize_nearest_kernel(const T* __restrict__ in, int in_cs, int in_co, int n,
                                                             int h, int w, int c, T* __restrict__ out, int out_cs,
                                                             int out_co, int oh, int ow) {
  const float sy = (float)h / (float)oh, sx = (float)w / (float)ow;
  const int64_t total = (int64_t)n * oh * ow * c;
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const int ch = (int)(idx % c);
    int64_t p = idx / c;
    const int ox = (int)(p % ow);
    p /= ow;
    const int oy = (int)(p % oh);
    const int b = (int)(p / oh);
    const int iy = min((int)floorf((float)oy * sy), h - 1), ix = min((int)floorf((float)ox * sx), w - 1);
    out[(((size_t)b * oh + oy) * ow + ox) * out_cs + out_co + ch] =
        in[(((size_t)b * h + iy) * w + ix) * in_cs + in_co + ch];
  }
}

void launch_resize_nearest(View iv, int n, int h, int w, int c, View ov, int oh, int ow, int dtype, hipStream_t s) {
  const int64_t total = (int64_t)n * oh * ow * c;
  if (total <= 0) return;
  const int g = grid_for(total, 256);
  if (dtype == RTDM_F16)
    hipLaunchKernelGGL(resize_nearest_kernel<_Float16>, dim3(g), dim3(256), 0, s, (const _Float16*)iv.ptr, iv.cs,
                       iv.co, n, h, w, c, (_Float16*)ov.ptr, ov.cs, ov.co, oh, ow);
  else
    hipLaunchKernelGGL(resize_nearest_kernel<float>, dim3(g), dim3(256), 0, s, (const float*)iv.ptr, iv.cs, iv.co, n,
                       h, w, c, (float*)ov.ptr, ov.cs, ov.co, oh, ow);
  RTDM_HIP(hipGetLastError());
}

void launch_copy_slice(View iv, int n, int h, int w, int c, View ov, int dtype, hipStream_t s) {
  launch_upsample(iv, n, h, w, c, 1, ov, dtype, s);
}

template <typename T>
__global__ __launch_bounds__(256) void to_nchw_kernel(const T* __restrict__ in, int cs, int co, int n, int h, int w,
                                                      int c, float* __restrict__ out) {
  const int64_t total = (int64_t)n * c * h * w;
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const int x = (int)(idx % w);
    int64_t p = idx / w;
    const int y = (int)(p % h);
    p /= h;
    const int ch = (int)(p % c);
    const int b = (int)(p / c);
    out[idx] = ldf(in + (((size_t)b * h + y) * w + x) * cs + co + ch);
  }
}

void launch_to_nchw_f32(View iv, int n, int h, int w, int c, float* out, int dtype, hipStream_t s) {
  const int64_t total = (int64_t)n * c * h * w;
  if (total <= 0) return;
  const int g = grid_for(total, 256);
  if (dtype == RTDM_F16)
    hipLaunchKernelGGL(to_nchw_kernel<_Float16>, dim3(g), dim3(256), 0, s, (const _Float16*)iv.ptr, iv.cs, iv.co, n,
                       h, w, c, out);
  else
    hipLaunchKernelGGL(to_nchw_kernel<float>, dim3(g), dim3(256), 0, s, (const float*)iv.ptr, iv.cs, iv.co, n, h, w,
                       c, out);
  RTDM_HIP(hipGetLastError());
}

// --------------------------------------------------------- classifier tail --
// conv2 1x1 C->5 (no bias) -> AvgPool2d(5, 1, pool_pad) (count_include_pad:
// divisor 25) -> view(-1, 5*ph*pw) in NCHW order -> Linear -> Softmax
// (squeeze_ernet.py:33-41, ernet.py:38-45).  One 1024-thread block per image.
template <typename T>
__global__ __launch_bounds__(1024) void cls_tail_kernel(const T* __restrict__ in, int h, int w, int c,
                                                       const float* __restrict__ w2, int pool_pad, int ph, int pw,
                                                       const float* __restrict__ fcw, const float* __restrict__ fcb,
                                                       float* __restrict__ logits, float* __restrict__ probs) {
  __shared__ float conv[5 * 64];  // [o][y*w+x], h*w <= 64
  __shared__ float feat[5 * 16];
  __shared__ float lg[5];
  const int b = blockIdx.x;
  const int hw = h * w;
  const T* src = in + (size_t)b * hw * c;
  // conv2: one wave per pixel, lanes stride the channels (coalesced), wave sum
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  for (int p = wid; p < hw; p += blockDim.x >> 6) {
    const T* x = src + (size_t)p * c;
    float acc[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
    for (int ch = lane; ch < c; ch += 64) {
      const float xv = ldf(x + ch);
#pragma unroll
      for (int o = 0; o < 5; ++o) acc[o] = fmaf(xv, w2[(size_t)o * c + ch], acc[o]);
    }
#pragma unroll
    for (int o = 0; o < 5; ++o) {
      float v = acc[o];
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
      if (lane == 0) conv[o * hw + p] = v;
    }
  }
  __syncthreads();
  const int nf = 5 * ph * pw;
  for (int t = threadIdx.x; t < nf; t += blockDim.x) {
    const int o = t / (ph * pw);
    const int r = t - o * ph * pw;
    const int i = r / pw, j = r - (r / pw) * pw;
    float s = 0.f;
    for (int dy = 0; dy < 5; ++dy) {
      const int y = i - pool_pad + dy;
      if ((unsigned)y >= (unsigned)h) continue;
      for (int dx = 0; dx < 5; ++dx) {
        const int x = j - pool_pad + dx;
        if ((unsigned)x >= (unsigned)w) continue;
        s += conv[o * hw + y * w + x];
      }
    }
    feat[t] = s / 25.f;
  }
  __syncthreads();
  if (threadIdx.x < 5) {
    const int k = threadIdx.x;
    float acc = 0.f;
    for (int q = 0; q < nf; ++q) acc = fmaf(feat[q], fcw[k * nf + q], acc);
    acc += fcb[k];
    lg[k] = acc;
    if (logits) logits[b * 5 + k] = acc;
  }
  __syncthreads();
  if (threadIdx.x < 5 && probs) {
    float mx = lg[0];
    for (int k = 1; k < 5; ++k) mx = fmaxf(mx, lg[k]);
    float sum = 0.f;
    for (int k = 0; k < 5; ++k) sum += expf(lg[k] - mx);
    probs[b * 5 + threadIdx.x] = expf(lg[threadIdx.x] - mx) / sum;
  }
}

void launch_cls_tail(const void* in, int n, int h, int w, int c, const float* w2, int pool_pad, int ph, int pw,
                     const float* fcw, const float* fcb, float* logits, float* probs, int dtype, hipStream_t s) {
  RTDM_REQUIRE(h * w <= 64 && ph * pw <= 16, RTDM_E_UNSUPPORTED, "classifier tail: feature map too large");
  if (n <= 0) return;
  if (dtype == RTDM_F16)
    hipLaunchKernelGGL(cls_tail_kernel<_Float16>, dim3(n), dim3(1024), 0, s, (const _Float16*)in, h, w, c, w2,
                       pool_pad, ph, pw, fcw, fcb, logits, probs);
  else
    hipLaunchKernelGGL(cls_tail_kernel<float>, dim3(n), dim3(1024), 0, s, (const float*)in, h, w, c, w2, pool_pad, ph,
                       pw, fcw, fcb, logits, probs);
  RTDM_HIP(hipGetLastError());
}

// ------------------------------------------------------------- preprocess --
// Pillow's antialiased BILINEAR resize for 8-bit images (Resample.c:
// precompute_coeffs + normalize_coeffs_8bpc, horizontal pass then vertical
// pass, PRECISION_BITS = 22, clip8), as torchvision.transforms.Resize calls
// it, followed by CenterCrop, ToTensor and Normalize (aider.py:421-426).
static constexpr int kPrecisionBits = 32 - 8 - 2;

static int precompute_coeffs(int in_size, int out_size, std::vector<int>& bounds, std::vector<double>& kk) {
  const double in0 = 0.0, in1 = (double)(float)in_size;
  double scale = (in1 - in0) / out_size;
  double filterscale = scale < 1.0 ? 1.0 : scale;
  const double support = 1.0 * filterscale;  // bilinear support = 1
  const int ksize = (int)std::ceil(support) * 2 + 1;
  bounds.assign(out_size * 2, 0);
  kk.assign((size_t)out_size * ksize, 0.0);
  for (int xx = 0; xx < out_size; ++xx) {
    const double center = in0 + (xx + 0.5) * scale;
    double ww = 0.0;
    const double ss = 1.0 / filterscale;
    int xmin = (int)(center - support + 0.5);
    if (xmin < 0) xmin = 0;
    int xmax = (int)(center + support + 0.5);
    if (xmax > in_size) xmax = in_size;
    xmax -= xmin;
    double* k = &kk[(size_t)xx * ksize];
    for (int x = 0; x < xmax; ++x) {
      double t = (x + xmin - center + 0.5) * ss;
      if (t < 0.0) t = -t;
      const double wv = t < 1.0 ? 1.0 - t : 0.0;
      k[x] = wv;
      ww += wv;
    }
    for (int x = 0; x < xmax; ++x)
      if (ww != 0.0) k[x] /= ww;
    bounds[xx * 2 + 0] = xmin;
    bounds[xx * 2 + 1] = xmax;
  }
  return ksize;
}

static std::vector<int> normalize_coeffs_8bpc(const std::vector<double>& kk) {
  std::vector<int> out(kk.size());
  for (size_t i = 0; i < kk.size(); ++i) {
    const double v = kk[i] * (double)(1 << kPrecisionBits);
    out[i] = kk[i] < 0 ? (int)(-0.5 + v) : (int)(0.5 + v);
  }
  return out;
}

void build_resize_plan(ResizePlan& p, int in_h, int in_w, int out_size, bool upload) {
  RTDM_REQUIRE(in_h > 0 && in_w > 0 && out_size > 0, RTDM_E_INVALID, "preprocess: bad sizes");
  p.in_h = in_h;
  p.in_w = in_w;
  p.out = out_size;
  // torchvision Resize(int): shorter side -> size, long side int(size * long / short)
  const int size = (int)(out_size * 1.14);
  if (in_w <= in_h) {
    p.rs_w = size;
    p.rs_h = (int)((double)size * in_h / in_w);
  } else {
    p.rs_h = size;
    p.rs_w = (int)((double)size * in_w / in_h);
  }
  RTDM_REQUIRE(p.rs_h >= out_size && p.rs_w >= out_size, RTDM_E_INVALID, "preprocess: crop larger than image");
  // CenterCrop: int(round((dim - crop) / 2.))  (Python round = half to even)
  auto pyround_half = [](int twice) {  // round(twice / 2)
    if (twice % 2 == 0) return twice / 2;
    const int lo = twice / 2;  // x.5 -> even
    return (lo % 2 == 0) ? lo : lo + 1;
  };
  p.crop_top = pyround_half(p.rs_h - out_size);
  p.crop_left = pyround_half(p.rs_w - out_size);

  std::vector<int> bh, bv;
  std::vector<double> kh, kv;
  const bool need_h = p.rs_w != in_w;
  const bool need_v = p.rs_h != in_h;
  if (need_h) {
    p.ksize_h = precompute_coeffs(in_w, p.rs_w, bh, kh);
  } else {  // identity pass: one tap of weight 1
    p.ksize_h = 1;
    bh.resize(p.rs_w * 2);
    kh.assign(p.rs_w, 1.0);
    for (int x = 0; x < p.rs_w; ++x) { bh[2 * x] = x; bh[2 * x + 1] = 1; }
  }
  if (need_v) {
    p.ksize_v = precompute_coeffs(in_h, p.rs_h, bv, kv);
  } else {
    p.ksize_v = 1;
    bv.resize(p.rs_h * 2);
    kv.assign(p.rs_h, 1.0);
    for (int y = 0; y < p.rs_h; ++y) { bv[2 * y] = y; bv[2 * y + 1] = 1; }
  }
  // restrict to the crop window
  std::vector<int> ch(out_size * 2), cv(out_size * 2);
  std::vector<int> kh8 = normalize_coeffs_8bpc(kh), kv8 = normalize_coeffs_8bpc(kv);
  std::vector<int> kch((size_t)out_size * p.ksize_h), kcv((size_t)out_size * p.ksize_v);
  int rmin = 1 << 30, rmax = 0;
  for (int i = 0; i < out_size; ++i) {
    const int x = p.crop_left + i;
    ch[2 * i] = bh[2 * x];
    ch[2 * i + 1] = bh[2 * x + 1];
    for (int k = 0; k < p.ksize_h; ++k) kch[(size_t)i * p.ksize_h + k] = kh8[(size_t)x * p.ksize_h + k];
    const int y = p.crop_top + i;
    cv[2 * i] = bv[2 * y];
    cv[2 * i + 1] = bv[2 * y + 1];
    for (int k = 0; k < p.ksize_v; ++k) kcv[(size_t)i * p.ksize_v + k] = kv8[(size_t)y * p.ksize_v + k];
    rmin = std::min(rmin, bv[2 * y]);
    rmax = std::max(rmax, bv[2 * y] + bv[2 * y + 1]);
  }
  p.row_first = rmin;
  p.rows = rmax - rmin;
  for (int i = 0; i < out_size; ++i) cv[2 * i] -= rmin;
  p.col_first = 1 << 30;
  int col_end = 0;
  for (int i = 0; i < out_size; ++i) {
    p.col_first = std::min(p.col_first, ch[2 * i]);
    col_end = std::max(col_end, ch[2 * i] + ch[2 * i + 1]);
  }
  p.col_end = col_end;
  p.band_rows8 = 0;
  for (int y0 = 0; y0 < out_size; y0 += 8) {  // kResizeBandS
    const int y1 = std::min(out_size, y0 + 8) - 1;
    p.band_rows8 = std::max(p.band_rows8, cv[2 * y1] + cv[2 * y1 + 1] - cv[2 * y0]);
  }
  p.band_rows = 0;
  p.band_rows17 = 0;
  for (int y0 = 0; y0 < out_size; y0 += 16) {  // kResizeBand
    const int y1 = std::min(out_size, y0 + 16) - 1, y2 = std::min(out_size, y0 + 17) - 1;
    p.band_rows = std::max(p.band_rows, cv[2 * y1] + cv[2 * y1 + 1] - cv[2 * y0]);
    p.band_rows17 = std::max(p.band_rows17, cv[2 * y2] + cv[2 * y2 + 1] - cv[2 * y0]);
  }
  if (!upload) return;
  auto up = [](DevBuf& d, const std::vector<int>& v) {
    d.alloc(v.size() * sizeof(int));
    RTDM_HIP(hipMemcpy(d.p, v.data(), v.size() * sizeof(int), hipMemcpyHostToDevice));
  };
  up(p.bounds_h, ch);
  up(p.coef_h, kch);
  up(p.bounds_v, cv);
  up(p.coef_v, kcv);
}

__device__ __forceinline__ int clip8(int v) {
  v >>= kPrecisionBits;
  return v < 0 ? 0 : (v > 255 ? 255 : v);
}

// horizontal pass: frames [n,in_h,in_w,3] -> tmp [n,rows,out,3] (crop columns only)
__global__ __launch_bounds__(256) void resize_h_kernel(const uint8_t* __restrict__ frames, int n, int in_h, int in_w,
                                                       int row_first, int rows, int out, int ksize,
                                                       const int* __restrict__ bounds, const int* __restrict__ coef,
                                                       uint8_t* __restrict__ tmp) {
  const int64_t total = (int64_t)n * rows * out;
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const int xx = (int)(idx % out);
    int64_t p = idx / out;
    const int r = (int)(p % rows);
    const int b = (int)(p / rows);
    const int xmin = bounds[2 * xx], xmax = bounds[2 * xx + 1];
    const int* k = coef + (size_t)xx * ksize;
    const uint8_t* src = frames + (((size_t)b * in_h + row_first + r) * in_w + xmin) * 3;
    int s0 = 1 << (kPrecisionBits - 1), s1 = s0, s2 = s0;
    for (int x = 0; x < xmax; ++x) {
      s0 += src[x * 3 + 0] * k[x];
      s1 += src[x * 3 + 1] * k[x];
      s2 += src[x * 3 + 2] * k[x];
    }
    uint8_t* dst = tmp + idx * 3;
    dst[0] = (uint8_t)clip8(s0);
    dst[1] = (uint8_t)clip8(s1);
    dst[2] = (uint8_t)clip8(s2);
  }
}

// vertical pass + ToTensor + Normalize: tmp -> out [n,out,out,3] NHWC (dtype) or NCHW f32
template <typename T>
__global__ __launch_bounds__(256) void resize_v_kernel(const uint8_t* __restrict__ tmp, int n, int rows, int out,
                                                       int ksize, const int* __restrict__ bounds,
                                                       const int* __restrict__ coef, T* __restrict__ dst, int nchw) {
  const float mean[3] = {0.485f, 0.456f, 0.406f};
  const float stdv[3] = {0.229f, 0.224f, 0.225f};
  const int64_t total = (int64_t)n * out * out;
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const int xx = (int)(idx % out);
    int64_t p = idx / out;
    const int yy = (int)(p % out);
    const int b = (int)(p / out);
    const int ymin = bounds[2 * yy], ymax = bounds[2 * yy + 1];
    const int* k = coef + (size_t)yy * ksize;
    int s[3] = {1 << (kPrecisionBits - 1), 1 << (kPrecisionBits - 1), 1 << (kPrecisionBits - 1)};
    for (int y = 0; y < ymax; ++y) {
      const uint8_t* src = tmp + (((size_t)b * rows + ymin + y) * out + xx) * 3;
#pragma unroll
      for (int ch = 0; ch < 3; ++ch) s[ch] += src[ch] * k[y];
    }
#pragma unroll
    for (int ch = 0; ch < 3; ++ch) {
      const float v = ((float)clip8(s[ch]) / 255.f - mean[ch]) / stdv[ch];
      if (nchw)
        dst[(((size_t)b * 3 + ch) * out + yy) * out + xx] = (T)v;
      else
        dst[idx * 3 + ch] = (T)v;
    }
  }
}

// Fused form: one block per (image, band of kResizeBand output rows).  The
// band's input rows get the horizontal pass straight from the frame into an
// LDS row buffer (uint8 after clip8, like Pillow's intermediate image), then
// the vertical pass + ToTensor + Normalize reads only LDS.  Same integer
// arithmetic as the two-kernel path (bit-exact with Pillow).
constexpr int kResizeBand = 16;

template <typename T>
__global__ __launch_bounds__(256) void resize_fused_kernel(const uint8_t* __restrict__ frames, int in_h, int in_w,
                                                           int row_first, int out, int kh_size, int kv_size,
                                                           const int* __restrict__ bh, const int* __restrict__ ch,
                                                           const int* __restrict__ bv, const int* __restrict__ cv,
                                                           T* __restrict__ dst, int nchw) {
  extern __shared__ __attribute__((aligned(16))) int rs_lds[];
  int* kcoef = rs_lds;                       // [out][kh_size]
  int* kb = kcoef + out * kh_size;           // [out][2]
  uint8_t* tmp = (uint8_t*)(kb + 2 * out);   // [band rows][out][3]
  const int bands = (out + kResizeBand - 1) / kResizeBand;
  const int b = blockIdx.x / bands;
  const int yy0 = (blockIdx.x - b * bands) * kResizeBand;
  const int yy1 = yy0 + kResizeBand < out ? yy0 + kResizeBand : out;
  const int r0 = bv[2 * yy0];
  const int r1 = bv[2 * (yy1 - 1)] + bv[2 * (yy1 - 1) + 1];
  for (int i = threadIdx.x; i < out * kh_size; i += 256) kcoef[i] = ch[i];
  for (int i = threadIdx.x; i < 2 * out; i += 256) kb[i] = bh[i];
  __syncthreads();
  // horizontal pass for input rows row_first + [r0, r1)
  const int nrow = r1 - r0;
  for (int i = threadIdx.x; i < nrow * out; i += 256) {
    const int r = i / out, xx = i - r * out;
    const int xmin = kb[2 * xx], xmax = kb[2 * xx + 1];
    const int* k = kcoef + xx * kh_size;
    const uint8_t* src = frames + (((size_t)b * in_h + row_first + r0 + r) * in_w + xmin) * 3;
    int s0 = 1 << (kPrecisionBits - 1), s1 = s0, s2 = s0;
    for (int x = 0; x < xmax; ++x) {
      const int kx = k[x];
      s0 += src[x * 3 + 0] * kx;
      s1 += src[x * 3 + 1] * kx;
      s2 += src[x * 3 + 2] * kx;
    }
    uint8_t* d = tmp + (size_t)i * 3;
    d[0] = (uint8_t)clip8(s0);
    d[1] = (uint8_t)clip8(s1);
    d[2] = (uint8_t)clip8(s2);
  }
  __syncthreads();
  const float mean[3] = {0.485f, 0.456f, 0.406f};
  const float stdv[3] = {0.229f, 0.224f, 0.225f};
  for (int i = threadIdx.x; i < (yy1 - yy0) * out; i += 256) {
    const int yr = i / out, xx = i - yr * out;
    const int yy = yy0 + yr;
    const int ymin = bv[2 * yy] - r0, ymax = bv[2 * yy + 1];
    const int* k = cv + (size_t)yy * kv_size;
    int acc[3] = {1 << (kPrecisionBits - 1), 1 << (kPrecisionBits - 1), 1 << (kPrecisionBits - 1)};
    for (int y = 0; y < ymax; ++y) {
      const uint8_t* t = tmp + ((size_t)(ymin + y) * out + xx) * 3;
      const int ky = k[y];
#pragma unroll
      for (int c = 0; c < 3; ++c) acc[c] += t[c] * ky;
    }
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const float v = ((float)clip8(acc[c]) / 255.f - mean[c]) / stdv[c];
      if (nchw)
        dst[(((size_t)b * 3 + c) * out + yy) * out + xx] = (T)v;
      else
        dst[(((size_t)b * out + yy) * out + xx) * 3 + c] = (T)v;
    }
  }
}

// Staged form of the fused kernel (used when each frame row is 16-byte aligned):
// the band's input rows (only the columns the crop reads) are first copied into
// LDS with coalesced 16-byte loads, so the horizontal taps read LDS instead of
// issuing per-byte global loads.  Same integer arithmetic (bit-exact with Pillow).
constexpr int kResizeBandS = 8;

template <typename T>
__global__ __launch_bounds__(256) void resize_staged_kernel(const uint8_t* __restrict__ frames, int in_h, int in_w,
                                                            int row_first, int out, int kh_size, int kv_size,
                                                            int col_first, int col_bytes16, const int* __restrict__ bh,
                                                            const int* __restrict__ ch, const int* __restrict__ bv,
                                                            const int* __restrict__ cv, T* __restrict__ dst, int nchw) {
  extern __shared__ __attribute__((aligned(16))) int rs_lds[];
  int* kcoef = rs_lds;                          // [out][kh_size]
  int* kb = kcoef + out * kh_size;              // [out][2]
  uint8_t* srow = (uint8_t*)(kb + 2 * out);     // [band input rows][col_bytes16]
  const int bands = (out + kResizeBandS - 1) / kResizeBandS;
  const int b = blockIdx.x / bands;
  const int yy0 = (blockIdx.x - b * bands) * kResizeBandS;
  const int yy1 = yy0 + kResizeBandS < out ? yy0 + kResizeBandS : out;
  const int r0 = bv[2 * yy0];
  const int r1 = bv[2 * (yy1 - 1)] + bv[2 * (yy1 - 1) + 1];
  const int nrow = r1 - r0;
  const int c0b = (col_first * 3) & ~15;        // first staged byte of a row (16-aligned)
  const int delta = col_first * 3 - c0b;
  const int v16 = col_bytes16 >> 4;
  const uint8_t* fb = frames + ((size_t)b * in_h + row_first + r0) * in_w * 3 + c0b;
  for (int i = threadIdx.x; i < nrow * v16; i += 256) {
    const int r = i / v16, v = i - r * v16;
    *(uint4*)(srow + (size_t)r * col_bytes16 + v * 16) = *(const uint4*)(fb + (size_t)r * in_w * 3 + v * 16);
  }
  for (int i = threadIdx.x; i < out * kh_size; i += 256) kcoef[i] = ch[i];
  for (int i = threadIdx.x; i < 2 * out; i += 256) kb[i] = bh[i];
  __syncthreads();
  uint8_t* tmp = srow + (size_t)nrow * col_bytes16;  // [nrow][out][3]
  for (int i = threadIdx.x; i < nrow * out; i += 256) {
    const int r = i / out, xx = i - r * out;
    const int xmin = kb[2 * xx], xmax = kb[2 * xx + 1];
    const int* k = kcoef + xx * kh_size;
    const uint8_t* src = srow + (size_t)r * col_bytes16 + delta + (xmin - col_first) * 3;
    int s0 = 1 << (kPrecisionBits - 1), s1 = s0, s2 = s0;
    for (int x = 0; x < xmax; ++x) {
      const int kx = k[x];
      s0 += src[x * 3 + 0] * kx;
      s1 += src[x * 3 + 1] * kx;
      s2 += src[x * 3 + 2] * kx;
    }
    uint8_t* d = tmp + (size_t)i * 3;
    d[0] = (uint8_t)clip8(s0);
    d[1] = (uint8_t)clip8(s1);
    d[2] = (uint8_t)clip8(s2);
  }
  __syncthreads();
  const float mean[3] = {0.485f, 0.456f, 0.406f};
  const float stdv[3] = {0.229f, 0.224f, 0.225f};
  for (int i = threadIdx.x; i < (yy1 - yy0) * out; i += 256) {
    const int yr = i / out, xx = i - yr * out;
    const int yy = yy0 + yr;
    const int ymin = bv[2 * yy] - r0, ymax = bv[2 * yy + 1];
    const int* k = cv + (size_t)yy * kv_size;
    int acc[3] = {1 << (kPrecisionBits - 1), 1 << (kPrecisionBits - 1), 1 << (kPrecisionBits - 1)};
    for (int y = 0; y < ymax; ++y) {
      const uint8_t* t = tmp + ((size_t)(ymin + y) * out + xx) * 3;
      const int ky = k[y];
#pragma unroll
      for (int c = 0; c < 3; ++c) acc[c] += t[c] * ky;
    }
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const float v = ((float)clip8(acc[c]) / 255.f - mean[c]) / stdv[c];
      if (nchw)
        dst[(((size_t)b * 3 + c) * out + yy) * out + xx] = (T)v;
      else
        dst[(((size_t)b * out + yy) * out + xx) * 3 + c] = (T)v;
    }
  }
}

// Streaming form: one thread per output column, one block per (image, band of
// kRsBand output rows).
//   rows    the band's input rows (the crop's columns) stream by buffer->LDS
//           DMA through a kRsRing-slot LDS ring, kRsDepth rows in flight;
//   H pass  each thread keeps its column's horizontal taps in registers and
//           writes the clip8'ed result of every input row (Pillow's uint8
//           intermediate) as one packed dword into an LDS column image;
//   V pass  per output row, taps unrolled with the band's coefficients staged in
//           LDS (broadcast reads; zero weights past ymax read rows that exist in
//           the padded image).
// Integer sums are Pillow's (bit-exact: zero-weight taps add 0); no divisions,
// one barrier per input row.
constexpr int kRsBand = 16;   // output rows per block (= kResizeBand: ResizePlan::band_rows)
constexpr int kRsTaps = 7;    // max taps per pass (ksize) held unrolled
constexpr int kRsDepth = 6;   // input rows in flight (buffer->LDS) per wave
constexpr int kRsDepth2 = 4;  // rows in flight with rows taken in pairs (RP 2)
constexpr int kRsRing = 8;    // LDS ring slots (>= kRsDepth + 2, >= kRsDepth2 + 4), power of two
constexpr int kRsRowB = 2048; // ring slot bytes: 128 16-byte chunks (2 issuing waves)

// The classifiers' conv1 fused behind the resize (STEM): 3 -> 16 channels, 3x3, stride 2,
// pad 0 (squeeze_ernet.py:11, ernet.py:10) on the band's fp16 rows, which never reach HBM.
struct RsStem {
  const _Float16* w = nullptr;  // conv_stem3's packed weights [16][64] (K16: + 32 the kh = 2 link)
  const float* bias = nullptr;  // [16]
  _Float16* out = nullptr;      // [n, oh, oh, 16] fp16 NHWC
  int oh = 0;
};

// ABL (diagnostic builds only, outputs wrong when non-zero): 1 = no H-pass LDS reads,
// 2 = no V pass / output stores (one store per thread), 4 = no row DMA.
// RP: input rows per wait + barrier (1 or 2)
// STEM: also compute the band's conv1 rows (a band of 16 output rows + the next band's first
// row feeds 8 stem rows) instead of storing the resized rows
template <typename T, int ABL, int RP = 2, bool STEM = false>
__global__ __launch_bounds__(256) void resize_stream_kernel(const uint8_t* __restrict__ frames, int in_h, int in_w,
                                                            int row_first, int out, int kh_size, int kv_size,
                                                            int col_first, int c0b, int v16, int band_rows,
                                                            const int* __restrict__ bh, const int* __restrict__ ch,
                                                            const int* __restrict__ bv, const int* __restrict__ cv,
                                                            T* __restrict__ dst, int nchw, RsStem stp) {
  constexpr int KB = STEM ? kRsBand + 1 : kRsBand;  // resized rows computed per block
  extern __shared__ __attribute__((aligned(16))) uint8_t rsx_lds[];
  const int rstride = kRsRowB;                             // ring slot (zero-weight taps may read past v16*16)
  uint8_t* ring = rsx_lds;                                  // [kRsRing][kRsRowB]
  uint32_t* himg = (uint32_t*)(rsx_lds + kRsRing * kRsRowB);  // [band_rows + kRsTaps][256] packed (r,g,b)
  int* kv = (int*)(himg + (band_rows + kRsTaps) * 256);    // [KB][kRsTaps]
  const int bands = (out + kRsBand - 1) / kRsBand;
  const int bl = xcd_block(blockIdx.x, gridDim.x);  // consecutive bands (shared tap rows) on one XCD
  const int b = bl / bands;
  const int yy0 = (bl - b * bands) * kRsBand;
  const int nyy = out - yy0 < KB ? out - yy0 : KB;
  const int r0 = bv[2 * yy0];
  const int r1 = bv[2 * (yy0 + nyy - 1)] + bv[2 * (yy0 + nyy - 1) + 1];
  const int xx = threadIdx.x;
  const bool col = xx < out;
  // ToTensor + Normalize of the 256 possible uint8 values, per channel: the same
  // float expression as the per-pixel form, evaluated once per block
  float* lut = (float*)(kv + KB * kRsTaps);  // [3][256]
  {
    const float mean[3] = {0.485f, 0.456f, 0.406f};
    const float stdv[3] = {0.229f, 0.224f, 0.225f};
#pragma unroll
    for (int c = 0; c < 3; ++c) lut[c * 256 + xx] = ((float)xx / 255.f - mean[c]) / stdv[c];
  }
  for (int i = xx; i < KB * kRsTaps; i += 256) {
    const int j = i / kRsTaps, t = i - j * kRsTaps;
    kv[i] = j < nyy && t < bv[2 * (yy0 + j) + 1] && t < kv_size ? cv[(yy0 + j) * kv_size + t] : 0;
  }
  // rows past the band (read with zero weight) must hold finite data: zero them
  for (int i = xx; i < kRsTaps * 256; i += 256) himg[(r1 - r0) * 256 + i] = 0u;
  // this column's horizontal filter (zero weights past xmax)
  int kx[kRsTaps];
  int xoff;
  {
    const int xc = col ? xx : 0;
    const int xmax = bh[2 * xc + 1];
    xoff = (bh[2 * xc] - col_first) * 3 + (col_first * 3 - c0b);
#pragma unroll
    for (int t = 0; t < kRsTaps; ++t) kx[t] = (col && t < xmax && t < kh_size) ? ch[xc * kh_size + t] : 0;
  }
  const size_t rowb = (size_t)in_w * 3;
  // Rows arrive by buffer->LDS DMA into a kRsRing-slot ring, kRsDepth rows ahead of
  // the row being filtered.  Wave w's lane l carries 16-byte chunk 64w + l of a row
  // (lanes past the row get an out-of-range offset: the DMA writes zeros).  The
  // loads retire in order, so "row r landed" is one counted vmcnt per wave + a raw
  // barrier.  Row r+kRsDepth goes to the slot last read for row r+kRsDepth-kRsRing
  // <= r-2, released by row r-1's barrier.
  typedef __attribute__((address_space(3))) void* lds_t;
  const int wid = xx >> 6, chunk = xx;
  const bool issuer = wid * 64 < v16;  // wave-uniform
  const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(frames + (size_t)b * in_h * rowb), 0, (int)(in_h * rowb), 0x00020000);
  auto issue = [&](int r, int slot) {
    if (issuer && !(ABL & 4)) {
      const int rr = r < r1 ? r : r1 - 1;
      const int vo = chunk < v16 ? (int)((row_first + rr) * rowb) + c0b + chunk * 16 : (int)0x80000000;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (lds_t)(ring + slot * rstride + wid * 1024), 16, vo, 0, 0, 0);
    }
  };
  // the H pass of one landed row (ring slot sl) into himg row r - r0
  auto hpass = [&](int r, int sl) {
    int s0 = 1 << (kPrecisionBits - 1), s1 = s0, s2 = s0;
    if constexpr ((ABL & 1) != 0) {
      himg[(r - r0) * 256 + xx] = (uint32_t)(r + xx);
    } else {
      // the 21 tap bytes from 7 aligned dword reads, realigned with v_alignbyte (a
      // byte-granular or misaligned wide LDS read costs far more than this)
      const uint32_t* dw = (const uint32_t*)(ring + sl * rstride + (xoff & ~3));
      const int sh = xoff & 3;
      uint32_t d[7], wv[6];
#pragma unroll
      for (int k = 0; k < 7; ++k) d[k] = dw[k];
#pragma unroll
      for (int k = 0; k < 6; ++k) wv[k] = __builtin_amdgcn_alignbyte(d[k + 1], d[k], sh);
#pragma unroll
      for (int t = 0; t < kRsTaps; ++t) {
        // bytes x non-negative 22-bit weights: 24-bit multiplies (full rate)
        const int b0 = 3 * t, b1 = 3 * t + 1, b2 = 3 * t + 2;
        s0 += (int)__umul24((wv[b0 >> 2] >> (8 * (b0 & 3))) & 255u, kx[t]);
        s1 += (int)__umul24((wv[b1 >> 2] >> (8 * (b1 & 3))) & 255u, kx[t]);
        s2 += (int)__umul24((wv[b2 >> 2] >> (8 * (b2 & 3))) & 255u, kx[t]);
      }
      himg[(r - r0) * 256 + xx] = (uint32_t)clip8(s0) | ((uint32_t)clip8(s1) << 8) | ((uint32_t)clip8(s2) << 16);
    }
  };
  if constexpr (RP == 2) {
    // rows in pairs: one wait + barrier per two rows, two independent H-pass chains per thread.
    // kRsDepth2 rows in flight; row r + D (+1) goes to the slot read for row r + D - 8 (- 7) <=
    // r - 3, finished before the previous pair's barrier
#pragma unroll
    for (int q = 0; q < kRsDepth2; ++q) issue(r0 + q, q);
    int slot = 0, islot = kRsDepth2;
    for (int r = r0; r < r1; r += 2) {
      issue(r + kRsDepth2, islot);
      issue(r + kRsDepth2 + 1, (islot + 1) & (kRsRing - 1));
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(kRsDepth2) : "memory");
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      hpass(r, slot);
      if (r + 1 < r1) hpass(r + 1, (slot + 1) & (kRsRing - 1));  // (row r1 - r0 is the zero row)
      slot = (slot + 2) & (kRsRing - 1);
      islot = (islot + 2) & (kRsRing - 1);
    }
  } else {
#pragma unroll
    for (int q = 0; q < kRsDepth; ++q) issue(r0 + q, q);
    int slot = 0, islot = kRsDepth;
    for (int r = r0; r < r1; ++r) {
      issue(r + kRsDepth, islot);
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(kRsDepth) : "memory");
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      hpass(r, slot);
      slot = (slot + 1) & (kRsRing - 1);
      islot = (islot + 1) & (kRsRing - 1);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if constexpr (STEM) {
    // V pass into registers (fp16 pairs, the values the resized image would hold), then the
    // ring / H image are dead: the stem image [KB][out + 1] of (c0, c1, c2, 0) pixels (column
    // x + 1 = input column x, conv_stem3's LDS layout) overlays them
    uint32_t sp0[KB], sp1[KB];
    const int xc = col ? xx : 0;
#pragma unroll
    for (int j = 0; j < KB; ++j) {
      // (rows past the band repeat its last row: computed, never staged; no branches, so the
      // compiler keeps one row's loads live at a time)
      const int jj = j < nyy ? j : nyy - 1;
      const uint32_t* hp = himg + (bv[2 * (yy0 + jj)] - r0) * 256 + xc;
      int a0 = 1 << (kPrecisionBits - 1), a1 = a0, a2 = a0;
#pragma unroll
      for (int t = 0; t < kRsTaps; ++t) {
        const uint32_t hv = hp[t * 256];
        const int k = kv[jj * kRsTaps + t];
        a0 += (int)__umul24(hv & 255u, k);
        a1 += (int)__umul24((hv >> 8) & 255u, k);
        a2 += (int)__umul24(hv >> 16, k);
      }
      const _Float16 h0 = (_Float16)lut[clip8(a0)], h1 = (_Float16)lut[256 + clip8(a1)],
                     h2 = (_Float16)lut[512 + clip8(a2)];
      sp0[j] = (uint32_t)__builtin_bit_cast(uint16_t, h0) | ((uint32_t)__builtin_bit_cast(uint16_t, h1) << 16);
      sp1[j] = (uint32_t)__builtin_bit_cast(uint16_t, h2);
    }
    __syncthreads();
    uint2* simg = (uint2*)rsx_lds;
    const int ls = out + 2;  // columns 0 and out + 1: zero (the kw = 3 pixel of an odd width's last tile)
    if (col) {
#pragma unroll
      for (int j = 0; j < KB; ++j)
        if (j < nyy) simg[j * ls + xx + 1] = make_uint2(sp0[j], sp1[j]);
    }
    if (xx < 2 * KB) simg[(xx >> 1) * ls + ((xx & 1) ? out + 1 : 0)] = make_uint2(0u, 0u);
    __syncthreads();
    // stem rows oy = yy0 / 2 + tr, tr < 8: input rows 2 tr .. 2 tr + 2 of the band; 16-pixel
    // tiles on v_mfma 16x16x32 (kh 0, 1) + 16x16x16 (kh 2), conv_stem3's links and epilogue
    typedef _Float16 h8s __attribute__((ext_vector_type(8)));
    typedef _Float16 h4s __attribute__((ext_vector_type(4)));
    typedef float f4s __attribute__((ext_vector_type(4)));
    typedef unsigned int u4s __attribute__((ext_vector_type(4)));
    const int lane = xx & 63, wid = xx >> 6, p = lane & 15, g = lane >> 4;
    const int kh0 = g >> 1, pr0 = g & 1;
    const h8s wa0 = *(const h8s*)(stp.w + (size_t)p * 64 + 8 * g);
    const h4s w16 = *(const h4s*)(stp.w + (size_t)p * 64 + 32 + 4 * g);
    float bias4[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) bias4[j] = stp.bias ? stp.bias[4 * g + j] : 0.f;
    const int oh = stp.oh, tiles_x = (oh + 15) >> 4, oy0 = yy0 >> 1;
    int one = 1;  // (two ds_read_b64, not a ds_read2_b64: conv_stem3)
    asm volatile("" : "+v"(one));
    for (int t = wid; t < tiles_x * 8; t += 4) {
      const int tr = t / tiles_x, tx = t - tr * tiles_x;
      const int oy = oy0 + tr;
      if (oy >= oh || 2 * tr + 2 >= nyy) continue;
      const int ox = tx * 16 + p;
      const bool valid = ox < oh;
      const int lx = (valid ? ox : oh - 1) * 2 + 1;
      const uint2* rowk0 = simg + (2 * tr + kh0) * ls;
      const uint2* rowk2 = simg + (2 * tr + 2) * ls;
      const uint2 b00 = rowk0[lx + 2 * pr0], b01 = rowk0[lx + 2 * pr0 + one];
      const h8s bf0 = __builtin_bit_cast(h8s, (u4s{b00.x, b00.y, b01.x, b01.y}));
      const h4s bk = __builtin_bit_cast(h4s, rowk2[lx + g]);
      f4s acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(wa0, bf0, f4s{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
      mfma_opcode_switch();
      acc = __builtin_amdgcn_mfma_f32_16x16x16f16(w16, bk, acc, 0, 0, 0);
      if (valid) {
        // conv_stem3's epilogue with its arguments here (in_scale 1, no activation or affine)
        float v[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float x = acc[j] * 1.f + bias4[j];
          v[j] = x * 1.f + 0.f;
        }
        const _Float16 q0 = (_Float16)v[0], q1 = (_Float16)v[1], q2 = (_Float16)v[2], q3 = (_Float16)v[3];
        _Float16* fp = stp.out + (((size_t)b * oh + oy) * oh + ox) * 16 + 4 * g;
        *(uint2*)fp = make_uint2((uint32_t)__builtin_bit_cast(uint16_t, q0) | ((uint32_t)__builtin_bit_cast(uint16_t, q1) << 16),
                                 (uint32_t)__builtin_bit_cast(uint16_t, q2) | ((uint32_t)__builtin_bit_cast(uint16_t, q3) << 16));
      }
    }
    return;
  }
  if (!col) return;
  if constexpr ((ABL & 2) != 0) {
    (void)lut;
    uint32_t acc = 0;
    for (int i = 0; i < r1 - r0; ++i) acc += himg[i * 256 + xx];
    dst[((size_t)b * out + yy0) * out * 3 + xx] = (T)(float)acc;
    return;
  }
#pragma unroll
  for (int j = 0; j < kRsBand; ++j) {
    if (j < nyy) {
      const int yy = yy0 + j;
      const uint32_t* hp = himg + (bv[2 * yy] - r0) * 256 + xx;
      int a0 = 1 << (kPrecisionBits - 1), a1 = a0, a2 = a0;
#pragma unroll
      for (int t = 0; t < kRsTaps; ++t) {
        const uint32_t hv = hp[t * 256];
        const int k = kv[j * kRsTaps + t];
        a0 += (int)__umul24(hv & 255u, k);
        a1 += (int)__umul24((hv >> 8) & 255u, k);
        a2 += (int)__umul24(hv >> 16, k);
      }
      const int av[3] = {a0, a1, a2};
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const float v = lut[c * 256 + clip8(av[c])];
        if (nchw)
          dst[(((size_t)b * 3 + c) * out + yy) * out + xx] = (T)v;
        else
          dst[(((size_t)b * out + yy) * out + xx) * 3 + c] = (T)v;
      }
    }
  }
}

int resize_stream_mode() { return tune().resize_stream; }

static size_t preprocess_stem_lds(const ResizePlan& p) {
  const size_t lds_rs = (size_t)kRsRing * kRsRowB + (size_t)(p.band_rows17 + kRsTaps) * 256 * 4 +
                        (kRsBand + 1) * kRsTaps * 4 + 3 * 256 * 4;
  const size_t lds_st = (size_t)(kRsBand + 1) * (p.out + 2) * 8;  // the stem image overlays the ring
  return std::max(lds_rs, lds_st);
}

bool preprocess_stem_ok(const ResizePlan& p, const uint8_t* frames, int stem_oh) {
  const int c0b = (p.col_first * 3) & ~15;
  const int col_bytes16 = (int)round_up((int64_t)p.col_end * 3 - c0b, 16);
  return preprocess_stem_lds(p) <= 160 * 1024 && tune().cls_front && tune().stem_k16 && resize_stream_mode() == 1 && p.out <= 255 &&
         (p.in_w * 3) % 16 == 0 && ((uintptr_t)frames & 15) == 0 && c0b + col_bytes16 <= p.in_w * 3 &&
         p.ksize_h <= kRsTaps && p.ksize_v <= kRsTaps && col_bytes16 + 32 <= kRsRowB &&
         (int64_t)p.in_h * p.in_w * 3 < (1ll << 31) && stem_oh == (p.out - 3) / 2 + 1;
}

void launch_preprocess_stem(const ResizePlan& p, const uint8_t* frames, int n, const void* w_stem, const float* bias,
                            void* stem_out, int stem_oh, hipStream_t s) {
  if (n <= 0) return;
  RTDM_REQUIRE(preprocess_stem_ok(p, frames, stem_oh), RTDM_E_INVALID, "preprocess_stem: unsupported geometry");
  const int c0b = (p.col_first * 3) & ~15;
  const int col_bytes16 = (int)round_up((int64_t)p.col_end * 3 - c0b, 16);
  const int v16 = col_bytes16 / 16;
  const size_t lds = preprocess_stem_lds(p);
  const int blocks = n * ((p.out + kRsBand - 1) / kRsBand);
  RsStem st;
  st.w = (const _Float16*)w_stem;
  st.bias = bias;
  st.out = (_Float16*)stem_out;
  st.oh = stem_oh;
  hipLaunchKernelGGL((resize_stream_kernel<_Float16, 0, 2, true>), dim3(blocks), dim3(256), lds, s, frames, p.in_h,
                     p.in_w, p.row_first, p.out, p.ksize_h, p.ksize_v, p.col_first, c0b, v16, p.band_rows17,
                     p.bounds_h.as<int>(), p.coef_h.as<int>(), p.bounds_v.as<int>(), p.coef_v.as<int>(),
                     (_Float16*)nullptr, 0, st);
  RTDM_HIP(hipGetLastError());
}

// LDS of the staged kernel: coefficients + bounds + band source rows + band tmp rows.
static size_t resize_staged_lds(const ResizePlan& p, int col_bytes16) {
  return (size_t)p.out * p.ksize_h * 4 + (size_t)p.out * 2 * 4 + (size_t)p.band_rows8 * col_bytes16 +
         (size_t)p.band_rows8 * p.out * 3;
}

static size_t resize_fused_lds(const ResizePlan& p) {
  return (size_t)p.out * p.ksize_h * 4 + (size_t)p.out * 2 * 4 + (size_t)p.band_rows * p.out * 3;
}

void launch_preprocess(const ResizePlan& p, const uint8_t* frames, int n, uint8_t* tmp, void* out, int out_layout,
                       int dtype, hipStream_t s) {
  if (n <= 0) return;
  // staged path: 16-byte aligned frame rows, band fits the LDS budget
  const int c0b = (p.col_first * 3) & ~15;
  const int col_bytes16 = (int)round_up((int64_t)p.col_end * 3 - c0b, 16);
  const bool rows16 = (p.in_w * 3) % 16 == 0 && ((uintptr_t)frames & 15) == 0 &&
                      c0b + col_bytes16 <= p.in_w * 3;
  const size_t slds = resize_staged_lds(p, col_bytes16);
  if (rows16 && resize_stream_mode() && p.out <= 256 && p.ksize_h <= kRsTaps && p.ksize_v <= kRsTaps &&
      col_bytes16 + 32 <= kRsRowB && (int64_t)p.in_h * p.in_w * 3 < (1ll << 31)) {
    const int v16 = col_bytes16 / 16;
    const size_t lds = (size_t)kRsRing * kRsRowB + (size_t)(p.band_rows + kRsTaps) * 256 * 4 + kRsBand * kRsTaps * 4 +
                       3 * 256 * 4;
    const int blocks = n * ((p.out + kRsBand - 1) / kRsBand);
    const int m = resize_stream_mode();
    if (m > 1 && !(out_layout == 1 || dtype == RTDM_F32)) {  // diagnostic ablations (tools/ab_cls.py)
      // 2..5 ablations; 6: one row per wait + barrier (the pre-r04 loop, A/B)
      auto k = m == 2 ? resize_stream_kernel<_Float16, 1> : m == 3 ? resize_stream_kernel<_Float16, 2>
             : m == 4 ? resize_stream_kernel<_Float16, 4> : m == 6 ? resize_stream_kernel<_Float16, 0, 1>
                                                                  : resize_stream_kernel<_Float16, 7>;
      hipLaunchKernelGGL(k, dim3(blocks), dim3(256), lds, s, frames, p.in_h, p.in_w, p.row_first, p.out, p.ksize_h,
                         p.ksize_v, p.col_first, c0b, v16, p.band_rows, p.bounds_h.as<int>(), p.coef_h.as<int>(),
                         p.bounds_v.as<int>(), p.coef_v.as<int>(), (_Float16*)out, 0, RsStem{});
    } else if (out_layout == 1 || dtype == RTDM_F32)
      hipLaunchKernelGGL((resize_stream_kernel<float, 0>), dim3(blocks), dim3(256), lds, s, frames, p.in_h, p.in_w,
                         p.row_first, p.out, p.ksize_h, p.ksize_v, p.col_first, c0b, v16, p.band_rows, p.bounds_h.as<int>(),
                         p.coef_h.as<int>(), p.bounds_v.as<int>(), p.coef_v.as<int>(), (float*)out,
                         out_layout == 1 ? 1 : 0, RsStem{});
    else
      hipLaunchKernelGGL((resize_stream_kernel<_Float16, 0>), dim3(blocks), dim3(256), lds, s, frames, p.in_h, p.in_w,
                         p.row_first, p.out, p.ksize_h, p.ksize_v, p.col_first, c0b, v16, p.band_rows, p.bounds_h.as<int>(),
                         p.coef_h.as<int>(), p.bounds_v.as<int>(), p.coef_v.as<int>(), (_Float16*)out, 0, RsStem{});
    RTDM_HIP(hipGetLastError());
    return;
  }
  if (rows16 && slds <= 64 * 1024) {
    const int blocks = n * ((p.out + kResizeBandS - 1) / kResizeBandS);
    if (out_layout == 1 || dtype == RTDM_F32)
      hipLaunchKernelGGL(resize_staged_kernel<float>, dim3(blocks), dim3(256), slds, s, frames, p.in_h, p.in_w,
                         p.row_first, p.out, p.ksize_h, p.ksize_v, p.col_first, col_bytes16, p.bounds_h.as<int>(),
                         p.coef_h.as<int>(), p.bounds_v.as<int>(), p.coef_v.as<int>(), (float*)out,
                         out_layout == 1 ? 1 : 0);
    else
      hipLaunchKernelGGL(resize_staged_kernel<_Float16>, dim3(blocks), dim3(256), slds, s, frames, p.in_h, p.in_w,
                         p.row_first, p.out, p.ksize_h, p.ksize_v, p.col_first, col_bytes16, p.bounds_h.as<int>(),
                         p.coef_h.as<int>(), p.bounds_v.as<int>(), p.coef_v.as<int>(), (_Float16*)out, 0);
    RTDM_HIP(hipGetLastError());
    return;
  }
  const size_t lds = resize_fused_lds(p);
  if (lds <= 64 * 1024) {
    const int blocks = n * ((p.out + kResizeBand - 1) / kResizeBand);
    if (out_layout == 1 || dtype == RTDM_F32)
      hipLaunchKernelGGL(resize_fused_kernel<float>, dim3(blocks), dim3(256), lds, s, frames, p.in_h, p.in_w,
                         p.row_first, p.out, p.ksize_h, p.ksize_v, p.bounds_h.as<int>(), p.coef_h.as<int>(),
                         p.bounds_v.as<int>(), p.coef_v.as<int>(), (float*)out, out_layout == 1 ? 1 : 0);
    else
      hipLaunchKernelGGL(resize_fused_kernel<_Float16>, dim3(blocks), dim3(256), lds, s, frames, p.in_h, p.in_w,
                         p.row_first, p.out, p.ksize_h, p.ksize_v, p.bounds_h.as<int>(), p.coef_h.as<int>(),
                         p.bounds_v.as<int>(), p.coef_v.as<int>(), (_Float16*)out, 0);
    RTDM_HIP(hipGetLastError());
    return;
  }
  const int64_t th = (int64_t)n * p.rows * p.out;
  hipLaunchKernelGGL(resize_h_kernel, dim3(grid_for(th, 256)), dim3(256), 0, s, frames, n, p.in_h, p.in_w,
                     p.row_first, p.rows, p.out, p.ksize_h, p.bounds_h.as<int>(), p.coef_h.as<int>(), tmp);
  const int64_t tv = (int64_t)n * p.out * p.out;
  if (out_layout == 1 || dtype == RTDM_F32)
    hipLaunchKernelGGL(resize_v_kernel<float>, dim3(grid_for(tv, 256)), dim3(256), 0, s, tmp, n, p.rows, p.out,
                       p.ksize_v, p.bounds_v.as<int>(), p.coef_v.as<int>(), (float*)out, out_layout == 1 ? 1 : 0);
  else
    hipLaunchKernelGGL(resize_v_kernel<_Float16>, dim3(grid_for(tv, 256)), dim3(256), 0, s, tmp, n, p.rows, p.out,
                       p.ksize_v, p.bounds_v.as<int>(), p.coef_v.as<int>(), (_Float16*)out, 0);
  RTDM_HIP(hipGetLastError());
}

// ------------------------------------------------------------ YOLO decode --
// YOLOLayer inference branch (models.py:252-258) on a raw NCHW head map.
// The anchors travel in the kernel arguments (no staging buffer, no host sync).
__global__ __launch_bounds__(256) void yolo_decode_kernel(const float* __restrict__ p, int n, int na, int no, int ny,
                                                          int nx, AnchorVec anchor_vec, float ystride,
                                                          float* __restrict__ io, int io_rows, int row_off) {
  const int64_t total = (int64_t)n * na * ny * nx * no;
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const int k = (int)(idx % no);
    int64_t q = idx / no;
    const int x = (int)(q % nx);
    q /= nx;
    const int y = (int)(q % ny);
    q /= ny;
    const int a = (int)(q % na);
    const int b = (int)(q / na);
    const float v = p[((((size_t)b * na + a) * no + k) * ny + y) * nx + x];
    float o;
    if (k < 2)
      o = (1.f / (1.f + expf(-v)) + (float)(k == 0 ? x : y)) * ystride;
    else if (k < 4)
      o = (expf(v) * anchor_vec.v[2 * a + (k - 2)]) * ystride;
    else
      o = 1.f / (1.f + expf(-v));
    const size_t row = (size_t)row_off + ((size_t)a * ny + y) * nx + x;
    io[((size_t)b * io_rows + row) * no + k] = o;
  }
}

void launch_yolo_decode(const float* p, int n, int na, int no, int ny, int nx, const AnchorVec& anchor_vec,
                        float ystride, float* io, int io_rows, int row_off, hipStream_t s) {
  const int64_t total = (int64_t)n * na * ny * nx * no;
  if (total <= 0) return;
  hipLaunchKernelGGL(yolo_decode_kernel, dim3(grid_for(total, 256)), dim3(256), 0, s, p, n, na, no, ny, nx,
                     anchor_vec, ystride, io, io_rows, row_off);
  RTDM_HIP(hipGetLastError());
}

// ------------------------------------------------- TensorRT YOLO plugin decode --
// CalDetection / CalDetection_NewCoords (tensorrt_inference/plugins/yolo_layer.cu:
// 203-306): one thread per (image, anchor, cell) -> Detection {x, y, w, h (top-left,
// normalised to the input), det_confidence, class_id, class_confidence}.  class id =
// first maximum raw class logit; sigmoid applied to it (not to each class) and to
// the objectness, which is not multiplied in.
__global__ __launch_bounds__(256) void yolo_trt_kernel(const float* __restrict__ in, int n, TrtYoloArgs t, int nchw,
                                                       float* __restrict__ out) {
  const int64_t total = (int64_t)n * t.rows;
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const int b = (int)(idx / t.rows);
    const int row = (int)(idx - (int64_t)b * t.rows);
    int hk = 0;
    while (hk + 1 < t.n_heads && row >= t.h[hk + 1].row0) ++hk;
    const TrtYoloHead& hd = t.h[hk];
    const int grids = hd.ny * hd.nx;
    const int r = row - hd.row0;
    const int ai = r / grids, cell = r - ai * grids;
    const int gy = cell / hd.nx, gx = cell - gy * hd.nx;
    // field k of this record: row layout (contiguous) or the plugin's NCHW plane
    const float* src;
    int64_t step;
    if (nchw) {
      src = in + ((int64_t)b * hd.na + ai) * t.no * grids + cell;
      step = grids;
    } else {
      src = in + idx * t.no;
      step = 1;
    }
    int cls = 0;
    float best = -INFINITY;
    for (int c = 0; c < t.nc; ++c) {
      const float l = src[(5 + c) * step];
      if (l > best) {
        best = l;
        cls = c;
      }
    }
    const float tx = src[0], ty = src[step], tw = src[2 * step], th = src[3 * step], to = src[4 * step];
    const float sxy = hd.scale_xy, off = (sxy - 1.0f) * 0.5f;
    float bx, by, bw, bh, det_conf, cls_conf;
    if (!hd.new_coords) {
      bx = ((float)gx + (sxy * (1.0f / (1.0f + expf(-tx))) - off)) / (float)hd.nx;
      by = ((float)gy + (sxy * (1.0f / (1.0f + expf(-ty))) - off)) / (float)hd.ny;
      bw = expf(tw) * hd.anchors[2 * ai] / (float)hd.in_w;
      bh = expf(th) * hd.anchors[2 * ai + 1] / (float)hd.in_h;
      det_conf = 1.0f / (1.0f + expf(-to));
      cls_conf = 1.0f / (1.0f + expf(-best));
    } else {  // scaled-YOLOv4 coordinates: the head already applied the sigmoid
      bx = ((float)gx + (sxy * tx - off)) / (float)hd.nx;
      by = ((float)gy + (sxy * ty - off)) / (float)hd.ny;
      bw = tw * tw * 4 * hd.anchors[2 * ai] / (float)hd.in_w;
      bh = th * th * 4 * hd.anchors[2 * ai + 1] / (float)hd.in_h;
      det_conf = to;
      cls_conf = best;
    }
    float* o = out + idx * 7;
    o[0] = bx - bw / 2;
    o[1] = by - bh / 2;
    o[2] = bw;
    o[3] = bh;
    o[4] = det_conf;
    o[5] = (float)cls;
    o[6] = cls_conf;
  }
}

void launch_yolo_trt(const float* in, int n, const TrtYoloArgs& t, int nchw, float* out, hipStream_t s) {
  const int64_t total = (int64_t)n * t.rows;
  if (total <= 0) return;
  hipLaunchKernelGGL(yolo_trt_kernel, dim3(grid_for(total, 256)), dim3(256), 0, s, in, n, t, nchw, out);
  RTDM_HIP(hipGetLastError());
}

// -------------------------------------------------------------------- NMS --
// non_max_suppression (utils.py:488-557, method 'vision_batch') with the
// greedy kernel of torchvision.ops.boxes.nms (CPU: descending score order,
// IoU = inter / (area_i + area_j - inter) in fp32, suppress if IoU > thr with
// the fp32 IoU promoted to double).  One 1024-thread workgroup per image.
//
// Candidate key = (~score_bits << 32) | (anchor * nc + class): ascending key
// order = descending score, ties -> lower (anchor, class) index, which is the
// row-major order of the reference's multi-label expansion (utils.py:524).
static constexpr int kNmsThreads = 1024;
static constexpr int kNmsLdsCap = 4096;
static constexpr int kNmsMaskCap = 512;  // LDS IoU-bitmask path: n * ceil(n/64) * 8 B <= 32 KiB
static constexpr int kNmsMaskCapG = 2048;  // workspace bitmask, scanned through LDS in chunks
static constexpr int kNmsRankCap = 2048;   // rank sort up to this many candidates

struct NmsWs {  // per-image slice of the workspace
  uint64_t* keys;
  float4* box;
  float* area;
  uint32_t* supp;
  int* keep;
  uint64_t* seg;  // candidate keys of anchor block k at seg + k * kNmsCandBlk * npa
  int* segcnt;    // [n_anchors / kNmsCandBlk] candidates per anchor block
  uint64_t* mask; // IoU bitmask [m][m/64], m = min(cap, kNmsMaskCapG)
};

// Candidate pass: one kNmsCandBlk-thread block per (image, anchor block).
static constexpr int kNmsCandBlk = 256;

static inline size_t nms_cap(int n_anchors, int nc) {
  size_t c = 1;
  while (c < (size_t)n_anchors * (size_t)(nc > 1 ? nc : 1)) c <<= 1;
  return c < 64 ? 64 : c;
}

__host__ __device__ inline int nms_nblk(int n_anchors) { return (n_anchors + kNmsCandBlk - 1) / kNmsCandBlk; }

__host__ __device__ inline size_t nms_per_image(size_t cap, int n_anchors, int nc) {
  const size_t npa = nc > 1 ? nc : 1;
  const size_t m = cap < (size_t)kNmsMaskCapG ? cap : (size_t)kNmsMaskCapG;
  return cap * (8 + 16 + 4 + 4) + (cap / 32 + 1) * 4 + 256 +
         round_up((int64_t)nms_nblk(n_anchors) * (kNmsCandBlk * npa * 8 + 4), 256) + m * (m / 64) * 8;
}

size_t nms_workspace_size(int n, int n_anchors, int nc) {
  return nms_per_image(nms_cap(n_anchors, nc), n_anchors, nc) * (size_t)n;
}

__device__ __forceinline__ NmsWs nms_ws(void* ws, int img, size_t cap, int n_anchors, int nc) {
  char* base = (char*)ws + nms_per_image(cap, n_anchors, nc) * img;
  NmsWs w;
  w.keys = (uint64_t*)base;
  w.box = (float4*)(base + cap * 8);
  w.area = (float*)(base + cap * 24);
  w.keep = (int*)(base + cap * 28);
  w.supp = (uint32_t*)(base + cap * 32);
  char* sb = base + cap * 32 + (cap / 32 + 1) * 4 + 256;
  w.seg = (uint64_t*)sb;
  w.segcnt = (int*)(sb + (size_t)nms_nblk(n_anchors) * kNmsCandBlk * (nc > 1 ? nc : 1) * 8);
  w.mask = (uint64_t*)(sb + round_up((int64_t)nms_nblk(n_anchors) * (kNmsCandBlk * (nc > 1 ? nc : 1) * 8 + 4), 256));
  return w;
}

// classes filter (utils.py:539-540): bit c of the mask; ~0 = every class (also the only
// mask accepted for nc > 64, checked in rtdm_nms)
__device__ __forceinline__ bool nms_class_ok(uint64_t class_mask, int c) {
  return class_mask == ~0ull || (c < 64 && ((class_mask >> c) & 1ull));
}

// 1. candidates (utils.py:505-536), spread over the whole chip: each block filters
// kNmsCandBlk anchors of one image and writes its keys to its own segment (+ count).
__global__ __launch_bounds__(kNmsCandBlk) void nms_cand_kernel(const float* __restrict__ io, int n_anchors, int no,
                                                               float conf, int multi_label, uint64_t class_mask,
                                                               void* ws, size_t cap) {
  __shared__ int s_n;
  const int img = blockIdx.y, blk = blockIdx.x, tid = threadIdx.x;
  const int nc = no - 5;
  const bool ml = multi_label && nc > 1;
  const int npa = nc > 1 ? nc : 1;
  NmsWs g = nms_ws(ws, img, cap, n_anchors, nc);
  uint64_t* seg = g.seg + (size_t)blk * kNmsCandBlk * npa;
  if (tid == 0) s_n = 0;
  __syncthreads();
  const int a = blk * kNmsCandBlk + tid;
  if (a < n_anchors) {
    const float* r = io + ((size_t)img * n_anchors + a) * no;
    const float obj = r[4];
    const float w = r[2], h = r[3];
    if ((obj > conf) && (w > 2.f) && (h > 2.f) && (w < 4096.f) && (h < 4096.f)) {
      const float x = r[0], y = r[1];
      const float hw = w / 2.f, hh = h / 2.f;
      const bool box_finite = isfinite(x - hw) && isfinite(y - hh) && isfinite(x + hw) && isfinite(y + hh);
      if (ml) {
        for (int j = 0; j < nc; ++j) {
          const float sc = r[5 + j] * obj;
          if (!(sc > conf)) continue;
          if (!nms_class_ok(class_mask, j)) continue;
          if (!box_finite || !isfinite(sc)) continue;
          seg[atomicAdd(&s_n, 1)] = ((uint64_t)(~__float_as_uint(sc)) << 32) | (uint32_t)(a * nc + j);
        }
      } else {
        float best = r[5] * obj;
        int bj = 0;
        for (int j = 1; j < nc; ++j) {
          const float sc = r[5 + j] * obj;
          if (sc > best) { best = sc; bj = j; }
        }
        if (nms_class_ok(class_mask, bj) && box_finite && isfinite(best))
          seg[atomicAdd(&s_n, 1)] = ((uint64_t)(~__float_as_uint(best)) << 32) | (uint32_t)(a * npa + bj);
      }
    }
  }
  __syncthreads();
  if (tid == 0) g.segcnt[blk] = s_n;
}

// OR of v over the 64 lanes of a full wave, as a wave-uniform value: rotations inside each
// 16-lane row (DPP row_ror 1 / 2 / 4 / 8) and the four rows' lane 0.  The __shfl_xor butterfly
// it replaces compiled to six dependent ds_bpermute_b32 per 32-bit half, an LDS round trip
// each, on the greedy scan's serial path.
__device__ __forceinline__ uint32_t wave_or_u32(uint32_t v) {
  v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x121, 0xf, 0xf, false);
  v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x122, 0xf, 0xf, false);
  v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x124, 0xf, 0xf, false);
  v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x128, 0xf, 0xf, false);
  return (uint32_t)__builtin_amdgcn_readlane((int)v, 0) | (uint32_t)__builtin_amdgcn_readlane((int)v, 16) |
         (uint32_t)__builtin_amdgcn_readlane((int)v, 32) | (uint32_t)__builtin_amdgcn_readlane((int)v, 48);
}

// v of lane (lane ^ J) for the bitonic stages inside a wave (lane = i & 63): J = 1, 2 one DPP
// quad permutation, J = 4, 8 a DPP row shift each way and a select (no LDS round trip),
// J = 16, 32 ds_bpermute (__shfl_xor)
template <int J>
__device__ __forceinline__ uint32_t lane_xor_u32(uint32_t v, int i) {
  if constexpr (J == 1) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xf, 0xf, false);  // quad_perm [1,0,3,2]
  } else if constexpr (J == 2) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xf, 0xf, false);  // quad_perm [2,3,0,1]
  } else if constexpr (J == 4 || J == 8) {
    const uint32_t up = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x100 + J, 0xf, 0xf, false);  // row_shl: lane + J
    const uint32_t dn = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x110 + J, 0xf, 0xf, false);  // row_shr: lane - J
    return (i & J) ? dn : up;
  } else {
    return (uint32_t)__shfl_xor((int)v, J);
  }
}

template <int J>
__device__ __forceinline__ uint64_t lane_xor_u64(uint64_t v, int i) {
  return ((uint64_t)lane_xor_u32<J>((uint32_t)(v >> 32), i) << 32) | lane_xor_u32<J>((uint32_t)v, i);
}

// 64-bit readlane (the builtin returns a signed int: widen it as unsigned)
__device__ __forceinline__ uint64_t readlane_u64(uint64_t v, int lane) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, lane);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), lane);
  return ((uint64_t)hi << 32) | lo;
}

// The greedy scan of an n <= kNmsMaskCap candidate bitmask (row i's word w at
// mask[i * W + w], columns j > i only), by one full wave (lane = tid < 64): lane b holds every
// mask word of row 64c + b in registers while word block c is scanned; the kept rows' masks
// reach the later words through one wave-wide OR per word.  Writes the kept rows to keep[] in score order and
// returns their count (wave-uniform).
template <typename MaskT>
__device__ __forceinline__ int nms_scan_wave(const MaskT* mask, int n, int W, int lane, int* __restrict__ keep) {
  int nk = 0;
  uint64_t removed[kNmsMaskCap / 64];
#pragma unroll
  for (int w = 0; w < kNmsMaskCap / 64; ++w) removed[w] = 0;
#pragma unroll
  for (int c = 0; c < kNmsMaskCap / 64; ++c) {
    if (c < W) {
      const int cnt = n - 64 * c < 64 ? n - 64 * c : 64;
      const int i = 64 * c + lane;
      uint64_t mrow[kNmsMaskCap / 64];
#pragma unroll
      for (int w = 0; w < kNmsMaskCap / 64; ++w) mrow[w] = (w >= c && w < W && lane < cnt) ? mask[(size_t)i * W + w] : 0ull;
      const uint64_t valid = cnt == 64 ? ~0ull : ((1ull << cnt) - 1ull);
      // The in-word greedy pass, wave-parallel.  sup (lane b): the rows a < b of this word
      // whose IoU with b is over the threshold -- the word's bit-matrix transposed, built from
      // the rows with any in-word bit only (usually few).  Then rounds over the undecided set
      // U: b is kept once none of its suppressors is kept or undecided, removed once one is
      // kept; the lowest undecided candidate is always decided, and the result is the serial
      // greedy's (each decision depends only on the decisions below it).
      uint64_t sup = 0;
      for (uint64_t nz = __builtin_amdgcn_ballot_w64(mrow[c] != 0ull); nz; nz &= nz - 1) {
        const int a = __builtin_ctzll(nz);
        sup |= ((readlane_u64(mrow[c], a) >> lane) & 1ull) << a;
      }
      uint64_t kept = 0;
      uint64_t und = valid & ~removed[c];
      while (und) {
        const bool in = (und >> lane) & 1ull;
        const uint64_t kk = __builtin_amdgcn_ballot_w64(in && (sup & (kept | und)) == 0ull);
        kept |= kk;
        const uint64_t rr = __builtin_amdgcn_ballot_w64(in && !((kk >> lane) & 1ull) && (sup & kept) != 0ull);
        und &= ~(kk | rr);
      }
      if ((kept >> lane) & 1ull) keep[nk + __popcll(kept & ((1ull << lane) - 1ull))] = i;
      nk += __popcll(kept);
      const bool mine = (kept >> lane) & 1ull;
#pragma unroll
      for (int w = c + 1; w < kNmsMaskCap / 64; ++w) {
        if (w < W) {
          const uint32_t lo = mine ? (uint32_t)mrow[w] : 0u, hi = mine ? (uint32_t)(mrow[w] >> 32) : 0u;
          removed[w] |= ((uint64_t)wave_or_u32(hi) << 32) | wave_or_u32(lo);
        }
      }
    }
  }
  return nk;
}

// 5. rows [x1,y1,x2,y2,conf,cls] in kept (descending score) order (utils.py:553-557)
__device__ __forceinline__ void nms_emit(const float* __restrict__ P, int no, int cls_div, const uint64_t* K,
                                         const int* __restrict__ keep, int nkeep, int max_det, int img, int tid,
                                         int nthreads, float* __restrict__ det, int32_t* __restrict__ idx_out,
                                         int32_t* __restrict__ count) {
  const int nout = nkeep < max_det ? nkeep : max_det;
  for (int r = tid; r < nout; r += nthreads) {
    const int i = keep[r];
    const uint64_t key = K[i];
    const uint32_t cand = (uint32_t)key;
    const int a = cand / cls_div, j = cand - (cand / cls_div) * cls_div;
    const float* rr = P + (size_t)a * no;
    const float x = rr[0], y = rr[1], w = rr[2], h = rr[3];
    float* d = det + ((size_t)img * max_det + r) * 6;
    d[0] = x - w / 2.f;
    d[1] = y - h / 2.f;
    d[2] = x + w / 2.f;
    d[3] = y + h / 2.f;
    d[4] = __uint_as_float(~(uint32_t)(key >> 32));
    d[5] = (float)j;
    if (idx_out) {
      idx_out[((size_t)img * max_det + r) * 2 + 0] = a;
      idx_out[((size_t)img * max_det + r) * 2 + 1] = j;
    }
  }
  if (tid == 0) count[img] = nkeep;
}

// split mode: the per-image candidate count the prep launch leaves for the mask / scan
// launches (-1: the prep launch finished the image itself), in the slice's slack bytes
__device__ __forceinline__ int* nms_split_n(const NmsWs& g, size_t cap) {
  return (int*)((char*)g.supp + (cap / 32 + 1) * 4 + 128);
}

__global__ __launch_bounds__(kNmsThreads) void nms_kernel(const float* __restrict__ io, int n_anchors, int no,
                                                          float conf, double iou_thr, int multi_label, int agnostic,
                                                          uint64_t class_mask, int max_det, void* ws, size_t cap,
                                                          float* __restrict__ det, int32_t* __restrict__ idx_out,
                                                          int32_t* __restrict__ count, int variant, int split) {
#pragma clang fp contract(off)
  __shared__ uint64_t s_keys[kNmsLdsCap];
  __shared__ float4 s_box[kNmsLdsCap];
  __shared__ float s_area[kNmsLdsCap];
  __shared__ uint32_t s_supp[kNmsLdsCap / 32];
  __shared__ uint64_t s_mask[kNmsMaskCap * (kNmsMaskCap / 64)];
  __shared__ int s_n;
  const int img = blockIdx.x;
  const int tid = threadIdx.x;
  const int nc = no - 5;
  const float* P = io + (size_t)img * n_anchors * no;
  NmsWs g = nms_ws(ws, img, cap, n_anchors, nc);
  // phase timestamps (100 MHz s_memrealtime) in the slice's slack bytes: diagnostics
  // for tools/nms_phases.py only (variant bit 2, rtdm_set_tuning("nms_variant", 4))
  uint64_t* stamps = (uint64_t*)((char*)g.supp + (cap / 32 + 1) * 4);
#define NMS_STAMP(k) \
  if ((variant & 4) && tid == 0) stamps[k] = __builtin_amdgcn_s_memrealtime()
  NMS_STAMP(0);
  __shared__ int s_off[kNmsThreads + 1];  // candidate offset of each anchor block (nms_cand_kernel)
  __shared__ int s_wsum[kNmsThreads / 64];

  // 1b. gather the anchor blocks' candidate segments (any order: the sort decides)
  const int nblk = nms_nblk(n_anchors);
  const int npa = nc > 1 ? nc : 1;
  int n = 0;
  for (int b0 = 0; b0 < nblk; b0 += kNmsThreads) {
    const int nb = nblk - b0 < kNmsThreads ? nblk - b0 : kNmsThreads;
    {  // exclusive offsets: wave-level inclusive scans + a scan of the 16 wave totals
      int v = tid < nb ? g.segcnt[b0 + tid] : 0;
      const int lane = tid & 63, wv = tid >> 6;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const int u = __shfl_up(v, d);
        if (lane >= d) v += u;
      }
      if (lane == 63) s_wsum[wv] = v;
      __syncthreads();
      if (tid == 0) {
        int acc = 0;
        for (int k = 0; k < kNmsThreads / 64; ++k) {
          const int t = s_wsum[k];
          s_wsum[k] = acc;
          acc += t;
        }
      }
      __syncthreads();
      s_off[tid + 1] = v + s_wsum[wv];
      if (tid == 0) s_off[0] = 0;
      __syncthreads();
    }
    const int tot = s_off[nb];
    const bool lds_keys = n + tot <= kNmsLdsCap;  // uniform
    for (int i = tid; i < tot; i += kNmsThreads) {
      int lo = 0, hi = nb - 1;  // segment k with s_off[k] <= i < s_off[k+1]
      while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (s_off[mid] <= i) lo = mid; else hi = mid - 1;
      }
      const uint64_t key = g.seg[(size_t)(b0 + lo) * kNmsCandBlk * npa + (i - s_off[lo])];
      g.keys[n + i] = key;
      if (lds_keys) s_keys[n + i] = key;
    }
    n += tot;
    __syncthreads();
  }
  NMS_STAMP(1);
  int npow = 1;
  while (npow < n) npow <<= 1;
  const bool lds = npow <= kNmsLdsCap;
  // Phases 2-5 are instantiated once with the LDS arrays and once with the workspace: a
  // pointer selected at run time between the two loses its address space, and every key,
  // box and mask access of the common (LDS) case became a flat instruction.
  auto phases = [&](auto lds_tag, uint64_t* K, float4* B, float* A, uint32_t* S) {
  for (int i = n + tid; i < npow; i += kNmsThreads) K[i] = ~0ull;  // sort padding
  __syncthreads();

  // 2. sort, ascending key: bitonic network (diagnostic variant bit 0: rank sort —
  // keys are unique, a key's rank = count of smaller keys; measured slower here).
  if (n <= kNmsRankCap && (variant & 1)) {
    uint64_t mine[kNmsRankCap / kNmsThreads];
    int rk[kNmsRankCap / kNmsThreads];
#pragma unroll
    for (int q = 0; q < kNmsRankCap / kNmsThreads; ++q) {
      const int i = tid + q * kNmsThreads;
      mine[q] = i < n ? K[i] : ~0ull;
      rk[q] = 0;
    }
    // 8 broadcast reads in flight per step (the loop is LDS-latency bound)
    int j = 0;
    for (; j + 8 <= n; j += 8) {
      uint64_t kj[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) kj[u] = K[j + u];
#pragma unroll
      for (int u = 0; u < 8; ++u)
#pragma unroll
        for (int q = 0; q < kNmsRankCap / kNmsThreads; ++q) rk[q] += kj[u] < mine[q] ? 1 : 0;
    }
    for (; j < n; ++j) {
      const uint64_t kj = K[j];
#pragma unroll
      for (int q = 0; q < kNmsRankCap / kNmsThreads; ++q) rk[q] += kj < mine[q] ? 1 : 0;
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < kNmsRankCap / kNmsThreads; ++q)
      if (tid + q * kNmsThreads < n) K[rk[q]] = mine[q];
    __syncthreads();
  } else {
  // bitonic network.  LDS keys (npow <= kNmsLdsCap): a thread keeps its keys in registers and
  // every stage of partner distance j < 64 runs inside the wave on lane shuffles with no
  // barrier; only the stages j >= 64 go through LDS, a barrier each (npow 512: 15 barriers,
  // not 45).  Keys are unique, so any correct sort yields the same order.
  auto cx_lds = [&](int k, int j) {
    for (int i = tid; i < npow; i += kNmsThreads) {
      const int ixj = i ^ j;
      if (ixj > i) {
        const uint64_t a = K[i], b = K[ixj];
        const bool up = (i & k) == 0;
        if ((a > b) == up) {
          K[i] = b;
          K[ixj] = a;
        }
      }
    }
    __syncthreads();
  };
  if constexpr (decltype(lds_tag)::value) {
    constexpr int EPT = kNmsLdsCap / kNmsThreads;
    uint64_t v[EPT];
#pragma unroll
    for (int m = 0; m < EPT; ++m) {
      const int i = tid + m * kNmsThreads;
      v[m] = i < npow ? K[i] : ~0ull;
    }
    for (int k = 2; k <= npow; k <<= 1) {
      if (k > 64) {
#pragma unroll
        for (int m = 0; m < EPT; ++m)
          if (tid + m * kNmsThreads < npow) K[tid + m * kNmsThreads] = v[m];
        __syncthreads();
        for (int j = k >> 1; j >= 64; j >>= 1) cx_lds(k, j);
#pragma unroll
        for (int m = 0; m < EPT; ++m)
          if (tid + m * kNmsThreads < npow) v[m] = K[tid + m * kNmsThreads];
      }
      const int j0 = (k >> 1) < 32 ? (k >> 1) : 32;
#pragma unroll
      for (int m = 0; m < EPT; ++m) {
        if (m * kNmsThreads + (tid & ~63) >= npow) continue;  // wave-uniform: no key of this wave
        const int i = tid + m * kNmsThreads;
        const bool up = (i & k) == 0;
        auto stage = [&](auto jc) {
          constexpr int j = decltype(jc)::value;
          const uint64_t p = lane_xor_u64<j>(v[m], i);
          const bool take_min = ((i & j) == 0) == up;  // the pair's lower index keeps min iff ascending
          v[m] = take_min ? (p < v[m] ? p : v[m]) : (p > v[m] ? p : v[m]);
        };
        if (j0 >= 32) stage(std::integral_constant<int, 32>{});
        if (j0 >= 16) stage(std::integral_constant<int, 16>{});
        if (j0 >= 8) stage(std::integral_constant<int, 8>{});
        if (j0 >= 4) stage(std::integral_constant<int, 4>{});
        if (j0 >= 2) stage(std::integral_constant<int, 2>{});
        stage(std::integral_constant<int, 1>{});
      }
    }
    __syncthreads();  // every wave's last LDS-stage reads are done before the write-back
#pragma unroll
    for (int m = 0; m < EPT; ++m)
      if (tid + m * kNmsThreads < npow) K[tid + m * kNmsThreads] = v[m];
    __syncthreads();
  } else {
    for (int k = 2; k <= npow; k <<= 1)
      for (int j = k >> 1; j > 0; j >>= 1) cx_lds(k, j);
  }
  }

  NMS_STAMP(2);
  // 3. offset boxes + areas (utils.py:547-552; torchvision areas)
  const int cls_div = nc > 1 ? nc : 1;
  for (int i = tid; i < n; i += kNmsThreads) {
    const uint32_t cand = (uint32_t)K[i];
    const int a = cand / cls_div, j = cand - (cand / cls_div) * cls_div;
    const float* r = P + (size_t)a * no;
    const float x = r[0], y = r[1], w = r[2], h = r[3];
    const float off = agnostic ? 0.f : (float)j * 4096.f;
    float4 bx;
    bx.x = (x - w / 2.f) + off;
    bx.y = (y - h / 2.f) + off;
    bx.z = (x + w / 2.f) + off;
    bx.w = (y + h / 2.f) + off;
    B[i] = bx;
    A[i] = (bx.z - bx.x) * (bx.w - bx.y);
  }
  for (int i = tid; i < (n + 31) / 32; i += kNmsThreads) S[i] = 0u;
  __syncthreads();

  if (split) {
    // split mode: an image whose bitmask fits the register scan hands its sorted keys,
    // boxes and areas to nms_mask_kernel / nms_scan_kernel; larger ones finish here
    if (decltype(lds_tag)::value && n <= kNmsMaskCap && !(variant & 2)) {
      for (int i = tid; i < n; i += kNmsThreads) {
        g.keys[i] = K[i];
        g.box[i] = B[i];
        g.area[i] = A[i];
      }
      if (tid == 0) *nms_split_n(g, cap) = n;
      return;
    }
    if (tid == 0) *nms_split_n(g, cap) = -1;
  }

  NMS_STAMP(3);
  // 4. greedy suppression.
  // n <= kNmsMaskCap: the torchvision-CUDA formulation — every (i, 64-column
  // word) IoU bitmask in parallel into LDS, then one wave scans candidates in
  // score order, OR-ing the masks of kept boxes (no workgroup barrier per
  // candidate).  Same IoU arithmetic and the same keep set as the greedy loop.
  // kNmsMaskCap < n <= kNmsMaskCapG: the same bitmask in the workspace, scanned in
  // chunks of rows staged through the LDS mask buffer.
  int nkeep = 0;
  if (n <= ((variant & 2) ? -1 : kNmsMaskCapG)) {
    const int W = (n + 63) >> 6;
    const bool in_lds = n <= kNmsMaskCap;
    // one (row i, 16-column quarter q of word w) per thread, rows fastest: the lanes of a
    // wave share (w, q), so each B[j] / A[j] read is one broadcast LDS address, and a
    // quarter word gives every wave of the block work at the typical n of 100-300
    // (LDS path: quarters ORed into the zeroed word; workspace path: whole words); the
    // division only where boxes meet
    const bool thr_nonneg = iou_thr >= 0.0;
    const int QS = in_lds ? 4 : 1, QW = 64 / QS;
    if (in_lds) {
      for (int p = tid; p < n * W; p += kNmsThreads) s_mask[p] = 0ull;
      __syncthreads();
    }
    auto build = [&](auto in_lds_tag, uint64_t* M) {
    for (int p = tid; p < n * W * QS; p += kNmsThreads) {
      const int r = p / n, i = p - r * n;
      const int w = r / QS, q = r - w * QS;
      const float4 bi = B[i];
      const float ai = A[i];
      uint64_t bits = 0;
      const int jw = w * 64, j0 = jw + q * QW;
      const int j1 = j0 + QW < n ? j0 + QW : n;
      // four columns per step with their box / area reads issued together (one LDS
      // latency per four IoUs; the per-column loop waited on each read behind the previous
      // column's divergent division branch)
      for (int jb = j0 > i + 1 ? j0 : i + 1; jb < j1; jb += 4) {
        float4 bq[4];
        float aq[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int j = jb + u < j1 ? jb + u : j1 - 1;
          bq[u] = B[j];
          aq[u] = A[j];
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const float4 bj = bq[u];
          const float xx1 = fmaxf(bi.x, bj.x);
          const float yy1 = fmaxf(bi.y, bj.y);
          const float xx2 = fminf(bi.z, bj.z);
          const float yy2 = fminf(bi.w, bj.w);
          const float w2 = fmaxf(0.f, xx2 - xx1);
          const float h2 = fmaxf(0.f, yy2 - yy1);
          const float inter = w2 * h2;
          if (jb + u < j1 && (inter > 0.f || !thr_nonneg)) {  // inter == 0: IoU 0 is never > a threshold >= 0
            const float ovr = inter / ((ai + aq[u]) - inter);
            if ((double)ovr > iou_thr) bits |= 1ull << (jb + u - jw);
          }
        }
      }
      if constexpr (decltype(in_lds_tag)::value) {
        if (bits) atomicOr((unsigned long long*)&M[(size_t)i * W + w], (unsigned long long)bits);
      } else {
        M[(size_t)i * W + w] = bits;
      }
    }
    };
    if (in_lds) build(std::true_type{}, s_mask);
    else build(std::false_type{}, g.mask);
    __syncthreads();
    NMS_STAMP(4);
    int nk = 0;
    if (in_lds) {
      if (tid < 64) nk = nms_scan_wave(s_mask, n, W, tid, g.keep);
    } else {
      // kMaskCap < n <= kNmsMaskCapG: the bitmask in the workspace, scanned in chunks of
      // whole 64-candidate words staged through the LDS mask buffer
      const int rows = ((kNmsMaskCap * (kNmsMaskCap / 64)) / W) & ~63;
      uint64_t removed = 0;  // wave 0: lane l < W holds word l of the suppressed set
      for (int c0 = 0; c0 < n; c0 += rows) {
        const int c1 = c0 + rows < n ? c0 + rows : n;
        for (int p = tid; p < (c1 - c0) * W; p += kNmsThreads) s_mask[p] = g.mask[(size_t)c0 * W + p];
        __syncthreads();
        if (tid < 64) {
          // word by word: the in-word greedy pass on scalars (lane b holds row 64w+b's
          // bits of word w), then every kept row's mask ORed into the later words
          for (int w = c0 >> 6; w * 64 < c1; ++w) {
            const int cnt = c1 - w * 64 < 64 ? c1 - w * 64 : 64;
            const int i = w * 64 + tid;
            const uint64_t mw = tid < cnt ? s_mask[(i - c0) * W + w] : 0ull;
            uint64_t rem = readlane_u64(removed, w);
            uint64_t kept = 0;
            for (int b = 0; b < cnt; ++b) {
              if ((rem >> b) & 1ull) continue;
              kept |= 1ull << b;
              rem |= readlane_u64(mw, b);
            }
            if ((kept >> tid) & 1ull) g.keep[nk + __popcll(kept & ((1ull << tid) - 1ull))] = i;
            nk += __popcll(kept);
            // kept rows' masks into the later words, 8 rows (LDS reads) in flight per step
            const int tl = tid < W ? tid : W - 1;
            for (uint64_t k = kept; k;) {
              int bs[8];
#pragma unroll
              for (int u = 0; u < 8; ++u) {
                bs[u] = k ? __builtin_ctzll(k) : -1;
                k &= k - 1;
              }
              uint64_t v[8];
#pragma unroll
              for (int u = 0; u < 8; ++u) v[u] = s_mask[(w * 64 + (bs[u] < 0 ? bs[0] : bs[u]) - c0) * W + tl];
#pragma unroll
              for (int u = 0; u < 8; ++u) removed |= bs[u] >= 0 ? v[u] : 0ull;
            }
          }
        }
        __syncthreads();  // the chunk's LDS rows are consumed before the next chunk lands
      }
    }
    if (tid == 0) s_n = nk;
    __syncthreads();
    nkeep = s_n;
  } else {
    for (int i = 0; i < n; ++i) {
      if ((S[i >> 5] >> (i & 31)) & 1u) continue;
      if (tid == 0) g.keep[nkeep] = i;
      ++nkeep;
      const float4 bi = B[i];
      const float ai = A[i];
      for (int j = i + 1 + tid; j < n; j += kNmsThreads) {
        if ((S[j >> 5] >> (j & 31)) & 1u) continue;
        const float4 bj = B[j];
        const float xx1 = fmaxf(bi.x, bj.x);
        const float yy1 = fmaxf(bi.y, bj.y);
        const float xx2 = fminf(bi.z, bj.z);
        const float yy2 = fminf(bi.w, bj.w);
        const float w = fmaxf(0.f, xx2 - xx1);
        const float h = fmaxf(0.f, yy2 - yy1);
        const float inter = w * h;
        const float ovr = inter / ((ai + A[j]) - inter);
        if ((double)ovr > iou_thr) atomicOr(&S[j >> 5], 1u << (j & 31));
      }
      __syncthreads();
    }
  }
  __syncthreads();  // g.keep written by wave 0 / thread 0 -> read by all below

  NMS_STAMP(5);
  nms_emit(P, no, cls_div, K, g.keep, nkeep, max_det, img, tid, kNmsThreads, det, idx_out, count);
  };
  if (lds) phases(std::true_type{}, s_keys, s_box, s_area, s_supp);
  else phases(std::false_type{}, g.keys, g.box, g.area, g.supp);
  NMS_STAMP(6);
#undef NMS_STAMP
}

// Split mode, launch 2: the IoU bitmask of every image the prep launch handed over, one
// 256-thread block per (64-column word w, 64-row block r <= w, image; a triangular grid): lane = row, wave =
// 16-column quarter of the word (broadcast column reads), quarters ORed through LDS.  Same
// IoU arithmetic as nms_kernel's mask, so the same bits; the worst image's mask spreads over
// up to 36 blocks instead of one.
__global__ __launch_bounds__(256) void nms_mask_kernel(int n_anchors, int nc, double iou_thr, void* ws, size_t cap) {
#pragma clang fp contract(off)
  __shared__ float4 s_b[64];
  __shared__ float s_a[64];
  __shared__ uint64_t s_part[4][64];
  // blockIdx.x enumerates the (w, r <= w) pairs row by row: t = w (w + 1) / 2 + r
  const int t = blockIdx.x, img = blockIdx.y, tid = threadIdx.x;
  int w = 0;
  while ((w + 1) * (w + 2) / 2 <= t) ++w;
  const int r = t - w * (w + 1) / 2;
  NmsWs g = nms_ws(ws, img, cap, n_anchors, nc);
  const int n = *nms_split_n(g, cap);
  if (n < 0 || 64 * w >= n) return;
  const int W = (n + 63) >> 6, jw = 64 * w, j1 = n < jw + 64 ? n : jw + 64;
  if (tid < j1 - jw) {
    s_b[tid] = g.box[jw + tid];
    s_a[tid] = g.area[jw + tid];
  }
  __syncthreads();
  const int lane = tid & 63, q = tid >> 6;
  const int i = 64 * r + lane;
  const bool thr_nonneg = iou_thr >= 0.0;
  uint64_t bits = 0;
  if (i < n) {
    const float4 bi = g.box[i];
    const float ai = g.area[i];
    const int c0 = jw + 16 * q, c1 = c0 + 16 < j1 ? c0 + 16 : j1;
    for (int j = c0 > i + 1 ? c0 : i + 1; j < c1; ++j) {
      const float4 bj = s_b[j - jw];
      const float xx1 = fmaxf(bi.x, bj.x);
      const float yy1 = fmaxf(bi.y, bj.y);
      const float xx2 = fminf(bi.z, bj.z);
      const float yy2 = fminf(bi.w, bj.w);
      const float w2 = fmaxf(0.f, xx2 - xx1);
      const float h2 = fmaxf(0.f, yy2 - yy1);
      const float inter = w2 * h2;
      if (inter > 0.f || !thr_nonneg) {  // inter == 0: IoU 0 is never > a threshold >= 0
        const float ovr = inter / ((ai + s_a[j - jw]) - inter);
        if ((double)ovr > iou_thr) bits |= 1ull << (j - jw);
      }
    }
  }
  s_part[q][lane] = bits;
  __syncthreads();
  if (q == 0 && i < n) g.mask[(size_t)i * W + w] = s_part[0][lane] | s_part[1][lane] | s_part[2][lane] | s_part[3][lane];
}

// Split mode, launch 3: the greedy scan (one wave) and the output rows of every image the prep
// launch handed over.
__global__ __launch_bounds__(256) void nms_scan_kernel(const float* __restrict__ io, int n_anchors, int no,
                                                       int max_det, void* ws, size_t cap, float* __restrict__ det,
                                                       int32_t* __restrict__ idx_out, int32_t* __restrict__ count) {
  __shared__ int s_n;
  __shared__ uint64_t s_mask[kNmsMaskCap * (kNmsMaskCap / 64)];
  __shared__ uint64_t s_key[kNmsMaskCap];
  __shared__ int s_keep[kNmsMaskCap];
  const int img = blockIdx.x, tid = threadIdx.x;
  const int nc = no - 5;
  NmsWs g = nms_ws(ws, img, cap, n_anchors, nc);
  const int n = *nms_split_n(g, cap);
  if (n < 0) return;
  const int W = (n + 63) >> 6;
  // the bitmask and the sorted keys into LDS by the whole block first, and the kept list kept
  // there: the launch is a chain of dependent memory round trips (count -> mask -> scan ->
  // kept rows -> keys -> io rows -> det), each global one ~1-2 us
  for (int i = tid; i < n; i += 256) {
    s_key[i] = g.keys[i];
    for (int w = i >> 6; w < W; ++w) s_mask[i * W + w] = g.mask[(size_t)i * W + w];  // (words left of the row's block: never read)
  }
  __syncthreads();
  if (tid < 64) {
    const int nk = nms_scan_wave(s_mask, n, W, tid, s_keep);
    if (tid == 0) s_n = nk;
  }
  __syncthreads();  // s_keep written by wave 0 -> read by all below
  nms_emit(io + (size_t)img * n_anchors * no, no, nc > 1 ? nc : 1, s_key, s_keep, s_n, max_det, img, tid, 256, det,
           idx_out, count);
}

void launch_nms(const float* io, int n, int n_anchors, int no, float conf, double iou, int multi_label, int agnostic,
                uint64_t class_mask, int max_det, void* ws, float* det, int32_t* idx, int32_t* count,
                hipStream_t s) {
  if (n <= 0) return;
  RTDM_REQUIRE(no >= 6, RTDM_E_INVALID, "nms: no must be >= 6 (5 + nc)");
  RTDM_REQUIRE(max_det >= 0, RTDM_E_INVALID, "nms: max_det < 0");
  const size_t cap = nms_cap(n_anchors, no - 5);
  hipLaunchKernelGGL(nms_cand_kernel, dim3(nms_nblk(n_anchors), n), dim3(kNmsCandBlk), 0, s, io, n_anchors, no, conf,
                     multi_label, class_mask, ws, cap);
  // split (default): images of <= kNmsMaskCap candidates take their IoU bitmask over many
  // blocks (nms_mask_kernel) and their scan in a third launch; 0 = one launch per image
  const int split = tune().nms_split && !(tune().nms_variant & 4) ? 1 : 0;
  hipLaunchKernelGGL(nms_kernel, dim3(n), dim3(kNmsThreads), 0, s, io, n_anchors, no, conf, iou, multi_label,
                     agnostic, class_mask, max_det, ws, cap, det, idx, count, tune().nms_variant, split);
  if (split) {
    const int wmax = (int)std::min<size_t>(cap, kNmsMaskCap) / 64;
    hipLaunchKernelGGL(nms_mask_kernel, dim3(wmax * (wmax + 1) / 2, n), dim3(256), 0, s, n_anchors, no - 5, iou, ws,
                       cap);
    hipLaunchKernelGGL(nms_scan_kernel, dim3(n), dim3(256), 0, s, io, n_anchors, no, max_det, ws, cap, det, idx,
                       count);
  }
  RTDM_HIP(hipGetLastError());
}

}  // namespace rtdm
