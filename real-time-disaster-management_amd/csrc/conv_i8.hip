// int8 support for the int8-quantised detector (RTDM_I8, BASELINE config 5: the CDNA4
// int8 MFMA path).  The GEMM itself is conv_pipe_i8 (conv_pipe.hip, the pipelined
// implicit GEMM on v_mfma_i32_16x16x64_i8); this file holds the two element-wise
// kernels around it:
//
//   chan_absmax_kernel  calibration: per-channel |x|max of an fp16 NHWC view (the
//                       input of an int8 conv) over the calibration frames.  The
//                       per-channel activation scale s_c = 2 |x|max_c / 127 is folded into
//                       the conv's weights on the host (with the detector's 2x headroom,
//                       detector.cpp kI8Headroom; W'[o][c] = W[o][c] * s_c, then
//                       symmetric per-output-channel int8: s_w[o] = max|W'[o]| / 127).
//   quantize_kernel     runtime: q = clamp(rint(x * (1 / s_c)), -127, 127), fp16 view ->
//                       contiguous int8 [pixels][cin] (symmetric: an out-of-image tap,
//                       read as 0 by the GEMM's buffer loads, is exactly x = 0).
//
// The reference has no numeric int8 path (its int8 artefacts are opaque TensorRT
// engines, calibration caches from calibrator.py:87-153); the scheme is the build's own.
#include "conv_epi.h"

#include <algorithm>

namespace rtdm {

// One block per pixel stripe; thread (g, p) covers channels 8g..8g+7 of every
// (blockDim / groups)-th pixel; per-channel maxima meet in LDS, then one atomicMax per
// channel per block on the float bits (|x| >= 0: IEEE order = unsigned order).
__global__ __launch_bounds__(256) void chan_absmax_kernel(const _Float16* __restrict__ p, int cs, int co, int64_t npix,
                                                          int cin, unsigned* __restrict__ out) {
  extern __shared__ unsigned s_max[];
  for (int i = threadIdx.x; i < cin; i += blockDim.x) s_max[i] = 0u;
  __syncthreads();
  const int groups = cin / 8;
  const int g = threadIdx.x % groups, lane_px = threadIdx.x / groups, px_per = blockDim.x / groups;
  float m[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (lane_px < px_per) {
    for (int64_t px = (int64_t)blockIdx.x * px_per + lane_px; px < npix; px += (int64_t)gridDim.x * px_per) {
      const h8 x = *(const h8*)(p + px * cs + co + g * 8);
#pragma unroll
      for (int j = 0; j < 8; ++j) m[j] = fmaxf(m[j], fabsf((float)x[j]));
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) atomicMax(&s_max[g * 8 + j], __float_as_uint(m[j]));
  }
  __syncthreads();
  for (int i = threadIdx.x; i < cin; i += blockDim.x)
    if (s_max[i]) atomicMax(&out[i], s_max[i]);
}

void launch_chan_absmax(View v, int n, int h, int w, int c, unsigned* out, hipStream_t s) {
  RTDM_REQUIRE(c % 8 == 0 && c <= 2048 && (v.cs | v.co) % 8 == 0, RTDM_E_INVALID, "absmax: view not 16-byte aligned");
  const int64_t npix = (int64_t)n * h * w;
  if (npix <= 0) return;
  const int px_per = std::max(1, 256 / (c / 8));
  const int blocks = (int)std::min<int64_t>((npix + px_per - 1) / px_per, 2048);
  hipLaunchKernelGGL(chan_absmax_kernel, dim3(blocks), dim3(256), c * sizeof(unsigned), s, (const _Float16*)v.ptr,
                     v.cs, v.co, npix, c, out);
  RTDM_HIP(hipGetLastError());
}

// 8 channels per thread: one 16-byte fp16 load, one 8-byte int8 store.  32-bit indices
// with a multiply-shift division by the channel-group count (the former 64-bit divide per
// element cost more than the 3 bytes of memory traffic), the 8 inverse scales as two
// 16-byte loads.
__global__ __launch_bounds__(256) void quantize_kernel(const _Float16* __restrict__ p, int cs, int co, int npix,
                                                       int cin, FastDiv fgroups, const float* __restrict__ inv_scale,
                                                       int8_t* __restrict__ q) {
  typedef float f4 __attribute__((ext_vector_type(4)));
  const int groups = cin / 8;
  const int total = npix * groups;
  // unsigned cursor: total < 2^31 and the stride < 2^31, so i + stride never wraps
  for (unsigned ui = blockIdx.x * blockDim.x + threadIdx.x; ui < (unsigned)total; ui += gridDim.x * blockDim.x) {
    const int i = (int)ui;
    const int px = fdiv(i, fgroups);
    const int g = i - px * groups;
    const h8 x = *(const h8*)(p + (size_t)px * cs + co + g * 8);
    const f4 s0 = *(const f4*)(inv_scale + g * 8), s1 = *(const f4*)(inv_scale + g * 8 + 4);
    uint32_t lo = 0, hi = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      int v = (int)rintf((float)x[j] * (j < 4 ? s0[j] : s1[j - 4]));
      v = v < -127 ? -127 : (v > 127 ? 127 : v);
      if (j < 4)
        lo |= ((uint32_t)v & 255u) << (8 * j);
      else
        hi |= ((uint32_t)v & 255u) << (8 * (j - 4));
    }
    *(uint2*)(q + (size_t)px * cin + g * 8) = make_uint2(lo, hi);
  }
}

void launch_quantize(View v, int n, int h, int w, int c, const float* inv_scale, int8_t* q, hipStream_t s) {
  RTDM_REQUIRE(c % 8 == 0 && (v.cs | v.co) % 8 == 0, RTDM_E_INVALID, "quantize: view not 16-byte aligned");
  const int64_t npix = (int64_t)n * h * w;
  const int64_t total = npix * (c / 8);
  if (total <= 0) return;
  RTDM_REQUIRE(total < (1ll << 31), RTDM_E_CAPACITY, "quantize: too many elements");
  const int blocks = (int)std::min<int64_t>((total + 255) / 256, 8192);
  hipLaunchKernelGGL(quantize_kernel, dim3(blocks), dim3(256), 0, s, (const _Float16*)v.ptr, v.cs, v.co, (int)npix, c,
                     make_fastdiv(c / 8), inv_scale, q);
  RTDM_HIP(hipGetLastError());
}

}  // namespace rtdm
