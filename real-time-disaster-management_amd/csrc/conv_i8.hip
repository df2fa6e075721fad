// int8 implicit-GEMM convolution for the int8-quantised detector (RTDM_I8,
// BASELINE config 5: the CDNA4 int8 MFMA path).
//
//   A  fp16 NHWC activations, quantised per tensor while staged into LDS:
//      q = clamp(rint(x * qscale), -127, 127), qscale = 127 / calibrated |x|max
//   B  int8 weights [cout_pad][kpad] (BN folded first), one scale per output channel
//   MFMA v_mfma_i32_16x16x64_i8: the int32 sum of a K-block is exact
//   epilogue  acc * deq[c] (deq = s_x * s_w[c]) -> the fp16 epilogue of conv_epi.h
//             (bias, LeakyReLU, fused 2x2 pool / x2 upsample / route slices)
//
// Activations stay fp16 in HBM, so every producer/consumer fusion of the fp16
// plan (route concats as channel slices, pooled/upsampled stores) is unchanged and
// no per-concat scale agreement is needed; int8 buys the 2x MFMA rate.
//
// Tile 128 x 128 x 64 (int8 K), 4 waves of 64 x 64 (4 x 4 accumulators), the
// conv_mfma_f16 register-staged double buffer (one barrier per K-block) and the
// same XCD-aware tile remap.  Replaces the same reference ops as conv.hip
// (victim_localization/yolov3/models.py:23-44 conv + BN + LeakyReLU).
#include "conv_epi.h"

#include <algorithm>

namespace rtdm {

namespace {
typedef int i32x4 __attribute__((ext_vector_type(4)));
constexpr int kQBM = 128, kQBN = 128, kQBK = 64;  // K-block in int8 elements
constexpr int kQLS = kQBK + 16;                    // LDS row bytes (padding: distinct bank slots)
constexpr int kQBuf = (kQBM + kQBN) * kQLS;        // bytes per staging buffer
constexpr int kQCstr = kQBN + 4;
constexpr int kQSmem = 2 * kQBuf > kQBM * kQCstr * 4 ? 2 * kQBuf : kQBM * kQCstr * 4;

__device__ __forceinline__ uint32_t q4(float a, float b, float c, float d) {
  auto q = [](float v) {
    const int i = (int)rintf(v);
    return (uint32_t)(i < -127 ? -127 : (i > 127 ? 127 : i)) & 255u;
  };
  return q(a) | (q(b) << 8) | (q(c) << 16) | (q(d) << 24);
}
}  // namespace

__global__ __launch_bounds__(256) void conv_i8(ConvArgs a) {
  constexpr int NT = 256, WM = 2, WN = 2;
  constexpr int KV = kQBK / 8;      // 8-half vectors per A row per K-block
  constexpr int RPP = NT / KV;      // A rows per pass (32)
  constexpr int VA = kQBM / RPP;    // 4
  constexpr int KVB = kQBK / 16;    // 16-byte vectors per B row per K-block
  constexpr int RPPB = NT / KVB;    // 64
  constexpr int VB = kQBN / RPPB;   // 2
  constexpr int TM = kQBM / WM / 16, TN = kQBN / WN / 16;
  __shared__ __attribute__((aligned(16))) unsigned char smem[kQSmem];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid - (wid / WN) * WN;
  const int nblk = gridDim.x, ntn = a.cout_pad / kQBN;
  int bid = blockIdx.x;
  {
    const int xcd = bid & 7, q = nblk >> 3, r = nblk & 7;
    bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  }
  const int m_base = (bid / ntn) * kQBM;
  const int n_base = (bid - (bid / ntn) * ntn) * kQBN;

  const int kvl = tid % KV, r0 = tid / KV;
  const int kvb = tid % KVB, rb0 = tid / KVB;
  const _Float16* __restrict__ in = (const _Float16*)a.in + a.in_co;
  const int8_t* __restrict__ wt = (const int8_t*)a.w8 + (size_t)(n_base + rb0) * a.kpad + kvb * 16;

  int a_pix[VA], a_iy[VA], a_ix[VA];
#pragma unroll
  for (int i = 0; i < VA; ++i) {
    const int m = m_base + r0 + i * RPP;
    int n = 0, oy = 0, ox = 0;
    if (m < a.M) row_to_pix(a, m, n, oy, ox);
    a_pix[i] = n * a.ih * a.iw;
    a_iy[i] = m < a.M ? oy * a.stride - a.pad : -(1 << 28);
    a_ix[i] = ox * a.stride - a.pad;
  }
  const int cvecs = a.cin >> 3, kvec_total = a.ks * a.ks * cvecs, nk = a.kpad / kQBK;
  const int ih = a.ih, iw = a.iw, ics = a.in_cs, ks = a.ks, kpad = a.kpad;
  const float qs = a.qscale;

  uint2 ra[VA];
  u32x4 rb[VB];
  auto gload = [&](int kb) {
    const int kv = kb * KV + kvl;
    const bool kval = kv < kvec_total;
    const int tap = kval ? kv / cvecs : 0;
    const int cv = kv - tap * cvecs;
    const int kh = tap / ks, kw = tap - kh * ks;
#pragma unroll
    for (int i = 0; i < VA; ++i) {
      const int iy = a_iy[i] + kh, ix = a_ix[i] + kw;
      const bool v = kval && (unsigned)iy < (unsigned)ih && (unsigned)ix < (unsigned)iw;
      const size_t off = v ? (size_t)(a_pix[i] + iy * iw + ix) * ics + cv * 8 : 0;
      const h8 t = *(const h8*)(in + off);
      const float s = v ? qs : 0.f;  // padding taps quantise to 0
      ra[i] = make_uint2(q4((float)t[0] * s, (float)t[1] * s, (float)t[2] * s, (float)t[3] * s),
                         q4((float)t[4] * s, (float)t[5] * s, (float)t[6] * s, (float)t[7] * s));
    }
#pragma unroll
    for (int j = 0; j < VB; ++j) rb[j] = *(const u32x4*)(wt + (size_t)j * RPPB * kpad + (size_t)kb * kQBK);
  };
  auto sstore = [&](int buf) {
    unsigned char* As = smem + buf * kQBuf;
    unsigned char* Bs = As + kQBM * kQLS;
#pragma unroll
    for (int i = 0; i < VA; ++i) *(uint2*)(As + (r0 + i * RPP) * kQLS + kvl * 8) = ra[i];
#pragma unroll
    for (int j = 0; j < VB; ++j) *(u32x4*)(Bs + (rb0 + j * RPPB) * kQLS + kvb * 16) = rb[j];
  };

  i32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = i32x4{0, 0, 0, 0};

  gload(0);
  sstore(0);
  __syncthreads();
  const int frow = lane & 15, fk = (lane >> 4) * 16;
  for (int kb = 0; kb < nk; ++kb) {
    const int buf = kb & 1;
    const bool more = kb + 1 < nk;
    if (more) gload(kb + 1);
    const unsigned char* As = smem + buf * kQBuf + (wm * 64 + frow) * kQLS + fk;
    const unsigned char* Bs = smem + buf * kQBuf + kQBM * kQLS + (wn * 64 + frow) * kQLS + fk;
    i32x4 af[TM], bf[TN];
#pragma unroll
    for (int tm = 0; tm < TM; ++tm) af[tm] = *(const i32x4*)(As + tm * 16 * kQLS);
#pragma unroll
    for (int tn = 0; tn < TN; ++tn) bf[tn] = *(const i32x4*)(Bs + tn * 16 * kQLS);
#pragma unroll
    for (int tm = 0; tm < TM; ++tm)
#pragma unroll
      for (int tn = 0; tn < TN; ++tn) acc[tm][tn] = __builtin_amdgcn_mfma_i32_16x16x64_i8(af[tm], bf[tn], acc[tm][tn], 0, 0, 0);
    if (more) sstore(buf ^ 1);
    __syncthreads();
  }

  // ---- epilogue: dequantise -> LDS C tile (fp32) -> 4 rows x 8 channels per thread ----
  float* Cs = reinterpret_cast<float*>(smem);
  const int rq = (lane >> 4) * 4;
#pragma unroll
  for (int tn = 0; tn < TN; ++tn) {
    const int col = wn * 64 + tn * 16 + frow;
    const float dq = n_base + col < a.cout ? a.deq[n_base + col] : 0.f;
#pragma unroll
    for (int tm = 0; tm < TM; ++tm) {
      const int row = wm * 64 + tm * 16 + rq;
#pragma unroll
      for (int j = 0; j < 4; ++j) Cs[(row + j) * kQCstr + col] = (float)acc[tm][tn][j] * dq;
    }
  }
  __syncthreads();
  constexpr int CG = kQBN / 8, UNITS = (kQBM / 4) * CG;
  for (int u = tid; u < UNITS; u += NT) {
    const int q = u / CG, gg = u - (u / CG) * CG;
    const int m0 = m_base + q * 4, c0 = n_base + gg * 8;
    if (m0 >= a.M || c0 >= a.cout) continue;
    float v[4][8];
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int j = 0; j < 8; ++j) v[r][j] = Cs[(q * 4 + r) * kQCstr + gg * 8 + j];
    epi_vec8(a, m0, c0, v);
  }
}

bool conv_i8_ok(const ConvArgs& a) {
  if (a.in_kind != IN_NHWC || a.w_f32 || (a.in_cs | a.in_co) % 8 != 0 || a.cin % 64 != 0) return false;
  if (a.cout_pad % kQBN != 0 || (a.ks != 1 && a.ks != 3) || a.kpad % kQBK != 0) return false;
  if (a.e.io || a.head_w) return false;
  return (int64_t)a.n * a.ih * a.iw * a.in_cs < (1ll << 31);
}

void launch_conv_i8(const ConvArgs& a, hipStream_t s) {
  RTDM_REQUIRE(conv_i8_ok(a) && a.w8 && a.deq, RTDM_E_INVALID, "conv_i8: unsupported layer");
  if (a.M <= 0) return;
  const int64_t nblk = (int64_t)((a.M + kQBM - 1) / kQBM) * (a.cout_pad / kQBN);
  RTDM_REQUIRE(nblk < (1ll << 31), RTDM_E_CAPACITY, "conv_i8: grid too large");
  hipLaunchKernelGGL(conv_i8, dim3((unsigned)nblk), dim3(256), 0, s, a);
  RTDM_HIP(hipGetLastError());
}

// |x|max of an NHWC fp16 view (calibration): block max, then one float atomic-max
// as an unsigned compare (|x| >= 0, so IEEE order = integer order).
__global__ __launch_bounds__(256) void absmax_kernel(const _Float16* __restrict__ p, int cs, int co, int64_t npix,
                                                     int cvec, unsigned* __restrict__ out) {
  float m = 0.f;
  const int64_t total = npix * cvec;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t px = i / cvec;
    const int v = (int)(i - px * cvec);
    const h8 x = *(const h8*)(p + px * cs + co + v * 8);
#pragma unroll
    for (int j = 0; j < 8; ++j) m = fmaxf(m, fabsf((float)x[j]));
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) m = fmaxf(m, __shfl_xor(m, off));
  __shared__ float wmax[4];
  if ((threadIdx.x & 63) == 0) wmax[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    const float b = fmaxf(fmaxf(wmax[0], wmax[1]), fmaxf(wmax[2], wmax[3]));
    atomicMax(out, __float_as_uint(b));
  }
}

// |x| histogram of an NHWC fp16 view over [0, amax] in kCalBins bins (calibration
// pass 2: the clip threshold that minimises the int8 quantisation MSE).
__global__ __launch_bounds__(256) void abshist_kernel(const _Float16* __restrict__ p, int cs, int co, int64_t npix,
                                                      int cvec, const unsigned* __restrict__ amax_bits,
                                                      unsigned* __restrict__ hist) {
  __shared__ unsigned h[kCalBins];
  for (int i = threadIdx.x; i < kCalBins; i += blockDim.x) h[i] = 0u;
  __syncthreads();
  const float amax = __uint_as_float(*amax_bits);
  const float inv = amax > 0.f ? (float)kCalBins / amax : 0.f;
  const int64_t total = npix * cvec;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t px = i / cvec;
    const int v = (int)(i - px * cvec);
    const h8 x = *(const h8*)(p + px * cs + co + v * 8);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int b = (int)(fabsf((float)x[j]) * inv);
      atomicAdd(&h[b < kCalBins ? b : kCalBins - 1], 1u);
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < kCalBins; i += blockDim.x)
    if (h[i]) atomicAdd(&hist[i], h[i]);
}

void launch_abshist(View v, int n, int h, int w, int c, const unsigned* amax, unsigned* hist, hipStream_t s) {
  const int64_t npix = (int64_t)n * h * w;
  const int64_t total = npix * (c / 8);
  if (total <= 0) return;
  const int blocks = (int)std::min<int64_t>((total + 255) / 256, 2048);
  hipLaunchKernelGGL(abshist_kernel, dim3(blocks), dim3(256), 0, s, (const _Float16*)v.ptr, v.cs, v.co, npix, c / 8,
                     amax, hist);
  RTDM_HIP(hipGetLastError());
}

void launch_absmax(View v, int n, int h, int w, int c, unsigned* out, hipStream_t s) {
  RTDM_REQUIRE(c % 8 == 0 && (v.cs | v.co) % 8 == 0, RTDM_E_INVALID, "absmax: view not 16-byte aligned");
  const int64_t npix = (int64_t)n * h * w;
  const int64_t total = npix * (c / 8);
  if (total <= 0) return;
  const int blocks = (int)std::min<int64_t>((total + 255) / 256, 4096);
  hipLaunchKernelGGL(absmax_kernel, dim3(blocks), dim3(256), 0, s, (const _Float16*)v.ptr, v.cs, v.co, npix, c / 8,
                     out);
  RTDM_HIP(hipGetLastError());
}

}  // namespace rtdm
