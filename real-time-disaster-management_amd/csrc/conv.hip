// Convolution as implicit GEMM on gfx950.
//
//   rows  (M) = output pixels (n, oy, ox) — linear or 2x2-"quad" ordered
//   cols  (N) = output channels
//   depth (K) = (kh, kw, cin), each tap's cin slice contiguous in NHWC
//
// Two bodies share one epilogue:
//   conv_mfma_f16  fp16 operands, fp32 accumulation on v_mfma_f32_16x16x32_f16,
//                  16-byte vector loads, double-buffered LDS (padded rows => no
//                  ds_read_b128 bank conflicts), one barrier per K-block.
//   conv_valu      fp32 FMA on VALU (parity mode, and the Cin=3 stems that read
//                  uint8 frames / NCHW model inputs directly).
//
// Replaces: nn.Conv2d (+ SyncBatchNorm eps 1e-4 + LeakyReLU 0.1) of
// victim_localization/yolov3/models.py:23-44 as run by Darknet.forward
// (:345-347), the shortcut add (:349-354, fused as a residual epilogue), the
// 2x2 maxpool (:57-64, fused via quad ordering), nearest upsample (:66-71,
// fused as a x2 store), the YOLOLayer decode (:252-258, fused into the head
// conv) and ACFF's fused 1x1 conv -> LeakyReLU(0.01) -> BatchNorm
// (disaster_detection/model/acff.py:49-53, BN applied as a post-activation affine).
#include "common.h"

namespace rtdm {

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));

template <typename T>
__device__ __forceinline__ float ldf(const T* p) {
  return (float)(*p);
}
template <typename T>
__device__ __forceinline__ void stf(T* p, float v) {
  *p = (T)v;
}

__device__ __forceinline__ void row_to_pix(const ConvArgs& a, int m, int& n, int& oy, int& ox) {
  if (a.quad) {
    const int q = m >> 2, d = m & 3;
    const int qx = q % a.qw;
    const int t = q / a.qw;
    const int qy = t % a.qh;
    n = t / a.qh;
    oy = 2 * qy + (d >> 1);
    ox = 2 * qx + (d & 1);
  } else {
    ox = m % a.ow;
    const int t = m / a.ow;
    oy = t % a.oh;
    n = t / a.oh;
  }
}

__device__ __forceinline__ float sigmoidf_(float x) { return 1.f / (1.f + expf(-x)); }

// Epilogue for the 4 accumulator values of rows m0..m0+3 (m0 % 4 == 0) in
// output channel c.  In quad mode the 4 rows are one 2x2 pixel quad.
template <typename T>
__device__ __forceinline__ void epi4(const ConvArgs& a, int m0, int c, const float* v) {
  const Epilogue& e = a.e;
  float vals[4];
  float pmax = -INFINITY;
  int pn = 0, poy = 0, pox = 0;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int m = m0 + r;
    if (m >= a.M) break;
    int n, oy, ox;
    row_to_pix(a, m, n, oy, ox);
    if (r == 0) { pn = n; poy = oy; pox = ox; }
    float x = v[r];
    if (e.bias) x += e.bias[c];
    if (e.act == ACT_LEAKY) {
      x = x > 0.f ? x : x * e.slope;
    } else if (e.act == ACT_SWISH) {
      x = x * sigmoidf_(x);
    }
    if (e.scale) x = x * e.scale[c] + e.shift[c];
    const size_t pix = ((size_t)n * a.oh + oy) * a.ow + ox;
    if (e.res.ptr) x += ldf((const T*)e.res.ptr + pix * e.res.cs + e.res.co + c);
    vals[r] = x;
    pmax = fmaxf(pmax, x);
    if (e.full.ptr) stf((T*)e.full.ptr + pix * e.full.cs + e.full.co + c, x);
    if (e.up.ptr) {
      const int uw = a.ow * 2;
      const size_t u0 = ((size_t)n * a.oh * 2 + 2 * oy) * uw + 2 * ox;
      T* up = (T*)e.up.ptr + e.up.co + c;
      const T hv = (T)x;
      up[u0 * e.up.cs] = hv;
      up[(u0 + 1) * e.up.cs] = hv;
      up[(u0 + uw) * e.up.cs] = hv;
      up[(u0 + uw + 1) * e.up.cs] = hv;
    }
    if (e.io) {
      const int ai = c / e.no, k = c - ai * e.no;
      float o;
      if (k < 2) {
        o = (sigmoidf_(x) + (float)(k == 0 ? ox : oy)) * e.ystride;
      } else if (k < 4) {
        o = (expf(x) * e.anchor_vec[2 * ai + (k - 2)]) * e.ystride;
      } else {
        o = sigmoidf_(x);
      }
      const size_t row = (size_t)e.io_off + ((size_t)ai * a.oh + oy) * a.ow + ox;
      e.io[((size_t)n * e.io_rows + row) * e.no + k] = o;
    }
  }
  (void)vals;
  if (e.pool.ptr && a.quad && m0 < a.M) {
    const size_t pp = ((size_t)pn * a.qh + (poy >> 1)) * a.qw + (pox >> 1);
    stf((T*)e.pool.ptr + pp * e.pool.cs + e.pool.co + c, pmax);
  }
}

// --------------------------------------------------------------------------
// fp16 MFMA implicit GEMM.  BM x BN block tile, BK-deep K-blocks, WM x WN waves.
// --------------------------------------------------------------------------
template <int BM, int BN, int BK, int WM, int WN>
__global__ __launch_bounds__(64 * WM * WN) void conv_mfma_f16(ConvArgs a) {
  constexpr int NT = 64 * WM * WN;
  constexpr int KV = BK / 8;          // 16-byte vectors per row of a K-block
  constexpr int LS = BK + 8;          // padded LDS row (halfs)
  constexpr int RPP = NT / KV;        // rows covered by one pass of the block
  constexpr int VA = BM / RPP;
  constexpr int VB = (BN + RPP - 1) / RPP;
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int TM = WTM / 16, TN = WTN / 16;
  static_assert(BM % RPP == 0, "BM must be a multiple of rows per pass");
  static_assert(TM >= 1 && TN >= 1, "wave tile too small");
  constexpr int BUF = (BM + BN) * LS;
  __shared__ __attribute__((aligned(16))) _Float16 smem[2 * BUF];

  const int tid = threadIdx.x;
  const int lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid - (wid / WN) * WN;
  const int m_base = blockIdx.x * BM;
  const int n_base = blockIdx.y * BN;

  const int kvl = tid % KV;
  const int r0 = tid / KV;

  const _Float16* __restrict__ in = (const _Float16*)a.in;
  const _Float16* __restrict__ wt = (const _Float16*)a.w;

  int a_pix[VA], a_iy[VA], a_ix[VA];
#pragma unroll
  for (int i = 0; i < VA; ++i) {
    const int m = m_base + r0 + i * RPP;
    if (m < a.M) {
      int n, oy, ox;
      row_to_pix(a, m, n, oy, ox);
      a_pix[i] = n * a.ih * a.iw;
      a_iy[i] = oy * a.stride - a.pad;
      a_ix[i] = ox * a.stride - a.pad;
    } else {
      a_pix[i] = 0;
      a_iy[i] = -(1 << 28);
      a_ix[i] = -(1 << 28);
    }
  }
  const int cvecs = a.cin >> 3;
  const int kvec_total = a.ks * a.ks * cvecs;
  const int nk = a.kpad / BK;

  uint4 ra[VA], rb[VB];
  const uint4 zero4 = make_uint4(0, 0, 0, 0);

  auto gload = [&](int kb) {
    const int kv = kb * KV + kvl;
    const bool kval = kv < kvec_total;
    const int tap = kval ? kv / cvecs : 0;
    const int cv = kv - tap * cvecs;
    const int kh = tap / a.ks;
    const int kw = tap - kh * a.ks;
#pragma unroll
    for (int i = 0; i < VA; ++i) {
      const int iy = a_iy[i] + kh, ix = a_ix[i] + kw;
      if (kval && (unsigned)iy < (unsigned)a.ih && (unsigned)ix < (unsigned)a.iw) {
        ra[i] = *(const uint4*)(in + (size_t)(a_pix[i] + iy * a.iw + ix) * a.in_cs + a.in_co + cv * 8);
      } else {
        ra[i] = zero4;
      }
    }
#pragma unroll
    for (int j = 0; j < VB; ++j) {
      const int r = r0 + j * RPP;
      if (r < BN) rb[j] = *(const uint4*)(wt + (size_t)(n_base + r) * a.kpad + kb * BK + kvl * 8);
    }
  };
  auto sstore = [&](int buf) {
    _Float16* As = smem + buf * BUF;
    _Float16* Bs = As + BM * LS;
#pragma unroll
    for (int i = 0; i < VA; ++i) *(uint4*)(As + (r0 + i * RPP) * LS + kvl * 8) = ra[i];
#pragma unroll
    for (int j = 0; j < VB; ++j) {
      const int r = r0 + j * RPP;
      if (r < BN) *(uint4*)(Bs + r * LS + kvl * 8) = rb[j];
    }
  };

  f4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};

  gload(0);
  sstore(0);
  __syncthreads();

  const int frow = lane & 15;
  const int fk = (lane >> 4) * 8;
  for (int kb = 0; kb < nk; ++kb) {
    const int buf = kb & 1;
    if (kb + 1 < nk) gload(kb + 1);
    const _Float16* As = smem + buf * BUF;
    const _Float16* Bs = As + BM * LS;
#pragma unroll
    for (int ks = 0; ks < BK / 32; ++ks) {
      h8 af[TM], bf[TN];
#pragma unroll
      for (int tm = 0; tm < TM; ++tm)
        af[tm] = *(const h8*)(As + (wm * WTM + tm * 16 + frow) * LS + ks * 32 + fk);
#pragma unroll
      for (int tn = 0; tn < TN; ++tn)
        bf[tn] = *(const h8*)(Bs + (wn * WTN + tn * 16 + frow) * LS + ks * 32 + fk);
#pragma unroll
      for (int tm = 0; tm < TM; ++tm)
#pragma unroll
        for (int tn = 0; tn < TN; ++tn)
          acc[tm][tn] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[tm], bf[tn], acc[tm][tn], 0, 0, 0);
    }
    if (kb + 1 < nk) sstore(buf ^ 1);
    __syncthreads();
  }

  const int rq = (lane >> 4) * 4;
#pragma unroll
  for (int tm = 0; tm < TM; ++tm) {
    const int m0 = m_base + wm * WTM + tm * 16 + rq;
#pragma unroll
    for (int tn = 0; tn < TN; ++tn) {
      const int c = n_base + wn * WTN + tn * 16 + frow;
      if (c < a.cout) {
        float v[4] = {acc[tm][tn][0], acc[tm][tn][1], acc[tm][tn][2], acc[tm][tn][3]};
        epi4<_Float16>(a, m0, c, v);
      }
    }
  }
}

// --------------------------------------------------------------------------
// VALU fp32 implicit GEMM: 64x64 block tile, 16-deep K-blocks, 4x4 per thread.
// Handles every input kind (NHWC activations, uint8 frames, NCHW tensors) and
// any Cin.  T = activation type of NHWC input/outputs; weights are fp32.
// --------------------------------------------------------------------------
template <typename T>
__device__ __forceinline__ float load_in(const ConvArgs& a, int n, int y, int x, int c) {
  switch (a.in_kind) {
    case IN_NHWC:
      return ldf((const T*)a.in + ((size_t)(n * a.ih + y) * a.iw + x) * a.in_cs + a.in_co + c);
    case IN_FRAME_U8:
      return (float)((const uint8_t*)a.in)[((size_t)(n * a.ih + y) * a.iw + x) * 3 + c] / 255.f;
    case IN_NCHW_F32:
      return ((const float*)a.in)[(((size_t)n * a.cin + c) * a.ih + y) * a.iw + x];
    default:
      return (float)((const _Float16*)a.in)[(((size_t)n * a.cin + c) * a.ih + y) * a.iw + x];
  }
}

template <typename T>
__global__ __launch_bounds__(256) void conv_valu(ConvArgs a) {
  constexpr int BM = 64, BN = 64, BK = 16;
  __shared__ float As[BK][BM + 4];
  __shared__ float Bs[BK][BN + 4];
  const int tid = threadIdx.x;
  const int tx = tid & 15, ty = tid >> 4;
  const int m_base = blockIdx.x * BM, n_base = blockIdx.y * BN;
  const float* __restrict__ wt = (const float*)a.w;
  const int ktot = a.ks * a.ks * a.cin;

  // A rows handled by this thread for loading: r = ty + 16*i, k_l = tx
  int ln[4], liy[4], lix[4];
  bool lval[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = m_base + ty + 16 * i;
    lval[i] = m < a.M;
    int n = 0, oy = 0, ox = 0;
    if (lval[i]) row_to_pix(a, m, n, oy, ox);
    ln[i] = n;
    liy[i] = oy * a.stride - a.pad;
    lix[i] = ox * a.stride - a.pad;
  }
  float acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = 0.f;

  for (int k0 = 0; k0 < ktot; k0 += BK) {
    const int k = k0 + tx;
    const bool kval = k < ktot;
    const int tap = kval ? k / a.cin : 0;
    const int c = k - tap * a.cin;
    const int kh = tap / a.ks, kw = tap - (tap / a.ks) * a.ks;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int iy = liy[i] + kh, ix = lix[i] + kw;
      float v = 0.f;
      if (kval && lval[i] && (unsigned)iy < (unsigned)a.ih && (unsigned)ix < (unsigned)a.iw)
        v = load_in<T>(a, ln[i], iy, ix, c);
      As[tx][ty + 16 * i] = v;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int col = n_base + ty + 16 * i;
      Bs[tx][ty + 16 * i] = (kval && col < a.cout_pad) ? wt[(size_t)col * a.kpad + k] : 0.f;
    }
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < BK; ++kk) {
      float av[4], bv[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) av[i] = As[kk][ty * 4 + i];
#pragma unroll
      for (int j = 0; j < 4; ++j) bv[j] = Bs[kk][tx + 16 * j];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = fmaf(av[i], bv[j], acc[i][j]);
    }
    __syncthreads();
  }
  const int m0 = m_base + ty * 4;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int c = n_base + tx + 16 * j;
    if (c < a.cout) {
      float v[4] = {acc[0][j], acc[1][j], acc[2][j], acc[3][j]};
      epi4<T>(a, m0, c, v);
    }
  }
}

// --------------------------------------------------------------------------
template <int BM, int BN, int BK, int WM, int WN>
static void launch_mfma(const ConvArgs& a, hipStream_t s) {
  RTDM_REQUIRE(a.cout_pad % BN == 0, RTDM_E_INVALID, "conv: cout_pad not a multiple of BN");
  RTDM_REQUIRE(a.kpad % BK == 0, RTDM_E_INVALID, "conv: kpad not a multiple of BK");
  dim3 grid((a.M + BM - 1) / BM, a.cout_pad / BN);
  hipLaunchKernelGGL((conv_mfma_f16<BM, BN, BK, WM, WN>), grid, dim3(64 * WM * WN), 0, s, a);
}

static bool mfma_ok(const ConvArgs& a) {
  return a.in_kind == IN_NHWC && a.cin % 8 == 0 && a.in_cs % 8 == 0 && a.in_co % 8 == 0;
}

const char* conv_kernel_name(const ConvArgs& a, int dtype) {
  if (dtype == RTDM_F16 && !a.w_f32) {
    if (a.cout_pad >= 128) return "conv_mfma_f16<128,128,64,2,2>";
    if (a.cout_pad == 64) return "conv_mfma_f16<128,64,64,2,2>";
    if (a.cout_pad == 32) return "conv_mfma_f16<128,32,64,4,1>";
    return "conv_mfma_f16<128,16,64,4,1>";
  }
  return dtype == RTDM_F16 ? "conv_valu<_Float16>" : "conv_valu<float>";
}

void launch_conv(const ConvArgs& a, int dtype, hipStream_t s) {
  if (a.M <= 0) return;
  RTDM_REQUIRE(!a.quad || (a.oh >= 2 && a.ow >= 2), RTDM_E_INVALID, "conv: quad ordering needs >= 2x2 output");
  RTDM_REQUIRE(!a.e.pool.ptr || a.quad, RTDM_E_INVALID, "conv: pooled output needs quad ordering");
  if (dtype == RTDM_F16 && !a.w_f32) {
    RTDM_REQUIRE(mfma_ok(a), RTDM_E_INVALID, "conv: fp16 MFMA weights but input view not 16-byte aligned NHWC");
    if (a.cout_pad >= 128)
      launch_mfma<128, 128, 64, 2, 2>(a, s);
    else if (a.cout_pad == 64)
      launch_mfma<128, 64, 64, 2, 2>(a, s);
    else if (a.cout_pad == 32)
      launch_mfma<128, 32, 64, 4, 1>(a, s);
    else
      launch_mfma<128, 16, 64, 4, 1>(a, s);
  } else {
    RTDM_REQUIRE(a.w_f32, RTDM_E_INVALID, "conv: VALU body needs fp32-packed weights");
    dim3 grid((a.M + 63) / 64, (a.cout_pad + 63) / 64);
    if (dtype == RTDM_F16)
      hipLaunchKernelGGL(conv_valu<_Float16>, grid, dim3(256), 0, s, a);
    else
      hipLaunchKernelGGL(conv_valu<float>, grid, dim3(256), 0, s, a);
  }
  RTDM_HIP(hipGetLastError());
}

}  // namespace rtdm
