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
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

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
    const int t = fdiv(q, a.fd_qw);
    const int qx = q - t * a.qw;
    n = fdiv(t, a.fd_qh);
    const int qy = t - n * a.qh;
    oy = 2 * qy + (d >> 1);
    ox = 2 * qx + (d & 1);
  } else {
    const int t = fdiv(m, a.fd_ow);
    ox = m - t * a.ow;
    n = fdiv(t, a.fd_oh);
    oy = t - n * a.oh;
  }
}

__device__ __forceinline__ float sigmoidf_(float x) { return 1.f / (1.f + expf(-x)); }

// Pixel of row m0 + r given the pixel (n, oy0, ox0) of row m0 (m0 % 4 == 0):
// quad order -> the 2x2 quad; linear order -> the next pixels of the same image
// row when they exist (row_to_pix otherwise).
__device__ __forceinline__ void row_pix4(const ConvArgs& a, int m0, int r, int n0, int oy0, int ox0, int& n, int& oy,
                                         int& ox) {
  if (a.quad) {
    n = n0;
    oy = oy0 + (r >> 1);
    ox = ox0 + (r & 1);
  } else if (ox0 + r < a.ow) {
    n = n0;
    oy = oy0;
    ox = ox0 + r;
  } else {
    row_to_pix(a, m0 + r, n, oy, ox);
  }
}

// Epilogue for the 4 accumulator values of rows m0..m0+3 (m0 % 4 == 0) in
// output channel c.  In quad mode the 4 rows are one 2x2 pixel quad.
template <typename T>
__device__ __forceinline__ void epi4(const ConvArgs& a, int m0, int c, f4 v) {
  const Epilogue& e = a.e;
  if (m0 >= a.M) return;
  const float bias = e.bias ? e.bias[c] : 0.f;
  const float sc = e.scale ? e.scale[c] : 1.f;
  const float sh = e.scale ? e.shift[c] : 0.f;
  float pmax = -INFINITY;
  int n0, oy0, ox0;
  row_to_pix(a, m0, n0, oy0, ox0);
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int m = m0 + r;
    if (m < a.M) {
      int n, oy, ox;
      row_pix4(a, m0, r, n0, oy0, ox0, n, oy, ox);
      float x = v[r] + bias;
      if (e.act == ACT_LEAKY) {
        x = x > 0.f ? x : x * e.slope;
      } else if (e.act == ACT_SWISH) {
        x = x * sigmoidf_(x);
      }
      if (e.scale) x = x * sc + sh;
      const size_t pix = ((size_t)n * a.oh + oy) * a.ow + ox;
      if (e.res.ptr) x += ldf((const T*)e.res.ptr + pix * e.res.cs + e.res.co + c);
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
  }
  if (e.pool.ptr && a.quad) {
    const size_t pp = ((size_t)n0 * a.qh + (oy0 >> 1)) * a.qw + (ox0 >> 1);
    stf((T*)e.pool.ptr + pp * e.pool.cs + e.pool.co + c, pmax);
  }
}

// Vector epilogue for a 2x2 quad / 4 consecutive rows (m0..m0+3) x 8 consecutive
// channels (c0..c0+7) of an fp16 output: bias -> act -> affine -> residual, then
// 16-byte stores of the full / pooled / upsampled views when they are 8-aligned
// (channel stride and offset multiples of 8), scalar stores otherwise; YOLO
// decode channels go to io as fp32 scalars.
typedef _Float16 h8v __attribute__((ext_vector_type(8)));
__device__ __forceinline__ void epi_vec8(const ConvArgs& a, int m0, int c0, const float (&v)[4][8]) {
  const Epilogue& e = a.e;
  const int nc = a.cout - c0 < 8 ? a.cout - c0 : 8;
  float bias[8], sc[8], sh[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const bool cv = j < nc;
    bias[j] = (e.bias && cv) ? e.bias[c0 + j] : 0.f;
    sc[j] = (e.scale && cv) ? e.scale[c0 + j] : 1.f;
    sh[j] = (e.scale && cv) ? e.shift[c0 + j] : 0.f;
  }
  const bool full8 = nc == 8;
  float pmax[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) pmax[j] = -INFINITY;
  int pn, poy, pox;
  row_to_pix(a, m0, pn, poy, pox);
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int m = m0 + r;
    if (m >= a.M) continue;
    int n, oy, ox;
    row_pix4(a, m0, r, pn, poy, pox, n, oy, ox);
    const size_t pix = ((size_t)n * a.oh + oy) * a.ow + ox;
    float x[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float t = v[r][j] + bias[j];
      if (e.act == ACT_LEAKY)
        t = t > 0.f ? t : t * e.slope;
      else if (e.act == ACT_SWISH)
        t = t * sigmoidf_(t);
      x[j] = t * sc[j] + sh[j];
    }
    if (e.res.ptr) {
      const _Float16* rp = (const _Float16*)e.res.ptr + pix * e.res.cs + e.res.co + c0;
      if (full8 && ((e.res.cs | e.res.co) & 7) == 0) {
        const h8v rv = *(const h8v*)rp;
#pragma unroll
        for (int j = 0; j < 8; ++j) x[j] += (float)rv[j];
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (j < nc) x[j] += (float)rp[j];
      }
    }
    h8v hv;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      hv[j] = (_Float16)x[j];
      pmax[j] = fmaxf(pmax[j], x[j]);
    }
    if (e.full.ptr) {
      _Float16* fp = (_Float16*)e.full.ptr + pix * e.full.cs + e.full.co + c0;
      if (full8 && ((e.full.cs | e.full.co) & 7) == 0) {
        *(h8v*)fp = hv;
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (j < nc) fp[j] = hv[j];
      }
    }
    if (e.up.ptr) {
      const int uw = a.ow * 2;
      const size_t u0 = ((size_t)n * a.oh * 2 + 2 * oy) * uw + 2 * ox;
      _Float16* up = (_Float16*)e.up.ptr + e.up.co + c0;
      const size_t uo[4] = {u0, u0 + 1, u0 + uw, u0 + uw + 1};
      if (full8 && ((e.up.cs | e.up.co) & 7) == 0) {
#pragma unroll
        for (int q = 0; q < 4; ++q) *(h8v*)(up + uo[q] * e.up.cs) = hv;
      } else {
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
          for (int j = 0; j < 8; ++j)
            if (j < nc) up[uo[q] * e.up.cs + j] = hv[j];
      }
    }
    if (e.io) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        if (j >= nc) continue;
        const int c = c0 + j;
        const int ai = c / e.no, k = c - ai * e.no;
        float o;
        if (k < 2)
          o = (sigmoidf_(x[j]) + (float)(k == 0 ? ox : oy)) * e.ystride;
        else if (k < 4)
          o = (expf(x[j]) * e.anchor_vec[2 * ai + (k - 2)]) * e.ystride;
        else
          o = sigmoidf_(x[j]);
        const size_t row = (size_t)e.io_off + ((size_t)ai * a.oh + oy) * a.ow + ox;
        e.io[((size_t)n * e.io_rows + row) * e.no + k] = o;
      }
    }
  }
  if (e.pool.ptr && a.quad && m0 < a.M) {
    const size_t pp = ((size_t)pn * a.qh + (poy >> 1)) * a.qw + (pox >> 1);
    _Float16* qp = (_Float16*)e.pool.ptr + pp * e.pool.cs + e.pool.co + c0;
    if (full8 && ((e.pool.cs | e.pool.co) & 7) == 0) {
      h8v pv;
#pragma unroll
      for (int j = 0; j < 8; ++j) pv[j] = (_Float16)pmax[j];
      *(h8v*)qp = pv;
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (j < nc) qp[j] = (_Float16)pmax[j];
    }
  }
}

// --------------------------------------------------------------------------
// fp16 MFMA implicit GEMM.  BM x BN block tile, BK-deep K-blocks, WM x WN waves.
// Register-staged double buffer: the global loads of K-block kb+1 are issued
// before the MFMAs of kb and written to the other LDS buffer after them (one
// barrier per K-block).  LDS rows are padded to BK+8 halfs so the 16 rows a
// ds_read_b128 lane group reads fall on 16 distinct 16-byte bank slots.
// Out-of-image taps (padding) and K padding load from a valid address and are
// zeroed by a select: no divergent branches around loads.
// Blocks are remapped so that consecutive tiles of one M row-panel (sharing the
// A rows) run on the same XCD (blocks b, b+8, ... share an XCD's L2).
// --------------------------------------------------------------------------
template <int BM, int BN, int BK, int WM, int WN>
__global__ __launch_bounds__(64 * WM * WN) void conv_mfma_f16(ConvArgs a) {
  constexpr int NT = 64 * WM * WN;
  constexpr int KV = BK / 8;          // 16-byte vectors per row of a K-block
  constexpr int LS = BK + 8;          // padded LDS row (halfs)
  constexpr int RPP = NT / KV;        // rows covered by one pass of the block
  constexpr int VA = BM / RPP;
  constexpr int VB = BN >= RPP ? BN / RPP : 1;
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int TM = WTM / 16, TN = WTN / 16;
  static_assert(BM % RPP == 0, "BM must be a multiple of rows per pass");
  static_assert(BN < RPP || BN % RPP == 0, "BN must be a multiple of rows per pass");
  static_assert(TM >= 1 && TN >= 1, "wave tile too small");
  constexpr int BUF = (BM + BN) * LS;
  __shared__ __attribute__((aligned(16))) _Float16 smem[2 * BUF];

  const int tid = threadIdx.x;
  const int lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid - (wid / WN) * WN;
  // XCD-aware bijective remap of the 1-D grid, then N-fastest tile order
  const int nblk = gridDim.x;
  const int ntn = a.cout_pad / BN;
  int bid = blockIdx.x;
  {
    const int xcd = bid & 7, q = nblk >> 3, r = nblk & 7;
    bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  }
  const int m_base = (bid / ntn) * BM;
  const int n_base = (bid - (bid / ntn) * ntn) * BN;

  const int kvl = tid % KV;
  const int r0 = tid / KV;
  const bool b_loader = BN >= RPP || r0 < BN;

  const _Float16* __restrict__ in = (const _Float16*)a.in + a.in_co;
  const _Float16* __restrict__ wt = (const _Float16*)a.w + (size_t)(n_base + (b_loader ? r0 : 0)) * a.kpad + kvl * 8;

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
  const int cvecs = a.cin >> 3;
  const int kvec_total = a.ks * a.ks * cvecs;
  const int nk = a.kpad / BK;
  const int ih = a.ih, iw = a.iw, ics = a.in_cs, ks = a.ks, kpad = a.kpad;

  u32x4 ra[VA], rb[VB];
  const u32x4 zero4 = {0u, 0u, 0u, 0u};

#define RTDM_GLOAD(kb_)                                                                  \
  {                                                                                      \
    const int kv = (kb_) * KV + kvl;                                                     \
    const bool kval = kv < kvec_total;                                                   \
    const int tap = kval ? kv / cvecs : 0;                                               \
    const int cv = kv - tap * cvecs;                                                     \
    const int kh = tap / ks;                                                             \
    const int kw = tap - kh * ks;                                                        \
    _Pragma("unroll") for (int i = 0; i < VA; ++i) {                                     \
      const int iy = a_iy[i] + kh, ix = a_ix[i] + kw;                                    \
      const bool v = kval && (unsigned)iy < (unsigned)ih && (unsigned)ix < (unsigned)iw; \
      const size_t off = v ? (size_t)(a_pix[i] + iy * iw + ix) * ics + cv * 8 : 0;       \
      const u32x4 t = *(const u32x4*)(in + off);                                         \
      ra[i] = v ? t : zero4;                                                             \
    }                                                                                    \
    _Pragma("unroll") for (int j = 0; j < VB; ++j)                                       \
      rb[j] = *(const u32x4*)(wt + (size_t)j * RPP * kpad + (kb_) * BK);                 \
  }
#define RTDM_SSTORE(buf_)                                                                \
  {                                                                                      \
    _Float16* As_ = smem + (buf_) * BUF;                                                 \
    _Float16* Bs_ = As_ + BM * LS;                                                       \
    _Pragma("unroll") for (int i = 0; i < VA; ++i)                                       \
      *(u32x4*)(As_ + (r0 + i * RPP) * LS + kvl * 8) = ra[i];                            \
    if (b_loader) {                                                                      \
      _Pragma("unroll") for (int j = 0; j < VB; ++j)                                     \
        *(u32x4*)(Bs_ + (r0 + j * RPP) * LS + kvl * 8) = rb[j];                          \
    }                                                                                    \
  }

  f4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};

  RTDM_GLOAD(0);
  RTDM_SSTORE(0);
  __syncthreads();

  const int frow = lane & 15;
  const int fk = (lane >> 4) * 8;
  for (int kb = 0; kb < nk; ++kb) {
    const int buf = kb & 1;
    const bool more = kb + 1 < nk;
    if (more) RTDM_GLOAD(kb + 1);
    const _Float16* As = smem + buf * BUF + (wm * WTM + frow) * LS + fk;
    const _Float16* Bs = smem + buf * BUF + BM * LS + (wn * WTN + frow) * LS + fk;
#pragma unroll
    for (int kk = 0; kk < BK / 32; ++kk) {
      h8 af[TM], bf[TN];
#pragma unroll
      for (int tm = 0; tm < TM; ++tm) af[tm] = *(const h8*)(As + tm * 16 * LS + kk * 32);
#pragma unroll
      for (int tn = 0; tn < TN; ++tn) bf[tn] = *(const h8*)(Bs + tn * 16 * LS + kk * 32);
#pragma unroll
      for (int tm = 0; tm < TM; ++tm)
#pragma unroll
        for (int tn = 0; tn < TN; ++tn)
          acc[tm][tn] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[tm], bf[tn], acc[tm][tn], 0, 0, 0);
    }
    if (more) RTDM_SSTORE(buf ^ 1);
    __syncthreads();
  }
#undef RTDM_GLOAD
#undef RTDM_SSTORE

  // ---- epilogue: accumulators -> LDS C tile -> 4 rows x 8 channels per thread ----
  constexpr int CSTR = BN + 4;
  static_assert(BM * CSTR * 4 <= 2 * BUF * 2, "C tile does not fit the staging LDS");
  float* Cs = reinterpret_cast<float*>(smem);
  const int rq = (lane >> 4) * 4;
#pragma unroll
  for (int tm = 0; tm < TM; ++tm)
#pragma unroll
    for (int tn = 0; tn < TN; ++tn) {
      const int row = wm * WTM + tm * 16 + rq;
      const int col = wn * WTN + tn * 16 + frow;
#pragma unroll
      for (int j = 0; j < 4; ++j) Cs[(row + j) * CSTR + col] = acc[tm][tn][j];
    }
  __syncthreads();
  constexpr int CG = BN / 8;
  constexpr int UNITS = (BM / 4) * CG;
  for (int u = tid; u < UNITS; u += NT) {
    const int q = u / CG, g = u - (u / CG) * CG;
    const int m0 = m_base + q * 4, c0 = n_base + g * 8;
    if (m0 >= a.M || c0 >= a.cout) continue;
    float v[4][8];
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int j = 0; j < 8; ++j) v[r][j] = Cs[(q * 4 + r) * CSTR + g * 8 + j];
    epi_vec8(a, m0, c0, v);
  }
}

// --------------------------------------------------------------------------
// fp16 MFMA stem: Cin = 3, 3x3, stride 1, pad 1 (the Darknet first conv, fed by
// uint8 frames or NCHW model inputs).  One block = one output row (linear M
// order) or one 2-row quad band (quad order, fused 2x2 maxpool).  The input
// rows the band needs are staged into LDS as fp16 (uint8 is exact in fp16; the
// /255 is folded into the uint8 weight copy), then every lane gathers its
// 8-element K slice (k = (kh*3 + kw)*3 + c, 27 padded to 32) for one
// v_mfma_f32_16x16x32_f16 per 16 output pixels per 16 output channels.
// --------------------------------------------------------------------------
constexpr int kStemMaxW = 1024;
__global__ __launch_bounds__(256) void conv_stem_mfma(ConvArgs a) {
  __shared__ _Float16 tile[4 * (kStemMaxW + 2) * 3];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int R = a.quad ? 2 : 1;                 // output rows per block
  const int rows_per_img = a.quad ? a.qh : a.oh;
  const int n = blockIdx.x / rows_per_img;
  const int yb = blockIdx.x - n * rows_per_img;  // quad row or output row
  const int y0 = yb * R;
  const int W = a.iw, H = a.ih;
  const int TW = W + 2;
  // ---- stage input rows y0-1 .. y0+R into LDS (zero border) ----
  const int nrow = R + 2;
  if (a.in_kind == IN_FRAME_U8 && (W * 3) % 16 == 0) {
    // 16-byte loads of whole frame rows (uint8 is exact in fp16)
    const int vpr = W * 3 / 16;
    for (int idx = tid; idx < nrow * vpr; idx += 256) {
      const int rr = idx / vpr, v = idx - (idx / vpr) * vpr;
      const int y = y0 - 1 + rr;
      u32x4 d = {0u, 0u, 0u, 0u};
      if ((unsigned)y < (unsigned)H) d = *(const u32x4*)((const uint8_t*)a.in + ((size_t)(n * H + y) * W) * 3 + v * 16);
      _Float16* dst = tile + (rr * TW + 1) * 3 + v * 16;
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int b = 0; b < 4; ++b) dst[q * 4 + b] = (_Float16)(float)((d[q] >> (8 * b)) & 0xffu);
    }
    for (int idx = tid; idx < nrow * 6; idx += 256) {  // left / right zero border
      const int rr = idx / 6, e = idx - (idx / 6) * 6;
      tile[(rr * TW + (e < 3 ? 0 : W + 1)) * 3 + (e % 3)] = (_Float16)0.f;
    }
  } else {
    for (int idx = tid; idx < nrow * TW * 3; idx += 256) {
      const int c = idx % 3;
      const int t = idx / 3;
      const int x = t % TW - 1;
      const int y = t / TW + y0 - 1;
      float v = 0.f;
      if ((unsigned)y < (unsigned)H && (unsigned)x < (unsigned)W) {
        if (a.in_kind == IN_FRAME_U8)
          v = (float)((const uint8_t*)a.in)[((size_t)(n * H + y) * W + x) * 3 + c];
        else if (a.in_kind == IN_NCHW_F32)
          v = ((const float*)a.in)[(((size_t)n * 3 + c) * H + y) * W + x];
        else
          v = (float)((const _Float16*)a.in)[(((size_t)n * 3 + c) * H + y) * W + x];
      }
      tile[idx] = (_Float16)v;
    }
  }
  // uint8 frames enter as 0..255: apply the /255 of detect.py:82 to the fp32 accumulator
  const float in_scale = a.in_kind == IN_FRAME_U8 ? 1.f / 255.f : 1.f;
  // ---- per-lane K slice: 8 LDS offsets relative to the pixel's window ----
  const int kg = (lane >> 4) * 8;
  int koff[8];
  bool kval[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int k = kg + j;
    kval[j] = k < 27;
    const int tap = k / 3, c = k - (k / 3) * 3;
    const int kh = tap / 3, kw = tap - (tap / 3) * 3;
    koff[j] = kval[j] ? (kh * TW + kw) * 3 + c : 0;
  }
  const _Float16* wsrc = (const _Float16*)a.w_stem;
  const int ntn = a.cout_pad / 16;
  __syncthreads();
  const int r = lane & 15;
  int groups;  // 16-pixel MFMA row groups in this block
  if (a.quad)
    groups = (a.qw + 3) / 4;
  else
    groups = (a.ow + 15) / 16;
  for (int g = wid; g < groups; g += 4) {
    int py, px;  // pixel of this lane's A row, relative to the band
    if (a.quad) {
      const int qx = g * 4 + (r >> 2), d = r & 3;
      py = d >> 1;
      px = 2 * qx + (d & 1);
    } else {
      py = 0;
      px = g * 16 + r;
    }
    const bool pv = px < a.ow;
    const int base = (py * TW + (pv ? px : 0)) * 3;
    h8 af;
#pragma unroll
    for (int j = 0; j < 8; ++j) af[j] = kval[j] ? tile[base + koff[j]] : (_Float16)0.f;
    // epilogue rows of this lane: 4 consecutive M rows
    int m0, nvalid;
    if (a.quad) {
      const int qx = g * 4 + (lane >> 4);
      m0 = ((n * a.qh + yb) * a.qw + qx) * 4;
      nvalid = qx < a.qw ? 4 : 0;
    } else {
      const int ox = g * 16 + (lane >> 4) * 4;
      m0 = (n * a.oh + y0) * a.ow + ox;
      nvalid = a.ow - ox < 4 ? (a.ow - ox > 0 ? a.ow - ox : 0) : 4;
    }
    for (int tn = 0; tn < ntn; ++tn) {
      const h8 bf = *(const h8*)(wsrc + (size_t)(tn * 16 + r) * 32 + kg);
      f4 acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(af, bf, f4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0) * in_scale;
      const int c = tn * 16 + r;
      if (c < a.cout && nvalid == 4) epi4<_Float16>(a, m0, c, acc);
      else if (c < a.cout && nvalid > 0) {
        f4 t = acc;
        ConvArgs b = a;
        b.M = m0 + nvalid;  // mask rows beyond the image row
        epi4<_Float16>(b, m0, c, t);
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
      epi4<T>(a, m0, c, f4{acc[0][j], acc[1][j], acc[2][j], acc[3][j]});
    }
  }
}

// --------------------------------------------------------------------------
template <int BM, int BN, int BK, int WM, int WN>
static void launch_mfma(const ConvArgs& a, hipStream_t s) {
  RTDM_REQUIRE(a.cout_pad % BN == 0, RTDM_E_INVALID, "conv: cout_pad not a multiple of BN");
  RTDM_REQUIRE(a.kpad % BK == 0, RTDM_E_INVALID, "conv: kpad not a multiple of BK");
  const int64_t nblk = (int64_t)((a.M + BM - 1) / BM) * (a.cout_pad / BN);
  RTDM_REQUIRE(nblk < (1ll << 31), RTDM_E_CAPACITY, "conv: grid too large");
  hipLaunchKernelGGL((conv_mfma_f16<BM, BN, BK, WM, WN>), dim3((unsigned)nblk), dim3(64 * WM * WN), 0, s, a);
}

static bool mfma_ok(const ConvArgs& a) {
  return a.in_kind == IN_NHWC && a.cin % 8 == 0 && a.in_cs % 8 == 0 && a.in_co % 8 == 0;
}

static bool stem_ok(const ConvArgs& a) {
  return a.w_stem && a.in_kind != IN_NHWC && a.cin == 3 && a.ks == 3 && a.stride == 1 && a.pad == 1 &&
         a.iw <= kStemMaxW && a.oh == a.ih && a.ow == a.iw && a.cout_pad % 16 == 0 &&
         (a.quad ? (a.oh % 2 == 0 && a.ow % 2 == 0) : true);
}

const char* conv_kernel_name(const ConvArgs& a, int dtype) {
  if (dtype == RTDM_F16 && stem_ok(a)) return "conv_stem_mfma";
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
  if (dtype == RTDM_F16 && stem_ok(a)) {
    const int blocks = a.n * (a.quad ? a.qh : a.oh);
    hipLaunchKernelGGL(conv_stem_mfma, dim3(blocks), dim3(256), 0, s, a);
  } else if (dtype == RTDM_F16 && !a.w_f32) {
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
