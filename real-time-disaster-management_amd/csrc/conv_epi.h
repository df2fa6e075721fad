// Device helpers shared by the implicit-GEMM convolution kernels (conv.hip,
// conv_pipe.hip): fragment vector types, GEMM row -> pixel mapping and the
// fused conv epilogues (bias -> activation -> BN affine -> residual -> full /
// pooled / upsampled stores / YOLO decode).
#pragma once

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
        if (e.raw) {
          o = x;
        } else if (k < 2) {
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
      // (anchor, field) of channel c0 by one division, then stepped per channel;
      // fp16 path: hardware exp / reciprocal (well inside the fp16 tolerance)
      int ai = c0 / e.no, k = c0 - ai * e.no;
      const size_t pix_io = (size_t)n * e.io_rows + e.io_off + (size_t)oy * a.ow + ox;
      const size_t plane = (size_t)a.oh * a.ow;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        if (j < nc) {
          float o;
          if (e.raw)
            o = x[j];
          else if (k < 2)
            o = (__frcp_rn(1.f + __expf(-x[j])) + (float)(k == 0 ? ox : oy)) * e.ystride;
          else if (k < 4)
            o = (__expf(x[j]) * e.anchor_vec[2 * ai + (k - 2)]) * e.ystride;
          else
            o = __frcp_rn(1.f + __expf(-x[j]));
          e.io[(pix_io + (size_t)ai * plane) * e.no + k] = o;
        }
        if (++k == e.no) {
          k = 0;
          ++ai;
        }
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

// Lean variant of epi_vec8 for the common Darknet conv (bias -> leaky/linear ->
// optional scale/shift -> full / 2x2-pool / x2-upsample outputs), with every view
// 8-channel aligned and 8 valid channels (checked on the host by epi_lean_ok).  No
// residual, swish or YOLO decode paths: the generic epilogue compiles to ~7k
// instructions, and fetching them cold at every tile's end cost ~10 us per tile
// round in the MFMA-bound convs (tools/ab_conv.py modes 8-10).
// RES: the fused shortcut add (weightedFeatureFusion, models.py:135-155) of a same-shape
// 8-aligned residual view, in epi_vec8's order (act -> affine -> + residual).
template <bool RES = false>
__device__ __forceinline__ void epi_vec8_lean(const ConvArgs& a, int m0, int c0, const float (&v)[4][8],
                                              const float (&bias)[8], const float (&sc)[8], const float (&sh)[8]) {
  const Epilogue& e = a.e;
  float pmax[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) pmax[j] = -INFINITY;
  int pn, poy, pox;
  row_to_pix(a, m0, pn, poy, pox);
  const float slp = e.act == ACT_LEAKY ? e.slope : 1.f;  // max(t, slope t), as pipe_epi_regs
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int m = m0 + r;
    if (m >= a.M) continue;
    int n, oy, ox;
    row_pix4(a, m0, r, pn, poy, pox, n, oy, ox);
    const size_t pix = ((size_t)n * a.oh + oy) * a.ow + ox;
    h8v rv;
    if constexpr (RES) rv = *(const h8v*)((const _Float16*)e.res.ptr + pix * e.res.cs + e.res.co + c0);
    h8v hv;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float t = v[r][j] + bias[j];
      t = fmaxf(t, t * slp);
      t = t * sc[j] + sh[j];
      if constexpr (RES) t += (float)rv[j];
      hv[j] = (_Float16)t;
      pmax[j] = fmaxf(pmax[j], t);
    }
    if (e.full.ptr) *(h8v*)((_Float16*)e.full.ptr + pix * e.full.cs + e.full.co + c0) = hv;
    if (e.up.ptr) {
      const int uw = a.ow * 2;
      const size_t u0 = ((size_t)n * a.oh * 2 + 2 * oy) * uw + 2 * ox;
      _Float16* up = (_Float16*)e.up.ptr + e.up.co + c0;
      *(h8v*)(up + u0 * e.up.cs) = hv;
      *(h8v*)(up + (u0 + 1) * e.up.cs) = hv;
      *(h8v*)(up + (u0 + uw) * e.up.cs) = hv;
      *(h8v*)(up + (u0 + uw + 1) * e.up.cs) = hv;
    }
  }
  if (e.pool.ptr && a.quad && m0 < a.M) {
    const size_t pp = ((size_t)pn * a.qh + (poy >> 1)) * a.qw + (pox >> 1);
    h8v pv;
#pragma unroll
    for (int j = 0; j < 8; ++j) pv[j] = (_Float16)pmax[j];
    *(h8v*)((_Float16*)e.pool.ptr + pp * e.pool.cs + e.pool.co + c0) = pv;
  }
}

// YOLO-head variant of epi_vec8: bias -> activation -> optional scale/shift -> decode
// (or raw) into io, the only output.  Same operations, in the same order, as the io
// branch of epi_vec8 (bit-identical), without the code of the other branches.
// Channel constants of the 8 channels c0..c0+7: bias, scale, shift and the anchor of
// the w/h channels (epi_io_consts; conv_pipe loads them at the tile's start).
__device__ __forceinline__ void epi_io_consts(const ConvArgs& a, int c0, float (&bias)[8], float (&sc)[8],
                                              float (&sh)[8], float (&anc)[8]) {
  const Epilogue& e = a.e;
  const int nc = a.cout - c0 < 8 ? a.cout - c0 : 8;
  int ai = c0 / e.no, k = c0 - ai * e.no;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const bool cv = j < nc;
    bias[j] = (e.bias && cv) ? e.bias[c0 + j] : 0.f;
    sc[j] = (e.scale && cv) ? e.scale[c0 + j] : 1.f;
    sh[j] = (e.scale && cv) ? e.shift[c0 + j] : 0.f;
    anc[j] = (cv && !e.raw && (k == 2 || k == 3)) ? e.anchor_vec[2 * ai + (k - 2)] : 0.f;
    if (++k == e.no) {
      k = 0;
      ++ai;
    }
  }
}

__device__ __forceinline__ void epi_vec8_io(const ConvArgs& a, int m0, int c0, const float (&v)[4][8],
                                            const float (&bias)[8], const float (&sc)[8], const float (&sh)[8],
                                            const float (&anc)[8]) {
  const Epilogue& e = a.e;
  const int nc = a.cout - c0 < 8 ? a.cout - c0 : 8;
  int pn, poy, pox;
  row_to_pix(a, m0, pn, poy, pox);
  const size_t plane = (size_t)a.oh * a.ow;
  const int ai0 = c0 / e.no, k0 = c0 - ai0 * e.no;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int m = m0 + r;
    if (m >= a.M) continue;
    int n, oy, ox;
    row_pix4(a, m0, r, pn, poy, pox, n, oy, ox);
    const size_t pix_io = (size_t)n * e.io_rows + e.io_off + (size_t)oy * a.ow + ox;
    int ai = ai0, k = k0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if (j < nc) {
        float t = v[r][j] + bias[j];
        if (e.act == ACT_LEAKY) t = t > 0.f ? t : t * e.slope;
        const float x = t * sc[j] + sh[j];
        float o;
        if (e.raw)
          o = x;
        else if (k < 2)
          o = (__frcp_rn(1.f + __expf(-x)) + (float)(k == 0 ? ox : oy)) * e.ystride;
        else if (k < 4)
          o = (__expf(x) * anc[j]) * e.ystride;
        else
          o = __frcp_rn(1.f + __expf(-x));
        e.io[(pix_io + (size_t)ai * plane) * e.no + k] = o;
      }
      if (++k == e.no) {
        k = 0;
        ++ai;
      }
    }
  }
}

// epi_vec8_io's arithmetic in place (v <- the io values of its 4 rows x 8 channels);
// the caller stores them (conv_pipe: coalesced per anchor plane)
__device__ __forceinline__ void epi_io_decode(const ConvArgs& a, int m0, int c0, float (&v)[4][8],
                                              const float (&bias)[8], const float (&sc)[8], const float (&sh)[8],
                                              const float (&anc)[8]) {
  const Epilogue& e = a.e;
  int pn, poy, pox;
  row_to_pix(a, m0, pn, poy, pox);
  const int ai0 = c0 / e.no, k0 = c0 - ai0 * e.no;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    int n, oy, ox;
    row_pix4(a, m0, r, pn, poy, pox, n, oy, ox);
    int k = k0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float t = v[r][j] + bias[j];
      if (e.act == ACT_LEAKY) t = t > 0.f ? t : t * e.slope;
      const float x = t * sc[j] + sh[j];
      float o;
      if (e.raw)
        o = x;
      else if (k < 2)
        o = (__frcp_rn(1.f + __expf(-x)) + (float)(k == 0 ? ox : oy)) * e.ystride;
      else if (k < 4)
        o = (__expf(x) * anc[j]) * e.ystride;
      else
        o = __frcp_rn(1.f + __expf(-x));
      v[r][j] = o;
      if (++k == e.no) k = 0;
    }
  }
}

__device__ __forceinline__ void epi_vec8_io(const ConvArgs& a, int m0, int c0, const float (&v)[4][8]) {
  float bias[8], sc[8], sh[8], anc[8];
  epi_io_consts(a, c0, bias, sc, sh, anc);
  epi_vec8_io(a, m0, c0, v, bias, sc, sh, anc);
}

inline bool epi_io_ok(const ConvArgs& a) {
  const Epilogue& e = a.e;
  return e.io && !e.res.ptr && !e.full.ptr && !e.pool.ptr && !e.up.ptr &&
         (e.act == ACT_LEAKY || e.act == ACT_LINEAR) && (!e.scale || e.shift);
}

inline bool epi_lean_ok(const ConvArgs& a, bool allow_res = false) {
  const Epilogue& e = a.e;
  if ((e.res.ptr && (!allow_res || ((e.res.cs | e.res.co) & 7) != 0)) || e.io ||
      (e.act != ACT_LEAKY && e.act != ACT_LINEAR) || a.cout % 8 != 0)
    return false;
  if (!e.bias || (e.scale && !e.shift)) return false;
  for (const View* v : {&e.full, &e.pool, &e.up})
    if (v->ptr && ((v->cs | v->co) & 7) != 0) return false;
  return !e.pool.ptr || a.quad;
}

typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef __attribute__((address_space(1))) void* gbl_ptr_t;

// Register epilogue of a lean conv_pipe / conv_wide tile (D^T accumulators: acc[tm][tn][r] =
// output channel n_base + wn*CW + tn*16 + 4g + r of GEMM row m_base + wm*RW + tm*16 + fr;
// RW / CW: rows / columns per wave).
// Same per-element operations, in the same order, as epi_vec8_lean.
// FIXED (cross-tile prefetch, see pipe_walk): the full-map output only (no pool / upsample,
// no BN affine),
// every store (and residual load) issued by every wave as a buffer op whose offset is out of
// range for invalid lanes, so the epilogue issues exactly pipe_epi_ops() vector-memory ops and
// the next tile can wait on its prefetched stage with an exact vmcnt.
template <bool RES, int FM, int FN>
__host__ __device__ constexpr int pipe_epi_ops() {
  return FM * FN * (RES ? 2 : 1);
}
template <bool RES, int FM, int FN, int RW, int CW, bool FIXED = false, typename AccT, int NDQ>
__device__ __forceinline__ void pipe_epi_regs(const ConvArgs& a, int m_base, int n_base, int wm, int wn, int lane,
                                              const AccT (&acc)[FM][FN], const f4 (&rb)[FN], const f4 (&dq4)[NDQ]) {
  constexpr bool I8 = !std::is_same_v<AccT, f4>;
  const Epilogue& e = a.e;
  const int fr = lane & 15, g = lane >> 4;
  // LeakyReLU as max(t, slope t): the planner's slopes are 0.1 / 0.01 (detector.cpp), for which
  // it equals t > 0 ? t : slope t on every non-NaN t (-0 included) without a compare + select;
  // linear layers take slope 1
  const float slp = e.act == ACT_LEAKY ? e.slope : 1.f;
  typedef _Float16 h4 __attribute__((ext_vector_type(4)));
  typedef int i2 __attribute__((ext_vector_type(2)));
  if constexpr (FIXED) {
    // byte offsets < 2^31 - 16 (pipe_pf_ok); 0x7FFFFFF8 is past num_records: no-op store / zero load
    const __amdgpu_buffer_rsrc_t rs_o =
        __builtin_amdgcn_make_buffer_rsrc((void*)((_Float16*)e.full.ptr + e.full.co), 0, 0x7FFFFFF0, 0x00020000);
    __amdgpu_buffer_rsrc_t rs_r = rs_o;
    if constexpr (RES)
      rs_r = __builtin_amdgcn_make_buffer_rsrc((void*)((const _Float16*)e.res.ptr + e.res.co), 0, 0x7FFFFFF0,
                                               0x00020000);
#pragma unroll
    for (int tm = 0; tm < FM; ++tm) {
      const int m = m_base + wm * RW + tm * 16 + fr;
      const bool mv = m < a.M;
      int n = 0, oy = 0, ox = 0;
      if (mv) row_to_pix(a, m, n, oy, ox);
      const int pix = (n * a.oh + oy) * a.ow + ox;
#pragma unroll
      for (int tn = 0; tn < FN; ++tn) {
        const int c0 = n_base + wn * CW + tn * 16 + 4 * g;
        const bool ok = mv && c0 < a.cout;
        f4 t;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          if constexpr (I8)
            t[r] = (float)acc[tm][tn][r] * dq4[NDQ == FN ? tn : 0][r];
          else
            t[r] = acc[tm][tn][r];
          t[r] = t[r] + rb[tn][r];
          t[r] = fmaxf(t[r], t[r] * slp);
        }
        if constexpr (RES) {
          const int ro = ok ? (pix * e.res.cs + c0) * 2 : 0x7FFFFFF8;
          const h4 rv = __builtin_bit_cast(h4, __builtin_amdgcn_raw_buffer_load_b64(rs_r, ro, 0, 0));
          // the unconditional add would contract with the LeakyReLU product into
          // fma(t, slope, r) (fp-contract=fast); the other epilogues round t * slope first
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            asm volatile("" : "+v"(t[r]));
            t[r] += (float)rv[r];
          }
        }
        h4 hv;
#pragma unroll
        for (int r = 0; r < 4; ++r) hv[r] = (_Float16)t[r];
        const int oo = ok ? (pix * e.full.cs + c0) * 2 : 0x7FFFFFF8;
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(i2, hv), rs_o, oo, 0, 0);
      }
    }
    return;
  }
#pragma unroll
  for (int tm = 0; tm < FM; ++tm) {
    const int m = m_base + wm * RW + tm * 16 + fr;
    const bool mv = m < a.M;
    int n = 0, oy = 0, ox = 0;
    if (mv) row_to_pix(a, m, n, oy, ox);
    const size_t pix = ((size_t)n * a.oh + oy) * a.ow + ox;
#pragma unroll
    for (int tn = 0; tn < FN; ++tn) {
      const int c0 = n_base + wn * CW + tn * 16 + 4 * g;
      const bool cv = c0 < a.cout;  // cout % 8 == 0 (epi_lean_ok): all 4 or none
      f4 t;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        if constexpr (I8)
          t[r] = (float)acc[tm][tn][r] * dq4[NDQ == FN ? tn : 0][r];
        else
          t[r] = acc[tm][tn][r];
        t[r] = t[r] + rb[tn][r];
        t[r] = fmaxf(t[r], t[r] * slp);
      }
      if (e.scale && cv) {
        const f4 sc = *(const f4*)(e.scale + c0), sh = *(const f4*)(e.shift + c0);
#pragma unroll
        for (int r = 0; r < 4; ++r) t[r] = t[r] * sc[r] + sh[r];
      }
      if constexpr (RES) {
        if (mv && cv) {
          const h4 rv = *(const h4*)((const _Float16*)e.res.ptr + pix * e.res.cs + e.res.co + c0);
#pragma unroll
          for (int r = 0; r < 4; ++r) t[r] += (float)rv[r];
        }
      }
      h4 hv;
#pragma unroll
      for (int r = 0; r < 4; ++r) hv[r] = (_Float16)t[r];
      if (mv && cv) {
        if (e.full.ptr) *(h4*)((_Float16*)e.full.ptr + pix * e.full.cs + e.full.co + c0) = hv;
        if (e.up.ptr) {
          const int uw = a.ow * 2;
          const size_t u0 = ((size_t)n * a.oh * 2 + 2 * oy) * uw + 2 * ox;
          _Float16* up = (_Float16*)e.up.ptr + e.up.co + c0;
          *(h4*)(up + u0 * e.up.cs) = hv;
          *(h4*)(up + (u0 + 1) * e.up.cs) = hv;
          *(h4*)(up + (u0 + uw) * e.up.cs) = hv;
          *(h4*)(up + (u0 + uw + 1) * e.up.cs) = hv;
        }
      }
      if (e.pool.ptr) {  // quad order: rows 4q..4q+3 = lanes fr 4q..4q+3 (a DPP quad)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float v = t[r];
          v = fmaxf(v, __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0xB1, 0xF, 0xF, false)));
          v = fmaxf(v, __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x4E, 0xF, 0xF, false)));
          t[r] = v;
        }
        if (mv && cv && (fr & 3) == 0) {
          const size_t pp = ((size_t)n * a.qh + (oy >> 1)) * a.qw + (ox >> 1);
          h4 pv;
#pragma unroll
          for (int r = 0; r < 4; ++r) pv[r] = (_Float16)t[r];
          *(h4*)((_Float16*)e.pool.ptr + pp * e.pool.cs + e.pool.co + c0) = pv;
        }
      }
    }
  }
}


}  // namespace rtdm
