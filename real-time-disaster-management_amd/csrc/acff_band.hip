// acff_band: one ACFF stage per launch over output row bands, for the classifier's
// small maps (ErNET acff3..acff6, Squeeze-ErNET acff3 / acff4, RedConv acff4), with the
// classifier tail fused into the last stage.
//
// disaster_detection/model/acff.py:37-59 per stage: three depthwise 3x3 branches
// (dilation 1 / 2 / 3, padding 0 / 1 / 2, + bias, acff.py:25-30) -> channel concat
// (acff.py:46) -> 1x1 conv (+bias) -> LeakyReLU(0.01) -> BatchNorm affine (eval) ->
// (the 2x2 MaxPool that follows acff3, ernet.py:33 / squeeze_ernet.py:31).  The last
// stage continues into the tail (ernet.py:38-45, squeeze_ernet.py:33-41): conv2 1x1 -> 5,
// AvgPool 5 (count_include_pad), NCHW flatten, Linear, Softmax.
//
// Why bands: acff_chain ran the whole small-map suffix in ONE workgroup per image (64 of
// 256 CUs at b64, 8 at b8) and spent ~60 % of it in the depthwise taps of all the
// image's pixels on one CU.  Here a workgroup owns `rows` output rows of one image and
// every output channel, so the depthwise work of a stage spreads over n x bands
// workgroups with no recomputation (a depthwise output is per pixel; only the input
// halo rows are re-read, from L2).  The maps between stages are a few MB (L2 / MALL
// resident); each stage is one launch of >= 40 workgroups at b8, hundreds at b64.
//
// Per workgroup (512 threads, 8 waves):
//   1. the band's input rows y0-2 .. y0+rows+3, columns -2 .. w+1 (the radius-3 halo of
//      the dilated branches, zero outside the image = their padding) -> LDS; meanwhile
//      each thread's depthwise taps (one branch x 8 channels: 72 fp32 + 8 biases) and the
//      first 1x1 weight fragments load into registers;
//   2. depthwise on VALU: a thread keeps one (branch, 8-channel group) and walks pixels;
//      per pixel bias then the 9 taps in (kh, kw) order as fp32 FMAs of fp16 inputs
//      (v_fma_mix_f32), rounded once to fp16 into the A tile [M][3 C] (k = branch*C + c,
//      torch.cat's order) -- acff_chain's exact operation sequence;
//   3. 1x1 GEMM [M x 3C] x [3C x cout] on v_mfma_f32_16x16x32_f16, k-steps of 32 in K order
//      (acff_chain's accumulation order), B fragments from the L2-resident packed weights
//      through a register ring issued ahead of use;
//   4. epilogue bias -> LeakyReLU -> BN affine (fmaf, acff_chain's) -> fp16 NHWC store,
//      or the 2x2 max of a quad (M in quad order: a lane's 4 accumulator rows are one
//      quad), or (tail) the fp16 map into LDS and the tail on it.
// Results are bit-identical to acff_chain on the non-pooled stages + tail
// (tests/test_gpu_parity.py::test_acff_band_bit_identical_to_chain).
//
// Measured (r06c, one box, alternating): OPT-IN, not the default.  Per launch it is the
// faster schedule at b8 (acff3..acff6 + tail 63 us against 80 for acff_persist + the
// chain), but in the two-stage bench it loses at b64 (46.1 / 45.7 k frames/s against
// 47.2 / 47.0 k with the chain) and ties at b8 (33.6 / 33.4 k against 33.3 / 33.5 k):
// with two batches in flight what a classifier launch costs is its CU-time, and the
// chain's 64 long workgroups hold 64 CUs x 62 us (4 CU-ms) where the banded launches hold
// the whole chip (32 CU-ms for acff3..acff6) -- each band workgroup is latency-bound
// (staging -> barrier -> depthwise -> barrier -> GEMM, 235 VGPRs: one 8-wave group per
// CU).  rtdm_set_tuning("acff_band", 1 | 2) selects it.
#include "common.h"

#include <algorithm>

namespace rtdm {

namespace {
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

constexpr int kBandThreads = 512;
constexpr int kBandKPre = 12;  // 1x1 weight k-steps in flight per wave (all of them for cin <= 128)

// fp32 = w (f32) * x (f16, low / high half of a packed pair) + acc: the exact cvt + fma in
// one VOP3P op
__device__ __forceinline__ float bmix_lo(float w, uint32_t x2, float acc) {
  float d;
  asm("v_fma_mix_f32 %0, %1, %2, %3 op_sel_hi:[0,1,0]" : "=v"(d) : "v"(w), "v"(x2), "v"(acc));
  return d;
}
__device__ __forceinline__ float bmix_hi(float w, uint32_t x2, float acc) {
  float d;
  asm("v_fma_mix_f32 %0, %1, %2, %3 op_sel:[0,1,0] op_sel_hi:[0,1,0]" : "=v"(d) : "v"(w), "v"(x2), "v"(acc));
  return d;
}
}  // namespace

struct AcffBandArgs {
  const _Float16* in;
  int in_cs, in_co;
  int h, w, cin;       // input map (h x w x cin per image)
  int rows, bands;     // output rows per band, bands per image (grid = n * bands)
  int oh_eff;          // output rows computed: oh, or 2 * (oh / 2) when pooled
  int halo_bytes;      // LDS offset of the A tile
  const float* dw_wt;  // [3][9][cin]
  const float* dw_b;   // [3][cin]
  const _Float16* pw;  // [cout_pad][kpad], k = branch * cin + c
  int kpad, cout, cout_pad;
  const float* bias;
  const float* scale;
  const float* shift;
  float slope;
  _Float16* out;       // NHWC [n][oh or oh/2][ow or ow/2][out_cs]
  int out_cs;
  // tail (TAIL: rows == oh, one band per image)
  const float* w2;     // [5][cout]
  int pool_pad, ph, pwid;
  const float* fcw;    // [5][5 * ph * pwid]
  const float* fcb;
  float* logits;
  float* probs;
};

// FMW: 16-row M tiles per wave; the 8 waves are WM (M) x WN (N) with WN = cout_pad / 32
// (every wave two 16-channel N tiles), WM = 8 / WN.
template <int FMW, bool POOL, bool TAIL>
__global__ __launch_bounds__(kBandThreads) void acff_band(AcffBandArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char band_lds[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, g = lane >> 4;
  const int C = a.cin, CG = C >> 3, PS = C + 8;
  const int W = a.w, OW = W - 2, HWc = W + 4, HR = a.rows + 6;
  const int img = blockIdx.x / a.bands, band = blockIdx.x - img * a.bands;
  const int y0 = band * a.rows;
  const int nrows = min(a.rows, a.oh_eff - y0);
  const int OWq = OW >> 1;                                  // quads per pooled row
  const int M = POOL ? (nrows >> 1) * OWq * 4 : nrows * OW;  // GEMM rows of this band
  const int K = 3 * C, AS = K + 8, nks = K >> 5;
  _Float16* X = (_Float16*)band_lds;                     // halo [HR][HWc][PS]
  _Float16* At = (_Float16*)(band_lds + a.halo_bytes);   // A tile [WM * FMW * 16][AS]

  // ---- 1x1 weight fragments of this wave (issued first: L2 latency under the staging) ----
  const int WN = a.cout_pad >> 5, WM = 8 / WN;
  const int wm = wid / WN, wn = wid - wm * WN;
  const int n0 = wn * 32;
  const _Float16* wrow = a.pw + (size_t)(n0 + fr) * a.kpad + g * 8;
  h8 bq[kBandKPre][2];
#pragma unroll
  for (int s = 0; s < kBandKPre; ++s)
    if (s < nks) {
      bq[s][0] = *(const h8*)(wrow + s * 32);
      bq[s][1] = *(const h8*)(wrow + (size_t)16 * a.kpad + s * 32);
    }

  // epilogue constants of this lane's two channels (loaded now: no wait after the GEMM)
  float e_b[2], e_s[2], e_t[2];
  bool e_ok[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int c = n0 + j * 16 + fr;
    e_ok[j] = c < a.cout;
    e_b[j] = e_ok[j] ? a.bias[c] : 0.f;
    e_s[j] = e_ok[j] && a.scale ? a.scale[c] : 1.f;
    e_t[j] = e_ok[j] && a.scale ? a.shift[c] : 0.f;
  }

  // ---- this thread's depthwise item set: one (branch, 8-channel group), pixels p0, p0 + pstep ----
  const int combos = 3 * CG;
  const int pstep = kBandThreads / combos;
  const int combo = tid % combos, p0 = tid / combos;
  const int br = combo / CG, gv = combo - br * CG;
  const bool dw_on = p0 < pstep;
  f4 wk[9][2], bk[2];
  if (dw_on) {
    const float* wb = a.dw_wt + (size_t)br * 9 * C + gv * 8;
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      wk[t][0] = *(const f4*)(wb + (size_t)t * C);
      wk[t][1] = *(const f4*)(wb + (size_t)t * C + 4);
    }
    bk[0] = *(const f4*)(a.dw_b + br * C + gv * 8);
    bk[1] = *(const f4*)(a.dw_b + br * C + gv * 8 + 4);
  }

  // ---- stage the band's input halo (zero outside the image) ----
  {
    const _Float16* src = a.in + (size_t)img * a.h * W * a.in_cs + a.in_co;
    const int nvec = HR * HWc * CG;
    for (int i = tid; i < nvec; i += kBandThreads) {
      const int pix = i / CG, v = i - pix * CG;
      const int r = pix / HWc, c = pix - r * HWc;
      const int y = y0 - 2 + r, x = c - 2;
      u32x4 d = {0u, 0u, 0u, 0u};
      if ((unsigned)y < (unsigned)a.h && (unsigned)x < (unsigned)W)
        d = *(const u32x4*)(src + ((size_t)y * W + x) * a.in_cs + v * 8);
      *(u32x4*)(X + (size_t)pix * PS + v * 8) = d;
    }
    // A rows past M (MFMA padding rows; their outputs are never stored): zero
    const int mrows = WM * FMW * 16;
    for (int i = tid; i < (mrows - M) * (K >> 3); i += kBandThreads) {
      const int r = M + i / (K >> 3), v = i - (i / (K >> 3)) * (K >> 3);
      *(u32x4*)(At + (size_t)r * AS + v * 8) = u32x4{0u, 0u, 0u, 0u};
    }
  }
  __syncthreads();

  // ---- depthwise -> A tile ----
  if (dw_on) {
    const int d = br + 1;
    auto item = [&](int m, int oy, int ox) {  // oy, ox: band-relative output pixel
      float t[8];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        t[j] = bk[0][j];
        t[4 + j] = bk[1][j];
      }
#pragma unroll
      for (int kh = 0; kh < 3; ++kh)
#pragma unroll
        for (int kw = 0; kw < 3; ++kw) {
          const int hr = oy + 3 + (kh - 1) * d, hc = ox + 3 + (kw - 1) * d;
          const u32x4 xv = *(const u32x4*)(X + (size_t)(hr * HWc + hc) * PS + gv * 8);
          const f4& w0 = wk[kh * 3 + kw][0];
          const f4& w1 = wk[kh * 3 + kw][1];
          t[0] = bmix_lo(w0[0], xv[0], t[0]);
          t[1] = bmix_hi(w0[1], xv[0], t[1]);
          t[2] = bmix_lo(w0[2], xv[1], t[2]);
          t[3] = bmix_hi(w0[3], xv[1], t[3]);
          t[4] = bmix_lo(w1[0], xv[2], t[4]);
          t[5] = bmix_hi(w1[1], xv[2], t[5]);
          t[6] = bmix_lo(w1[2], xv[3], t[6]);
          t[7] = bmix_hi(w1[3], xv[3], t[7]);
        }
      h8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) asm volatile("" : "+v"(t[j]));  // (each f32 sum rounds on its own)
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = (_Float16)t[j];
      *(h8*)(At + (size_t)m * AS + br * C + gv * 8) = o;
    };
    if constexpr (POOL) {
      // quads q = (pooled row, pooled column) of the band; M row 4 q + (dy * 2 + dx)
      const int nq = M >> 2;
      int qy = p0 / OWq, qx = p0 - (p0 / OWq) * OWq;
      const int dq = pstep / OWq, dr = pstep - dq * OWq;
      for (int q = p0; q < nq; q += pstep) {
#pragma unroll
        for (int e = 0; e < 4; ++e) item(4 * q + e, 2 * qy + (e >> 1), 2 * qx + (e & 1));
        qx += dr;
        qy += dq;
        if (qx >= OWq) {
          qx -= OWq;
          ++qy;
        }
      }
    } else {
      int oy = p0 / OW, ox = p0 - (p0 / OW) * OW;
      const int dq = pstep / OW, dr = pstep - dq * OW;
      for (int m = p0; m < M; m += pstep) {
        item(m, oy, ox);
        ox += dr;
        oy += dq;
        if (ox >= OW) {
          ox -= OW;
          ++oy;
        }
      }
    }
  }
  __syncthreads();

  // ---- 1x1 GEMM: this wave's FMW M tiles x 2 N tiles over k = 0 .. 3C ----
  f4 acc[FMW][2];
#pragma unroll
  for (int i = 0; i < FMW; ++i) acc[i][0] = acc[i][1] = f4{0.f, 0.f, 0.f, 0.f};
  const int mt0 = wm * FMW;
  const _Float16* arow = At + (size_t)(mt0 * 16 + fr) * AS + g * 8;
  for (int k0 = 0; k0 < nks; k0 += kBandKPre) {
#pragma unroll
    for (int s = 0; s < kBandKPre; ++s) {
      const int ks = k0 + s;
      if (ks < nks) {
        h8 af[FMW];
#pragma unroll
        for (int i = 0; i < FMW; ++i) af[i] = *(const h8*)(arow + (size_t)i * 16 * AS + ks * 32);
#pragma unroll
        for (int i = 0; i < FMW; ++i) {
          acc[i][0] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[i], bq[s][0], acc[i][0], 0, 0, 0);
          acc[i][1] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[i], bq[s][1], acc[i][1], 0, 0, 0);
        }
        if (ks + kBandKPre < nks) {
          bq[s][0] = *(const h8*)(wrow + (ks + kBandKPre) * 32);
          bq[s][1] = *(const h8*)(wrow + (size_t)16 * a.kpad + (ks + kBandKPre) * 32);
        }
      }
    }
  }

  // ---- epilogue: bias -> LeakyReLU -> BN affine (acff_chain's operations) ----
  auto act = [&](float x, int j) {
    x += e_b[j];
    x = x > 0.f ? x : x * a.slope;
    return fmaf(x, e_s[j], e_t[j]);
  };
  if constexpr (TAIL) {
    // the stage's fp16 map into LDS (over the halo, no longer read): Y [M][cout + 8]
    __syncthreads();
    _Float16* Y = X;
    const int YS = a.cout + 8;
#pragma unroll
    for (int i = 0; i < FMW; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        if (!e_ok[j]) continue;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = (mt0 + i) * 16 + g * 4 + r;
          if (m < M) Y[(size_t)m * YS + n0 + j * 16 + fr] = (_Float16)act(acc[i][j][r], j);
        }
      }
    __syncthreads();
    // ---- tail: conv2 1x1 (cout -> 5) -> AvgPool 5 -> flatten -> Linear -> Softmax ----
    const int c = a.cout, hw = M, h = OW;  // square map: oh == ow
    float* conv = (float*)At;              // [5][hw] (the A tile is dead)
    float* w2s = conv + 5 * 64;            // [5][c]
    const int nf = 5 * a.ph * a.pwid;
    float* fcs = w2s + 5 * c;              // [5][nf]
    float* feat = fcs + 5 * nf;            // [nf]
    float* lg = feat + nf;                 // [5]
    for (int i = tid; i < 5 * c; i += kBandThreads) w2s[i] = a.w2[i];
    for (int i = tid; i < 5 * nf; i += kBandThreads) fcs[i] = a.fcw[i];
    __syncthreads();
    for (int t = tid; t < 5 * hw; t += kBandThreads) {  // four partial sums over the channels
      const int o = t / hw, p = t - o * hw;
      const _Float16* x = Y + (size_t)p * YS;
      const float* w = w2s + o * c;
      float s4[4] = {0.f, 0.f, 0.f, 0.f};
      for (int ch = 0; ch < c; ch += 8) {
        const h8 xv = *(const h8*)(x + ch);
        const f4 w0 = *(const f4*)(w + ch), w1 = *(const f4*)(w + ch + 4);
#pragma unroll
        for (int j = 0; j < 4; ++j) s4[j] = fmaf((float)xv[j], w0[j], s4[j]);
#pragma unroll
        for (int j = 0; j < 4; ++j) s4[j] = fmaf((float)xv[4 + j], w1[j], s4[j]);
      }
      conv[o * hw + p] = (s4[0] + s4[1]) + (s4[2] + s4[3]);
    }
    __syncthreads();
    for (int t = tid; t < nf; t += kBandThreads) {  // AvgPool2d(5, 1, pool_pad), count_include_pad
      const int o = t / (a.ph * a.pwid), r = t - o * a.ph * a.pwid;
      const int i = r / a.pwid, j = r - (r / a.pwid) * a.pwid;
      float sum = 0.f;
      for (int dy = 0; dy < 5; ++dy) {
        const int y = i - a.pool_pad + dy;
        if ((unsigned)y >= (unsigned)h) continue;
        for (int dx = 0; dx < 5; ++dx) {
          const int x = j - a.pool_pad + dx;
          if ((unsigned)x >= (unsigned)h) continue;
          sum += conv[o * hw + y * h + x];
        }
      }
      feat[t] = sum / 25.f;
    }
    __syncthreads();
    if (tid < 5) {  // Linear on the NCHW flatten (feat is [o][i][j])
      float s1 = 0.f;
      for (int q = 0; q < nf; ++q) s1 = fmaf(feat[q], fcs[tid * nf + q], s1);
      s1 += a.fcb[tid];
      lg[tid] = s1;
      if (a.logits) a.logits[img * 5 + tid] = s1;
    }
    __syncthreads();
    if (tid < 5 && a.probs) {
      float mx = lg[0];
      for (int k = 1; k < 5; ++k) mx = fmaxf(mx, lg[k]);
      float sum = 0.f;
      for (int k = 0; k < 5; ++k) sum += expf(lg[k] - mx);
      a.probs[img * 5 + tid] = expf(lg[tid] - mx) / sum;
    }
  } else if constexpr (POOL) {
    const int owp = OWq, ohp = a.oh_eff >> 1;
    _Float16* outn = a.out + (size_t)img * ohp * owp * a.out_cs + n0 + fr;
#pragma unroll
    for (int i = 0; i < FMW; ++i) {
      const int q = (mt0 + i) * 4 + g;  // this lane's quad
      if (4 * q >= M) continue;
      const int qy = q / owp, qx = q - (q / owp) * owp;
      _Float16* o = outn + ((size_t)((y0 >> 1) + qy) * owp + qx) * a.out_cs;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        if (!e_ok[j]) continue;
        const float v0 = act(acc[i][j][0], j), v1 = act(acc[i][j][1], j);
        const float v2 = act(acc[i][j][2], j), v3 = act(acc[i][j][3], j);
        o[j * 16] = (_Float16)fmaxf(fmaxf(v0, v1), fmaxf(v2, v3));
      }
    }
  } else {
    _Float16* outn = a.out + (size_t)img * (a.h - 2) * OW * a.out_cs + (size_t)y0 * OW * a.out_cs + n0 + fr;
#pragma unroll
    for (int i = 0; i < FMW; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = (mt0 + i) * 16 + g * 4 + r;
        if (m >= M) continue;
#pragma unroll
        for (int j = 0; j < 2; ++j)
          if (e_ok[j]) outn[(size_t)m * a.out_cs + j * 16] = (_Float16)act(acc[i][j][r], j);
      }
  }
}

int acff_band_mode() { return tune().acff_band; }

namespace {
struct BandGeom {
  int rows = 0, bands = 0, oh_eff = 0, fmw = 0, halo = 0, lds = 0;
};
BandGeom band_geom(int h, int w, int cin, int cout_pad, int pool, bool tail, int rows_pref) {
  BandGeom b;
  const int oh = h - 2, ow = w - 2;
  b.oh_eff = pool ? 2 * (oh / 2) : oh;
  b.rows = tail ? oh : std::max(pool ? 2 : 1, std::min(rows_pref, b.oh_eff));
  if (pool) b.rows &= ~1;
  if (b.rows <= 0) return BandGeom{};
  b.bands = (b.oh_eff + b.rows - 1) / b.rows;
  const int M = pool ? (b.rows / 2) * (ow / 2) * 4 : b.rows * ow;
  const int WM = 8 / (cout_pad / 32);
  b.fmw = ((M + 15) / 16 + WM - 1) / WM;
  b.halo = (int)round_up((int64_t)(b.rows + 6) * (w + 4) * (cin + 8) * 2, 16);
  const int a_bytes = WM * b.fmw * 16 * (3 * cin + 8) * 2;
  int tail_bytes = 0;
  if (tail) {
    // Y over the halo; conv [5][64] + w2 [5][cout] + fc [5][nf] + feat + logits over the A tile
    b.halo = std::max(b.halo, (int)round_up((int64_t)M * (cout_pad + 8) * 2, 16));
    tail_bytes = (5 * 64 + 5 * cout_pad + 5 * 5 * 16 + 5 * 16 + 8) * 4;
  }
  b.lds = b.halo + std::max(a_bytes, tail_bytes);
  return b;
}
}  // namespace

bool acff_band_ok(int h, int w, int cin, int cout, int cout_pad, int kpad, int pool, bool tail) {
  if (cin % 32 != 0 || cin > 128 || kpad < 3 * cin) return false;
  if (cout_pad != 128 && cout_pad != 256) return false;
  if (cout > cout_pad) return false;
  if (tail && (pool || h != w || (h - 2) * (w - 2) > 64)) return false;
  if (h - 2 < 1 || w - 2 < (pool ? 2 : 1)) return false;
  const BandGeom b = band_geom(h, w, cin, cout_pad, pool, tail, 2);
  return b.fmw >= 1 && b.fmw <= 4 && b.lds <= 160 * 1024;
}

void launch_acff_band(const void* in, int in_cs, int in_co, int n, int h, int w, int cin, const float* dw_wt,
                      const float* dw_b, const void* pw, int kpad, int cout, int cout_pad, const float* bias,
                      const float* scale, const float* shift, float slope, void* out, int out_cs, int pool,
                      const AcffBandTail* tail, hipStream_t s) {
  RTDM_REQUIRE(acff_band_ok(h, w, cin, cout, cout_pad, kpad, pool, tail != nullptr), RTDM_E_INVALID,
               "acff_band: unsupported shape");
  RTDM_REQUIRE((in_cs % 8) == 0 && (in_co % 8) == 0, RTDM_E_INVALID, "acff_band: input view not 16-byte aligned");
  RTDM_REQUIRE(slope > 0.f && slope <= 1.f, RTDM_E_INVALID, "acff_band: LeakyReLU slope outside (0, 1]");
  if (n <= 0) return;
  const BandGeom b = band_geom(h, w, cin, cout_pad, pool, tail != nullptr, tune().acff_band_rows);
  RTDM_REQUIRE(b.fmw >= 1 && b.fmw <= 4 && b.lds <= 160 * 1024, RTDM_E_INVALID, "acff_band: band too large");
  AcffBandArgs a;
  a.in = (const _Float16*)in;
  a.in_cs = in_cs;
  a.in_co = in_co;
  a.h = h;
  a.w = w;
  a.cin = cin;
  a.rows = b.rows;
  a.bands = b.bands;
  a.oh_eff = b.oh_eff;
  a.halo_bytes = b.halo;
  a.dw_wt = dw_wt;
  a.dw_b = dw_b;
  a.pw = (const _Float16*)pw;
  a.kpad = kpad;
  a.cout = cout;
  a.cout_pad = cout_pad;
  a.bias = bias;
  a.scale = scale;
  a.shift = shift;
  a.slope = slope;
  a.out = (_Float16*)out;
  a.out_cs = out_cs;
  a.w2 = tail ? tail->w2 : nullptr;
  a.pool_pad = tail ? tail->pool_pad : 0;
  a.ph = tail ? tail->ph : 0;
  a.pwid = tail ? tail->pw : 0;
  a.fcw = tail ? tail->fcw : nullptr;
  a.fcb = tail ? tail->fcb : nullptr;
  a.logits = tail ? tail->logits : nullptr;
  a.probs = tail ? tail->probs : nullptr;
  if (tail) RTDM_REQUIRE(a.ph * a.pwid <= 16, RTDM_E_UNSUPPORTED, "acff_band: pooled tail too large");
  const int64_t blocks = (int64_t)n * b.bands;
  RTDM_REQUIRE(blocks < (1ll << 31), RTDM_E_CAPACITY, "acff_band: too many bands");
  auto go = [&](auto kern) {
    hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(kBandThreads), (size_t)b.lds, s, a);
  };
#define RTDM_BAND_GO(P, T)                  \
  switch (b.fmw) {                          \
    case 1: go(acff_band<1, P, T>); break;  \
    case 2: go(acff_band<2, P, T>); break;  \
    case 3: go(acff_band<3, P, T>); break;  \
    default: go(acff_band<4, P, T>); break; \
  }
  if (tail) {
    RTDM_BAND_GO(false, true)
  } else if (pool) {
    RTDM_BAND_GO(true, false)
  } else {
    RTDM_BAND_GO(false, false)
  }
#undef RTDM_BAND_GO
  RTDM_HIP(hipGetLastError());
}

}  // namespace rtdm
