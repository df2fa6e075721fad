// Fused ACFF block on gfx950 (fp16 activations, fp32 accumulation).
//
// disaster_detection/model/acff.py:37-59 in one launch:
//   three depthwise 3x3 branches (dilation 1/2/3, padding 0/1/2, + bias each,
//   acff.py:25-30) -> channel concat (acff.py:46) -> 1x1 conv (+bias) ->
//   LeakyReLU(0.01) -> BatchNorm affine (eval; acff.py:51-53, BN after the
//   activation so it stays an epilogue affine) -> optional 2x2 floor maxpool
//   (the MaxPool2d(2,2) that follows acff1..3 in squeeze_ernet.py:27-35 / ernet.py).
// The concat never touches HBM: a block owns an 8x8 output tile, builds the
// tile's depthwise outputs for all 3*Cin concat channels in LDS (the MFMA A
// operand, k = branch*Cin + c like the reference's torch.cat) and multiplies
// it by the packed 1x1 weights on v_mfma_f32_16x16x32_f16.
//
//   phase 1 (per 32-channel chunk): input tile rows oy0-2..oy0+11, cols
//            ox0-2..ox0+11 (radius-3 halo of the centre pixel (oy+1, ox+1))
//            -> LDS, zero outside the image (the padding of the dilated branches).
//   phase 2: depthwise taps on VALU, fp32 accumulate, one (pixel, 8 channels,
//            branch) item per thread per pass, 16-byte LDS reads, stored as fp16
//            into the A tile (the fp16 rounding the unfused path applies when it
//            writes the concat to HBM).
//   phase 3: 2x2 waves over (64 pixels) x (cout_pad): A fragments from LDS,
//            B fragments (weights, L2-resident) from global, prefetched one
//            k-step ahead.
//   phase 4: epilogue in registers.  Tile pixels are in 2x2-quad order, so each
//            lane's 4 accumulator rows are one quad and the pool is in-lane.
#include "common.h"

namespace rtdm {

namespace {
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));

constexpr int kTile = 8;              // output tile side
constexpr int kHalo = kTile + 6;      // staged input tile side
constexpr int kPix = kTile * kTile;   // 64 output pixels per block
}  // namespace

struct AcffArgs {
  const _Float16* in;
  int in_cs, in_co;
  int n, h, w, cin;
  int lim_h, lim_w;        // only outputs oy < lim_h, ox < lim_w are stored
  const float* dw_wt;      // [3][9][cin] (tap-major)
  const float* dw_b;       // [3][cin]
  const _Float16* pw;      // [cout_pad][kpad], k = branch*cin + c
  int kpad, cout, cout_pad;
  const float* bias;       // [cout]
  const float* scale;      // [cout] or null
  const float* shift;
  float slope;
  _Float16* out;           // NHWC [n, oh, ow, cout] or pooled [n, oh/2, ow/2, cout]
  int out_cs, pool;
  int cc;                  // channels per staging chunk (multiple of 8)
};

static inline size_t acff_lds_bytes(int cc, int kpad, int cin) {
  return (size_t)kHalo * kHalo * cc * 2            // input tile chunk
         + (size_t)(3 * 9 + 3) * cc * 4            // dw weights + bias chunk
         + (size_t)kPix * (kpad + 8) * 2;          // A tile (rows padded by 8 halfs)
}

// pixel m (0..63) of the tile in quad order -> (py, px)
__device__ __forceinline__ void tile_pix(int m, int& py, int& px) {
  const int q = m >> 2, d = m & 3;
  py = 2 * (q >> 2) + (d >> 1);
  px = 2 * (q & 3) + (d & 1);
}

template <int NTW>
__global__ __launch_bounds__(256) void acff_fused(AcffArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char acff_lds[];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int cc = a.cc;
  const int LS = a.kpad + 8;  // A-tile row stride (halfs)
  _Float16* xt = (_Float16*)acff_lds;                                   // [kHalo][kHalo][cc]
  float* wsm = (float*)(acff_lds + (size_t)kHalo * kHalo * cc * 2);     // [3][9][cc] then bias [3][cc]
  float* bsm = wsm + 27 * cc;
  _Float16* At = (_Float16*)(acff_lds + (size_t)kHalo * kHalo * cc * 2 + (size_t)30 * cc * 4);  // [64][LS]

  const int oh = a.h - 2, ow = a.w - 2;
  const int tiles_x = (a.lim_w + kTile - 1) / kTile;
  const int tiles_y = (a.lim_h + kTile - 1) / kTile;
  const int per_img = tiles_x * tiles_y;
  const int n = blockIdx.x / per_img;
  const int tt = blockIdx.x - n * per_img;
  const int oy0 = (tt / tiles_x) * kTile, ox0 = (tt - (tt / tiles_x) * tiles_x) * kTile;
  const int K = 3 * a.cin;

  // zero the K padding of the A tile
  if (K < a.kpad) {
    const int padw = a.kpad - K;
    for (int i = tid; i < kPix * padw; i += 256) {
      const int m = i / padw, k = K + (i - (i / padw) * padw);
      At[m * LS + k] = (_Float16)0.f;
    }
  }

  const _Float16* src = a.in + (size_t)n * a.h * a.w * a.in_cs + a.in_co;
  for (int c0 = 0; c0 < a.cin; c0 += cc) {
    const int ccn = a.cin - c0 < cc ? a.cin - c0 : cc;  // channels in this chunk (multiple of 8)
    const int cv = ccn >> 3;
    // ---- phase 1: stage input tile chunk + dw weights ----
    for (int i = tid; i < kHalo * kHalo * cv; i += 256) {
      const int pix = i / cv, v = i - pix * cv;
      const int r = pix / kHalo, c = pix - r * kHalo;
      const int y = oy0 - 2 + r, x = ox0 - 2 + c;
      uint4 d = make_uint4(0u, 0u, 0u, 0u);
      if ((unsigned)y < (unsigned)a.h && (unsigned)x < (unsigned)a.w)
        d = *(const uint4*)(src + ((size_t)y * a.w + x) * a.in_cs + c0 + v * 8);
      *(uint4*)(xt + (size_t)pix * cc + v * 8) = d;
    }
    for (int i = tid; i < 30 * ccn; i += 256) {
      const int row = i / ccn, c = i - row * ccn;
      if (row < 27)
        wsm[row * cc + c] = a.dw_wt[(size_t)row * a.cin + c0 + c];
      else
        bsm[(row - 27) * cc + c] = a.dw_b[(size_t)(row - 27) * a.cin + c0 + c];
    }
    __syncthreads();
    // ---- phase 2: depthwise branches -> A tile ----
    const int items = kPix * cv * 3;
    for (int i = tid; i < items; i += 256) {
      const int v = i % cv;
      const int t2 = i / cv;
      const int m = t2 & (kPix - 1);
      const int br = t2 >> 6;
      const int d = br + 1;
      int py, px;
      tile_pix(m, py, px);
      float acc[8];
      const float4 b0 = *(const float4*)(bsm + br * cc + v * 8);
      const float4 b1 = *(const float4*)(bsm + br * cc + v * 8 + 4);
      acc[0] = b0.x; acc[1] = b0.y; acc[2] = b0.z; acc[3] = b0.w;
      acc[4] = b1.x; acc[5] = b1.y; acc[6] = b1.z; acc[7] = b1.w;
#pragma unroll
      for (int kh = 0; kh < 3; ++kh)
#pragma unroll
        for (int kw = 0; kw < 3; ++kw) {
          const int r = py + 3 + (kh - 1) * d, c = px + 3 + (kw - 1) * d;
          const h8 xv = *(const h8*)(xt + (size_t)(r * kHalo + c) * cc + v * 8);
          const float* wp = wsm + (br * 9 + kh * 3 + kw) * cc + v * 8;
          const float4 w0 = *(const float4*)wp;
          const float4 w1 = *(const float4*)(wp + 4);
          acc[0] = fmaf(w0.x, (float)xv[0], acc[0]);
          acc[1] = fmaf(w0.y, (float)xv[1], acc[1]);
          acc[2] = fmaf(w0.z, (float)xv[2], acc[2]);
          acc[3] = fmaf(w0.w, (float)xv[3], acc[3]);
          acc[4] = fmaf(w1.x, (float)xv[4], acc[4]);
          acc[5] = fmaf(w1.y, (float)xv[5], acc[5]);
          acc[6] = fmaf(w1.z, (float)xv[6], acc[6]);
          acc[7] = fmaf(w1.w, (float)xv[7], acc[7]);
        }
      h8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = (_Float16)acc[j];
      *(h8*)(At + m * LS + br * a.cin + c0 + v * 8) = o;
    }
    __syncthreads();
  }

  // ---- phase 3: [64 x kpad] x [kpad x cout_pad] on MFMA ----
  const int wm = wid >> 1, wn = wid & 1;
  const int n_base = wn * (a.cout_pad >> 1);
  const int fr = lane & 15, fk = (lane >> 4) * 8;
  f4 acc[2][NTW];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < NTW; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
  const _Float16* wrow = a.pw + (size_t)(n_base + fr) * a.kpad + fk;
  const int nks = a.kpad >> 5;
  h8 bcur[NTW], bnext[NTW];
#pragma unroll
  for (int j = 0; j < NTW; ++j) bcur[j] = *(const h8*)(wrow + (size_t)j * 16 * a.kpad);
  const _Float16* arow = At + (wm * 32 + fr) * LS + fk;
  for (int ks = 0; ks < nks; ++ks) {
    if (ks + 1 < nks) {
#pragma unroll
      for (int j = 0; j < NTW; ++j) bnext[j] = *(const h8*)(wrow + (size_t)j * 16 * a.kpad + (ks + 1) * 32);
    }
    const h8 a0 = *(const h8*)(arow + ks * 32);
    const h8 a1 = *(const h8*)(arow + 16 * LS + ks * 32);
#pragma unroll
    for (int j = 0; j < NTW; ++j) {
      acc[0][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a0, bcur[j], acc[0][j], 0, 0, 0);
      acc[1][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a1, bcur[j], acc[1][j], 0, 0, 0);
    }
#pragma unroll
    for (int j = 0; j < NTW; ++j) bcur[j] = bnext[j];
  }

  // ---- phase 4: bias -> LeakyReLU -> BN affine -> (pool) -> fp16 store ----
  const int rq = lane >> 4;
#pragma unroll
  for (int j = 0; j < NTW; ++j) {
    const int c = n_base + j * 16 + fr;
    if (c >= a.cout) continue;
    const float bb = a.bias[c];
    const float sc = a.scale ? a.scale[c] : 1.f;
    const float sh = a.scale ? a.shift[c] : 0.f;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int q = wm * 8 + i * 4 + rq;  // quad of this lane's 4 rows
      const int qy = q >> 2, qx = q & 3;
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float x = acc[i][j][r] + bb;
        x = x > 0.f ? x : x * a.slope;
        v[r] = x * sc + sh;
      }
      if (a.pool) {
        const int py = (oy0 >> 1) + qy, px = (ox0 >> 1) + qx;
        if (py < (oh >> 1) && px < (ow >> 1)) {
          const float mx = fmaxf(fmaxf(v[0], v[1]), fmaxf(v[2], v[3]));
          a.out[(((size_t)n * (oh >> 1) + py) * (ow >> 1) + px) * a.out_cs + c] = (_Float16)mx;
        }
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int y = oy0 + 2 * qy + (r >> 1), x = ox0 + 2 * qx + (r & 1);
          if (y < a.lim_h && x < a.lim_w) a.out[(((size_t)n * oh + y) * ow + x) * a.out_cs + c] = (_Float16)v[r];
        }
      }
    }
  }
}

// Largest staging chunk (32 / 16 / 8 channels) whose LDS footprint fits 64 KiB; 0 if none.
static int acff_chunk(int cin, int kpad) {
  for (int cc = 32; cc >= 8; cc >>= 1) {
    const int c = cin < cc ? cin : cc;
    if (acff_lds_bytes(c, kpad, cin) <= 64 * 1024) return c;
  }
  return 0;
}

bool acff_fused_ok(int cin, int cout_pad, int kpad) {
  if (cin % 8 != 0 || kpad % 32 != 0) return false;
  if (cout_pad != 64 && cout_pad != 128 && cout_pad != 256) return false;
  return acff_chunk(cin, kpad) > 0;
}

void launch_acff_fused(const void* in, int in_cs, int in_co, int n, int h, int w, int cin, int lim_h, int lim_w,
                       const float* dw_wt, const float* dw_b, const void* pw, int kpad, int cout, int cout_pad,
                       const float* bias, const float* scale, const float* shift, float slope, void* out, int out_cs,
                       int pool, hipStream_t s) {
  RTDM_REQUIRE(acff_fused_ok(cin, cout_pad, kpad), RTDM_E_INVALID, "acff_fused: unsupported shape");
  RTDM_REQUIRE((in_cs % 8) == 0 && (in_co % 8) == 0, RTDM_E_INVALID, "acff_fused: input view not 16-byte aligned");
  AcffArgs a;
  a.in = (const _Float16*)in;
  a.in_cs = in_cs;
  a.in_co = in_co;
  a.n = n;
  a.h = h;
  a.w = w;
  a.cin = cin;
  a.lim_h = lim_h;
  a.lim_w = lim_w;
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
  a.pool = pool;
  a.cc = acff_chunk(cin, kpad);
  const int tiles = ((lim_h + kTile - 1) / kTile) * ((lim_w + kTile - 1) / kTile);
  const int64_t blocks = (int64_t)n * tiles;
  if (blocks <= 0) return;
  const size_t lds = acff_lds_bytes(a.cc, kpad, cin);
  if (cout_pad == 64)
    hipLaunchKernelGGL(acff_fused<2>, dim3((unsigned)blocks), dim3(256), lds, s, a);
  else if (cout_pad == 128)
    hipLaunchKernelGGL(acff_fused<4>, dim3((unsigned)blocks), dim3(256), lds, s, a);
  else
    hipLaunchKernelGGL(acff_fused<8>, dim3((unsigned)blocks), dim3(256), lds, s, a);
  RTDM_HIP(hipGetLastError());
}

}  // namespace rtdm
