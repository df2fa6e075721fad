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

#include <map>
#include <mutex>

#include <algorithm>
#include <type_traits>

namespace rtdm {

namespace {
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

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
      for (int j = 0; j < 8; ++j) asm volatile("" : "+v"(acc[j]));  // (f32 sums round on their own)
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
        v[r] = fmaf(x, sc, sh);  // explicit FMA: acff_chain repeats it bit for bit
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

// --------------------------------------------------------------------------
// acff_persist: the same block for the large-map ACFF layers (ErNET acff1..3,
// Squeeze acff1..3), built for throughput:
//   * persistent blocks (occupancy-sized grid) walk (tile, channel chunk) work
//     items; the next item's input halo is prefetched into registers while the
//     current one is computed (double-buffered LDS halo);
//   * 8 x 16 output tiles (halo 14 x 22: 2.4x input reads per output instead of
//     3x for 8 x 8);
//   * depthwise: one wave owns an 8-channel group for 64 pixels (lane = pixel),
//     so the 27 tap weights of a branch are wave-uniform scalar loads (SGPR
//     operands of the FMAs), inputs one ds_read_b128 per tap;
//   * the 1x1 GEMM accumulates over channel chunks of CC channels: K order
//     (chunk, branch, channel) — weights repacked host-side to match — on
//     v_mfma_f32_16x16x32_f16, B fragments straight from global (L2-resident).
// Tile pixels are in 2x2-quad order, so the pooled epilogue stays in-lane.
// --------------------------------------------------------------------------
struct AcffPArgs {
  const _Float16* in;
  int in_cs, in_co;
  int n, h, w, cin;
  int lim_h, lim_w;
  const float* dw_wt;   // [3][9][cin]
  const float* dw_b;    // [3][cin]
  const _Float16* pw;   // [cout_pad][nch * KC], k = chunk*KC + branch*CC + c
  int cout, cout_pad;
  const float* bias;
  const float* scale;
  const float* shift;
  float slope;
  _Float16* out;
  int out_cs, pool;
  // int8 1x1 fusion (RTDM_I8 classifiers, BASELINE config 5): the depthwise concat is
  // quantised per concat channel (x * inv_s[branch][c], symmetric, +-127) into an int8 A
  // tile; the per-channel activation scales are folded into per-output-channel int8
  // weights pw8 [cout_pad][nch * 64] (k = chunk*64 + branch*CC + c), exact int32 sums
  // dequantised by deq[o].
  const int8_t* pw8;
  const float* deq;
  const float* inv_s;  // [3][cin]
  unsigned* amax;      // calibration (fp16 path): |x|max of every concat channel [3][cin]
};

// Wave-uniform reads through the constant address space become scalar loads
// (SGPR operands of the depthwise FMAs).
typedef const __attribute__((address_space(4))) float* cfloat_p;

template <int CC>
struct AcffPGeom {
  // HW: staged halo columns, 2 past the 22 the taps read: with a row pitch of 24 pixels the
  // quad-ordered depthwise reads of a 16-lane group fall in 16 distinct 4-bank slots (at 22,
  // 2-way conflicts: 25 % of the kernel's LDS cycles, PMC r04c)
  static constexpr int TH = 8, TW = 16, HH = TH + 6, HW = TW + 8, NPIX = TH * TW;
  static constexpr int PS = CC + 8;                    // halo pixel stride (halfs)
  static constexpr int CG = CC / 8;                    // 8-channel groups per chunk
  static constexpr int KC = (3 * CC + 31) / 32 * 32;   // K per chunk (zero-padded)
  static constexpr int AS = KC + 8;                    // A-tile row stride (halfs)
  static constexpr int HALO = HH * HW * CG;            // 16-byte vectors per halo chunk
  static constexpr int PV = (HALO + 255) / 256;        // prefetch registers per thread
  // RP: halo row pitch (halfs), 4 past HW * PS: the depthwise reads are ds_read_b64 of 4
  // channels for pixels of two tile rows per 32-lane half, and a row offset of 2 mod 4 dwords
  // puts the second row on the other two banks of each 4-bank slot (conflict-free); the
  // staging then writes 8-byte halves (a row start is only 8-byte aligned)
  static constexpr int RP = HW * PS + 4;
  static constexpr int XS = HH * RP;                   // halfs per halo buffer
};

// fp32 = w (SGPR f32) * x (f16, low / high half of a packed pair) + acc, exact like
// cvt + fma but one VOP3P instruction.
__device__ __forceinline__ float fma_mix_lo(float w, uint32_t x2, float acc) {
  float d;
  asm("v_fma_mix_f32 %0, %1, %2, %3 op_sel_hi:[0,1,0]" : "=v"(d) : "s"(w), "v"(x2), "v"(acc));
  return d;
}
__device__ __forceinline__ float fma_mix_hi(float w, uint32_t x2, float acc) {
  float d;
  asm("v_fma_mix_f32 %0, %1, %2, %3 op_sel:[0,1,0] op_sel_hi:[0,1,0]" : "=v"(d) : "s"(w), "v"(x2), "v"(acc));
  return d;
}
// the same with the weight in a VGPR (broadcast from LDS)
__device__ __forceinline__ float fma_mix_lo_v(float w, uint32_t x2, float acc) {
  float d;
  asm("v_fma_mix_f32 %0, %1, %2, %3 op_sel_hi:[0,1,0]" : "=v"(d) : "v"(w), "v"(x2), "v"(acc));
  return d;
}
__device__ __forceinline__ float fma_mix_hi_v(float w, uint32_t x2, float acc) {
  float d;
  asm("v_fma_mix_f32 %0, %1, %2, %3 op_sel:[0,1,0] op_sel_hi:[0,1,0]" : "=v"(d) : "v"(w), "v"(x2), "v"(acc));
  return d;
}
constexpr int kAcffPMaxCin = 128;  // depthwise taps + biases of the whole layer in LDS

// MODE: 0 fp16, 1 int8 1x1 fusion, 2 fp16 + calibration (records the concat's |x|max)
template <int CC, int NF, int ABL = 0, int MODE = 0>  // ABL (diagnostics, wrong outputs): 1 no taps, 2 no GEMM, 4 no tap-weight reads
__global__ __launch_bounds__(256, NF == 2 ? 3 : 2) void acff_persist(AcffPArgs a) {  // NF 2: <= 168 VGPRs, 3 waves / SIMD
  constexpr bool I8 = MODE == 1, CAL = MODE == 2;
  using G = AcffPGeom<CC>;
  constexpr int TH = G::TH, TW = G::TW, HW = G::HW, PS = G::PS, CG = G::CG, KC = G::KC, AS = G::AS, RP = G::RP;
  constexpr int HALO = G::HALO, PV = G::PV, XS = G::XS;
  constexpr int KC8 = (3 * CC + 63) / 64 * 64, AS8 = KC8 + 16;  // int8 A tile: K per chunk, row bytes
  static_assert(!I8 || G::NPIX * AS8 <= G::NPIX * AS * 2, "int8 A tile reuses the fp16 one");
  __shared__ __attribute__((aligned(16))) _Float16 xs[2 * XS];
  __shared__ __attribute__((aligned(16))) _Float16 At[G::NPIX * AS];
  int8_t* const At8 = reinterpret_cast<int8_t*>(At);
  // depthwise taps [27][cin], biases [3][cin] (int8: + inverse activation scales [3][cin]):
  // LDS broadcast reads, pipelined by the compiler (as wave-uniform scalar loads every tap
  // waited on its own s_load latency)
  extern __shared__ __attribute__((aligned(16))) float s_dw[];  // dynamic: (I8 ? 33 : 30) * cin floats
  const int tid = threadIdx.x, lane = tid & 63;
  // LDS layout [chunk][NW][CC]: every tap / bias / scale offset inside a chunk is a
  // compile-time immediate from one per-item base (with [NW][cin] each read needed its own
  // wave-uniform address moved into a VGPR)
  constexpr int NW = I8 ? 33 : 30;
  for (int i = tid; i < NW * a.cin; i += 256) {
    const int chk = i / (NW * CC), r = i - chk * (NW * CC);
    const int t = r / CC, c = chk * CC + (r - t * CC);
    s_dw[i] = t < 27 ? a.dw_wt[t * a.cin + c] : t < 30 ? a.dw_b[(t - 27) * a.cin + c] : a.inv_s[(t - 30) * a.cin + c];
  }
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, g = lane >> 4;
  const int oh = a.h - 2, ow = a.w - 2;
  const int tiles_x = (a.lim_w + TW - 1) / TW, tiles_y = (a.lim_h + TH - 1) / TH;
  const int ntiles = a.n * tiles_x * tiles_y;
  const int nch = a.cin / CC;
  const int ktot = nch * KC;
  if constexpr (I8) {  // zero K padding of the int8 A tile (never overwritten)
    constexpr int padw = KC8 - 3 * CC;
    for (int i = tid; i < G::NPIX * padw; i += 256) At8[(i / padw) * AS8 + 3 * CC + i % padw] = 0;
  } else if (KC > 3 * CC) {  // zero K padding of the A tile (never overwritten)
    constexpr int padw = KC - 3 * CC;
    for (int i = tid; i < G::NPIX * padw; i += 256) At[(i / padw) * AS + 3 * CC + i % padw] = (_Float16)0.f;
  }
  const _Float16* __restrict__ in = a.in + a.in_co;
  // work items of this block: tiles t0, t0 + tstep, ... < tend (XCD-contiguous walk:
  // neighbouring tiles' halos share the XCD's L2), each over the channel chunks 0 .. nch-1.
  // Two cursors (the item being computed, the one being prefetched two ahead) step the
  // (chunk, tile x, tile y, image) coordinates with carries: no per-item integer divisions
  // (each was ~10 VALU; the launch keeps every input offset below 2^31, so 32-bit offsets)
  int t0, tend, tstep;
  xcd_span(blockIdx.x, gridDim.x, ntiles, t0, tend, tstep);
  const int tpi = tiles_x * tiles_y;
  const int sn = tstep / tpi, sy = (tstep - sn * tpi) / tiles_x, sx = tstep - sn * tpi - sy * tiles_x;
  struct Cur {
    int ch, tx, ty, n, tile;
  };
  auto cur_at = [&](int tile) {
    Cur c;
    c.ch = 0;
    c.tile = tile;
    c.tx = tile % tiles_x;
    const int t1 = tile / tiles_x;
    c.ty = t1 % tiles_y;
    c.n = t1 / tiles_y;
    return c;
  };
  auto advance = [&](Cur& c) {
    if (++c.ch < nch) return;
    c.ch = 0;
    c.tile += tstep;
    c.tx += sx;
    if (c.tx >= tiles_x) {
      c.tx -= tiles_x;
      ++c.ty;
    }
    c.ty += sy;
    if (c.ty >= tiles_y) {
      c.ty -= tiles_y;
      ++c.n;
    }
    c.n += sn;
  };
  auto prefetch = [&](u32x4(&pre)[PV], const Cur& it) {
    const int ch = it.ch, tx = it.tx, ty = it.ty, n = it.n;
#pragma unroll
    for (int k = 0; k < PV; ++k) {
      const int i = tid + 256 * k;
      const int pix = i / CG, v = i - pix * CG;
      const int r = pix / HW, c = pix - r * HW;
      const int y = ty * TH - 2 + r, x = tx * TW - 2 + c;
      u32x4 d = {0u, 0u, 0u, 0u};
      if (i < HALO && (unsigned)y < (unsigned)a.h && (unsigned)x < (unsigned)a.w)
        d = *(const u32x4*)(in + (unsigned)(((n * a.h + y) * a.w + x) * a.in_cs + ch * CC + v * 8));
      pre[k] = d;
    }
  };
  auto stage = [&](const u32x4(&pre)[PV], _Float16* xb) {
#pragma unroll
    for (int k = 0; k < PV; ++k) {
      const int i = tid + 256 * k;
      if (i < HALO) {
        const int pix = i / CG, v = i - pix * CG;
        const int r = pix / HW, c = pix - r * HW;
        uint2* dst = (uint2*)(xb + r * RP + c * PS + v * 8);
        dst[0] = make_uint2(pre[k][0], pre[k][1]);
        dst[1] = make_uint2(pre[k][2], pre[k][3]);
      }
    }
  };
  const int wm = wid >> 1, wn = wid & 1;
  typedef int i32x4 __attribute__((ext_vector_type(4)));
  using AccT = std::conditional_t<I8, i32x4, f4>;
  AccT acc[4][NF];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int jn = 0; jn < NF; ++jn) acc[i][jn] = AccT{0, 0, 0, 0};
  h8 bf[KC / 32][NF];
  i32x4 bf8[KC8 / 64][NF];
  int bf_ch = -1;
  const int ktot8 = nch * KC8;
  // 1x1 weight fragments of item j's chunk (global, L2-resident; once when nch == 1).
  // Issued BEFORE the halo prefetch of j+2: vmcnt retires in order, so waiting for
  // these never waits for the prefetch.
  auto load_bf = [&](int ch) {
    if (ch == bf_ch) return;
    if constexpr (I8) {
#pragma unroll
      for (int ks = 0; ks < KC8 / 64; ++ks)
#pragma unroll
        for (int tn = 0; tn < NF; ++tn)
          bf8[ks][tn] = *(const i32x4*)(a.pw8 + (size_t)(wn * NF * 16 + tn * 16 + fr) * ktot8 + ch * KC8 + ks * 64 + g * 16);
    } else {
#pragma unroll
      for (int ks = 0; ks < KC / 32; ++ks)
#pragma unroll
        for (int tn = 0; tn < NF; ++tn)
          bf[ks][tn] = *(const h8*)(a.pw + (size_t)(wn * NF * 16 + tn * 16 + fr) * ktot + ch * KC + ks * 32 + g * 8);
    }
    bf_ch = ch;
  };
  // epilogue constants of this lane's channels, hoisted out of the item loop (a load
  // in the loop would wait for the in-flight prefetch)
  float e_b[NF], e_s[NF], e_t[NF], e_d[NF];
  bool e_ok[NF];
#pragma unroll
  for (int tn = 0; tn < NF; ++tn) {
    const int c = wn * NF * 16 + tn * 16 + fr;
    const bool cv = c < a.cout;
    e_ok[tn] = cv;
    e_d[tn] = I8 && cv ? a.deq[c] : 1.f;
    e_b[tn] = cv ? a.bias[c] : 0.f;
    e_s[tn] = (cv && a.scale) ? a.scale[c] : 1.f;
    e_t[tn] = (cv && a.scale) ? a.shift[c] : 0.f;
  }

  auto process = [&](const Cur& it, const _Float16* xb) {
    const int ch = it.ch;
    int cal_ok = 0;  // calibration: this lane's pixel lies inside the output map
    if constexpr (CAL) {
      const int tx = it.tx, ty = it.ty;
      const int m = lane, q = m >> 2, dq = m & 3;  // pixel of lane (pixel block 0 / 1 differ by 4 rows)
      const int py = 2 * (q >> 3) + (dq >> 1), px = 2 * (q & 7) + (dq & 1);
      cal_ok = (ty * TH + py < oh ? 1 : 0) | (ty * TH + py + 4 < oh ? 2 : 0);
      if (tx * TW + px >= ow) cal_ok = 0;
    }
    // ---- depthwise branches -> A tile (fp16, or int8 quantised per concat channel).
    //      A wave owns 4 channels (c4) of BOTH 64-pixel halves (lane = pixel m and m + 64,
    //      4 tile rows apart): each tap's 4 weights (one broadcast ds_read_b128) serve 8 FMAs,
    //      half the weight reads per FMA of one pixel x 8 channels per lane (the weight reads
    //      were 57 % of the kernel's LDS instructions; without them acff1 ran 15 % faster,
    //      r05ah).  Every output takes the same operations in the same order. ----
#pragma unroll
    for (int u0 = 0; u0 < CC / 4; u0 += 4) {
      const int c4 = u0 + wid;
      if (c4 < CC / 4) {
        const int m = lane;  // pixel block 0; block 1 is m + 64, 4 rows down
        const int q = m >> 2, dq = m & 3;
        const int py = 2 * (q >> 3) + (dq >> 1), px = 2 * (q & 7) + (dq & 1);
        const int cbase = ch * CC + c4 * 4;
        const float* wc = s_dw + ch * (NW * CC) + c4 * 4;  // this chunk's [NW][CC] block, lane's 4 channels
#pragma unroll
        for (int br = 0; br < 3; ++br) {
          const int d = br + 1;
          const f4 bb = *(const f4*)(wc + (27 + br) * CC);
          float s0[4] = {bb[0], bb[1], bb[2], bb[3]}, s1[4] = {bb[0], bb[1], bb[2], bb[3]};
#pragma unroll
          for (int kh = 0; kh < 3; ++kh)
#pragma unroll
            for (int kw = 0; kw < 3; ++kw) {
              if constexpr ((ABL & 1) != 0) continue;
              const int hr = py + 3 + (kh - 1) * d, hc = px + 3 + (kw - 1) * d;
              const _Float16* xp = xb + hr * RP + hc * PS + c4 * 4;
              const uint2 x0 = *(const uint2*)xp, x1 = *(const uint2*)(xp + 4 * RP);
              f4 w;
              if constexpr ((ABL & 4) != 0) {  // (diagnostic: no tap-weight LDS reads)
                w = f4{0.5f, 0.25f, 0.125f, 0.5f};
              } else {
                w = *(const f4*)(wc + (br * 9 + kh * 3 + kw) * CC);
              }
              s0[0] = fma_mix_lo_v(w[0], x0.x, s0[0]);
              s0[1] = fma_mix_hi_v(w[1], x0.x, s0[1]);
              s0[2] = fma_mix_lo_v(w[2], x0.y, s0[2]);
              s0[3] = fma_mix_hi_v(w[3], x0.y, s0[3]);
              s1[0] = fma_mix_lo_v(w[0], x1.x, s1[0]);
              s1[1] = fma_mix_hi_v(w[1], x1.x, s1[1]);
              s1[2] = fma_mix_lo_v(w[2], x1.y, s1[2]);
              s1[3] = fma_mix_hi_v(w[3], x1.y, s1[3]);
            }
          if constexpr (I8) {
            const f4 is = *(const f4*)(wc + (30 + br) * CC);
            uint32_t q0 = 0, q1 = 0;
#pragma unroll
            for (int jj = 0; jj < 4; ++jj) {
              int v0 = (int)rintf(s0[jj] * is[jj]), v1 = (int)rintf(s1[jj] * is[jj]);
              v0 = v0 < -127 ? -127 : (v0 > 127 ? 127 : v0);
              v1 = v1 < -127 ? -127 : (v1 > 127 ? 127 : v1);
              q0 |= ((uint32_t)v0 & 255u) << (8 * jj);
              q1 |= ((uint32_t)v1 & 255u) << (8 * jj);
            }
            *(uint32_t*)(At8 + m * AS8 + br * CC + c4 * 4) = q0;
            *(uint32_t*)(At8 + (m + 64) * AS8 + br * CC + c4 * 4) = q1;
          } else {
            typedef _Float16 h4v __attribute__((ext_vector_type(4)));
            h4v o0, o1;
#pragma unroll
            for (int jj = 0; jj < 4; ++jj) {
              o0[jj] = (_Float16)s0[jj];
              o1[jj] = (_Float16)s1[jj];
            }
            *(h4v*)(At + m * AS + br * CC + c4 * 4) = o0;
            *(h4v*)(At + (m + 64) * AS + br * CC + c4 * 4) = o1;
            if constexpr (CAL) {  // calibration: per concat channel |x|max over the wave's valid pixels
#pragma unroll
              for (int jj = 0; jj < 4; ++jj) {
                float v = fmaxf((cal_ok & 1) ? fabsf(s0[jj]) : 0.f, (cal_ok & 2) ? fabsf(s1[jj]) : 0.f);
#pragma unroll
                for (int off = 32; off > 0; off >>= 1) v = fmaxf(v, __shfl_xor(v, off));
                if (lane == 0 && v > 0.f) atomicMax(a.amax + br * a.cin + cbase + jj, __float_as_uint(v));
              }
            }
          }
        }
      }
    }
    __syncthreads();
    // ---- 1x1 GEMM over this chunk: [128 px x KC] x [KC x cout_pad] ----
    if constexpr (I8) {
#pragma unroll
      for (int ks = 0; ks < ((ABL & 2) ? 0 : KC8 / 64); ++ks) {
        i32x4 af[4];
#pragma unroll
        for (int tm = 0; tm < 4; ++tm) af[tm] = *(const i32x4*)(At8 + (wm * 64 + tm * 16 + fr) * AS8 + ks * 64 + g * 16);
#pragma unroll
        for (int tm = 0; tm < 4; ++tm)
#pragma unroll
          for (int tn = 0; tn < NF; ++tn)
            acc[tm][tn] = __builtin_amdgcn_mfma_i32_16x16x64_i8(af[tm], bf8[ks][tn], acc[tm][tn], 0, 0, 0);
      }
    } else {
#pragma unroll
      for (int ks = 0; ks < ((ABL & 2) ? 0 : KC / 32); ++ks) {
        h8 af[4];
#pragma unroll
        for (int tm = 0; tm < 4; ++tm) af[tm] = *(const h8*)(At + (wm * 64 + tm * 16 + fr) * AS + ks * 32 + g * 8);
#pragma unroll
        for (int tm = 0; tm < 4; ++tm)
#pragma unroll
          for (int tn = 0; tn < NF; ++tn)
            acc[tm][tn] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[tm], bf[ks][tn], acc[tm][tn], 0, 0, 0);
      }
    }
    if (ch == nch - 1) {
      // ---- epilogue: bias -> LeakyReLU (0 < slope < 1: max(x, slope x)) -> BN affine ->
      //      (2x2 max) -> fp16; 32-bit offsets from a per-image base ----
      const int tx = it.tx, ty = it.ty, n = it.n;
      const int oy0 = ty * TH, ox0 = tx * TW;
      const int ohp = oh >> 1, owp = ow >> 1;
      _Float16* outn = a.out + (size_t)n * (a.pool ? ohp * owp : oh * ow) * a.out_cs + wn * NF * 16 + fr;
#pragma unroll
      for (int tm = 0; tm < 4; ++tm) {
        const int qd = (wm * 64 + tm * 16 + g * 4) >> 2;
        const int qy = qd >> 3, qx = qd & 7;
        float v[NF][4];
#pragma unroll
        for (int tn = 0; tn < NF; ++tn)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float x = (I8 ? (float)acc[tm][tn][r] * e_d[tn] : (float)acc[tm][tn][r]) + e_b[tn];
            v[tn][r] = fmaxf(x, x * a.slope) * e_s[tn] + e_t[tn];
          }
        if (a.pool) {
          const int py = (oy0 >> 1) + qy, px = (ox0 >> 1) + qx;
          if (2 * py < a.lim_h && 2 * px < a.lim_w) {
            _Float16* o = outn + (py * owp + px) * a.out_cs;
#pragma unroll
            for (int tn = 0; tn < NF; ++tn)
              if (e_ok[tn]) o[tn * 16] = (_Float16)fmaxf(fmaxf(v[tn][0], v[tn][1]), fmaxf(v[tn][2], v[tn][3]));
          }
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int y = oy0 + 2 * qy + (r >> 1), x = ox0 + 2 * qx + (r & 1);
            if (y < a.lim_h && x < a.lim_w) {
              _Float16* o = outn + (y * ow + x) * a.out_cs;
#pragma unroll
              for (int tn = 0; tn < NF; ++tn)
                if (e_ok[tn]) o[tn * 16] = (_Float16)v[tn][r];
            }
          }
        }
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int jn = 0; jn < NF; ++jn) acc[i][jn] = AccT{0, 0, 0, 0};
    }
  };

  // two register prefetch sets: item j+2's halo is in flight while item j computes
  u32x4 preA[PV], preB[PV];
  Cur cc = cur_at(t0), pc = cc;  // computed item, prefetched item (two ahead)
  if (pc.tile < tend) prefetch(preA, pc);
  advance(pc);
  if (pc.tile < tend) prefetch(preB, pc);
  advance(pc);
  while (cc.tile < tend) {
    stage(preA, xs);
    __syncthreads();
    load_bf(cc.ch);
    if (pc.tile < tend) prefetch(preA, pc);
    advance(pc);
    process(cc, xs);
    advance(cc);
    if (cc.tile >= tend) break;
    stage(preB, xs + XS);
    __syncthreads();
    load_bf(cc.ch);
    if (pc.tile < tend) prefetch(preB, pc);
    advance(pc);
    process(cc, xs + XS);
    advance(cc);
  }
}

int acff_persist_mode() { return tune().acff_persist; }

// Channel chunk of the persistent kernel for cin (0 = not eligible).
int acff_persist_chunk(int cin, int cout_pad, int oh) {
  if (cout_pad != 64 && cout_pad != 96 && cout_pad != 128) return 0;
  if (oh < 24) return 0;  // small maps: 8 x 16 tiles would mostly idle
  if (cin > kAcffPMaxCin) return 0;
  // 16-channel chunks for every cin: (CC = 32 chunks need ~40 more VGPRs and spill)
  return cin % 16 == 0 ? 16 : 0;
}

void launch_acff_persist(const void* in, int in_cs, int in_co, int n, int h, int w, int cin, int lim_h, int lim_w,
                         const float* dw_wt, const float* dw_b, const void* pwc, int cout, int cout_pad,
                         const float* bias, const float* scale, const float* shift, float slope, void* out, int out_cs,
                         int pool, hipStream_t s, const AcffI8* q) {
  const int cc = acff_persist_chunk(cin, cout_pad, h - 2);
  RTDM_REQUIRE(cc > 0, RTDM_E_INVALID, "acff_persist: unsupported shape");
  RTDM_REQUIRE((in_cs % 8) == 0 && (in_co % 8) == 0, RTDM_E_INVALID, "acff_persist: input view not 16-byte aligned");
  RTDM_REQUIRE(!pool || ((lim_h | lim_w) & 1) == 0, RTDM_E_INVALID, "acff_persist: odd pooled limit");
  RTDM_REQUIRE((int64_t)n * h * w * in_cs < (1ll << 31), RTDM_E_CAPACITY, "acff_persist: input map over 2^31 elements");
  AcffPArgs a;
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
  a.pw = (const _Float16*)pwc;
  a.cout = cout;
  a.cout_pad = cout_pad;
  a.bias = bias;
  a.scale = scale;
  a.shift = shift;
  a.slope = slope;
  a.out = (_Float16*)out;
  a.out_cs = out_cs;
  a.pool = pool;
  const bool i8 = q && q->w8;
  a.pw8 = i8 ? (const int8_t*)q->w8 : nullptr;
  a.deq = i8 ? q->deq : nullptr;
  a.inv_s = i8 ? q->inv_s : nullptr;
  a.amax = q && !i8 ? q->amax : nullptr;
  const int64_t tiles = (int64_t)n * ((lim_h + 7) / 8) * ((lim_w + 15) / 16);
  if (tiles <= 0) return;
  RTDM_REQUIRE(tiles < (1ll << 31), RTDM_E_CAPACITY, "acff_persist: too many tiles");
  // CU count and resident blocks per (kernel, LDS bytes) queried once per process: these
  // host calls ran on every launch, and the small per-rank batches are launch-bound on the host
  static const int cus = [] {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v < 1)
      v = 256;
    return v;
  }();
  const size_t lds = (size_t)(i8 ? 33 : 30) * cin * sizeof(float);
  auto go = [&](auto kern) {
    static std::mutex mu;
    static std::map<std::pair<const void*, size_t>, int> occ;
    int per_cu = 1;
    {
      std::lock_guard<std::mutex> lk(mu);
      const auto key = std::make_pair((const void*)kern, lds);
      auto it = occ.find(key);
      if (it == occ.end()) {
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, 256, lds) != hipSuccess || per_cu < 1) per_cu = 1;
        occ.emplace(key, per_cu);
      } else {
        per_cu = it->second;
      }
    }
    const int64_t blocks = std::min<int64_t>(tiles, (int64_t)per_cu * cus);
    hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(256), lds, s, a);
  };
  const int abl = acff_persist_mode() - 1;  // >1: diagnostic ablations
  if (cc == 16) {
    RTDM_REQUIRE(cout_pad != 96 || (!i8 && abl <= 0), RTDM_E_INVALID,
                 "acff_persist: 96 output rows are for the fp16 / calibration kernels");
    if (i8) cout_pad == 64 ? go(acff_persist<16, 2, 0, 1>) : go(acff_persist<16, 4, 0, 1>);
    else if (a.amax) cout_pad == 64 ? go(acff_persist<16, 2, 0, 2>) : cout_pad == 96 ? go(acff_persist<16, 3, 0, 2>) : go(acff_persist<16, 4, 0, 2>);
    else if (cout_pad == 96) go(acff_persist<16, 3>);
    else if (abl == 1) cout_pad == 64 ? go(acff_persist<16, 2, 1>) : go(acff_persist<16, 4, 1>);
    else if (abl == 2) cout_pad == 64 ? go(acff_persist<16, 2, 2>) : go(acff_persist<16, 4, 2>);
    else if (abl == 4) cout_pad == 64 ? go(acff_persist<16, 2, 4>) : go(acff_persist<16, 4, 4>);
    else cout_pad == 64 ? go(acff_persist<16, 2>) : go(acff_persist<16, 4>);
  }
  RTDM_HIP(hipGetLastError());
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


// --------------------------------------------------------------------------
// acff_chain: the classifier's small-map suffix in ONE launch, one 512-thread
// block per image: ACFF stages without pooling (ErNET acff4..6, Squeeze acff4)
// run back to back on an LDS-resident activation map, then the tail (conv2 1x1
// -> AvgPool -> view -> Linear -> Softmax, squeeze_ernet.py:33-41 /
// ernet.py:38-45).  Per stage, per dilation branch: depthwise taps (VALU, fp32
// accumulate, same FMA order as acff_fused) -> fp16 A chunk [M][C] in LDS ->
// this branch's K slice of the 1x1 GEMM on v_mfma_f32_16x16x32_f16 (B fragments
// from the L2-resident packed weights; K order branch*C + c, so the fp32
// accumulation sequence is acff_fused's) -> bias / LeakyReLU / BN affine ->
// fp16 map for the next stage.  The activations never leave the CU: the
// unfused path's 3 launches + tail and their HBM round trips become one launch,
// bit-identical results.
// --------------------------------------------------------------------------
static constexpr int kChainMaxStages = 4;
static constexpr int kChainThreads = 512;

struct AcffChainStage {
  const float* dw_wt;   // [3][9][cin]
  const float* dw_b;    // [3][cin]
  const _Float16* pw;   // [cout_pad][kpad], k = branch*cin + c
  const int8_t* pw8;    // int8: [cout_pad][3 cin], k = branch*cin + c (AcffI8)
  const float* deq;
  const float* inv_s;   // [3][cin]
  unsigned* amax;       // calibration (fp16 run)
  const float* bias;
  const float* scale;
  const float* shift;
  int cin, cout, cout_pad, kpad, h;  // square input side h
};

struct AcffChainArgs {
  const _Float16* in;
  int in_cs, in_co;
  int nst;
  AcffChainStage st[kChainMaxStages];
  float slope;
  int act_bytes;  // bytes of each of the two LDS activation buffers
  int a_bytes;    // bytes of the A chunk
  // tail
  const float* w2;  // [5][c]
  int pool_pad, ph, pw;
  const float* fcw;
  const float* fcb;
  float* logits;
  float* probs;
  int abl;  // diagnostics (wrong outputs): 1 no depthwise, 2 no 1x1 MFMA, 4 no tail
  unsigned long long* stamps;  // diagnostics (acff_chain mode 16): block 0's s_memtime at each phase
};

template <int MODE>  // 0 fp16, 1 int8 1x1 fusion, 2 fp16 + calibration
__global__ __launch_bounds__(kChainThreads) void acff_chain(AcffChainArgs a) {
  constexpr bool I8 = MODE == 1, CAL = MODE == 2;
  extern __shared__ __attribute__((aligned(16))) unsigned char chain_lds[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int img = blockIdx.x;
  int nst_ = 0;
  auto stamp = [&]() {
    if (a.stamps && img == 0 && tid == 0) a.stamps[nst_] = __builtin_amdgcn_s_memtime();
    ++nst_;
  };
  stamp();
  // the two activation maps as byte offsets into chain_lds: a runtime-indexed array of the
  // two pointers lost their LDS address space (every depthwise tap became a flat load that
  // also waited on the in-flight global weight loads)
  auto act = [&](int k) { return (_Float16*)(chain_lds + k * a.act_bytes); };
  _Float16* At = (_Float16*)(chain_lds + 2 * a.act_bytes);
  int8_t* const At8 = (int8_t*)At;  // int8 A chunk [M][C + 16] bytes (inside the fp16 one)
  float* wsm = (float*)(chain_lds + 2 * a.act_bytes + a.a_bytes);  // [3][9][C], bias [3][C] (int8: inv_s [3][C])
  typedef int i32x4 __attribute__((ext_vector_type(4)));
  using AccT = std::conditional_t<I8, i32x4, f4>;

  {  // input map of stage 0: [h*h][cin] fp16 from the NHWC view
    const int h = a.st[0].h, C = a.st[0].cin, CG = C >> 3;
    const _Float16* src = a.in + (size_t)img * h * h * a.in_cs + a.in_co;
    for (int i = tid; i < h * h * CG; i += kChainThreads) {
      const int px = i / CG, v = i - px * CG;
      *(uint4*)(act(0) + (size_t)px * (C + 8) + v * 8) = *(const uint4*)(src + (size_t)px * a.in_cs + v * 8);
    }
  }
  int cur = 0;
  const int fr = lane & 15, g = lane >> 4;
  // depthwise taps + biases of a stage -> wsm.  Stage 0 here; stage si + 1's are loaded into
  // registers while stage si runs and stored once its last depthwise phase is done (each
  // stage used to start by waiting on these global loads).
  constexpr int NW = I8 ? 33 : 30;  // floats per channel in wsm
  constexpr int kWPre = (NW * 128 + kChainThreads - 1) / kChainThreads;  // cin <= 128
  auto wload = [&](const AcffChainStage& st, float (&pre)[kWPre]) {
#pragma unroll
    for (int k = 0; k < kWPre; ++k) {
      const int i = tid + k * kChainThreads;
      pre[k] = i < 27 * st.cin   ? st.dw_wt[i]
               : i < 30 * st.cin ? st.dw_b[i - 27 * st.cin]
               : (I8 && i < 33 * st.cin) ? st.inv_s[i - 30 * st.cin]
                                          : 0.f;
    }
  };
  auto wstore = [&](const AcffChainStage& st, const float (&pre)[kWPre]) {
#pragma unroll
    for (int k = 0; k < kWPre; ++k) {
      const int i = tid + k * kChainThreads;
      if (i < NW * st.cin) wsm[i] = pre[k];
    }
  };
  if (a.nst > 0) {
    float pre0[kWPre];
    wload(a.st[0], pre0);
    wstore(a.st[0], pre0);
  }
  for (int si = 0; si < a.nst; ++si) {
    const AcffChainStage& st = a.st[si];
    const int H = st.h, OH = H - 2, M = OH * OH, C = st.cin, CG = C >> 3, AS = C + 8;
    float wpre[kWPre];
    if (si + 1 < a.nst) wload(a.st[si + 1], wpre);
    // this lane's epilogue constants (2 channels), loaded now so the epilogue does not wait
    float e_b[2], e_s[2], e_t[2], e_d[2];
    {
      const int wn0 = st.cout_pad >> 5, wni0 = wid - (wid / wn0) * wn0;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int c = wni0 * 32 + j * 16 + fr;
        const bool cv = c < st.cout;
        e_d[j] = I8 && cv ? st.deq[c] : 1.f;
        e_b[j] = cv ? st.bias[c] : 0.f;
        e_s[j] = cv && st.scale ? st.scale[c] : 1.f;
        e_t[j] = cv && st.scale ? st.shift[c] : 0.f;
      }
    }
    __syncthreads();  // input map + dw weights ready; the previous stage's A reads are done
    stamp();
    const _Float16* X = act(cur);
    _Float16* Y = act(cur ^ 1);
    const int wn = st.cout_pad >> 5, wm = 8 / wn;  // wave grid: wm (M) x wn (N), 32 channels per wave
    const int wmi = wid / wn, wni = wid - wmi * wn;
    const int mtiles = (M + 15) >> 4;
    const int fm = (mtiles + wm - 1) / wm;  // <= 4 (plan-time check)
    const int m_base = wmi * fm * 16, n_base = wni * 32;
    AccT acc[4][2];
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[i][0] = acc[i][1] = AccT{0, 0, 0, 0};
    const int AS8 = C + 16;
    for (int br = 0; br < 3; ++br) {
      const int d = br + 1;
      const float* wb = wsm + br * 9 * C;
      const float* bb = wsm + 27 * C + br * C;
      // this branch's 1x1 weight fragments (global, L2-resident), issued before the
      // depthwise phase so their latency hides under it (C <= 128: 4 k-steps)
      const _Float16* wrow = st.pw + (size_t)(n_base + fr) * st.kpad + br * C + g * 8;
      const int nks = C / 32;
      h8 bpre[I8 ? 1 : 4][2];
      i32x4 bpre8[I8 ? 2 : 1][2];
      if constexpr (I8) {  // k-steps of 64: C / 64 <= 2
        const int8_t* w8row = st.pw8 + (size_t)(n_base + fr) * 3 * C + br * C + g * 16;
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
          if (ks < C / 64) {
            bpre8[ks][0] = *(const i32x4*)(w8row + ks * 64);
            bpre8[ks][1] = *(const i32x4*)(w8row + (size_t)16 * 3 * C + ks * 64);
          }
      } else {
#pragma unroll
        for (int ks = 0; ks < 4; ++ks)
          if (ks < nks && C <= 128) {
            bpre[ks][0] = *(const h8*)(wrow + ks * 32);
            bpre[ks][1] = *(const h8*)(wrow + (size_t)16 * st.kpad + ks * 32);
          }
      }
      // one (pixel m, 8-channel group v) item: bias, then the 9 taps in (kh, kw) order (fp32
      // FMAs, acff_fused's sequence) -> the A chunk (fp16, or int8 quantised)
      auto dw_item = [&](int m, int oy, int ox, int v, const f4 (&wk)[9][2], const f4 (&bk)[2]) {
        float t[8];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          t[j] = bk[0][j];
          t[4 + j] = bk[1][j];
        }
        // the centre tap's offset once per item; each tap adds a wave-uniform shift, and the
        // border tests are per tap row / column (d = 1 taps never leave the map: padding 0)
        const int pc = ((oy + 1) * H + ox + 1) * (C + 8) + v * 8;
        const int dp = d * (C + 8), dr = d * H * (C + 8);
        const bool r0 = oy + 1 - d >= 0, r2 = oy + 1 + d < H, c0 = ox + 1 - d >= 0, c2 = ox + 1 + d < H;
#pragma unroll
        for (int kh = 0; kh < 3; ++kh)
#pragma unroll
          for (int kw = 0; kw < 3; ++kw) {
            const bool ok = (kh == 0 ? r0 : kh == 2 ? r2 : true) && (kw == 0 ? c0 : kw == 2 ? c2 : true);
            h8 xv = h8{0, 0, 0, 0, 0, 0, 0, 0};
            if (ok) xv = *(const h8*)(X + pc + (kh - 1) * dr + (kw - 1) * dp);
            const f4& w0 = wk[kh * 3 + kw][0];
            const f4& w1 = wk[kh * 3 + kw][1];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              t[j] = fmaf(w0[j], (float)xv[j], t[j]);
              t[4 + j] = fmaf(w1[j], (float)xv[4 + j], t[4 + j]);
            }
          }
        if constexpr (I8) {
          const float* ip = wsm + 30 * C + br * C + v * 8;
          uint32_t lo = 0, hi = 0;
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            int q = (int)rintf(t[j] * ip[j]);
            q = q < -127 ? -127 : (q > 127 ? 127 : q);
            if (j < 4)
              lo |= ((uint32_t)q & 255u) << (8 * j);
            else
              hi |= ((uint32_t)q & 255u) << (8 * (j - 4));
          }
          *(uint2*)(At8 + (size_t)m * AS8 + v * 8) = make_uint2(lo, hi);
        } else {
          h8 o;
          // (opaque: the f32 sums round to fp16 on their own, as in the per-stage kernels,
          // instead of folding the last tap's FMA into an fp16-result mix op)
#pragma unroll
          for (int j = 0; j < 8; ++j) asm volatile("" : "+v"(t[j]));
#pragma unroll
          for (int j = 0; j < 8; ++j) o[j] = (_Float16)t[j];
          *(h8*)(At + (size_t)m * AS + v * 8) = o;
          if constexpr (CAL) {  // calibration: |x|max per concat channel
#pragma unroll
            for (int j = 0; j < 8; ++j)
              if (t[j] != 0.f) atomicMax(st.amax + br * C + v * 8 + j, __float_as_uint(fabsf(t[j])));
          }
        }
      };
      auto wtaps = [&](int v, f4 (&wk)[9][2], f4 (&bk)[2]) {
#pragma unroll
        for (int k = 0; k < 9; ++k) {
          wk[k][0] = *(const f4*)(wb + k * C + v * 8);
          wk[k][1] = *(const f4*)(wb + k * C + v * 8 + 4);
        }
        bk[0] = *(const f4*)(bb + v * 8);
        bk[1] = *(const f4*)(bb + v * 8 + 4);
      };
      if (!(a.abl & 1)) {
        // a thread keeps one channel group (its 72 tap weights + 8 biases in registers) and
        // walks the pixels: per tap one 16-byte LDS read (the activation) instead of three
        const int pstep = kChainThreads / CG, v = tid % CG;
        if (tid < pstep * CG) {
          f4 wk[9][2], bk[2];
          wtaps(v, wk, bk);
          // (pixel m -> (oy, ox) stepped, not divided: an integer division per item was ~20
          // VALU against its 72 FMAs)
          const int m0 = tid / CG, dq = pstep / OH, dr = pstep - dq * OH;
          int oy = m0 / OH, ox = m0 - oy * OH;
          for (int m = m0; m < M; m += pstep) {
            dw_item(m, oy, ox, v, wk, bk);
            ox += dr;
            oy += dq;
            if (ox >= OH) {
              ox -= OH;
              ++oy;
            }
          }
        }
      }
      __syncthreads();
      stamp();
      // this branch's K slice: k = br*C + [0, C)
      auto kstep8 = [&](int ks, const i32x4& b0, const i32x4& b1) {
#pragma unroll
        for (int tm = 0; tm < 4; ++tm) {
          if (tm < fm && m_base + tm * 16 < M) {
            const int row = m_base + tm * 16 + fr;
            const i32x4 av = *(const i32x4*)(At8 + (size_t)(row < M ? row : M - 1) * AS8 + ks * 64 + g * 16);
            if constexpr (I8) {
              acc[tm][0] = __builtin_amdgcn_mfma_i32_16x16x64_i8(av, b0, acc[tm][0], 0, 0, 0);
              acc[tm][1] = __builtin_amdgcn_mfma_i32_16x16x64_i8(av, b1, acc[tm][1], 0, 0, 0);
            }
          }
        }
      };
      auto kstep = [&](int ks, const h8& b0, const h8& b1) {
#pragma unroll
        for (int tm = 0; tm < 4; ++tm) {
          if (tm < fm && m_base + tm * 16 < M) {
            const int row = m_base + tm * 16 + fr;
            const h8 av = *(const h8*)(At + (size_t)(row < M ? row : M - 1) * AS + ks * 32 + g * 8);
            if constexpr (!I8) {
              acc[tm][0] = __builtin_amdgcn_mfma_f32_16x16x32_f16(av, b0, acc[tm][0], 0, 0, 0);
              acc[tm][1] = __builtin_amdgcn_mfma_f32_16x16x32_f16(av, b1, acc[tm][1], 0, 0, 0);
            }
          }
        }
      };
      if (a.abl & 2) {
      } else if constexpr (I8) {
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
          if (ks < C / 64) kstep8(ks, bpre8[ks][0], bpre8[ks][1]);
      } else if (C <= 128) {
#pragma unroll
        for (int ks = 0; ks < 4; ++ks)
          if (ks < nks) kstep(ks, bpre[ks][0], bpre[ks][1]);
      } else {
        for (int ks = 0; ks < nks; ++ks)
          kstep(ks, *(const h8*)(wrow + ks * 32), *(const h8*)(wrow + (size_t)16 * st.kpad + ks * 32));
      }
      if (br == 2 && si + 1 < a.nst) wstore(a.st[si + 1], wpre);  // this stage's taps are no longer read
      __syncthreads();  // the A chunk is rewritten by the next branch
      stamp();
    }
    // epilogue: bias -> LeakyReLU -> BN affine -> fp16 map Y [M][cout]
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int c = n_base + j * 16 + fr;
      if (c >= st.cout) continue;
      const float bc = e_b[j], sc = e_s[j], sh = e_t[j], dq = e_d[j];
#pragma unroll
      for (int tm = 0; tm < 4; ++tm) {
        if (!(tm < fm)) continue;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = m_base + tm * 16 + g * 4 + r;
          if (m < M) {
            float x = (I8 ? (float)acc[tm][j][r] * dq : (float)acc[tm][j][r]) + bc;
            x = x > 0.f ? x : x * a.slope;
            Y[(size_t)m * (st.cout + 8) + c] = (_Float16)fmaf(x, sc, sh);  // pixel stride cout + 8
          }
        }
      }
    }
    cur ^= 1;
  }
  __syncthreads();
  stamp();
  if (a.abl & 4) return;
  // ---- tail on the last map: [hw][c], c = last cout ----
  const int h = a.nst > 0 ? a.st[a.nst - 1].h - 2 : a.st[0].h, hw = h * h;
  const int c = a.nst > 0 ? a.st[a.nst - 1].cout : a.st[0].cin;
  const _Float16* X = act(cur);
  float* conv = (float*)At;  // [5][hw]
  // conv2 1x1 (c -> 5): one (output, pixel) pair per thread, weights from LDS, four partial
  // sums over the channels (was a wave per pixel with shuffle reductions)
  // (pixel stride c + 8 halfs: consecutive pixels' lanes read distinct banks; with stride c
  // every lane of a 16-lane group hit the same four)
  float* w2s = wsm;  // [5][c], the stage taps are dead
  const int nf = 5 * a.ph * a.pw;
  float* fcs = wsm + 5 * c;  // [5][nf] fc weights, staged with w2 (the fc read them from global)
  for (int i = tid; i < 5 * c; i += kChainThreads) w2s[i] = a.w2[i];
  for (int i = tid; i < 5 * nf; i += kChainThreads) fcs[i] = a.fcw[i];
  __syncthreads();
  stamp();
  for (int t = tid; t < 5 * hw; t += kChainThreads) {
    const int o = t / hw, p = t - o * hw;
    const _Float16* x = X + (size_t)p * (c + 8);
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
  stamp();
  float* feat = conv + 5 * hw;  // [5*ph*pw]
  for (int t = tid; t < nf; t += kChainThreads) {
    const int o = t / (a.ph * a.pw);
    const int r = t - o * a.ph * a.pw;
    const int i = r / a.pw, j = r - (r / a.pw) * a.pw;
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
  stamp();
  float* lg = feat + nf;
  if (tid < 5) {
    float s1 = 0.f;
    for (int q = 0; q < nf; ++q) s1 = fmaf(feat[q], fcs[tid * nf + q], s1);
    s1 += a.fcb[tid];
    lg[tid] = s1;
    if (a.logits) a.logits[img * 5 + tid] = s1;
  }
  __syncthreads();
  stamp();
  if (tid < 5 && a.probs) {
    float mx = lg[0];
    for (int k = 1; k < 5; ++k) mx = fmaxf(mx, lg[k]);
    float sum = 0.f;
    for (int k = 0; k < 5; ++k) sum += expf(lg[k] - mx);
    a.probs[img * 5 + tid] = expf(lg[tid] - mx) / sum;
  }
  stamp();
}

int acff_chain_mode() { return tune().acff_chain; }

size_t acff_chain_lds(const AcffChainPlan& p) {
  size_t act = 0, ab = 0;
  int cmax = 0;
  for (int i = 0; i < p.nst; ++i) {
    const int h = p.h[i], oh = h - 2;
    act = std::max(act, (size_t)h * h * (p.cin[i] + 8) * 2);  // pixel stride C + 8 (banks)
    act = std::max(act, (size_t)oh * oh * (p.cout[i] + 8) * 2);
    ab = std::max(ab, (size_t)oh * oh * (p.cin[i] + 8) * 2);
    cmax = std::max(cmax, p.cin[i]);
  }
  act = (size_t)round_up((int64_t)act, 16);
  const int oh = p.h[p.nst - 1] - 2;
  ab = std::max(ab, (size_t)(5 * oh * oh + 5 * 16 + 8) * 4);  // the tail reuses the A chunk
  ab = (size_t)round_up((int64_t)ab, 16);
  return 2 * act + ab + (size_t)33 * cmax * 4;  // wsm: taps, biases (+ int8 inverse scales)
}

bool acff_chain_ok(const AcffChainPlan& p) {
  if (p.nst < 1 || p.nst > kChainMaxStages) return false;
  for (int i = 0; i < p.nst; ++i) {
    const int oh = p.h[i] - 2, M = oh * oh;
    if (p.cin[i] % 32 != 0 || p.kpad[i] < 3 * p.cin[i] || oh < 1) return false;
    const int wn = p.cout_pad[i] / 32;
    if (p.cout_pad[i] % 32 != 0 || (wn != 1 && wn != 2 && wn != 4 && wn != 8)) return false;
    const int wm = 8 / wn, mtiles = (M + 15) / 16;
    if ((mtiles + wm - 1) / wm > 4) return false;
    if (i > 0 && (p.h[i] != p.h[i - 1] - 2 || p.cin[i] != p.cout[i - 1])) return false;
  }
  const int oh = p.h[p.nst - 1] - 2;
  if (oh * oh > 64 * 16) return false;
  int cmax = 0;
  for (int i = 0; i < p.nst; ++i) cmax = std::max(cmax, p.cin[i]);
  const int clast = p.cout[p.nst - 1];
  if (cmax > 128 || clast % 8 != 0 || 5 * clast + 5 * 5 * 16 > 30 * cmax) return false;  // register prefetch; tail conv2 + fc weights in wsm
  return acff_chain_lds(p) <= 160 * 1024;
}

void launch_acff_chain(const AcffChainPlan& p, const void* in, int in_cs, int in_co, int n, const float* const* dw_wt,
                       const float* const* dw_b, const void* const* pw, const float* const* bias,
                       const float* const* scale, const float* const* shift, float slope, const float* w2,
                       int pool_pad, int ph, int pwid, const float* fcw, const float* fcb, float* logits, float* probs,
                       hipStream_t s, const AcffI8* q) {
  RTDM_REQUIRE(acff_chain_ok(p), RTDM_E_INVALID, "acff_chain: unsupported plan");
  RTDM_REQUIRE((in_cs % 8) == 0 && (in_co % 8) == 0, RTDM_E_INVALID, "acff_chain: input view not 16-byte aligned");
  RTDM_REQUIRE(ph * pwid <= 16, RTDM_E_UNSUPPORTED, "acff_chain: pooled tail too large");
  if (n <= 0) return;
  AcffChainArgs a;
  a.in = (const _Float16*)in;
  a.in_cs = in_cs;
  a.in_co = in_co;
  a.nst = acff_chain_mode() == 2 ? 0 : p.nst;  // 2: tail only (diagnostics; stages skipped -> wrong)
  a.abl = acff_chain_mode() >= 8 && acff_chain_mode() < 16 ? (acff_chain_mode() - 8) & 7 : 0;  // 8 + bits: ablations
  static unsigned long long* stamps_dev = nullptr;  // mode 16: phase timestamps of block 0 (diagnostics)
  if (acff_chain_mode() == 16 && !stamps_dev) RTDM_HIP(hipMalloc(&stamps_dev, 64 * sizeof(unsigned long long)));
  a.stamps = acff_chain_mode() == 16 ? stamps_dev : nullptr;
  for (int i = 0; i < p.nst; ++i) {
    AcffChainStage& t = a.st[i];
    t.dw_wt = dw_wt[i];
    t.dw_b = dw_b[i];
    t.pw = (const _Float16*)pw[i];
    t.bias = bias[i];
    t.scale = scale[i];
    t.shift = shift[i];
    t.cin = p.cin[i];
    t.cout = p.cout[i];
    t.cout_pad = p.cout_pad[i];
    t.kpad = p.kpad[i];
    t.h = p.h[i];
    const bool i8 = q && q[i].w8;
    t.pw8 = i8 ? (const int8_t*)q[i].w8 : nullptr;
    t.deq = i8 ? q[i].deq : nullptr;
    t.inv_s = i8 ? q[i].inv_s : nullptr;
    t.amax = q && !i8 ? q[i].amax : nullptr;
  }
  const bool i8 = q && q[0].w8;
  for (int i = 0; i < p.nst; ++i)
    RTDM_REQUIRE(!q || (q[i].w8 != nullptr) == i8, RTDM_E_INVALID, "acff_chain: int8 on some stages only");
  if (i8)
    for (int i = 0; i < p.nst; ++i)
      RTDM_REQUIRE(p.cin[i] % 64 == 0, RTDM_E_UNSUPPORTED, "acff_chain: int8 needs cin % 64 == 0");
  a.slope = slope;
  size_t act = 0, ab = 0;
  for (int i = 0; i < p.nst; ++i) {
    const int h = p.h[i], oh = h - 2;
    act = std::max(act, (size_t)h * h * (p.cin[i] + 8) * 2);  // pixel stride C + 8 (banks)
    act = std::max(act, (size_t)oh * oh * (p.cout[i] + 8) * 2);
    ab = std::max(ab, (size_t)oh * oh * (p.cin[i] + 8) * 2);
  }
  const int ohl = p.h[p.nst - 1] - 2;
  ab = std::max(ab, (size_t)(5 * ohl * ohl + 5 * 16 + 8) * 4);
  a.act_bytes = (int)round_up((int64_t)act, 16);
  a.a_bytes = (int)round_up((int64_t)ab, 16);
  a.w2 = w2;
  a.pool_pad = pool_pad;
  a.ph = ph;
  a.pw = pwid;
  a.fcw = fcw;
  a.fcb = fcb;
  a.logits = logits;
  a.probs = probs;
  const size_t lds = acff_chain_lds(p);
  if (i8)
    hipLaunchKernelGGL(acff_chain<1>, dim3(n), dim3(kChainThreads), lds, s, a);
  else if (q && q[0].amax)
    hipLaunchKernelGGL(acff_chain<2>, dim3(n), dim3(kChainThreads), lds, s, a);
  else
    hipLaunchKernelGGL(acff_chain<0>, dim3(n), dim3(kChainThreads), lds, s, a);
  RTDM_HIP(hipGetLastError());
  if (a.stamps) {  // diagnostics: print block 0's phase durations (synchronises the stream)
    unsigned long long h[64] = {};
    RTDM_HIP(hipMemcpyAsync(h, a.stamps, sizeof h, hipMemcpyDeviceToHost, s));
    RTDM_HIP(hipStreamSynchronize(s));
    fprintf(stderr, "acff_chain phases (s_memtime ticks, n=%d):", n);
    for (int i = 1; i < 64 && h[i] >= h[i - 1] && h[i]; ++i) fprintf(stderr, " %llu", h[i] - h[i - 1]);
    fprintf(stderr, "\n");
  }
}

}  // namespace rtdm
