// Cin-32 3x3 convolutions (Darknet-53's stride-2 conv 32 -> 64 and the first residual
// block's 3x3 32 -> 64 + shortcut, yolov3 / yolov3-spp L1 and L3): a persistent MFMA kernel
// with the layer's weights resident in LDS and the input tile's halo staged once per tile.
//
// Replaces: nn.Conv2d(32, 64, 3, stride s, pad 1) + folded BatchNorm + LeakyReLU 0.1 of
// victim_localization/yolov3/models.py:23-44 as run by Darknet.forward (:345-347), with the
// shortcut add (:349-354) fused.
//
// These layers move ~6 bytes of HBM per MAC-row and do little arithmetic (K = 288): the
// generic implicit-GEMM tiles (conv_mfma: 128 x 64, K-blocks of 64 gathered per tap through
// registers) and the direct kernel (16 x 16 tiles, one Cin chunk, 8-byte NHWC stores) ran
// them at 0.11 / 0.14 ms per b16 416 frame batch, 2-3x their HBM time.  Here:
//   * a workgroup (4 waves; 8 at stride 2) loads the 64 x 288 weights into LDS once and walks output tiles
//     (TH x 16 pixels, grid-stride), so the weights are not re-read per tile;
//   * per tile the (TH-1)S+3 x 15S+3 halo (32 channels = 4 x 16 B per pixel) is staged
//     through registers: the next tile's halo loads are issued before this tile's MFMAs;
//   * K step = one tap's 32 channels = one v_mfma_f32_16x16x32_f16 k-depth: A = 16 weight
//     rows from LDS, B = 16 pixels of a tile row read at the tap's offset in the halo;
//   * the weight rows are stored so that MFMA row i of N-fragment n is output channel
//     (i/4)*16 + 4n + i%4: a lane's 4 fragments then hold 16 consecutive channels of one
//     pixel (channels 16g .. 16g+15), stored as two 16-byte vectors (4 lanes = one 128-byte
//     pixel line) after bias -> LeakyReLU -> (+ residual), epi_vec8_lean's operations.
// LDS pitches (pixel 48 / 40 halfs for stride 1 / 2, weight row 304 halfs, weight rows in
// fragment order) put the 16 lanes of each ds_read_b128 group on distinct bank slots.
// K order per output: taps 0..8, each tap's 32 channels inside one MFMA, as conv_mfma's
// K-blocks (k = tap*32 + c) and conv3_direct's k-steps.
#include "conv_epi.h"

#include <algorithm>

namespace rtdm {

constexpr int kC32TW = 16;  // tile columns (one fragment of pixels)
constexpr int kC32WP = 304;  // weight row pitch (halfs)

template <int S, int NW = 4>  // NW: waves per workgroup
struct C32Geom {
  static constexpr int RW = S == 1 ? 4 : 2;   // tile rows per wave
  static constexpr int TH = NW * RW;          // tile rows
  static constexpr int NT = 64 * NW;          // threads
  static constexpr int HR = (TH - 1) * S + 3, HW = (kC32TW - 1) * S + 3;
  static constexpr int PP = S == 1 ? 48 : 40;
  static constexpr int HALO = HR * HW * PP;        // halfs
  static constexpr int NVEC = HR * HW * 4;         // 16-byte vectors per halo
  static constexpr int NV = (NVEC + NT - 1) / NT;  // per thread
  static constexpr size_t LDS = (size_t)(HALO + 64 * kC32WP) * 2;
};

template <int S, bool RES, int NW>
__global__ __launch_bounds__(64 * NW) void conv3_c32(ConvArgs a, int ntiles) {
  using G = C32Geom<S, NW>;
  extern __shared__ __attribute__((aligned(16))) _Float16 c32_lds[];
  _Float16* const hs = c32_lds;
  _Float16* const ws = c32_lds + G::HALO;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int j = lane & 15, g = lane >> 4;
  const int tx_n = (a.ow + kC32TW - 1) / kC32TW, ty_n = (a.oh + G::TH - 1) / G::TH;
  const _Float16* __restrict__ in = (const _Float16*)a.in + a.in_co;

  auto tile_of = [&](int t, int& n, int& ty, int& tx) {
    tx = t % tx_n;
    const int t2 = t / tx_n;
    ty = t2 % ty_n;
    n = t2 / ty_n;
  };
  auto hload = [&](int t, u32x4 (&r)[G::NV]) {
    int n, ty, tx;
    tile_of(t, n, ty, tx);
    const int iy0 = ty * G::TH * S - 1, ix0 = tx * kC32TW * S - 1;
#pragma unroll
    for (int k = 0; k < G::NV; ++k) {
      const int v = tid + k * G::NT;
      const int pix = v >> 2, c = v & 3;
      const int hr = pix / G::HW, col = pix - hr * G::HW;
      const int y = iy0 + hr, x = ix0 + col;
      const bool ok = v < G::NVEC && (unsigned)y < (unsigned)a.ih && (unsigned)x < (unsigned)a.iw;
      r[k] = u32x4{0u, 0u, 0u, 0u};
      if (ok) r[k] = *(const u32x4*)(in + ((size_t)(n * a.ih + y) * a.iw + x) * a.in_cs + c * 8);
    }
  };
  auto hstore = [&](const u32x4 (&r)[G::NV]) {
#pragma unroll
    for (int k = 0; k < G::NV; ++k) {
      const int v = tid + k * G::NT;
      if (v < G::NVEC) *(u32x4*)(hs + (v >> 2) * G::PP + (v & 3) * 8) = r[k];
    }
  };

  int t = blockIdx.x;
  u32x4 pre[G::NV];
  if (t < ntiles) hload(t, pre);
  // weights -> LDS, row q = 16n + i holds output channel (i/4)*16 + 4n + i%4 (k = tap*32 + c)
  for (int v = tid; v < 64 * 36; v += G::NT) {
    const int q = v / 36, kv = v - q * 36;
    const int n = q >> 4, i = q & 15;
    const int co = (i >> 2) * 16 + 4 * n + (i & 3);
    *(u32x4*)(ws + q * kC32WP + kv * 8) = *(const u32x4*)((const _Float16*)a.w + (size_t)co * a.kpad + kv * 8);
  }
  // this lane's 16 channels: bias
  const Epilogue& e = a.e;
  const int c0 = 16 * g;
  const bool cval = c0 < a.cout;  // cout % 16 == 0 (c32_ok)
  float bias[16];
#pragma unroll
  for (int q = 0; q < 16; ++q) bias[q] = cval && e.bias ? e.bias[c0 + q] : 0.f;
  const float slp = e.act == ACT_LEAKY ? e.slope : 1.f;  // LeakyReLU as max(x, slope x) (c32_ok)

  for (; t < ntiles; t += gridDim.x) {
    hstore(pre);
    __syncthreads();  // halo (and, first time round, the weights) visible
    if (t + (int)gridDim.x < ntiles) hload(t + gridDim.x, pre);  // lands under this tile's MFMAs
    f4 acc[G::RW][4];
#pragma unroll
    for (int f = 0; f < G::RW; ++f)
#pragma unroll
      for (int n = 0; n < 4; ++n) acc[f][n] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      const int kh = tap / 3, kw = tap % 3;
      h8 wf[4];
#pragma unroll
      for (int n = 0; n < 4; ++n) wf[n] = *(const h8*)(ws + (n * 16 + j) * kC32WP + tap * 32 + g * 8);
#pragma unroll
      for (int f = 0; f < G::RW; ++f) {
        const h8 xf = *(const h8*)(hs + (((wid * G::RW + f) * S + kh) * G::HW + j * S + kw) * G::PP + g * 8);
#pragma unroll
        for (int n = 0; n < 4; ++n) acc[f][n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wf[n], xf, acc[f][n], 0, 0, 0);
      }
    }
    __syncthreads();  // every wave is done with the halo before the next tile's store
    int n, ty, tx;
    tile_of(t, n, ty, tx);
    const int ox = tx * kC32TW + j;
#pragma unroll
    for (int f = 0; f < G::RW; ++f) {
      const int oy = ty * G::TH + wid * G::RW + f;
      if (!cval || oy >= a.oh || ox >= a.ow) continue;
      const size_t pix = ((size_t)n * a.oh + oy) * a.ow + ox;
      h8v rv[2];
      if constexpr (RES) {
        const _Float16* rp = (const _Float16*)e.res.ptr + pix * e.res.cs + e.res.co + c0;
        rv[0] = *(const h8v*)rp;
        rv[1] = *(const h8v*)(rp + 8);
      }
      h8v hv[2];
#pragma unroll
      for (int nn = 0; nn < 4; ++nn)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int q = 4 * nn + r;  // channel c0 + q
          float x = acc[f][nn][r] + bias[q];
          x = fmaxf(x, x * slp);
          // (opaque: x * slope rounds to fp32 before the fp16 conversion, as in the other
          // epilogues, instead of folding into one single-rounding fp16-result mix op)
          asm volatile("" : "+v"(x));
          x = x * 1.f + 0.f;  // epi_vec8_lean's (absent) BN affine: -0 -> +0 as there
          if constexpr (RES) x += (float)rv[q >> 3][q & 7];
          hv[q >> 3][q & 7] = (_Float16)x;
        }
      _Float16* op = (_Float16*)e.full.ptr + pix * e.full.cs + e.full.co + c0;
      *(h8v*)op = hv[0];
      *(h8v*)(op + 8) = hv[1];
    }
  }
}

// conv3_c32r: Darknet-53's first residual block in one launch — the 1x1 reduce (64 -> 32,
// Darknet.forward models.py:345-347), the 3x3 (32 -> 64) and the shortcut add (:349-354) —
// for a 16 x 16 output tile per step of a persistent walk:
//   1. the tile's 18 x 18 halo of the block input X (64 channels, pitch 80 halfs) is staged
//      from registers (the next tile's halo loads are issued before this tile's MFMAs);
//   2. the 1x1 runs on every halo pixel inside the image (21 fragments of 16 pixels over the 4
//      waves, 2 k-steps of 32 channels, conv_mfma's order), bias -> LeakyReLU (rounded to
//      fp32) -> fp16 into the Y halo (32 channels, pitch 48); pixels outside the image are
//      zero (the 3x3's padding);
//   3. the 3x3 is conv3_c32<1>'s loop on the Y halo, and its residual is X at the tile's
//      pixels, read from the staged halo instead of HBM.
// The reduce map (Y) never reaches HBM: per output pixel 128 B of X in (with the halo) and
// 128 B out, against 128 + 64 + 64 + 128 + 128 B for the two launches.  Every value takes
// the unfused kernels' operations in their order: bit-identical (tests/test_gpu_c32.py).
constexpr int kC32rPX = 80;                           // X halo pixel pitch (halfs)
constexpr int kC32rHP = C32Geom<1>::HR * C32Geom<1>::HW;  // 324 halo pixels
constexpr int kC32rXV = kC32rHP * 8;                  // 16-byte vectors of the X halo
constexpr size_t kC32rLDS = (size_t)(kC32rHP * kC32rPX + C32Geom<1>::HALO + 64 * kC32WP) * 2;

template <int NW>  // waves per workgroup (4 | 8)
__global__ __launch_bounds__(64 * NW) void conv3_c32r(ConvArgs a1, ConvArgs a, int ntiles) {
  using G = C32Geom<1>;
  constexpr int NT = 64 * NW, RW = G::TH / NW;        // threads; tile rows per wave
  constexpr int kC32rNV = (kC32rXV + NT - 1) / NT;    // X halo vectors per thread
  extern __shared__ __attribute__((aligned(16))) _Float16 c32r_lds[];
  _Float16* const xs = c32r_lds;                      // X halo [324][80]
  _Float16* const hs = xs + kC32rHP * kC32rPX;        // Y halo [324][48]
  _Float16* const ws = hs + G::HALO;                  // 3x3 weights
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int j = lane & 15, g = lane >> 4;
  const int tx_n = (a.ow + kC32TW - 1) / kC32TW, ty_n = (a.oh + G::TH - 1) / G::TH;
  const _Float16* __restrict__ in = (const _Float16*)a1.in + a1.in_co;

  auto tile_of = [&](int t, int& n, int& ty, int& tx) {
    tx = t % tx_n;
    const int t2 = t / tx_n;
    ty = t2 % ty_n;
    n = t2 / ty_n;
  };
  auto hload = [&](int t, u32x4 (&r)[kC32rNV]) {
    int n, ty, tx;
    tile_of(t, n, ty, tx);
    const int iy0 = ty * G::TH - 1, ix0 = tx * kC32TW - 1;
#pragma unroll
    for (int k = 0; k < kC32rNV; ++k) {
      const int v = tid + k * NT;
      const int pix = v >> 3, c = v & 7;
      const int hr = pix / G::HW, col = pix - hr * G::HW;
      const int y = iy0 + hr, x = ix0 + col;
      const bool ok = v < kC32rXV && (unsigned)y < (unsigned)a1.ih && (unsigned)x < (unsigned)a1.iw;
      r[k] = u32x4{0u, 0u, 0u, 0u};
      if (ok) r[k] = *(const u32x4*)(in + ((size_t)(n * a1.ih + y) * a1.iw + x) * a1.in_cs + c * 8);
    }
  };

  int t = blockIdx.x;
  u32x4 pre[kC32rNV];
  if (t < ntiles) hload(t, pre);
  // 3x3 weights -> LDS (conv3_c32's fragment-ordered rows)
  for (int v = tid; v < 64 * 36; v += NT) {
    const int q = v / 36, kv = v - q * 36;
    const int n = q >> 4, i = q & 15;
    const int co = (i >> 2) * 16 + 4 * n + (i & 3);
    *(u32x4*)(ws + q * kC32WP + kv * 8) = *(const u32x4*)((const _Float16*)a.w + (size_t)co * a.kpad + kv * 8);
  }
  // 1x1 weight fragments (A, registers): N-fragment n row i = reduce channel (i/4)*8 + 4n + i%4,
  // so a lane's two fragments hold reduce channels 8g .. 8g+7 of one pixel
  h8 w1[2][2];
#pragma unroll
  for (int n = 0; n < 2; ++n)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int co = (j >> 2) * 8 + 4 * n + (j & 3);
      w1[n][ks] = *(const h8*)((const _Float16*)a1.w + (size_t)co * a1.kpad + ks * 32 + g * 8);
    }
  const Epilogue& e1 = a1.e;
  const Epilogue& e = a.e;
  float b1[8], bias[16];
#pragma unroll
  for (int q = 0; q < 8; ++q) b1[q] = e1.bias ? e1.bias[8 * g + q] : 0.f;
  const int c0 = 16 * g;
#pragma unroll
  for (int q = 0; q < 16; ++q) bias[q] = e.bias ? e.bias[c0 + q] : 0.f;
  const float slp1 = e1.act == ACT_LEAKY ? e1.slope : 1.f, slp = e.act == ACT_LEAKY ? e.slope : 1.f;

  for (; t < ntiles; t += gridDim.x) {
#pragma unroll
    for (int k = 0; k < kC32rNV; ++k) {
      const int v = tid + k * NT;
      if (v < kC32rXV) *(u32x4*)(xs + (v >> 3) * kC32rPX + (v & 7) * 8) = pre[k];
    }
    __syncthreads();  // X halo (and the 3x3 weights) visible; the previous tile's reads done
    if (t + (int)gridDim.x < ntiles) hload(t + gridDim.x, pre);
    int n, ty, tx;
    tile_of(t, n, ty, tx);
    // ---- 1x1 reduce over the halo pixels -> Y halo ----
    for (int f = wid; f * 16 < kC32rHP; f += NW) {
      const int q = f * 16 + j;  // this lane's halo pixel (B column)
      const int qc = q < kC32rHP ? q : kC32rHP - 1;
      const h8 xa = *(const h8*)(xs + qc * kC32rPX + g * 8);
      const h8 xb = *(const h8*)(xs + qc * kC32rPX + 32 + g * 8);
      f4 acc[2];
#pragma unroll
      for (int nn = 0; nn < 2; ++nn) {
        acc[nn] = __builtin_amdgcn_mfma_f32_16x16x32_f16(w1[nn][0], xa, f4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
        acc[nn] = __builtin_amdgcn_mfma_f32_16x16x32_f16(w1[nn][1], xb, acc[nn], 0, 0, 0);
      }
      const int hr = qc / G::HW, col = qc - hr * G::HW;
      const int y = ty * G::TH - 1 + hr, x = tx * kC32TW - 1 + col;
      const bool inside = (unsigned)y < (unsigned)a.ih && (unsigned)x < (unsigned)a.iw;
      h8v yv;
#pragma unroll
      for (int nn = 0; nn < 2; ++nn)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int qq = 4 * nn + r;  // reduce channel 8g + qq
          float v = acc[nn][r] + b1[qq];
          v = fmaxf(v, v * slp1);
          asm volatile("" : "+v"(v));  // (x * slope rounds to fp32 first, as in the other epilogues)
          v = v * 1.f + 0.f;           // epi_vec8_lean's (absent) BN affine
          yv[qq] = inside ? (_Float16)v : (_Float16)0.f;
        }
      if (q < kC32rHP) *(h8v*)(hs + q * G::PP + 8 * g) = yv;
    }
    __syncthreads();  // Y halo complete
    // ---- 3x3 (conv3_c32<1>) on the Y halo ----
    f4 acc[RW][4];
#pragma unroll
    for (int f = 0; f < RW; ++f)
#pragma unroll
      for (int nn = 0; nn < 4; ++nn) acc[f][nn] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      const int kh = tap / 3, kw = tap % 3;
      h8 wf[4];
#pragma unroll
      for (int nn = 0; nn < 4; ++nn) wf[nn] = *(const h8*)(ws + (nn * 16 + j) * kC32WP + tap * 32 + g * 8);
#pragma unroll
      for (int f = 0; f < RW; ++f) {
        const h8 xf = *(const h8*)(hs + (((wid * RW + f) + kh) * G::HW + j + kw) * G::PP + g * 8);
#pragma unroll
        for (int nn = 0; nn < 4; ++nn) acc[f][nn] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wf[nn], xf, acc[f][nn], 0, 0, 0);
      }
    }
    const int ox = tx * kC32TW + j;
#pragma unroll
    for (int f = 0; f < RW; ++f) {
      const int row = wid * RW + f;
      const int oy = ty * G::TH + row;
      // residual: X at this output pixel = halo pixel (row + 1, j + 1)
      const _Float16* rp = xs + ((row + 1) * G::HW + j + 1) * kC32rPX + c0;
      h8v rv[2];
      rv[0] = *(const h8v*)rp;
      rv[1] = *(const h8v*)(rp + 8);
      if (oy >= a.oh || ox >= a.ow) continue;
      const size_t pix = ((size_t)n * a.oh + oy) * a.ow + ox;
      h8v hv[2];
#pragma unroll
      for (int nn = 0; nn < 4; ++nn)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int q = 4 * nn + r;
          float x = acc[f][nn][r] + bias[q];
          x = fmaxf(x, x * slp);
          asm volatile("" : "+v"(x));
          x = x * 1.f + 0.f;
          x += (float)rv[q >> 3][q & 7];
          hv[q >> 3][q & 7] = (_Float16)x;
        }
      _Float16* op = (_Float16*)e.full.ptr + pix * e.full.cs + e.full.co + c0;
      *(h8v*)op = hv[0];
      *(h8v*)(op + 8) = hv[1];
    }
    __syncthreads();  // X / Y halo reads done before the next tile's stores
  }
}

// conv3_c64r: Darknet-53's 104 x 104 residual blocks (yolov3 / yolov3-spp blocks 2 and 3 at
// 416: the 1x1 reduce 128 -> 64, Darknet.forward models.py:345-347, the 3x3 64 -> 128 and the
// shortcut add :349-354) in one launch.  The 3x3's weights (128 x 576) do not fit in LDS
// beside a halo, so each workgroup owns one half of its output channels (64 x 576 weights
// resident, 74 KB) and the two halves of a tile run on workgroups b and b ^ 8, which sit on
// the same XCD: the second half's reads of the block input X hit that XCD's L2.  Per 16 x 16
// output tile:
//   1. the 1x1 on the 18 x 18 halo pixels inside the image (21 fragments of 16 pixels over the
//      8 waves, 4 k-steps of 32 channels in conv_mfma's order), its B operands straight from
//      X in HBM / L2 (loaded for the next tile under this tile's 3x3), its weights in LDS;
//      bias -> LeakyReLU (rounded to fp32) -> fp16 into the Y halo, zero outside the image;
//   2. the 3x3 on the Y halo, taps 0..8 x two 32-channel k-steps (conv_pipe's K-blocks for
//      Cin 64), bias -> LeakyReLU -> + X at the output pixel -> fp16 (epi_vec8_lean<true>).
// Both halves compute the reduce (1.27 x the 1x1's MACs per half for the halo, +28 % MFMA
// work); the Y map never reaches HBM: per output pixel 256 B of X in, 256 B out, against
// 256 + 128 + 128 + 256 + 256 B for the two launches.  Bit-identical (tests/test_gpu_c32.py).
constexpr int kC64rYP = 80;                     // Y halo pixel pitch (halfs)
constexpr int kC64rWP = 592;                    // 3x3 weight row pitch (halfs: 576 + 16)
constexpr int kC64rW1P = 144;                   // 1x1 weight row pitch (halfs: 128 + 16)
constexpr int kC64rHP = 324;                    // halo pixels (18 x 18)
constexpr int kC64rNF = (kC64rHP + 15) / 16;    // halo fragments (21)
constexpr int kC64rFW = (kC64rNF + 7) / 8;      // fragments per wave (3)
constexpr size_t kC64rLDS = (size_t)(kC64rHP * kC64rYP + 64 * kC64rWP + 64 * kC64rW1P) * 2;

__global__ __launch_bounds__(512) void conv3_c64r(ConvArgs a1, ConvArgs a, int ntiles) {
  extern __shared__ __attribute__((aligned(16))) _Float16 c64r_lds[];
  _Float16* const ys = c64r_lds;                  // Y halo [324][80]
  _Float16* const ws = ys + kC64rHP * kC64rYP;    // this half's 3x3 weights [64][592]
  _Float16* const w1s = ws + 64 * kC64rWP;        // 1x1 weights [64][144]
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int j = lane & 15, g = lane >> 4;
  const int half = (blockIdx.x >> 3) & 1;                         // output channels 64 half ..
  const int pair = (blockIdx.x & 7) | ((blockIdx.x >> 4) << 3);   // b and b ^ 8: one XCD
  const int npairs = gridDim.x >> 1;
  const int tx_n = (a.ow + 15) >> 4, ty_n = (a.oh + 15) >> 4;
  const _Float16* __restrict__ X = (const _Float16*)a1.in + a1.in_co;

  auto tile_of = [&](int t, int& n, int& ty, int& tx) {
    tx = t % tx_n;
    const int t2 = t / tx_n;
    ty = t2 % ty_n;
    n = t2 / ty_n;
  };
  // this lane's X operands of the wave's halo fragments (zero outside the image)
  auto xload = [&](int t, u32x4 (&xr)[kC64rFW][4]) {
    int n, ty, tx;
    tile_of(t, n, ty, tx);
#pragma unroll
    for (int fi = 0; fi < kC64rFW; ++fi) {
      const int q = (wid + 8 * fi) * 16 + j;
      const int hr = q / 18, col = q - hr * 18;
      const int y = ty * 16 - 1 + hr, x = tx * 16 - 1 + col;
      const bool ok = q < kC64rHP && (unsigned)y < (unsigned)a1.ih && (unsigned)x < (unsigned)a1.iw;
      const _Float16* src = X + ((size_t)(n * a1.ih + y) * a1.iw + x) * a1.in_cs + g * 8;
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        xr[fi][ks] = u32x4{0u, 0u, 0u, 0u};
        if (ok) xr[fi][ks] = *(const u32x4*)(src + ks * 32);
      }
    }
  };

  int t = pair;
  u32x4 xr[kC64rFW][4];
  if (t < ntiles) xload(t, xr);
  // 3x3 weights of this half: row q = 16n + i holds output channel 64 half + (i/4)*16 + 4n + i%4
  for (int v = tid; v < 64 * 72; v += 512) {
    const int q = v / 72, kv = v - q * 72;
    const int n = q >> 4, i = q & 15;
    const int co = 64 * half + (i >> 2) * 16 + 4 * n + (i & 3);
    *(u32x4*)(ws + q * kC64rWP + kv * 8) = *(const u32x4*)((const _Float16*)a.w + (size_t)co * a.kpad + kv * 8);
  }
  // 1x1 weights: row q = 16n + i holds reduce channel (i/4)*16 + 4n + i%4
  for (int v = tid; v < 64 * 16; v += 512) {
    const int q = v >> 4, kv = v & 15;
    const int n = q >> 4, i = q & 15;
    const int co = (i >> 2) * 16 + 4 * n + (i & 3);
    *(u32x4*)(w1s + q * kC64rW1P + kv * 8) = *(const u32x4*)((const _Float16*)a1.w + (size_t)co * a1.kpad + kv * 8);
  }
  const Epilogue& e1 = a1.e;
  const Epilogue& e = a.e;
  const int c0 = 64 * half + 16 * g;  // this lane's 16 output channels
  float b1[16], bias[16];
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    b1[q] = e1.bias ? e1.bias[16 * g + q] : 0.f;
    bias[q] = e.bias ? e.bias[c0 + q] : 0.f;
  }
  // LeakyReLU as max(x, slope x) (c64r_ok: 0 < slope <= 1; linear = slope 1): the same value
  // as x > 0 ? x : slope x for every non-NaN x, -0 included, in one compare-free op
  const float slp1 = e1.act == ACT_LEAKY ? e1.slope : 1.f, slp = e.act == ACT_LEAKY ? e.slope : 1.f;
  __syncthreads();  // weights visible

  for (; t < ntiles; t += npairs) {
    int n, ty, tx;
    tile_of(t, n, ty, tx);
    // ---- 1x1 reduce over the halo pixels -> Y halo ----
#pragma unroll
    for (int fi = 0; fi < kC64rFW; ++fi) {
      const int f = wid + 8 * fi;
      if (f >= kC64rNF) break;  // wave-uniform
      f4 acc1[4];
#pragma unroll
      for (int nn = 0; nn < 4; ++nn) acc1[nn] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        const h8 xb = __builtin_bit_cast(h8, xr[fi][ks]);
#pragma unroll
        for (int nn = 0; nn < 4; ++nn) {
          const h8 wa = *(const h8*)(w1s + (nn * 16 + j) * kC64rW1P + ks * 32 + g * 8);
          acc1[nn] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wa, xb, acc1[nn], 0, 0, 0);
        }
      }
      const int q = f * 16 + j;
      const int hr = q / 18, col = q - hr * 18;
      const int y = ty * 16 - 1 + hr, x = tx * 16 - 1 + col;
      const bool inside = (unsigned)y < (unsigned)a1.ih && (unsigned)x < (unsigned)a1.iw;
      h8v yv[2];
#pragma unroll
      for (int nn = 0; nn < 4; ++nn)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int qq = 4 * nn + r;  // reduce channel 16g + qq
          float v = acc1[nn][r] + b1[qq];
          v = fmaxf(v, v * slp1);
          asm volatile("" : "+v"(v));  // (x * slope rounds to fp32 first, as in the other epilogues)
          v = v * 1.f + 0.f;           // epi_vec8_lean's (absent) BN affine
          yv[qq >> 3][qq & 7] = (_Float16)v;
        }
      if (!inside) yv[0] = yv[1] = h8v{};
      if (q < kC64rHP) {
        *(h8v*)(ys + q * kC64rYP + 16 * g) = yv[0];
        *(h8v*)(ys + q * kC64rYP + 16 * g + 8) = yv[1];
      }
    }
    if (t + npairs < ntiles) xload(t + npairs, xr);  // lands under the 3x3
    __syncthreads();  // Y halo complete
    // ---- 3x3 on the Y halo: wave rows 2 wid, 2 wid + 1 ----
    f4 acc[2][4];
#pragma unroll
    for (int f = 0; f < 2; ++f)
#pragma unroll
      for (int nn = 0; nn < 4; ++nn) acc[f][nn] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      const int kh = tap / 3, kw = tap % 3;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        h8 wf[4];
#pragma unroll
        for (int nn = 0; nn < 4; ++nn) wf[nn] = *(const h8*)(ws + (nn * 16 + j) * kC64rWP + tap * 64 + ks * 32 + g * 8);
#pragma unroll
        for (int f = 0; f < 2; ++f) {
          const h8 xf = *(const h8*)(ys + ((2 * wid + f + kh) * 18 + j + kw) * kC64rYP + ks * 32 + g * 8);
#pragma unroll
          for (int nn = 0; nn < 4; ++nn) acc[f][nn] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wf[nn], xf, acc[f][nn], 0, 0, 0);
        }
      }
    }
    const int ox = tx * 16 + j;
#pragma unroll
    for (int f = 0; f < 2; ++f) {
      const int oy = ty * 16 + 2 * wid + f;
      if (oy >= a.oh || ox >= a.ow) continue;
      const size_t pix = ((size_t)n * a.oh + oy) * a.ow + ox;
      const _Float16* rp = (const _Float16*)e.res.ptr + pix * e.res.cs + e.res.co + c0;
      h8v rv[2];
      rv[0] = *(const h8v*)rp;
      rv[1] = *(const h8v*)(rp + 8);
      h8v hv[2];
#pragma unroll
      for (int nn = 0; nn < 4; ++nn)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int q = 4 * nn + r;  // channel c0 + q
          float x = acc[f][nn][r] + bias[q];
          x = fmaxf(x, x * slp);
          asm volatile("" : "+v"(x));
          x = x * 1.f + 0.f;
          x += (float)rv[q >> 3][q & 7];
          hv[q >> 3][q & 7] = (_Float16)x;
        }
      _Float16* op = (_Float16*)e.full.ptr + pix * e.full.cs + e.full.co + c0;
      *(h8v*)op = hv[0];
      *(h8v*)(op + 8) = hv[1];
    }
    __syncthreads();  // Y halo reads done before the next tile's 1x1 stores
  }
}

static bool view8(const View& v) { return ((v.cs | v.co) & 7) == 0; }

bool c32_ok(const ConvArgs& a) {
  if (!tune().conv_c32 || a.in_kind != IN_NHWC || a.w_f32 || a.cin != 32 || a.ks != 3 || a.pad != 1) return false;
  if ((a.stride != 1 && a.stride != 2) || a.quad || a.cout_pad != 64 || a.cout % 16 || a.kpad < 288) return false;
  if ((a.in_cs | a.in_co) & 7 || a.in_cs < a.in_co + 32) return false;
  if (a.oh != (a.ih + 2 - 3) / a.stride + 1 || a.ow != (a.iw + 2 - 3) / a.stride + 1) return false;
  const Epilogue& e = a.e;
  if (!e.full.ptr || e.pool.ptr || e.up.ptr || e.io || e.scale || e.act == ACT_SWISH) return false;
  if (e.act == ACT_LEAKY && !(e.slope > 0.f && e.slope <= 1.f)) return false;  // max(x, slope x)
  if (!view8(e.full) || (e.res.ptr && !view8(e.res))) return false;
  return (int64_t)a.n * a.ih * a.iw * a.in_cs < (1ll << 31) && (int64_t)a.n * a.oh * a.ow * e.full.cs < (1ll << 31);
}

// waves per workgroup: stride 1 4 (70 KB of LDS, two workgroups per CU); stride 2 8, one
// 126 KB workgroup per CU with a 16 x 16 output tile (the 4-wave 8 x 16 tile's 84 KB fits
// only once per CU, leaving one wave per SIMD to hide the halo loads)
constexpr int kC32NW1 = 4, kC32NW2 = 8;

static int c32_tiles(const ConvArgs& a) {
  const int th = a.stride == 1 ? C32Geom<1, kC32NW1>::TH : C32Geom<2, kC32NW2>::TH;
  return a.n * ((a.oh + th - 1) / th) * ((a.ow + kC32TW - 1) / kC32TW);
}

// The residual pair: a1 = the 1x1 reduce (64 -> 32, reading X), a = the 3x3 (32 -> 64) reading
// a1's output with the shortcut X as its residual view.
bool c32r_ok(const ConvArgs& a1, const ConvArgs& a) {
  if (!c32_ok(a) || a.stride != 1 || !a.e.res.ptr || a.cout != 64) return false;
  const Epilogue& e1 = a1.e;
  if (a1.in_kind != IN_NHWC || a1.w_f32 || a1.ks != 1 || a1.stride != 1 || a1.pad != 0 || a1.quad) return false;
  if (a1.cin != 64 || a1.cout != 32 || a1.cout_pad != 32 || a1.kpad < 64 || (a1.in_cs | a1.in_co) & 7) return false;
  if (!e1.full.ptr || e1.pool.ptr || e1.up.ptr || e1.io || e1.res.ptr || e1.scale || e1.act == ACT_SWISH) return false;
  if (e1.act == ACT_LEAKY && !(e1.slope > 0.f && e1.slope <= 1.f)) return false;  // max(x, slope x)
  if (a1.ih != a.ih || a1.iw != a.iw || a1.oh != a.ih || a1.ow != a.iw || a1.n != a.n) return false;
  // a reads a1's output; a's residual is a1's input (same view)
  if (a.in != e1.full.ptr || a.in_cs != e1.full.cs || a.in_co != e1.full.co) return false;
  if (a.e.res.ptr != a1.in || a.e.res.cs != a1.in_cs || a.e.res.co != a1.in_co) return false;
  return (int64_t)a1.n * a1.ih * a1.iw * a1.in_cs < (1ll << 31);
}

void launch_c32r(const ConvArgs& a1, const ConvArgs& a, hipStream_t s) {
  const int nt = c32_tiles(a);
  if (nt <= 0) return;
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1)
    cus = 256;
  const int per_cu = (int)std::max<size_t>(1, (160 * 1024) / kC32rLDS);
  const dim3 grid(std::min(nt, cus * per_cu));
  if (tune().res_fuse == 2)
    hipLaunchKernelGGL(conv3_c32r<4>, grid, dim3(256), kC32rLDS, s, a1, a, nt);
  else
    hipLaunchKernelGGL(conv3_c32r<8>, grid, dim3(512), kC32rLDS, s, a1, a, nt);
  RTDM_HIP(hipGetLastError());
}

// The 104 x 104 residual pair: a1 = the 1x1 reduce (128 -> 64, reading X), a = the 3x3
// (64 -> 128) reading a1's output with X as its residual view.
bool c64r_ok(const ConvArgs& a1, const ConvArgs& a) {
  if (tune().res_fuse != 1) return false;
  if (a.in_kind != IN_NHWC || a.w_f32 || a.cin != 64 || a.cout != 128 || a.cout_pad != 128 || a.ks != 3 ||
      a.stride != 1 || a.pad != 1 || a.quad || a.kpad < 576 || a.oh != a.ih || a.ow != a.iw)
    return false;
  const Epilogue& e = a.e;
  if (!e.full.ptr || !e.res.ptr || e.pool.ptr || e.up.ptr || e.io || e.scale || e.act == ACT_SWISH) return false;
  if (!view8(e.full) || !view8(e.res)) return false;
  const Epilogue& e1 = a1.e;
  for (const Epilogue* ep : {&e, &e1})  // the kernel's max(x, slope x) LeakyReLU
    if (ep->act == ACT_LEAKY && !(ep->slope > 0.f && ep->slope <= 1.f)) return false;
  if (a1.in_kind != IN_NHWC || a1.w_f32 || a1.ks != 1 || a1.stride != 1 || a1.pad != 0 || a1.quad) return false;
  if (a1.cin != 128 || a1.cout != 64 || a1.cout_pad != 64 || a1.kpad < 128 || (a1.in_cs | a1.in_co) & 7) return false;
  if (a1.in_cs < a1.in_co + 128 || e.res.cs < e.res.co + 128 || e.full.cs < e.full.co + 128) return false;
  if (!e1.full.ptr || e1.pool.ptr || e1.up.ptr || e1.io || e1.res.ptr || e1.scale || e1.act == ACT_SWISH) return false;
  if (a1.ih != a.ih || a1.iw != a.iw || a1.oh != a.ih || a1.ow != a.iw || a1.n != a.n) return false;
  if (a.in != e1.full.ptr || a.in_cs != e1.full.cs || a.in_co != e1.full.co) return false;
  if (a.e.res.ptr != a1.in || a.e.res.cs != a1.in_cs || a.e.res.co != a1.in_co) return false;
  return (int64_t)a1.n * a1.ih * a1.iw * a1.in_cs < (1ll << 31) && (int64_t)a.n * a.oh * a.ow * e.full.cs < (1ll << 31);
}

void launch_c64r(const ConvArgs& a1, const ConvArgs& a, hipStream_t s) {
  const int nt = a.n * ((a.oh + 15) / 16) * ((a.ow + 15) / 16);
  if (nt <= 0) return;
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1)
    cus = 256;
  // one workgroup per CU (LDS); a multiple of 16 so that b and b ^ 8 pair every workgroup
  const int grid = 16 * std::max(1, std::min(cus, 2 * nt) / 16);
  hipLaunchKernelGGL(conv3_c64r, dim3(grid), dim3(512), kC64rLDS, s, a1, a, nt);
  RTDM_HIP(hipGetLastError());
}

const char* c32_name(const ConvArgs& a) {
  static const char* names[2][2] = {{"conv3_c32<1,false>", "conv3_c32<1,true>"}, {"conv3_c32<2,false>", "conv3_c32<2,true>"}};
  return names[a.stride == 2][a.e.res.ptr != nullptr];
}

template <int S, bool RES>
static void launch_c32_t(const ConvArgs& a, int ntiles, hipStream_t s) {
  constexpr int NW = S == 1 ? kC32NW1 : kC32NW2;
  using G = C32Geom<S, NW>;
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1)
    cus = 256;
  // workgroups per CU the LDS allows (160 KB per CU)
  const int per_cu = (int)std::max<size_t>(1, (160 * 1024) / G::LDS);
  const int grid = std::min(ntiles, cus * per_cu);
  hipLaunchKernelGGL((conv3_c32<S, RES, NW>), dim3(grid), dim3(G::NT), G::LDS, s, a, ntiles);
  RTDM_HIP(hipGetLastError());
}

void launch_c32(const ConvArgs& a, hipStream_t s) {
  const int nt = c32_tiles(a);
  if (nt <= 0) return;
  const bool res = a.e.res.ptr != nullptr;
  if (a.stride == 1)
    res ? launch_c32_t<1, true>(a, nt, s) : launch_c32_t<1, false>(a, nt, s);
  else
    res ? launch_c32_t<2, true>(a, nt, s) : launch_c32_t<2, false>(a, nt, s);
}

}  // namespace rtdm
