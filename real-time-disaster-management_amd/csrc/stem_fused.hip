// Fused Darknet stem pair: conv 3->16 3x3/s1 + maxpool 2x2  ->  conv 16->32 3x3/s1 + maxpool 2x2
// (yolov4-tiny / yolov3-tiny cfg layers 0-3: victim_localization/yolov3/models.py:23-44 conv +
// BN + LeakyReLU and :64-72 maxpool, as run by Darknet.forward :345-347) in ONE launch.
//
// The unfused pair (conv_stem3<true> then conv3_pool_small<16,32>) writes the 16-channel pooled
// stem map (2x the frame bytes in fp16: 189 MB per b64 batch at 608) and reads it back.  Here a
// workgroup owns an 8 x 8 tile of the SECOND pooled map and builds everything it needs in LDS:
//   input   38 x 40 frame pixels (u8 -> fp16, 4 channels per pixel, zero outside the frame);
//   stem    the 18 x 18 tile of pooled stem outputs its 3x3 conv reads (the 16 x 16 tile + the
//           1-pixel halo; zero outside the map = the conv's padding): 81 MFMA tiles of 4 2x2
//           quads, each 2 x v_mfma_f32_16x16x32_f16 on conv_stem3's K layout, the quad max in
//           lane, the epilogue, one fp16 per lane into conv3_pool_small's LDS tile layout;
//   conv2   conv3_pool_small<16,32,16,4,2>'s K loop and pooled epilogue on that tile.
// Every value is produced by the same operations in the same order as the unfused kernels
// (stem: same K layout, same MFMA pair, max -> fma(x, 1/255, bias) -> max(x, slope x);
// conv2: same K order, same DPP pool), so the output is bit-identical to them.  The halo
// recompute costs 1.27x the stem's MFMAs (36 x 36 stem outputs per 32 x 32).
// Persistent: each workgroup keeps both layers' weights in registers and walks a contiguous
// run of its XCD's tiles, prefetching the next tile's frame pixels into registers during the
// second conv.
#include "common.h"

namespace rtdm {

namespace {
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

constexpr int kSpIR = 38, kSpIC = 40;  // staged frame rows / pixel columns (4-pixel aligned)
constexpr int kSpG4 = kSpIC / 4;       // 4-pixel groups per staged row
constexpr int kSpItems = kSpIR * kSpG4;
constexpr int kSpPV = (kSpItems + 255) / 256;
constexpr int kSpL1 = 18;              // stem tile side (16 + halo)
constexpr int kSpPS = 24;              // stem tile pixel stride (halfs): 16 channels + 8 (bank spread)
constexpr int kSpNQ = 9 * 2;           // 8-channel groups in conv2's K (Cin 16)
constexpr int kSpNKS = (kSpNQ + 3) / 4;

__device__ __forceinline__ uint32_t sp_pack_h2(float a, float b) {
  const _Float16 ha = (_Float16)a, hb = (_Float16)b;
  return (uint32_t)__builtin_bit_cast(uint16_t, ha) | ((uint32_t)__builtin_bit_cast(uint16_t, hb) << 16);
}
__device__ __forceinline__ float sp_dpp_xor1(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0xB1, 0xF, 0xF, 0));
}
}  // namespace

// ABL (diagnostics, wrong outputs): 1 no frame loads, 2 no stem MFMAs, 4 no conv2 MFMAs, 8 no stores
// U: stem MFMA tiles in flight per wave (independent LDS -> MFMA -> epilogue chains; each wave
// has 21 of a tile's 81)
template <int ABL, int U>
__global__ __launch_bounds__(256, 3) void conv_stem_pool2(ConvArgs a0, ConvArgs a2) {
  constexpr int kSpU = U;
  __shared__ __attribute__((aligned(16))) uint2 xin[kSpIR * kSpIC];
  __shared__ __attribute__((aligned(16))) _Float16 l1[kSpL1 * kSpL1 * kSpPS];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int p = lane & 15, g = lane >> 4;
  const int H = a0.ih, W = a0.iw;            // frame
  const int H1 = a0.oh >> 1, W1 = a0.ow >> 1;  // pooled stem map
  const int QH = a2.oh >> 1, QW = a2.ow >> 1;  // pooled conv2 map
  const int tiles_x = QW >> 3, tiles_y = QH >> 3;
  const int ntiles = a0.n * tiles_y * tiles_x;

  // ---- per-lane constants ----
  // stem weights (conv_stem3 layout, B operand: K group g, channel p) and epilogue
  const _Float16* w0p = (const _Float16*)a0.w_stem + (size_t)p * 64 + 8 * g;
  const h8 wa0 = *(const h8*)w0p, wa1 = *(const h8*)(w0p + 32);
  const float bias0 = a0.e.bias ? a0.e.bias[p] : 0.f;
  const float slp0 = a0.e.act == ACT_LEAKY ? a0.e.slope : 1.f;
  constexpr float in_scale = 1.f / 255.f;
  // conv2 weights for the whole K (conv3_pool_small layout, A operand: channel 16t + p, K group)
  h8 wf[kSpNKS][2];
#pragma unroll
  for (int s = 0; s < kSpNKS; ++s)
#pragma unroll
    for (int t = 0; t < 2; ++t) wf[s][t] = *(const h8*)((const _Float16*)a2.w + (size_t)(16 * t + p) * a2.kpad + 8 * (4 * s + g));
  int kofs[kSpNKS];
#pragma unroll
  for (int s = 0; s < kSpNKS; ++s) {
    int q = 4 * s + g;
    q = q < kSpNQ ? q : kSpNQ - 1;
    const int tap = q >> 1, cg = q & 1;
    const int kh = tap / 3, kw = tap - kh * 3;
    kofs[s] = (kh * kSpL1 + kw) * kSpPS + cg * 8;
  }
  float bias2[2][4];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) bias2[t][r] = a2.e.bias ? a2.e.bias[16 * t + 4 * g + r] : 0.f;
  const float slp2 = a2.e.act == ACT_LEAKY ? a2.e.slope : 1.f;

  // ---- frame staging: item i = (row i / 10, 4-pixel group i % 10), 12 bytes ----
  int it_r[kSpPV], it_g[kSpPV];
#pragma unroll
  for (int k = 0; k < kSpPV; ++k) {
    const int i = tid + 256 * k;
    it_r[k] = i < kSpItems ? i / kSpG4 : -(1 << 20);
    it_g[k] = i - (i / kSpG4) * kSpG4;
  }
  uint32_t pre[kSpPV][3];
  auto fetch = [&](int tile) {
    const int tx = tile % tiles_x, t1 = tile / tiles_x;
    const int ty = t1 % tiles_y, n = t1 / tiles_y;
    const uint8_t* img = (const uint8_t*)a0.in + (size_t)n * H * W * 3;
#pragma unroll
    for (int k = 0; k < kSpPV; ++k) {
      const int y = 32 * ty - 3 + it_r[k], x0 = 32 * tx - 4 + 4 * it_g[k];
      pre[k][0] = pre[k][1] = pre[k][2] = 0u;
      if (!(ABL & 1) && (unsigned)y < (unsigned)H && x0 >= 0 && x0 + 4 <= W) {
        const uint32_t* src = (const uint32_t*)(img + ((size_t)y * W + x0) * 3);
        pre[k][0] = src[0];
        pre[k][1] = src[1];
        pre[k][2] = src[2];
      }
    }
  };
  auto stage = [&]() {
#pragma unroll
    for (int k = 0; k < kSpPV; ++k) {
      if (it_r[k] < 0) continue;
      const uint32_t d0 = pre[k][0], d1 = pre[k][1], d2 = pre[k][2];
      const uint32_t b[12] = {d0 & 255u, (d0 >> 8) & 255u, (d0 >> 16) & 255u, d0 >> 24,
                              d1 & 255u, (d1 >> 8) & 255u, (d1 >> 16) & 255u, d1 >> 24,
                              d2 & 255u, (d2 >> 8) & 255u, (d2 >> 16) & 255u, d2 >> 24};
      uint2* dst = xin + it_r[k] * kSpIC + 4 * it_g[k];
#pragma unroll
      for (int q = 0; q < 4; ++q)
        dst[q] = make_uint2(sp_pack_h2((float)b[3 * q], (float)b[3 * q + 1]), sp_pack_h2((float)b[3 * q + 2], 0.f));
    }
  };

  // stem MFMA tile of this lane: A row p = pixel d of quad q (the 4 quads are stem-tile pixels
  // 4 t0 + q in row-major order); per k-step one 2-pixel x 4-channel group (conv_stem3's K layout:
  // G = g: kh = g >> 1, kw pair 2 (g & 1); G = 4 + g: kh = 2, g >= 2 against zero weights)
  const int q = p >> 2, d = p & 3;
  const int kh0 = g >> 1, kwp = 2 * (g & 1);

  int tile, tend, tstep;
  xcd_span(blockIdx.x, gridDim.x, ntiles, tile, tend, tstep);
  if (tile < tend) fetch(tile);
  for (; tile < tend; tile += tstep) {
    const int tx = tile % tiles_x, t1 = tile / tiles_x;
    const int ty = t1 % tiles_y, n = t1 / tiles_y;
    stage();
    __syncthreads();  // frame tile staged; the previous tile's conv2 reads of l1 are done
    // ---- stem + pool -> l1 (fp16): the wave's MFMA tiles t0 = wid + 4 k, kSpU independent
    //      LDS -> MFMA -> epilogue chains at a time (one chain per iteration left the wave
    //      waiting on each chain's LDS and MFMA latency in turn) ----
    constexpr int kTiles = (kSpL1 * kSpL1) / 4, kPerWave = (kTiles + 3) / 4;
#pragma unroll 1
    for (int k0 = 0; k0 < kPerWave; k0 += kSpU) {
      h8 bf0[kSpU], bf1[kSpU];
#pragma unroll
      for (int u = 0; u < kSpU; ++u) {
        int t0 = wid + 4 * (k0 + u);
        t0 = t0 < kTiles ? t0 : kTiles - 1;  // (past the last tile: a valid address, not stored)
        const int li = 4 * t0 + q;
        const int r1 = li / kSpL1, c1 = li - r1 * kSpL1;
        const int i = 2 * r1 + (d >> 1), j = 2 * c1 + (d & 1);  // stem output pixel (tile-local)
        const uint2* b0 = xin + (i + kh0) * kSpIC + j + 1 + kwp;
        const uint2* b1 = xin + (i + 2) * kSpIC + j + 1 + kwp;
        const uint2 x00 = b0[0], x01 = b0[1], x10 = b1[0], x11 = b1[1];
        bf0[u] = __builtin_bit_cast(h8, (u32x4{x00.x, x00.y, x01.x, x01.y}));
        bf1[u] = __builtin_bit_cast(h8, (u32x4{x10.x, x10.y, x11.x, x11.y}));
      }
      f4 acc[kSpU];
#pragma unroll
      for (int u = 0; u < kSpU; ++u) {
        if constexpr ((ABL & 2) != 0) {
          acc[u] = f4{(float)bf0[u][0], (float)bf0[u][1], (float)bf1[u][2], (float)bf1[u][3]};
        } else {
          acc[u] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bf0[u], wa0, f4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
          acc[u] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bf1[u], wa1, acc[u], 0, 0, 0);
        }
      }
#pragma unroll
      for (int u = 0; u < kSpU; ++u) {
        const int t0 = wid + 4 * (k0 + u);
        if (t0 >= kTiles) continue;
        // lane: channel p, quad g = stem-tile pixel 4 t0 + g
        const int lo = 4 * t0 + g;
        const int ro = lo / kSpL1, co = lo - ro * kSpL1;
        const int R = 16 * ty - 1 + ro, C = 16 * tx - 1 + co;  // pooled stem map coordinates
        const float x = fmaf(fmaxf(fmaxf(acc[u][0], acc[u][1]), fmaxf(acc[u][2], acc[u][3])), in_scale, bias0);
        float m = fmaxf(x, x * slp0) + 0.f;
        if ((unsigned)R >= (unsigned)H1 || (unsigned)C >= (unsigned)W1) m = 0.f;  // conv2's zero padding
        l1[lo * kSpPS + p] = (_Float16)m;
      }
    }
    __syncthreads();
    if (tile + tstep < tend) fetch(tile + tstep);  // the next frame tile, in flight during conv2
    // ---- conv2 + pool: wave = 4 rows x 16 columns x 32 channels ----
    const _Float16* xb = l1 + (wid * 4 * kSpL1 + p) * kSpPS;
    f4 acc2[4][2];
#pragma unroll
    for (int jr = 0; jr < 4; ++jr)
#pragma unroll
      for (int t = 0; t < 2; ++t) acc2[jr][t] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < kSpNKS; ++s) {
      const _Float16* bp = xb + kofs[s];
#pragma unroll
      for (int jr = 0; jr < 4; ++jr) {
        const h8 b = *(const h8*)(bp + jr * kSpL1 * kSpPS);
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          if constexpr ((ABL & 4) != 0)
            acc2[jr][t][0] += (float)b[t];
          else
            acc2[jr][t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wf[s][t], b, acc2[jr][t], 0, 0, 0);
        }
      }
    }
    // pooled epilogue (conv3_pool_small's): lane = conv2 column 16 tx + p, rows jr;
    // channels 16 t + 4 g + r
    const int px = (16 * tx + p) >> 1;
    const int py0 = 8 * ty + 2 * wid;
    _Float16* const prow = (_Float16*)a2.e.pool.ptr + a2.e.pool.co + 4 * g + ((size_t)(n * QH + py0) * QW + px) * a2.e.pool.cs;
    const bool lane_st = (p & 1) == 0;
#pragma unroll
    for (int jr = 0; jr < 4; jr += 2) {
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        float m[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float t2 = fmaxf(acc2[jr][t][r], acc2[jr + 1][t][r]);
          const float x = fmaxf(t2, sp_dpp_xor1(t2)) + bias2[t][r];
          m[r] = fmaxf(x, x * slp2);
        }
        if (lane_st && (!(ABL & 8) || m[0] == 12345.f))
          *(uint2*)(prow + (size_t)(jr / 2) * QW * a2.e.pool.cs + 16 * t) =
              make_uint2(sp_pack_h2(m[0], m[1]), sp_pack_h2(m[2], m[3]));
      }
    }
  }
}

// ---- host side ----
// a0: the pooled stem (conv_stem3<true,1> shape: frame u8, Cin 3 -> 16, 3x3 / s1 / p1, LeakyReLU or
// linear, no post-activation affine, pooled output only); a2: conv3_pool_small<16,32>'s layer whose
// input is a0's pooled map.  Both maps tile exactly by 32 frame pixels.
bool stem_pool2_ok(const ConvArgs& a0, const ConvArgs& a2) {
  if (a0.in_kind != IN_FRAME_U8 || !a0.w_stem || a0.cin != 3 || a0.ks != 3 || a0.stride != 1 || a0.pad != 1) return false;
  if (a0.cout != 16 || a0.cout_pad != 16 || !a0.quad || !a0.e.pool.ptr || a0.e.full.ptr || a0.e.up.ptr || a0.e.res.ptr ||
      a0.e.io || a0.e.scale)
    return false;
  if (!(a0.e.act == ACT_LEAKY || a0.e.act == ACT_LINEAR) || (a0.e.act == ACT_LEAKY && !(a0.e.slope > 0.f && a0.e.slope <= 1.f)))
    return false;
  if (a0.ih != a0.oh || a0.iw != a0.ow || a0.ih % 32 != 0 || a0.iw % 32 != 0) return false;
  if ((int64_t)a0.ih * a0.iw * 3 >= (1ll << 31)) return false;
  if (a2.in_kind != IN_NHWC || a2.cin != 16 || a2.cout != 32 || a2.cout_pad != 32 || a2.ks != 3 || a2.stride != 1 ||
      a2.pad != 1 || a2.w_f32 || !a2.quad)
    return false;
  if (a2.ih != a0.oh / 2 || a2.iw != a0.ow / 2 || a2.oh != a2.ih || a2.ow != a2.iw || a2.n != a0.n) return false;
  if (!a2.e.pool.ptr || a2.e.full.ptr || a2.e.up.ptr || a2.e.res.ptr || a2.e.io || a2.e.scale || a2.e.act == ACT_SWISH)
    return false;
  if (a2.e.act == ACT_LEAKY && !(a2.e.slope > 0.f && a2.e.slope <= 1.f)) return false;
  if ((a2.e.pool.cs | a2.e.pool.co) & 3) return false;
  return a2.kpad >= 32 * kSpNKS;  // weights read up to k = 32 * NKS (zero-padded)
}

void launch_stem_pool2(const ConvArgs& a0, const ConvArgs& a2, int abl, hipStream_t s) {
  RTDM_REQUIRE(stem_pool2_ok(a0, a2), RTDM_E_INVALID, "conv_stem_pool2: unsupported layer pair");
  const int64_t tiles = (int64_t)a0.n * (a0.oh / 32) * (a0.ow / 32);
  if (tiles <= 0) return;
  RTDM_REQUIRE(tiles < (1ll << 31), RTDM_E_CAPACITY, "conv_stem_pool2: too many tiles");
  static const int per_cu = [] {
    int nb = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, conv_stem_pool2<0, 7>, 256, 0) != hipSuccess || nb < 1) nb = 1;
    return nb;
  }();
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  const dim3 grid((unsigned)std::min<int64_t>(tiles, (int64_t)per_cu * cus));
  // tune().stem_fuse: 1 = 7 chains per wave (default), 2 = 3, 3 = 1 (A/B diagnostics)
  const int mode = tune().stem_fuse;
  switch (abl) {
    case 1: hipLaunchKernelGGL((conv_stem_pool2<1, 7>), grid, dim3(256), 0, s, a0, a2); break;
    case 2: hipLaunchKernelGGL((conv_stem_pool2<2, 7>), grid, dim3(256), 0, s, a0, a2); break;
    case 4: hipLaunchKernelGGL((conv_stem_pool2<4, 7>), grid, dim3(256), 0, s, a0, a2); break;
    case 8: hipLaunchKernelGGL((conv_stem_pool2<8, 7>), grid, dim3(256), 0, s, a0, a2); break;
    default:
      if (mode == 2)
        hipLaunchKernelGGL((conv_stem_pool2<0, 3>), grid, dim3(256), 0, s, a0, a2);
      else if (mode == 3)
        hipLaunchKernelGGL((conv_stem_pool2<0, 1>), grid, dim3(256), 0, s, a0, a2);
      else
        hipLaunchKernelGGL((conv_stem_pool2<0, 7>), grid, dim3(256), 0, s, a0, a2);
      break;
  }
  RTDM_HIP(hipGetLastError());
}

}  // namespace rtdm
