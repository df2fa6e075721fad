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
#include "conv_epi.h"

#include <type_traits>

#include <algorithm>

namespace rtdm {

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
// EK: epilogue instantiation — 0 generic epi_vec8, 1 epi_vec8_lean, 2 epi_vec8_io
template <int BM, int BN, int BK, int WM, int WN, int EK = 0>
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
  float lb[8], ls[8], lh[8];
  if constexpr (EK == 1) {
    static_assert(NT % CG == 0, "channel group per thread");
    const int c0 = n_base + (tid % CG) * 8;
    const bool cv = c0 < a.cout;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      lb[j] = cv ? a.e.bias[c0 + j] : 0.f;
      ls[j] = cv && a.e.scale ? a.e.scale[c0 + j] : 1.f;
      lh[j] = cv && a.e.scale ? a.e.shift[c0 + j] : 0.f;
    }
  }
  for (int u = tid; u < UNITS; u += NT) {
    const int q = u / CG, g = u - (u / CG) * CG;
    const int m0 = m_base + q * 4, c0 = n_base + g * 8;
    if (m0 >= a.M || c0 >= a.cout) continue;
    float v[4][8];
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int j = 0; j < 8; ++j) v[r][j] = Cs[(q * 4 + r) * CSTR + g * 8 + j];
    if constexpr (EK == 1)
      epi_vec8_lean(a, m0, c0, v, lb, ls, lh);
    else if constexpr (EK == 2)
      epi_vec8_io(a, m0, c0, v);
    else
      epi_vec8(a, m0, c0, v);
  }
}

// --------------------------------------------------------------------------
// fp16 MFMA stem: Cin = 3, 3x3, stride 1|2, pad 0|1 — the Darknet first conv
// (uint8 frames or NCHW model inputs, detect.py:80-82 /255 applied to the fp32
// accumulator) and the ACFF classifiers' conv1 (squeeze_ernet.py:11, ernet.py:10;
// fp16 NHWC output of the fused CLI transform or NCHW model inputs).
//
// Output-channel-major GEMM, D[cout][pixel] = W[cout][k] x X[k][pixel], on
// v_mfma_f32_16x16x32_f16: the weight fragments (A) are loaded once per block
// and stay in registers; each lane's B fragment is 8 contiguous fp16 of the LDS
// input image, so one MFMA tile costs 2 x (2 ds_read_b64) per lane.
//   LDS image: the block's input rows, every pixel padded to 4 channels
//              (c0,c1,c2,0) = 8 bytes, zero columns/rows for the padding.
//   K (64 = 2 MFMA k-steps): group G = 0..5 -> (kh = G>>1, pixel pair
//              kw in {0,1} | {2,3}), 8 values = 2 pixels x 4 channels; G = 6,7
//              are zero.  Weights for kw = 3 and c = 3 are zero.
//   D layout:  lane = pixel (lane & 15), 4 consecutive channels per lane
//              ((lane >> 4) * 4 + j) -> 8-byte NHWC stores; in quad order the
//              16 pixels are 4 2x2 quads on lane groups of 4, so the fused 2x2
//              maxpool is two DPP quad_perm max steps.
// One block = kStemRows output rows of one image, 4 waves stride over the
// 16-pixel tiles of those rows.
// --------------------------------------------------------------------------
constexpr int kStemRows = 4;      // output rows per block, plain stem
constexpr int kStemRowsPool = 4;  // output rows per block, pooled stem (2 waves per quad row; 8 measured slower)
__host__ __device__ constexpr int stem_rows(bool pool) { return pool ? kStemRowsPool : kStemRows; }
// LDS columns past the staged row that the pooled loop's last two tiles may read: quad
// x <= qw + 10 -> column <= (ow + 21) * s + 4, i.e. 22 * s + pad past the staged columns
__host__ __device__ constexpr int stem_xcols(bool pool, int s) { return pool ? 22 * s + 2 : 0; }

// two byte values as an fp16 pair: one v_cvt_pkrtz (0..255 are exact in fp16, so the
// round-toward-zero conversion gives pack_h2's bits)
__device__ __forceinline__ uint32_t pack_u8x2(uint32_t a, uint32_t b) {
  return __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_pkrtz((float)a, (float)b));
}

__device__ __forceinline__ uint32_t pack_h2(float a, float b) {
  const _Float16 ha = (_Float16)a, hb = (_Float16)b;
  return (uint32_t)__builtin_bit_cast(uint16_t, ha) | ((uint32_t)__builtin_bit_cast(uint16_t, hb) << 16);
}

// The kh = 2 third of K on one 16-deep MFMA (K16, the default): lane group g supplies the
// pixel at kw = g (4 channels; kw = 3 meets zero weights), so K = 32 + 16 instead of 32 + 32
// with lane groups 2, 3 re-reading kh = 2 pixels against zero weights — the same nonzero
// products, bit-identical (tests/test_gpu_stem.py).  The 16-deep link reads the 32-deep
// link's accumulator as SrcC; mfma_opcode_switch() keeps the two opcodes apart (see there).
// ABL (diagnostic builds only, outputs wrong when non-zero): 1 = no frame loads,
// 2 = no output stores, 4 = no MFMA.
template <bool POOL, int NTN, bool K16, int ABL = 0>
__global__ __launch_bounds__(256, 5) void conv_stem3(ConvArgs a) {  // 5: the LDS bound (<= 31 KB per block at 608); lets the compiler keep the fragment reads in flight
  extern __shared__ __attribute__((aligned(16))) uint2 stem_lds[];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int s = a.stride, pad = a.pad;
  constexpr int ROWS = stem_rows(POOL);
  const int bpi = (a.oh + ROWS - 1) / ROWS;
  const int bl = xcd_block(blockIdx.x, gridDim.x);  // consecutive bands (shared halo rows) on one XCD
  const int n = bl / bpi;
  const int oy0 = (bl - n * bpi) * ROWS;
  const int nrows = (ROWS - 1) * s + 3;
  const int cols = (a.ow - 1) * s - pad + 5;  // LDS column = x + 1, x in [-1, (ow-1)*s - pad + 3]
  const int ls = cols + stem_xcols(POOL, s);   // LDS row stride (overrun columns: never staged)
  const int iy0 = oy0 * s - pad;
  const int H = a.ih, W = a.iw;

  // ---- stage the input rows iy0 .. iy0+nrows-1 (fp16, 4 channels / pixel) ----
  if (a.in_kind == IN_FRAME_U8 && (W & 3) == 0 && cols >= W + 1) {
    const int gpr = W >> 2;  // 4-pixel groups per row (12 bytes)
    // (row, group) items flattened over all 256 threads (a per-row loop left 256 - gpr
    // threads idle every row: 104 of 256 at 608 columns), four items per thread per pass
    // with all their loads issued before the first conversion (one load latency per pass,
    // not per item)
    int r = tid / gpr, g = tid - r * gpr;
    while (r < nrows) {
      uint32_t d[4][3];
      int rk[4], gk[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        rk[k] = r;
        gk[k] = g;
        d[k][0] = d[k][1] = d[k][2] = 0u;
        const int y = iy0 + r;
        if (r < nrows && (unsigned)y < (unsigned)H && !(ABL & 1)) {
          const uint32_t* src = (const uint32_t*)((const uint8_t*)a.in + ((size_t)(n * H + y) * W + 4 * g) * 3);
          d[k][0] = src[0];
          d[k][1] = src[1];
          d[k][2] = src[2];
        }
        g += 256;
        while (g >= gpr) {
          g -= gpr;
          ++r;
        }
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        if (rk[k] >= nrows) break;
        const uint32_t d0 = d[k][0], d1 = d[k][1], d2 = d[k][2];
        const uint32_t b[12] = {d0 & 255u, (d0 >> 8) & 255u, (d0 >> 16) & 255u, d0 >> 24,
                                d1 & 255u, (d1 >> 8) & 255u, (d1 >> 16) & 255u, d1 >> 24,
                                d2 & 255u, (d2 >> 8) & 255u, (d2 >> 16) & 255u, d2 >> 24};
        uint2* dst = stem_lds + rk[k] * ls + 4 * gk[k] + 1;
#pragma unroll
        for (int p = 0; p < 4; ++p)
          dst[p] = make_uint2(pack_u8x2(b[3 * p], b[3 * p + 1]), pack_u8x2(b[3 * p + 2], 0u));
      }
    }
    const int npad = cols - W;  // LDS column 0 and columns W+1 .. cols-1 are padding
    for (int idx = tid; idx < nrows * npad; idx += 256) {
      const int r = idx / npad, k = idx - r * npad;
      stem_lds[r * ls + (k == 0 ? 0 : W + k)] = make_uint2(0u, 0u);
    }
  } else {
    for (int idx = tid; idx < nrows * cols; idx += 256) {
      const int r = idx / cols, lc = idx - r * cols;
      const int y = iy0 + r, x = lc - 1;
      float v[3] = {0.f, 0.f, 0.f};
      if ((unsigned)y < (unsigned)H && (unsigned)x < (unsigned)W) {
#pragma unroll
        for (int c = 0; c < 3; ++c) {
          if (a.in_kind == IN_FRAME_U8)
            v[c] = (float)((const uint8_t*)a.in)[((size_t)(n * H + y) * W + x) * 3 + c];
          else if (a.in_kind == IN_NCHW_F32)
            v[c] = ((const float*)a.in)[(((size_t)n * 3 + c) * H + y) * W + x];
          else if (a.in_kind == IN_NCHW_F16)
            v[c] = (float)((const _Float16*)a.in)[(((size_t)n * 3 + c) * H + y) * W + x];
          else
            v[c] = (float)((const _Float16*)a.in)[((size_t)(n * H + y) * W + x) * a.in_cs + a.in_co + c];
        }
      }
      stem_lds[r * ls + lc] = make_uint2(pack_h2(v[0], v[1]), pack_h2(v[2], 0.f));
    }
  }

  // ---- per-lane constants: weight fragments and epilogue vectors ----
  // POOL (pixel-major, D[pixel][cout]): lane = channel (lane & 15), 4 pixels per
  //   lane = one 2x2 quad -> the maxpool is in-lane; 2-byte stores.
  // !POOL (channel-major, D[cout][pixel]): lane = pixel, 4 channels per lane ->
  //   8-byte stores.
  const int p = lane & 15, g = lane >> 4;
  const Epilogue& e = a.e;
  h8 wa[NTN][2];
  constexpr int NE = POOL ? 1 : 4;  // epilogue channels per lane per cout tile
  float bias[NTN][NE], sc[NTN][NE], sh[NTN][NE];
#pragma unroll
  for (int t = 0; t < NTN; ++t) {
    const _Float16* wp = (const _Float16*)a.w_stem + (size_t)(16 * t + p) * 64 + 8 * g;
    wa[t][0] = *(const h8*)wp;
    wa[t][1] = *(const h8*)(wp + 32);
#pragma unroll
    for (int j = 0; j < NE; ++j) {
      const int c = POOL ? 16 * t + p : 16 * t + 4 * g + j;
      const bool cv = c < a.cout;
      bias[t][j] = (e.bias && cv) ? e.bias[c] : 0.f;
      sc[t][j] = (e.scale && cv) ? e.scale[c] : 1.f;
      sh[t][j] = (e.scale && cv) ? e.shift[c] : 0.f;
    }
  }
  const float in_scale = a.in_kind == IN_FRAME_U8 ? 1.f / 255.f : 1.f;
  const int act = e.act;
  const float slope = e.slope;
  __syncthreads();

  auto epi = [&](float x, int t, int j) {
    x = x * in_scale + bias[t][j];
    if (act == ACT_LEAKY)
      x = x > 0.f ? x : x * slope;
    else if (act == ACT_SWISH)
      x = x * sigmoidf_(x);
    return x * sc[t][j] + sh[t][j];
  };
  const int kh0 = g >> 1, pr0 = g & 1;
  typedef _Float16 h4s __attribute__((ext_vector_type(4)));
  h4s w16[NTN];
#pragma unroll
  for (int t = 0; t < NTN; ++t) w16[t] = *(const h4s*)((const _Float16*)a.w_stem + (size_t)(16 * t + p) * 64 + 32 + 4 * g);
  if (POOL) {
    // waves 0,1 -> quad row 0, waves 2,3 -> quad row 1 (ROWS == 4); a wave's
    // tiles are 4 consecutive quads, striding by 2 tiles.
    static_assert(!POOL || ROWS == 4, "two waves per quad row");
    const int qw = a.ow >> 1, qh = a.oh >> 1;
    const int tr = __builtin_amdgcn_readfirstlane(wid >> 1);  // wave-uniform: the pooled row's buffer base in SGPRs
    const int py = (oy0 >> 1) + tr;
    if (py >= qh) return;
    const int d = p & 3;
    const int ly = 2 * tr + (d >> 1);  // LDS row of kh = 0 (stride 1 / 2 scaled below)
    // lane's LDS reads for the wave's first tile (tx = wid & 1); a tile step of 2 is 16*s
    // columns and the loop step of 4 tiles 32*s.  Pixels past the row (qx >= qw) read the
    // overrun columns and are never stored.  The second K half's lanes g >= 2 (G = 6, 7)
    // read kh = 2 pixels again, against zero weights (pack_stem): finite x 0, no masking.
    const int lx0 = (2 * ((wid & 1) * 4 + (p >> 2)) + (d & 1)) * s - pad + 1;
    const uint2* rk0 = stem_lds + (ly * s + kh0) * ls + lx0 + 2 * pr0;
    const uint2* rk2 = stem_lds + (ly * s + 2) * ls + lx0 + 2 * (g & 1);
    const uint2* rk2s = stem_lds + (ly * s + 2) * ls + lx0 + g;
    _Float16* pool_row = (_Float16*)e.pool.ptr + ((size_t)n * qh + py) * qw * e.pool.cs + e.pool.co;
    // the pooled row as a buffer (wave-uniform base, 32-bit lane offsets); a lane with no
    // output stores at an offset past the row's records, which the buffer unit drops
    const __amdgpu_buffer_rsrc_t rs_pool =
        __builtin_amdgcn_make_buffer_rsrc((void*)pool_row, 0, qw * e.pool.cs * 2, 0x00020000);
    // Darknet stem (no BN affine after the fold, LeakyReLU / linear): LeakyReLU as
    // max(x, slope x) (0 < slope < 1; 1 = linear), no per-value branches
    const bool lean = !e.scale && act != ACT_SWISH && (act != ACT_LEAKY || (slope > 0.f && slope <= 1.f));
    const float slp = act == ACT_LEAKY ? slope : 1.f;
    // two 4-quad tiles per iteration (tx, tx + 2): two independent LDS -> MFMA -> epilogue
    // chains per wave instead of one latency-bound chain; the loop is unswitched on `lean`
    // the pixel pair as two ds_read_b64 (2 LDS cycles each, 64 banks) rather than the one
    // ds_read2_b64 the compiler would merge them into (8 cycles, 32 banks: 55 % of the LDS
    // cycles were conflicts): an offset it cannot see keeps them apart
    int one = 1;
    asm volatile("" : "+v"(one));
    auto run = [&](auto lean_c) {
    constexpr bool LEAN = decltype(lean_c)::value;
    for (int tx0 = wid & 1, off = 0; tx0 * 4 < qw; tx0 += 4, off += 32 * s) {
      h8 bf0[2], bf1[2];
      h4s bk[2];
      int oq[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int tx = tx0 + 2 * u, o = off + u * 16 * s;
        const uint2 b00 = rk0[o], b01 = rk0[o + one];
        bf0[u] = __builtin_bit_cast(h8, (u32x4{b00.x, b00.y, b01.x, b01.y}));
        if constexpr (K16) {
          bk[u] = __builtin_bit_cast(h4s, rk2s[o]);
        } else {
          const uint2 b10 = rk2[o], b11 = rk2[o + 1];
          bf1[u] = __builtin_bit_cast(h8, (u32x4{b10.x, b10.y, b11.x, b11.y}));
        }
        oq[u] = tx * 4 + g;  // pooled x of this lane's output quad
      }
      f4 accs[NTN][2];
      if constexpr ((ABL & 4) != 0) {
#pragma unroll
        for (int t = 0; t < NTN; ++t)
#pragma unroll
          for (int u = 0; u < 2; ++u)
            accs[t][u] = K16 ? f4{(float)bf0[u][0], (float)bf0[u][1], (float)bk[u][2], (float)bk[u][3]}
                             : f4{(float)bf0[u][0], (float)bf0[u][1], (float)bf1[u][2], (float)bf1[u][3]};
      } else {
        // every chain's 32-deep link, then (K16) the fence, then every 16-deep link
#pragma unroll
        for (int t = 0; t < NTN; ++t)
#pragma unroll
          for (int u = 0; u < 2; ++u)
            accs[t][u] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bf0[u], wa[t][0], f4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
        if constexpr (K16) mfma_opcode_switch();
#pragma unroll
        for (int t = 0; t < NTN; ++t)
#pragma unroll
          for (int u = 0; u < 2; ++u) {
            if constexpr (K16)
              accs[t][u] = __builtin_amdgcn_mfma_f32_16x16x16f16(bk[u], w16[t], accs[t][u], 0, 0, 0);
            else
              accs[t][u] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bf1[u], wa[t][1], accs[t][u], 0, 0, 0);
          }
      }
#pragma unroll
      for (int t = 0; t < NTN; ++t) {
        const f4* acc = accs[t];
        const int c = 16 * t + p;
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          // bias, LeakyReLU/linear and the positive 1/255 scale are monotone non-decreasing
          // (and so is their fp32 rounding): pool first, then one epilogue per quad
          float m;
          if constexpr (LEAN) {
            const float x = fmaxf(fmaxf(acc[u][0], acc[u][1]), fmaxf(acc[u][2], acc[u][3])) * in_scale + bias[t][0];
            m = fmaxf(x, x * slp) + 0.f;  // + 0: epi's "* 1 + 0" affine (-0 -> +0), bit-identical
          } else {
            m = e.scale || act == ACT_SWISH
                    ? fmaxf(fmaxf(epi(acc[u][0], t, 0), epi(acc[u][1], t, 0)), fmaxf(epi(acc[u][2], t, 0), epi(acc[u][3], t, 0)))
                    : epi(fmaxf(fmaxf(acc[u][0], acc[u][1]), fmaxf(acc[u][2], acc[u][3])), t, 0);
          }
          if (!(ABL & 2) || m == 12345.f) {
            const int po = oq[u] < qw && c < a.cout ? (oq[u] * e.pool.cs + c) * 2 : 0x7FFFFFF0;
            __builtin_amdgcn_raw_buffer_store_b16(__builtin_bit_cast(unsigned short, (_Float16)m), rs_pool, po, 0, 0);
          }
        }
      }
    }
    };
    if (lean)
      run(std::true_type{});
    else
      run(std::false_type{});
  } else {
    const int tiles_x = (a.ow + 15) >> 4;
    const int ntiles = tiles_x * ROWS;
    for (int t = wid; t < ntiles; t += 4) {
      const int tr = t / tiles_x, tx = t - tr * tiles_x;
      const int oy = oy0 + tr;
      if (oy >= a.oh) break;
      const int ox = tx * 16 + p;
      const bool valid = ox < a.ow;
      const int lx = (valid ? ox : a.ow - 1) * s - pad + 1;
      const uint2* rowk0 = stem_lds + (tr * s + kh0) * ls;
      const uint2* rowk2 = stem_lds + (tr * s + 2) * ls;
      int one = 1;  // (two ds_read_b64, not a ds_read2_b64: see the pooled path)
      asm volatile("" : "+v"(one));
      const uint2 b00 = rowk0[lx + 2 * pr0], b01 = rowk0[lx + 2 * pr0 + one];
      const h8 bf0 = __builtin_bit_cast(h8, (u32x4{b00.x, b00.y, b01.x, b01.y}));
      h8 bf1;
      h4s bk;
      if constexpr (K16) {
        bk = __builtin_bit_cast(h4s, rowk2[lx + g]);  // kw = g (kw = 3: zero weights, staged pixel)
      } else {
        uint2 b10 = rowk2[lx + 2 * (g & 1)], b11 = rowk2[lx + 2 * (g & 1) + 1];
        if (g >= 2) b10 = b11 = make_uint2(0u, 0u);
        bf1 = __builtin_bit_cast(h8, (u32x4{b10.x, b10.y, b11.x, b11.y}));
      }
      const size_t pix = ((size_t)n * a.oh + oy) * a.ow + ox;
      f4 accs[NTN];
#pragma unroll
      for (int tt = 0; tt < NTN; ++tt)
        accs[tt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wa[tt][0], bf0, f4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
      if constexpr (K16) mfma_opcode_switch();
#pragma unroll
      for (int tt = 0; tt < NTN; ++tt) {
        if constexpr (K16)
          accs[tt] = __builtin_amdgcn_mfma_f32_16x16x16f16(w16[tt], bk, accs[tt], 0, 0, 0);
        else
          accs[tt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wa[tt][1], bf1, accs[tt], 0, 0, 0);
      }
#pragma unroll
      for (int tt = 0; tt < NTN; ++tt) {
        const f4 acc = accs[tt];
        float v[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = epi(acc[j], tt, j);
        const int c0 = 16 * tt + 4 * g;
        if (valid && e.full.ptr) {
          _Float16* fp = (_Float16*)e.full.ptr + pix * e.full.cs + e.full.co + c0;
          if (c0 + 4 <= a.cout) {
            *(uint2*)fp = make_uint2(pack_h2(v[0], v[1]), pack_h2(v[2], v[3]));
          } else {
#pragma unroll
            for (int j = 0; j < 4; ++j)
              if (c0 + j < a.cout) fp[j] = (_Float16)v[j];
          }
        }
      }
    }
  }
}

static size_t stem3_lds_bytes(const ConvArgs& a) {
  const int nrows = (stem_rows(a.quad != 0) - 1) * a.stride + 3;
  const int cols = (a.ow - 1) * a.stride - a.pad + 5 + stem_xcols(a.quad != 0, a.stride);
  return (size_t)nrows * cols * sizeof(uint2);
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
// fp16 implicit GEMM with direct global->LDS staging (global_load_lds_dwordx4).
// 128 x 128 block tile, BK = 64, 4 waves (2 x 2, 64 x 64 each), two LDS
// buffers: the loads of K-block kb+1 are issued before the MFMAs of kb and
// retired by the one __syncthreads() (vmcnt(0) + barrier) per K-block.
// glds writes each wave-instruction's 64 x 16 bytes lane-linearly (8 rows of
// 128 B), so the bank-conflict swizzle lives in the per-lane SOURCE address:
// LDS slot s of row r holds k-vector s ^ ((r >> 1) & 7), and a fragment read
// of k-vector v in row r reads slot v ^ ((r >> 1) & 7) — the 16 rows a
// ds_read_b128 lane group touches then cover all 64 banks.  Out-of-image taps,
// K padding and rows past M read a 16-byte zero block (a.zero) instead.
// --------------------------------------------------------------------------

template <int BM, int NS>
__global__ __launch_bounds__(BM * 2, (BM == 128 && NS == 2) ? 2 : 1) void conv_glds_f16(ConvArgs a) {
  constexpr int BN = 128, BK = 64;
  constexpr int WAVES = BM / 32;         // 4 (128 x 128 tile) or 8 (256 x 128 tile)
  constexpr int NT = 64 * WAVES;
  constexpr int NB = BN / (8 * WAVES);   // B-tile wave-instructions per wave per stage
  constexpr int VM = 4 + NB;             // vm ops per wave per stage (exact, for counted vmcnt)
  constexpr int BUF = (BM + BN) * BK;    // halfs per stage buffer
  constexpr int CSTR = BN + 4;
  constexpr int SMEM = (NS * BUF * 2 > BM * CSTR * 4) ? NS * BUF * 2 : BM * CSTR * 4;
  __shared__ __attribute__((aligned(16))) unsigned char smem_raw[SMEM];
  _Float16* smem = reinterpret_cast<_Float16*>(smem_raw);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);  // provably wave-uniform (scalar LDS addresses)
  const int wm = wid >> 1, wn = wid & 1;
  const int nblk = gridDim.x;
  const int ntn = a.cout_pad / BN;
  int bid = blockIdx.x;
  {
    const int xcd = bid & 7, q = nblk >> 3, r = nblk & 7;
    bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  }
  const int m_base = (bid / ntn) * BM;
  const int n_base = (bid - (bid / ntn) * ntn) * BN;

  // ---- staging rows: A instr j covers rows 32*wid + 8*j + lane/8, B instr j rows
  //      (8*NB)*wid + 8*j + lane/8; slot lane%8 holds k-vector slot ^ ((row >> 1) & 7) ----
  const int slot = lane & 7;
  const _Float16* __restrict__ in = (const _Float16*)a.in + a.in_co;
  const _Float16* __restrict__ zero = (const _Float16*)a.zero;
  int a_pix[4], a_iy[4], a_ix[4], kofs[4];
  int voff_a[4];
  uint32_t vmask[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int r = 32 * wid + 8 * j + (lane >> 3);
    kofs[j] = 8 * (slot ^ ((r >> 1) & 7));
    const int m = m_base + r;
    int n = 0, oy = 0, ox = 0;
    if (m < a.M) row_to_pix(a, m, n, oy, ox);
    a_pix[j] = n * a.ih * a.iw;
    a_iy[j] = m < a.M ? oy * a.stride - a.pad : -(1 << 28);
    a_ix[j] = ox * a.stride - a.pad;
    voff_a[j] = m < a.M ? ((a_pix[j] + a_iy[j] * a.iw + a_ix[j]) * a.in_cs + kofs[j]) * 2 : 0;
    uint32_t msk = 0;
    for (int t = 0; t < a.ks * a.ks; ++t) {
      const int kh = a.ks == 3 ? (t * 11) >> 5 : 0, kw = t - kh * a.ks;
      const int iy = a_iy[j] + kh, ix = a_ix[j] + kw;
      if ((unsigned)iy < (unsigned)a.ih && (unsigned)ix < (unsigned)a.iw) msk |= 1u << t;
    }
    vmask[j] = msk;
  }
  int kofs_b[NB], voff_b[NB];
  const _Float16* b_src[NB];
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    const int r = 8 * NB * wid + 8 * j + (lane >> 3);
    kofs_b[j] = 8 * (slot ^ ((r >> 1) & 7));
    voff_b[j] = (r * a.kpad + kofs_b[j]) * 2;
    b_src[j] = (const _Float16*)a.w + (size_t)(n_base + r) * a.kpad + kofs_b[j];
  }
  const int K = a.ks * a.ks * a.cin;
  const int nk = a.kpad / BK;
  const FastDiv fd_cin = a.fd_cin;
  // Uniform path (Cin % 64 == 0, tensor < 2^30 elements): a K-block never straddles a
  // tap, so the tap and channel block are wave-uniform scalars advanced once per
  // K-block.  Loads are buffer_load ... lds through one descriptor per operand: per
  // row a 32-bit byte offset and a 9-bit tap-validity mask fixed at the start; an
  // invalid tap / row gets an offset past num_records, which the buffer unit returns
  // as zeros (the convolution's zero padding).  B offsets are fixed per lane, the
  // K-block advance rides in soffset.
  const bool uni = a.glds_uni;
  __amdgpu_buffer_rsrc_t rs_in, rs_w;
  if (uni) {
    const int64_t in_bytes = ((int64_t)a.n * a.ih * a.iw * a.in_cs - a.in_co) * 2;
    rs_in = __builtin_amdgcn_make_buffer_rsrc((void*)in, 0, (int)in_bytes, 0x00020000);
    rs_w = __builtin_amdgcn_make_buffer_rsrc((void*)((const _Float16*)a.w + (size_t)n_base * a.kpad), 0,
                                             BN * a.kpad * 2, 0x00020000);
  }
  const int cpt = a.cin / BK;  // K-blocks per tap (uniform path)
  int st_tap = 0, st_c = 0;     // uniform-path cursor: the next K-block to stage

  auto stage = [&](int buf, int kb) {
    _Float16* As = smem + buf * BUF;
    _Float16* Bs = As + BM * BK;
    if (uni) {
      const int kh = a.ks == 3 ? (st_tap * 11) >> 5 : 0, kw = st_tap - kh * a.ks;
      const int tapoff = ((kh * a.iw + kw) * a.in_cs + st_c * BK) * 2;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int vo = ((vmask[j] >> st_tap) & 1u) ? voff_a[j] + tapoff : (int)0x80000000;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs_in, (lds_ptr_t)(As + (32 * wid + 8 * j) * BK), 16, vo, 0, 0, 0);
      }
      const int soff = kb * BK * 2;
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        _Float16* bdst = Bs + (8 * NB * wid + 8 * j) * BK;
        const int vob = voff_b[j];
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs_w, (lds_ptr_t)bdst, 16, vob, soff, 0, 0);
      }
      if (++st_c == cpt) {
        st_c = 0;
        ++st_tap;
      }
      return;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int kg = kb * BK + kofs[j];
      const int tap = fdiv(kg, fd_cin);
      const int c = kg - tap * a.cin;
      const int kh = a.ks == 3 ? (tap * 11) >> 5 : 0;
      const int kw = tap - kh * a.ks;
      const int iy = a_iy[j] + kh, ix = a_ix[j] + kw;
      const bool v = kg < K && (unsigned)iy < (unsigned)a.ih && (unsigned)ix < (unsigned)a.iw;
      const _Float16* src = v ? in + (size_t)(a_pix[j] + iy * a.iw + ix) * a.in_cs + c : zero;
      __builtin_amdgcn_global_load_lds((gbl_ptr_t)src, (lds_ptr_t)(As + (32 * wid + 8 * j) * BK), 16, 0, 0);
    }
#pragma unroll
    for (int j = 0; j < NB; ++j)
      __builtin_amdgcn_global_load_lds((gbl_ptr_t)(b_src[j] + kb * BK), (lds_ptr_t)(Bs + (8 * NB * wid + 8 * j) * BK),
                                       16, 0, 0);
  };

  f4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};

  const int fr = lane & 15, g = lane >> 4;
  const int rsw = (fr >> 1) & 7;  // swizzle key of this lane's fragment rows
  const int s0 = 8 * ((0 + g) ^ rsw), s1 = 8 * ((4 + g) ^ rsw);

  // NS = 2: loads of kb+1 in flight during kb, retired by __syncthreads (vmcnt(0)).
  // NS = 3: loads of kb+1 and kb+2 in flight; every stage is exactly VM buffer/global
  // LDS-DMA ops per wave, so "s_waitcnt vmcnt(VM)" + raw s_barrier retires stage kb+1
  // while kb+2 stays in flight across the barrier (no other vector-memory ops in the loop).
  stage(0, 0);
  if (NS == 3 && nk > 1) {
    stage(1, 1);
    if (VM == 8)
      asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else
      asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  } else {
    __syncthreads();
  }
  for (int kb = 0; kb < nk; ++kb) {
    const int cur = NS == 2 ? (kb & 1) : kb % 3;
    if (NS == 2) {
      if (kb + 1 < nk) stage(cur ^ 1, kb + 1);
    } else {
      if (kb + 2 < nk) stage(cur == 0 ? 2 : cur - 1, kb + 2);
    }
    const _Float16* As = smem + cur * BUF + (wm * 64 + fr) * BK;
    const _Float16* Bs = smem + cur * BUF + BM * BK + (wn * 64 + fr) * BK;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int so = kk ? s1 : s0;
      h8 af[4], bf[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) af[t] = *(const h8*)(As + t * 16 * BK + so);
#pragma unroll
      for (int t = 0; t < 4; ++t) bf[t] = *(const h8*)(Bs + t * 16 * BK + so);
#pragma unroll
      for (int tm = 0; tm < 4; ++tm)
#pragma unroll
        for (int tn = 0; tn < 4; ++tn)
          acc[tm][tn] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[tm], bf[tn], acc[tm][tn], 0, 0, 0);
    }
    if (NS == 2) {
      __syncthreads();
    } else {
      if (kb + 2 < nk) {
        if (VM == 8)
          asm volatile("s_waitcnt vmcnt(8) lgkmcnt(0)" ::: "memory");
        else
          asm volatile("s_waitcnt vmcnt(6) lgkmcnt(0)" ::: "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      }
      __builtin_amdgcn_s_barrier();
    }
  }
  if (NS == 3) __syncthreads();

  // ---- epilogue: accumulators -> LDS C tile -> 4 rows x 8 channels per thread ----
  float* Cs = reinterpret_cast<float*>(smem_raw);
  const int rq = g * 4;
#pragma unroll
  for (int tm = 0; tm < 4; ++tm)
#pragma unroll
    for (int tn = 0; tn < 4; ++tn) {
      const int row = wm * 64 + tm * 16 + rq;
      const int col = wn * 64 + tn * 16 + fr;
#pragma unroll
      for (int j = 0; j < 4; ++j) Cs[(row + j) * CSTR + col] = acc[tm][tn][j];
    }
  __syncthreads();
  constexpr int CG = BN / 8;
  constexpr int UNITS = (BM / 4) * CG;
  for (int u = tid; u < UNITS; u += NT) {
    const int q = u / CG, gg = u - (u / CG) * CG;
    const int m0 = m_base + q * 4, c0 = n_base + gg * 8;
    if (m0 >= a.M || c0 >= a.cout) continue;
    float v[4][8];
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int j = 0; j < 8; ++j) v[r][j] = Cs[(q * 4 + r) * CSTR + gg * 8 + j];
    epi_vec8(a, m0, c0, v);
  }
}

static bool glds_ok(const ConvArgs& a) {
  return a.zero && a.in_kind == IN_NHWC && !a.w_f32 && a.cin % 8 == 0 && (a.in_cs | a.in_co) % 8 == 0 &&
         a.cout_pad % 128 == 0 && a.kpad % 64 == 0 && (a.ks == 1 || a.ks == 3);
}

// conv_glds_f16 variant (RTDM_GLDS=<BM>x<stages>, e.g. 128x2, 256x3).
struct GldsCfg {
  int bm, ns;
};
static GldsCfg glds_cfg() {
  static GldsCfg v = [] {
    GldsCfg c{128, 2};
    if (const char* e = getenv("RTDM_GLDS")) {
      int bm = 0, ns = 0;
      if (sscanf(e, "%dx%d", &bm, &ns) == 2 && (bm == 128 || bm == 256) && (ns == 2 || ns == 3)) c = {bm, ns};
    }
    return c;
  }();
  return v;
}

// Uniform-tap staging applies when every K-block lies inside one tap and the
// input view's element offsets fit in 30 bits.
static int glds_uniform(const ConvArgs& a) {
  const int64_t elems = (int64_t)a.n * a.ih * a.iw * a.in_cs;
  return a.cin % 64 == 0 && a.kpad == a.ks * a.ks * a.cin && elems < (1ll << 30);
}

// --------------------------------------------------------------------------
// Direct 3x3 / stride 1 / pad 1 convolution on MFMA with an LDS-resident input
// tile (the early, small-Cin Darknet layers, where im2col re-reads dominate).
//
// A block owns a TH x 16 output tile x BN output channels.  Per Cin chunk of CC
// channels (a power of two <= 64) it stages the 10 x 18 input halo tile into
// LDS once (pixel stride CC+8 halfs: consecutive pixels land 4 banks apart, so
// the 16 lanes of a fragment read conflict-free), then runs the chunk's 9*CC/32
// k-steps: K = (tap, channel) in the packed-weight order of pack_conv
// (k = tap*Cin + c), each lane's 8 k-values = 8 channels of one tap.
// Channel-major product D[cout][pixel] = W x X: the weight fragment (A) comes
// from global (L2-resident) one k-step ahead, the pixel fragment (B) from LDS
// at a per-lane tap offset.  Each lane ends with 4 consecutive channels of one
// pixel per fragment -> 8-byte NHWC stores; the 2x2 maxpool combines two
// fragments in-lane and lane pairs through DPP.
// Waves WPX (pixels) x 4/WPX (channels): wave (wp, wc) = tile rows 4wp..4wp+3
// x TC 16-channel tiles; TH = 4*WPX, BN = 16*TC*(4/WPX).  Small Cout uses
// WPX = 4 (every wave owns all BN channels of its 64 pixels).
// --------------------------------------------------------------------------
constexpr int kDirTW = 16, kDirHW = kDirTW + 2;

__device__ __forceinline__ float dpp_xor1(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0xB1, 0xF, 0xF, 0));
}

template <int TC, int WPX>
__global__ __launch_bounds__(256) void conv3_direct(ConvArgs a, int cc_log2) {
  constexpr int WCH = 4 / WPX;           // waves along channels
  constexpr int BN = 16 * TC * WCH;      // channels per block
  constexpr int kDirTH = 4 * WPX;        // tile rows
  extern __shared__ __attribute__((aligned(16))) _Float16 dir_lds[];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int cc = 1 << cc_log2, PS = cc + 8;
  const int tiles_x = (a.ow + kDirTW - 1) / kDirTW, tiles_y = (a.oh + kDirTH - 1) / kDirTH;
  const int nbn = a.cout_pad / BN;
  int bid = blockIdx.x;
  {
    const int nblk = gridDim.x, xcd = bid & 7, q = nblk >> 3, r = nblk & 7;
    bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  }
  const int nb = bid % nbn;
  int t = bid / nbn;
  const int tx = t % tiles_x;
  t /= tiles_x;
  const int ty = t % tiles_y;
  const int n = t / tiles_y;
  const int oy0 = ty * kDirTH, ox0 = tx * kDirTW;
  const int wp = wid / WCH, wc = wid - (wid / WCH) * WCH;
  const int p = lane & 15, g = lane >> 4;
  const int co_base = nb * BN + wc * (16 * TC);

  const _Float16* __restrict__ in = (const _Float16*)a.in + a.in_co;
  const _Float16* __restrict__ wt = (const _Float16*)a.w + (size_t)(co_base + p) * a.kpad;
  f4 acc[TC][4];
#pragma unroll
  for (int i = 0; i < TC; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};

  const int cgl = cc_log2 - 3;  // log2(8-channel groups per tap)
  for (int c0 = 0; c0 < a.cin; c0 += cc) {
    if (c0) __syncthreads();
    const int cv = cc >> 3;
    for (int i = tid; i < (kDirTH + 2) * kDirHW * cv; i += 256) {
      const int pix = i >> cgl, v = i & (cv - 1);
      const int r = pix / kDirHW, c = pix - r * kDirHW;
      const int y = oy0 - 1 + r, x = ox0 - 1 + c;
      u32x4 d = {0u, 0u, 0u, 0u};
      if ((unsigned)y < (unsigned)a.ih && (unsigned)x < (unsigned)a.iw)
        d = *(const u32x4*)(in + ((size_t)(n * a.ih + y) * a.iw + x) * a.in_cs + c0 + v * 8);
      *(u32x4*)(dir_lds + pix * PS + v * 8) = d;
    }
    __syncthreads();
    const int nq = 9 << cgl;         // 8-channel groups in this chunk's K
    const int nks = (nq + 3) >> 2;   // 32-deep k-steps
    auto wload = [&](int s, h8 (&w)[TC]) {
      const int q0 = 4 * s + g;
      const bool kv = q0 < nq;
      const int q = kv ? q0 : 0;  // no out-of-range address even if the load is speculated
      const int tap = q >> cgl, cg = q & ((1 << cgl) - 1);
      const size_t k = (size_t)tap * a.cin + c0 + cg * 8;
#pragma unroll
      for (int i = 0; i < TC; ++i) {
        const h8 z = {};
        w[i] = kv ? *(const h8*)(wt + (size_t)i * 16 * a.kpad + k) : z;
      }
    };
    h8 wcur[TC], wnext[TC];
    wload(0, wcur);
    for (int s = 0; s < nks; ++s) {
      if (s + 1 < nks) wload(s + 1, wnext);
      const int q = 4 * s + g;
      const bool kv = q < nq;
      const int tap = kv ? q >> cgl : 0, cg = q & ((1 << cgl) - 1);
      const int kh = tap / 3, kw = tap - (tap / 3) * 3;
      const _Float16* bp = dir_lds + ((4 * wp + kh) * kDirHW + p + kw) * PS + cg * 8;
      h8 b[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const h8 z = {};
        const h8 v = *(const h8*)(bp + j * kDirHW * PS);
        b[j] = kv ? v : z;
      }
#pragma unroll
      for (int i = 0; i < TC; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wcur[i], b[j], acc[i][j], 0, 0, 0);
#pragma unroll
      for (int i = 0; i < TC; ++i) wcur[i] = wnext[i];
    }
  }

  // ---- epilogue: lane = pixel (oy0 + 4wp + j, ox0 + p), 4 channels per fragment ----
  const Epilogue& e = a.e;
  const int ox = ox0 + p;
  if (e.pool.ptr && !e.full.ptr && !e.up.ptr && !e.res.ptr && e.act != ACT_SWISH) {
    // pooled output only: bias + LeakyReLU are monotone, so max-pool the raw
    // accumulators (2 fragments in-lane, lane pairs by DPP) and run the epilogue
    // once per pooled pixel — bit-identical to pooling the activated values.
    const int qh = a.oh >> 1, qw = a.ow >> 1;
#pragma unroll
    for (int i = 0; i < TC; ++i) {
      const int c0 = co_base + i * 16 + 4 * g;
      const bool cval = c0 < a.cout;
      float bias[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) bias[r] = (e.bias && cval) ? e.bias[c0 + r] : 0.f;
#pragma unroll
      for (int j = 0; j < 4; j += 2) {
        float m[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float t2 = fmaxf(acc[i][j][r], acc[i][j + 1][r]);
          float x = fmaxf(t2, dpp_xor1(t2)) + bias[r];
          if (e.act == ACT_LEAKY) x = x > 0.f ? x : x * e.slope;
          m[r] = x;
        }
        const int py = (oy0 + 4 * wp + j) >> 1, px = ox >> 1;
        if (cval && (p & 1) == 0 && py < qh && px < qw) {
          const size_t pp = ((size_t)n * qh + py) * qw + px;
          *(uint2*)((_Float16*)e.pool.ptr + pp * e.pool.cs + e.pool.co + c0) =
              make_uint2(pack_h2(m[0], m[1]), pack_h2(m[2], m[3]));
        }
      }
    }
    return;
  }
#pragma unroll
  for (int i = 0; i < TC; ++i) {
    const int c0 = co_base + i * 16 + 4 * g;
    const bool cval = c0 < a.cout;
    float bias[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) bias[r] = (e.bias && cval) ? e.bias[c0 + r] : 0.f;
    float v[4][4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int oy = oy0 + 4 * wp + j;
      const bool pv = cval && oy < a.oh && ox < a.ow;
      const size_t pix = ((size_t)n * a.oh + oy) * a.ow + ox;
      float x[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float t2 = acc[i][j][r] + bias[r];
        if (e.act == ACT_LEAKY)
          t2 = t2 > 0.f ? t2 : t2 * e.slope;
        else if (e.act == ACT_SWISH)
          t2 = t2 * sigmoidf_(t2);
        x[r] = t2;
      }
      if (e.res.ptr && pv) {
        const uint2 rv = *(const uint2*)((const _Float16*)e.res.ptr + pix * e.res.cs + e.res.co + c0);
        const _Float16* rh = (const _Float16*)&rv;
#pragma unroll
        for (int r = 0; r < 4; ++r) x[r] += (float)rh[r];
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) v[j][r] = x[r];
      const uint2 hv = make_uint2(pack_h2(x[0], x[1]), pack_h2(x[2], x[3]));
      if (e.full.ptr && pv) *(uint2*)((_Float16*)e.full.ptr + pix * e.full.cs + e.full.co + c0) = hv;
      if (e.up.ptr && pv) {
        const int uw = a.ow * 2;
        const size_t u0 = ((size_t)n * a.oh * 2 + 2 * oy) * uw + 2 * ox;
        _Float16* up = (_Float16*)e.up.ptr + e.up.co + c0;
        *(uint2*)(up + u0 * e.up.cs) = hv;
        *(uint2*)(up + (u0 + 1) * e.up.cs) = hv;
        *(uint2*)(up + (u0 + uw) * e.up.cs) = hv;
        *(uint2*)(up + (u0 + uw + 1) * e.up.cs) = hv;
      }
    }
    if (e.pool.ptr) {
      const int qh = a.oh >> 1, qw = a.ow >> 1;
#pragma unroll
      for (int j = 0; j < 4; j += 2) {
        float m[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float t2 = fmaxf(v[j][r], v[j + 1][r]);
          m[r] = fmaxf(t2, dpp_xor1(t2));
        }
        const int py = (oy0 + 4 * wp + j) >> 1, px = ox >> 1;
        if (cval && (p & 1) == 0 && py < qh && px < qw) {
          const size_t pp = ((size_t)n * qh + py) * qw + px;
          *(uint2*)((_Float16*)e.pool.ptr + pp * e.pool.cs + e.pool.co + c0) =
              make_uint2(pack_h2(m[0], m[1]), pack_h2(m[2], m[3]));
        }
      }
    }
  }
}

// --------------------------------------------------------------------------
// conv3_pool_small: 3x3 / s1 / p1 convolution + fused 2x2 maxpool for the
// small-Cin early layers (Cin 16 / 32, Cout 32 / 64; the 608x608 Darknet's
// layers 2 and 4, where the work per output is tiny and address arithmetic,
// not MFMA, sets the speed).  Everything that does not depend on the tile is
// hoisted out of the K loop:
//   * each lane's weight fragments for the whole K (NKS k-steps x WCH channel
//     tiles) are loaded once into registers;
//   * each lane's LDS offset for every k-step (tap, 8-channel group) is
//     computed once; per k-step the B fragment of tile row j is one
//     ds_read_b128 at that offset + a compile-time row stride;
//   * the 2x2 maxpool runs on the raw accumulators (bias + LeakyReLU are
//     monotone): in-lane over tile rows j, j+1 and across the lane pair
//     (p, p^1) by DPP, then one bias/activation/store per pooled pixel.
// Block: TH x 16 output pixels x COUT channels; waves = (TH / WROWS) row
// groups x (COUT / 16 / WCH) channel groups = 4.  LDS: the 18 x 18 input halo,
// pixel stride PS halfs (below: chosen so the B-fragment reads are conflict-free).
// --------------------------------------------------------------------------
// NWV: waves per block (4, or 8 for Cin 64 -> Cout 128: one 16-channel tile per wave, 18
// k-steps of weights = 72 registers).  A full-resolution output view (a.e.full) is written
// too when present (Cin 64: yolov4-tiny L6, whose map a route reads).
template <int CIN, int COUT, int TH, int WROWS, int WCH, int PF = 1, int NWV = 4>
__global__ __launch_bounds__(64 * NWV, NWV == 8 ? 1 : (CIN == 16 || WCH == 1) && !(CIN == 32 && PF > 1) ? 3 : 2) void conv3_pool_small(ConvArgs a) {  // 3 blocks per CU (<= 168 registers): CIN 16, and CIN 32 with one 16-channel tile per wave (WCH 1: half the weight registers; with WCH 2 it would spill)
  // PS: halo pixel stride (halfs).  Cin 32: 48, so the B-fragment reads of a 16-lane group
  // (16 pixels x 2 channel groups) fall in 16 distinct 4-bank slots (at 40: 2-way conflicts,
  // half the kernel's LDS cycles, PMC r04f)
  // Cin 64: 80 (the 1x1-style pattern, 16 pixels x 4 channel groups per k-step: conflict-free)
  // Cin 16: 16, unpadded -- a k-step's lane groups pair the two channel halves of one tap
  // (+16 B), which at 32-B pixels fill all 16 slots (at 24: 18 extra cycles per 5 k-steps)
  constexpr int TW = 16, HW = TW + 2, PS = CIN == 32 ? 48 : CIN == 64 ? 80 : CIN == 16 ? 16 : CIN + 8;
  constexpr int NT = 64 * NWV;
  constexpr int CG = CIN / 8;                // 8-channel groups per tap
  constexpr int NQ = 9 * CG;                 // 8-channel groups in K
  constexpr int NKS = (NQ + 3) / 4;          // 32-deep k-steps
  constexpr int RG = TH / WROWS;             // row groups of waves
  constexpr int HALO = (TH + 2) * HW * CG;   // 16-byte vectors per staged tile
  constexpr int PV = (HALO + NT - 1) / NT;   // prefetch registers per thread
  constexpr int XS = (TH + 2) * HW * PS;     // halfs per LDS buffer
  static_assert(RG * (COUT / 16 / WCH) == NWV, "wave layout must cover the block's waves");
  __shared__ __attribute__((aligned(16))) _Float16 xs[2 * XS];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int p = lane & 15, g = lane >> 4;
  const int tiles_x = (a.ow + TW - 1) / TW, tiles_y = (a.oh + TH - 1) / TH;
  const int ntiles = a.n * tiles_y * tiles_x;
  const int wr = wid % RG, wc = wid / RG;
  const int co0 = wc * WCH * 16;

  // weights for the whole K stay in registers across all tiles of this (persistent) block
  h8 wf[NKS][WCH];
#pragma unroll
  for (int s = 0; s < NKS; ++s) {
    const int q = 4 * s + g;  // k = 8q (zero-padded weights beyond 9*CIN)
#pragma unroll
    for (int t = 0; t < WCH; ++t) wf[s][t] = *(const h8*)((const _Float16*)a.w + (size_t)(co0 + 16 * t + p) * a.kpad + 8 * q);
  }
  // per-lane LDS offset of every k-step (tap clamped for the zero-weight tail)
  // (Cin 64: a k-step is half of one tap's channels, so the offset is a compile-time constant
  // per k-step plus 8 g: no per-k-step registers, which the 8-wave variant cannot spare)
  int kofs[CIN == 64 ? 1 : NKS];
  if constexpr (CIN != 64) {
#pragma unroll
    for (int s = 0; s < NKS; ++s) {
      int q = 4 * s + g;
      q = q < NQ ? q : NQ - 1;
      const int tap = q / CG, cg = q - tap * CG;
      const int kh = tap / 3, kw = tap - kh * 3;
      kofs[s] = (kh * HW + kw) * PS + cg * 8;
    }
  }
  const int g8 = 8 * g;
  auto kofs_of = [&](int s) {
    if constexpr (CIN == 64) {
      const int tap = s >> 1, kh = tap / 3, kw = tap - kh * 3;
      return (kh * HW + kw) * PS + (s & 1) * 32 + g8;
    } else {
      return kofs[s];
    }
  };
  float bias[WCH][4];
#pragma unroll
  for (int t = 0; t < WCH; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) bias[t][r] = a.e.bias ? a.e.bias[co0 + 16 * t + 4 * g + r] : 0.f;

  const _Float16* __restrict__ in = (const _Float16*)a.in + a.in_co;
  // per-thread halo slots, fixed across tiles: (row, column) of the 16-byte vector k and
  // its LDS offset (the prefetch addressing was ~30 VALU per vector when recomputed)
  int hr[PV], hc[PV], hoff[PV], soff[PV];
#pragma unroll
  for (int k = 0; k < PV; ++k) {
    const int i = tid + NT * k;
    const int pix = i / CG, v = i - pix * CG;
    hr[k] = i < HALO ? pix / HW : -(1 << 20);  // out of range: never loaded
    hc[k] = pix - (pix / HW) * HW;
    hoff[k] = v * 8;
    soff[k] = pix * PS + v * 8;
  }
  const int img = a.ih * a.iw * a.in_cs;  // halfs per image (< 2^31: planner limits)
  // PF halo register sets: tiles t + tstep .. t + PF*tstep in flight while tile t computes
  // (PF 2: twice the bytes in flight per CU; these layers are HBM-latency bound)
  u32x4 pre[PV], pre2[PF > 1 ? PV : 1];
  auto prefetch_to = [&](int tile, u32x4 (&dst)[PV]) {
    // (tile -> (n, ty, tx) by multiply-shift: as integer divisions they were ~1/3 of the
    // kernel's VALU)
    const int t1 = fdiv(tile, a.fd_tx), tx = tile - t1 * tiles_x;
    const int n = fdiv(t1, a.fd_ty), ty = t1 - n * tiles_y;
    const _Float16* base = in + (size_t)n * img;
    const int y0 = ty * TH - 1, x0 = tx * TW - 1;
#pragma unroll
    for (int k = 0; k < PV; ++k) {
      const int y = y0 + hr[k], x = x0 + hc[k];
      u32x4 d = {0u, 0u, 0u, 0u};
      if ((unsigned)y < (unsigned)a.ih && (unsigned)x < (unsigned)a.iw)
        d = *(const u32x4*)(base + (y * a.iw + x) * a.in_cs + hoff[k]);
      dst[k] = d;
    }
  };
  const Epilogue& e = a.e;
  const int qh = a.oh >> 1, qw = a.ow >> 1;
  // LeakyReLU as max(x, slope x) (0 < slope < 1; slope 1 = linear): same values, no branch
  const float slope = e.act == ACT_LEAKY ? e.slope : 1.f;
  int buf = 0;
  int tile, tend, tstep;  // XCD-contiguous tile walk (horizontal neighbours share the halo columns)
  xcd_span(blockIdx.x, gridDim.x, ntiles, tile, tend, tstep);
  if constexpr (PF == 1) {
    if (tile < tend) prefetch_to(tile, pre);
    for (; tile < tend; tile += tstep) {
      _Float16* xb_w = xs + buf * XS;
#pragma unroll
      for (int k = 0; k < PV; ++k)
        if (tid + NT * k < HALO) *(u32x4*)(xb_w + soff[k]) = pre[k];
      __syncthreads();
      const int t1 = fdiv(tile, a.fd_tx), tx = tile - t1 * tiles_x;
      const int n = fdiv(t1, a.fd_ty), ty = t1 - n * tiles_y;
      if (tile + tstep < tend) prefetch_to(tile + tstep, pre);  // in flight during the MFMAs
      const _Float16* xb = xb_w + (wr * WROWS * HW + p) * PS;
      f4 acc[WROWS][WCH];
#pragma unroll
      for (int j = 0; j < WROWS; ++j)
#pragma unroll
        for (int t = 0; t < WCH; ++t) acc[j][t] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < NKS; ++s) {
        const _Float16* bp = xb + kofs_of(s);
#pragma unroll
        for (int j = 0; j < WROWS; ++j) {
          const h8 b = *(const h8*)(bp + j * HW * PS);
#pragma unroll
          for (int t = 0; t < WCH; ++t)
            acc[j][t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wf[s][t], b, acc[j][t], 0, 0, 0);
        }
        if constexpr (CIN == 64) {  // one k-step's reads, then its MFMAs: no reads hoisted further
          __builtin_amdgcn_sched_group_barrier(0x100, WROWS, 0);
          __builtin_amdgcn_sched_group_barrier(0x008, WROWS * WCH, 0);
        }
      }
      // pooled epilogue: lane = pixel column ox0 + p, rows j; channels co0 + 16t + 4g + r.
      // One pooled-row pointer per tile; rows j step by qw pixels.
      const int px = (tx * TW + p) >> 1;
      const int py0 = (ty * TH + wr * WROWS) >> 1;
      _Float16* const prow = (_Float16*)e.pool.ptr + e.pool.co + co0 + 4 * g +
                            ((size_t)(n * qh + py0) * qw + px) * e.pool.cs;
      const bool lane_st = (p & 1) == 0 && px < qw;
#pragma unroll
      for (int j = 0; j < WROWS; j += 2) {
        const bool st = lane_st && py0 + j / 2 < qh;
#pragma unroll
        for (int t = 0; t < WCH; ++t) {
          if (e.full.ptr) {  // rows j, j+1 at full resolution: bias -> LeakyReLU -> fp16
            const int ox = tx * TW + p;
#pragma unroll
            for (int jj = 0; jj < 2; ++jj) {
              const int oy = ty * TH + wr * WROWS + j + jj;
              float v[4];
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                const float x = acc[j + jj][t][r] + bias[t][r];
                v[r] = fmaxf(x, x * slope);
              }
              if (ox < a.ow && oy < a.oh)
                *(uint2*)((_Float16*)e.full.ptr + ((size_t)(n * a.oh + oy) * a.ow + ox) * e.full.cs + e.full.co + co0 +
                          16 * t + 4 * g) = make_uint2(pack_h2(v[0], v[1]), pack_h2(v[2], v[3]));
            }
          }
          float m[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float t2 = fmaxf(acc[j][t][r], acc[j + 1][t][r]);
            const float x = fmaxf(t2, dpp_xor1(t2)) + bias[t][r];
            m[r] = fmaxf(x, x * slope);
          }
          if (st)
            *(uint2*)(prow + (size_t)(j / 2) * qw * e.pool.cs + 16 * t) =
                make_uint2(pack_h2(m[0], m[1]), pack_h2(m[2], m[3]));
        }
      }
      buf ^= 1;
    }
  } else {
    if (tile < tend) prefetch_to(tile, pre);
    if (tile + tstep < tend) prefetch_to(tile + tstep, pre2);
    auto body = [&](u32x4 (&cur)[PV]) {
      _Float16* xb_w = xs + buf * XS;
#pragma unroll
      for (int k = 0; k < PV; ++k)
        if (tid + NT * k < HALO) *(u32x4*)(xb_w + soff[k]) = cur[k];
      __syncthreads();
      const int t1 = fdiv(tile, a.fd_tx), tx = tile - t1 * tiles_x;
      const int n = fdiv(t1, a.fd_ty), ty = t1 - n * tiles_y;
      if (tile + 2 * tstep < tend) prefetch_to(tile + 2 * tstep, cur);  // two tiles in flight
      // (the tile's MFMAs + pooled epilogue as in the PF 1 loop, written out: as a shared lambda
      // the compiler allocated ~27 more VGPRs, 135 -> 162)
      const _Float16* xb = xb_w + (wr * WROWS * HW + p) * PS;
      f4 acc[WROWS][WCH];
#pragma unroll
      for (int j = 0; j < WROWS; ++j)
#pragma unroll
        for (int t = 0; t < WCH; ++t) acc[j][t] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < NKS; ++s) {
        const _Float16* bp = xb + kofs_of(s);
#pragma unroll
        for (int j = 0; j < WROWS; ++j) {
          const h8 b = *(const h8*)(bp + j * HW * PS);
#pragma unroll
          for (int t = 0; t < WCH; ++t)
            acc[j][t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wf[s][t], b, acc[j][t], 0, 0, 0);
        }
        if constexpr (CIN == 64) {  // one k-step's reads, then its MFMAs: no reads hoisted further
          __builtin_amdgcn_sched_group_barrier(0x100, WROWS, 0);
          __builtin_amdgcn_sched_group_barrier(0x008, WROWS * WCH, 0);
        }
      }
      // pooled epilogue: lane = pixel column ox0 + p, rows j; channels co0 + 16t + 4g + r.
      // One pooled-row pointer per tile; rows j step by qw pixels.
      const int px = (tx * TW + p) >> 1;
      const int py0 = (ty * TH + wr * WROWS) >> 1;
      _Float16* const prow = (_Float16*)e.pool.ptr + e.pool.co + co0 + 4 * g +
                            ((size_t)(n * qh + py0) * qw + px) * e.pool.cs;
      const bool lane_st = (p & 1) == 0 && px < qw;
#pragma unroll
      for (int j = 0; j < WROWS; j += 2) {
        const bool st = lane_st && py0 + j / 2 < qh;
#pragma unroll
        for (int t = 0; t < WCH; ++t) {
          if (e.full.ptr) {  // rows j, j+1 at full resolution: bias -> LeakyReLU -> fp16
            const int ox = tx * TW + p;
#pragma unroll
            for (int jj = 0; jj < 2; ++jj) {
              const int oy = ty * TH + wr * WROWS + j + jj;
              float v[4];
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                const float x = acc[j + jj][t][r] + bias[t][r];
                v[r] = fmaxf(x, x * slope);
              }
              if (ox < a.ow && oy < a.oh)
                *(uint2*)((_Float16*)e.full.ptr + ((size_t)(n * a.oh + oy) * a.ow + ox) * e.full.cs + e.full.co + co0 +
                          16 * t + 4 * g) = make_uint2(pack_h2(v[0], v[1]), pack_h2(v[2], v[3]));
            }
          }
          float m[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float t2 = fmaxf(acc[j][t][r], acc[j + 1][t][r]);
            const float x = fmaxf(t2, dpp_xor1(t2)) + bias[t][r];
            m[r] = fmaxf(x, x * slope);
          }
          if (st)
            *(uint2*)(prow + (size_t)(j / 2) * qw * e.pool.cs + 16 * t) =
                make_uint2(pack_h2(m[0], m[1]), pack_h2(m[2], m[3]));
        }
      }
      buf ^= 1;
      tile += tstep;
    };
    while (tile < tend) {
      body(pre);
      if (tile < tend) body(pre2);
    }
  }
}

static bool pool_small_ok(const ConvArgs& a) {
  if (a.in_kind != IN_NHWC || a.ks != 3 || a.stride != 1 || a.pad != 1 || a.w_f32) return false;
  const bool c64 = a.cin == 64 && a.cout == 128 && tune().pool_small64;
  if (!((a.cin == 16 && a.cout == 32) || (a.cin == 32 && a.cout == 64) || c64)) return false;
  if (a.cout_pad != a.cout || (a.in_cs | a.in_co) & 7 || a.oh != a.ih || a.ow != a.iw || (a.oh | a.ow) & 1) return false;
  if (!a.e.pool.ptr || (a.e.full.ptr && !c64) || a.e.up.ptr || a.e.res.ptr || a.e.io || a.e.scale || a.e.act == ACT_SWISH)
    return false;
  if (a.e.full.ptr && ((a.e.full.cs | a.e.full.co) & 3)) return false;
  if ((a.e.pool.cs | a.e.pool.co) & 3) return false;
  if (a.e.act == ACT_LEAKY && !(a.e.slope > 0.f && a.e.slope <= 1.f)) return false;  // max(x, slope x)
  if ((int64_t)a.ih * a.iw * a.in_cs >= (1ll << 31)) return false;                  // 32-bit image offsets
  return a.kpad >= 32 * ((9 * a.cin / 8 + 3) / 4);  // weights read up to k = 32 * NKS
}

// Resident blocks per CU of a kernel (occupancy API, cached by the caller).
template <class K>
static int resident_blocks(K kernel, int threads, size_t lds) {
  int nb = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kernel, threads, lds) != hipSuccess || nb < 1) nb = 1;
  return nb;
}

static int cu_count() {
  static int n = [] {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v < 1)
      v = 256;
    return v;
  }();
  return n;
}

static void launch_pool_small(const ConvArgs& a_in, hipStream_t s) {
  const int th = a_in.cin == 16 ? 16 : 8;
  ConvArgs a = a_in;
  a.fd_tx = make_fastdiv((a.ow + 15) / 16);
  a.fd_ty = make_fastdiv((a.oh + th - 1) / th);
  if (a.cin == 64) {  // 8 waves, one 16-channel tile each
    const int64_t tiles64 = (int64_t)a.n * ((a.oh + 7) / 8) * ((a.ow + 15) / 16);
    RTDM_REQUIRE(tiles64 < (1ll << 31), RTDM_E_CAPACITY, "conv: too many tiles");
    static const int per_cu = resident_blocks(conv3_pool_small<64, 128, 8, 4, 2, 1, 8>, 512, 0);
    const int64_t blocks = std::min<int64_t>(tiles64, (int64_t)per_cu * cu_count());
    hipLaunchKernelGGL((conv3_pool_small<64, 128, 8, 4, 2, 1, 8>), dim3((unsigned)blocks), dim3(512), 0, s, a);
    return;
  }
  const int64_t tiles = (int64_t)a.n * ((a.oh + th - 1) / th) * ((a.ow + 15) / 16);
  RTDM_REQUIRE(tiles < (1ll << 31), RTDM_E_CAPACITY, "conv: too many tiles");
  // persistent blocks: exactly the resident count, each streaming tiles with its weights in registers
  // halo tiles in flight per block: 2 for Cin 16 (b64 L2 0.082 -> 0.077 ms), 1 for Cin 32 (at 2
  // it needs 210 VGPRs, 2 blocks per CU: 0.056 -> 0.058 ms; profiles/r04s_pool_small_pf.txt);
  // rtdm_set_tuning("pool_small_pf", 1 | 2) forces one (0 = this choice)
  const bool pf2 = tune().pool_small_pf ? tune().pool_small_pf >= 2 : a.cin == 16;
  if (a.cin == 16) {
    static const int per_cu = resident_blocks(conv3_pool_small<16, 32, 16, 4, 2>, 256, 0);
    static const int per_cu2 = resident_blocks(conv3_pool_small<16, 32, 16, 4, 2, 2>, 256, 0);
    const int64_t blocks = std::min<int64_t>(tiles, (int64_t)(pf2 ? per_cu2 : per_cu) * cu_count());
    if (pf2)
      hipLaunchKernelGGL((conv3_pool_small<16, 32, 16, 4, 2, 2>), dim3((unsigned)blocks), dim3(256), 0, s, a);
    else
      hipLaunchKernelGGL((conv3_pool_small<16, 32, 16, 4, 2>), dim3((unsigned)blocks), dim3(256), 0, s, a);
  } else {
    static const int per_cu = resident_blocks(conv3_pool_small<32, 64, 8, 8, 1>, 256, 0);
    static const int per_cu2 = resident_blocks(conv3_pool_small<32, 64, 8, 8, 1, 2>, 256, 0);
    const int64_t blocks = std::min<int64_t>(tiles, (int64_t)(pf2 ? per_cu2 : per_cu) * cu_count());
    if (pf2)
      hipLaunchKernelGGL((conv3_pool_small<32, 64, 8, 8, 1, 2>), dim3((unsigned)blocks), dim3(256), 0, s, a);
    else
      hipLaunchKernelGGL((conv3_pool_small<32, 64, 8, 8, 1>), dim3((unsigned)blocks), dim3(256), 0, s, a);
  }
}

static int direct_cc_log2(int cin) {
  for (int l = 6; l >= 3; --l)
    if (cin % (1 << l) == 0) return l;
  return -1;
}

// Direct-conv configuration for cout_pad: (TC, WPX) and channels per block.
struct DirCfg {
  int tc, wpx, bn, th;
};
static DirCfg direct_cfg(int cout_pad) {
  if (cout_pad == 32) return {2, 4, 32, 16};
  if (cout_pad == 64) return {4, 4, 64, 16};
  return {4, 2, 128, 8};
}

static size_t direct_lds_bytes(int cc_log2, int th) {
  return (size_t)(th + 2) * kDirHW * ((1 << cc_log2) + 8) * 2;
}

static bool direct_ok(const ConvArgs& a) {
  if (a.in_kind != IN_NHWC || a.ks != 3 || a.stride != 1 || a.pad != 1 || a.w_f32) return false;
  if (a.cin % 16 || a.cin > 32 || (a.in_cs | a.in_co) & 7 || a.cout % 4 || a.e.io || a.e.scale) return false;
  if (a.cout_pad != 32 && a.cout_pad != 64 && a.cout_pad % 128) return false;
  if (a.oh != a.ih || a.ow != a.iw || a.ow < 64) return false;
  const View* vs[4] = {&a.e.full, &a.e.pool, &a.e.up, &a.e.res};
  for (const View* v : vs)
    if (v->ptr && ((v->cs | v->co) & 3)) return false;
  if (a.e.pool.ptr && ((a.oh | a.ow) & 1)) return false;
  return direct_cc_log2(a.cin) >= 4;
}

static void launch_direct(const ConvArgs& a, hipStream_t s) {
  const int l = direct_cc_log2(a.cin);
  const DirCfg c = direct_cfg(a.cout_pad);
  const int64_t blocks = (int64_t)a.n * ((a.oh + c.th - 1) / c.th) * ((a.ow + kDirTW - 1) / kDirTW) * (a.cout_pad / c.bn);
  const size_t lds = direct_lds_bytes(l, c.th);
  if (c.bn == 128)
    hipLaunchKernelGGL((conv3_direct<4, 2>), dim3((unsigned)blocks), dim3(256), lds, s, a, l);
  else if (c.bn == 64)
    hipLaunchKernelGGL((conv3_direct<4, 4>), dim3((unsigned)blocks), dim3(256), lds, s, a, l);
  else
    hipLaunchKernelGGL((conv3_direct<2, 4>), dim3((unsigned)blocks), dim3(256), lds, s, a, l);
}

// --------------------------------------------------------------------------
template <int BM, int BN, int BK, int WM, int WN>
static void launch_mfma(const ConvArgs& a, hipStream_t s) {
  RTDM_REQUIRE(a.cout_pad % BN == 0, RTDM_E_INVALID, "conv: cout_pad not a multiple of BN");
  RTDM_REQUIRE(a.kpad % BK == 0, RTDM_E_INVALID, "conv: kpad not a multiple of BK");
  const int64_t nblk = (int64_t)((a.M + BM - 1) / BM) * (a.cout_pad / BN);
  RTDM_REQUIRE(nblk < (1ll << 31), RTDM_E_CAPACITY, "conv: grid too large");
  const dim3 grid((unsigned)nblk), block(64 * WM * WN);
  if (epi_lean_ok(a))
    hipLaunchKernelGGL((conv_mfma_f16<BM, BN, BK, WM, WN, 1>), grid, block, 0, s, a);
  else if (epi_io_ok(a))
    hipLaunchKernelGGL((conv_mfma_f16<BM, BN, BK, WM, WN, 2>), grid, block, 0, s, a);
  else
    hipLaunchKernelGGL((conv_mfma_f16<BM, BN, BK, WM, WN, 0>), grid, block, 0, s, a);
}

static bool mfma_ok(const ConvArgs& a) {
  return a.in_kind == IN_NHWC && a.cin % 8 == 0 && a.in_cs % 8 == 0 && a.in_co % 8 == 0;
}

static bool stem_ok(const ConvArgs& a) {
  if (!a.w_stem || a.cin != 3 || a.ks != 3 || (a.stride != 1 && a.stride != 2) || a.pad < 0 || a.pad > 1) return false;
  if (a.in_kind == IN_NHWC && (a.in_cs < 3)) return false;
  if (a.cout_pad % 16 != 0 || (a.cout_pad != 16 && a.cout_pad != 32 && a.cout_pad != 64)) return false;
  if (a.e.res.ptr || a.e.up.ptr || a.e.io) return false;
  if (a.e.full.ptr && ((a.e.full.cs | a.e.full.co) & 3)) return false;
  // pooled variant: output only the 2x2-pooled view (quad order); plain variant: full view only
  if (a.quad ? (!a.e.pool.ptr || a.e.full.ptr || (a.oh | a.ow) & 1) : (!a.e.full.ptr || a.e.pool.ptr)) return false;
  return stem3_lds_bytes(a) <= 64 * 1024;
}

// Pipelined 256x128 kernel (conv_pipe.hip) for the Cin % 64 == 0 layers; 0 = off
// (conv_glds_f16 takes them).  RTDM_CONV_PIPE in the environment, or
// rtdm_set_tuning("conv_pipe", v), for A/B runs.
int stem_abl() { return tune().stem_abl; }
int conv_pipe_mode() { return tune().conv_pipe; }

// Stand-alone YOLO head convs on head1x1_f16 (head.hip); 0 = conv_pipe's decode epilogue
// (rtdm_set_tuning("head1x1", v), for A/B runs; bit-identical either way).

static bool use_pipe(const ConvArgs& a, int dtype) {
  return dtype == RTDM_F16 && (conv_pipe_mode() > 0 || a.head_w) && conv_pipe_ok(a);
}

const char* conv_kernel_name(const ConvArgs& a, int dtype) {
  if (dtype == RTDM_F16 && stem_ok(a)) {
    static const char* names[2][2][3] = {
        {{"conv_stem3<false,1>", "conv_stem3<false,2>", "conv_stem3<false,4>"},
         {"conv_stem3<true,1>", "conv_stem3<true,2>", "conv_stem3<true,4>"}},
        {{"conv_stem3<false,1,k16>", "conv_stem3<false,2,k16>", "conv_stem3<false,4,k16>"},
         {"conv_stem3<true,1,k16>", "conv_stem3<true,2,k16>", "conv_stem3<true,4,k16>"}}};
    const int ntn = a.cout_pad / 16;
    return names[tune().stem_k16 ? 1 : 0][a.quad ? 1 : 0][ntn == 1 ? 0 : ntn == 2 ? 1 : 2];
  }
  if (dtype == RTDM_F16 && pool_small_ok(a))
    return a.cin == 16   ? "conv3_pool_small<16,32,16,4,2>"
           : a.cin == 64 ? "conv3_pool_small<64,128,8,4,2,1,8>"
                         : "conv3_pool_small<32,64,8,8,1>";
  if (dtype == RTDM_F16 && c32_ok(a)) return c32_name(a);
  if (dtype == RTDM_F16 && direct_ok(a)) {
    const int bn = direct_cfg(a.cout_pad).bn;
    return bn == 128 ? "conv3_direct<4,2>" : bn == 64 ? "conv3_direct<4,4>" : "conv3_direct<2,4>";
  }
  if (dtype == RTDM_F16 && tune().head1x1 && head1x1_ok(a)) return head1x1_name(a);
  if (use_pipe(a, dtype)) return conv_pipe_name(a);
  if (dtype == RTDM_F16 && glds_ok(a)) {
    static const char* names[2][2] = {{"conv_glds_f16<128,2>", "conv_glds_f16<128,3>"},
                                      {"conv_glds_f16<256,2>", "conv_glds_f16<256,3>"}};
    const GldsCfg c = glds_cfg();
    return names[c.bm == 256][c.ns == 3];
  }
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
  RTDM_REQUIRE(!a.head_w || use_pipe(a, dtype), RTDM_E_INVALID, "conv: fused head on a shape conv_pipe_f16 does not take");
  RTDM_REQUIRE(!a.quad || (a.oh >= 2 && a.ow >= 2), RTDM_E_INVALID, "conv: quad ordering needs >= 2x2 output");
  RTDM_REQUIRE(!a.e.pool.ptr || a.quad, RTDM_E_INVALID, "conv: pooled output needs quad ordering");
  if (dtype == RTDM_F16 && stem_ok(a)) {
    const int rows = stem_rows(a.quad != 0);
    const int blocks = a.n * ((a.oh + rows - 1) / rows);
    const size_t lds = stem3_lds_bytes(a);
    const int ntn = a.cout_pad / 16;
    const int abl = stem_abl();
    const bool k16 = tune().stem_k16 != 0;
    if (a.quad && abl) {  // diagnostic ablation builds (tools/ab_conv.py --key stem_abl)
      RTDM_REQUIRE(ntn == 1 && k16 && (abl == 1 || abl == 2 || abl == 4 || abl == 7), RTDM_E_INVALID,
                   "stem_abl: 1 | 2 | 4 | 7 on the 16-channel K16 pooled stem");
      if (abl == 1) hipLaunchKernelGGL((conv_stem3<true, 1, true, 1>), dim3(blocks), dim3(256), lds, s, a);
      else if (abl == 2) hipLaunchKernelGGL((conv_stem3<true, 1, true, 2>), dim3(blocks), dim3(256), lds, s, a);
      else if (abl == 4) hipLaunchKernelGGL((conv_stem3<true, 1, true, 4>), dim3(blocks), dim3(256), lds, s, a);
      else hipLaunchKernelGGL((conv_stem3<true, 1, true, 7>), dim3(blocks), dim3(256), lds, s, a);
    } else {
      auto go = [&](auto pool_c, auto k16_c) {
        constexpr bool P = decltype(pool_c)::value, K = decltype(k16_c)::value;
        if (ntn == 1) hipLaunchKernelGGL((conv_stem3<P, 1, K>), dim3(blocks), dim3(256), lds, s, a);
        else if (ntn == 2) hipLaunchKernelGGL((conv_stem3<P, 2, K>), dim3(blocks), dim3(256), lds, s, a);
        else hipLaunchKernelGGL((conv_stem3<P, 4, K>), dim3(blocks), dim3(256), lds, s, a);
      };
      if (a.quad && k16) go(std::true_type{}, std::true_type{});
      else if (a.quad) go(std::true_type{}, std::false_type{});
      else if (k16) go(std::false_type{}, std::true_type{});
      else go(std::false_type{}, std::false_type{});
    }
  } else if (dtype == RTDM_F16 && pool_small_ok(a)) {
    launch_pool_small(a, s);
  } else if (dtype == RTDM_F16 && c32_ok(a)) {
    launch_c32(a, s);
  } else if (dtype == RTDM_F16 && direct_ok(a)) {
    launch_direct(a, s);
  } else if (dtype == RTDM_F16 && tune().head1x1 && head1x1_ok(a)) {
    launch_head1x1(a, s);
  } else if (use_pipe(a, dtype)) {
    launch_conv_pipe(a, s);
  } else if (dtype == RTDM_F16 && glds_ok(a)) {
    const GldsCfg c = glds_cfg();
    const int64_t nblk = (int64_t)((a.M + c.bm - 1) / c.bm) * (a.cout_pad / 128);
    RTDM_REQUIRE(nblk < (1ll << 31), RTDM_E_CAPACITY, "conv: grid too large");
    ConvArgs b = a;
    b.glds_uni = glds_uniform(a);
    const dim3 grid((unsigned)nblk), block(2 * c.bm);
    if (c.bm == 128 && c.ns == 2)
      hipLaunchKernelGGL((conv_glds_f16<128, 2>), grid, block, 0, s, b);
    else if (c.bm == 128)
      hipLaunchKernelGGL((conv_glds_f16<128, 3>), grid, block, 0, s, b);
    else if (c.ns == 2)
      hipLaunchKernelGGL((conv_glds_f16<256, 2>), grid, block, 0, s, b);
    else
      hipLaunchKernelGGL((conv_glds_f16<256, 3>), grid, block, 0, s, b);
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
