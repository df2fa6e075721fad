// Darknet's first two conv layers as ONE persistent row-band launch: conv 3 -> 16 3x3/s1/p1 on
// the uint8 frame + 2x2 maxpool, then conv 16 -> 32 3x3/s1/p1 + 2x2 maxpool (yolov4-tiny /
// yolov3-tiny cfg layers 0-3: victim_localization/yolov3/models.py:23-44 conv + BN + LeakyReLU
// and :57-64 maxpool, as Darknet.forward runs them :345-347).
//
// The two-launch path (conv_stem3<true,1,k16> then conv3_pool_small<16,32>) writes the 16-channel
// pooled stem map P0 (fp16: 189 MB per b64 batch at 608) and reads it back.  Here a workgroup owns
// a band of rows of the SECOND pooled map P2 over the whole image width and walks down it; P0 only
// ever exists as a 6-row ring in LDS:
//   frame ring  12 frame rows, u8 -> fp16 4-channel pixels (conv_stem3's LDS image), zero outside
//               the frame; the rows of phase k + 1 are converted during phase k (loaded during
//               phase k - 1), so the next rows are in flight while this phase computes;
//   phase k     the stem for P0 rows 2k+1, 2k+2 (conv_stem3's pooled tile: 4 quads x 16 channels
//               on v_mfma_f32_16x16x32_f16 + the kh = 2 third on v_mfma_f32_16x16x16f16, quad max
//               in lane, max -> x / 255 + bias -> LeakyReLU) into the P0 ring, AND the 16 -> 32
//               conv for P2 row k - 1 from P0 rows 2k-3 .. 2k (conv3_pool_small<16,32>'s K loop and
//               DPP pool) -- independent work, one barrier per phase;
// so no P0 row is computed twice along a band (one halo row per band edge) and none crosses HBM.
// Every value takes the two kernels' operations in their order: the io is BIT-IDENTICAL to the
// two-launch path (tests/test_gpu_stem.py).
#include "conv_epi.h"

namespace rtdm {

namespace {
constexpr int kSbFR = 12;            // frame ring rows
constexpr int kSbPR = 6;             // P0 ring rows
constexpr int kSbPS = 16;            // P0 pixel stride (halfs): the 16 channels, unpadded -- conflict-free for
                                     // conv2's ds_read_b128 lane groups (see the conv2 loop)
constexpr int kSbFC0 = 4;            // frame ring column of frame pixel 0 (left pad 4: 32-B aligned item stores)
constexpr int kSbNQ = 18, kSbNKS = 5;  // conv2: 8-channel groups in K (9 taps x 2), 32-deep k-steps

__device__ __forceinline__ uint32_t sb_pack_h2(float a, float b) {
  const _Float16 ha = (_Float16)a, hb = (_Float16)b;
  return (uint32_t)__builtin_bit_cast(uint16_t, ha) | ((uint32_t)__builtin_bit_cast(uint16_t, hb) << 16);
}
__device__ __forceinline__ float sb_dpp_xor1(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0xB1, 0xF, 0xF, true));
}
}  // namespace

// frame ring: kSbFR rows x fcols uint2 pixels (column = x + kSbFC0); P0 ring: kSbPR rows x pcols
// pixels x kSbPS halfs (column = x + 1)
__host__ __device__ inline int sb_fcols(int W) { return W + 12; }
__host__ __device__ inline int sb_pcols(int W1) { return (W1 + 15) / 16 * 16 + 2; }
static inline size_t sb_lds_bytes(int W) {
  return (size_t)kSbFR * sb_fcols(W) * 8 + (size_t)kSbPR * sb_pcols(W / 2) * kSbPS * 2;
}

// a0: the pooled stem (frame u8, Cin 3 -> 16, 3x3/s1/p1, lean epilogue); a2: the conv reading its
// pooled map (Cin 16 -> 32, 3x3/s1/p1, pooled output only).  nb: bands per image.
// WAVES waves a workgroup; ITEMS frame items (4 pixels = 12 bytes) per thread per phase
template <int WAVES, int ITEMS, int DIAG = 0>
__global__ __launch_bounds__(64 * WAVES, 1) void conv_stem_band(ConvArgs a0, ConvArgs a2, int nb) {
  constexpr int kSbWaves = WAVES, kSbNT = 64 * WAVES, kSbItems = ITEMS;
  extern __shared__ __attribute__((aligned(16))) unsigned char sb_lds[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);  // (wave-uniform: the walks below are scalar)
  const int p = lane & 15, g = lane >> 4;
  const int H = a0.ih, W = a0.iw;                  // frame
  const int H1 = a0.oh >> 1, W1 = a0.ow >> 1;      // P0
  const int QH = a2.oh >> 1, QW = a2.ow >> 1;      // P2
  const int fcols = sb_fcols(W), pcols = sb_pcols(W1);
  uint2* const fr = reinterpret_cast<uint2*>(sb_lds);
  _Float16* const pr = reinterpret_cast<_Float16*>(sb_lds + (size_t)kSbFR * fcols * 8);
  const int n = blockIdx.x / nb, band = blockIdx.x - n * nb;
  const int r0 = (int)((int64_t)band * QH / nb), r1 = (int)((int64_t)(band + 1) * QH / nb);

  // ---- zero both rings once: the pad columns stay zero (the padding of both convs) ----
  for (int i = tid; i < kSbFR * fcols; i += kSbNT) fr[i] = make_uint2(0u, 0u);
  for (int i = tid; i < kSbPR * pcols * kSbPS / 8; i += kSbNT) reinterpret_cast<u32x4*>(pr)[i] = u32x4{0u, 0u, 0u, 0u};

  // ---- per-lane constants ----
  // stem (conv_stem3 pooled layout: B = weights, channel p, K group g)
  const _Float16* w0p = (const _Float16*)a0.w_stem + (size_t)p * 64 + 8 * g;
  const h8 wa0 = *(const h8*)w0p;
  typedef _Float16 h4s __attribute__((ext_vector_type(4)));
  const h4s w16 = *(const h4s*)((const _Float16*)a0.w_stem + (size_t)p * 64 + 32 + 4 * g);
  const float bias0 = a0.e.bias ? a0.e.bias[p] : 0.f;
  const float slp0 = a0.e.act == ACT_LEAKY ? a0.e.slope : 1.f;
  constexpr float in_scale = 1.f / 255.f;
  // stem lane geometry (conv_stem3's pooled layout): MFMA row p = pre-pool pixel (quad p >> 2,
  // dx = p & 1, dy = (p >> 1) & 1), K group g = (kh0 = g >> 1, pixel pair g & 1) for the 32-deep
  // link (taps kh 0, 1) and kw = g for the 16-deep one (kh 2).  Frame ring column = x + 1.
  const int sx = 2 * (p >> 2) + (p & 1);
  const int lrow_a = ((p >> 1) & 1) + (g >> 1), lrow_k = ((p >> 1) & 1) + 2;  // frame row - (4k + 1), less 2 rp
  const int lx_a = (sx + 2 * (g & 1) + kSbFC0 - 1) * 8, lx_k = (sx + g + kSbFC0 - 1) * 8;  // column bytes (tile 0)
  const int lp_out = (g + 1) * kSbPS + p;                                       // P0 ring: pixel 4 tile + g, channel p
  // conv2 (conv3_pool_small<16,32> layout: A = weights, channel 16t + p, K group g)
  h8 wf[kSbNKS][2];
#pragma unroll
  for (int s = 0; s < kSbNKS; ++s)
#pragma unroll
    for (int t = 0; t < 2; ++t)
      wf[s][t] = *(const h8*)((const _Float16*)a2.w + (size_t)(16 * t + p) * a2.kpad + 8 * (4 * s + g));
  int kh_s[kSbNKS], kofs_s[kSbNKS];  // per k-step: the tap row and the in-row offset (halfs)
#pragma unroll
  for (int s = 0; s < kSbNKS; ++s) {
    int q = 4 * s + g;
    q = q < kSbNQ ? q : kSbNQ - 1;  // (zero weights past K: any valid pixel)
    const int tap = q >> 1, cg = q & 1, kh = tap / 3, kw = tap - kh * 3;
    kh_s[s] = kh;
    kofs_s[s] = (p + kw) * kSbPS + cg * 8;
  }
  float bias2[2][4];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) bias2[t][r] = a2.e.bias ? a2.e.bias[16 * t + 4 * g + r] : 0.f;
  const float slp2 = a2.e.act == ACT_LEAKY ? a2.e.slope : 1.f;
  const Epilogue& e2 = a2.e;

  // ---- frame rows: phase k's stem reads frame rows 4k+1 .. 4k+6; rows 4k+3 .. 4k+6 are new ----
  const int gpr = W >> 2;  // 4-pixel items per row
  const uint8_t* frame = (const uint8_t*)a0.in + (size_t)n * H * W * 3;
  uint32_t fd[kSbItems][3];
  auto fload = [&](int y0, int rows) {  // items of frame rows y0 .. y0 + rows - 1 -> registers
#pragma unroll
    for (int k = 0; k < kSbItems; ++k) {
      const int i = tid + kSbNT * k, r = i / gpr, y = y0 + r;
      fd[k][0] = fd[k][1] = fd[k][2] = 0u;
      if (r < rows && (unsigned)y < (unsigned)H) {
        const uint32_t* src = (const uint32_t*)(frame + ((size_t)y * W + 4 * (i - r * gpr)) * 3);
        fd[k][0] = src[0];
        fd[k][1] = src[1];
        fd[k][2] = src[2];
      }
    }
  };
  auto fstore = [&](int y0, int rows) {  // registers -> frame ring (zero rows outside the frame)
#pragma unroll
    for (int k = 0; k < kSbItems; ++k) {
      const int i = tid + kSbNT * k, r = i / gpr;
      if (r < rows) {
        const int y = y0 + r, gi = i - r * gpr;
        uint2* dst = fr + (size_t)(((y % kSbFR) + kSbFR) % kSbFR) * fcols + 4 * gi + kSbFC0;
        const uint32_t d0 = fd[k][0], d1 = fd[k][1], d2 = fd[k][2];
        const uint32_t b[12] = {d0 & 255u, (d0 >> 8) & 255u, (d0 >> 16) & 255u, d0 >> 24,
                                d1 & 255u, (d1 >> 8) & 255u, (d1 >> 16) & 255u, d1 >> 24,
                                d2 & 255u, (d2 >> 8) & 255u, (d2 >> 16) & 255u, d2 >> 24};
        uint32_t px[8];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          px[2 * q] = sb_pack_h2((float)b[3 * q], (float)b[3 * q + 1]);
          px[2 * q + 1] = sb_pack_h2((float)b[3 * q + 2], 0.f);
        }
        reinterpret_cast<u32x4*>(dst)[0] = u32x4{px[0], px[1], px[2], px[3]};  // (2-way ds_write_b128 vs 4-way b64)
        reinterpret_cast<u32x4*>(dst)[1] = u32x4{px[4], px[5], px[6], px[7]};
      }
    }
  };
  // prologue: phase r0 - 1 needs frame rows 4r0 - 3 .. 4r0 + 2 (6 rows), phase r0 rows 4r0 + 3 .. 4r0 + 6
  __syncthreads();
  for (int y0 = 4 * r0 - 3; y0 < 4 * r0 + 7; y0 += 4) {  // (3 passes of up to 4 rows)
    const int rows = 4 * r0 + 7 - y0 < 4 ? 4 * r0 + 7 - y0 : 4;
    fload(y0, rows);
    fstore(y0, rows);
  }
  if (r0 + 1 <= r1 - 1) fload(4 * (r0 + 1) + 3, 4);  // phase r0 + 1's new rows, in flight
  __syncthreads();

  // ---- work split per phase: conv tasks (P2 row, 16-pixel column tile: 20 MFMAs) round robin;
  //      stem tasks (P0 row, 4-quad tile: 2 MFMAs) spread so every wave has about as many
  //      MFMAs ----
  const int ctiles = (a2.ow + 15) >> 4;       // conv2 column tiles of a row
  const int stiles = (W1 + 3) >> 2;           // stem tiles of a P0 row
  // stem units (per wave) so that 10 x conv + stem is level: cumulative split of 2 * stiles
  int sbeg, send;
  {
    const int tot = 2 * stiles + 10 * ctiles;  // MFMA pairs per phase
    int acc_c = 0, acc_s = 0;
    sbeg = send = 0;
    for (int w = 0; w < kSbWaves; ++w) {
      const int nc = ctiles / kSbWaves + (w < ctiles % kSbWaves ? 1 : 0);
      acc_c += nc;
      int want = (int)(((int64_t)(w + 1) * tot) / kSbWaves) - 10 * acc_c;  // stem units up to wave w
      want = want < acc_s ? acc_s : want > 2 * stiles ? 2 * stiles : want;
      if (w == kSbWaves - 1) want = 2 * stiles;
      if (w == wid) {
        sbeg = acc_s;
        send = want;
      }
      acc_s = want;
    }
  }

  for (int k = r0 - 1; k <= r1; ++k) {
    // frame rows of phase k + 1 (loaded during phase k - 1) into the ring; phase k + 2's in flight
    if (k + 1 >= r0 + 1 && k + 1 <= r1 - 1) {
      fstore(4 * (k + 1) + 3, 4);
      if (k + 2 <= r1 - 1) fload(4 * (k + 2) + 3, 4);
    }
    // ---- stem: P0 rows 2k+1, 2k+2 (row pair rp 0 / 1, 4-quad tiles).  Per phase each lane
    //      computes its two frame-ring bases per row pair (frame rows 4k+1 .. 4k+6 sit in ring
    //      slots fs0 + 0..5 mod kSbFR); a unit then adds only its tile offset.  SU independent
    //      LDS -> MFMA -> epilogue chains per iteration ----
    if (k <= r1 - 1) {
      constexpr int SU = DIAG == 2 ? 8 : 4;
      // the pixel pair as two ds_read_b64 (2 LDS cycles each, 64 banks), not one ds_read2_b64
      // (8 cycles, 32 banks): an offset the compiler cannot see keeps it from merging them
      int off8 = 8;
      asm volatile("" : "+v"(off8));
      const int fs0 = ((4 * k + 1) % kSbFR + kSbFR) % kSbFR;
#pragma unroll
      for (int rp = 0; rp < 2; ++rp) {
        const int tb = max(sbeg - rp * stiles, 0), te = min(send - rp * stiles, stiles);  // this wave's tiles
        if (tb >= te) continue;
        int sa = fs0 + 2 * rp + lrow_a, sk = fs0 + 2 * rp + lrow_k;
        sa -= sa >= kSbFR ? kSbFR : 0;
        sk -= sk >= kSbFR ? kSbFR : 0;
        const int base_a = sa * fcols * 8 + lx_a, base_k = sk * fcols * 8 + lx_k;  // LDS bytes
        const int i = 2 * k + 1 + rp;  // P0 row
        const bool live = i >= 0 && i < H1;
        int ps = i % kSbPR;
        ps += ps < 0 ? kSbPR : 0;
        _Float16* const pdst = pr + (size_t)ps * pcols * kSbPS + lp_out;
        for (int t0 = tb; t0 < te; t0 += SU) {
          h8 bf0[SU];
          h4s bk[SU];
          f4 acc[SU];
#pragma unroll
          for (int v = 0; v < SU; ++v) {
            const int tt = min(t0 + v, te - 1);  // (past the range: recompute the last tile, never stored)
            const unsigned char* fa = sb_lds + base_a + tt * 64;
            const uint2 b00 = *(const uint2*)fa, b01 = *(const uint2*)(fa + off8);
            bf0[v] = __builtin_bit_cast(h8, (u32x4{b00.x, b00.y, b01.x, b01.y}));
            bk[v] = __builtin_bit_cast(h4s, *(const uint2*)(sb_lds + base_k + tt * 64));
          }
#pragma unroll
          for (int v = 0; v < SU; ++v)
            acc[v] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bf0[v], wa0, f4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
          mfma_opcode_switch();
#pragma unroll
          for (int v = 0; v < SU; ++v) acc[v] = __builtin_amdgcn_mfma_f32_16x16x16f16(bk[v], w16, acc[v], 0, 0, 0);
#pragma unroll
          for (int v = 0; v < SU; ++v) {
            if (t0 + v >= te) break;
            float m = 0.f;
            if (live) {  // (rows outside the map: zeros, the padding conv2 reads)
              const float x = fmaxf(fmaxf(acc[v][0], acc[v][1]), fmaxf(acc[v][2], acc[v][3])) * in_scale + bias0;
              m = fmaxf(x, x * slp0) + 0.f;
            }
            // columns past the map: zero (conv2's right padding)
            pdst[(size_t)(t0 + v) * 4 * kSbPS] = (_Float16)(4 * (t0 + v) + g < W1 ? m : 0.f);
          }
        }
      }
    }
    // ---- conv2: P2 row k - 1 from P0 rows 2k-3 .. 2k (ring slots ps0 + 0..3, mod kSbPR) ----
    const int rc = k - 1;
    if (rc >= r0) {
      int ps0 = (2 * rc - 1) % kSbPR;  // slot of P0 row 2rc - 1 (output row 2rc, kh = 0)
      ps0 += ps0 < 0 ? kSbPR : 0;
      const _Float16* rowp[kSbNKS][2];  // per k-step and output row: this lane's tap pointer (column tile 0)
#pragma unroll
      for (int s = 0; s < kSbNKS; ++s)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          int sl = ps0 + j + kh_s[s];
          sl -= sl >= kSbPR ? kSbPR : 0;
          rowp[s][j] = pr + (size_t)sl * pcols * kSbPS + kofs_s[s];
        }
      for (int ct = wid; ct < ctiles; ct += kSbWaves) {
        f4 acc[2][2];
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int t = 0; t < 2; ++t) acc[j][t] = f4{0.f, 0.f, 0.f, 0.f};
        h8 bv[kSbNKS][2];  // every operand in flight before the first MFMA
#pragma unroll
        for (int s = 0; s < kSbNKS; ++s)
#pragma unroll
          for (int j = 0; j < 2; ++j) bv[s][j] = *(const h8*)(rowp[s][j] + ct * 16 * kSbPS);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int s = 0; s < kSbNKS; ++s)
#pragma unroll
          for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int t = 0; t < 2; ++t) acc[j][t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wf[s][t], bv[s][j], acc[j][t], 0, 0, 0);
        // pooled epilogue (conv3_pool_small's): lane = pixel column, channels 16t + 4g + r
        const int px = (ct * 16 + p) >> 1;
        const bool st = (p & 1) == 0 && px < QW && rc < QH;
        _Float16* const prow = (_Float16*)e2.pool.ptr + e2.pool.co + 4 * g + ((size_t)(n * QH + rc) * QW + px) * e2.pool.cs;
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          float m[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float t2 = fmaxf(acc[0][t][r], acc[1][t][r]);
            const float x = fmaxf(t2, sb_dpp_xor1(t2)) + bias2[t][r];
            m[r] = fmaxf(x, x * slp2);
          }
          if (st) *(uint2*)(prow + 16 * t) = make_uint2(sb_pack_h2(m[0], m[1]), sb_pack_h2(m[2], m[3]));
        }
      }
    }
    if constexpr (DIAG != 1) __syncthreads();  // (DIAG 1: no phase barrier -- timing only, wrong io)
  }
}

bool stem_band_ok(const ConvArgs& a0, const ConvArgs& a2) {
  if (a0.in_kind != IN_FRAME_U8 || !a0.w_stem || a0.cin != 3 || a0.ks != 3 || a0.stride != 1 || a0.pad != 1) return false;
  if (a0.cout != 16 || a0.cout_pad != 16 || !a0.quad || !a0.e.pool.ptr || a0.e.full.ptr || a0.e.scale) return false;
  if (a0.e.act == ACT_SWISH || (a0.e.act == ACT_LEAKY && !(a0.e.slope > 0.f && a0.e.slope <= 1.f))) return false;
  if (a0.oh != a0.ih || a0.ow != a0.iw || ((a0.ih | a0.iw) & 3)) return false;  // W % 4 (frame items), H1, W1 even
  if (a2.in_kind != IN_NHWC || a2.cin != 16 || a2.cout != 32 || a2.cout_pad != 32 || a2.ks != 3 || a2.stride != 1 ||
      a2.pad != 1 || a2.w_f32)
    return false;
  if (a2.ih != (a0.oh >> 1) || a2.iw != (a0.ow >> 1) || a2.oh != a2.ih || a2.ow != a2.iw) return false;
  if (!a2.e.pool.ptr || a2.e.full.ptr || a2.e.up.ptr || a2.e.res.ptr || a2.e.io || a2.e.scale || a2.e.act == ACT_SWISH)
    return false;
  if (a2.e.act == ACT_LEAKY && !(a2.e.slope > 0.f && a2.e.slope <= 1.f)) return false;
  if ((a2.e.pool.cs | a2.e.pool.co) & 3) return false;
  if (a2.kpad < 32 * kSbNKS) return false;
  if (a0.iw > 2 * 512) return false;  // 4 rows of 4-pixel items per pass: 2 items x 512 threads
  return sb_lds_bytes(a0.iw) <= 160 * 1024;
}

void launch_stem_band(const ConvArgs& a0, const ConvArgs& a2, hipStream_t s) {
  RTDM_REQUIRE(stem_band_ok(a0, a2), RTDM_E_INVALID, "conv_stem_band: unsupported layer pair");
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1)
    cus = 256;
  const int QH = a2.oh >> 1;
  // bands per image: one workgroup per CU over the batch, at least 4 P2 rows a band
  int nb = (cus + a0.n - 1) / a0.n;
  nb = std::max(1, std::min(nb, QH / 4));
  const int64_t blocks = (int64_t)a0.n * nb;
  RTDM_REQUIRE(blocks < (1ll << 31), RTDM_E_CAPACITY, "conv_stem_band: grid too large");
  const size_t lds = sb_lds_bytes(a0.iw);
  const int waves = tune().stem_fuse == 3 ? 16 : tune().stem_fuse == 2 ? 12 : 8;
  if (waves == 16 && a0.iw <= 768)
    hipLaunchKernelGGL((conv_stem_band<12, 1, 2>), dim3((unsigned)blocks), dim3(768), lds, s, a0, a2, nb);
  else if (waves == 12 && a0.iw <= 768)
    hipLaunchKernelGGL((conv_stem_band<12, 1>), dim3((unsigned)blocks), dim3(768), lds, s, a0, a2, nb);
  else
    hipLaunchKernelGGL((conv_stem_band<8, 2>), dim3((unsigned)blocks), dim3(512), lds, s, a0, a2, nb);
  RTDM_HIP(hipGetLastError());
}

}  // namespace rtdm
