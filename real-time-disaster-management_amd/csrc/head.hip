// Stand-alone YOLO head conv: the 1x1 conv (Cin % 128 == 0, <= 32 outputs) in front of a
// [yolo] layer whose producer cannot carry it as a fused head (Cin > 128: yolov4-tiny L15 /
// L22, the three yolov3 / yolov3-spp heads), plus the YOLOLayer inference decode into io
// (victim_localization/yolov3/models.py:23-44 conv, :204-258 YOLOLayer, create_grids
// :422-436).
//
// conv_pipe's tile (128 output channels, LDS ring, C tile through LDS, barriers) spent
// most of a head launch in per-tile latency: 28 real columns of 128, 2-8 K-blocks, then
// three barrier-separated epilogue phases.  Here each wave owns 16 * FM rows and all 32
// (padded) head channels and needs no LDS and no barrier: A fragments (8 input channels
// of one pixel per lane) and B fragments (8 K of one head channel) come straight from
// global memory (the weights, 32 x Cin fp16, stay in L1/L2), two 128-deep K chunks in
// flight, v_mfma_f32_16x16x32_f16 in the same K order as conv_pipe (bit-identical
// accumulators), and the decode runs on the accumulators in registers with the same
// per-element operations as epi_io_decode.
#include "conv_epi.h"

namespace rtdm {

namespace {
constexpr int kHeadCh = 4;  // 32-deep K steps per chunk (128 K)
}

// ONE: Cin == 128, one K chunk (no second register set: FM 4 then fits 2 waves per SIMD)
template <int FM, bool ONE = false>
__global__ __launch_bounds__(256) void head1x1_f16(ConvArgs a) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int fr = lane & 15, g = lane >> 4;
  const int m_base = (blockIdx.x * 4 + wid) * (16 * FM);
  if (m_base >= a.M) return;
  const Epilogue& e = a.e;

  // per-lane operand rows: A = pixel m_base + 16 tm + fr (clamped; its outputs are not
  // stored), K slice 8g..8g+7 of each 32-deep step; B = head channel 16 tn + fr
  const _Float16* ap[FM];
#pragma unroll
  for (int tm = 0; tm < FM; ++tm) {
    int m = m_base + tm * 16 + fr;
    m = m < a.M ? m : a.M - 1;
    ap[tm] = (const _Float16*)a.in + (size_t)m * a.in_cs + a.in_co + 8 * g;
  }
  const _Float16* bp[2];
#pragma unroll
  for (int tn = 0; tn < 2; ++tn) bp[tn] = (const _Float16*)a.w + (size_t)(tn * 16 + fr) * a.kpad + 8 * g;

  f4 acc[FM][2];
#pragma unroll
  for (int tm = 0; tm < FM; ++tm)
#pragma unroll
    for (int tn = 0; tn < 2; ++tn) acc[tm][tn] = f4{0.f, 0.f, 0.f, 0.f};

  h8 a0[kHeadCh][FM], b0[kHeadCh][2], a1[ONE ? 1 : kHeadCh][FM], b1[ONE ? 1 : kHeadCh][2];
  auto load = [&](int k0, h8(&A)[kHeadCh][FM], h8(&B)[kHeadCh][2]) {
#pragma unroll
    for (int s = 0; s < kHeadCh; ++s) {
#pragma unroll
      for (int tm = 0; tm < FM; ++tm) A[s][tm] = *(const h8*)(ap[tm] + k0 + 32 * s);
#pragma unroll
      for (int tn = 0; tn < 2; ++tn) B[s][tn] = *(const h8*)(bp[tn] + k0 + 32 * s);
    }
  };
  auto mma = [&](const h8(&A)[kHeadCh][FM], const h8(&B)[kHeadCh][2]) {
#pragma unroll
    for (int s = 0; s < kHeadCh; ++s)
#pragma unroll
      for (int tm = 0; tm < FM; ++tm)
#pragma unroll
        for (int tn = 0; tn < 2; ++tn)
          acc[tm][tn] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A[s][tm], B[s][tn], acc[tm][tn], 0, 0, 0);
  };
  const int K = a.cin, CK = 32 * kHeadCh;
  load(0, a0, b0);
  if constexpr (ONE) {
    (void)a1;
    (void)b1;
    __builtin_amdgcn_sched_barrier(0);  // every load in flight before the first MFMA waits
    mma(a0, b0);
  } else {
    int k0 = 0;
    for (; k0 + 2 * CK <= K; k0 += 2 * CK) {
      load(k0 + CK, a1, b1);
      mma(a0, b0);
      if (k0 + 2 * CK < K) load(k0 + 2 * CK, a0, b0);
      mma(a1, b1);
    }
    if (k0 < K) mma(a0, b0);  // odd chunk count: the last chunk was loaded into a0/b0
  }

  // ---- decode (epi_io_decode's per-element operations) and io stores.  Accumulator
  //      acc[tm][tn][j] = row m_base + 16 tm + 4 g + j, head channel 16 tn + fr. ----
  float bias[2], sc[2], sh[2], anc[2];
  int kk[2], ai[2];
  bool cv[2];
#pragma unroll
  for (int tn = 0; tn < 2; ++tn) {
    const int c = tn * 16 + fr;
    cv[tn] = c < a.cout;
    ai[tn] = c / e.no;
    kk[tn] = c - ai[tn] * e.no;
    bias[tn] = (e.bias && cv[tn]) ? e.bias[c] : 0.f;
    sc[tn] = (e.scale && cv[tn]) ? e.scale[c] : 1.f;
    sh[tn] = (e.scale && cv[tn]) ? e.shift[c] : 0.f;
    anc[tn] = (cv[tn] && !e.raw && (kk[tn] == 2 || kk[tn] == 3)) ? e.anchor_vec[2 * ai[tn] + (kk[tn] - 2)] : 0.f;
  }
  // decoded values -> the wave's LDS tile T[c][px] (px stride 16 FM + 1: a store's 16 channel
  // lanes hit distinct banks), then each anchor plane's 16 FM pixels x no values leave as one
  // contiguous run of io (consecutive lanes, consecutive dwords) instead of 4-byte scatters
  constexpr int PX = 16 * FM, PXS = PX + 1;
  __shared__ float hs_tile[4][32 * PXS];
  float* T = hs_tile[wid];
  // The decode branch is per lane (the head channel k = lane's column) and so divergent
  // across the wave: every path's operations as selects instead, the same operations on the
  // same values per element (xy: rcp(1 + exp(-x)) + grid, wh: exp(x) * anchor, obj / cls:
  // rcp(1 + exp(-x))), bit-identical to epi_io_decode.  A lane's 4 rows j of block tm are
  // consecutive pixels: one row_to_pix per block, row_pix4 for the others.
#pragma unroll
  for (int tm = 0; tm < FM; ++tm) {
    const int r0 = min(m_base + tm * 16 + 4 * g, a.M - 1);
    int n0_, oy0_, ox0_;
    row_to_pix(a, r0, n0_, oy0_, ox0_);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int px = tm * 16 + 4 * g + j;
      int n, oy, ox;
      row_pix4(a, r0, j, n0_, oy0_, ox0_, n, oy, ox);  // (rows past M: any pixel, never stored)
#pragma unroll
      for (int tn = 0; tn < 2; ++tn) {
        if (!cv[tn]) continue;
        float t = acc[tm][tn][j] + bias[tn];
        if (e.act == ACT_LEAKY) t = t > 0.f ? t : t * e.slope;
        const float x = t * sc[tn] + sh[tn];
        const int k = kk[tn];
        float o;
        if (e.raw) {
          o = x;
        } else {
          const bool wh = k == 2 || k == 3;
          const float v = __expf(wh ? x : -x);
          const float s = __frcp_rn(1.f + v);
          o = k < 2 ? (s + (float)(k == 0 ? ox : oy)) * e.ystride : wh ? (v * anc[tn]) * e.ystride : s;
        }
        T[(tn * 16 + fr) * PXS + px] = o;
      }
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  const int rows = min(PX, a.M - m_base), no = e.no, na = a.cout / no;
  const size_t plane = (size_t)a.oh * a.ow;
  int n0, oy0, ox0;
  row_to_pix(a, m_base, n0, oy0, ox0);
  const int p0 = oy0 * a.ow + ox0;
  const bool one_image = p0 + rows <= (int)plane;  // the wave's rows are consecutive pixels of one image
  const int ne = rows * no;
  // el / no by a multiply-shift (exact for el < 2112 and no <= 32, checked host-side in
  // head1x1_ok): a run-time integer division per element was a third of the kernel's VALU
  const uint32_t inv_no = (65536u + (uint32_t)no - 1u) / (uint32_t)no;
  for (int ai = 0; ai < na; ++ai) {
    const float* Ta = T + ai * no * PXS;
    float* dst = e.io + ((size_t)n0 * e.io_rows + e.io_off + (size_t)ai * plane + p0) * no;
    for (int el = lane; el < ne; el += 64) {
      const int px = (int)(((uint32_t)el * inv_no) >> 16), k = el - px * no;
      const float v = Ta[k * PXS + px];
      if (one_image) {
        dst[el] = v;
      } else {
        int n, oy, ox;
        row_to_pix(a, m_base + px, n, oy, ox);
        e.io[((size_t)n * e.io_rows + e.io_off + (size_t)ai * plane + (size_t)oy * a.ow + ox) * no + k] = v;
      }
    }
  }
}

bool head1x1_ok(const ConvArgs& a) {
  return a.ks == 1 && a.stride == 1 && a.pad == 0 && !a.quad && a.in_kind == IN_NHWC && !a.w_f32 && a.w &&
         !a.head_w && epi_io_ok(a) && a.cout >= 1 && a.cout <= 32 && a.cout_pad >= 32 && a.cin % 128 == 0 &&
         a.kpad >= a.cin && (a.in_cs | a.in_co) % 8 == 0 && a.kpad % 8 == 0 && a.ih == a.oh && a.iw == a.ow &&
         a.e.no > 0 && a.e.no <= 32;  // (the store loop's multiply-shift division: rows <= 64, no <= 32)
}

static int head_fm(const ConvArgs& a) {
  static int cus = [] {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v < 1)
      v = 256;
    return v;
  }();
  // more rows per wave once the grid has them to spare: a wave's loads are all issued before
  // its first MFMA, so its bytes in flight (16 FM rows x Cin) set the launch's memory-level
  // parallelism (yolov4-tiny@608 b64 L29, 369664 x 128: FM 2 -> 4)
  if (a.cin == 128 && (a.M + 255) / 256 >= 4 * cus) return 4;
  return (a.M + 127) / 128 >= 2 * cus ? 2 : 1;  // 2 fragments per wave once the grid is >= 2 per CU
}

const char* head1x1_name(const ConvArgs& a) {
  const int fm = head_fm(a);
  return fm == 4 ? "head1x1_f16<4>" : fm == 2 ? "head1x1_f16<2>" : "head1x1_f16<1>";
}

void launch_head1x1(const ConvArgs& a, hipStream_t s) {
  RTDM_REQUIRE(head1x1_ok(a), RTDM_E_INVALID, "head1x1: unsupported layer");
  const int fm = head_fm(a);
  const int64_t blocks = ((int64_t)a.M + 64 * fm - 1) / (64 * fm);
  RTDM_REQUIRE(blocks < (1ll << 31), RTDM_E_CAPACITY, "head1x1: grid too large");
  if (fm == 4)
    hipLaunchKernelGGL((head1x1_f16<4, true>), dim3((unsigned)blocks), dim3(256), 0, s, a);
  else if (fm == 2)
    hipLaunchKernelGGL((head1x1_f16<2>), dim3((unsigned)blocks), dim3(256), 0, s, a);
  else
    hipLaunchKernelGGL((head1x1_f16<1>), dim3((unsigned)blocks), dim3(256), 0, s, a);
  RTDM_HIP(hipGetLastError());
}

}  // namespace rtdm
