// Wide-tile fp16 implicit-GEMM convolution for the big 3x3 / s1 Darknet layers
// (yolov4-tiny@608 L10 / L12 / L14 / L21, the Darknet-53 3x3 residual convs): the same
// window-mode data path as conv_pipew (conv_pipe.hip), on 256 x 256 output tiles.
//
//   tile        256 pixels x 256 output channels, K-blocks of 64 (one tap of one 64-channel
//               block), channel-block-outer K order: every output is the same fp32 dot product
//               in the same order as conv_pipe's, so the results are bit-identical to it.
//   waves       8 = 4 (M) x 2 (N), each 64 pixels x 128 channels: FM x FN = 4 x 8 accumulators
//               of v_mfma_f32_16x16x32_f16 (128 registers), operands swapped (weights as A) so a
//               lane's accumulator holds 4 consecutive channels of one pixel (register epilogue).
//               Per K-block and wave: 64 MFMAs on 24 ds_read_b128 (conv_pipe's 64 x 64 waves:
//               32 on 16), i.e. 3/4 of the LDS read bytes per FLOP and half the barriers.
//   fragments   one rolling set: the 8 weight fragments of the next half K-block are read into
//               the registers of the current ones as each is consumed (4 MFMAs each), the 4
//               activation fragments into a second set: 64 fragment registers, not 96.
//   LDS         two window buffers (channel blocks alternate) of 336 rows x 64 channels: per
//               channel block the tile's input rows m0 - W - 1 .. m0 + 256 + W sit in LDS once,
//               the 9 taps read shifted views (out-of-image taps read a zero area); a 2-stage
//               weight ring of 256 x 64 (32 KB each).  150 KB in all.  With 64 MFMAs per wave
//               per K-block (~2,000 SIMD cycles) one stage of look-ahead covers the LDS-DMA
//               latency: K-block s + 1's loads fly during the half K-blocks s - 1 / 2 and s / 1.
//   loads       buffer_load ... lds (LDS-DMA): per K-block 4 weight ops + at most 1 window op per
//               thread (the next channel block's window, one 64-row slice per tap 0..5).
//   walk        persistent, one workgroup per CU over a contiguous run of its XCD's tiles.
//
// Replaces the same reference op as conv_pipe (victim_localization/yolov3/models.py:23-44 conv
// + BN + LeakyReLU as run by Darknet.forward :345-347; the fused shortcut of :349-354).
#include "conv_epi.h"

#include <type_traits>
#include <utility>

namespace rtdm {

namespace {
constexpr int kWM = 256, kWN = 256, kWK = 64;  // tile rows (pixels), columns (channels), K-block
constexpr int kWRows = 336;                     // window rows per buffer: 256 + 2W + 2 <= 336 (W <= 39)
constexpr int kWWin = kWRows * kWK * 2;         // bytes per window buffer
constexpr int kWB = kWN * kWK * 2;              // bytes per weight stage
constexpr int kWOffB = 2 * kWWin;               // weight ring
constexpr int kWOffZ = kWOffB + 2 * kWB;        // 1 KB zero area (out-of-image taps)
constexpr int kWOffJ = kWOffZ + 1024;           // 1 KB junk area (window rows past kWRows)
constexpr int kWSmem = kWOffJ + 1024;
static_assert(kWSmem <= 163840, "wide-tile LDS");
static_assert(kWRows % 8 == 0, "a wave's 8-row DMA block is wholly inside or past the window");

// acc += A x B on v_mfma_f32_16x16x32_f16 with the accumulator tied to AGPRs: the 128
// accumulator registers of a wave stay in the AGPR half of the register file, in place (the
// builtin's VGPR-form MFMAs left the register allocator renaming and copying accumulators
// around the K-loop, with the fragments and addresses spilled to scratch).  The asm is
// volatile, so the MFMAs keep program order; its inputs are waited on (lgkmcnt) by the
// compiler like any use of a ds_read result.
__device__ __forceinline__ void mfma_a(f4& acc, const h8& a, const h8& b) {
  asm volatile("v_mfma_f32_16x16x32_f16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
}

template <class F, int... I>
__device__ __forceinline__ void wunroll(F&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
}  // namespace

// One 256 x 256 output tile.  RES: the fused shortcut add (ABL 896).
// DG (diagnostics, wrong outputs): 1 no in-loop weight loads, 2 no in-loop window loads
template <bool RES, int DG = 0>
__device__ __forceinline__ void wide_tile(const ConvArgs& a, unsigned char* smem, int tile) {
  constexpr int FM = 4, FN = 8;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid >> 1, wn = wid & 1;
  const int fr = lane & 15, g = lane >> 4, slot = lane & 7;
  const int nbn = (a.cout_pad + kWN - 1) / kWN;
  const int mt = tile / nbn;
  const int m_base = mt * kWM, n_base = (tile - mt * nbn) * kWN;
  const int W = a.iw;
  const int wr = kWM + 2 * W + 2;  // window rows used
  const int ncb = a.cin / kWK;

  typedef __attribute__((address_space(3))) char lds_char;
  lds_char* const lds0 = (lds_char*)(lds_ptr_t)smem;
  const char* in = (const char*)a.in + (size_t)a.in_co * 2;
  const int in_bytes = (int)(((int64_t)a.n * a.ih * a.iw * a.in_cs - a.in_co) * 2);  // < 2^30 (conv_wide_ok)
  const __amdgpu_buffer_rsrc_t rs_in = __builtin_amdgcn_make_buffer_rsrc((void*)in, 0, in_bytes, 0x00020000);
  // rows past cout_pad read as zeros (out of the buffer's range)
  const __amdgpu_buffer_rsrc_t rs_w =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.w, 0, a.cout_pad * a.kpad * 2, 0x00020000);

  // ---- staging (LDS-DMA).  Weight op j of wave w fills stage rows 32w + 8j + lane/8; window
  //      slice j of wave w rows 64j + 8w + lane/8.  LDS slot lane%8 of a row holds k-vector
  //      slot ^ (row & 7) (applied on the source side; the reads apply the same involution). ----
  // (rows 8j apart share the swizzle: op j = op 0 + j * 16 * kpad bytes, a scalar offset)
  const int voff_b = (32 * wid + (lane >> 3)) * a.kpad * 2 + 16 * (slot ^ (lane >> 3));
  const int koff_n = n_base * a.kpad * 2;  // the tile's weight panel
  const int wrow0 = 8 * wid + (lane >> 3);
  const int wv0 = (m_base - W - 1 + wrow0) * a.in_cs * 2 + 16 * (slot ^ (wrow0 & 7));
  // weight columns of K-block (channel block cb, tap t) into ring stage st
  // Opaque per-body copies (Z: asm the compiler cannot see through, fresh in every K-block body)
  // of the layer constants the per-tap values derive from (the tap shifts, weight-column and
  // window-slice offsets, tap-validity masks): otherwise the compiler precomputes those values
  // for all 9 taps / 6 slices ahead of the channel-block loop, and they do not fit the registers
  // (spilled, their scratch reloads' vmcnt(0) drain the LDS-DMA pipeline).
  struct Z {
    int cin, in_cs, w, z, wv;  // wv: the window source offset wv0 (per lane)
  };
  auto stage_b1 = [&](int cb, int t, int st, const Z& z, int j) {  // weight op j
    const int koff = koff_n + (t * z.cin + cb * kWK + j * 8 * a.kpad) * 2;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs_w, (lds_ptr_t)(lds0 + kWOffB + st * kWB + (32 * wid + 8 * j) * 128), 16,
                                             voff_b, koff, 0, 0);
  };
  auto stage_b = [&](int cb, int t, int st, const Z& z) {
#pragma unroll
    for (int j = 0; j < 4; ++j) stage_b1(cb, t, st, z, j);
  };
  // window slice j of channel block cw.  Rows before / past the batch are out of the buffer's
  // range (zeros: negative offsets wrap past 2^31 > in_bytes); a slice wholly past the window
  // is pushed out of range by 2^31; rows past kWRows go to the junk area.
  auto stage_w = [&](int j, int cw, const Z& z) {
    const int r0 = 64 * j + 8 * wid;
    const int dofs = r0 < kWRows ? (cw & 1) * kWWin + r0 * 128 : kWOffJ;
    const uint32_t so = (uint32_t)((64 * j * z.in_cs + cw * kWK) * 2) + (64 * j < wr ? 0u : 0x80000000u);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs_in, (lds_ptr_t)(lds0 + dofs), 16, (int)((uint32_t)z.wv + so), 0, 0, 0);
  };

  // ---- read side.  Activation fragment tm of tap (KH, KW): window row wm*64 + tm*16 + fr + sh
  //      (sh = KH*W + KW), slot (4h + g) ^ (row & 7); an out-of-image tap reads the zero area.
  //      Half 1 = half 0 ^ 64 (row bases are multiples of 128).  Weight fragment tn: stage row
  //      wn*128 + tn*16 + fr, immediates 2048 tn. ----
  uint32_t amask[FM];  // (packed below: tm 0 / 1 in the halves of am01, 2 / 3 of am23)
#pragma unroll
  for (int tm = 0; tm < FM; ++tm) {
    const int m = m_base + wm * 64 + tm * 16 + fr;
    uint32_t msk = 0;
    if (m < a.M) {
      int n, oy, ox;
      row_to_pix(a, m, n, oy, ox);
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const int kh = t / 3, kw = t % 3;
        if ((unsigned)(oy + kh - 1) < (unsigned)a.ih && (unsigned)(ox + kw - 1) < (unsigned)a.iw) msk |= 1u << t;
      }
    }
    amask[tm] = msk;
  }
  const uint32_t am[2] = {amask[0] | (amask[1] << 16), amask[2] | (amask[3] << 16)};
  uint32_t wtab = 0;  // g ^ ((fr + r) & 7) for r = 0..7, 3 bits each
#pragma unroll
  for (int r = 0; r < 8; ++r) wtab |= (uint32_t)((g ^ ((fr + r) & 7)) & 7) << (3 * r);
  const int lrow = (wm * 64 + fr) * 128;
  const int boff0 = kWOffB + (wn * 128 + fr) * 128 + 16 * (g ^ (fr & 7));
  int aoff[FM];
  auto waddr = [&](auto tt_, int par, const Z& z) {
    constexpr int TT = decltype(tt_)::value, KH = TT / 3, KW = TT % 3;
    const int sh = KH * z.w + KW;
    const int off = lrow + par * kWWin + (sh << 7) + (int)(((wtab >> (3 * (sh & 7))) & 7u) << 4);
#pragma unroll
    for (int tm = 0; tm < FM; ++tm) {
      const bool valid = (am[tm >> 1] >> (TT + 16 * (tm & 1) + z.z)) & 1u;  // tap TT valid for this row
      aoff[tm] = valid ? off + tm * 2048 : kWOffZ;
    }
  };

  f4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
  h8 fa0[FM], fa1[FM], fb[FN];
  auto rd = [&](int off) { return *(const h8*)(smem + off); };
  f4 rb[FN];  // register-epilogue bias (loaded in the last K-block)

  // ---- prologue: channel block 0's window, K-blocks 0 / 1 into stages 0 / 1 ----
  const Z z0{a.cin, a.in_cs, W, 0, wv0};
#pragma unroll
  for (int j = 0; j < 6; ++j) stage_w(j, 0, z0);
  stage_b(0, 0, 0, z0);
  stage_b(0, 1, 1, z0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
  waddr(std::integral_constant<int, 0>{}, 0, z0);
#pragma unroll
  for (int tm = 0; tm < FM; ++tm) fa0[tm] = rd(aoff[tm]);
#pragma unroll
  for (int tn = 0; tn < FN; ++tn) fb[tn] = rd(boff0 + tn * 2048);  // (prologue: once per tile)

  // ---- K-block s = 9 cb + T (T a compile-time constant).  Phase 1: the MFMAs of half 0 (fa0,
  //      fb) with the reads of half 1 (fa1, fb rolling).  Then: retire K-block s + 1's loads
  //      (every wave's vmcnt(0) + the barrier; lgkmcnt(0): this stage's reads are done before any
  //      wave restages it), issue K-block s + 2's loads into this stage (and slice T of channel
  //      block cb + 1's window), phase 2: the MFMAs of half 1 (fa1, fb) with the reads of half 0
  //      of s + 1 (fa0, fb rolling).  Each accumulator sees K-blocks in order, half 0 before half
  //      1, as conv_pipe's: bit-identical. ----
  auto body = [&](auto t_, auto stg_, auto wop_, auto nxt_, int cb) {
    constexpr int T = decltype(t_)::value;
    constexpr bool STG = decltype(stg_)::value, WOP = decltype(wop_)::value, NXT = decltype(nxt_)::value;
    const int bs = ((cb + T) & 1) * kWB;  // this K-block's stage (and K-block s + 2's)
    Z z{a.cin, a.in_cs, W, 0, wv0};
    asm volatile("" : "+s"(z.cin), "+s"(z.in_cs), "+s"(z.w), "+s"(z.z), "+v"(z.wv));
    // phase 1.  Each group (4 MFMAs on fb[tn], then the read of fb[tn]'s next value into its
    // register) is fenced by sched_barrier: with the MFMAs in program order the rolling reuse of
    // the fragment registers holds (a free scheduler interleaves the groups' MFMAs and then
    // needs both values of every fb[tn] at once, and renames the accumulators)
    // this body's weight-fragment base (opaque: the 8 fragments are then one address register
    // plus ds_read immediates, not 8 precomputed addresses)
    int bh1 = (boff0 + bs) ^ 64;
    asm volatile("" : "+v"(bh1));
#pragma unroll
    for (int tm = 0; tm < FM; ++tm) fa1[tm] = rd(aoff[tm] ^ 64);
#pragma unroll
    for (int tn = 0; tn < FN; ++tn) {
#pragma unroll
      for (int tm = 0; tm < FM; ++tm)
        mfma_a(acc[tm][tn], fb[tn], fa0[tm]);
      fb[tn] = rd(bh1 + tn * 2048);
      __builtin_amdgcn_sched_barrier(0);
    }
    if constexpr (!NXT) {  // the tile's last K-block
      const __amdgpu_buffer_rsrc_t rs_bias =
          __builtin_amdgcn_make_buffer_rsrc((void*)a.e.bias, 0, a.cout * 4, 0x00020000);
#pragma unroll
      for (int tn = 0; tn < FN; ++tn) {
        const int c0 = n_base + wn * 128 + tn * 16 + 4 * g;  // out-of-range channels load zeros
        rb[tn] = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(rs_bias, c0 * 4, 0, 0));
      }
#pragma unroll
      for (int tn = 0; tn < FN; ++tn) {
#pragma unroll
        for (int tm = 0; tm < FM; ++tm)
          mfma_a(acc[tm][tn], fb[tn], fa1[tm]);
        __builtin_amdgcn_sched_barrier(0);
      }
      return;
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    // phase 2: the LDS-DMA ops of K-block s + 2 one per MFMA group
    waddr(std::integral_constant<int, (T + 1) % 9>{}, (cb + (T == 8 ? 1 : 0)) & 1, z);
    int bh0 = boff0 + ((cb + T + 1) & 1) * kWB;  // K-block s + 1's stage
    asm volatile("" : "+v"(bh0));
#pragma unroll
    for (int tm = 0; tm < FM; ++tm) fa0[tm] = rd(aoff[tm]);
    constexpr int T2 = (T + 2) % 9;
    const int cb2 = cb + (T >= 7 ? 1 : 0);
#pragma unroll
    for (int tn = 0; tn < FN; ++tn) {
#pragma unroll
      for (int tm = 0; tm < FM; ++tm)
        mfma_a(acc[tm][tn], fb[tn], fa1[tm]);
      fb[tn] = rd(bh0 + tn * 2048);
      if constexpr (STG) {
        if (!(DG & 1) && tn < 4) stage_b1(cb2, T2, (cb + T) & 1, z, tn);
        if (!(DG & 2) && WOP && tn == 4) stage_w(T, cb + 1, z);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  using T_ = std::true_type;
  using F_ = std::false_type;
  int cb = 0;
  for (; cb < ncb - 1; ++cb)
    wunroll(
        [&](auto t_) {
          constexpr int T = decltype(t_)::value;
          body(t_, T_{}, std::bool_constant<(T * 64 < kWRows)>{}, T_{}, cb);
        },
        std::make_integer_sequence<int, 9>{});
  wunroll(
      [&](auto t_) {
        constexpr int T = decltype(t_)::value;
        body(t_, std::bool_constant<(T <= 6)>{}, F_{}, std::bool_constant<(T <= 7)>{}, cb);
      },
      std::make_integer_sequence<int, 9>{});

  // the epilogue's pixel of each row derives from an opaque copy of m_base: otherwise the
  // compiler reuses the prologue's row_to_pix (the tap masks) and keeps its results live
  // across the K-loop
  int mb = m_base;
  asm volatile("" : "+s"(mb));
  // the last MFMAs' results are read by VALU next: their passes must be complete (the compiler
  // does not see the MFMAs inside the asm, so it inserts no wait states for them)
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
  f4 dq4[1];
  pipe_epi_regs<RES, FM, FN, 64, 128>(a, mb, n_base, wm, wn, lane, acc, rb, dq4);
}

template <int ABL, int DG = 0>
__global__ __launch_bounds__(512, 1) void conv_wide_f16(ConvArgs a, int ntiles) {
  __shared__ __attribute__((aligned(16))) unsigned char smem[kWSmem];
  if (threadIdx.x < 64) reinterpret_cast<u32x4*>(smem + kWOffZ)[threadIdx.x] = u32x4{0u, 0u, 0u, 0u};
  // persistent XCD walk: XCD x (blocks b with b % 8 == x) takes a contiguous run of tiles
  const int nb = gridDim.x, xcd = blockIdx.x & 7, l = blockIdx.x >> 3;
  const int q = ntiles >> 3, r = ntiles & 7;
  const int lo = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  const int hi = lo + q + (xcd < r ? 1 : 0);
  const int bx = (nb - xcd + 7) >> 3;
  for (int t = lo + l; t < hi; t += bx) {
    __syncthreads();  // the previous tile's LDS reads are done (and, first, the zero area is written)
    wide_tile<(ABL & 256) != 0, DG>(a, smem, t);
  }
}

// ---- host side ----
bool conv_wide_ok(const ConvArgs& a, int abl) {
  if (abl != 640 && abl != 896) return false;  // register epilogue (+ fused shortcut) layers
  if (!a.w || a.w_f32 || a.head_w || a.in_kind != IN_NHWC || (a.in_cs | a.in_co) % 8 != 0) return false;
  if (a.ks != 3 || a.stride != 1 || a.pad != 1 || a.quad || a.ih != a.oh || a.iw != a.ow) return false;
  if (a.cin % kWK != 0 || a.kpad != 9 * a.cin || a.cout_pad % 128 != 0) return false;
  if (kWM + 2 * a.iw + 2 > kWRows) return false;
  if ((int64_t)a.n * a.ih * a.iw * a.in_cs * 2 >= (1ll << 30)) return false;  // the window op's 2^31 skip
  if ((int64_t)a.cout_pad * a.kpad * 2 >= (1ll << 31)) return false;
  return true;
}

int64_t conv_wide_tiles(const ConvArgs& a) {
  return (int64_t)((a.M + kWM - 1) / kWM) * ((a.cout_pad + kWN - 1) / kWN);
}

void launch_conv_wide(const ConvArgs& a, int abl, int ntiles, int cus, hipStream_t s) {
  RTDM_REQUIRE(conv_wide_ok(a, abl), RTDM_E_INVALID, "conv_wide: unsupported layer");
  RTDM_REQUIRE(ntiles > 0 && ntiles <= conv_wide_tiles(a), RTDM_E_INVALID, "conv_wide: bad tile count");
  const dim3 grid((unsigned)(ntiles < cus ? ntiles : cus));
  const int dg = tune().pipe_wide >= 10 ? tune().pipe_wide - 10 : 0;  // conv_wide 11 / 12 / 13: ablations
  if (abl == 896)
    hipLaunchKernelGGL((conv_wide_f16<896>), grid, dim3(512), 0, s, a, ntiles);
  else if (dg == 1)
    hipLaunchKernelGGL((conv_wide_f16<640, 1>), grid, dim3(512), 0, s, a, ntiles);
  else if (dg == 2)
    hipLaunchKernelGGL((conv_wide_f16<640, 2>), grid, dim3(512), 0, s, a, ntiles);
  else if (dg == 3)
    hipLaunchKernelGGL((conv_wide_f16<640, 3>), grid, dim3(512), 0, s, a, ntiles);
  else
    hipLaunchKernelGGL((conv_wide_f16<640>), grid, dim3(512), 0, s, a, ntiles);
  RTDM_HIP(hipGetLastError());
}

}  // namespace rtdm
