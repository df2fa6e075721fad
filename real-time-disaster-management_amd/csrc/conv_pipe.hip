// Pipelined fp16 implicit-GEMM convolution for the MFMA-bound Darknet layers
// (3x3 / 1x1, Cin % 64 == 0): the conv_glds_f16 data path (direct
// global->LDS buffer loads, source-swizzled LDS image, scalar tap cursor) in a
// schedule built for one workgroup per CU.
//
//   tile        BM (pixels) x 128 (output channels), BK = 64; BM = 256, 128 or 64,
//               picked per launch from the tile count (pipe_bm): small per-rank
//               batches (M = 8 frames x 19^2 = 2,888 rows) need the smaller tiles to
//               reach every CU.  Every BM accumulates each output in the same K
//               order, so the results are bit-identical across BM (batch-invariant).
//   waves       8: BM 256 = 4 (M) x 2 (N) waves of 64 x 64 outputs (FM x FN = 4 x 4
//               accumulators of v_mfma_f32_16x16x32_f16); BM 128 = 2 x 4 waves of
//               64 x 32; BM 64 = 2 x 4 waves of 32 x 32.  2 waves per SIMD.
//               (Measured alternative: 4 waves of 128 x 64 — 3/4 of the LDS read
//               bytes per FLOP — ran 30 % slower: one wave per SIMD, and hipcc
//               spills the 128 accumulators into AGPR copy chains in the loop.)
//   LDS         3 stages x 48 KB: loads of K-block kb+2 are issued while kb is
//               multiplied and kb+1 is landing; a counted "s_waitcnt vmcnt(VM)"
//               (VM = buffer->LDS ops per thread per stage) retires kb+1 while
//               kb+2 stays in flight across the one raw s_barrier per K-block
//   fragments   two register sets: the LDS reads of the next half K-block are
//               interleaved with the MFMAs of the current one
//
// Replaces the same reference ops as conv.hip (victim_localization/yolov3/
// models.py:23-44 conv + BN + LeakyReLU as run by Darknet.forward :345-347,
// with the fused epilogues of conv_epi.h).
#include "conv_epi.h"

#include <algorithm>
#include <mutex>
#include <set>
#include <string>
#include <type_traits>
#include <utility>

namespace rtdm {

namespace {
constexpr int kPBN = 128, kPBK = 64, kPNS = 3;
constexpr int kPCstr = kPBN + 4;
// NS: LDS stages (the ring code takes any NS >= 3; deeper rings for the 128- / 64-row
// tiles, 4 x 32 KB / 6 x 24 KB, measured no faster at b8: r02an).
template <int BM>
struct PipeCfg {
  static constexpr int WM = BM == 256 ? 4 : 2, WN = 8 / WM;
  static constexpr int NS = 3;
  static constexpr int Stage = (BM + kPBN) * kPBK;  // halfs per stage
  static constexpr int Smem = NS * Stage * 2 > BM * kPCstr * 4 ? NS * Stage * 2 : BM * kPCstr * 4;
};

// Window mode (3x3 / stride 1 / pad 1, linear row order): per 64-channel block the tile's
// input rows m_base - W - 1 .. m_base + BM + W (BM + 2W + 2 pixels, at most kWinRows) sit
// in LDS once; the 9 taps read shifted views of it.  Layout: two window buffers (channel
// blocks alternate), the 3-stage B ring, a 1 KB zero area (out-of-image taps read it; a
// per-row swizzled 2 KB zero area removes the border reads' bank conflicts but its
// per-K-block address VALU cost more: r02ck).
constexpr int kWinRows = 440;
// + a 1 KB junk area: the tap-unrolled loop's window slice 6 rows past kWinRows land there
constexpr int kWinSmem = (2 * kWinRows * kPBK + kPNS * kPBN * kPBK + 16 * kPBK) * 2;
static_assert(kWinSmem <= 163840, "window LDS");

// s_waitcnt vmcnt(N) lgkmcnt(0), any N < 64 (gfx9 encoding: vmcnt bits 3:0 and 15:14)
template <int N>
__device__ __forceinline__ void wait_vmn_lgkm0() {
  static_assert(N >= 0 && N < 64, "vmcnt");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4));
}
template <int N>
__device__ __forceinline__ void wait_vm_lgkm0() {
  if constexpr (N == 6)
    asm volatile("s_waitcnt vmcnt(6) lgkmcnt(0)" ::: "memory");
  else if constexpr (N == 4)
    asm volatile("s_waitcnt vmcnt(4) lgkmcnt(0)" ::: "memory");
  else if constexpr (N == 3)
    asm volatile("s_waitcnt vmcnt(3) lgkmcnt(0)" ::: "memory");
  else if constexpr (N == 12)
    asm volatile("s_waitcnt vmcnt(12) lgkmcnt(0)" ::: "memory");
  else if constexpr (N == 8)
    asm volatile("s_waitcnt vmcnt(8) lgkmcnt(0)" ::: "memory");
  else if constexpr (N == 2)
    asm volatile("s_waitcnt vmcnt(2) lgkmcnt(0)" ::: "memory");
  else if constexpr (N == 1)
    asm volatile("s_waitcnt vmcnt(1) lgkmcnt(0)" ::: "memory");
  else
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
}
// f(integral_constant<int, I>) for I = 0 .. N-1, unrolled at compile time
template <class F, int... I>
__device__ __forceinline__ void unroll_seq(F&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
}  // namespace

// Fused-head epilogue for the 4 rows m0..m0+3 of head channel c (YOLOLayer
// inference branch, models.py:252-258): bias -> activation -> decode -> io.
// bias / anc: the channel's head bias and (w / h channels) anchor, loaded by the caller.
__device__ __forceinline__ void head_epi4(const ConvArgs& a, int m0, int c, f4 v, float bias, float anc) {
  const Epilogue& e = a.head_e;
  if (m0 >= a.M) return;
  const int ai = c / e.no, k = c - ai * e.no;
  int n0, oy0, ox0;
  row_to_pix(a, m0, n0, oy0, ox0);
  const size_t plane = (size_t)a.oh * a.ow;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    if (m0 + r >= a.M) break;
    int n, oy, ox;
    row_pix4(a, m0, r, n0, oy0, ox0, n, oy, ox);
    float x = v[r] + bias;
    if (e.act == ACT_LEAKY) x = x > 0.f ? x : x * e.slope;
    float o;
    if (e.raw)
      o = x;
    else if (k < 2)
      o = (__frcp_rn(1.f + __expf(-x)) + (float)(k == 0 ? ox : oy)) * e.ystride;
    else if (k < 4)
      o = (__expf(x) * anc) * e.ystride;
    else
      o = __frcp_rn(1.f + __expf(-x));
    const size_t row = (size_t)n * e.io_rows + e.io_off + (size_t)ai * plane + (size_t)oy * a.ow + ox;
    e.io[row * e.no + k] = o;
  }
}

// ABL: ablation bits for diagnostic builds only (outputs are wrong when non-zero):
// 1 = no buffer->LDS loads in the K-loop, 2 = no fragment ds_reads in the K-loop,
// 4 = no wait + barrier in the K-loop, 16 = no epilogue (one guarded store keeps the
// MFMAs live), 32 = no K-loop (prologue + epilogue only).  Bit 8 (not an ablation):
// fused YOLO head; bit 128 (not an ablation): lean epilogue (epi_vec8_lean); bit 256 with
// 128: lean epilogue with the fused shortcut add.
// One BM x 128 output tile (logical tile index bid, M-major over N tiles).
// I8 (RTDM_I8 detectors, BASELINE config 5): int8 activations (a quantised copy of the
// input view, per-channel scales folded into the weights) and int8 weights, the same
// 128-byte LDS rows holding 128 K-elements instead of 64, v_mfma_i32_16x16x64_i8 in place
// of v_mfma_f32_16x16x32_f16 (same issue count per K-block, twice the K), exact int32
// sums dequantised per output channel (a.deq) before the unchanged fp32 epilogues.
// WIN: window mode (see kWinRows): per K-block B ops + ONE window op (a 64-row slice of
// the next channel block's window, or a dummy zero load into the zero area, so every
// stage issues the same op count for the counted waits).
template <int ABL, int BM, bool I8 = false, bool WIN = false>
__device__ __forceinline__ void pipe_tile(const ConvArgs& a, unsigned char* smem_raw, int bid, bool pf, int next,
                                          bool pre) {
  constexpr int WM = PipeCfg<BM>::WM, WN = PipeCfg<BM>::WN;
  constexpr int BN = kPBN, BK = kPBK;              // LDS row: BK halfs = 128 bytes
  constexpr int ES = I8 ? 1 : 2, BKE = I8 ? 128 : 64;  // element bytes, K-elements per K-block
  constexpr int kPStage = WIN ? BN * BK : PipeCfg<BM>::Stage;  // halfs per ring stage
  constexpr int WAVES = WM * WN, NT = 64 * WAVES;
  constexpr int FM = BM / WM / 16, FN = BN / WN / 16;  // accumulators per wave
  constexpr int NA = WIN ? 1 : BM * BK * 2 / (NT * 16);  // A buffer->LDS ops per thread per stage
  constexpr int NB = BN * BK * 2 / (NT * 16);          // B ops
  constexpr int VM = NA + NB;
  constexpr int NSt = WIN ? kPNS : PipeCfg<BM>::NS;  // LDS ring stages (window mode: the 3-stage B ring)
  constexpr int WAITN = (NSt - 2) * VM;               // ops of the stages younger than kb+1
  static_assert(WAITN == 3 || WAITN == 4 || WAITN == 6 || WAITN == 8 || WAITN == 12, "wait literal");
  static_assert(!WIN || BM >= 128, "window mode: 256- / 128-row tiles");
  static_assert(VM == 6 || VM == 4 || VM == 3, "wait literal");
  _Float16* smem = reinterpret_cast<_Float16*>(smem_raw);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WN, wn = wid % WN;
  const int ntn = a.cout_pad / BN;
  const int mt = bid / ntn;
  const int m_base = mt * BM, n_base = (bid - mt * ntn) * BN;

  // Register epilogue (ABL bit 512, lean layers without pool / upsample outputs, whose
  // scattered 8-byte stores measured slower than the LDS path): the MFMA operands are swapped (weights as
  // A, activations as B), so a lane's accumulator holds 4 consecutive output channels
  // of one pixel (D^T; every output is the same K-ordered dot product, bit-identical)
  // and bias -> act -> affine -> stores run straight from registers, 8 bytes per lane
  // per 16x16 block, with the 2x2 pool as two DPP max steps over quad-order rows: no
  // fp32 C tile through LDS and no barrier between the K-loop and the stores.
  constexpr bool REG = (ABL & 512) != 0;
  // window mode with the taps unrolled (see the WLOOP loop below); ABL bit 4096 selects the
  // generic cursor loop instead (A/B diagnostics)
  constexpr bool WLOOP = WIN && !(ABL & 4096);
  // the same tap-unrolled loop for the per-tap-load (non-window) 3x3 layers (channel-block-outer
  // K order), chosen at run time; 1x1 layers keep the generic cursor loop
  constexpr bool ULOOP = !(ABL & 4096) && !(ABL & 32);
  const bool uloop = ULOOP && (WIN || (a.ks == 3 && a.pipe_corder != 0 && a.pipe_u != 0));
  constexpr bool RES_ = (ABL & 256) != 0;
  // cross-tile prefetch (pf, register epilogue only: the LDS ring is free during it)
  constexpr bool HEAD = (ABL & 8) != 0;
  constexpr bool PF = REG || HEAD;
  // Epilogue channel constants, loaded at the tile's start so their latency hides under
  // the K-loop.  Register epilogue: the 4 channels (4g..4g+3 of each 16-column block)
  // of this lane's accumulators.  Fused head: the FN columns of this lane's accumulators.
  constexpr int CG = BN / 8;
  float lb[8], ls[8], lh[8], la[8];
  // (register epilogue: its bias is loaded after the K-loop, load_rb, so that its 4 FN
  // registers are not live across the loop)
  f4 rb[REG ? FN : 1];
  auto load_rb = [&]() {
    const __amdgpu_buffer_rsrc_t rs_bias = __builtin_amdgcn_make_buffer_rsrc((void*)a.e.bias, 0, a.cout * 4, 0x00020000);
#pragma unroll
    for (int tn = 0; tn < FN; ++tn) {
      const int c0 = n_base + wn * (BN / WN) + tn * 16 + 4 * (lane >> 4);
      // buffer load: out-of-range channels (c0 >= cout) load zeros
      rb[tn] = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(rs_bias, c0 * 4, 0, 0));
    }
  };
  // WLOOP: the register epilogue's bias / the fused head's constants are loaded in the last
  // K-block body (their registers are not live across the loop); elsewhere at the tile start
  if constexpr (REG) {
    if (!uloop) load_rb();
  } else if constexpr ((ABL & 128) != 0) {
    const int c0 = n_base + (tid % CG) * 8;
    const bool cv = c0 < a.cout;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      lb[j] = cv ? a.e.bias[c0 + j] : 0.f;
      ls[j] = cv && a.e.scale ? a.e.scale[c0 + j] : 1.f;
      lh[j] = cv && a.e.scale ? a.e.shift[c0 + j] : 0.f;
    }
  } else if constexpr ((ABL & 1024) != 0) {  // stand-alone head: + the w/h anchors
    const int c0 = n_base + (tid % CG) * 8;
    if (c0 < a.cout) epi_io_consts(a, c0, lb, ls, lh, la);
  }
  float dq[FN];  // int8: per-output-channel dequantisation of this lane's accumulator columns
  f4 dq4[REG && I8 ? FN : 1];
  if constexpr (I8 && REG) {
#pragma unroll
    for (int tn = 0; tn < FN; ++tn) {
      const int c0 = n_base + wn * (BN / WN) + tn * 16 + 4 * (lane >> 4);
      dq4[tn] = c0 < a.cout ? *(const f4*)(a.deq + c0) : f4{0.f, 0.f, 0.f, 0.f};
    }
  } else if constexpr (I8) {
#pragma unroll
    for (int tn = 0; tn < FN; ++tn) {
      const int col = n_base + wn * (BN / WN) + tn * 16 + (lane & 15);
      dq[tn] = col < a.cout ? a.deq[col] : 0.f;
    }
  }
  float hb[FN], hs[FN], hh[FN];  // fused head: loaded after the K-loop (load_hconst)
  auto load_hconst = [&]() {
#pragma unroll
    for (int tn = 0; tn < FN; ++tn) {
      const int col = wn * (BN / WN) + tn * 16 + (lane & 15);
      const bool cv = col < a.cout;
      hb[tn] = cv ? a.e.bias[col] : 0.f;
      hs[tn] = (cv && a.e.scale) ? a.e.scale[col] : 1.f;
      hh[tn] = (cv && a.e.scale) ? a.e.shift[col] : 0.f;
    }
  };
  if (HEAD && !uloop) load_hconst();

  // ---- per-lane staging state.  A op j of wave w fills tile rows 8(NA w + j) + lane/8,
  //      B op j rows 8(NB w + j) + lane/8; LDS slot lane%8 of a row holds k-vector
  //      slot ^ (row & 7) (the read side applies the same involution).  ds_read_b128 serves
  //      a wave in 4 lane groups of 16, each mixing 8 lanes of one 16-lane row block (rows
  //      R..R+15 by fr, one k-slot group g) with 8 of the next (g ^ 1): with slot = g ^ (row & 7)
  //      the 16 reads hit 16 distinct 4-bank groups (8·(row & 1) + slot) for ANY row offset R,
  //      so the window mode's tap-shifted rows read conflict-free too (the former
  //      (row >> 1) & 7 swizzle was conflict-free only for even R: 31 % of the window
  //      kernel's LDS cycles were bank conflicts, profiles/r02ci_pmc_table.txt).
  //      Per-tile part (PipeGeo): A row offsets / tap masks, the window origin, the weight
  //      panel; built for this tile and, for the cross-tile prefetch, for the next one. ----
  const int slot = lane & 7;
  struct Geo {
    int m_base, koff_n;                // koff_n: byte offset of the tile's weight panel
    int voff_a[WIN ? 1 : NA];
    uint32_t vmask[WIN ? 1 : NA];
    int wp0, wv0;                      // window mode: first window row's pixel / source offset
  };
  const int wrow0 = 8 * wid + (lane >> 3);
  auto make_geo = [&](int tile) {
    Geo G;
    const int tmt = tile / ntn;
    G.m_base = tmt * BM;
    G.koff_n = (tile - tmt * ntn) * BN * a.kpad * ES;
#pragma unroll
    for (int j = 0; j < (WIN ? 0 : NA); ++j) {
      const int r = 8 * (NA * wid + j) + (lane >> 3);
      const int kofs = 16 * (slot ^ (r & 7));  // bytes
      const int m = G.m_base + r;
      int n = 0, oy = 0, ox = 0;
      if (m < a.M) row_to_pix(a, m, n, oy, ox);
      const int iy0 = m < a.M ? oy * a.stride - a.pad : -(1 << 28);
      const int ix0 = ox * a.stride - a.pad;
      G.voff_a[j] = m < a.M ? (n * a.ih * a.iw + iy0 * a.iw + ix0) * a.in_cs * ES + kofs : 0;
      uint32_t msk = 0;
      for (int t = 0; t < a.ks * a.ks; ++t) {
        const int kh = a.ks == 3 ? (t * 11) >> 5 : 0, kw = t - kh * a.ks;
        const int iy = iy0 + kh, ix = ix0 + kw;
        if ((unsigned)iy < (unsigned)a.ih && (unsigned)ix < (unsigned)a.iw) msk |= 1u << t;
      }
      G.vmask[j] = msk;
    }
    if constexpr (WIN) {
      G.wp0 = G.m_base - a.iw - 1 + wrow0;
      G.wv0 = G.wp0 * a.in_cs * ES + 16 * (slot ^ (wrow0 & 7));  // + 64j rows keeps the swizzle
    } else {
      G.wp0 = G.wv0 = 0;
    }
    return G;
  };
  const Geo G0 = make_geo(bid);
  int voff_b[NB];
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    const int r = 8 * (NB * wid + j) + (lane >> 3);
    voff_b[j] = r * a.kpad * ES + 16 * (slot ^ (r & 7));
  }
  const char* in = (const char*)a.in + (size_t)a.in_co * ES;
  const int64_t in_bytes = ((int64_t)a.n * a.ih * a.iw * a.in_cs - a.in_co) * ES;
  const __amdgpu_buffer_rsrc_t rs_in = __builtin_amdgcn_make_buffer_rsrc((void*)in, 0, (int)in_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rs_w = __builtin_amdgcn_make_buffer_rsrc((void*)(I8 ? a.w8 : a.w), 0,
                                                                        a.cout_pad * a.kpad * ES, 0x00020000);
  const int nk = a.kpad / BKE;
  const int cpt = a.cin / BKE;  // K-blocks per tap
  const int ntap = a.ks * a.ks;
  // K-block cursor: inner counter st_i (limit ni) and outer st_o; channel-block outer
  // (pipe_corder) walks the taps inside, tap outer the channel blocks.  Plain scalars
  // selected by value (a by-reference select of the counter to bump sends the cursor to
  // scratch, and its loads' vmcnt(0) then drains the LDS-DMA pipeline every K-block).
  const bool corder = a.pipe_corder != 0;
  const int ni = corder ? ntap : cpt;
  int st_i = 0, st_o = 0, st_buf = 0;

  // window mode: buffers, window geometry (rows of the channel block's window: pixels
  // m_base - W - 1 + row of the flattened batch, zero outside it)
  _Float16* const Bring = WIN ? smem + 2 * kWinRows * BK : smem;
  _Float16* const zarea = smem + 2 * kWinRows * BK + kPNS * BN * BK;
  _Float16* const jarea = zarea + 8 * BK;
  typedef __attribute__((address_space(3))) char lds_char;
  lds_char* const lds0 = (lds_char*)(lds_ptr_t)smem_raw;
  const int wr = BM + 2 * a.iw + 2;              // window rows used
  const int npix = a.n * a.ih * a.iw;
  const int ncb = a.cin / BKE;
  // one 64-row slice j of channel block cw's window (or a dummy zero load)
  // (branch-free: a divergent branch here would split the loop body, and the MFMA /
  // DS-read / VMEM interleave groups do not cross basic blocks)
  // per-lane row of slice 0 (this wave's 8 rows, lane / 8) and its source offset
  auto win_op = [&](const Geo& G, int j, int cw, bool live) {
    const int r0 = 64 * j + 8 * wid;  // this wave's 8 rows
    const bool real = live & (r0 < kWinRows);
    _Float16* dst = real ? smem + ((cw & 1) * kWinRows + r0) * BK : zarea;
    const int p = G.wp0 + 64 * j;
    const int vraw = G.wv0 + (64 * j * a.in_cs + cw * BKE) * ES;
    const bool ok = real & (wrow0 < wr - 64 * j) & ((unsigned)p < (unsigned)npix);
    const int vo = vraw | (int)((uint32_t)!ok << 31);  // >= 2^31: out of range, loads 0
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs_in, (lds_ptr_t)dst, 16, vo, 0, 0, 0);
  };

  // Issue the VM buffer->LDS ops of the next K-block (cursor si / so) of tile G into stage sb.
  auto stage_g = [&](const Geo& G, int& si, int& so, int& sb) {
    _Float16* As = smem + sb * kPStage;
    _Float16* Bs = WIN ? Bring + sb * kPStage : As + BM * BK;
    const int st_tap = __builtin_amdgcn_readfirstlane(corder ? si : so);
    const int st_c = __builtin_amdgcn_readfirstlane(corder ? so : si);
    const int kh = a.ks == 3 ? (st_tap * 11) >> 5 : 0, kw = st_tap - kh * a.ks;
    if constexpr (WIN) {
      // K-block s = 9 st_c + st_tap is staged during body s - 2: it carries slice
      // j = st_tap - 2 (taps 2..8 -> slices 0..6) of channel block st_c + 1's window
      const int j = st_tap - 2, cw = st_c + 1;
      win_op(G, j < 0 ? 0 : j, cw, j >= 0 && cw < ncb && 64 * j < wr);
    } else {
      const int tapoff = ((kh * a.iw + kw) * a.in_cs + st_c * BKE) * ES;
#pragma unroll
      for (int j = 0; j < NA; ++j) {
        const int vo = ((G.vmask[j] >> st_tap) & 1u) ? G.voff_a[j] + tapoff : (int)0x80000000;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs_in, (lds_ptr_t)(As + 8 * (NA * wid + j) * BK), 16, vo, 0, 0, 0);
      }
    }
    // weight column of this K-block (tap-major packing) in the tile's panel
    const int koff = G.koff_n + (st_tap * a.cin + st_c * BKE) * ES;
#pragma unroll
    for (int j = 0; j < NB; ++j)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs_w, (lds_ptr_t)(Bs + 8 * (NB * wid + j) * BK), 16, voff_b[j], koff,
                                               0, 0);
    if (++si == ni) {
      si = 0;
      ++so;
    }
    sb = sb == NSt - 1 ? 0 : sb + 1;
  };
  auto stage = [&]() { stage_g(G0, st_i, st_o, st_buf); };
  // prologue loads of tile G (window mode: channel block 0's whole window, then K-blocks
  // 0 .. NSt-2), from a fresh cursor; returns nothing, the caller waits
  auto prologue_issue = [&](const Geo& G) {
    int si = 0, so = 0, sb = 0;
    if constexpr (WIN) {
      for (int j = 0; 64 * j < wr; ++j) win_op(G, j, 0, true);
    }
#pragma unroll
    for (int i = 0; i < NSt - 1; ++i) stage_g(G, si, so, sb);
  };

  const int fr = lane & 15, g = lane >> 4;
  const int rsw = fr & 7;  // fragment rows start at multiples of 16
  const int so0 = 8 * ((0 + g) ^ rsw), so1 = 8 * ((4 + g) ^ rsw);
  const int a_row = (wm * (BM / WM) + fr) * BK, b_row = ((WIN ? 0 : BM) + wn * (BN / WN) + fr) * BK;

  // window mode read side: validity of the 9 taps for this lane's FM fragment rows
  // (out-of-image taps, and window rows of a neighbouring image, read the zero area)
  // and the LDS byte offsets of the next K-block's A fragments (half 1: ^ 64)
  uint32_t amask[WIN ? FM : 1];
  int aoff[WIN ? FM : 1];
  int rd_i = 0, rd_o = 0;  // cursor of the next K-block read0 reads
  if constexpr (WIN) {
#pragma unroll
    for (int tm = 0; tm < FM; ++tm) {
      const int m = m_base + wm * (BM / WM) + tm * 16 + fr;
      uint32_t msk = 0;
      if (m < a.M) {
        int n, oy, ox;
        row_to_pix(a, m, n, oy, ox);
        for (int t = 0; t < 9; ++t) {
          const int kh = (t * 11) >> 5, kw = t - 3 * kh;
          if ((unsigned)(oy + kh - 1) < (unsigned)a.ih && (unsigned)(ox + kw - 1) < (unsigned)a.iw) msk |= 1u << t;
        }
      }
      amask[tm] = msk;
    }
  }
  // byte offsets; the 16-row fragment blocks tm share the swizzle of block 0 (rows + 16 tm)
  const int zoff = (2 * kWinRows * BK + kPNS * BN * BK + 8 * g) * 2;
  const int wrd0 = wm * (BM / WM) + fr;
  auto win_addr = [&]() {  // aoff for K-block (rd_o, rd_i), then advance the read cursor
    const int t = __builtin_amdgcn_readfirstlane(rd_i);
    const int kh = (t * 11) >> 5, kw = t - 3 * kh;
    const int i = wrd0 + kh * a.iw + kw;
    const int off = ((rd_o & 1) * kWinRows + i) * BK * 2 + 16 * (g ^ (i & 7));
#pragma unroll
    for (int tm = 0; tm < FM; ++tm) aoff[tm] = ((amask[tm] >> t) & 1u) ? off + tm * 16 * BK * 2 : zoff;
    if (++rd_i == 9) {
      rd_i = 0;
      ++rd_o;
    }
  };

  typedef int i32x4 __attribute__((ext_vector_type(4)));
  using AccT = std::conditional_t<I8, i32x4, f4>;
  AccT acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = AccT{0, 0, 0, 0};
  auto mfma = [&](const h8& x_, const h8& y_, AccT c) -> AccT {
    const h8& x = REG ? y_ : x_;  // register epilogue: weights as A (D^T)
    const h8& y = REG ? x_ : y_;
    if constexpr (I8)
      return __builtin_amdgcn_mfma_i32_16x16x64_i8(__builtin_bit_cast(i32x4, x), __builtin_bit_cast(i32x4, y), c, 0, 0,
                                                   0);
    else
      return __builtin_amdgcn_mfma_f32_16x16x32_f16(x, y, c, 0, 0, 0);
  };

  h8 fa0[FM], fb0[FN], fa1[FM], fb1[FN];
  auto read0 = [&](int buf) {
    const _Float16* S = (WIN ? Bring : smem) + buf * kPStage;
    if constexpr (WIN) {
#pragma unroll
      for (int t = 0; t < FM; ++t) fa0[t] = *(const h8*)(smem_raw + aoff[t]);
    } else {
#pragma unroll
      for (int t = 0; t < FM; ++t) fa0[t] = *(const h8*)(S + a_row + t * 16 * BK + so0);
    }
#pragma unroll
    for (int t = 0; t < FN; ++t) fb0[t] = *(const h8*)(S + b_row + t * 16 * BK + so0);
  };
  auto read1 = [&](int buf) {
    const _Float16* S = (WIN ? Bring : smem) + buf * kPStage;
    if constexpr (WIN) {
#pragma unroll
      for (int t = 0; t < FM; ++t) fa1[t] = *(const h8*)(smem_raw + (aoff[t] ^ 64));
    } else {
#pragma unroll
      for (int t = 0; t < FM; ++t) fa1[t] = *(const h8*)(S + a_row + t * 16 * BK + so1);
    }
#pragma unroll
    for (int t = 0; t < FN; ++t) fb1[t] = *(const h8*)(S + b_row + t * 16 * BK + so1);
  };
  // WLOOP read side.  The tap TT of a K-block is a compile-time constant: its row shift
  // sh = kh * W + kw is one scalar, the 16-byte slot g ^ ((row + sh) & 7) comes from a
  // per-lane table of the 8 residues (3 bits each), and the fragment blocks tm = 1..3 are
  // ds_read immediate offsets (tm * 2048).  An out-of-image tap reads the zero area: its
  // address is zb - tm * 2048, so address + immediate = zb (half 1: zb ^ 64, both inside
  // the 1 KB zero area; 2048 tm and the window parity offset are multiples of 128, so the
  // half-1 XOR commutes with them).
  const int zb = (2 * kWinRows * BK + kPNS * BN * BK) * 2;
  static_assert(((2 * kWinRows * kPBK + kPNS * kPBN * kPBK) * 2) % 256 == 0, "zero area 256-byte aligned");
  uint32_t wtab = 0;
  if constexpr (WLOOP) {
#pragma unroll
    for (int r = 0; r < 8; ++r) wtab |= (uint32_t)((g ^ ((wm * (BM / WM) + fr + r) & 7)) & 7) << (3 * r);
  }
  const int lrow = (wm * (BM / WM) + fr) * BK * 2;
  // The per-tap values derive from an opaque zero zo, re-made opaque in every body by an empty
  // asm the compiler cannot see through (it must assume any value): otherwise the compiler
  // hoists the 9 taps' shifts, weight-column offsets and tap-validity masks out of the
  // channel-block loop, and the SGPRs / VGPRs they need spill (VGPR-lane reloads in the loop,
  // scratch reloads whose vmcnt(0) drain the LDS-DMA pipeline).  (Round 3 used a loop-carried
  // zo *= a.pipe_z with a host-side zero, which a compiler that specialised on the argument
  // could have seen through.)
  int zo = 0;
  auto waddr = [&](auto tt_, int par) {
    constexpr int TT = decltype(tt_)::value, KH = TT / 3, KW = TT % 3;
    const int iw_o = a.iw + zo;
    const int sh = KH * iw_o + KW;
    const int off = lrow + ((par * kWinRows + sh) << 7) + (int)(((wtab >> (3 * (sh & 7))) & 7u) << 4);
    // an out-of-image tap reads the zero area at its own offset mod 256 (zb is 256-aligned), so
    // it takes the bank slot its in-image read would have: a 16-lane group stays conflict-free
    // (one shared zero address collided with the group's in-image reads: 20 % of the 19^2
    // layers' LDS cycles were bank conflicts, PMC r05g; now 0 %, the layers 0.2-0.5 % faster,
    // bit-identical, profiles/r05w_zero_area_ab.txt)
    const int zl = zb + (off & 255);
#pragma unroll
    for (int tm = 0; tm < FM; ++tm) {
      const int keep = (int)(amask[tm] << (31 - TT + zo)) >> 31;  // 0 / -1: tap TT valid for this row
      aoff[tm] = (off & keep) | ((zl - tm * 2048) & ~keep);
    }
  };
  auto wread0 = [&](auto buf_) {
    const _Float16* S = Bring + decltype(buf_)::value * kPStage;
#pragma unroll
    for (int t = 0; t < FM; ++t) fa0[t] = *(const h8*)(smem_raw + aoff[t] + t * 2048);
#pragma unroll
    for (int t = 0; t < FN; ++t) fb0[t] = *(const h8*)(S + b_row + t * 16 * BK + so0);
  };
  auto wread1 = [&](auto buf_) {
    const _Float16* S = Bring + decltype(buf_)::value * kPStage;
#pragma unroll
    for (int t = 0; t < FM; ++t) fa1[t] = *(const h8*)(smem_raw + (aoff[t] ^ 64) + t * 2048);
#pragma unroll
    for (int t = 0; t < FN; ++t) fb1[t] = *(const h8*)(S + b_row + t * 16 * BK + so1);
  };
  constexpr int NMF = FM * FN, NRD = FM + FN;
  // MFMA / DS-read interleave of one cluster: NRD reads spread over the NMF MFMAs
  auto interleave_reads = [&]() {
    constexpr int per = NMF / NRD > 0 ? NMF / NRD : 1;
#pragma unroll
    for (int i = 0; i < NRD; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x008, per, 0);  // MFMA
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);    // DS read
    }
  };

  // prologue: (window mode: channel block 0's whole window,) K-blocks 0 and 1 in flight,
  // wait for 0
  // (cross-tile prefetch: the previous tile of this workgroup issued them before its
  // epilogue, whose exactly EPI vector-memory ops are younger than K-block NSt-2)
  if constexpr (WLOOP)
    waddr(std::integral_constant<int, 0>{}, 0);
  else if constexpr (WIN)
    win_addr();
  // the tile cursor past the prologue's NSt-1 K-blocks (issued here or by the previous tile)
  auto skip_prologue = [&]() {
#pragma unroll
    for (int i = 0; i < NSt - 1; ++i) {
      if (++st_i == ni) {
        st_i = 0;
        ++st_o;
      }
      st_buf = st_buf == NSt - 1 ? 0 : st_buf + 1;
    }
  };
  if (PF && pre) {
    skip_prologue();
    // (fused head: its io stores are per-lane conditional, so younger than K-block NSt-2
    // only a lower bound of them: none — the wait also covers them)
    wait_vmn_lgkm0<WAITN + (HEAD ? 0 : pipe_epi_ops<RES_, FM, FN>())>();
  } else if (nk >= NSt - 1) {
    prologue_issue(G0);
    skip_prologue();
    wait_vm_lgkm0<WAITN>();
  } else {
    if constexpr (WIN) {
      for (int j = 0; 64 * j < wr; ++j) win_op(G0, j, 0, true);
    }
    for (int i = 0; i < nk; ++i) stage();
    wait_vm_lgkm0<0>();
  }
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
  if constexpr (WLOOP)
    wread0(std::integral_constant<int, 0>{});
  else
    read0(0);

  // Cluster A (half 0 of kb): MFMAs on fa0/fb0, interleaved with the reads of half 1
  // (fa1/fb1) and the buffer->LDS loads of kb+NSt-1.  Cluster B (half 1): MFMAs on
  // fa1/fb1, interleaved with the reads of half 0 of kb+1 (after the barrier that
  // publishes kb+1).  The loop is peeled so the steady-state body is one basic
  // block (interleave groups do not cross branches): STG = loads of kb+NSt-1 go out,
  // NXT = kb+1 exists (wait for it, barrier, read its half 0).
  int cur = 0;
  auto body = [&](auto stg, auto nxt_c) {
    constexpr bool STG = decltype(stg)::value, NXT = decltype(nxt_c)::value;
    const int nxt = cur == NSt - 1 ? 0 : cur + 1;
    if constexpr (!(ABL & 2)) read1(cur);
    if constexpr (STG && !(ABL & 1)) stage();
#pragma unroll
    for (int tm = 0; tm < FM; ++tm)
#pragma unroll
      for (int tn = 0; tn < FN; ++tn)
        acc[tm][tn] = mfma(fa0[tm], fb0[tn], acc[tm][tn]);
    if constexpr (STG && !(ABL & 1)) {
      // reads in the first half of the cluster, the VM loads in the second
      constexpr int half = NMF / 2;
      constexpr int per_r = half / NRD > 0 ? half / NRD : 1;
      constexpr int per_v = (NMF - half) / VM > 0 ? (NMF - half) / VM : 1;
#pragma unroll
      for (int i = 0; i < NRD; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, per_r, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      }
#pragma unroll
      for (int i = 0; i < VM; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, per_v, 0);
        __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
      }
      __builtin_amdgcn_sched_group_barrier(0x008, NMF, 0);
    } else {
      interleave_reads();
      __builtin_amdgcn_sched_group_barrier(0x008, NMF, 0);
    }
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (NXT && WIN) win_addr();
    if constexpr (NXT) {
      // retire kb+1 (kb+2 stays in flight); lgkmcnt(0): this stage's reads are done
      // in every wave before any wave restages it (kb+3, issued after this barrier)
      if constexpr (!(ABL & 4)) {
        if constexpr (STG)
          wait_vm_lgkm0<WAITN>();
        else
          wait_vm_lgkm0<0>();
        __builtin_amdgcn_s_barrier();
      }
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (!(ABL & 2)) read0(nxt);
    }
#pragma unroll
    for (int tm = 0; tm < FM; ++tm)
#pragma unroll
      for (int tn = 0; tn < FN; ++tn)
        acc[tm][tn] = mfma(fa1[tm], fb1[tn], acc[tm][tn]);
    if constexpr (NXT) interleave_reads();
    __builtin_amdgcn_sched_group_barrier(0x008, NMF, 0);
    __builtin_amdgcn_sched_barrier(0);
    cur = nxt;
  };
  using T_ = std::true_type;
  using F_ = std::false_type;
  // ---- WLOOP: window mode with the 9 taps of a channel block unrolled.  K-block s = 9 cb + t
  //      with t a compile-time constant in each body, so everything the generic loop derives
  //      from its cursor per K-block is fixed: the tap's row shift (waddr), the ring stage
  //      (s % 3 = t % 3: 9 K-blocks per channel block), the K-block staged with it (s + 2:
  //      tap (t + 2) % 9) and its window slice (slice t of channel block cb + 1's window for
  //      t <= 6, none for t = 7, 8: no dummy loads), and so the counted vmcnt.  The last
  //      channel block (no next window; nothing to stage after tap 6) is its own unrolled
  //      copy.  Per wave and K-block the generic loop spent ~40 SALU + ~25 VALU on cursor,
  //      window-op and address arithmetic, serially between two MFMAs; here one VALU per
  //      window op and the fragment address selects remain.  Every accumulator sees the
  //      same MFMA sequence: bit-identical to the generic loop.
  //      Non-window 3x3 layers (uloop, !WIN): the same unrolled loop with the per-tap A loads
  //      of conv_pipe (tap offset one scalar, validity bit test per A op) and the A fragments
  //      at fixed LDS offsets of the compile-time ring stage.
  if (uloop) {
    static_assert(ULOOP == false || NSt == 3, "ring stage s % 3 = tap % 3 (9 taps per channel block)");
    auto wbody = [&](auto t_, auto stg_, auto wop_, auto nxt_, int cb) {
      constexpr int T = decltype(t_)::value;
      constexpr bool STG = decltype(stg_)::value, WOP = decltype(wop_)::value, NXT = decltype(nxt_)::value;
      // ops of K-block s + 2 issued here (ABL bits 8192 / 16384: diagnostics without the window
      // slices / without the B loads)
      constexpr int VMS = STG ? ((ABL & 16384) ? 0 : NB) + (WIN ? (WOP && !(ABL & 8192) ? 1 : 0) : NA) : 0;
      asm volatile("" : "+s"(zo));  // opaque: any value, as far as the compiler knows
      if constexpr (!(ABL & 2)) {
        if constexpr (WIN)
          wread1(std::integral_constant<int, T % 3>{});
        else
          read1(T % 3);
      }
      if constexpr (!NXT) {  // the tile's last K-block: the epilogue constants
        if constexpr (REG) load_rb();
        if constexpr (HEAD) load_hconst();
      }
      if constexpr (STG && !(ABL & 1) && !WIN) {
        // A: tap (T + 2) % 9 of channel block cb + (T >= 7); out-of-image taps load zeros
        constexpr int T2 = (T + 2) % 9, KH2 = T2 / 3, KW2 = T2 % 3;
        const int tapoff = ((KH2 * (a.iw + zo) + KW2) * (a.in_cs + zo) + (cb + (T >= 7 ? 1 : 0)) * BKE) * ES;
        _Float16* As = smem + ((T + 2) % 3) * kPStage;
#pragma unroll
        for (int j = 0; j < NA; ++j) {
          const int vo = ((G0.vmask[j] >> (T2 + zo)) & 1u) ? G0.voff_a[j] + tapoff : (int)0x80000000;
          __builtin_amdgcn_raw_ptr_buffer_load_lds(rs_in, (lds_ptr_t)(As + 8 * (NA * wid + j) * BK), 16, vo, 0, 0, 0);
        }
      }
      if constexpr (STG && !(ABL & 1)) {
        if constexpr (WIN && WOP && !(ABL & 8192)) {
          // slice T of channel block cb + 1's window: one VALU add.  Rows before / past the
          // batch are out of the buffer's range (zeros); rows past the window (>= wr) load
          // data no tap reads, except a slice wholly past it, which is pushed out of range by
          // the scalar 2^31 (pipe_win_ok: input < 2^30 bytes, so even the first tile's
          // negative offsets stay out of range); rows past kWinRows go to the junk area.
          const int cw = cb + 1;
          const int r0 = 64 * T + 8 * wid;
          // (the destination as an LDS byte offset: a select of two generic LDS pointers
          // makes the compiler emit an illegal null check of the shared aperture)
          const int dofs = r0 < kWinRows ? ((cw & 1) * kWinRows + r0) * BK * 2 : (int)((jarea - smem) * 2);
          // (offsets in unsigned arithmetic: with the 2^31 skip the sum wraps by design)
          const uint32_t so = (uint32_t)((64 * T * (a.in_cs + zo) + cw * BKE) * ES) + (64 * T < wr ? 0u : 0x80000000u);
          __builtin_amdgcn_raw_ptr_buffer_load_lds(rs_in, (lds_ptr_t)(lds0 + dofs), 16, (int)((uint32_t)G0.wv0 + so), 0, 0,
                                                   0);
        }
        constexpr int T2 = (T + 2) % 9;
        const int koff = G0.koff_n + (T2 * (a.cin + zo) + (cb + (T >= 7 ? 1 : 0)) * BKE) * ES;
        _Float16* Bs = WIN ? Bring + ((T + 2) % 3) * kPStage : smem + ((T + 2) % 3) * kPStage + BM * BK;
#pragma unroll
        for (int j = 0; j < ((ABL & 16384) ? 0 : NB); ++j)
          __builtin_amdgcn_raw_ptr_buffer_load_lds(rs_w, (lds_ptr_t)(Bs + 8 * (NB * wid + j) * BK), 16, voff_b[j],
                                                   koff, 0, 0);
      }
#pragma unroll
      for (int tm = 0; tm < FM; ++tm)
#pragma unroll
        for (int tn = 0; tn < FN; ++tn) acc[tm][tn] = mfma(fa0[tm], fb0[tn], acc[tm][tn]);
      if constexpr (STG && !(ABL & 1)) {
        constexpr int half = NMF / 2;
        constexpr int per_r = half / NRD > 0 ? half / NRD : 1;
        constexpr int per_v = VMS > 0 && (NMF - half) / VMS > 0 ? (NMF - half) / VMS : 1;
#pragma unroll
        for (int i = 0; i < NRD; ++i) {
          __builtin_amdgcn_sched_group_barrier(0x008, per_r, 0);
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        }
#pragma unroll
        for (int i = 0; i < VMS; ++i) {
          __builtin_amdgcn_sched_group_barrier(0x008, per_v, 0);
          __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
        }
        __builtin_amdgcn_sched_group_barrier(0x008, NMF, 0);
      } else {
        interleave_reads();
        __builtin_amdgcn_sched_group_barrier(0x008, NMF, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (NXT) {
        if constexpr (WIN) waddr(std::integral_constant<int, (T + 1) % 9>{}, (cb + (T == 8 ? 1 : 0)) & 1);
        // retire K-block s + 1 (s + 2 stays in flight); lgkmcnt(0): this stage's reads are
        // done in every wave before any wave restages it
        if constexpr (!(ABL & 4)) {
          wait_vm_lgkm0<VMS>();
          __builtin_amdgcn_s_barrier();
        }
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (!(ABL & 2)) {
          if constexpr (WIN)
            wread0(std::integral_constant<int, (T + 1) % 3>{});
          else
            read0((T + 1) % 3);
        }
      }
#pragma unroll
      for (int tm = 0; tm < FM; ++tm)
#pragma unroll
        for (int tn = 0; tn < FN; ++tn) acc[tm][tn] = mfma(fa1[tm], fb1[tn], acc[tm][tn]);
      if constexpr (NXT) interleave_reads();
      __builtin_amdgcn_sched_group_barrier(0x008, NMF, 0);
      __builtin_amdgcn_sched_barrier(0);
    };
    int cb = 0;
    for (; cb < ncb - 1; ++cb)
      unroll_seq(
          [&](auto t_) {
            constexpr int T = decltype(t_)::value;
            wbody(t_, T_{}, std::bool_constant<(T <= 6)>{}, T_{}, cb);
          },
          std::make_integer_sequence<int, 9>{});
    unroll_seq(
        [&](auto t_) {
          constexpr int T = decltype(t_)::value;
          wbody(t_, std::bool_constant<(T <= 6)>{}, F_{}, std::bool_constant<(T <= 7)>{}, cb);
        },
        std::make_integer_sequence<int, 9>{});
  } else if constexpr (!(ABL & 32) && !WLOOP) {
    int kb = 0;
    for (; kb + NSt - 1 < nk; ++kb) body(T_{}, T_{});  // stages kb + NSt - 1
    for (; kb + 1 < nk; ++kb) body(F_{}, T_{});        // tail: nothing left to stage (waits vmcnt(0))
    body(F_{}, F_{});
  }
  if constexpr (REG) {
    if (pf) {
      if (next >= 0) {  // prefetch the next tile's prologue under this tile's epilogue
        // (WLOOP: the bias loads of the last K-block body are the only older vector-memory
        // ops; retired here, so the epilogue's use of them never waits on the prefetch)
        if (uloop)
          asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        else
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();  // every wave is past its last fragment read
        __builtin_amdgcn_sched_barrier(0);
        prologue_issue(make_geo(next));
        __builtin_amdgcn_sched_barrier(0);
      }
      pipe_epi_regs<RES_, FM, FN, BM / WM, BN / WN, true>(a, m_base, n_base, wm, wn, lane, acc, rb, dq4);
    } else {
      pipe_epi_regs<RES_, FM, FN, BM / WM, BN / WN>(a, m_base, n_base, wm, wn, lane, acc, rb, dq4);
    }
    return;
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __syncthreads();
  f4 accf[FM][FN];
#pragma unroll
  for (int tm = 0; tm < FM; ++tm)
#pragma unroll
    for (int tn = 0; tn < FN; ++tn) {
      if constexpr (I8) {
#pragma unroll
        for (int j = 0; j < 4; ++j) accf[tm][tn][j] = (float)acc[tm][tn][j] * dq[tn];
      } else {
        accf[tm][tn] = acc[tm][tn];
      }
    }

  if constexpr ((ABL & 8) != 0) {
    // ---- fused head: activated conv output (fp16, the value the unfused path would
    //      store) -> LDS tile [256][128] (16-B slot swizzle: slot ^ (row & 15)) ->
    //      1x1 head GEMM on MFMA -> YOLO decode -> io.  Same fp16 operands and K
    //      order as the unfused head conv.
    _Float16* Hs = smem;
    const Epilogue& e = a.e;
    // head weight fragments and decode constants first: their loads are older than the
    // next tile's prefetch, and their latency hides under the activated-tile writes
    const _Float16* hw = (const _Float16*)a.head_w;  // [32][128]
    h8 hbf[BN / 32][2];
#pragma unroll
    for (int ks = 0; ks < BN / 32; ++ks)
#pragma unroll
      for (int t = 0; t < 2; ++t) hbf[ks][t] = *(const h8*)(hw + (16 * t + fr) * BN + 32 * ks + 8 * g);
    float hbias[2], hanc[2];
#pragma unroll
    for (int tq = 0; tq < 2; ++tq) {
      const int c = 16 * tq + fr;
      const bool cv = c < a.head_cout;
      const int ai = c / a.head_e.no, k = c - ai * a.head_e.no;
      hbias[tq] = cv ? a.head_e.bias[c] : 0.f;
      hanc[tq] = cv && (k == 2 || k == 3) ? a.head_e.anchor_vec[2 * ai + (k - 2)] : 0.f;
    }
#pragma unroll
    for (int tn = 0; tn < FN; ++tn) {
      const int col = wn * (BN / WN) + tn * 16 + fr;
      const bool cv = col < a.cout;
      const float bias = hb[tn], sc = hs[tn], sh = hh[tn];
#pragma unroll
      for (int tm = 0; tm < FM; ++tm)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int row = wm * (BM / WM) + tm * 16 + g * 4 + j;
          float x = accf[tm][tn][j] + bias;
          if (e.act == ACT_LEAKY)
            x = x > 0.f ? x : x * e.slope;
          else if (e.act == ACT_SWISH)  // yolov4-tiny-swish.cfg (models.py:43-44)
            x = x * sigmoidf_(x);
          x = cv ? x * sc + sh : 0.f;
          Hs[row * BN + 8 * ((col >> 3) ^ (row & 15)) + (col & 7)] = (_Float16)x;
        }
    }
    __syncthreads();
    // each wave: BM / 8 rows (HT fragments of 16) x the 32 head channels
    constexpr int HR = BM / WAVES, HT = HR / 16;
    static_assert(HT >= 1, "fused head needs BM >= 128");
    f4 hacc[HT][2];
#pragma unroll
    for (int i = 0; i < HT; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) hacc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < BN / 32; ++ks) {
      h8 af[HT];
#pragma unroll
      for (int t = 0; t < HT; ++t) {
        const int row = HR * wid + 16 * t + fr;
        af[t] = *(const h8*)(Hs + row * BN + 8 * ((4 * ks + g) ^ (row & 15)));
      }
#pragma unroll
      for (int tm = 0; tm < HT; ++tm)
#pragma unroll
        for (int tq = 0; tq < 2; ++tq)
          hacc[tm][tq] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[tm], hbf[ks][tq], hacc[tm][tq], 0, 0, 0);
    }
    if (pf && next >= 0) {  // the activated tile is consumed: prefetch under the decode / io stores
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      prologue_issue(make_geo(next));
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int tm = 0; tm < HT; ++tm)
#pragma unroll
      for (int tq = 0; tq < 2; ++tq) {
        const int c = 16 * tq + fr;
        if (c < a.head_cout)
          head_epi4(a, m_base + HR * wid + 16 * tm + 4 * g, c, hacc[tm][tq], hbias[tq], hanc[tq]);
      }
    return;
  }

  if constexpr ((ABL & 16) != 0) {
    float t = 0.f;
#pragma unroll
    for (int tm = 0; tm < FM; ++tm)
#pragma unroll
      for (int tn = 0; tn < FN; ++tn) t += accf[tm][tn][0] + accf[tm][tn][1] + accf[tm][tn][2] + accf[tm][tn][3];
    if (t == 1234.5f) ((float*)a.e.full.ptr)[tid] = t;
    return;
  }
  // ---- epilogue: accumulators -> LDS C tile (fp32) -> 4 rows x 8 channels per thread ----
  float* Cs = reinterpret_cast<float*>(smem_raw);
  const int rq = g * 4;
#pragma unroll
  for (int tm = 0; tm < FM; ++tm)
#pragma unroll
    for (int tn = 0; tn < FN; ++tn) {
      const int row = wm * (BM / WM) + tm * 16 + rq;
      const int col = wn * (BN / WN) + tn * 16 + fr;
#pragma unroll
      for (int j = 0; j < 4; ++j) Cs[(row + j) * kPCstr + col] = accf[tm][tn][j];
    }
  __syncthreads();
  constexpr int UNITS = (BM / 4) * CG;
  static_assert(NT % CG == 0, "channel group per thread");
  if constexpr ((ABL & 1024) != 0) {
    if (!a.quad) {  // (head convs are never quad-ordered; the per-unit stores below stay for them)
      // stand-alone YOLO head: decode in place in the C tile (same operations as
      // epi_vec8_io), then write io anchor plane by anchor plane: a plane's rows of
      // consecutive pixels are one contiguous run of io, stored by consecutive lanes
      // (the per-unit stores were 4-byte scatters, one io row per lane)
      for (int u = tid; u < UNITS; u += NT) {
        const int q = u / CG, gg = u - (u / CG) * CG;
        const int m0 = m_base + q * 4, c0 = n_base + gg * 8;
        if (m0 >= a.M || c0 >= a.cout) continue;
        float v[4][8];
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
          for (int j = 0; j < 8; ++j) v[r][j] = Cs[(q * 4 + r) * kPCstr + gg * 8 + j];
        epi_io_decode(a, m0, c0, v, lb, ls, lh, la);
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
          for (int j = 0; j < 8; ++j) Cs[(q * 4 + r) * kPCstr + gg * 8 + j] = v[r][j];
      }
      __syncthreads();
      const Epilogue& e = a.e;
      const int no = e.no, plane = a.oh * a.ow;
      const int rows = a.M - m_base < BM ? a.M - m_base : BM;
      const int nch = a.cout - n_base < BN ? a.cout - n_base : BN;
      const int per_a = rows * no;
      for (int ai = 0; ai * no < nch; ++ai) {
        const size_t aoff = (size_t)(n_base / no + ai) * plane;
        for (int f = tid; f < per_a; f += NT) {
          const int r = f / no, k = f - r * no;
          const int m = m_base + r, n = m / plane, p = m - n * plane;
          e.io[((size_t)n * e.io_rows + e.io_off + p + aoff) * no + k] = Cs[r * kPCstr + ai * no + k];
        }
      }
      return;
    }
  }
  for (int u = tid; u < UNITS; u += NT) {
    const int q = u / CG, gg = u - (u / CG) * CG;
    if constexpr ((ABL & 64) != 0) {
      if (Cs[(q * 4) * kPCstr + gg * 8] == 1234.5f) ((float*)a.e.full.ptr)[tid] = 0.f;
      continue;
    }
    const int m0 = m_base + q * 4, c0 = n_base + gg * 8;
    if (m0 >= a.M || c0 >= a.cout) continue;
    float v[4][8];
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int j = 0; j < 8; ++j) v[r][j] = Cs[(q * 4 + r) * kPCstr + gg * 8 + j];
    if constexpr ((ABL & 128) != 0)
      epi_vec8_lean<(ABL & 256) != 0>(a, m0, c0, v, lb, ls, lh);
    else if constexpr ((ABL & 1024) != 0)
      epi_vec8_io(a, m0, c0, v, lb, ls, lh, la);  // stand-alone YOLO head: decode -> io only
    else
      epi_vec8(a, m0, c0, v);
  }
}

// Persistent over tiles: one workgroup per CU walks a contiguous run of tiles of its
// XCD (A panels shared in that XCD's L2), so a tile's epilogue stores drain while the
// next tile's first K-blocks load, instead of every CU storing, then loading, in
// lockstep rounds.  Between tiles only LDS is fenced (lgkmcnt): the stores stay in flight.
// Tile walk order.  Linear walk index t -> logical tile (M-major: mt * ntn + nt).  With
// a.pipe_g = g (a divisor of ntn, 0 < g < ntn) the walk is N-group major: the g N-panels of
// one group, M-tile by M-tile, then the next group.  An XCD's 32 CUs then hold 32/g M-tiles
// x g weight panels at a time instead of 32/ntn x ntn: fewer weight panels live per L2.
__device__ __forceinline__ int pipe_tile_map(const ConvArgs& a, int t, int ntiles) {
  const int ntn = a.cout_pad / kPBN, g = a.pipe_g;
  if (g <= 0 || g >= ntn) return t;
  const int ntm = ntiles / ntn, per_grp = ntm * g;
  const int grp = t / per_grp, r = t - grp * per_grp;
  const int mt = r / g, j = r - mt * g;
  return mt * ntn + grp * g + j;
}

template <int ABL, int BM, bool I8, bool WIN>
__device__ __forceinline__ void pipe_walk(const ConvArgs& a, unsigned char* smem_raw, int ntiles, bool pf) {
  // tiles [a.pipe_t0, ntiles)
  const int nb = gridDim.x, xcd = blockIdx.x & 7, l = blockIdx.x >> 3;
  const int cnt = ntiles - a.pipe_t0;
  const int q = cnt >> 3, r = cnt & 7;
  const int lo = a.pipe_t0 + (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q);
  const int hi = lo + q + (xcd < r ? 1 : 0);
  const int bx = (nb - xcd + 7) >> 3;  // workgroups on this XCD (>= 1: this one)
  if constexpr (WIN) {  // the zero area: written once, outside every epilogue's LDS use
    if (threadIdx.x < 64) {
      u32x4* z = reinterpret_cast<u32x4*>(smem_raw + (2 * kWinRows * kPBK + kPNS * kPBN * kPBK) * 2);
      z[threadIdx.x] = u32x4{0u, 0u, 0u, 0u};
    }
    __syncthreads();
  }
  bool pre = false;
  for (int t = lo + l; t < hi; t += bx) {
    const int nx = pf && t + bx < hi ? pipe_tile_map(a, t + bx, ntiles) : -1;
    pipe_tile<ABL, BM, I8, WIN>(a, smem_raw, pipe_tile_map(a, t, ntiles), pf, nx, pre);
    pre = nx >= 0;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  }
}
template <int BM, bool WIN>
constexpr int pipe_smem() {
  return WIN && kWinSmem > PipeCfg<BM>::Smem ? kWinSmem : PipeCfg<BM>::Smem;
}

template <int ABL, int BM>
__global__ __launch_bounds__(512, 1) void conv_pipe_f16(ConvArgs a, int ntiles, int pf) {
  __shared__ __attribute__((aligned(16))) unsigned char smem_raw[pipe_smem<BM, false>()];
  pipe_walk<ABL, BM, false, false>(a, smem_raw, ntiles, pf != 0);
}
// window mode (3x3 / s1 / p1, linear rows): see kWinRows
template <int ABL, int BM>
__global__ __launch_bounds__(512, 1) void conv_pipew_f16(ConvArgs a, int ntiles, int pf) {
  __shared__ __attribute__((aligned(16))) unsigned char smem_raw[pipe_smem<BM, true>()];
  pipe_walk<ABL, BM, false, true>(a, smem_raw, ntiles, pf != 0);
}
// int8 twins (same persistent XCD walk)
template <int ABL, int BM>
__global__ __launch_bounds__(512, 1) void conv_pipe_i8(ConvArgs a, int ntiles, int pf) {
  __shared__ __attribute__((aligned(16))) unsigned char smem_raw[pipe_smem<BM, false>()];
  pipe_walk<ABL, BM, true, false>(a, smem_raw, ntiles, pf != 0);
}
template <int ABL, int BM>
__global__ __launch_bounds__(512, 1) void conv_pipew_i8(ConvArgs a, int ntiles, int pf) {
  __shared__ __attribute__((aligned(16))) unsigned char smem_raw[pipe_smem<BM, true>()];
  pipe_walk<ABL, BM, true, true>(a, smem_raw, ntiles, pf != 0);
}

bool conv_pipe_ok(const ConvArgs& a) {
  if (!a.zero || a.in_kind != IN_NHWC || a.w_f32 || (a.in_cs | a.in_co) % 8 != 0) return false;
  if (a.cin % 64 != 0 || a.cout_pad % kPBN != 0 || (a.ks != 1 && a.ks != 3)) return false;
  if (a.kpad != a.ks * a.ks * a.cin) return false;
  const int64_t elems = (int64_t)a.n * a.ih * a.iw * a.in_cs;
  if (elems >= (1ll << 30) || (int64_t)a.cout_pad * a.kpad * 2 >= (1ll << 31)) return false;
  if (a.head_w) {  // fused head: one N tile, head K = 128, output only through the head
    if (a.cout_pad != kPBN || a.head_cout < 1 || a.head_cout > 32 || !a.head_e.io || !a.head_e.bias) return false;
    if (a.e.full.ptr || a.e.pool.ptr || a.e.up.ptr || a.e.res.ptr || a.e.io || a.quad) return false;
  }
  return true;
}

// mode (conv_pipe_mode): 1 = the kernel; 2..5 = ablation builds for diagnostics
// (tools/ab_conv.py; outputs wrong): 2 no loads, 3 no ds_reads, 4 neither, 5 no
// barrier, 6 no epilogue, 7 bare MFMA loop (no loads, reads or epilogue), 8 no K-loop,
// 9 neither K-loop nor epilogue, 10 no K-loop and no global epilogue stores (bit 64),
// 11 the generic epilogue where the lean one applies (correct outputs).
static int pipe_cus() {
  static int n = [] {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v < 1)
      v = 256;
    return v;
  }();
  return n;
}

// Tile rows per launch.  A tile of BM rows costs about BM/256 of a 256-row tile's
// K-loop at a lower per-CU rate (fewer MFMAs per LDS byte and per barrier) plus a
// fixed prologue / epilogue; the launch takes ceil(tiles / CUs) such rounds.  The
// smallest estimated time wins (ties: the larger tile).  rtdm_set_tuning("conv_pipe_bm",
// 256 | 128 | 64) forces one (0 = this model).  Batch-invariant: only the tiling changes.
static int pipe_bm_nk(const ConvArgs& a, int nk, double* est = nullptr);
int pipe_bm(const ConvArgs& a) { return pipe_bm_nk(a, a.kpad / kPBK); }
// Objective of the tile-rows model: 0 = latency (rounds of tiles over the CUs: a launch that
// has the GPU to itself), 1 = throughput (CU-time: tiles x per-tile time, for several batches
// in flight whose launches fill each other's idle CUs).  rtdm_set_tuning("conv_pipe_cost", v);
// bench.py sets 1 with more than one batch in flight.  Throughput favours 256-row tiles:
// b8 31.8k -> 33.0k, b16 36.9k -> 39.3k frames/s with 4 in flight (r03an, forced 256 rows).
static bool pipe_win_ok(const ConvArgs& a, int bm);
static bool pipe_unroll(int abl);
static int pipe_abl(const ConvArgs& a);
static int pipe_bm_nk(const ConvArgs& a, int nk, double* est) {
  const bool head = a.head_w != nullptr;
  if (est) *est = 1e300;
  if (tune().pipe_bm && !(head && tune().pipe_bm == 64)) return tune().pipe_bm;
  const int ntn = a.cout_pad / kPBN, cus = pipe_cus();
  static const int bms[3] = {256, 128, 64};
  // 256-row tiles of window-mode layers run the tap-unrolled window loop: ~1.2x the K-loop
  // rate of the per-tap-load 256-row tiles (b64 L10 / L14 on 256-row window tiles 0.0614 /
  // 0.0682 ms against 0.0664 / 0.0710 on the 128-row tiles this model picked without it, r03ak)
  // (only when that launch will run the unrolled window loop: register-epilogue layers; the
  // LDS-epilogue window layers run the cursor loop, launch_abl_w0)
  const double eff[3] = {!head && pipe_win_ok(a, 256) && pipe_unroll(pipe_abl(a)) ? 1.2 : 1.0, 0.85,
                         0.65};
  const double ovh = 3.0 + (head ? 4.0 : 0.0);
  int best = 256;
  double best_t = 1e300;
  for (int i = 0; i < (head ? 2 : 3); ++i) {
    const int64_t tiles = (int64_t)((a.M + bms[i] - 1) / bms[i]) * ntn;
    const double rounds = tune().pipe_cost ? (double)tiles : (double)((tiles + cus - 1) / cus);
    const double t = rounds * (bms[i] / 256.0 * nk / eff[i] + ovh * bms[i] / 256.0 + 1.0);
    if (t < best_t * 0.97) {
      best_t = t;
      best = bms[i];
    }
  }
  if (est) *est = best_t;
  return best;
}

static int g_pipe_korder_get() { return tune().pipe_korder; }

// Epilogue instantiation (ABL) of a launch: 8 fused head; 1024 stand-alone YOLO head
// (decode into io only, epi_vec8_io); lean layers 640 (register
// epilogue) / 128 (LDS C tile: layers with pool or upsample outputs), +256 with the fused
// shortcut add; 0 the generic epilogue.
static int pipe_abl(const ConvArgs& a) {
  if (a.head_w) return 8;
  if (epi_io_ok(a)) return 1024;
  // (pool / upsample layers: the LDS C tile; the register epilogue, which pools the
  // quad-ordered rows across lane quads by DPP, measured slower there: r02cg, r04r)
  const int reg = !a.e.pool.ptr && !a.e.up.ptr ? 512 : 0;
  if (epi_lean_ok(a)) return 128 | reg;
  if (epi_lean_ok(a, true)) return 384 | reg;
  return 0;
}

// Window mode eligibility (3x3 / s1 / p1 over a linear-order NHWC input whose window of
// BM + 2W + 2 rows fits kWinRows; channel-block-outer K order; 256-row tiles: with the
// 128-row tiles' 16 MFMAs per K-block the window addressing VALU costs more than the
// A loads it saves, measured +10 % on yolov4-tiny L10 / L14).  rtdm_set_tuning("conv_pipe_win", 0)
// turns it off (bit-identical either way).
static bool pipe_win_ok(const ConvArgs& a, int bm) {
  return tune().pipe_win && bm == 256 && a.cin % 64 == 0 && a.ks == 3 && a.stride == 1 && a.pad == 1 && !a.quad && a.pipe_corder &&
         a.ih == a.oh && a.iw == a.ow && bm + 2 * a.iw + 2 <= kWinRows &&
         (int64_t)a.n * a.ih * a.iw * a.in_cs * 2 < (1ll << 30);  // (the window op's 2^31 skip)
}

// Cross-tile prefetch (register-epilogue layers): a workgroup issues its next tile's
// prologue loads (window + K-blocks 0 .. NSt-2) right after its K-loop, before the
// epilogue, whose stores then drain under the next tile's first K-blocks instead of in
// front of them.  Needs nk >= NSt - 1 and byte offsets of the output / residual views
// below 2^31 - 16 (the epilogue's fixed-count buffer ops).  rtdm_set_tuning("conv_pipe_pf", 0)
// turns it off (bit-identical either way).

// Tile walk (pipe_tile_map): N-panels per group; 0 = the M-major walk.  rtdm_set_tuning(
// "conv_pipe_walk", g).  Bit-identical for every g (only the order tiles run in changes).
// Default 2: yolov4-tiny@608 b64 L12 (8 N-panels) fetches 39 % fewer bytes past L2 (PMC
// FETCH_SIZE, r03l) at the same time (0.2007 vs 0.2009 ms).
// 3x3 K-loops: 1 = taps unrolled (default: WLOOP for window mode, the run-time uloop path for
// the per-tap-load layers), 0 = the generic cursor loop (window mode: ABL bit 4096; A/B
// diagnostics).  rtdm_set_tuning("conv_pipe_wloop", v); bit-identical either way.
// Per epilogue (pipe_unroll): the unrolled loop for the register-epilogue layers only.  The
// LDS C-tile epilogues (pooled / upsampled outputs, ABL 128 / 384) and the fused head (ABL 8)
// measured 2-3 % slower with it at b64 (r03aa: L6 0.1047 -> 0.1081 ms, L28 0.2592 -> 0.2662):
// their kernels hold more registers across the loop and the unrolled loop's spill reloads
// land in the tile prologue.
static bool pipe_unroll(int abl) { return tune().pipe_wloop && (abl & 512) != 0; }
static int pipe_walk_g(const ConvArgs& a) {
  const int ntn = a.cout_pad / kPBN;
  return tune().pipe_walk > 0 && tune().pipe_walk < ntn && ntn % tune().pipe_walk == 0 ? tune().pipe_walk : 0;
}

static bool pipe_pf_ok(const ConvArgs& a, int abl, int nk) {
  if (!tune().pipe_pf || nk < kPNS - 1) return false;
  if (abl == 8) return true;  // fused head: prefetch after the head GEMM, before the decode
  if (!(abl & 512) || !a.e.full.ptr || a.e.pool.ptr || a.e.up.ptr || a.e.scale) return false;
  const int64_t pix = (int64_t)a.n * a.oh * a.ow;
  const int64_t lim = (1ll << 31) - 16;
  if ((pix * a.e.full.cs) * 2 >= lim) return false;
  if (a.e.res.ptr && (pix * a.e.res.cs) * 2 >= lim) return false;
  return true;
}

#define RTDM_PIPE_KERNEL(NAME)                                                                  \
  template <int ABL, int BM>                                                                    \
  struct NAME##_k {                                                                             \
    static void go(dim3 g, hipStream_t s, const ConvArgs& a, int nt, int pf) {                  \
      hipLaunchKernelGGL((NAME<ABL, BM>), g, dim3(512), 0, s, a, nt, pf);                      \
    }                                                                                           \
  };
RTDM_PIPE_KERNEL(conv_pipe_f16)
RTDM_PIPE_KERNEL(conv_pipew_f16)
RTDM_PIPE_KERNEL(conv_pipe_i8)
RTDM_PIPE_KERNEL(conv_pipew_i8)
#undef RTDM_PIPE_KERNEL

template <template <int, int> class K, int BM>
static void launch_abl(int abl, dim3 g, hipStream_t s, const ConvArgs& a, int nt, int pf) {
  switch (abl) {
    case 8:
      if constexpr (BM >= 128) K<8, BM>::go(g, s, a, nt, pf);
      break;
    case 128: K<128, BM>::go(g, s, a, nt, pf); break;
    case 384: K<384, BM>::go(g, s, a, nt, pf); break;
    case 640: K<640, BM>::go(g, s, a, nt, pf); break;
    case 896: K<896, BM>::go(g, s, a, nt, pf); break;
    case 1024: K<1024, BM>::go(g, s, a, nt, pf); break;
    default: K<0, BM>::go(g, s, a, nt, pf); break;
  }
}

// the generic-cursor window loop (ABL bit 4096), 256-row tiles only
template <template <int, int> class K, int BM>
static void launch_abl_w0(int abl, dim3 g, hipStream_t s, const ConvArgs& a, int nt, int pf) {
  if constexpr (BM == 256) {
    switch (abl) {
      case 8: K<8 | 4096, BM>::go(g, s, a, nt, pf); break;
      case 128: K<128 | 4096, BM>::go(g, s, a, nt, pf); break;
      case 384: K<384 | 4096, BM>::go(g, s, a, nt, pf); break;
      case 640: K<640 | 4096, BM>::go(g, s, a, nt, pf); break;
      case 896: K<896 | 4096, BM>::go(g, s, a, nt, pf); break;
      case 1024: K<1024 | 4096, BM>::go(g, s, a, nt, pf); break;
      default: K<4096, BM>::go(g, s, a, nt, pf); break;
    }
  }
}

template <int BM>
static void launch_pipe_bm(const ConvArgs& a, hipStream_t s, int ntiles, dim3 grid, bool win) {
  const int abl = pipe_abl(a), pf = pipe_pf_ok(a, abl, a.kpad / kPBK) ? 1 : 0;
  if constexpr (BM >= 128) {
    if (win && BM == 256 && !pipe_unroll(abl)) return launch_abl_w0<conv_pipew_f16_k, BM>(abl, grid, s, a, ntiles, pf);
    if (win) return launch_abl<conv_pipew_f16_k, BM>(abl, grid, s, a, ntiles, pf);
  }
  launch_abl<conv_pipe_f16_k, BM>(abl, grid, s, a, ntiles, pf);
}

// kernel symbol of a launch, e.g. conv_pipew_f16<640,256>; the strings live in a set (stable
// pointers)
static const char* pipe_name(bool i8, bool win, int abl, int bm) {
  static std::mutex mu;  // (handles may be planned on several threads)
  std::lock_guard<std::mutex> lk(mu);
  static std::set<std::string> names;
  char b[48];
  snprintf(b, sizeof b, "conv_pipe%s_%s<%d,%d>", win ? ((abl & 4096) ? "w0" : "w") : "", i8 ? "i8" : "f16",
           abl & ~4096, bm);
  return names.insert(b).first->c_str();
}

const char* conv_pipe_name(const ConvArgs& a_in) {
  ConvArgs a = a_in;
  a.pipe_corder = g_pipe_korder_get() && a.ks == 3 && a.cin % 64 == 0 ? 1 : 0;
  const int bm = conv_pipe_mode() > 1 && conv_pipe_mode() != 13 ? 256 : pipe_bm(a);
  const bool abl_mode = a.head_w || conv_pipe_mode() <= 1 || conv_pipe_mode() == 13;
  const bool win = abl_mode && pipe_win_ok(a, bm);
  return pipe_name(false, win, pipe_abl(a) | (win && !pipe_unroll(pipe_abl(a)) ? 4096 : 0), bm);
}

// K order of the implicit GEMM: 0 = tap outer (each tap's whole channel run), 1 = 64-channel
// block outer (the 9 taps of one channel slice back to back, so the shifted input rows
// a tap re-reads are the slice's: an L2 working set of 1/(cin/64) of the tap-outer one).
// rtdm_set_tuning("conv_pipe_korder", v).  Changes the fp32 summation order (not batch
// invariance): results differ from the other order in the last bits.

void launch_conv_pipe(const ConvArgs& a_in, hipStream_t s) {
  ConvArgs a = a_in;
  a.pipe_corder = tune().pipe_korder && a.ks == 3 && a.cin % 64 == 0 ? 1 : 0;
  a.pipe_g = pipe_walk_g(a);
  a.pipe_u = pipe_unroll(pipe_abl(a)) ? 1 : 0;
  const int bm = conv_pipe_mode() > 1 && conv_pipe_mode() != 13 ? 256 : pipe_bm(a);
  const int64_t nt = (int64_t)((a.M + bm - 1) / bm) * (a.cout_pad / kPBN);
  RTDM_REQUIRE(nt < (1ll << 31), RTDM_E_CAPACITY, "conv: grid too large");
  const int ntiles = (int)nt;
  // mode 13: one workgroup per tile (non-persistent), for A/B runs
  const int cap = conv_pipe_mode() == 13 ? ntiles : pipe_cus();
  const dim3 grid((unsigned)(ntiles < cap ? ntiles : cap));
  switch (a.head_w ? 1 : conv_pipe_mode()) {
    case 2: hipLaunchKernelGGL((conv_pipe_f16<1, 256>), grid, dim3(512), 0, s, a, ntiles, 0); break;
    case 3: hipLaunchKernelGGL((conv_pipe_f16<2, 256>), grid, dim3(512), 0, s, a, ntiles, 0); break;
    case 4: hipLaunchKernelGGL((conv_pipe_f16<3, 256>), grid, dim3(512), 0, s, a, ntiles, 0); break;
    case 5: hipLaunchKernelGGL((conv_pipe_f16<4, 256>), grid, dim3(512), 0, s, a, ntiles, 0); break;
    case 6: hipLaunchKernelGGL((conv_pipe_f16<16, 256>), grid, dim3(512), 0, s, a, ntiles, 0); break;
    case 7: hipLaunchKernelGGL((conv_pipe_f16<19, 256>), grid, dim3(512), 0, s, a, ntiles, 0); break;
    case 8: hipLaunchKernelGGL((conv_pipe_f16<32, 256>), grid, dim3(512), 0, s, a, ntiles, 0); break;
    case 9: hipLaunchKernelGGL((conv_pipe_f16<48, 256>), grid, dim3(512), 0, s, a, ntiles, 0); break;
    case 10: hipLaunchKernelGGL((conv_pipe_f16<96, 256>), grid, dim3(512), 0, s, a, ntiles, 0); break;
    case 11: hipLaunchKernelGGL((conv_pipe_f16<0, 256>), grid, dim3(512), 0, s, a, ntiles, 0); break;
    // tap-unrolled window loop ablations (diagnostics; window-mode register-epilogue layers
    // only, every other layer runs its normal kernel): 31 no LDS-DMA loads, 32 no fragment
    // reads, 33 neither, 34 no wait + barrier, 35 no window-slice loads (B loads kept), 36 no B
    // loads (window slices kept)
    case 31:
    case 32:
    case 33:
    case 34:
    case 35:
    case 36:
      if (pipe_win_ok(a, 256) && pipe_abl(a) == 640) {
        switch (conv_pipe_mode()) {
          case 31: hipLaunchKernelGGL((conv_pipew_f16<641, 256>), grid, dim3(512), 0, s, a, ntiles, 0); break;
          case 32: hipLaunchKernelGGL((conv_pipew_f16<642, 256>), grid, dim3(512), 0, s, a, ntiles, 0); break;
          case 33: hipLaunchKernelGGL((conv_pipew_f16<643, 256>), grid, dim3(512), 0, s, a, ntiles, 0); break;
          case 35: hipLaunchKernelGGL((conv_pipew_f16<640 | 8192, 256>), grid, dim3(512), 0, s, a, ntiles, 0); break;
          case 36: hipLaunchKernelGGL((conv_pipew_f16<640 | 16384, 256>), grid, dim3(512), 0, s, a, ntiles, 0); break;
          default: hipLaunchKernelGGL((conv_pipew_f16<644, 256>), grid, dim3(512), 0, s, a, ntiles, 0); break;
        }
        break;
      }
      [[fallthrough]];
    default: {
      const bool win = pipe_win_ok(a, bm);
      if (bm == 256)
        launch_pipe_bm<256>(a, s, ntiles, grid, win);
      else if (bm == 128)
        launch_pipe_bm<128>(a, s, ntiles, grid, win);
      else
        launch_pipe_bm<64>(a, s, ntiles, grid, false);
      break;
    }
  }
}

// ---- int8 (RTDM_I8): the quantised input copy is contiguous [n*ih*iw][cin] int8 ----
bool conv_pipe_i8_ok(const ConvArgs& a) {
  if (!a.zero || a.in_kind != IN_NHWC || !a.w8 || !a.deq || (a.in_cs | a.in_co) % 16 != 0) return false;
  if (a.cin % 128 != 0 || a.cout_pad % kPBN != 0 || (a.ks != 1 && a.ks != 3) || a.kpad != a.ks * a.ks * a.cin)
    return false;
  if ((int64_t)a.n * a.ih * a.iw * a.in_cs >= (1ll << 31) || (int64_t)a.cout_pad * a.kpad >= (1ll << 31)) return false;
  if (a.head_w) {
    if (a.cout_pad != kPBN || a.head_cout < 1 || a.head_cout > 32 || !a.head_e.io || !a.head_e.bias) return false;
    if (a.e.full.ptr || a.e.pool.ptr || a.e.up.ptr || a.e.res.ptr || a.e.io || a.quad) return false;
  }
  return true;
}

const char* conv_pipe_i8_name(const ConvArgs& a_in) {
  ConvArgs a = a_in;
  a.pipe_corder = tune().pipe_korder && a.ks == 3 ? 1 : 0;
  const int bm = pipe_bm_nk(a, a.kpad / 128);
  const bool win = pipe_win_ok(a, bm);
  return pipe_name(true, win, pipe_abl(a) | (win && !pipe_unroll(pipe_abl(a)) ? 4096 : 0), bm);
}

void launch_conv_pipe_i8(const ConvArgs& a_in, hipStream_t s) {
  ConvArgs a = a_in;
  RTDM_REQUIRE(conv_pipe_i8_ok(a), RTDM_E_INVALID, "conv_pipe_i8: unsupported layer");
  a.pipe_corder = tune().pipe_korder && a.ks == 3 ? 1 : 0;
  a.pipe_g = pipe_walk_g(a);
  a.pipe_u = pipe_unroll(pipe_abl(a)) ? 1 : 0;
  const int bm = pipe_bm_nk(a, a.kpad / 128);
  const int64_t nt = (int64_t)((a.M + bm - 1) / bm) * (a.cout_pad / kPBN);
  RTDM_REQUIRE(nt < (1ll << 31), RTDM_E_CAPACITY, "conv: grid too large");
  const int ntiles = (int)nt;
  const dim3 grid((unsigned)(ntiles < pipe_cus() ? ntiles : pipe_cus()));
  const bool win = pipe_win_ok(a, bm);
  const int abl = pipe_abl(a), pf = pipe_pf_ok(a, abl, a.kpad / 128) ? 1 : 0;
  if (bm == 256) {
    if (win && !pipe_unroll(abl))  // the cursor window loop, as the f16 path (launch_pipe_bm)
      launch_abl_w0<conv_pipew_i8_k, 256>(abl, grid, s, a, ntiles, pf);
    else if (win)
      launch_abl<conv_pipew_i8_k, 256>(abl, grid, s, a, ntiles, pf);
    else
      launch_abl<conv_pipe_i8_k, 256>(abl, grid, s, a, ntiles, pf);
  } else if (bm == 128) {
    if (win)
      launch_abl<conv_pipew_i8_k, 128>(abl, grid, s, a, ntiles, pf);
    else
      launch_abl<conv_pipe_i8_k, 128>(abl, grid, s, a, ntiles, pf);
  } else {
    launch_abl<conv_pipe_i8_k, 64>(abl, grid, s, a, ntiles, pf);
  }
  RTDM_HIP(hipGetLastError());
}

}  // namespace rtdm
