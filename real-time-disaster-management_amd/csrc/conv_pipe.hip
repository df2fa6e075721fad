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

#include <type_traits>

namespace rtdm {

namespace {
constexpr int kPBN = 128, kPBK = 64, kPNS = 3;
constexpr int kPCstr = kPBN + 4;
template <int BM>
struct PipeCfg {
  static constexpr int WM = BM == 256 ? 4 : 2, WN = 8 / WM;
  static constexpr int Stage = (BM + kPBN) * kPBK;  // halfs per stage
  static constexpr int Smem = kPNS * Stage * 2 > BM * kPCstr * 4 ? kPNS * Stage * 2 : BM * kPCstr * 4;
};

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
  else
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
}
}  // namespace

// Fused-head epilogue for the 4 rows m0..m0+3 of head channel c (YOLOLayer
// inference branch, models.py:252-258): bias -> activation -> decode -> io.
__device__ __forceinline__ void head_epi4(const ConvArgs& a, int m0, int c, f4 v) {
  const Epilogue& e = a.head_e;
  if (m0 >= a.M) return;
  const float bias = e.bias[c];
  const int ai = c / e.no, k = c - ai * e.no;
  const float anc = k == 2 || k == 3 ? e.anchor_vec[2 * ai + (k - 2)] : 0.f;
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
template <int ABL, int BM, bool I8 = false>
__device__ __forceinline__ void pipe_tile(const ConvArgs& a, unsigned char* smem_raw, int bid) {
  constexpr int WM = PipeCfg<BM>::WM, WN = PipeCfg<BM>::WN;
  constexpr int BN = kPBN, BK = kPBK;              // LDS row: BK halfs = 128 bytes
  constexpr int ES = I8 ? 1 : 2, BKE = I8 ? 128 : 64;  // element bytes, K-elements per K-block
  constexpr int kPStage = PipeCfg<BM>::Stage;
  constexpr int WAVES = WM * WN, NT = 64 * WAVES;
  constexpr int FM = BM / WM / 16, FN = BN / WN / 16;  // accumulators per wave
  constexpr int NA = BM * BK * 2 / (NT * 16);          // A buffer->LDS ops per thread per stage
  constexpr int NB = BN * BK * 2 / (NT * 16);          // B ops
  constexpr int VM = NA + NB;
  static_assert(VM == 6 || VM == 4 || VM == 3, "wait literal");
  _Float16* smem = reinterpret_cast<_Float16*>(smem_raw);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WN, wn = wid % WN;
  const int ntn = a.cout_pad / BN;
  const int mt = bid / ntn;
  const int m_base = mt * BM, n_base = (bid - mt * ntn) * BN;

  // Epilogue channel constants, loaded at the tile's start so their latency hides under
  // the K-loop.  Lean epilogue: this thread's 8 channels are the same in both of its
  // units (NT % CG == 0).  Fused head: the FN columns of this lane's accumulators.
  constexpr int CG = BN / 8;
  float lb[8], ls[8], lh[8];
  if constexpr ((ABL & 128) != 0) {
    const int c0 = n_base + (tid % CG) * 8;
    const bool cv = c0 < a.cout;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      lb[j] = cv ? a.e.bias[c0 + j] : 0.f;
      ls[j] = cv && a.e.scale ? a.e.scale[c0 + j] : 1.f;
      lh[j] = cv && a.e.scale ? a.e.shift[c0 + j] : 0.f;
    }
  }
  float dq[FN];  // int8: per-output-channel dequantisation of this lane's accumulator columns
  if constexpr (I8) {
#pragma unroll
    for (int tn = 0; tn < FN; ++tn) {
      const int col = n_base + wn * (BN / WN) + tn * 16 + (lane & 15);
      dq[tn] = col < a.cout ? a.deq[col] : 0.f;
    }
  }
  float hb[FN], hs[FN], hh[FN];
  if constexpr ((ABL & 8) != 0) {
#pragma unroll
    for (int tn = 0; tn < FN; ++tn) {
      const int col = wn * (BN / WN) + tn * 16 + (lane & 15);
      const bool cv = col < a.cout;
      hb[tn] = cv ? a.e.bias[col] : 0.f;
      hs[tn] = (cv && a.e.scale) ? a.e.scale[col] : 1.f;
      hh[tn] = (cv && a.e.scale) ? a.e.shift[col] : 0.f;
    }
  }

  // ---- per-lane staging state.  A op j of wave w fills tile rows 8(NA w + j) + lane/8,
  //      B op j rows 8(NB w + j) + lane/8; LDS slot lane%8 of a row holds k-vector
  //      slot ^ ((row >> 1) & 7) (the read side applies the same involution). ----
  const int slot = lane & 7;
  int voff_a[NA];
  uint32_t vmask[NA];
#pragma unroll
  for (int j = 0; j < NA; ++j) {
    const int r = 8 * (NA * wid + j) + (lane >> 3);
    const int kofs = 16 * (slot ^ ((r >> 1) & 7));  // bytes
    const int m = m_base + r;
    int n = 0, oy = 0, ox = 0;
    if (m < a.M) row_to_pix(a, m, n, oy, ox);
    const int iy0 = m < a.M ? oy * a.stride - a.pad : -(1 << 28);
    const int ix0 = ox * a.stride - a.pad;
    voff_a[j] = m < a.M ? (n * a.ih * a.iw + iy0 * a.iw + ix0) * a.in_cs * ES + kofs : 0;
    uint32_t msk = 0;
    for (int t = 0; t < a.ks * a.ks; ++t) {
      const int kh = a.ks == 3 ? (t * 11) >> 5 : 0, kw = t - kh * a.ks;
      const int iy = iy0 + kh, ix = ix0 + kw;
      if ((unsigned)iy < (unsigned)a.ih && (unsigned)ix < (unsigned)a.iw) msk |= 1u << t;
    }
    vmask[j] = msk;
  }
  int voff_b[NB];
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    const int r = 8 * (NB * wid + j) + (lane >> 3);
    voff_b[j] = r * a.kpad * ES + 16 * (slot ^ ((r >> 1) & 7));
  }
  const char* in = (const char*)a.in + (size_t)a.in_co * ES;
  const int64_t in_bytes = ((int64_t)a.n * a.ih * a.iw * a.in_cs - a.in_co) * ES;
  const __amdgpu_buffer_rsrc_t rs_in = __builtin_amdgcn_make_buffer_rsrc((void*)in, 0, (int)in_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rs_w = __builtin_amdgcn_make_buffer_rsrc(
      (void*)((const char*)(I8 ? a.w8 : a.w) + (size_t)n_base * a.kpad * ES), 0, BN * a.kpad * ES, 0x00020000);
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

  // Issue the VM buffer->LDS ops of the next K-block (cursor st_*) into stage st_buf.
  auto stage = [&]() {
    _Float16* As = smem + st_buf * kPStage;
    _Float16* Bs = As + BM * BK;
    const int st_tap = __builtin_amdgcn_readfirstlane(corder ? st_i : st_o);
    const int st_c = __builtin_amdgcn_readfirstlane(corder ? st_o : st_i);
    const int kh = a.ks == 3 ? (st_tap * 11) >> 5 : 0, kw = st_tap - kh * a.ks;
    const int tapoff = ((kh * a.iw + kw) * a.in_cs + st_c * BKE) * ES;
#pragma unroll
    for (int j = 0; j < NA; ++j) {
      const int vo = ((vmask[j] >> st_tap) & 1u) ? voff_a[j] + tapoff : (int)0x80000000;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs_in, (lds_ptr_t)(As + 8 * (NA * wid + j) * BK), 16, vo, 0, 0, 0);
    }
    const int koff = (st_tap * a.cin + st_c * BKE) * ES;  // weight column of this K-block (tap-major packing)
#pragma unroll
    for (int j = 0; j < NB; ++j)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs_w, (lds_ptr_t)(Bs + 8 * (NB * wid + j) * BK), 16, voff_b[j], koff,
                                               0, 0);
    if (++st_i == ni) {
      st_i = 0;
      ++st_o;
    }
    st_buf = st_buf == kPNS - 1 ? 0 : st_buf + 1;
  };

  const int fr = lane & 15, g = lane >> 4;
  const int rsw = (fr >> 1) & 7;
  const int so0 = 8 * ((0 + g) ^ rsw), so1 = 8 * ((4 + g) ^ rsw);
  const int a_row = (wm * (BM / WM) + fr) * BK, b_row = (BM + wn * (BN / WN) + fr) * BK;

  typedef int i32x4 __attribute__((ext_vector_type(4)));
  using AccT = std::conditional_t<I8, i32x4, f4>;
  AccT acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = AccT{0, 0, 0, 0};
  auto mfma = [&](const h8& x, const h8& y, AccT c) -> AccT {
    if constexpr (I8)
      return __builtin_amdgcn_mfma_i32_16x16x64_i8(__builtin_bit_cast(i32x4, x), __builtin_bit_cast(i32x4, y), c, 0, 0,
                                                   0);
    else
      return __builtin_amdgcn_mfma_f32_16x16x32_f16(x, y, c, 0, 0, 0);
  };

  h8 fa0[FM], fb0[FN], fa1[FM], fb1[FN];
  auto read0 = [&](int buf) {
    const _Float16* S = smem + buf * kPStage;
#pragma unroll
    for (int t = 0; t < FM; ++t) fa0[t] = *(const h8*)(S + a_row + t * 16 * BK + so0);
#pragma unroll
    for (int t = 0; t < FN; ++t) fb0[t] = *(const h8*)(S + b_row + t * 16 * BK + so0);
  };
  auto read1 = [&](int buf) {
    const _Float16* S = smem + buf * kPStage;
#pragma unroll
    for (int t = 0; t < FM; ++t) fa1[t] = *(const h8*)(S + a_row + t * 16 * BK + so1);
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

  // prologue: K-blocks 0 and 1 in flight, wait for 0
  stage();
  if (nk > 1) {
    stage();
    wait_vm_lgkm0<VM>();
  } else {
    wait_vm_lgkm0<0>();
  }
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
  read0(0);

  // Cluster A (half 0 of kb): MFMAs on fa0/fb0, interleaved with the reads of half 1
  // (fa1/fb1) and the buffer->LDS loads of kb+2.  Cluster B (half 1): MFMAs on
  // fa1/fb1, interleaved with the reads of half 0 of kb+1 (after the barrier that
  // publishes kb+1).  The loop is peeled so the steady-state body is one basic
  // block (interleave groups do not cross branches): STG = loads of kb+2 go out,
  // NXT = kb+1 exists (wait for it, barrier, read its half 0).
  int cur = 0;
  auto body = [&](auto stg, auto nxt_c) {
    constexpr bool STG = decltype(stg)::value, NXT = decltype(nxt_c)::value;
    const int nxt = cur == kPNS - 1 ? 0 : cur + 1;
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
    if constexpr (NXT) {
      // retire kb+1 (kb+2 stays in flight); lgkmcnt(0): this stage's reads are done
      // in every wave before any wave restages it (kb+3, issued after this barrier)
      if constexpr (!(ABL & 4)) {
        if constexpr (STG)
          wait_vm_lgkm0<VM>();
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
  if constexpr (!(ABL & 32)) {
    for (int kb = 0; kb + 2 < nk; ++kb) body(T_{}, T_{});
    if (nk >= 2) body(F_{}, T_{});
    body(F_{}, F_{});
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
    const _Float16* hw = (const _Float16*)a.head_w;  // [32][128]
#pragma unroll
    for (int ks = 0; ks < BN / 32; ++ks) {
      h8 af[HT], bf[2];
#pragma unroll
      for (int t = 0; t < HT; ++t) {
        const int row = HR * wid + 16 * t + fr;
        af[t] = *(const h8*)(Hs + row * BN + 8 * ((4 * ks + g) ^ (row & 15)));
      }
#pragma unroll
      for (int t = 0; t < 2; ++t) bf[t] = *(const h8*)(hw + (16 * t + fr) * BN + 32 * ks + 8 * g);
#pragma unroll
      for (int tm = 0; tm < HT; ++tm)
#pragma unroll
        for (int tq = 0; tq < 2; ++tq)
          hacc[tm][tq] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[tm], bf[tq], hacc[tm][tq], 0, 0, 0);
    }
#pragma unroll
    for (int tm = 0; tm < HT; ++tm)
#pragma unroll
      for (int tq = 0; tq < 2; ++tq) {
        const int c = 16 * tq + fr;
        if (c < a.head_cout) head_epi4(a, m_base + HR * wid + 16 * tm + 4 * g, c, hacc[tm][tq]);
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
    else
      epi_vec8(a, m0, c0, v);
  }
}

// Persistent over tiles: one workgroup per CU walks a contiguous run of tiles of its
// XCD (A panels shared in that XCD's L2), so a tile's epilogue stores drain while the
// next tile's first K-blocks load, instead of every CU storing, then loading, in
// lockstep rounds.  Between tiles only LDS is fenced (lgkmcnt): the stores stay in flight.
template <int ABL, int BM>
__global__ __launch_bounds__(512, 1) void conv_pipe_f16(ConvArgs a, int ntiles) {
  __shared__ __attribute__((aligned(16))) unsigned char smem_raw[PipeCfg<BM>::Smem];
  const int nb = gridDim.x, xcd = blockIdx.x & 7, l = blockIdx.x >> 3;
  const int q = ntiles >> 3, r = ntiles & 7;
  const int lo = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  const int hi = lo + q + (xcd < r ? 1 : 0);
  const int bx = (nb - xcd + 7) >> 3;  // workgroups on this XCD (>= 1: this one)
  for (int t = lo + l; t < hi; t += bx) {
    pipe_tile<ABL, BM>(a, smem_raw, t);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  }
}


// int8 twin of conv_pipe_f16 (same persistent XCD walk)
template <int ABL, int BM>
__global__ __launch_bounds__(512, 1) void conv_pipe_i8(ConvArgs a, int ntiles) {
  __shared__ __attribute__((aligned(16))) unsigned char smem_raw[PipeCfg<BM>::Smem];
  const int nb = gridDim.x, xcd = blockIdx.x & 7, l = blockIdx.x >> 3;
  const int q = ntiles >> 3, r = ntiles & 7;
  const int lo = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  const int hi = lo + q + (xcd < r ? 1 : 0);
  const int bx = (nb - xcd + 7) >> 3;
  for (int t = lo + l; t < hi; t += bx) {
    pipe_tile<ABL, BM, true>(a, smem_raw, t);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  }
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
static int g_pipe_bm = 0;
void set_pipe_bm(int v) { g_pipe_bm = (v == 256 || v == 128 || v == 64) ? v : 0; }
static int pipe_bm_nk(const ConvArgs& a, int nk);
int pipe_bm(const ConvArgs& a) { return pipe_bm_nk(a, a.kpad / kPBK); }
static int pipe_bm_nk(const ConvArgs& a, int nk) {
  const bool head = a.head_w != nullptr;
  if (g_pipe_bm && !(head && g_pipe_bm == 64)) return g_pipe_bm;
  const int ntn = a.cout_pad / kPBN, cus = pipe_cus();
  static const int bms[3] = {256, 128, 64};
  static const double eff[3] = {1.0, 0.85, 0.65};
  const double ovh = 3.0 + (head ? 4.0 : 0.0);
  int best = 256;
  double best_t = 1e300;
  for (int i = 0; i < (head ? 2 : 3); ++i) {
    const int64_t tiles = (int64_t)((a.M + bms[i] - 1) / bms[i]) * ntn;
    const double rounds = (double)((tiles + cus - 1) / cus);
    const double t = rounds * (bms[i] / 256.0 * nk / eff[i] + ovh * bms[i] / 256.0 + 1.0);
    if (t < best_t * 0.97) {
      best_t = t;
      best = bms[i];
    }
  }
  return best;
}

template <int BM>
static void launch_pipe_bm(const ConvArgs& a, hipStream_t s, int ntiles, dim3 grid) {
  if (a.head_w) {
    if constexpr (BM >= 128) hipLaunchKernelGGL((conv_pipe_f16<8, BM>), grid, dim3(512), 0, s, a, ntiles);
  } else if (epi_lean_ok(a)) {
    hipLaunchKernelGGL((conv_pipe_f16<128, BM>), grid, dim3(512), 0, s, a, ntiles);
  } else if (epi_lean_ok(a, true)) {
    hipLaunchKernelGGL((conv_pipe_f16<384, BM>), grid, dim3(512), 0, s, a, ntiles);
  } else {
    hipLaunchKernelGGL((conv_pipe_f16<0, BM>), grid, dim3(512), 0, s, a, ntiles);
  }
}

const char* conv_pipe_name(const ConvArgs& a) {
  const int bm = pipe_bm(a);
  if (a.head_w) return bm == 256 ? "conv_pipe_f16<8,256>" : "conv_pipe_f16<8,128>";
  if (epi_lean_ok(a)) return bm == 256 ? "conv_pipe_f16<128,256>" : bm == 128 ? "conv_pipe_f16<128,128>" : "conv_pipe_f16<128,64>";
  if (epi_lean_ok(a, true))
    return bm == 256 ? "conv_pipe_f16<384,256>" : bm == 128 ? "conv_pipe_f16<384,128>" : "conv_pipe_f16<384,64>";
  return bm == 256 ? "conv_pipe_f16<0,256>" : bm == 128 ? "conv_pipe_f16<0,128>" : "conv_pipe_f16<0,64>";
}

// K order of the implicit GEMM: 0 = tap outer (each tap's whole channel run), 1 = 64-channel
// block outer (the 9 taps of one channel slice back to back, so the shifted input rows
// a tap re-reads are the slice's: an L2 working set of 1/(cin/64) of the tap-outer one).
// rtdm_set_tuning("conv_pipe_korder", v).  Changes the fp32 summation order (not batch
// invariance): results differ from the other order in the last bits.
static int g_pipe_korder = 1;
void set_pipe_korder(int v) { g_pipe_korder = v ? 1 : 0; }

void launch_conv_pipe(const ConvArgs& a_in, hipStream_t s) {
  ConvArgs a = a_in;
  a.pipe_corder = g_pipe_korder && a.ks == 3 ? 1 : 0;
  const int bm = conv_pipe_mode() > 1 && conv_pipe_mode() != 13 ? 256 : pipe_bm(a);
  const int64_t nt = (int64_t)((a.M + bm - 1) / bm) * (a.cout_pad / kPBN);
  RTDM_REQUIRE(nt < (1ll << 31), RTDM_E_CAPACITY, "conv: grid too large");
  const int ntiles = (int)nt;
  // mode 13: one workgroup per tile (non-persistent), for A/B runs
  const int cap = conv_pipe_mode() == 13 ? ntiles : pipe_cus();
  const dim3 grid((unsigned)(ntiles < cap ? ntiles : cap));
  switch (a.head_w ? 1 : conv_pipe_mode()) {
    case 2: hipLaunchKernelGGL((conv_pipe_f16<1, 256>), grid, dim3(512), 0, s, a, ntiles); break;
    case 3: hipLaunchKernelGGL((conv_pipe_f16<2, 256>), grid, dim3(512), 0, s, a, ntiles); break;
    case 4: hipLaunchKernelGGL((conv_pipe_f16<3, 256>), grid, dim3(512), 0, s, a, ntiles); break;
    case 5: hipLaunchKernelGGL((conv_pipe_f16<4, 256>), grid, dim3(512), 0, s, a, ntiles); break;
    case 6: hipLaunchKernelGGL((conv_pipe_f16<16, 256>), grid, dim3(512), 0, s, a, ntiles); break;
    case 7: hipLaunchKernelGGL((conv_pipe_f16<19, 256>), grid, dim3(512), 0, s, a, ntiles); break;
    case 8: hipLaunchKernelGGL((conv_pipe_f16<32, 256>), grid, dim3(512), 0, s, a, ntiles); break;
    case 9: hipLaunchKernelGGL((conv_pipe_f16<48, 256>), grid, dim3(512), 0, s, a, ntiles); break;
    case 10: hipLaunchKernelGGL((conv_pipe_f16<96, 256>), grid, dim3(512), 0, s, a, ntiles); break;
    case 11: hipLaunchKernelGGL((conv_pipe_f16<0, 256>), grid, dim3(512), 0, s, a, ntiles); break;
    default:
      if (bm == 256)
        launch_pipe_bm<256>(a, s, ntiles, grid);
      else if (bm == 128)
        launch_pipe_bm<128>(a, s, ntiles, grid);
      else
        launch_pipe_bm<64>(a, s, ntiles, grid);
      break;
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

const char* conv_pipe_i8_name(const ConvArgs& a) {
  const int bm = pipe_bm_nk(a, a.kpad / 128);
  if (a.head_w) return bm == 256 ? "conv_pipe_i8<8,256>" : "conv_pipe_i8<8,128>";
  if (epi_lean_ok(a)) return bm == 256 ? "conv_pipe_i8<128,256>" : bm == 128 ? "conv_pipe_i8<128,128>" : "conv_pipe_i8<128,64>";
  if (epi_lean_ok(a, true))
    return bm == 256 ? "conv_pipe_i8<384,256>" : bm == 128 ? "conv_pipe_i8<384,128>" : "conv_pipe_i8<384,64>";
  return bm == 256 ? "conv_pipe_i8<0,256>" : bm == 128 ? "conv_pipe_i8<0,128>" : "conv_pipe_i8<0,64>";
}

template <int BM>
static void launch_pipe_i8_bm(const ConvArgs& a, hipStream_t s, int ntiles, dim3 grid) {
  if (a.head_w) {
    if constexpr (BM >= 128) hipLaunchKernelGGL((conv_pipe_i8<8, BM>), grid, dim3(512), 0, s, a, ntiles);
  } else if (epi_lean_ok(a)) {
    hipLaunchKernelGGL((conv_pipe_i8<128, BM>), grid, dim3(512), 0, s, a, ntiles);
  } else if (epi_lean_ok(a, true)) {
    hipLaunchKernelGGL((conv_pipe_i8<384, BM>), grid, dim3(512), 0, s, a, ntiles);
  } else {
    hipLaunchKernelGGL((conv_pipe_i8<0, BM>), grid, dim3(512), 0, s, a, ntiles);
  }
}

void launch_conv_pipe_i8(const ConvArgs& a_in, hipStream_t s) {
  ConvArgs a = a_in;
  RTDM_REQUIRE(conv_pipe_i8_ok(a), RTDM_E_INVALID, "conv_pipe_i8: unsupported layer");
  a.pipe_corder = g_pipe_korder && a.ks == 3 ? 1 : 0;
  const int bm = pipe_bm_nk(a, a.kpad / 128);
  const int64_t nt = (int64_t)((a.M + bm - 1) / bm) * (a.cout_pad / kPBN);
  RTDM_REQUIRE(nt < (1ll << 31), RTDM_E_CAPACITY, "conv: grid too large");
  const int ntiles = (int)nt;
  const dim3 grid((unsigned)(ntiles < pipe_cus() ? ntiles : pipe_cus()));
  if (bm == 256)
    launch_pipe_i8_bm<256>(a, s, ntiles, grid);
  else if (bm == 128)
    launch_pipe_i8_bm<128>(a, s, ntiles, grid);
  else
    launch_pipe_i8_bm<64>(a, s, ntiles, grid);
  RTDM_HIP(hipGetLastError());
}

}  // namespace rtdm
