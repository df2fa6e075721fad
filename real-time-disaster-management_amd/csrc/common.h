// Shared definitions for the rtdm HIP runtime (gfx950 / CDNA4 only).
#pragma once

#include <hip/hip_runtime.h>
#include <hip/hip_fp16.h>

#include <cstdint>
#include <cstdio>
#include <memory>
#include <string>
#include <vector>

#include "../../include/rtdm.h"

namespace rtdm {

// ---------------------------------------------------------------- errors ----
void set_error(const std::string& msg);
const char* get_error();

struct Error {
  rtdm_status code;
  std::string msg;
};

#define RTDM_HIP(expr)                                                                     \
  do {                                                                                     \
    hipError_t e__ = (expr);                                                               \
    if (e__ != hipSuccess)                                                                 \
      throw ::rtdm::Error{RTDM_E_HIP, std::string(#expr) + ": " + hipGetErrorString(e__)}; \
  } while (0)

#define RTDM_REQUIRE(cond, code, msg)                       \
  do {                                                      \
    if (!(cond)) throw ::rtdm::Error{(code), (msg)};        \
  } while (0)

// Runs f, converting exceptions into a status + thread-local message.
template <class F>
rtdm_status guard(F&& f) {
  try {
    f();
    return RTDM_OK;
  } catch (const Error& e) {
    set_error(e.msg);
    return e.code;
  } catch (const std::bad_alloc&) {
    set_error("host allocation failed");
    return RTDM_E_OOM;
  } catch (const std::exception& e) {
    set_error(e.what());
    return RTDM_E_INVALID;
  }
}

// ------------------------------------------------------------- device mem ----
// Owning device allocation (hipMalloc); freed in the destructor.
struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
  DevBuf() = default;
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
  ~DevBuf() {
    if (p) (void)hipFree(p);
  }
  void reset() {
    if (p) (void)hipFree(p);
    p = nullptr;
    bytes = 0;
  }
  void alloc(size_t n) {
    reset();
    if (n == 0) n = 16;
    hipError_t e = hipMalloc(&p, n);
    if (e != hipSuccess) throw Error{RTDM_E_OOM, "hipMalloc(" + std::to_string(n) + ") failed"};
    bytes = n;
  }
  template <class T>
  T* as() const {
    return reinterpret_cast<T*>(p);
  }
};

__host__ __device__ inline int64_t round_up(int64_t x, int64_t m) { return (x + m - 1) / m * m; }

// ------------------------------------------------------------ activations ----
enum Act : int { ACT_LINEAR = 0, ACT_LEAKY = 1, ACT_SWISH = 2 };

// Input element kinds for conv / stem kernels.
enum InKind : int {
  IN_NHWC = 0,     // activation buffer, NHWC with channel stride/offset, element = dtype
  IN_FRAME_U8 = 1, // uint8 NHWC RGB frame, value = u8 / 255.f   (detect.py:80-82)
  IN_NCHW_F32 = 2, // fp32 NCHW model input tensor
  IN_NCHW_F16 = 3  // fp16 NCHW model input tensor
};

// A view of an NHWC activation tensor living inside a (possibly wider) buffer:
// element (n,y,x,c) is at ptr[((n*H + y)*W + x)*cs + co + c].
struct View {
  void* ptr = nullptr;
  int cs = 0;  // channel stride (elements per pixel in the buffer)
  int co = 0;  // channel offset inside the pixel
};

// Epilogue of a convolution-as-GEMM.  Per output element (pixel m, channel c):
//   v = acc + bias[c]; v = act(v); v = v*scale[c] + shift[c] (opt);
//   v += residual(m, c) (opt); store to full / 2x2-max-pooled / x2-upsampled
//   views and/or YOLO-decode it into io.
struct Epilogue {
  const float* bias = nullptr;
  const float* scale = nullptr;
  const float* shift = nullptr;
  int act = ACT_LINEAR;
  float slope = 0.f;
  View res;   // residual (shortcut), same geometry as the full-res output
  View full;  // full-resolution output
  View pool;  // 2x2 stride-2 max pooled output (requires quad ordering)
  View up;    // nearest x2 upsampled output
  // YOLO decode into io [n, io_rows, no] (YOLOLayer inference branch, models.py:252-258)
  float* io = nullptr;
  int io_rows = 0, io_off = 0, na = 0, no = 0;
  float ystride = 0.f;
  const float* anchor_vec = nullptr;  // device [na][2]: anchors / stride, fp32 like models.py:431
  // raw = 1: write the head conv's output itself (no decode) into the io rows: the
  // YOLOLayer training-branch p (models.py:249-250) that the TensorRT plugin decodes
  int raw = 0;
};

// Branch-free unsigned division by a runtime-invariant divisor (round-up
// multiplier, Hacker's Delight 10-8 / libdivide u32 "add" variant): valid for
// 0 <= n < 2^31.  Built on the host, 4-5 VALU ops on the device.
struct FastDiv {
  uint32_t m = 0;
  int l = 0;  // ceil(log2 d)
  int d = 1;
};
inline FastDiv make_fastdiv(int d) {
  FastDiv f;
  f.d = d < 1 ? 1 : d;
  int l = 0;
  while ((1ll << l) < f.d) ++l;
  f.l = l;
  f.m = l == 0 ? 0u : (uint32_t)(((((uint64_t)1 << 32) * (((uint64_t)1 << l) - (uint64_t)f.d)) / (uint64_t)f.d) + 1);
  return f;
}
__device__ __forceinline__ int fdiv(int n, const FastDiv& f) {
  if (f.l == 0) return n;
  const uint32_t t = __umulhi((uint32_t)n, f.m);
  return (int)((t + (((uint32_t)n - t) >> 1)) >> (f.l - 1));
}

// XCD-contiguous work order.  The dispatcher deals blockIdx round-robin over the 8 XCDs
// (XCD = blockIdx % 8); these maps give each XCD one contiguous run of the logical order,
// so neighbouring tiles / row bands (whose halos overlap) share that XCD's L2 instead of
// each XCD fetching the shared rows from HBM.
// One logical block per launched block (a bijection of [0, nb)):
__device__ __forceinline__ int xcd_block(int bid, int nb) {
  const int x = bid & 7, q = nb >> 3, r = nb & 7;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (bid >> 3);
}
// Persistent blocks over ntiles tiles: block bid walks first, first + step, ... < end.
// Every XCD that owns tiles has a block when nb >= 8 or ntiles <= nb; otherwise the plain
// grid-stride order.
__device__ __forceinline__ void xcd_span(int bid, int nb, int ntiles, int& first, int& end, int& step) {
  if (nb < 8 && ntiles > nb) {
    first = bid, end = ntiles, step = nb;
    return;
  }
  const int x = bid & 7, q = ntiles >> 3, r = ntiles & 7;
  const int lo = x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q;
  first = lo + (bid >> 3);
  end = lo + q + (x < r ? 1 : 0);
  step = (nb - x + 7) >> 3;
}

// Between an accumulation chain's MFMA of one opcode and its next link of ANOTHER opcode that
// reads the first one's accumulator as SrcC (the stem's 16x16x32 -> 16x16x16 chain).  The
// compiler's hazard model inserts no wait states for a full-register SrcC overlap whatever the
// opcodes, and back to back the 16-deep link read a stale accumulator: NaN / wrong values in
// round 4 (the swish stem, the channel-major stem).  sched_barrier keeps every chain's first
// link before the fence and every second link after it.  With several chains (NTN > 1) at
// least one independent MFMA sits between a chain's two links; with a single chain (the
// non-pooled stem at NTN == 1: the classifiers' conv1, conv_stem3<false, 1, k16>) the two
// s_nop 7 (16 wait states) are the ONLY guard.  16 covers the gfx950 requirement for an XDL
// write followed by a SrcC read of a different opcode (the 16-pass 32-deep link's latency):
// do not lower the nop count or lengthen the first link's MFMA shape without re-checking
// tests/test_gpu_stem.py, which asserts bit-identity for that single-chain stem.
constexpr int kMfmaOpcodeSwitchWaitStates = 16;  // the two s_nop 7 below (8 wait states each)
__device__ __forceinline__ void mfma_opcode_switch() {
  static_assert(kMfmaOpcodeSwitchWaitStates == 2 * 8, "keep the s_nop count in step with the hazard note");
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_nop 7\n\ts_nop 7" ::);
  __builtin_amdgcn_sched_barrier(0);
}

// Tuning knobs (rtdm_set_tuning keys in api.cpp): kernel-choice / A/B switches and the
// cost-model objectives.  default_tuning() holds the process defaults; a detector / classifier
// handle copies them when it is created (rtdm_*_set_tuning changes its own copy), and every
// call on a handle runs under a TuningScope of the handle's set, so two handles in one process
// can differ (e.g. a latency pipeline and a throughput pipeline).  tune() is the active set
// (the calling thread's scope, else the defaults).
struct Tuning {
  int conv_pipe = 1;        // conv_pipe mode (1 the kernels; 0 off; > 1 diagnostics, conv_pipe.hip)
  int stem_abl = 0;         // conv_stem3 ablations (diagnostics)
  int head1x1 = 1;          // stand-alone YOLO head convs on head1x1_f16
  int pipe_bm = 0;          // conv_pipe tile rows: 0 cost model, else forced 256 / 128 / 64
  int pipe_cost = 0;        // conv_pipe tile objective: 0 latency (rounds), 1 throughput (CU-time)
  int pipe_korder = 1;      // conv_pipe K order: 0 tap outer, 1 channel-block outer
  int pipe_win = 1;         // conv_pipe window mode
  int pipe_pf = 1;          // conv_pipe cross-tile prologue prefetch
  int pipe_walk = 2;        // conv_pipe tile walk: N-panels per group (0 = M-major)
  int pipe_wloop = 1;       // conv_pipe tap-unrolled 3x3 K-loops
  int dw3_tile = 1;         // YOLO-ACFF depthwise on the LDS-tiled kernel (1) or the vector one (0)
  int resize_stream = 1;    // classifier preprocessing kernel
  int nms_split = 1;        // NMS: bitmask + scan of <= 512-candidate images in two more launches (0: one launch)
  int nms_variant = 0;      // NMS diagnostics
  int acff_persist = 1;     // acff_persist for the large-map ACFF stages (> 1: ablations)
  int acff_chain = 1;       // acff_chain for the small-map suffix
  int acff_band = 0;        // acff_band for the small-map stages + tail (fp16 handles; before acff_chain; 2: only the chain's stages). Off: -2.5 % in the b64 bench, neutral at b8 (r06c)
  int acff_band_rows = 2;   // acff_band output rows per workgroup (non-tail stages)
  int fuse_head = 0;        // fused YOLO head convs (plan time; 0: the 3x3 on the unrolled window kernel + head1x1_f16, measured faster r04h)
  int two_streams = 1;      // detector head branches on a second stream (plan time)
  int pool_sep = 1;         // separable stride-1 max pools (K 5 / 9 / 13: the SPP block)
  int pool_small64 = 1;     // conv3_pool_small for 3x3 Cin 64 -> 128 + pool (+ full map)
  int pool_small_pf = 0;    // conv3_pool_small halo tiles in flight per block (0 auto | 1 | 2)
  int stem_k16 = 1;         // pooled MFMA stem: the kh = 2 third of K as a 16-deep MFMA (0: 32-deep)
  int conv_c32 = 1;         // conv3_c32 for the Cin-32 3x3 convs (conv_c32.hip)
  int res_fuse = 1;         // conv3_c32r (+ conv3_c64r): Darknet-53's residual blocks as one launch (1: c32r on 8 waves + c64r, 2: c32r on 4 waves, 3: c32r on 8 waves only)
  int cls_front = 1;        // classifier uint8 frames: CLI transform + conv1 in one launch (0: two launches)
};
Tuning& default_tuning();
const Tuning& tune();
struct TuningScope {
  explicit TuningScope(const Tuning* t);
  ~TuningScope();
  TuningScope(const TuningScope&) = delete;
  TuningScope& operator=(const TuningScope&) = delete;
  const Tuning* prev;
};
// key -> knob (RTDM_E_INVALID on an unknown key)
void tuning_set(Tuning& t, const char* key, int value);
// keys read only when a detector handle is planned (fuse_head, two_streams): a created
// handle refuses them (rtdm_detector_set_tuning), they apply through rtdm_set_tuning
bool tuning_is_plan_time(const char* key);

struct ConvArgs {
  const void* in = nullptr;
  int in_cs = 0, in_co = 0, in_kind = IN_NHWC;
  int n = 0, ih = 0, iw = 0, cin = 0;
  int ks = 1, stride = 1, pad = 0;
  int oh = 0, ow = 0, cout = 0;
  int quad = 0;  // M ordering: 1 => groups of 4 rows are 2x2 pixel quads
  int qh = 0, qw = 0;
  int M = 0;     // rows of the implicit GEMM
  FastDiv fd_ow, fd_oh, fd_qw, fd_qh;  // set by conv_set_rows
  const void* w = nullptr;  // packed weights [cout_pad][kpad], k = (kh*ks+kw)*cin + c
  int kpad = 0, cout_pad = 0;
  int w_f32 = 0;            // weights packed fp32 for the VALU body (else fp16 MFMA layout)
  const void* w_stem = nullptr;  // MFMA stem (Cin=3, 3x3): fp16 [cout_pad][64] (pack_stem)
  const void* zero = nullptr;    // >= 16 zero bytes in device memory (glds padding source)
  FastDiv fd_cin;                // set by conv_set_rows
  FastDiv fd_tx, fd_ty;          // conv3_pool_small: tiles per row / per column (set at its launch)
  int glds_uni = 0;              // conv_glds_f16: uniform-tap staging (set by launch_conv)
  int pipe_corder = 0;           // conv_pipe_f16: channel-block-outer K order (set by launch_conv_pipe)
  int pipe_g = 0;                // conv_pipe: N-panels per tile-walk group (0: M-major walk; set at launch)
  int pipe_u = 1;                // conv_pipe: tap-unrolled loop for the per-tap-load 3x3 layers (set at launch)
  int pipe_t0 = 0;               // conv_pipe: first tile of the launch
  Epilogue e;
  // Fused YOLO head (conv_pipe_f16 only): a 1x1 conv over this conv's activated
  // output (cout <= 128 = one N tile), head_w fp16 [head_cout_pad][cout_pad] (k = c),
  // applied in the epilogue with head_e (bias, activation, YOLO decode into io);
  // this conv's own output is then never written.
  const void* head_w = nullptr;
  int head_cout = 0;
  Epilogue head_e;
  // int8 path (conv_pipe_i8): int8 weights [cout_pad][kpad] with the input's per-channel
  // activation scales folded in, per-output-channel dequantisation deq[o] = s_w[o]
  const void* w8 = nullptr;
  const float* deq = nullptr;
};

// Launchers (conv.hip).  dtype = RTDM_F16 / RTDM_F32 (activation + weight type).
void launch_conv(const ConvArgs& a, int dtype, hipStream_t s);
// conv_i8.hip: int8 calibration (per-channel |x|max of an fp16 view, float bits) and the
// per-channel quantisation of an fp16 view into a contiguous int8 copy
void launch_chan_absmax(View v, int n, int h, int w, int c, unsigned* out, hipStream_t s);
void launch_quantize(View v, int n, int h, int w, int c, const float* inv_scale, int8_t* q, hipStream_t s);
// conv_pipe.hip: pipelined 256x128 implicit GEMM for Cin % 64 == 0 layers
bool conv_pipe_ok(const ConvArgs& a);
void launch_conv_pipe(const ConvArgs& a, hipStream_t s);
// head.hip: stand-alone YOLO head (1x1, Cin % 128 == 0, <= 32 outputs, decode into io)
bool head1x1_ok(const ConvArgs& a);
void launch_head1x1(const ConvArgs& a, hipStream_t s);
const char* head1x1_name(const ConvArgs& a);
int conv_pipe_mode();
int pipe_bm(const ConvArgs& a);           // tile rows the launch will use (256 / 128 / 64)
const char* conv_pipe_name(const ConvArgs& a);  // kernel symbol of that launch
// conv_c32.hip: persistent Cin-32 3x3 kernel (stride 1 / 2, Cout 64, optional residual)
bool c32_ok(const ConvArgs& a);
void launch_c32(const ConvArgs& a, hipStream_t s);
const char* c32_name(const ConvArgs& a);
// ... and Darknet-53's first residual block (1x1 64 -> 32, 3x3 32 -> 64, shortcut) as one launch
bool c32r_ok(const ConvArgs& a1, const ConvArgs& a);
void launch_c32r(const ConvArgs& a1, const ConvArgs& a, hipStream_t s);
bool c64r_ok(const ConvArgs& a1, const ConvArgs& a);
void launch_c64r(const ConvArgs& a1, const ConvArgs& a, hipStream_t s);
// int8 twin (RTDM_I8): a.in = quantised contiguous int8 copy of the input, a.w8 int8
// weights (per-channel activation scales folded in), a.deq per-output-channel scales
bool conv_pipe_i8_ok(const ConvArgs& a);
void launch_conv_pipe_i8(const ConvArgs& a, hipStream_t s);
const char* conv_pipe_i8_name(const ConvArgs& a);
// diagnostics: conv_stem3 ablation builds (tools/ab_conv.py --key stem_abl)
int stem_abl();
// detector.cpp: plan conv -> 1x1 head -> [yolo] as one fused launch (default 1)
int fuse_head();
// detector.cpp: run independent branches (heads) on a second stream (default 1)
int two_streams_mode();
// Kernel symbol (template instantiation) launch_conv will pick for a / dtype.
const char* conv_kernel_name(const ConvArgs& a, int dtype);
// Row geometry helpers shared by host planners.
inline void conv_set_rows(ConvArgs& a) {
  if (a.quad) {
    a.qh = a.oh / 2;
    a.qw = a.ow / 2;
    a.M = a.n * a.qh * a.qw * 4;
  } else {
    a.M = a.n * a.oh * a.ow;
  }
  a.fd_ow = make_fastdiv(a.ow);
  a.fd_cin = make_fastdiv(a.cin);
  a.fd_oh = make_fastdiv(a.oh);
  a.fd_qw = make_fastdiv(a.qw);
  a.fd_qh = make_fastdiv(a.qh);
}

// ----------------------------------------------------------- other ops ----
// ops.hip
void launch_dw3_acff(const void* in, int in_cs, int in_co, int n, int h, int w, int c, int lim_h, int lim_w,
                     const float* wts /*[3][c][9]*/, const float* bias /*[3][c]*/, void* out /*[n,h-2,w-2,3c]*/,
                     int dtype, hipStream_t s);
// YOLO-ACFF (models.py:296-302): the three branches ADDED into one [n,h-2,w-2,c] map;
// wts [27][c] (branch-major taps), bsum [c] = b1 + b2 + b3
void launch_dw3_sum(const void* in, int in_cs, int in_co, int n, int h, int w, int c, const float* wts,
                    const float* bsum, void* out, int dtype, hipStream_t s);
bool dw3_sum_vec_ok(int c, int in_cs, int in_co, int dtype);
bool dw3_sum_tile_ok(int c, int in_cs, int in_co, int dtype);
// acff.hip: fused ACFF block (dw3 -> concat -> 1x1 -> LeakyReLU -> BN affine -> opt. 2x2 pool), fp16
bool acff_fused_ok(int cin, int cout_pad, int kpad);
void launch_acff_fused(const void* in, int in_cs, int in_co, int n, int h, int w, int cin, int lim_h, int lim_w,
                       const float* dw_wt /*[3][9][cin]*/, const float* dw_b /*[3][cin]*/, const void* pw, int kpad,
                       int cout, int cout_pad, const float* bias, const float* scale, const float* shift, float slope,
                       void* out, int out_cs, int pool, hipStream_t s);
// int8 1x1 fusion of an ACFF stage (RTDM_I8 classifiers): w8 non-null runs the int8 GEMM
// (the concat quantised per channel with inv_s [3][cin], per-output-channel int8 weights in
// the kernel's K order, dequantised by deq); w8 null and amax non-null records the fp16
// run's |x|max of every concat channel (calibration).
struct AcffI8 {
  const void* w8 = nullptr;
  const float* deq = nullptr;
  const float* inv_s = nullptr;
  unsigned* amax = nullptr;
};
// acff.hip: persistent ACFF for the large maps (channel chunk from acff_persist_chunk;
// pwc = 1x1 weights in (chunk, branch, channel) K order; int8: k = chunk*64 + branch*CC + c)
int acff_persist_chunk(int cin, int cout_pad, int oh);
void launch_acff_persist(const void* in, int in_cs, int in_co, int n, int h, int w, int cin, int lim_h, int lim_w,
                         const float* dw_wt, const float* dw_b, const void* pwc, int cout, int cout_pad,
                         const float* bias, const float* scale, const float* shift, float slope, void* out, int out_cs,
                         int pool, hipStream_t s, const AcffI8* q = nullptr);
// acff.hip: the classifier's non-pooled small-map ACFF suffix + tail in one launch
struct AcffChainPlan {
  int nst = 0;
  int h[4] = {}, cin[4] = {}, cout[4] = {}, cout_pad[4] = {}, kpad[4] = {};
};
bool acff_chain_ok(const AcffChainPlan& p);
size_t acff_chain_lds(const AcffChainPlan& p);
void launch_acff_chain(const AcffChainPlan& p, const void* in, int in_cs, int in_co, int n, const float* const* dw_wt,
                       const float* const* dw_b, const void* const* pw, const float* const* bias,
                       const float* const* scale, const float* const* shift, float slope, const float* w2,
                       int pool_pad, int ph, int pwid, const float* fcw, const float* fcb, float* logits, float* probs,
                       hipStream_t s, const AcffI8* q = nullptr /* [nst]; int8: k = branch*cin + c */);
int acff_chain_mode();  // 1 = use acff_chain when the plan allows (default), 0 = per-stage kernels + tail
// acff_band.hip: one small-map ACFF stage per launch over output row bands (all output
// channels per workgroup; optional 2x2 pool), the last stage with the classifier tail
struct AcffBandTail {
  const float* w2 = nullptr;  // conv2 [5][cout]
  int pool_pad = 0, ph = 0, pw = 0;
  const float* fcw = nullptr;
  const float* fcb = nullptr;
  float* logits = nullptr;
  float* probs = nullptr;
};
bool acff_band_ok(int h, int w, int cin, int cout, int cout_pad, int kpad, int pool, bool tail);
void launch_acff_band(const void* in, int in_cs, int in_co, int n, int h, int w, int cin, const float* dw_wt,
                      const float* dw_b, const void* pw, int kpad, int cout, int cout_pad, const float* bias,
                      const float* scale, const float* shift, float slope, void* out, int out_cs, int pool,
                      const AcffBandTail* tail, hipStream_t s);
int acff_band_mode();  // 1 = acff_band for the classifier's small-map stages + tail, 2 = only the chain's stages, 0 = off (default)
int acff_persist_mode();
void launch_maxpool(const void* in, View iv, int n, int h, int w, int c, int k, int stride, int pad, int zero_pad_rb,
                    View ov, int oh, int ow, int dtype, hipStream_t s);
void launch_upsample(View iv, int n, int h, int w, int c, int f, View ov, int dtype, hipStream_t s);
// F.interpolate(mode="nearest", size=(oh, ow)): src = min(floor(dst * (in / out)), in - 1)
// out = a + b (fp32 sum, rounded once), NHWC views of one shape
void launch_add(View a, View b, int n, int h, int w, int c, int cb, View ov, int dtype, hipStream_t s);
void launch_resize_nearest(View iv, int n, int h, int w, int c, View ov, int oh, int ow, int dtype, hipStream_t s);
void launch_copy_slice(View iv, int n, int h, int w, int c, View ov, int dtype, hipStream_t s);
void launch_cls_tail(const void* in, int n, int h, int w, int c, const float* w2 /*[5][c]*/, int pool_pad,
                     int ph, int pw, const float* fcw /*[5][5*ph*pw]*/, const float* fcb, float* logits,
                     float* probs, int dtype, hipStream_t s);
void launch_to_nchw_f32(View iv, int n, int h, int w, int c, float* out, int dtype, hipStream_t s);

struct ResizePlan {  // Pillow 8bpc antialiased bilinear, restricted to a center crop
  int in_h = 0, in_w = 0, rs_h = 0, rs_w = 0, out = 0;
  int crop_top = 0, crop_left = 0;
  int ksize_h = 0, ksize_v = 0;
  int row_first = 0, rows = 0;  // input rows needed by the vertical pass
  int band_rows = 0;            // max input rows of one 16-output-row band (fused kernel)
  int band_rows17 = 0;          // ... of 17 output rows from a band start (the resize + conv1 kernel)
  int band_rows8 = 0;           // ... of one 8-output-row band (staged kernel)
  int col_first = 0, col_end = 0;  // input columns the crop reads
  DevBuf bounds_h, coef_h, bounds_v, coef_v;  // int32 device arrays
};
void build_resize_plan(ResizePlan& p, int in_h, int in_w, int out_size, bool upload);
// 1 = streaming resize kernel (default), 0 = the staged band kernel (A/B knob)
int resize_stream_mode();
// frames -> tmp (horizontal pass) -> out (vertical pass + crop + ToTensor + Normalize)
void launch_preprocess(const ResizePlan& p, const uint8_t* frames, int n, uint8_t* tmp, void* out,
                       int out_layout /*0: NHWC dtype, 1: NCHW f32*/, int dtype, hipStream_t s);
// The same transform with the classifiers' conv1 (3 -> 16, 3x3, stride 2, pad 0, conv_stem3's
// packed weights + bias) fused: writes the [n, stem_oh, stem_oh, 16] fp16 stem map only.
bool preprocess_stem_ok(const ResizePlan& p, const uint8_t* frames, int stem_oh);
void launch_preprocess_stem(const ResizePlan& p, const uint8_t* frames, int n, const void* w_stem, const float* bias,
                            void* stem_out, int stem_oh, hipStream_t s);

// Letterbox (datasets.py:599-631): cv2 INTER_AREA resize to new_w x new_h at (left, top)
// of an out_h x out_w canvas of pad_rgb; uint8 3-channel frames (row pitch in bytes).
void launch_letterbox(const uint8_t* frames, int n, int in_h, int in_w, int pitch, int new_h, int new_w, int out_h,
                      int out_w, int top, int left, uint32_t pad_rgb, int swap_rb, uint8_t* out, hipStream_t s,
                      int interp = 0 /*0: INTER_AREA rules, 1: INTER_LINEAR*/);

struct AnchorVec {  // anchor_vec = anchors / stride of one [yolo] head (<= 8 anchors), by value
  float v[16];
};
void launch_yolo_decode(const float* p, int n, int na, int no, int ny, int nx, const AnchorVec& anchor_vec, float ystride,
                        float* io, int io_rows, int row_off, hipStream_t s);

// TensorRT YoloLayer_TRT decode (CalDetection / CalDetection_NewCoords,
// tensorrt_inference/plugins/yolo_layer.cu:203-306) -> Detection records of 7 floats
static constexpr int kTrtMaxHeads = 8;
static constexpr int kTrtMaxAnchors = 6;  // MAX_ANCHORS, yolo_layer.h:11
struct TrtYoloHead {
  int row0 = 0, na = 0, ny = 0, nx = 0;  // rows [row0, row0 + na*ny*nx) of the row layout
  int in_w = 0, in_h = 0;                // mInputWidth / mInputHeight
  float scale_xy = 1.f;
  int new_coords = 0;
  float anchors[2 * kTrtMaxAnchors] = {};  // pixels
};
struct TrtYoloArgs {
  int n_heads = 0, rows = 0, no = 0, nc = 0;
  TrtYoloHead h[kTrtMaxHeads];
};
// nchw = 0: in = rows [n, rows, no] (the raw YOLOLayer p of every head, io order);
// nchw = 1: in = one head's map [n, na*no, ny, nx] (the plugin's input binding).
// out: [n, rows, 7] (plugin output order: anchor, then grid cell).
void launch_yolo_trt(const float* in, int n, const TrtYoloArgs& t, int nchw, float* out, hipStream_t s);

size_t nms_workspace_size(int n, int n_anchors, int nc);
void launch_nms(const float* io, int n, int n_anchors, int no, float conf, double iou, int multi_label,
                int agnostic, uint64_t class_mask, int max_det, void* ws, float* det, int32_t* idx,
                int32_t* count, hipStream_t s);

}  // namespace rtdm
