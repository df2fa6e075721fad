// ACFF classifier runtime: Squeeze-ErNET / Squeeze-ErNET-RedConv / ErNET.
//
// Mirrors disaster_detection/model/{squeeze_ernet,squeeze_ernet_redconv,ernet}.py
// forward passes as a fixed launch sequence over NHWC device buffers:
//   [preprocess] -> stem conv 3x3/s2 (VALU, Cin=3) -> per ACFF block:
//   dw3 (three dilated depthwise branches, concat layout) -> 1x1 GEMM with
//   epilogue bias -> LeakyReLU(0.01) -> BN affine (-> fused 2x2 floor maxpool)
//   -> tail (1x1 ->5, AvgPool 5, NCHW flatten, Linear, Softmax).
// RedConv's conv_red1 is folded into the stem (linear o linear); conv_red2
// absorbs acff2's BN affine.
#include <cstdio>
#include <cmath>
#include <cstring>
#include <map>

#include "weights.h"

namespace rtdm {

struct AcffStage {
  int cin = 0, cout = 0, h = 0, w = 0;  // input geometry
  bool pool = false;                    // 2x2 floor maxpool after the block
  bool affine = true;                   // BN as post-activation affine in epilogue
  size_t dw_w = 0, dw_b = 0;            // [3][cin][9], [3][cin]
  size_t dw_wt = 0;                     // [3][9][cin] (tap-major copy for the fused kernel)
  bool fused = false;                   // fp16 fused ACFF kernel (acff.hip)
  int persist_cc = 0;                   // acff_persist channel chunk (0 = acff_fused)
  int persist_cp = 0;                   // acff_persist output channels padded to 32 (fp16 / calibration
                                        // runs; int8 keeps pw.cout_pad): rows of pwc_off
  size_t pwc_off = 0;                   // 1x1 weights in (chunk, branch, channel) K order
  PackedConv pw;                        // fused 1x1 conv
  size_t d_buf = 0, out_buf = 0;        // arena offsets (elements) per image
  int oh = 0, ow = 0;                   // dw/1x1 output geometry
  int out_h = 0, out_w = 0;             // after optional pool
  // optional trailing 1x1 reducer (RedConv): conv_red2 / conv_red3
  bool red = false;
  bool red_pool = false;
  PackedConv redw;
  size_t red_buf = 0;
  int red_h = 0, red_w = 0;
  size_t mid_buf = 0;  // ACFF output before the reducer (when red)
  // int8 1x1 fusion (RTDM_I8 handles: acff_persist and acff_chain stages): blob slots of
  // the int8 weights (kernel K order), per-output dequantisation, inverse activation
  // scales [3][cin]; fp32 fusion weights [cout][3 cin] kept for the calibration
  bool q8 = false;
  size_t w8_off = 0, deq_off = 0, inv_off = 0;
  int amax_off = 0;
  std::vector<float> wf;
};

}  // namespace rtdm

struct rtdm_classifier_s {
  int kind = 0, dtype = 0, S = 0, max_batch = 0, dev = 0;
  rtdm::Tuning tuning;  // this handle's knobs (rtdm_classifier_set_tuning; the defaults at create)
  rtdm::DevBlob blob;
  rtdm::PackedConv stem;
  int stem_oh = 0, stem_cout = 0;
  std::vector<rtdm::AcffStage> stages;
  size_t tail_w2 = 0, tail_fcw = 0, tail_fcb = 0;
  int tail_pool_pad = 0, tail_ph = 0, tail_pw = 0, tail_h = 0, tail_c = 0;
  // arena (elements of dtype per image)
  size_t x0_buf = 0, stem_buf = 0, per_image = 0;
  rtdm::DevBuf arena;
  // preprocessing plans per frame size
  std::map<std::pair<int, int>, std::unique_ptr<rtdm::ResizePlan>> resize;
  rtdm::DevBuf resize_tmp;
  size_t resize_tmp_bytes = 0;
  // stages [chain_start, end) + tail run as one acff_chain launch (-1: none)
  int chain_start = -1;
  // stages [band_start, end) run as acff_band launches, the last with the tail (-1: none;
  // fp16 handles; takes precedence over the chain when acff_band_mode())
  int band_start = -1;
  rtdm::AcffChainPlan chain;
  // RTDM_I8: fp16 activations everywhere, int8 1x1 fusion GEMMs in the persistent and
  // chained ACFF stages once calibrated (rtdm_classifier_calibrate); calibrating = the
  // fp16 forward recording every int8 stage's concat |x|max into amax
  bool int8 = false, calibrated = false, calibrating = false;
  rtdm::DevBuf amax;
  int q_channels = 0;
  // optional per-launch timing (rtdm_classifier_enable_timing): events[call][2 * seg + {0,1}]
  // around each launch of rtdm_classify; names / algorithmic HBM bytes of the launches
  static constexpr int kMaxSeg = 24;
  bool timing = false;
  int timing_cap = 0, timing_calls = 0, n_seg = 0, seg_n = 0;
  std::vector<int> call_segs;  // launches recorded by each timed call
  std::vector<hipEvent_t> events;
  std::vector<std::string> seg_name;
  std::vector<double> seg_bytes;
  ~rtdm_classifier_s() {
    for (hipEvent_t e : events) (void)hipEventDestroy(e);
  }
};

namespace rtdm {

namespace {

struct ParamMap {
  std::map<std::string, const rtdm_param*> m;
  ParamMap(const rtdm_param* p, int n) {
    for (int i = 0; i < n; ++i) {
      RTDM_REQUIRE(p[i].name, RTDM_E_INVALID, "classifier: parameter with NULL name");
      m[p[i].name] = &p[i];
    }
  }
  const float* get(const std::string& k, int64_t numel) const {
    auto it = m.find(k);
    RTDM_REQUIRE(it != m.end(), RTDM_E_INVALID, "classifier: missing parameter '" + k + "'");
    RTDM_REQUIRE(it->second->numel == numel, RTDM_E_INVALID,
                 "classifier: parameter '" + k + "' has " + std::to_string(it->second->numel) + " elements, expected " +
                     std::to_string(numel));
    RTDM_REQUIRE(it->second->data, RTDM_E_INVALID, "classifier: parameter '" + k + "' has NULL data");
    return it->second->data;
  }
};

size_t esize(int dtype) { return dtype == RTDM_F16 ? 2 : 4; }

// BN eval affine y = (x - mean) / sqrt(var + eps) * g + b  ==  x*s + t
void bn_affine(const float* g, const float* b, const float* mean, const float* var, int c, double eps,
               std::vector<double>& s, std::vector<double>& t) {
  s.resize(c);
  t.resize(c);
  for (int i = 0; i < c; ++i) {
    s[i] = (double)g[i] / std::sqrt((double)var[i] + eps);
    t[i] = (double)b[i] - (double)mean[i] * s[i];
  }
}

std::vector<float> to_f32(const std::vector<double>& v) { return std::vector<float>(v.begin(), v.end()); }

}  // namespace

static void build_classifier(rtdm_classifier_s& h, const ParamMap& pm) {
  Blob blob;
  const bool f16 = h.dtype == RTDM_F16;
  const int S = h.S;
  // ---- stem (squeeze_ernet.py:11 / ernet.py:10) ----
  const float* w1 = pm.get("conv1.weight", 16 * 3 * 9);
  h.stem_oh = (S - 3) / 2 + 1;
  if (h.kind == RTDM_SQUEEZE_REDCONV) {
    // conv_red1 (squeeze_ernet_redconv.py:12) folded: W' = Wr . W1, b' = br
    const float* wr = pm.get("conv_red1.weight", 8 * 16);
    const float* br = pm.get("conv_red1.bias", 8);
    std::vector<float> wf(8 * 27);
    for (int o = 0; o < 8; ++o)
      for (int q = 0; q < 27; ++q) {
        double acc = 0.0;
        for (int k = 0; k < 16; ++k) acc += (double)wr[o * 16 + k] * w1[k * 27 + q];
        wf[o * 27 + q] = (float)acc;
      }
    h.stem = pack_conv(blob, wf.data(), 8, 3, 3, nullptr, false);
    if (f16) h.stem.stem_off = pack_stem(blob, wf.data(), 8, nullptr);
    h.stem.b_off = blob.add(br, 8 * sizeof(float));
    h.stem_cout = 8;
  } else {
    h.stem = pack_conv(blob, w1, 16, 3, 3, nullptr, false);
    if (f16) h.stem.stem_off = pack_stem(blob, w1, 16, nullptr);
    h.stem_cout = 16;
  }

  // ---- ACFF stages ----
  struct Spec {
    const char* name;
    int cin, cout;
    bool pool;
    const char* red;  // reducer module name or nullptr
    int red_out;
    bool red_before_pool;  // conv_red2 sits between acff2 and pool2
  };
  std::vector<Spec> specs;
  if (h.kind == RTDM_SQUEEZE_ERNET) {
    specs = {{"acff1", 16, 64, true, nullptr, 0, false},
             {"acff2", 64, 96, true, nullptr, 0, false},
             {"acff3", 96, 128, true, nullptr, 0, false},
             {"acff4", 128, 256, false, nullptr, 0, false}};
  } else if (h.kind == RTDM_SQUEEZE_REDCONV) {
    specs = {{"acff1", 8, 64, true, nullptr, 0, false},
             {"acff2", 64, 96, true, "conv_red2", 48, true},
             {"acff3", 48, 128, true, "conv_red3", 64, false},
             {"acff4", 64, 256, false, nullptr, 0, false}};
  } else {
    specs = {{"acff1", 16, 64, true, nullptr, 0, false},  {"acff2", 64, 96, true, nullptr, 0, false},
             {"acff3", 96, 128, true, nullptr, 0, false}, {"acff4", 128, 128, false, nullptr, 0, false},
             {"acff5", 128, 128, false, nullptr, 0, false}, {"acff6", 128, 256, false, nullptr, 0, false}};
  }
  size_t off = 0;
  auto take = [&](size_t elems) {
    const size_t o = off;
    off += (size_t)round_up((int64_t)elems, 64);
    return o;
  };
  h.x0_buf = take((size_t)S * S * 3);
  h.stem_buf = take((size_t)h.stem_oh * h.stem_oh * h.stem_cout);
  int ch = h.stem_oh, cc = h.stem_cout;
  for (const Spec& sp : specs) {
    AcffStage st;
    st.cin = sp.cin;
    st.cout = sp.cout;
    RTDM_REQUIRE(cc == sp.cin, RTDM_E_INVALID, "classifier: channel mismatch at " + std::string(sp.name));
    st.h = st.w = ch;
    st.oh = st.ow = ch - 2;
    const std::string p = sp.name;
    // depthwise branches (acff.py:25-30)
    std::vector<float> dww(3 * sp.cin * 9), dwb(3 * sp.cin);
    for (int br = 0; br < 3; ++br) {
      const std::string cn = p + ".conv" + std::to_string(br + 1);
      const float* w = pm.get(cn + ".weight", (int64_t)sp.cin * 9);
      const float* b = pm.get(cn + ".bias", sp.cin);
      std::memcpy(&dww[(size_t)br * sp.cin * 9], w, sizeof(float) * sp.cin * 9);
      std::memcpy(&dwb[(size_t)br * sp.cin], b, sizeof(float) * sp.cin);
    }
    st.dw_w = blob.add_f32(dww);
    st.dw_b = blob.add_f32(dwb);
    std::vector<float> dwt(dww.size());
    for (int br = 0; br < 3; ++br)
      for (int t = 0; t < 9; ++t)
        for (int c = 0; c < sp.cin; ++c) dwt[((size_t)br * 9 + t) * sp.cin + c] = dww[((size_t)br * sp.cin + c) * 9 + t];
    st.dw_wt = blob.add_f32(dwt);
    // fused 1x1 conv + BN (acff.py:31-34)
    const float* fw = pm.get(p + ".fused_conv.weight", (int64_t)sp.cout * 3 * sp.cin);
    const float* fb = pm.get(p + ".fused_conv.bias", sp.cout);
    std::vector<double> bs, bt;
    bn_affine(pm.get(p + ".batch_norm.weight", sp.cout), pm.get(p + ".batch_norm.bias", sp.cout),
              pm.get(p + ".batch_norm.running_mean", sp.cout), pm.get(p + ".batch_norm.running_var", sp.cout), sp.cout,
              1e-5, bs, bt);
    if (h.int8) st.wf.assign(fw, fw + (size_t)sp.cout * 3 * sp.cin);
    st.pw = pack_conv(blob, fw, sp.cout, 3 * sp.cin, 1, nullptr, f16);
    st.pw.b_off = blob.add(fb, sizeof(float) * sp.cout);
    st.fused = f16 && acff_fused_ok(sp.cin, st.pw.cout_pad, st.pw.kpad);
    if (st.fused && !(sp.red && sp.red_before_pool)) st.persist_cc = acff_persist_chunk(sp.cin, st.pw.cout_pad, st.oh);
    if (st.persist_cc) {
      // [persist_cp][nch * KC] fp16, k = chunk*KC + branch*CC + c (zero K/row padding); rows
      // padded to 32 only (two waves x NF 16-channel tiles): ErNET acff2's 96 outputs as NF 3
      // instead of 128 rows of which a quarter were zero MFMA work
      st.persist_cp = (sp.cout + 31) / 32 * 32;
      const int CCk = st.persist_cc, nch = sp.cin / CCk, KC = (3 * CCk + 31) / 32 * 32;
      std::vector<_Float16> wc((size_t)st.persist_cp * nch * KC, (_Float16)0.f);
      for (int o = 0; o < sp.cout; ++o)
        for (int chk = 0; chk < nch; ++chk)
          for (int br = 0; br < 3; ++br)
            for (int cl = 0; cl < CCk; ++cl)
              wc[(size_t)o * nch * KC + chk * KC + br * CCk + cl] =
                  (_Float16)fw[(size_t)o * 3 * sp.cin + br * sp.cin + chk * CCk + cl];
      st.pwc_off = blob.add(wc.data(), wc.size() * sizeof(_Float16));
    }
    st.d_buf = take((size_t)st.oh * st.ow * 3 * sp.cin);
    if (sp.red && sp.red_before_pool) {
      // acff2 -> conv_red2 -> pool2: BN affine folded into conv_red2
      st.affine = false;
      st.red = true;
      st.red_pool = sp.pool;
      st.pool = false;
      st.mid_buf = take((size_t)st.oh * st.ow * sp.cout);
      const std::string rn = sp.red;
      const float* rw = pm.get(rn + ".weight", (int64_t)sp.red_out * sp.cout);
      const float* rb = pm.get(rn + ".bias", sp.red_out);
      std::vector<float> wf((size_t)sp.red_out * sp.cout), bf(sp.red_out);
      for (int o = 0; o < sp.red_out; ++o) {
        double acc = rb[o];
        for (int c = 0; c < sp.cout; ++c) {
          wf[(size_t)o * sp.cout + c] = (float)((double)rw[(size_t)o * sp.cout + c] * bs[c]);
          acc += (double)rw[(size_t)o * sp.cout + c] * bt[c];
        }
        bf[o] = (float)acc;
      }
      st.redw = pack_conv(blob, wf.data(), sp.red_out, sp.cout, 1, nullptr, f16);
      st.redw.b_off = blob.add_f32(bf);
      st.red_h = st.red_w = st.oh / 2;
      st.red_buf = take((size_t)st.red_h * st.red_w * sp.red_out);
      st.out_h = st.out_w = st.red_h;
      ch = st.red_h;
      cc = sp.red_out;
    } else {
      st.affine = true;
      st.pw.s_off = blob.add_f32(to_f32(bs));
      st.pw.t_off = blob.add_f32(to_f32(bt));
      st.pool = sp.pool;
      st.out_h = st.out_w = sp.pool ? st.oh / 2 : st.oh;
      st.out_buf = take((size_t)st.out_h * st.out_w * sp.cout);
      ch = st.out_h;
      cc = sp.cout;
      if (sp.red) {  // acff3 -> pool3 -> conv_red3
        st.red = true;
        st.red_pool = false;
        const std::string rn = sp.red;
        const float* rw = pm.get(rn + ".weight", (int64_t)sp.red_out * sp.cout);
        const float* rb = pm.get(rn + ".bias", sp.red_out);
        st.redw = pack_conv(blob, rw, sp.red_out, sp.cout, 1, nullptr, f16);
        st.redw.b_off = blob.add(rb, sizeof(float) * sp.red_out);
        st.red_h = st.red_w = st.out_h;
        st.red_buf = take((size_t)st.red_h * st.red_w * sp.red_out);
        cc = sp.red_out;
      }
    }
    h.stages.push_back(st);
  }
  // ---- tail (squeeze_ernet.py:19-22 / ernet.py:19-22) ----
  RTDM_REQUIRE(cc == 256, RTDM_E_INVALID, "classifier: tail expects 256 channels");
  h.tail_h = ch;
  h.tail_c = cc;
  h.tail_pool_pad = h.kind == RTDM_ERNET ? 0 : 1;
  h.tail_ph = h.tail_pw = (ch + 2 * h.tail_pool_pad - 5) + 1;
  const int nf = 5 * h.tail_ph * h.tail_pw;
  h.tail_w2 = blob.add(pm.get("conv2.weight", 5 * 256), 5 * 256 * sizeof(float));
  h.tail_fcw = blob.add(pm.get("fc.weight", 5 * nf), (size_t)5 * nf * sizeof(float));
  h.tail_fcb = blob.add(pm.get("fc.bias", 5), 5 * sizeof(float));
  // ---- small-map suffix: non-pooled, reducer-free acff_fused stages (+ tail) in one launch ----
  if (f16) {
    int first = (int)h.stages.size();
    while (first > 0) {
      const AcffStage& st = h.stages[first - 1];
      if (!st.fused || st.persist_cc || st.pool || st.red || !st.affine) break;
      --first;
    }
    const int nst = (int)h.stages.size() - first;
    if (nst >= 1 && nst <= 4) {
      AcffChainPlan cp;
      cp.nst = nst;
      for (int i = 0; i < nst; ++i) {
        const AcffStage& st = h.stages[first + i];
        cp.h[i] = st.h;
        cp.cin[i] = st.cin;
        cp.cout[i] = st.cout;
        cp.cout_pad[i] = st.pw.cout_pad;
        cp.kpad[i] = st.pw.kpad;
      }
      if (acff_chain_ok(cp)) {
        h.chain_start = first;
        h.chain = cp;
      }
    }
  }
  // ---- small-map stages on acff_band (fp16): the last stage with the tail, earlier ones with
  //      maps up to 32 rows, pooled or not, as long as each is a plain ACFF (no reducer) ----
  if (f16 && !h.int8) {
    int first = (int)h.stages.size();
    while (first > 0) {
      const AcffStage& st = h.stages[first - 1];
      const bool last = first == (int)h.stages.size();
      if (st.red || !st.affine || (!last && st.oh > 32) || (last && st.pool) ||
          !acff_band_ok(st.h, st.w, st.cin, st.cout, st.pw.cout_pad, st.pw.kpad, st.pool ? 1 : 0, last))
        break;
      --first;
    }
    if (first < (int)h.stages.size()) h.band_start = first;
  }
  if (h.int8) {  // int8 slots for the persistent stages and (all or none of) the chained ones
    bool chain_q = h.chain_start >= 0;
    for (int i = std::max(0, h.chain_start); chain_q && i < (int)h.stages.size(); ++i)
      chain_q = h.stages[i].cin % 64 == 0;
    for (int i = 0; i < (int)h.stages.size(); ++i) {
      AcffStage& st = h.stages[i];
      const bool in_chain = h.chain_start >= 0 && i >= h.chain_start;
      if (!(st.persist_cc || (in_chain && chain_q))) {
        st.wf.clear();
        continue;
      }
      const int cp = st.pw.cout_pad;
      const size_t kq = st.persist_cc ? (size_t)(st.cin / st.persist_cc) * 64 : (size_t)3 * st.cin;
      st.q8 = true;
      st.w8_off = blob.add(nullptr, (size_t)cp * kq);
      st.deq_off = blob.add(nullptr, (size_t)cp * sizeof(float));
      st.inv_off = blob.add(nullptr, (size_t)3 * st.cin * sizeof(float));
      st.amax_off = h.q_channels;
      h.q_channels += 3 * st.cin;
    }
    h.amax.alloc((size_t)std::max(1, h.q_channels) * sizeof(unsigned));
    // zeroed: a first rtdm_classifier_calibrate(reset = 0) folds its maxima into these
    RTDM_HIP(hipMemset(h.amax.p, 0, (size_t)std::max(1, h.q_channels) * sizeof(unsigned)));
  }
  h.per_image = off;
  h.blob.upload(blob);
  h.arena.alloc(h.per_image * esize(h.dtype) * h.max_batch);
}

// conv1 (3x3/s2, 3 -> stem_cout) over n images whose input fields (in, in_kind, in_cs, in_co)
// are already in a: the one construction classify() launches and describe() names.
static void stem_conv_args(const rtdm_classifier_s& h, ConvArgs& a, int n, View out) {
  a.n = n;
  a.ih = a.iw = h.S;
  a.cin = 3;
  a.ks = 3;
  a.stride = 2;
  a.pad = 0;
  a.oh = a.ow = h.stem_oh;
  a.cout = h.stem_cout;
  a.quad = 0;
  conv_set_rows(a);
  a.w = h.blob.at<void>(h.stem.w_off);
  a.kpad = h.stem.kpad;
  a.cout_pad = h.stem.cout_pad;
  a.w_f32 = h.stem.mfma ? 0 : 1;
  a.w_stem = h.blob.at<void>(h.stem.stem_off);
  a.e.bias = h.blob.at<float>(h.stem.b_off);
  a.e.full = out;
}

// uint8 frames: the CLI transform and conv1 as one launch (launch_preprocess_stem) when the
// stem is the fp16 16-channel one (not RedConv's folded 8-channel stem) and cls_front is on
static bool front_fusable(const rtdm_classifier_s& h) {
  return h.dtype == RTDM_F16 && h.stem_cout == 16 && h.stem.cout_pad == 16 && h.stem.stem_off != SIZE_MAX &&
         tune().cls_front && tune().stem_k16;
}

static void run_classifier(rtdm_classifier_s& h, const void* x, int x_kind, int n, int in_h, int in_w, float* logits,
                           float* probs, hipStream_t s) {
  RTDM_REQUIRE(n >= 0 && n <= h.max_batch, RTDM_E_CAPACITY,
               "classify: batch " + std::to_string(n) + " exceeds max_batch " + std::to_string(h.max_batch));
  RTDM_REQUIRE(!h.int8 || h.calibrated || h.calibrating || h.q_channels == 0, RTDM_E_INVALID,
               "classify: int8 classifier not calibrated (rtdm_classifier_calibrate)");
  // before any launch: an int8 handle's quantised stages only exist in the chained schedule
  RTDM_REQUIRE(!h.int8 || (h.chain_start >= 0 && acff_chain_mode()) || h.chain_start < 0, RTDM_E_INVALID,
               "classify: int8 handle needs acff_chain mode");
  if (n == 0) return;
  RTDM_REQUIRE(x, RTDM_E_INVALID, "classify: NULL input");
  const size_t es = esize(h.dtype);
  // per-launch timing: seg(name, bytes) before a launch, seg_end() after it
  hipEvent_t* ev = nullptr;
  int si = 0;
  if (h.timing && !h.calibrating && h.timing_calls < h.timing_cap) {
    ev = &h.events[(size_t)h.timing_calls * 2 * rtdm_classifier_s::kMaxSeg];
    if (h.timing_calls == 0) {
      h.seg_name.clear();
      h.seg_bytes.clear();
      h.call_segs.assign(h.timing_cap, 0);
    }
    ++h.timing_calls;
  }
  auto seg = [&](const std::string& name, double bytes) {
    if (!ev) return;
    RTDM_REQUIRE(si < rtdm_classifier_s::kMaxSeg, RTDM_E_INVALID, "classify timing: too many launches");
    if (h.timing_calls == 1) {
      h.seg_name.push_back(name);
      h.seg_bytes.push_back(bytes);
    }
    RTDM_HIP(hipEventRecord(ev[2 * si], s));
  };
  auto seg_end = [&]() {
    if (!ev) return;
    RTDM_HIP(hipEventRecord(ev[2 * si + 1], s));
    h.n_seg = ++si;
    h.call_segs[h.timing_calls - 1] = si;
  };
  const double nb = (double)n;
  char* base = h.arena.as<char>();
  auto buf = [&](size_t off) { return (void*)(base + off * es * h.max_batch); };
  const int S = h.S;
  // ---- input ----
  ConvArgs a;
  bool stem_done = false;
  if (x_kind == RTDM_INPUT_FRAME_U8) {
    auto key = std::make_pair(in_h, in_w);
    auto it = h.resize.find(key);
    if (it == h.resize.end()) {
      auto p = std::make_unique<ResizePlan>();
      build_resize_plan(*p, in_h, in_w, S, true);
      it = h.resize.emplace(key, std::move(p)).first;
    }
    const ResizePlan& rp = *it->second;
    const size_t need = (size_t)h.max_batch * rp.rows * rp.out * 3;
    if (need > h.resize_tmp_bytes) {
      RTDM_HIP(hipStreamSynchronize(s));
      h.resize_tmp.alloc(need);
      h.resize_tmp_bytes = need;
    }
    // CLI transform + conv1 in one launch (fp16, the 16-channel stem): the transformed image
    // never leaves LDS; the stem map is bit-identical to the two-launch form's
    if (front_fusable(h) && preprocess_stem_ok(rp, (const uint8_t*)x, h.stem_oh)) {
      seg("preprocess+stem", nb * ((double)in_h * in_w * 3 + (double)h.stem_oh * h.stem_oh * h.stem_cout * es));
      launch_preprocess_stem(rp, (const uint8_t*)x, n, h.blob.at<void>(h.stem.stem_off), h.blob.at<float>(h.stem.b_off),
                             buf(h.stem_buf), h.stem_oh, s);
      seg_end();
      stem_done = true;
    } else {
      // bytes: the frames in, the S x S x 3 model input out
      seg("preprocess", nb * ((double)in_h * in_w * 3 + (double)S * S * 3 * es));
      launch_preprocess(rp, (const uint8_t*)x, n, h.resize_tmp.as<uint8_t>(), buf(h.x0_buf), 0, h.dtype, s);
      seg_end();
      a.in = buf(h.x0_buf);
      a.in_kind = IN_NHWC;
      a.in_cs = 3;
      a.in_co = 0;
    }
  } else if (x_kind == RTDM_INPUT_NCHW_F32 || x_kind == RTDM_INPUT_NCHW_F16) {
    RTDM_REQUIRE(in_h == S && in_w == S, RTDM_E_UNSUPPORTED,
                 "classify: model expects " + std::to_string(S) + "x" + std::to_string(S) + " input, got " +
                     std::to_string(in_h) + "x" + std::to_string(in_w));
    a.in = x;
    a.in_kind = x_kind == RTDM_INPUT_NCHW_F32 ? IN_NCHW_F32 : IN_NCHW_F16;
  } else {
    throw Error{RTDM_E_INVALID, "classify: unknown input kind"};
  }
  // ---- stem ----
  if (!stem_done) {
    stem_conv_args(h, a, n, View{buf(h.stem_buf), h.stem_cout, 0});
    seg("stem", nb * ((double)S * S * 3 * (x_kind == RTDM_INPUT_NCHW_F32 ? 4 : es) +
                      (double)h.stem_oh * h.stem_oh * h.stem_cout * es));
    launch_conv(a, h.dtype, s);
    seg_end();
  }

  View cur{buf(h.stem_buf), h.stem_cout, 0};
  const bool chain = h.chain_start >= 0 && acff_chain_mode();
  // int8 / calibration arguments of a stage (nullptr: the plain fp16 kernels)
  auto q8 = [&](const AcffStage& st, AcffI8& q) -> const AcffI8* {
    if (!st.q8) return nullptr;
    if (h.calibrating) {
      q.amax = h.amax.as<unsigned>() + st.amax_off;
      return &q;
    }
    q.w8 = h.blob.at<void>(st.w8_off);
    q.deq = h.blob.at<float>(st.deq_off);
    q.inv_s = h.blob.at<float>(st.inv_off);
    return &q;
  };
  const bool band = h.band_start >= 0 && acff_band_mode() && !h.calibrating;
  // acff_band 2 (tests): bands only from the chain's first stage, so the result is the chain's bit for bit
  const int band_start = acff_band_mode() == 2 ? std::max(h.band_start, h.chain_start) : h.band_start;
  for (size_t si = 0; si < h.stages.size(); ++si) {
    if (band && (int)si == band_start) break;
    if (chain && (int)si == h.chain_start) break;
    const AcffStage& st = h.stages[si];
    const int lim = st.pool || st.red_pool ? (st.oh / 2) * 2 : st.oh;
    if (st.fused) {
      const float* sc = st.affine ? h.blob.at<float>(st.pw.s_off) : nullptr;
      const float* sh = st.affine ? h.blob.at<float>(st.pw.t_off) : nullptr;
      const bool pool_here = st.pool && !st.red_pool;
      void* dst = st.red && st.red_pool ? buf(st.mid_buf) : buf(st.out_buf);
      AcffI8 qa;
      // bytes: the stage input map in, its (pooled) output out
      seg("acff" + std::to_string(si + 1),
          nb * ((double)st.h * st.w * st.cin + (double)(pool_here ? (lim / 2) * (lim / 2) : lim * lim) * st.cout) * es);
      if (st.persist_cc && (acff_persist_mode() || st.q8)) {
        const AcffI8* qp = q8(st, qa);
        launch_acff_persist(cur.ptr, cur.cs, cur.co, n, st.h, st.w, st.cin, lim, lim, h.blob.at<float>(st.dw_wt),
                            h.blob.at<float>(st.dw_b), h.blob.at<void>(st.pwc_off), st.cout,
                            qp && qp->w8 ? st.pw.cout_pad : st.persist_cp, h.blob.at<float>(st.pw.b_off), sc, sh,
                            0.01f, dst, st.cout, pool_here ? 1 : 0, s, qp);
      } else
      launch_acff_fused(cur.ptr, cur.cs, cur.co, n, st.h, st.w, st.cin, lim, lim, h.blob.at<float>(st.dw_wt),
                        h.blob.at<float>(st.dw_b), h.blob.at<void>(st.pw.w_off), st.pw.kpad, st.cout, st.pw.cout_pad,
                        h.blob.at<float>(st.pw.b_off), sc, sh, 0.01f, dst, st.cout, pool_here ? 1 : 0, s);
      seg_end();
      if (st.red && st.red_pool) {
        ConvArgs r;
        r.in = buf(st.mid_buf);
        r.in_cs = st.cout;
        r.n = n;
        r.ih = r.iw = st.oh;
        r.cin = st.cout;
        r.ks = 1;
        r.oh = r.ow = st.oh;
        r.cout = st.redw.cout;
        r.quad = 1;
        conv_set_rows(r);
        r.w = h.blob.at<void>(st.redw.w_off);
        r.kpad = st.redw.kpad;
        r.cout_pad = st.redw.cout_pad;
        r.w_f32 = st.redw.mfma ? 0 : 1;
        r.e.bias = h.blob.at<float>(st.redw.b_off);
        r.e.pool = View{buf(st.red_buf), st.redw.cout, 0};
        seg("conv_red", nb * ((double)r.ih * r.iw * r.cin + (double)(r.e.pool.ptr ? (r.oh / 2) * (r.ow / 2) : r.oh * r.ow) * r.cout) * es);
        launch_conv(r, h.dtype, s);
        seg_end();
        cur = View{buf(st.red_buf), st.redw.cout, 0};
        continue;
      }
      cur = View{buf(st.out_buf), st.cout, 0};
      if (st.red) {  // conv_red3 on the pooled output
        ConvArgs r;
        r.in = cur.ptr;
        r.in_cs = st.cout;
        r.n = n;
        r.ih = r.iw = st.out_h;
        r.cin = st.cout;
        r.ks = 1;
        r.oh = r.ow = st.out_h;
        r.cout = st.redw.cout;
        conv_set_rows(r);
        r.w = h.blob.at<void>(st.redw.w_off);
        r.kpad = st.redw.kpad;
        r.cout_pad = st.redw.cout_pad;
        r.w_f32 = st.redw.mfma ? 0 : 1;
        r.e.bias = h.blob.at<float>(st.redw.b_off);
        r.e.full = View{buf(st.red_buf), st.redw.cout, 0};
        seg("conv_red", nb * ((double)r.ih * r.iw * r.cin + (double)(r.e.pool.ptr ? (r.oh / 2) * (r.ow / 2) : r.oh * r.ow) * r.cout) * es);
        launch_conv(r, h.dtype, s);
        seg_end();
        cur = View{buf(st.red_buf), st.redw.cout, 0};
      }
      continue;
    }
    launch_dw3_acff(cur.ptr, cur.cs, cur.co, n, st.h, st.w, st.cin, lim, lim, h.blob.at<float>(st.dw_w),
                    h.blob.at<float>(st.dw_b), buf(st.d_buf), h.dtype, s);
    ConvArgs g;
    g.in = buf(st.d_buf);
    g.in_cs = 3 * st.cin;
    g.in_kind = IN_NHWC;
    g.n = n;
    g.ih = st.oh;
    g.iw = st.ow;
    g.cin = 3 * st.cin;
    g.ks = 1;
    g.oh = st.oh;
    g.ow = st.ow;
    g.cout = st.cout;
    g.w = h.blob.at<void>(st.pw.w_off);
    g.kpad = st.pw.kpad;
    g.cout_pad = st.pw.cout_pad;
    g.w_f32 = st.pw.mfma ? 0 : 1;
    g.e.bias = h.blob.at<float>(st.pw.b_off);
    g.e.act = ACT_LEAKY;
    g.e.slope = 0.01f;  // ACFF's LeakyReLU(0.01); the epilogues' max(t, slope t) needs 0 < slope <= 1
    RTDM_REQUIRE(g.e.slope > 0.f && g.e.slope <= 1.f, RTDM_E_INVALID, "classifier: LeakyReLU slope outside (0, 1]");
    if (st.affine) {
      g.e.scale = h.blob.at<float>(st.pw.s_off);
      g.e.shift = h.blob.at<float>(st.pw.t_off);
    }
    if (st.red && st.red_pool) {
      // acff2 (-> mid, full) ; conv_red2 (+BN folded) with fused pool
      g.quad = 1;  // only the even region is consumed by the pooled reducer
      conv_set_rows(g);
      g.e.full = View{buf(st.mid_buf), st.cout, 0};
      launch_conv(g, h.dtype, s);
      ConvArgs r;
      r.in = buf(st.mid_buf);
      r.in_cs = st.cout;
      r.n = n;
      r.ih = r.iw = st.oh;
      r.cin = st.cout;
      r.ks = 1;
      r.oh = r.ow = st.oh;
      r.cout = st.redw.cout;
      r.quad = 1;
      conv_set_rows(r);
      r.w = h.blob.at<void>(st.redw.w_off);
      r.kpad = st.redw.kpad;
      r.cout_pad = st.redw.cout_pad;
      r.w_f32 = st.redw.mfma ? 0 : 1;
      r.e.bias = h.blob.at<float>(st.redw.b_off);
      r.e.pool = View{buf(st.red_buf), st.redw.cout, 0};
      seg("conv_red", nb * ((double)r.ih * r.iw * r.cin + (double)(r.e.pool.ptr ? (r.oh / 2) * (r.ow / 2) : r.oh * r.ow) * r.cout) * es);
      launch_conv(r, h.dtype, s);
      seg_end();
      cur = View{buf(st.red_buf), st.redw.cout, 0};
      continue;
    }
    g.quad = st.pool ? 1 : 0;
    conv_set_rows(g);
    if (st.pool)
      g.e.pool = View{buf(st.out_buf), st.cout, 0};
    else
      g.e.full = View{buf(st.out_buf), st.cout, 0};
    launch_conv(g, h.dtype, s);
    cur = View{buf(st.out_buf), st.cout, 0};
    if (st.red) {  // conv_red3 on the pooled output
      ConvArgs r;
      r.in = cur.ptr;
      r.in_cs = st.cout;
      r.n = n;
      r.ih = r.iw = st.out_h;
      r.cin = st.cout;
      r.ks = 1;
      r.oh = r.ow = st.out_h;
      r.cout = st.redw.cout;
      conv_set_rows(r);
      r.w = h.blob.at<void>(st.redw.w_off);
      r.kpad = st.redw.kpad;
      r.cout_pad = st.redw.cout_pad;
      r.w_f32 = st.redw.mfma ? 0 : 1;
      r.e.bias = h.blob.at<float>(st.redw.b_off);
      r.e.full = View{buf(st.red_buf), st.redw.cout, 0};
      seg("conv_red", nb * ((double)r.ih * r.iw * r.cin + (double)(r.e.pool.ptr ? (r.oh / 2) * (r.ow / 2) : r.oh * r.ow) * r.cout) * es);
      launch_conv(r, h.dtype, s);
      seg_end();
      cur = View{buf(st.red_buf), st.redw.cout, 0};
    }
  }
  if (band) {
    for (size_t si = band_start; si < h.stages.size(); ++si) {
      const AcffStage& st = h.stages[si];
      const bool last = si + 1 == h.stages.size();
      AcffBandTail tl;
      if (last) {
        tl.w2 = h.blob.at<float>(h.tail_w2);
        tl.pool_pad = h.tail_pool_pad;
        tl.ph = h.tail_ph;
        tl.pw = h.tail_pw;
        tl.fcw = h.blob.at<float>(h.tail_fcw);
        tl.fcb = h.blob.at<float>(h.tail_fcb);
        tl.logits = logits;
        tl.probs = probs;
      }
      const int lo = st.pool ? (st.oh / 2) * (st.ow / 2) : st.oh * st.ow;
      seg("acff" + std::to_string(si + 1) + (last ? "+tail" : ""),
          nb * ((double)st.h * st.w * st.cin * es + (last ? 2.0 * 5 * 4 : (double)lo * st.cout * es)));
      launch_acff_band(cur.ptr, cur.cs, cur.co, n, st.h, st.w, st.cin, h.blob.at<float>(st.dw_wt),
                       h.blob.at<float>(st.dw_b), h.blob.at<void>(st.pw.w_off), st.pw.kpad, st.cout, st.pw.cout_pad,
                       h.blob.at<float>(st.pw.b_off), h.blob.at<float>(st.pw.s_off), h.blob.at<float>(st.pw.t_off),
                       0.01f, last ? nullptr : buf(st.out_buf), st.cout, st.pool ? 1 : 0, last ? &tl : nullptr, s);
      seg_end();
      cur = View{buf(st.out_buf), st.cout, 0};
    }
    return;
  }
  if (chain) {
    const int k = h.chain.nst;
    AcffI8 qs[4];
    bool any_q = false;
    const float* dw_wt[4];
    const float* dw_b[4];
    const void* pw[4];
    const float* bias[4];
    const float* sc[4];
    const float* sh[4];
    for (int i = 0; i < k; ++i) {
      const AcffStage& st = h.stages[h.chain_start + i];
      dw_wt[i] = h.blob.at<float>(st.dw_wt);
      dw_b[i] = h.blob.at<float>(st.dw_b);
      pw[i] = h.blob.at<void>(st.pw.w_off);
      bias[i] = h.blob.at<float>(st.pw.b_off);
      sc[i] = h.blob.at<float>(st.pw.s_off);
      sh[i] = h.blob.at<float>(st.pw.t_off);
      any_q = q8(st, qs[i]) != nullptr || any_q;
    }
    {
      const AcffStage& st0 = h.stages[h.chain_start];
      seg("acff_chain", nb * ((double)st0.h * st0.w * st0.cin * es + 2.0 * 5 * 4));
    }
    launch_acff_chain(h.chain, cur.ptr, cur.cs, cur.co, n, dw_wt, dw_b, pw, bias, sc, sh, 0.01f,
                      h.blob.at<float>(h.tail_w2), h.tail_pool_pad, h.tail_ph, h.tail_pw, h.blob.at<float>(h.tail_fcw),
                      h.blob.at<float>(h.tail_fcb), logits, probs, s, any_q ? qs : nullptr);
    seg_end();
    return;
  }
  seg("tail", nb * ((double)h.tail_h * h.tail_h * h.tail_c * es + 2.0 * 5 * 4));
  launch_cls_tail(cur.ptr, n, h.tail_h, h.tail_h, h.tail_c, h.blob.at<float>(h.tail_w2), h.tail_pool_pad, h.tail_ph,
                  h.tail_pw, h.blob.at<float>(h.tail_fcw), h.blob.at<float>(h.tail_fcb), logits, probs, h.dtype, s);
  seg_end();
}

}  // namespace rtdm

using namespace rtdm;

extern "C" {

rtdm_status rtdm_classifier_create(int kind, int dtype, const rtdm_param* params, int n_params, int max_batch,
                                   rtdm_classifier* out) {
  return guard([&] {
    RTDM_REQUIRE(out, RTDM_E_INVALID, "classifier_create: NULL out");
    *out = nullptr;
    RTDM_REQUIRE(kind >= RTDM_SQUEEZE_ERNET && kind <= RTDM_ERNET, RTDM_E_INVALID, "classifier_create: bad kind");
    RTDM_REQUIRE(dtype == RTDM_F32 || dtype == RTDM_F16 || dtype == RTDM_I8, RTDM_E_INVALID,
                 "classifier_create: bad dtype");
    RTDM_REQUIRE(max_batch > 0, RTDM_E_INVALID, "classifier_create: max_batch must be > 0");
    RTDM_REQUIRE(params && n_params > 0, RTDM_E_INVALID, "classifier_create: no parameters");
    auto h = std::make_unique<rtdm_classifier_s>();
    h->tuning = default_tuning();
    TuningScope ts_(&h->tuning);
    h->kind = kind;
    h->int8 = dtype == RTDM_I8;
    h->dtype = h->int8 ? RTDM_F16 : dtype;  // int8 handles keep fp16 activations
    h->S = kind == RTDM_ERNET ? 240 : 140;
    h->max_batch = max_batch;
    RTDM_HIP(hipGetDevice(&h->dev));
    ParamMap pm(params, n_params);
    build_classifier(*h, pm);
    *out = h.release();
  });
}

rtdm_status rtdm_classifier_set_tuning(rtdm_classifier h, const char* key, int value) {
  return guard([&] {
    RTDM_REQUIRE(h, RTDM_E_INVALID, "classifier_set_tuning: NULL handle");
    tuning_set(h->tuning, key, value);
  });
}

rtdm_status rtdm_classifier_destroy(rtdm_classifier h) {
  return guard([&] { delete h; });
}

rtdm_status rtdm_classifier_enable_timing(rtdm_classifier h, int max_calls) {
  return guard([&] {
    TuningScope ts_(h ? &h->tuning : nullptr);
    RTDM_REQUIRE(h, RTDM_E_INVALID, "classifier_enable_timing: NULL handle");
    for (hipEvent_t e : h->events) (void)hipEventDestroy(e);
    h->events.clear();
    h->timing = max_calls > 0;
    h->timing_cap = max_calls > 0 ? max_calls : 0;
    h->timing_calls = 0;
    h->n_seg = 0;
    const size_t ne = (size_t)h->timing_cap * 2 * rtdm_classifier_s::kMaxSeg;
    h->events.resize(ne);
    for (size_t i = 0; i < ne; ++i) RTDM_HIP(hipEventCreateWithFlags(&h->events[i], hipEventDisableSystemFence));
  });
}

rtdm_status rtdm_classifier_read_timing(rtdm_classifier h, double* ms_per_launch, double* bytes_per_launch,
                                        char* names, int name_stride, int* n_launches, int* calls) {
  return guard([&] {
    TuningScope ts_(h ? &h->tuning : nullptr);
    RTDM_REQUIRE(h, RTDM_E_INVALID, "classifier_read_timing: NULL handle");
    // every timed call must have recorded the first call's launches (the names / bytes are the
    // first call's): a call with another launch sequence (frames vs NCHW input, another
    // chain mode) is refused, not summed into mismatched slots
    const int ns = h->timing_calls > 0 ? (int)h->seg_name.size() : 0;
    for (int c = 0; c < h->timing_calls; ++c)
      RTDM_REQUIRE(h->call_segs[c] == ns, RTDM_E_INVALID,
                   "classifier_read_timing: timed call " + std::to_string(c) + " recorded " +
                       std::to_string(h->call_segs[c]) + " launches, the first " + std::to_string(ns));
    for (int i = 0; i < ns; ++i) {
      double t = 0.0;
      for (int c = 0; c < h->timing_calls; ++c) {
        hipEvent_t* ev = &h->events[(size_t)c * 2 * rtdm_classifier_s::kMaxSeg];
        float ms = 0.f;
        RTDM_HIP(hipEventSynchronize(ev[2 * i + 1]));
        RTDM_HIP(hipEventElapsedTime(&ms, ev[2 * i], ev[2 * i + 1]));
        t += ms;
      }
      if (ms_per_launch) ms_per_launch[i] = t;
      if (bytes_per_launch) bytes_per_launch[i] = i < (int)h->seg_bytes.size() ? h->seg_bytes[i] : 0.0;
      if (names && name_stride > 0) {
        const std::string& nm = i < (int)h->seg_name.size() ? h->seg_name[i] : std::string();
        std::snprintf(names + (size_t)i * name_stride, name_stride, "%s", nm.c_str());
      }
    }
    if (n_launches) *n_launches = ns;
    if (calls) *calls = h->timing_calls;
  });
}

int rtdm_classifier_input_size(rtdm_classifier h) { return h ? h->S : 0; }

int64_t rtdm_classifier_describe(rtdm_classifier h, char* buf, int64_t buf_len) {
  if (!h) return 0;
  TuningScope ts_(&h->tuning);
  std::string s = "classifier S " + std::to_string(h->S) + " dtype " +
                  (h->int8 ? "i8" : h->dtype == RTDM_F16 ? "f16" : "f32") + " max_batch " +
                  std::to_string(h->max_batch) + "\n";
  {  // conv1 as classify() launches it on the transformed (NHWC) frames
    ConvArgs a;
    a.in_kind = IN_NHWC;
    a.in_cs = 3;
    // (any non-null output view: only its presence is read)
    stem_conv_args(*h, a, 1, View{h->blob.at<void>(0), h->stem_cout, 0});
    s += std::string("conv1 kernel ") + conv_kernel_name(a, h->dtype) + "\n";
    if (front_fusable(*h))
      s += "conv1 on frames: fused with the transform (resize_stream_kernel<stem>, frame rows 16-byte multiples)\n";
  }
  const bool chain = h->chain_start >= 0 && acff_chain_mode();
  const bool band = h->band_start >= 0 && acff_band_mode();
  for (int i = 0; i < (int)h->stages.size(); ++i) {
    const AcffStage& st = h->stages[i];
    const int band_start = acff_band_mode() == 2 ? std::max(h->band_start, h->chain_start) : h->band_start;
    const char* k = band && i >= band_start                          ? "acff_band"
                    : chain && i >= h->chain_start                   ? "acff_chain"
                    : st.persist_cc && (acff_persist_mode() || st.q8) ? "acff_persist"
                    : st.fused                                        ? "acff_fused"
                                                                      : "dw3+gemm";
    s += "acff" + std::to_string(i + 1) + " cin " + std::to_string(st.cin) + " cout " + std::to_string(st.cout) +
         " in " + std::to_string(st.h) + "x" + std::to_string(st.w) + " kernel " + k + " pool " +
         std::to_string(st.pool ? 1 : 0) + " red " + std::to_string(st.red ? 1 : 0) + " int8 " +
         std::to_string(st.q8 ? 1 : 0) + "\n";
  }
  const int64_t need = (int64_t)s.size() + 1;
  if (buf && buf_len >= need) std::memcpy(buf, s.c_str(), need);
  return need;
}

rtdm_status rtdm_classifier_calibrate(rtdm_classifier h, const void* x, int x_kind, int n, int in_h, int in_w,
                                      int reset, void* stream) {
  return guard([&] {
    TuningScope ts_(h ? &h->tuning : nullptr);
    RTDM_REQUIRE(h, RTDM_E_INVALID, "classifier_calibrate: NULL handle");
    RTDM_REQUIRE(h->int8, RTDM_E_INVALID, "classifier_calibrate: handle is not RTDM_I8");
    if (h->q_channels == 0) {
      h->calibrated = true;
      return;
    }
    RTDM_REQUIRE(acff_chain_mode() == 1 || h->chain_start < 0, RTDM_E_INVALID, "classifier_calibrate: acff_chain mode");
    const hipStream_t s = (hipStream_t)stream;
    if (reset) RTDM_HIP(hipMemsetAsync(h->amax.p, 0, (size_t)h->q_channels * sizeof(unsigned), s));
    if (n > 0) {
      DevBuf out;
      out.alloc((size_t)n * 10 * sizeof(float));
      h->calibrating = true;  // fp16 forward, |x|max of every int8 stage's depthwise concat
      try {
        run_classifier(*h, x, x_kind, n, in_h, in_w, out.as<float>(), out.as<float>() + (size_t)n * 5, s);
      } catch (...) {
        h->calibrating = false;
        throw;
      }
      h->calibrating = false;
    }
    // per int8 stage, per concat channel k = branch*cin + c: s_k = |x|max_k / 127 folded into
    // the fusion weights (W'[o][k] = W[o][k] s_k), symmetric per-output-channel int8 of W'
    // (s_w[o] = max_k |W'[o][k]| / 127, W8 = rint(W' / s_w[o]), deq[o] = s_w[o]) — the
    // detector's scheme (rtdm_detector_calibrate) on the ACFF concat
    std::vector<unsigned> am(h->q_channels);
    RTDM_HIP(hipMemcpyAsync(am.data(), h->amax.p, am.size() * sizeof(unsigned), hipMemcpyDeviceToHost, s));
    RTDM_HIP(hipStreamSynchronize(s));
    for (const AcffStage& st : h->stages) {
      if (!st.q8) continue;
      const int K = 3 * st.cin, cp = st.pw.cout_pad;
      std::vector<float> sx(K), inv(K);
      for (int k = 0; k < K; ++k) {
        float mx;
        std::memcpy(&mx, &am[st.amax_off + k], sizeof(float));
        RTDM_REQUIRE(std::isfinite(mx), RTDM_E_INVALID, "classifier_calibrate: non-finite activations");
        sx[k] = mx > 0.f ? mx / 127.f : 1.f;
        inv[k] = 1.f / sx[k];
      }
      const int cc = st.persist_cc, nch = cc ? st.cin / cc : 1;
      const size_t kq = cc ? (size_t)nch * 64 : (size_t)K;
      std::vector<int8_t> w8((size_t)cp * kq, 0);
      std::vector<float> dq(cp, 0.f);
      for (int o = 0; o < st.cout; ++o) {
        const float* row = &st.wf[(size_t)o * K];
        double mx = 0.0;
        for (int k = 0; k < K; ++k) mx = std::max(mx, std::fabs((double)row[k] * sx[k]));
        const double sw = mx > 0.0 ? mx / 127.0 : 1.0;
        dq[o] = (float)sw;
        for (int k = 0; k < K; ++k) {
          const long q = std::max(-127L, std::min(127L, std::lround((double)row[k] * sx[k] / sw)));
          size_t dst = (size_t)k;  // chain: k = branch*cin + c
          if (cc) {                // persist: chunk*64 + branch*cc + c_local
            const int br = k / st.cin, c = k - br * st.cin;
            dst = (size_t)(c / cc) * 64 + br * cc + c % cc;
          }
          w8[(size_t)o * kq + dst] = (int8_t)q;
        }
      }
      RTDM_HIP(hipMemcpy(h->blob.at<void>(st.w8_off), w8.data(), w8.size(), hipMemcpyHostToDevice));
      RTDM_HIP(hipMemcpy(h->blob.at<void>(st.deq_off), dq.data(), dq.size() * sizeof(float), hipMemcpyHostToDevice));
      RTDM_HIP(hipMemcpy(h->blob.at<void>(st.inv_off), inv.data(), inv.size() * sizeof(float), hipMemcpyHostToDevice));
    }
    h->calibrated = true;
  });
}

rtdm_status rtdm_classify(rtdm_classifier h, const void* x, int x_kind, int n, int in_h, int in_w, float* logits,
                          float* probs, void* stream) {
  return guard([&] {
    TuningScope ts_(h ? &h->tuning : nullptr);
    RTDM_REQUIRE(h, RTDM_E_INVALID, "classify: NULL handle");
    run_classifier(*h, x, x_kind, n, in_h, in_w, logits, probs, (hipStream_t)stream);
  });
}

}  // extern "C"
