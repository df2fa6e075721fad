// Darknet (cfg-driven YOLO) detector runtime.
//
// Parses a Darknet .cfg like parse_model_cfg (yolov3/utils/parse_config.py:6-52),
// infers shapes like create_modules (yolov3/models.py:9-123), loads the darknet
// weight stream like load_darknet_weights (models.py:449-486, BN folded into
// the conv: eps 1e-4), and plans Darknet.forward (models.py:332-395) as a
// sequence of kernel launches over NHWC buffers with these fusions:
//   conv -> maxpool(2,2)         : 2x2 max in the conv epilogue (quad rows)
//   conv -> upsample(2)          : x2 nearest stores in the conv epilogue
//   conv -> shortcut             : residual add in the conv epilogue
//   conv -> yolo                 : YOLOLayer decode in the conv epilogue -> io
//   route (concat)               : producers write straight into channel
//                                  slices of the concat buffer (zero copy)
// Anything else runs as its own kernel (maxpool k/s, upsample, slice copy).
#include <map>
#include <sstream>

#include "weights.h"

namespace rtdm {

struct CfgBlock {
  std::string type;
  std::map<std::string, std::string> kv;
  bool has(const std::string& k) const { return kv.count(k) != 0; }
  std::string str(const std::string& k, const std::string& def = "") const {
    auto it = kv.find(k);
    return it == kv.end() ? def : it->second;
  }
  int i(const std::string& k, int def) const {
    auto it = kv.find(k);
    if (it == kv.end()) return def;
    try {
      return std::stoi(it->second);
    } catch (...) {
      throw Error{RTDM_E_INVALID, "cfg: [" + type + "] " + k + "=" + it->second + " is not an integer"};
    }
  }
  std::vector<int> ints(const std::string& k) const {
    std::vector<int> out;
    std::stringstream ss(str(k));
    std::string tok;
    while (std::getline(ss, tok, ',')) out.push_back(std::stoi(tok));
    return out;
  }
  std::vector<double> floats(const std::string& k) const {
    std::vector<double> out;
    std::stringstream ss(str(k));
    std::string tok;
    while (std::getline(ss, tok, ',')) out.push_back(std::stod(tok));
    return out;
  }
};

static std::string strip(const std::string& s) {
  size_t a = 0, b = s.size();
  while (a < b && isspace((unsigned char)s[a])) ++a;
  while (b > a && isspace((unsigned char)s[b - 1])) --b;
  return s.substr(a, b - a);
}

// parse_config.py:6-52
static std::vector<CfgBlock> parse_cfg(const std::string& text) {
  std::vector<CfgBlock> defs;
  std::stringstream ss(text);
  std::string line;
  while (std::getline(ss, line)) {
    if (line.empty() || line[0] == '#') continue;
    line = strip(line);
    if (line.empty()) continue;
    if (line[0] == '[') {
      CfgBlock b;
      b.type = strip(line.substr(1, line.size() - 2));
      if (b.type == "convolutional") b.kv["batch_normalize"] = "0";
      defs.push_back(b);
    } else {
      const size_t eq = line.find('=');
      RTDM_REQUIRE(eq != std::string::npos, RTDM_E_INVALID, "cfg: line without '=': " + line);
      RTDM_REQUIRE(!defs.empty(), RTDM_E_INVALID, "cfg: key before first [section]");
      defs.back().kv[strip(line.substr(0, eq))] = strip(line.substr(eq + 1));
    }
  }
  RTDM_REQUIRE(!defs.empty() && (defs[0].type == "net" || defs[0].type == "network"), RTDM_E_INVALID,
               "cfg: first section must be [net]");
  return defs;
}

// ST_DW3: an [acff] block's three dilated depthwise branches, ADDED (models.py:302), into a
// [C] scratch map (its 1x1 fusion is the ST_CONV after it); ST_RESIZE: the route's nearest resize of the
// narrower of two maps (models.py:364-375)
// ST_ADD: a [shortcut] that cannot ride the previous conv's epilogue (that conv's pre-add
// output is also routed elsewhere): out = in + res
enum StepKind { ST_CONV = 0, ST_MAXPOOL = 1, ST_UPSAMPLE = 2, ST_COPY = 3, ST_DW3 = 4, ST_RESIZE = 5, ST_ADD = 6 };

struct Tensor {
  int c = 0, h = 0, w = 0;
  int home = -1;         // concat tensor id this one lives in (slice), or -1
  int home_co = 0;       // channel offset inside home
  bool own = false;      // has its own buffer
  size_t off = 0;        // arena offset (elements per image) of own buffer
  bool materialised = false;
  std::string what;
};

struct Step {
  int kind = ST_CONV;
  int layer = -1;
  int in_t = -1;  // -1 = network input
  // conv
  PackedConv pc;
  int ks = 1, stride = 1, pad = 0, act = ACT_LINEAR, cin = 0, cout = 0;
  int ih = 0, iw = 0, oh = 0, ow = 0;
  int full_t = -1, pool_t = -1, up_t = -1, res_t = -1;
  int yolo = -1;  // index into yolo heads
  bool quad = false;
  // Darknet-53's first residual block: this 1x1 reduce (64 -> 32), whose map only the next
  // step (3x3 32 -> 64 with this step's input as its shortcut) reads, runs with it as one
  // conv3_c32r launch when the shapes fit (c32r_ok)
  bool fuse_r = false;
  float slope = 0.1f;  // LeakyReLU slope: 0.1 Darknet conv (models.py:40), 0.01 ACFF (:291)
  // [acff] (models.py:46-55, ACFF :265-315): this ST_CONV is the 1x1 fusion over the
  // ST_DW3 map b1+b2+b3 with the fused_conv weights [F][C]; BN is the post-activation
  // affine a_bn = [gamma | beta | mean | var], eps 1e-5
  bool acff = false;
  std::vector<float> a_W;
  const float* a_bn = nullptr;
  const float* a_dw = nullptr;  // ST_DW3: [w1 C*9 | b1 C | w2 | b2 | w3 | b3]
  size_t dw_w_off = SIZE_MAX, dw_b_off = SIZE_MAX;
  // fused 1x1 head conv (layer + 1) feeding a [yolo] (layer + 2): conv_pipe_f16 head
  // epilogue; this conv's own output is not materialised
  bool head = false;
  int head_cout = 0, head_act = ACT_LINEAR;
  bool head_bn = false;
  const float *h_beta = nullptr, *h_gamma = nullptr, *h_mean = nullptr, *h_var = nullptr, *h_bias = nullptr,
              *h_W = nullptr;
  PackedConv hpc;
  bool bn = false;  // raw darknet weights (host), packed after planning
  const float *w_beta = nullptr, *w_gamma = nullptr, *w_mean = nullptr, *w_var = nullptr, *w_bias = nullptr,
              *w_W = nullptr;
  // int8 (RTDM_I8 handles): slot of this conv among the int8 convs (-1: fp16 conv); its
  // BN-folded fp32 weights [cout][k] (host, k = tap * cin + c) for the calibration that
  // folds the per-channel activation scales in; device slots of the int8 weights, the
  // dequantisation scales deq[o] and the input's inverse activation scales; the offsets
  // of its per-channel |x|max (amax) and of its quantised input copy (qarena, per image)
  int q = -1;
  size_t w8_off = SIZE_MAX, deq_off = SIZE_MAX, inv_off = SIZE_MAX;
  std::vector<float> wf;
  size_t amax_off = 0, qbuf_off = 0;
  // two-stream schedule (schedule_streams): stream 0 = the caller's, 1 = the side stream
  int stream = 0;
  std::vector<int> deps;    // earlier steps writing a buffer this step reads
  bool signal = false;      // a step on the other stream waits for this one
  // maxpool / upsample / copy
  int out_t = -1;
  int k = 0, s = 0, p = 0, zero_rb = 0, f = 0;
};

struct YoloHead {
  int layer = 0, na = 0, no = 0, ny = 0, nx = 0, io_off = 0;
  float ystride = 0.f;
  std::vector<float> anchor_vec;
  // TensorRT YoloLayer_TRT fields for rtdm_detect_trt (yolo_layer.cu:352-419): masked
  // anchors in pixels, [yolo] scale_x_y / new_coords (default 1 / 0)
  std::vector<float> anchor_px;
  float scale_xy = 1.f;
  int new_coords = 0;
  size_t anchor_off = 0;  // device copy in the weight blob
};

}  // namespace rtdm

struct rtdm_detector_s {
  int img_h = 0, img_w = 0, dtype = 0, max_batch = 0, dev = 0;
  rtdm::Tuning tuning;  // this handle's knobs (rtdm_detector_set_tuning; the defaults at create)
  bool planning_only = true;
  // RTDM_I8: activations fp16 (dtype = RTDM_F16) in the arena; the Cin % 128 == 0 convs
  // run conv_pipe_i8 on a per-channel int8 copy of their input once calibrated
  // (rtdm_detector_calibrate); calibrating = the fp16 forward recording every int8
  // conv's per-channel input |x|max
  bool int8 = false, calibrated = false;
  int calibrating = 0;
  int n_q = 0;
  size_t q_channels = 0, q_bytes = 0;  // sum of int8 conv input channels; int8 copy bytes per image
  rtdm::DevBuf amax, qarena;           // [q_channels] float bits; [max_batch * q_bytes] int8
  std::vector<rtdm::CfgBlock> defs;  // without [net]
  std::vector<rtdm::Tensor> tensors;
  std::vector<rtdm::Step> steps;
  std::vector<rtdm::YoloHead> heads;
  std::vector<int> layer_tensor;  // cfg layer -> tensor id
  int n_anchors_total = 0, no = 0, nc = 0;
  int64_t weight_floats = 0;
  double flop = 0.0;
  size_t per_image = 0;  // arena elements per image
  rtdm::DevBlob blob;
  rtdm::DevBuf arena;
  rtdm::DevBuf zero;  // 256 zero bytes: padding source of the glds conv kernel
  rtdm::DevBuf raw_buf;  // raw head rows for rtdm_detect_trt (allocated on first use)
  int last_n = 0;
  std::vector<int> fused_away;  // tensors the last rtdm_detect call never wrote (fused stem pairs)
  // optional per-step timing: events[call][2*step + {0,1}] recorded around each step
  // on the stream it runs on
  bool timing = false;
  int timing_cap = 0, timing_calls = 0;
  std::vector<hipEvent_t> events;
  // two-stream execution of independent branches (heads): side stream + one
  // event per signalling step, plus fork / join events
  bool two_streams = false;
  hipStream_t side = nullptr;
  std::vector<hipEvent_t> step_ev;
  hipEvent_t fork_ev = nullptr, join_ev = nullptr;
  ~rtdm_detector_s() {
    for (hipEvent_t e : events) (void)hipEventDestroy(e);
    for (hipEvent_t e : step_ev)
      if (e) (void)hipEventDestroy(e);
    if (fork_ev) (void)hipEventDestroy(fork_ev);
    if (join_ev) (void)hipEventDestroy(join_ev);
    if (side) (void)hipStreamDestroy(side);
  }
};

namespace rtdm {

int fuse_head() { return tune().fuse_head; }

static size_t esize_of(int dtype) { return dtype == RTDM_F16 ? 2 : 4; }

static bool implicit_input(const std::string& t) {
  return t == "convolutional" || t == "acff" || t == "maxpool" || t == "upsample" || t == "shortcut" || t == "yolo";
}

static int resolve_ref(int layer, int l) { return l < 0 ? layer + l : l; }

// int8 activation scale headroom over the calibration |x|max (rtdm.h RTDM_I8)
constexpr float kI8Headroom = 2.0f;

static void plan(rtdm_detector_s& h, const float* weights, int64_t n_floats) {
  auto& defs = h.defs;
  const int L = (int)defs.size();
  const bool f16 = h.dtype == RTDM_F16;
  // ---- consumers (who reads out[i]) ----
  std::vector<std::vector<int>> consumers(L);
  for (int j = 0; j < L; ++j) {
    const std::string& t = defs[j].type;
    if (j > 0 && implicit_input(t)) consumers[j - 1].push_back(j);
    if (t == "route")
      for (int l : defs[j].ints("layers")) {
        const int s = resolve_ref(j, l);
        RTDM_REQUIRE(s >= 0 && s < j, RTDM_E_INVALID, "cfg: route " + std::to_string(j) + " references bad layer");
        consumers[s].push_back(j);
      }
    if (t == "shortcut")
      for (int l : defs[j].ints("from")) {
        const int s = resolve_ref(j, l);
        RTDM_REQUIRE(s >= 0 && s < j, RTDM_E_INVALID, "cfg: shortcut " + std::to_string(j) + " references bad layer");
        consumers[s].push_back(j);
      }
  }
  auto new_tensor = [&](int c, int hh, int ww, const std::string& what) {
    Tensor t;
    t.c = c;
    t.h = hh;
    t.w = ww;
    t.what = what;
    h.tensors.push_back(t);
    return (int)h.tensors.size() - 1;
  };
  h.layer_tensor.assign(L, -1);
  std::vector<bool> fused(L, false);
  int cur_c = 3, cur_h = h.img_h, cur_w = h.img_w;  // shape of x
  int cur_t = -1;
  int64_t wptr = 0;
  Blob blob;
  auto take_w = [&](int64_t n) -> const float* {
    const int64_t at = wptr;
    wptr += n;
    if (!weights) return nullptr;
    RTDM_REQUIRE(wptr <= n_floats, RTDM_E_INVALID,
                 "darknet weights: stream too short (" + std::to_string(n_floats) + " floats)");
    return weights + at;
  };
  std::vector<int> out_c(L), out_h(L), out_w(L);
  int nc_all = -1;
  for (int i = 0; i < L; ++i) {
    const CfgBlock& d = defs[i];
    const std::string& t = d.type;
    if (fused[i]) {  // produced by the previous conv's epilogue; shape already set
      out_c[i] = cur_c;
      out_h[i] = cur_h;
      out_w[i] = cur_w;
      continue;
    }
    if (t == "convolutional" || t == "acff") {
      const bool is_acff = t == "acff";
      const int bn = is_acff ? 0 : d.i("batch_normalize", 0);
      const int filters = d.i("filters", 0);
      const int size = is_acff ? 1 : d.i("size", 1);
      RTDM_REQUIRE(is_acff || d.has("stride"), RTDM_E_UNSUPPORTED, "cfg: conv without stride (stride_x/stride_y) unsupported");
      const int stride = is_acff ? 1 : d.i("stride", 1);
      const int pad = is_acff ? 0 : d.i("pad", 0) ? (size - 1) / 2 : 0;
      RTDM_REQUIRE(d.i("groups", 1) == 1, RTDM_E_UNSUPPORTED, "cfg: grouped conv unsupported");
      const std::string actn = is_acff ? "leaky" : d.str("activation", "linear");
      int act = ACT_LINEAR;
      if (actn == "leaky")
        act = ACT_LEAKY;
      else if (actn == "swish")
        act = ACT_SWISH;
      const int acff_c = cur_c;
      if (is_acff) {
        // three dilated depthwise branches d1p0 / d2p1 / d3p2, each [C, H-2, W-2] (+bias),
        // summed into one [C] map for the 1x1 fusion conv below
        RTDM_REQUIRE(d.i("size", 3) == 3, RTDM_E_UNSUPPORTED, "cfg: acff size must be 3");
        RTDM_REQUIRE(cur_h > 2 && cur_w > 2 && cur_t >= 0, RTDM_E_UNSUPPORTED, "cfg: acff input too small");
        Step dw;
        dw.kind = ST_DW3;
        dw.layer = i;
        dw.in_t = cur_t;
        dw.cin = cur_c;
        dw.ih = cur_h;
        dw.iw = cur_w;
        dw.oh = cur_h - 2;
        dw.ow = cur_w - 2;
        dw.a_dw = take_w(3 * ((int64_t)cur_c * 9 + cur_c));
        h.tensors[cur_t].materialised = true;
        dw.out_t = new_tensor(cur_c, dw.oh, dw.ow, "acffdw" + std::to_string(i));
        h.tensors[dw.out_t].materialised = true;
        h.flop += 2.0 * dw.oh * dw.ow * 3.0 * cur_c * 9;
        h.steps.push_back(dw);
        cur_t = dw.out_t;
        cur_h -= 2;
        cur_w -= 2;
      }
      // create_modules adds no module for any other activation (models.py:40-44): identity
      Step s;
      s.kind = ST_CONV;
      s.layer = i;
      s.in_t = cur_t;
      s.ks = size;
      s.stride = stride;
      s.pad = pad;
      s.act = act;
      s.cin = cur_c;
      s.cout = filters;
      s.ih = cur_h;
      s.iw = cur_w;
      s.oh = (cur_h + 2 * pad - size) / stride + 1;
      s.ow = (cur_w + 2 * pad - size) / stride + 1;
      RTDM_REQUIRE(s.oh > 0 && s.ow > 0, RTDM_E_UNSUPPORTED, "cfg: conv output empty at layer " + std::to_string(i));
      h.flop += 2.0 * s.oh * s.ow * (double)filters * (is_acff ? acff_c : cur_c) * size * size;
      // weights: [bn: beta gamma mean var | bias] then W
      const float *beta = nullptr, *gamma = nullptr, *mean = nullptr, *var = nullptr, *bias = nullptr;
      if (bn) {
        beta = take_w(filters);
        gamma = take_w(filters);
        mean = take_w(filters);
        var = take_w(filters);
      } else if (!is_acff) {
        bias = take_w(filters);
      }
      const float* W = nullptr;
      if (is_acff) {  // fused_conv weight [F][C], bias [F], then BN gamma/beta/mean/var
        const float* w1 = take_w((int64_t)filters * acff_c);
        bias = take_w(filters);
        s.a_bn = take_w(4 * (int64_t)filters);
        if (w1) s.a_W.assign(w1, w1 + (size_t)filters * acff_c);
        s.acff = true;
        s.slope = 0.01f;
      } else {
        W = take_w((int64_t)filters * cur_c * size * size);
      }
      s.bn = bn != 0;
      s.w_beta = beta;
      s.w_gamma = gamma;
      s.w_mean = mean;
      s.w_var = var;
      s.w_bias = bias;
      s.w_W = W;
      const int full = new_tensor(filters, s.oh, s.ow, "conv" + std::to_string(i));
      s.full_t = full;
      h.layer_tensor[i] = full;
      cur_c = filters;
      cur_h = s.oh;
      cur_w = s.ow;
      cur_t = full;
      // ---- epilogue fusion with layer i+1 ----
      std::vector<int> others;
      for (int c : consumers[i])
        if (c != i + 1) others.push_back(c);
      bool need_full = !others.empty();
      if (i + 1 < L) {
        const CfgBlock& nx = defs[i + 1];
        const bool only_next = consumers[i].size() == 1 && consumers[i][0] == i + 1;
        if (nx.type == "maxpool" && nx.i("size", 0) == 2 && nx.i("stride", 0) == 2 && s.oh % 2 == 0 &&
            s.ow % 2 == 0) {
          s.quad = true;
          s.pool_t = new_tensor(filters, s.oh / 2, s.ow / 2, "pool" + std::to_string(i + 1));
          h.tensors[s.pool_t].materialised = true;
          fused[i + 1] = true;
          h.layer_tensor[i + 1] = s.pool_t;
          cur_t = s.pool_t;
          cur_h = s.oh / 2;
          cur_w = s.ow / 2;
        } else if (nx.type == "upsample" && nx.i("stride", 0) == 2 && only_next) {
          s.up_t = new_tensor(filters, s.oh * 2, s.ow * 2, "up" + std::to_string(i + 1));
          h.tensors[s.up_t].materialised = true;
          fused[i + 1] = true;
          h.layer_tensor[i + 1] = s.up_t;
          cur_t = s.up_t;
          cur_h = s.oh * 2;
          cur_w = s.ow * 2;
        } else if (nx.type == "shortcut" && only_next && nx.ints("from").size() == 1 &&
                   resolve_ref(i + 1, nx.ints("from")[0]) != i && !nx.has("weights_type") &&
                   h.layer_tensor[resolve_ref(i + 1, nx.ints("from")[0])] >= 0 &&
                   h.tensors[h.layer_tensor[resolve_ref(i + 1, nx.ints("from")[0])]].c == filters) {
          // same-channel shortcut fused as the residual epilogue; a channel mismatch runs the
          // unfused ST_ADD below (weightedFeatureFusion's slicing)
          const int src = resolve_ref(i + 1, nx.ints("from")[0]);
          const int st = h.layer_tensor[src];
          RTDM_REQUIRE(st >= 0, RTDM_E_UNSUPPORTED, "cfg: shortcut source not materialisable");
          RTDM_REQUIRE(h.tensors[st].c == filters && h.tensors[st].h == s.oh && h.tensors[st].w == s.ow,
                       RTDM_E_UNSUPPORTED, "cfg: shortcut with channel/shape mismatch unsupported");
          s.res_t = st;
          fused[i + 1] = true;
          h.layer_tensor[i] = -1;        // the pre-add conv output is never materialised
          h.layer_tensor[i + 1] = full;  // conv output with the residual added
          need_full = !consumers[i + 1].empty();
        } else if (f16 && fuse_head() && !is_acff && nx.type == "convolutional" && only_next && i + 2 < L && defs[i + 2].type == "yolo" &&
                   consumers[i + 1].size() == 1 && consumers[i + 1][0] == i + 2 && consumers[i + 2].empty() &&
                   nx.i("size", 1) == 1 && nx.i("stride", 1) == 1 && nx.i("groups", 1) == 1 &&
                   nx.i("filters", 0) <= 32 && filters > 64 && filters <= 128 &&
                   s.cin % 64 == 0 && (size == 1 || size == 3) &&
                   (nx.str("activation", "linear") == "linear" || nx.str("activation", "linear") == "leaky")) {
          // conv -> 1x1 head conv -> YOLOLayer (models.py:185-258): the head GEMM and the
          // decode run in this conv's epilogue (conv_pipe_f16 head variant)
          const int hf = nx.i("filters", 0);
          const int hbn = nx.i("batch_normalize", 0);
          s.head = true;
          s.head_cout = hf;
          s.head_act = nx.str("activation", "linear") == "leaky" ? ACT_LEAKY : ACT_LINEAR;
          s.head_bn = hbn != 0;
          if (hbn) {
            s.h_beta = take_w(hf);
            s.h_gamma = take_w(hf);
            s.h_mean = take_w(hf);
            s.h_var = take_w(hf);
          } else {
            s.h_bias = take_w(hf);
          }
          s.h_W = take_w((int64_t)hf * filters);
          h.flop += 2.0 * s.oh * s.ow * (double)hf * filters;
          const CfgBlock& yb = defs[i + 2];
          YoloHead yh;
          yh.layer = i + 2;
          const std::vector<int> mask = yb.ints("mask");
          const std::vector<double> anc = yb.floats("anchors");
          const int ncls = yb.i("classes", 0);
          yh.na = (int)mask.size();
          yh.no = ncls + 5;
          yh.ny = s.oh;
          yh.nx = s.ow;
          RTDM_REQUIRE(yh.na > 0 && yh.na <= 8, RTDM_E_UNSUPPORTED, "cfg: yolo with more than 8 anchors");
          RTDM_REQUIRE(hf == yh.na * yh.no, RTDM_E_INVALID,
                       "cfg: yolo head conv has " + std::to_string(hf) + " filters, expected na*(nc+5)");
          RTDM_REQUIRE(nc_all < 0 || nc_all == ncls, RTDM_E_UNSUPPORTED, "cfg: yolo heads disagree on classes");
          nc_all = ncls;
          const double isz = std::max(h.img_h, h.img_w);
          const double ystride = isz / (double)std::max(s.oh, s.ow);
          yh.ystride = (float)ystride;
          for (int a : mask) {
            RTDM_REQUIRE(2 * a + 1 < (int)anc.size(), RTDM_E_INVALID, "cfg: yolo mask out of range");
            yh.anchor_vec.push_back((float)anc[2 * a] / (float)ystride);
            yh.anchor_vec.push_back((float)anc[2 * a + 1] / (float)ystride);
            yh.anchor_px.push_back((float)anc[2 * a]);
            yh.anchor_px.push_back((float)anc[2 * a + 1]);
          }
          yh.scale_xy = yb.has("scale_x_y") ? (float)std::stod(yb.str("scale_x_y")) : 1.f;
          yh.new_coords = yb.i("new_coords", 0);
          yh.io_off = h.n_anchors_total;
          h.n_anchors_total += yh.na * yh.ny * yh.nx;
          s.yolo = (int)h.heads.size();
          h.heads.push_back(yh);
          const int ht = new_tensor(hf, s.oh, s.ow, "conv" + std::to_string(i + 1));
          fused[i + 1] = true;
          fused[i + 2] = true;
          h.layer_tensor[i] = -1;
          h.layer_tensor[i + 1] = ht;  // never materialised: only the decoded io leaves the kernel
          h.layer_tensor[i + 2] = ht;
          need_full = false;
        } else if (nx.type == "yolo" && only_next) {
          // YOLOLayer (models.py:185-258) fused into this head conv
          YoloHead yh;
          yh.layer = i + 1;
          const std::vector<int> mask = nx.ints("mask");
          const std::vector<double> anc = nx.floats("anchors");
          const int ncls = nx.i("classes", 0);
          yh.na = (int)mask.size();
          yh.no = ncls + 5;
          yh.ny = s.oh;
          yh.nx = s.ow;
          RTDM_REQUIRE(yh.na > 0 && yh.na <= 8, RTDM_E_UNSUPPORTED, "cfg: yolo with more than 8 anchors");
          RTDM_REQUIRE(filters == yh.na * yh.no, RTDM_E_INVALID,
                       "cfg: yolo head conv has " + std::to_string(filters) + " filters, expected na*(nc+5)");
          RTDM_REQUIRE(nc_all < 0 || nc_all == ncls, RTDM_E_UNSUPPORTED, "cfg: yolo heads disagree on classes");
          nc_all = ncls;
          // create_grids: img_size = max(img), stride = img_size / max(ng) (models.py:424-425)
          const double isz = std::max(h.img_h, h.img_w);
          const double ystride = isz / (double)std::max(s.oh, s.ow);
          yh.ystride = (float)ystride;
          for (int a : mask) {
            RTDM_REQUIRE(2 * a + 1 < (int)anc.size(), RTDM_E_INVALID, "cfg: yolo mask out of range");
            yh.anchor_vec.push_back((float)anc[2 * a] / (float)ystride);
            yh.anchor_vec.push_back((float)anc[2 * a + 1] / (float)ystride);
            yh.anchor_px.push_back((float)anc[2 * a]);
            yh.anchor_px.push_back((float)anc[2 * a + 1]);
          }
          yh.scale_xy = nx.has("scale_x_y") ? (float)std::stod(nx.str("scale_x_y")) : 1.f;
          yh.new_coords = nx.i("new_coords", 0);
          yh.io_off = h.n_anchors_total;
          h.n_anchors_total += yh.na * yh.ny * yh.nx;
          s.yolo = (int)h.heads.size();
          h.heads.push_back(yh);
          fused[i + 1] = true;
          h.layer_tensor[i + 1] = full;
          need_full = need_full || !consumers[i + 1].empty();
        }
      }
      h.tensors[full].materialised = need_full || (s.pool_t < 0 && s.up_t < 0 && s.yolo < 0);
      if (s.head) {
        // shape bookkeeping continues from the head conv's output (layer i+2 = yolo)
        cur_c = s.head_cout;
        cur_t = h.layer_tensor[i + 1];
      }
      if (!h.tensors[full].materialised) s.full_t = -1;
      if (s.quad && h.tensors[full].materialised) {
        RTDM_REQUIRE(s.oh % 2 == 0 && s.ow % 2 == 0, RTDM_E_INVALID, "internal: quad with odd full output");
      }
      h.steps.push_back(s);
    } else if (t == "maxpool") {
      const int k = d.i("size", 2), st = d.i("stride", 2);
      Step s;
      s.kind = ST_MAXPOOL;
      s.layer = i;
      s.in_t = cur_t;
      s.k = k;
      s.s = st;
      s.cin = cur_c;
      s.ih = cur_h;
      s.iw = cur_w;
      if (k == 2 && st == 1) {  // ZeroPad2d((0,1,0,1)) + MaxPool2d(2,1) (models.py:62-64)
        s.zero_rb = 1;
        s.p = 0;
        s.oh = (cur_h + 1 - k) / st + 1;
        s.ow = (cur_w + 1 - k) / st + 1;
      } else {
        s.p = (k - 1) / 2;
        s.oh = (cur_h + 2 * s.p - k) / st + 1;
        s.ow = (cur_w + 2 * s.p - k) / st + 1;
      }
      RTDM_REQUIRE(cur_t >= 0, RTDM_E_UNSUPPORTED, "cfg: maxpool on the network input");
      s.out_t = new_tensor(cur_c, s.oh, s.ow, "maxpool" + std::to_string(i));
      h.tensors[s.out_t].materialised = true;
      h.layer_tensor[i] = s.out_t;
      cur_h = s.oh;
      cur_w = s.ow;
      cur_t = s.out_t;
      h.steps.push_back(s);
    } else if (t == "upsample") {
      Step s;
      s.kind = ST_UPSAMPLE;
      s.layer = i;
      s.in_t = cur_t;
      s.f = d.i("stride", 2);
      s.cin = cur_c;
      s.ih = cur_h;
      s.iw = cur_w;
      s.oh = cur_h * s.f;
      s.ow = cur_w * s.f;
      RTDM_REQUIRE(cur_t >= 0, RTDM_E_UNSUPPORTED, "cfg: upsample on the network input");
      s.out_t = new_tensor(cur_c, s.oh, s.ow, "upsample" + std::to_string(i));
      h.tensors[s.out_t].materialised = true;
      h.layer_tensor[i] = s.out_t;
      cur_h = s.oh;
      cur_w = s.ow;
      cur_t = s.out_t;
      h.steps.push_back(s);
    } else if (t == "route") {
      const std::vector<int> ls = d.ints("layers");
      RTDM_REQUIRE(!ls.empty(), RTDM_E_INVALID, "cfg: route without layers");
      if (ls.size() == 1) {
        const int src = resolve_ref(i, ls[0]);
        const int tt = h.layer_tensor[src];
        RTDM_REQUIRE(tt >= 0, RTDM_E_UNSUPPORTED, "cfg: route to a layer without output");
        h.layer_tensor[i] = tt;
        cur_t = tt;
        cur_c = h.tensors[tt].c;
        cur_h = h.tensors[tt].h;
        cur_w = h.tensors[tt].w;
      } else {
        if (ls.size() == 2) {
          // models.py:364-375: maps of different widths -> the narrower one is nearest-resized
          // to size (W, W) of the wider one, replacing that layer's stored output
          const int s0 = resolve_ref(i, ls[0]), s1 = resolve_ref(i, ls[1]);
          const int t0 = h.layer_tensor[s0], t1 = h.layer_tensor[s1];
          RTDM_REQUIRE(t0 >= 0 && t1 >= 0, RTDM_E_UNSUPPORTED, "cfg: route to a layer without output");
          const int w0 = h.tensors[t0].w, w1 = h.tensors[t1].w;
          if (w0 != w1) {
            const bool big0 = w0 > w1;  // max((w, num)): ties cannot happen here
            const int src = big0 ? s1 : s0, st_ = big0 ? t1 : t0, sz = big0 ? w0 : w1;
            Step rz;
            rz.kind = ST_RESIZE;
            rz.layer = i;
            rz.in_t = st_;
            rz.cin = h.tensors[st_].c;
            rz.ih = h.tensors[st_].h;
            rz.iw = h.tensors[st_].w;
            rz.oh = sz;
            rz.ow = sz;
            h.tensors[st_].materialised = true;
            rz.out_t = new_tensor(rz.cin, sz, sz, "resize" + std::to_string(src));
            h.layer_tensor[src] = rz.out_t;
            h.steps.push_back(rz);
          }
        }
        int csum = 0, hh = -1, ww = -1;
        for (int l : ls) {
          const int tt = h.layer_tensor[resolve_ref(i, l)];
          RTDM_REQUIRE(tt >= 0, RTDM_E_UNSUPPORTED, "cfg: route to a layer without output");
          if (hh < 0) {
            hh = h.tensors[tt].h;
            ww = h.tensors[tt].w;
          }
          RTDM_REQUIRE(h.tensors[tt].h == hh && h.tensors[tt].w == ww, RTDM_E_UNSUPPORTED,
                       "cfg: route of differently sized maps (reorg) unsupported");
          csum += h.tensors[tt].c;
        }
        const int ct = new_tensor(csum, hh, ww, "route" + std::to_string(i));
        h.tensors[ct].materialised = true;
        h.tensors[ct].own = true;
        // home sources inside the concat buffer where possible, else copy
        int co = 0;
        for (int l : ls) {
          const int tt = h.layer_tensor[resolve_ref(i, l)];
          Tensor& src = h.tensors[tt];
          src.materialised = true;
          if (src.home < 0 && !src.own) {
            src.home = ct;
            src.home_co = co;
          } else {
            Step s;
            s.kind = ST_COPY;
            s.layer = i;
            s.in_t = tt;
            s.out_t = ct;
            s.k = co;  // channel offset in the concat
            s.cin = src.c;
            s.ih = hh;
            s.iw = ww;
            h.steps.push_back(s);
          }
          co += src.c;
        }
        h.layer_tensor[i] = ct;
        cur_t = ct;
        cur_c = csum;
        cur_h = hh;
        cur_w = ww;
      }
    } else if (t == "shortcut") {
      // unfused weightedFeatureFusion (models.py:135-155), unweighted; channel counts may differ
      // (dc > 0: the residual is added into the first ac channels; dc < 0: only its first nc
      // channels are read), spatial shapes must agree
      RTDM_REQUIRE(!d.has("weights_type") && d.ints("from").size() == 1 && cur_t >= 0, RTDM_E_UNSUPPORTED,
                   "cfg: unsupported shortcut at layer " + std::to_string(i));
      const int rt = h.layer_tensor[resolve_ref(i, d.ints("from")[0])];
      RTDM_REQUIRE(rt >= 0 && h.tensors[rt].h == cur_h && h.tensors[rt].w == cur_w, RTDM_E_UNSUPPORTED,
                   "cfg: shortcut with spatial shape mismatch unsupported (layer " + std::to_string(i) + ")");
      Step ad;
      ad.kind = ST_ADD;
      ad.layer = i;
      ad.in_t = cur_t;
      ad.res_t = rt;
      ad.cin = cur_c;
      ad.ih = ad.oh = cur_h;
      ad.iw = ad.ow = cur_w;
      h.tensors[cur_t].materialised = true;
      h.tensors[rt].materialised = true;
      ad.out_t = new_tensor(cur_c, cur_h, cur_w, "add" + std::to_string(i));
      h.tensors[ad.out_t].materialised = true;
      h.layer_tensor[i] = ad.out_t;
      cur_t = ad.out_t;
      h.steps.push_back(ad);
    } else if (t == "yolo") {
      throw Error{RTDM_E_UNSUPPORTED, "cfg: yolo not preceded by a fusable head conv (layer " + std::to_string(i) + ")"};
    } else {
      throw Error{RTDM_E_UNSUPPORTED, "cfg: unsupported layer type [" + t + "] at layer " + std::to_string(i)};
    }
    out_c[i] = cur_c;
    out_h[i] = cur_h;
    out_w[i] = cur_w;
  }
  RTDM_REQUIRE(!h.heads.empty(), RTDM_E_UNSUPPORTED, "cfg: no [yolo] layers");
  h.nc = nc_all;
  h.no = nc_all + 5;
  h.weight_floats = wptr;
  if (weights)
    RTDM_REQUIRE(wptr == n_floats, RTDM_E_INVALID,
                 "darknet weights: stream has " + std::to_string(n_floats) + " floats, cfg needs " +
                     std::to_string(wptr));
  // ---- fused residual pairs (conv3_c32r) ----
  for (size_t i = 0; i + 1 < h.steps.size(); ++i) {
    Step& a = h.steps[i];
    const Step& b = h.steps[i + 1];
    // (64 -> 32 -> 64: conv3_c32r; 128 -> 64 -> 128: conv3_c64r)
    const bool c32 = a.cin == 64 && a.cout == 32 && b.cin == 32 && b.cout == 64;
    const bool c64 = a.cin == 128 && a.cout == 64 && b.cin == 64 && b.cout == 128;
    if (a.kind != ST_CONV || b.kind != ST_CONV || a.in_t < 0 || a.full_t < 0 || a.ks != 1 || a.stride != 1 ||
        !(c32 || c64) || a.pool_t >= 0 || a.up_t >= 0 || a.res_t >= 0 || a.yolo >= 0 || a.head ||
        a.acff || b.ks != 3 || b.stride != 1 || b.in_t != a.full_t ||
        b.res_t != a.in_t || b.pool_t >= 0 || b.up_t >= 0 || b.yolo >= 0 || b.head || b.acff)
      continue;
    bool other = h.tensors[a.full_t].home >= 0;
    for (size_t j = 0; j < h.steps.size() && !other; ++j)
      if (j != i + 1 && (h.steps[j].in_t == a.full_t || h.steps[j].res_t == a.full_t)) other = true;
    for (const Tensor& t : h.tensors)
      if (t.home == a.full_t) other = true;
    a.fuse_r = !other;
  }
  // ---- own buffers for materialised tensors that are not homed in a concat ----
  size_t off = 0;
  for (Tensor& t : h.tensors) {
    if (!t.materialised) continue;
    if (t.home >= 0) continue;
    t.own = true;
    t.off = off;
    off += (size_t)round_up((int64_t)t.c * t.h * t.w, 64);
  }
  h.per_image = off;
  // ---- pack conv weights: MFMA layout iff the input view is 16-byte aligned NHWC ----
  for (Step& st : h.steps) {
    if (st.kind == ST_DW3 && weights) {  // [27][C] taps (branch-major), [C] bias sums (launch_dw3_sum)
      const int c = st.cin;
      std::vector<float> w((size_t)27 * c), b((size_t)c, 0.f);
      for (int r = 0; r < 3; ++r) {
        const float* src = st.a_dw + (size_t)r * (c * 9 + c);  // conv{r+1}.weight [C][1][3][3], .bias [C]
        for (int ch = 0; ch < c; ++ch)
          for (int t = 0; t < 9; ++t) w[(size_t)(r * 9 + t) * c + ch] = src[(size_t)ch * 9 + t];
        for (int ch = 0; ch < c; ++ch) b[ch] += src[(size_t)c * 9 + ch];  // (b1 + b2) + b3
      }
      st.dw_w_off = blob.add_f32(w);
      st.dw_b_off = blob.add_f32(b);
      st.a_dw = nullptr;
    }
    if (st.kind != ST_CONV) continue;
    bool use_mfma = f16 && st.in_t >= 0 && st.cin % 8 == 0;
    if (use_mfma) {
      const Tensor& it = h.tensors[st.in_t];
      const int cs = it.home >= 0 ? h.tensors[it.home].c : it.c;
      const int co = it.home >= 0 ? it.home_co : 0;
      use_mfma = cs % 8 == 0 && co % 8 == 0;
    }
    const int filters = st.cout, size = st.ks;
    const bool stem = f16 && st.in_t < 0 && st.cin == 3 && size == 3 && (st.stride == 1 || st.stride == 2) && st.pad <= 1;
    // stand-alone YOLO head convs (1x1 -> 3|4 x (5 + nc), decode epilogue) whose input
    // conv_pipe takes: padded to one 128-channel N tile so they run on conv_pipe (io
    // epilogue) instead of the small-tile conv_mfma (b8 L15: 27 -> ~6 us)
    const int pad_to = use_mfma && st.yolo >= 0 && !st.head && !st.acff && filters <= 128 && st.cin % 64 == 0 &&
                               (size == 1 || size == 3)
                           ? 128
                           : 0;
    if (weights) {
      std::vector<double> sc(filters, 1.0);
      std::vector<float> b(filters);
      for (int o = 0; o < filters; ++o) {
        if (st.bn) {
          sc[o] = (double)st.w_gamma[o] / std::sqrt((double)st.w_var[o] + 1e-4);
          b[o] = (float)((double)st.w_beta[o] - (double)st.w_mean[o] * sc[o]);
        } else {
          b[o] = st.w_bias[o];
        }
      }
      st.pc = pack_conv(blob, st.acff ? st.a_W.data() : st.w_W, filters, st.cin, size, st.bn ? sc.data() : nullptr,
                        use_mfma, pad_to);
      st.pc.b_off = blob.add_f32(b);
      if (st.acff) {  // BatchNorm2d after the LeakyReLU (acff.py order), eps 1e-5
        std::vector<float> as(filters), at(filters);
        for (int o = 0; o < filters; ++o) {
          const double g = st.a_bn[o], be = st.a_bn[filters + o], mu = st.a_bn[2 * filters + o],
                       var = st.a_bn[3 * filters + o];
          const double k = g / std::sqrt(var + 1e-5);
          as[o] = (float)k;
          at[o] = (float)(be - mu * k);
        }
        st.pc.s_off = blob.add_f32(as);
        st.pc.t_off = blob.add_f32(at);
        st.a_W.clear();
        st.a_W.shrink_to_fit();
        st.a_bn = nullptr;
      }
      if (st.head) {
        std::vector<double> hsc(st.head_cout, 1.0);
        std::vector<float> hb(st.head_cout);
        for (int o = 0; o < st.head_cout; ++o) {
          if (st.head_bn) {
            hsc[o] = (double)st.h_gamma[o] / std::sqrt((double)st.h_var[o] + 1e-4);
            hb[o] = (float)((double)st.h_beta[o] - (double)st.h_mean[o] * hsc[o]);
          } else {
            hb[o] = st.h_bias[o];
          }
        }
        // [cout_pad(32)][kpad(128)] fp16, k = input channel: the head GEMM's B operand
        st.hpc = pack_conv(blob, st.h_W, st.head_cout, filters, 1, st.head_bn ? hsc.data() : nullptr, true);
        st.hpc.b_off = blob.add_f32(hb);
        RTDM_REQUIRE(st.hpc.kpad == 128 && st.hpc.cout_pad == 32, RTDM_E_INVALID, "internal: head packing");
      }
      if (stem) st.pc.stem_off = pack_stem(blob, st.w_W, filters, st.bn ? sc.data() : nullptr);
      // int8 convs: 3x3, Cin % 128, not a head conv, and not a conv whose output only a YOLO
      // head conv reads.  1x1 convs stay fp16: with the quantize pass of their input they
      // measured slower than fp16 (b16 L13 / L18 / L25: 14.2 / 12.0 / 16.4 us fp16 vs 17.0 /
      // 15.7 / 21.5 us int8, tools/det_int8_timing.py r05q).  A pre-head conv's rounding reaches
      // the logits with no layer after it to average it out: the scheme model
      // (tools/int8_scope.py, 16 frames) loses 4 % of the two-sided matches with L28 int8
      // (stride-8 head); L14 (stride 32) costs nothing there, but at b16 it is no faster in
      // int8 (r05s: 25.9 + the quantize pass vs 25.2 us), so it stays fp16 too.
      // oracle/int8.py eligible() mirrors this rule.
      const bool pre_head = consumers[st.layer].size() == 1 && consumers[st.layer][0] + 1 < L &&
                            defs[consumers[st.layer][0]].type == "convolutional" &&
                            defs[consumers[st.layer][0] + 1].type == "yolo";
      if (h.int8 && use_mfma && !st.acff && st.yolo < 0 && !st.head && !pre_head && st.cin % 128 == 0 &&
          size == 3 && st.pc.cout_pad % 128 == 0 && st.pc.kpad == size * size * st.cin) {
        // BN-folded fp32 rows [cout][k] kept for calibration; int8 slots filled there
        const int kp = st.pc.kpad, cp = st.pc.cout_pad;
        st.wf.assign((size_t)filters * kp, 0.f);
        for (int o = 0; o < filters; ++o)
          for (int c = 0; c < st.cin; ++c)
            for (int kh = 0; kh < size; ++kh)
              for (int kw = 0; kw < size; ++kw) {
                double v = st.w_W[(((size_t)o * st.cin + c) * size + kh) * size + kw];
                if (st.bn) v *= sc[o];
                st.wf[(size_t)o * kp + (size_t)(kh * size + kw) * st.cin + c] = (float)v;
              }
        st.w8_off = blob.add(nullptr, (size_t)cp * kp);
        st.deq_off = blob.add(nullptr, (size_t)cp * sizeof(float));
        st.inv_off = blob.add(nullptr, (size_t)st.cin * sizeof(float));
        st.q = h.n_q++;
        st.amax_off = h.q_channels;
        h.q_channels += st.cin;
        st.qbuf_off = h.q_bytes;
        h.q_bytes += (size_t)round_up((int64_t)st.ih * st.iw * st.cin, 256);
      }
    } else {
      st.pc.cout = filters;
      st.pc.cin = st.cin;
      st.pc.ks = size;
      st.pc.mfma = use_mfma;
      st.pc.kpad = (int)round_up((int64_t)size * size * st.cin, 64);
      st.pc.cout_pad = pad_to > 0 ? pad_to : cout_pad_for(filters);
      if (stem) st.pc.stem_off = 0;  // planning only: marks the stem kernel for step_info
    }
    st.w_beta = st.w_gamma = st.w_mean = st.w_var = st.w_bias = st.w_W = nullptr;
    st.h_beta = st.h_gamma = st.h_mean = st.h_var = st.h_bias = st.h_W = nullptr;
  }
  for (YoloHead& y : h.heads) y.anchor_off = blob.add_f32(y.anchor_vec);
  // the shared epilogues compute LeakyReLU as max(t, slope t), which is the reference's
  // t > 0 ? t : slope t only for 0 < slope <= 1 (conv_epi.h)
  for (const Step& st : h.steps)
    RTDM_REQUIRE(st.kind != ST_CONV || (st.act != ACT_LEAKY && !st.acff) || (st.slope > 0.f && st.slope <= 1.f),
                 RTDM_E_INVALID, "plan: LeakyReLU slope outside (0, 1] at layer " + std::to_string(st.layer));
  if (weights) {
    RTDM_HIP(hipGetDevice(&h.dev));
    h.blob.upload(blob);
    h.arena.alloc(h.per_image * esize_of(h.dtype) * h.max_batch);
    h.zero.alloc(256);
    RTDM_HIP(hipMemset(h.zero.p, 0, 256));
    if (h.n_q) {
      h.amax.alloc(h.q_channels * sizeof(unsigned));
      RTDM_HIP(hipMemset(h.amax.p, 0, h.q_channels * sizeof(unsigned)));
      h.qarena.alloc(h.q_bytes * h.max_batch);
    }
  }
}

// View of tensor t for a batch arena.
static View tensor_view(const rtdm_detector_s& h, int t) {
  if (t < 0) return View{};
  const Tensor& x = h.tensors[t];
  if (!x.materialised) return View{};
  const size_t es = esize_of(h.dtype);
  char* base = h.arena.as<char>();
  if (x.home >= 0) {
    const Tensor& c = h.tensors[x.home];
    return View{base + c.off * es * h.max_batch, c.c, x.home_co};
  }
  return View{base + x.off * es * h.max_batch, x.c, 0};
}

// Run-time arguments of a conv step (views of this call's buffers).
static ConvArgs run_args(rtdm_detector_s& h, const Step& st, const void* x, int in_kind, int n, float* io, int raw) {
  ConvArgs a;
  if (st.in_t < 0) {
    a.in = x;
    a.in_kind = in_kind;
  } else {
    const View v = tensor_view(h, st.in_t);
    a.in = v.ptr;
    a.in_cs = v.cs;
    a.in_co = v.co;
    a.in_kind = IN_NHWC;
  }
  a.n = n;
  a.ih = st.ih;
  a.iw = st.iw;
  a.cin = st.cin;
  a.ks = st.ks;
  a.stride = st.stride;
  a.pad = st.pad;
  a.oh = st.oh;
  a.ow = st.ow;
  a.cout = st.cout;
  a.quad = st.quad ? 1 : 0;
  conv_set_rows(a);
  a.w = h.blob.at<void>(st.pc.w_off);
  a.kpad = st.pc.kpad;
  a.cout_pad = st.pc.cout_pad;
  a.e.bias = h.blob.at<float>(st.pc.b_off);
  a.e.act = st.act;
  a.e.slope = st.slope;
  if (st.pc.s_off != SIZE_MAX) {
    a.e.scale = h.blob.at<float>(st.pc.s_off);
    a.e.shift = h.blob.at<float>(st.pc.t_off);
  }
  a.e.full = tensor_view(h, st.full_t);
  a.e.pool = tensor_view(h, st.pool_t);
  a.e.up = tensor_view(h, st.up_t);
  a.e.res = tensor_view(h, st.res_t);
  if (st.head) {
    const YoloHead& y = h.heads[st.yolo];
    a.head_w = h.blob.at<void>(st.hpc.w_off);
    a.head_cout = st.head_cout;
    a.head_e.bias = h.blob.at<float>(st.hpc.b_off);
    a.head_e.act = st.head_act;
    a.head_e.slope = 0.1f;
    a.head_e.io = io;
    a.head_e.io_rows = h.n_anchors_total;
    a.head_e.io_off = y.io_off;
    a.head_e.na = y.na;
    a.head_e.no = y.no;
    a.head_e.ystride = y.ystride;
    a.head_e.anchor_vec = h.blob.at<float>(y.anchor_off);
    a.head_e.raw = raw;
  } else if (st.yolo >= 0) {
    const YoloHead& y = h.heads[st.yolo];
    a.e.io = io;
    a.e.io_rows = h.n_anchors_total;
    a.e.io_off = y.io_off;
    a.e.na = y.na;
    a.e.no = y.no;
    a.e.ystride = y.ystride;
    a.e.anchor_vec = h.blob.at<float>(y.anchor_off);
    a.e.raw = raw;
  }
  // the mfma/valu choice was fixed when the weights were packed
  a.w_f32 = st.pc.mfma ? 0 : 1;
  a.w_stem = h.blob.at<void>(st.pc.stem_off);
  a.zero = h.zero.p;
  return a;
}

static void run_detector(rtdm_detector_s& h, const void* x, int x_kind, int n, float* io, hipStream_t s,
                         int raw = 0) {
  RTDM_REQUIRE(!h.planning_only, RTDM_E_INVALID, "detect: handle was created without weights");
  RTDM_REQUIRE(!h.int8 || h.calibrated || h.calibrating != 0 || h.n_q == 0, RTDM_E_INVALID,
               "detect: int8 detector not calibrated (rtdm_detector_calibrate)");
  RTDM_REQUIRE(n >= 0 && n <= h.max_batch, RTDM_E_CAPACITY,
               "detect: batch " + std::to_string(n) + " exceeds max_batch " + std::to_string(h.max_batch));
  if (n == 0) return;
  RTDM_REQUIRE(x && io, RTDM_E_INVALID, "detect: NULL input or io");
  int in_kind;
  if (x_kind == RTDM_INPUT_FRAME_U8)
    in_kind = IN_FRAME_U8;
  else if (x_kind == RTDM_INPUT_NCHW_F32)
    in_kind = IN_NCHW_F32;
  else if (x_kind == RTDM_INPUT_NCHW_F16)
    in_kind = IN_NCHW_F16;
  else
    throw Error{RTDM_E_INVALID, "detect: unknown input kind"};
  hipEvent_t* ev = nullptr;
  if (h.timing && h.timing_calls < h.timing_cap) {
    ev = &h.events[(size_t)h.timing_calls * 2 * h.steps.size()];
    ++h.timing_calls;
  }
  const bool two = h.two_streams && h.side;
  if (two) {  // the side stream starts after everything already queued on s (input, previous call)
    RTDM_HIP(hipEventRecord(h.fork_ev, s));
    RTDM_HIP(hipStreamWaitEvent(h.side, h.fork_ev, 0));
  }
  hipStream_t s0 = s;
  bool fused_next = false;
  h.fused_away.clear();
  for (size_t si = 0; si < h.steps.size(); ++si) {
    const Step& st = h.steps[si];
    s = two && st.stream == 1 ? h.side : s0;
    if (two)
      for (int d : st.deps)
        if (h.steps[d].stream != st.stream) RTDM_HIP(hipStreamWaitEvent(s, h.step_ev[d], 0));
    if (ev) RTDM_HIP(hipEventRecord(ev[2 * si], s));
    if (fused_next) {  // this step ran inside the previous step's launch (conv3_c32r)
      fused_next = false;
    } else if (st.kind == ST_CONV) {
      ConvArgs a = run_args(h, st, x, in_kind, n, io, raw);
      if (st.fuse_r && tune().res_fuse && st.q < 0 && h.steps[si + 1].q < 0) {
        const Step& nx = h.steps[si + 1];
        const ConvArgs b = run_args(h, nx, x, in_kind, n, io, raw);
        const bool r32 = c32r_ok(a, b), r64 = !r32 && c64r_ok(a, b);
        if ((!two || nx.stream == st.stream) && (r32 || r64)) {
          if (two)
            for (int d : nx.deps)
              if (h.steps[d].stream != nx.stream) RTDM_HIP(hipStreamWaitEvent(s, h.step_ev[d], 0));
          if (r32)
            launch_c32r(a, b, s);
          else
            launch_c64r(a, b, s);
          fused_next = true;
          h.fused_away.push_back(st.full_t);
        }
      }
      if (fused_next) {
      } else if (st.q >= 0 && h.calibrating) {
        launch_chan_absmax(tensor_view(h, st.in_t), n, st.ih, st.iw, st.cin, h.amax.as<unsigned>() + st.amax_off, s);
        launch_conv(a, h.dtype, s);
      } else if (st.q >= 0) {
        int8_t* qb = h.qarena.as<int8_t>() + st.qbuf_off * h.max_batch;
        launch_quantize(tensor_view(h, st.in_t), n, st.ih, st.iw, st.cin, h.blob.at<float>(st.inv_off), qb, s);
        a.in = qb;
        a.in_cs = st.cin;
        a.in_co = 0;
        a.w8 = h.blob.at<void>(st.w8_off);
        a.deq = h.blob.at<float>(st.deq_off);
        launch_conv_pipe_i8(a, s);
      } else {
        launch_conv(a, h.dtype, s);
      }
    } else if (st.kind == ST_MAXPOOL) {
      launch_maxpool(nullptr, tensor_view(h, st.in_t), n, st.ih, st.iw, st.cin, st.k, st.s, st.p, st.zero_rb,
                     tensor_view(h, st.out_t), st.oh, st.ow, h.dtype, s);
    } else if (st.kind == ST_UPSAMPLE) {
      launch_upsample(tensor_view(h, st.in_t), n, st.ih, st.iw, st.cin, st.f, tensor_view(h, st.out_t), h.dtype, s);
    } else if (st.kind == ST_COPY) {
      View o = tensor_view(h, st.out_t);
      o.co += st.k;
      launch_copy_slice(tensor_view(h, st.in_t), n, st.ih, st.iw, st.cin, o, h.dtype, s);
    } else if (st.kind == ST_DW3) {
      const View iv = tensor_view(h, st.in_t), ov = tensor_view(h, st.out_t);
      RTDM_REQUIRE(ov.cs == st.cin && ov.co == 0, RTDM_E_INVALID, "internal: acff branch map view");
      launch_dw3_sum(iv.ptr, iv.cs, iv.co, n, st.ih, st.iw, st.cin, h.blob.at<float>(st.dw_w_off),
                     h.blob.at<float>(st.dw_b_off), ov.ptr, h.dtype, s);
    } else if (st.kind == ST_ADD) {
      launch_add(tensor_view(h, st.in_t), tensor_view(h, st.res_t), n, st.ih, st.iw, st.cin,
                 std::min(st.cin, h.tensors[st.res_t].c), tensor_view(h, st.out_t), h.dtype, s);
    } else if (st.kind == ST_RESIZE) {
      launch_resize_nearest(tensor_view(h, st.in_t), n, st.ih, st.iw, st.cin, tensor_view(h, st.out_t), st.oh, st.ow,
                            h.dtype, s);
    }
    if (ev) RTDM_HIP(hipEventRecord(ev[2 * si + 1], s));
    if (two && st.signal) RTDM_HIP(hipEventRecord(h.step_ev[si], s));
  }
  if (two) {  // everything on the side stream finishes before later work on the caller's stream
    RTDM_HIP(hipEventRecord(h.join_ev, h.side));
    RTDM_HIP(hipStreamWaitEvent(s0, h.join_ev, 0));
  }
  h.last_n = n;
}

// Geometry of tensor t's view (pointer is a non-null placeholder) for kernel selection.
static View view_geom(const rtdm_detector_s& h, int t) {
  if (t < 0 || !h.tensors[t].materialised) return View{};
  const Tensor& x = h.tensors[t];
  if (x.home >= 0) return View{(void*)64, h.tensors[x.home].c, x.home_co};
  return View{(void*)64, x.c, 0};
}

// Kernel symbol, FLOPs and compulsory HBM bytes per image of one step.
// Geometry-only arguments of a conv step (placeholder pointers) for kernel selection.
static ConvArgs geom_args(const rtdm_detector_s& h, const Step& st) {
  ConvArgs a;
  a.in_kind = st.in_t < 0 ? IN_FRAME_U8 : IN_NHWC;
  a.cout_pad = st.pc.cout_pad;
  a.w_f32 = st.pc.mfma ? 0 : 1;
  a.cin = st.cin;
  a.ks = st.ks;
  a.stride = st.stride;
  a.pad = st.pad;
  a.ih = st.ih;
  a.iw = st.iw;
  a.oh = st.oh;
  a.ow = st.ow;
  a.quad = st.quad ? 1 : 0;
  a.w_stem = st.pc.stem_off != SIZE_MAX ? (const void*)1 : nullptr;
  a.zero = (const void*)64;
  a.kpad = st.pc.kpad;
  a.cout = st.cout;
  // the kernel instance depends on the batch (conv_pipe tile rows): the last
  // rtdm_detect call's, max_batch before any
  a.n = h.last_n > 0 ? h.last_n : h.max_batch;
  conv_set_rows(a);
  a.e.bias = (const float*)64;
  a.e.act = st.act;
  a.e.slope = st.slope;  // kernel choice depends on it (pool_small_ok)
  if (st.pc.s_off != SIZE_MAX) {
    a.e.scale = (const float*)64;
    a.e.shift = (const float*)64;
  }
  if (st.in_t >= 0) {
    const View iv = view_geom(h, st.in_t);
    a.in = iv.ptr;  // (the placeholder every view carries: c32r_ok compares views)
    a.in_cs = iv.cs;
    a.in_co = iv.co;
  }
  a.e.full = view_geom(h, st.full_t);
  a.e.pool = view_geom(h, st.pool_t);
  a.e.up = view_geom(h, st.up_t);
  a.e.res = view_geom(h, st.res_t);
  if (st.head) {
    a.head_w = (const void*)64;
    a.head_cout = st.head_cout;
    a.head_e.io = (float*)64;
    a.head_e.bias = (const float*)64;
  } else if (st.yolo >= 0) {
    a.e.io = (float*)64;
    a.e.no = h.heads[st.yolo].no;
  }
  if (st.pc.mfma) a.w = (const void*)64;
  if (st.q >= 0) {
    a.in_cs = st.cin;
    a.in_co = 0;
    a.w8 = (const void*)64;
    a.deq = (const float*)64;
  }
  return a;
}

static void step_info(const rtdm_detector_s& h, const Step& st, std::string& name, double& flop, double& bytes) {
  const double es = (double)esize_of(h.dtype);
  if (st.kind == ST_CONV) {
    const ConvArgs a = geom_args(h, st);
    name = st.q >= 0 ? conv_pipe_i8_name(a) : conv_kernel_name(a, h.dtype);
    flop = 2.0 * st.oh * st.ow * (double)st.cout * st.cin * st.ks * st.ks +
           (st.head ? 2.0 * st.oh * st.ow * (double)st.head_cout * st.cout : 0.0);
    double out = 0;
    if (st.full_t >= 0) out += (double)st.oh * st.ow * st.cout;
    if (st.pool_t >= 0) out += (double)(st.oh / 2) * (st.ow / 2) * st.cout;
    if (st.up_t >= 0) out += 4.0 * st.oh * st.ow * st.cout;
    if (st.res_t >= 0) out += (double)st.oh * st.ow * st.cout;
    const double in = (double)st.ih * st.iw * st.cin * (st.in_t < 0 ? 1.0 / es : 1.0);
    bytes = (in + out) * es + (st.yolo >= 0 ? (double)st.oh * st.ow * (st.head ? st.head_cout : st.cout) * 4.0 : 0.0);
  } else if (st.kind == ST_MAXPOOL) {
    name = "maxpool_kernel";
    flop = 0;
    bytes = ((double)st.ih * st.iw + (double)st.oh * st.ow) * st.cin * es;
  } else if (st.kind == ST_DW3) {
    const View iv = view_geom(h, st.in_t);
    const bool vec = dw3_sum_vec_ok(st.cin, iv.cs, iv.co, h.dtype);
    name = dw3_sum_tile_ok(st.cin, iv.cs, iv.co, h.dtype) ? "dw3_sum_tile_kernel" : vec ? (h.dtype == RTDM_F16 ? "dw3_sum_kernel<_Float16,8>" : "dw3_sum_kernel<float,4>")
               : (h.dtype == RTDM_F16 ? "dw3_sum_kernel<_Float16,1>" : "dw3_sum_kernel<float,1>");
    flop = 2.0 * st.oh * st.ow * 3.0 * st.cin * 9;
    bytes = ((double)st.ih * st.iw + (double)st.oh * st.ow) * st.cin * es;
  } else if (st.kind == ST_ADD) {
    name = "add_kernel";
    flop = 0;
    bytes = 3.0 * st.ih * st.iw * st.cin * es;
  } else if (st.kind == ST_RESIZE) {
    name = "resize_nearest_kernel";
    flop = 0;
    bytes = ((double)st.ih * st.iw + (double)st.oh * st.ow) * st.cin * es;
  } else {
    name = "upsample_kernel";
    flop = 0;
    bytes = ((double)st.ih * st.iw + (double)st.oh * st.ow) * st.cin * es;
  }
}

// Two-stream schedule of the step list.  Dependencies come from the buffers each
// step reads and writes (a route concat is one buffer written by several
// producers).  A step's primary producer is its latest dependency; among the
// steps sharing a primary producer, the one with the longest remaining path
// (FLOP + 312 FLOP per HBM byte ~ time at the chip's peaks) stays on the
// producer's stream and the others run on the other stream — in the YOLO
// graphs these are the detection-head branches, which then overlap the trunk.
int two_streams_mode() { return tune().two_streams; }

static void schedule_streams(rtdm_detector_s& h) {
  const int ns = (int)h.steps.size();
  auto buf_of = [&](int t) { return t < 0 ? -1 : (h.tensors[t].home >= 0 ? h.tensors[t].home : t); };
  std::vector<std::vector<int>> reads(ns), writes(ns);
  std::vector<double> cost(ns, 0.0);
  for (int i = 0; i < ns; ++i) {
    const Step& st = h.steps[i];
    auto rd = [&](int t) {
      if (buf_of(t) >= 0) reads[i].push_back(buf_of(t));
    };
    auto wr = [&](int t) {
      if (t >= 0 && h.tensors[t].materialised) writes[i].push_back(buf_of(t));
    };
    rd(st.in_t);
    if (st.kind == ST_ADD) rd(st.res_t);
    if (st.kind == ST_CONV) {
      rd(st.res_t);
      wr(st.full_t);
      wr(st.pool_t);
      wr(st.up_t);
    } else {
      wr(st.out_t);
    }
    std::string name;
    double f = 0, b = 0;
    step_info(h, st, name, f, b);
    cost[i] = f + 312.0 * b;
  }
  for (int i = 0; i < ns; ++i) {
    Step& st = h.steps[i];
    st.deps.clear();
    for (int j = 0; j < i; ++j) {
      bool dep = false;
      for (int rb : reads[i])
        for (int wb : writes[j]) dep = dep || rb == wb;
      if (dep) st.deps.push_back(j);
    }
  }
  std::vector<double> lp(ns, 0.0);  // longest path from step i to the end
  for (int i = ns - 1; i >= 0; --i) {
    double m = 0.0;
    for (int j = i + 1; j < ns; ++j)
      for (int d : h.steps[j].deps)
        if (d == i) m = std::max(m, lp[j]);
    lp[i] = cost[i] + m;
  }
  for (int i = 0; i < ns; ++i) {
    Step& st = h.steps[i];
    st.stream = 0;
    st.signal = false;
    if (st.deps.empty()) continue;
    const int p = st.deps.back();
    // the heaviest child of p keeps p's stream
    int best = -1;
    for (int j = p + 1; j < ns; ++j)
      if (!h.steps[j].deps.empty() && h.steps[j].deps.back() == p && (best < 0 || lp[j] > lp[best])) best = j;
    st.stream = best == i ? h.steps[p].stream : 1 - h.steps[p].stream;
  }
  bool any_side = false;
  for (int i = 0; i < ns; ++i) {
    any_side = any_side || h.steps[i].stream == 1;
    for (int d : h.steps[i].deps)
      if (h.steps[d].stream != h.steps[i].stream) h.steps[d].signal = true;
  }
  h.two_streams = any_side && two_streams_mode();
  if (h.two_streams && !h.planning_only) {
    RTDM_HIP(hipStreamCreateWithFlags(&h.side, hipStreamNonBlocking));
    h.step_ev.assign(ns, nullptr);
    for (int i = 0; i < ns; ++i)
      if (h.steps[i].signal) RTDM_HIP(hipEventCreateWithFlags(&h.step_ev[i], hipEventDisableTiming));
    RTDM_HIP(hipEventCreateWithFlags(&h.fork_ev, hipEventDisableTiming));
    RTDM_HIP(hipEventCreateWithFlags(&h.join_ev, hipEventDisableTiming));
  }
}

static std::string describe(const rtdm_detector_s& h) {
  std::ostringstream o;
  o << "darknet plan: img " << h.img_h << "x" << h.img_w << " dtype " << (h.int8 ? "i8" : h.dtype == RTDM_F16 ? "f16" : "f32")
    << " layers " << h.defs.size() << " steps " << h.steps.size() << " anchors " << h.n_anchors_total << " no " << h.no
    << " GFLOP/img " << h.flop * 1e-9 << " arena/img " << h.per_image << " elems\n";
  auto tn = [&](int t) -> std::string {
    if (t < 0) return "-";
    const Tensor& x = h.tensors[t];
    std::ostringstream s;
    s << x.what << "[" << x.c << "x" << x.h << "x" << x.w;
    if (x.home >= 0) s << " @" << h.tensors[x.home].what << "+" << x.home_co;
    s << "]";
    return s.str();
  };
  for (const Step& st : h.steps) {
    o << "  L" << st.layer << " ";
    if (st.kind == ST_CONV) {
      o << "conv" << st.ks << "x" << st.ks << "/" << st.stride << " " << st.cin << "->" << st.cout << " "
        << (st.pc.mfma ? "mfma" : "valu") << (st.quad ? " quad" : "") << " in=" << (st.in_t < 0 ? "input" : tn(st.in_t))
        << " full=" << tn(st.full_t) << " pool=" << tn(st.pool_t) << " up=" << tn(st.up_t) << " res=" << tn(st.res_t);
      if (st.head) o << " head1x1->" << st.head_cout;
      if (h.two_streams && st.stream == 1) o << " [side stream]";
      if (st.yolo >= 0) o << " yolo" << st.yolo << "(off " << h.heads[st.yolo].io_off << ")";
    } else if (st.kind == ST_MAXPOOL) {
      o << "maxpool k" << st.k << " s" << st.s << (st.zero_rb ? " zeropad" : "") << " " << tn(st.in_t) << " -> "
        << tn(st.out_t);
    } else if (st.kind == ST_UPSAMPLE) {
      o << "upsample x" << st.f << " " << tn(st.in_t) << " -> " << tn(st.out_t);
    } else if (st.kind == ST_DW3) {
      o << "acff dw3x3 d1/d2/d3 " << tn(st.in_t) << " -> " << tn(st.out_t);
    } else if (st.kind == ST_ADD) {
      o << "shortcut add " << tn(st.in_t) << " + " << tn(st.res_t) << " -> " << tn(st.out_t);
    } else if (st.kind == ST_RESIZE) {
      o << "resize nearest " << tn(st.in_t) << " -> " << tn(st.out_t);
    } else {
      o << "copy " << tn(st.in_t) << " -> " << tn(st.out_t) << "+" << st.k;
    }
    o << "\n";
  }
  return o.str();
}

}  // namespace rtdm

using namespace rtdm;

extern "C" {

rtdm_status rtdm_detector_create(const char* cfg_text, int img_h, int img_w, int dtype, const float* weights,
                                 int64_t n_floats, int max_batch, rtdm_detector* out) {
  return guard([&] {
    RTDM_REQUIRE(out, RTDM_E_INVALID, "detector_create: NULL out");
    *out = nullptr;
    RTDM_REQUIRE(cfg_text, RTDM_E_INVALID, "detector_create: NULL cfg");
    RTDM_REQUIRE(img_h > 0 && img_w > 0, RTDM_E_INVALID, "detector_create: bad image size");
    RTDM_REQUIRE(dtype == RTDM_F32 || dtype == RTDM_F16 || dtype == RTDM_I8, RTDM_E_INVALID,
                 "detector_create: bad dtype");
    RTDM_REQUIRE(max_batch > 0, RTDM_E_INVALID, "detector_create: max_batch must be > 0");
    auto h = std::make_unique<rtdm_detector_s>();
    h->tuning = default_tuning();
    TuningScope ts_(&h->tuning);  // the plan (fused heads, streams) follows this handle's knobs
    h->img_h = img_h;
    h->img_w = img_w;
    h->int8 = dtype == RTDM_I8;
    h->dtype = h->int8 ? RTDM_F16 : dtype;  // int8 handles keep fp16 activations
    h->max_batch = max_batch;
    h->planning_only = weights == nullptr;
    std::vector<CfgBlock> defs = parse_cfg(cfg_text);
    const CfgBlock& net = defs[0];
    RTDM_REQUIRE(net.i("channels", 3) == 3, RTDM_E_UNSUPPORTED, "cfg: only 3-channel input supported");
    h->defs.assign(defs.begin() + 1, defs.end());
    plan(*h, weights, n_floats);
    schedule_streams(*h);
    *out = h.release();
  });
}

rtdm_status rtdm_detector_set_tuning(rtdm_detector h, const char* key, int value) {
  return guard([&] {
    RTDM_REQUIRE(h, RTDM_E_INVALID, "detector_set_tuning: NULL handle");
    RTDM_REQUIRE(key && !tuning_is_plan_time(key), RTDM_E_INVALID,
                 std::string("detector_set_tuning: ") + (key ? key : "(null)") +
                     " is a plan-time key (set it with rtdm_set_tuning before rtdm_detector_create)");
    tuning_set(h->tuning, key, value);
  });
}

rtdm_status rtdm_detector_destroy(rtdm_detector h) {
  return guard([&] { delete h; });
}

rtdm_status rtdm_detector_get_info(rtdm_detector h, rtdm_detector_info* info) {
  return guard([&] {
    TuningScope ts_(h ? &h->tuning : nullptr);
    RTDM_REQUIRE(h && info, RTDM_E_INVALID, "detector_get_info: NULL argument");
    info->img_h = h->img_h;
    info->img_w = h->img_w;
    info->n_layers = (int)h->defs.size();
    info->n_yolo = (int)h->heads.size();
    info->n_anchors_total = h->n_anchors_total;
    info->no = h->no;
    info->nc = h->nc;
    info->weight_floats = h->weight_floats;
    info->device_bytes = (int64_t)(h->blob.buf.bytes + h->arena.bytes);
    info->flop_per_image = h->flop;
  });
}

int64_t rtdm_detector_describe(rtdm_detector h, char* buf, int64_t buf_len) {
  if (!h) return 0;
  TuningScope ts_(&h->tuning);
  const std::string s = describe(*h);
  const int64_t need = (int64_t)s.size() + 1;
  if (buf && buf_len >= need) std::memcpy(buf, s.c_str(), need);
  return need;
}

int rtdm_detector_num_steps(rtdm_detector h) { return h ? (int)h->steps.size() : 0; }

rtdm_status rtdm_detector_step_info(rtdm_detector h, int step, char* name, int name_len, int* layer,
                                    double* flop_per_image, double* bytes_per_image) {
  return guard([&] {
    TuningScope ts_(h ? &h->tuning : nullptr);
    RTDM_REQUIRE(h && step >= 0 && step < (int)h->steps.size(), RTDM_E_INVALID, "step_info: bad step");
    std::string nm;
    double f = 0, b = 0;
    step_info(*h, h->steps[step], nm, f, b);
    // a fused residual pair (run_detector's conv3_c32r / conv3_c64r choice): the first step
    // reports the launch (both layers' FLOPs), the second an empty step
    const auto res_pair = [&](int i) -> int {  // 0: no, 32: conv3_c32r, 64: conv3_c64r
      if (i < 0 || i + 1 >= (int)h->steps.size()) return 0;
      const Step& a = h->steps[i];
      const Step& c = h->steps[i + 1];
      if (!(a.fuse_r && tune().res_fuse && a.q < 0 && c.q < 0 && (!(h->two_streams && h->side) || c.stream == a.stream)))
        return 0;
      const ConvArgs ga = geom_args(*h, a), gc = geom_args(*h, c);
      return c32r_ok(ga, gc) ? 32 : c64r_ok(ga, gc) ? 64 : 0;
    };
    if (const int rp = res_pair(step)) {
      const Step& a = h->steps[step];
      const Step& c = h->steps[step + 1];
      std::string n2;
      double f2 = 0, b2 = 0;
      step_info(*h, c, n2, f2, b2);
      nm = rp == 32 ? "conv3_c32r" : "conv3_c64r";
      f += f2;
      b = ((double)a.ih * a.iw * a.cin + (double)c.oh * c.ow * c.cout) * (double)esize_of(h->dtype);
    } else if (const int rq = res_pair(step - 1)) {
      nm = rq == 32 ? "conv3_c32r:fused" : "conv3_c64r:fused";
      f = 0;
      b = 0;
    }
    if (name && name_len > 0) {
      std::strncpy(name, nm.c_str(), name_len - 1);
      name[name_len - 1] = 0;
    }
    if (layer) *layer = h->steps[step].layer;
    if (flop_per_image) *flop_per_image = f;
    if (bytes_per_image) *bytes_per_image = b;
  });
}

rtdm_status rtdm_detector_enable_timing(rtdm_detector h, int max_calls) {
  return guard([&] {
    TuningScope ts_(h ? &h->tuning : nullptr);
    RTDM_REQUIRE(h && !h->planning_only, RTDM_E_INVALID, "enable_timing: bad handle");
    for (hipEvent_t e : h->events) (void)hipEventDestroy(e);
    h->events.clear();
    h->timing = max_calls > 0;
    h->timing_cap = max_calls > 0 ? max_calls : 0;
    h->timing_calls = 0;
    const size_t ne = (size_t)h->timing_cap * 2 * h->steps.size();
    h->events.resize(ne);
    for (size_t i = 0; i < ne; ++i) RTDM_HIP(hipEventCreateWithFlags(&h->events[i], hipEventDisableSystemFence));
  });
}

rtdm_status rtdm_detector_read_timing(rtdm_detector h, double* ms_per_step, int* calls) {
  return guard([&] {
    TuningScope ts_(h ? &h->tuning : nullptr);
    RTDM_REQUIRE(h, RTDM_E_INVALID, "read_timing: NULL handle");
    const size_t ns = h->steps.size();
    for (size_t i = 0; i < ns; ++i) ms_per_step[i] = 0.0;
    for (int c = 0; c < h->timing_calls; ++c) {
      hipEvent_t* ev = &h->events[(size_t)c * 2 * ns];
      for (size_t i = 0; i < ns; ++i) {
        float ms = 0.f;
        RTDM_HIP(hipEventSynchronize(ev[2 * i + 1]));
        RTDM_HIP(hipEventElapsedTime(&ms, ev[2 * i], ev[2 * i + 1]));
        ms_per_step[i] += ms;
      }
    }
    if (calls) *calls = h->timing_calls;
  });
}

rtdm_status rtdm_detect(rtdm_detector h, const void* x, int x_kind, int n, float* io, void* stream) {
  return guard([&] {
    TuningScope ts_(h ? &h->tuning : nullptr);
    RTDM_REQUIRE(h, RTDM_E_INVALID, "detect: NULL handle");
    run_detector(*h, x, x_kind, n, io, (hipStream_t)stream);
  });
}

rtdm_status rtdm_detector_calibrate(rtdm_detector h, const void* x, int x_kind, int n, int reset, void* stream) {
  return guard([&] {
    TuningScope ts_(h ? &h->tuning : nullptr);
    RTDM_REQUIRE(h, RTDM_E_INVALID, "calibrate: NULL handle");
    RTDM_REQUIRE(h->int8, RTDM_E_INVALID, "calibrate: handle is not RTDM_I8");
    if (h->n_q == 0) {
      h->calibrated = true;
      return;
    }
    const hipStream_t s = (hipStream_t)stream;
    if (reset) RTDM_HIP(hipMemsetAsync(h->amax.p, 0, h->q_channels * sizeof(unsigned), s));
    if (n > 0) {
      const size_t need = (size_t)h->max_batch * h->n_anchors_total * h->no * sizeof(float);
      if (h->raw_buf.bytes < need) h->raw_buf.alloc(need);
      h->calibrating = 1;  // fp16 forward, per-channel |x|max of every int8 conv's input
      try {
        run_detector(*h, x, x_kind, n, h->raw_buf.as<float>(), s);
      } catch (...) {
        h->calibrating = 0;
        throw;
      }
      h->calibrating = 0;
    }
    // per int8 conv: s_c = kI8Headroom * |x|max_c / 127 per input channel (headroom: frames
    // past the calibration set's extremes round instead of clamping -- clamped peaks are
    // the activations detections come from), folded into the weights
    // (W'[o][k] = W[o][k] * s_c(k)); symmetric per-output-channel int8 of W':
    // s_w[o] = max_k |W'[o][k]| / 127, W8 = rint(W' / s_w[o]); deq[o] = s_w[o]
    std::vector<unsigned> am(h->q_channels);
    RTDM_HIP(hipMemcpyAsync(am.data(), h->amax.p, am.size() * sizeof(unsigned), hipMemcpyDeviceToHost, s));
    RTDM_HIP(hipStreamSynchronize(s));
    for (Step& st : h->steps) {
      if (st.q < 0) continue;
      const int cin = st.cin, kp = st.pc.kpad, cp = st.pc.cout_pad, cout = st.cout;
      std::vector<float> sx(cin), inv(cin);
      for (int c = 0; c < cin; ++c) {
        float mx;
        std::memcpy(&mx, &am[st.amax_off + c], sizeof(float));
        RTDM_REQUIRE(std::isfinite(mx), RTDM_E_INVALID, "calibrate: non-finite activations");
        sx[c] = mx > 0.f ? mx * kI8Headroom / 127.f : 1.f;
        inv[c] = 1.f / sx[c];
      }
      std::vector<int8_t> w8((size_t)cp * kp, 0);
      std::vector<float> dq(cp, 0.f);
      for (int o = 0; o < cout; ++o) {
        const float* row = &st.wf[(size_t)o * kp];
        double mx = 0.0;
        for (int k = 0; k < kp; ++k) mx = std::max(mx, std::fabs((double)row[k] * sx[k % cin]));
        const double sw = mx > 0.0 ? mx / 127.0 : 1.0;
        dq[o] = (float)sw;
        for (int k = 0; k < kp; ++k) {
          const long q = std::lround((double)row[k] * sx[k % cin] / sw);
          w8[(size_t)o * kp + k] = (int8_t)std::max(-127L, std::min(127L, q));
        }
      }
      RTDM_HIP(hipMemcpy(h->blob.at<void>(st.w8_off), w8.data(), w8.size(), hipMemcpyHostToDevice));
      RTDM_HIP(hipMemcpy(h->blob.at<void>(st.deq_off), dq.data(), dq.size() * sizeof(float), hipMemcpyHostToDevice));
      RTDM_HIP(hipMemcpy(h->blob.at<void>(st.inv_off), inv.data(), inv.size() * sizeof(float), hipMemcpyHostToDevice));
    }
    h->calibrated = true;
  });
}

rtdm_status rtdm_detect_raw(rtdm_detector h, const void* x, int x_kind, int n, float* p, void* stream) {
  return guard([&] {
    TuningScope ts_(h ? &h->tuning : nullptr);
    RTDM_REQUIRE(h, RTDM_E_INVALID, "detect_raw: NULL handle");
    run_detector(*h, x, x_kind, n, p, (hipStream_t)stream, 1);
  });
}

rtdm_status rtdm_detect_trt(rtdm_detector h, const void* x, int x_kind, int n, float* dets, void* stream) {
  return guard([&] {
    TuningScope ts_(h ? &h->tuning : nullptr);
    RTDM_REQUIRE(h, RTDM_E_INVALID, "detect_trt: NULL handle");
    RTDM_REQUIRE(!h->planning_only, RTDM_E_INVALID, "detect_trt: handle was created without weights");
    RTDM_REQUIRE(n >= 0 && n <= h->max_batch, RTDM_E_CAPACITY, "detect_trt: batch exceeds max_batch");
    if (n == 0) return;
    RTDM_REQUIRE(dets, RTDM_E_INVALID, "detect_trt: NULL dets");
    RTDM_REQUIRE((int)h->heads.size() <= kTrtMaxHeads, RTDM_E_UNSUPPORTED, "detect_trt: too many [yolo] heads");
    TrtYoloArgs t;
    t.n_heads = (int)h->heads.size();
    t.rows = h->n_anchors_total;
    t.no = h->no;
    t.nc = h->nc;
    for (int k = 0; k < t.n_heads; ++k) {
      const YoloHead& y = h->heads[k];
      RTDM_REQUIRE(y.na <= kTrtMaxAnchors, RTDM_E_UNSUPPORTED,
                   "detect_trt: more than 6 anchors per head (yolo_layer.h MAX_ANCHORS)");
      TrtYoloHead& d = t.h[k];
      d.row0 = y.io_off;
      d.na = y.na;
      d.ny = y.ny;
      d.nx = y.nx;
      // the engine's input size is yolo_width * inputMultiplier (yolo_layer.cu:416)
      d.in_w = y.nx * (h->img_w / y.nx);
      d.in_h = y.ny * (h->img_h / y.ny);
      d.scale_xy = y.scale_xy;
      d.new_coords = y.new_coords;
      for (int j = 0; j < 2 * y.na; ++j) d.anchors[j] = y.anchor_px[j];
    }
    const size_t need = (size_t)h->max_batch * h->n_anchors_total * h->no * sizeof(float);
    if (h->raw_buf.bytes < need) h->raw_buf.alloc(need);
    run_detector(*h, x, x_kind, n, h->raw_buf.as<float>(), (hipStream_t)stream, 1);
    launch_yolo_trt(h->raw_buf.as<float>(), n, t, 0, dets, (hipStream_t)stream);
  });
}

rtdm_status rtdm_detector_layer_output(rtdm_detector h, int layer, int n, float* out, int64_t out_numel, int* c,
                                       int* hgt, int* wid, void* stream) {
  return guard([&] {
    TuningScope ts_(h ? &h->tuning : nullptr);
    RTDM_REQUIRE(h, RTDM_E_INVALID, "layer_output: NULL handle");
    RTDM_REQUIRE(layer >= 0 && layer < (int)h->defs.size(), RTDM_E_INVALID, "layer_output: bad layer");
    const int t = h->layer_tensor[layer];
    RTDM_REQUIRE(t >= 0 && h->tensors[t].materialised, RTDM_E_UNSUPPORTED,
                 "layer_output: layer " + std::to_string(layer) + " output is fused away (not materialised)");
    const Tensor& x = h->tensors[t];
    if (c) *c = x.c;
    if (hgt) *hgt = x.h;
    if (wid) *wid = x.w;
    if (!out) return;
    RTDM_REQUIRE(std::find(h->fused_away.begin(), h->fused_away.end(), t) == h->fused_away.end(), RTDM_E_UNSUPPORTED,
                 "layer_output: layer " + std::to_string(layer) +
                     " output was fused away in the last detect (conv3_c32r / conv3_c64r; rtdm_detector_set_tuning res_fuse 0 keeps it)");
    RTDM_REQUIRE(n > 0 && n <= h->last_n, RTDM_E_INVALID, "layer_output: n exceeds the last detect batch");
    RTDM_REQUIRE(out_numel >= (int64_t)n * x.c * x.h * x.w, RTDM_E_CAPACITY, "layer_output: out too small");
    launch_to_nchw_f32(tensor_view(*h, t), n, x.h, x.w, x.c, out, h->dtype, (hipStream_t)stream);
  });
}

}  // extern "C"
