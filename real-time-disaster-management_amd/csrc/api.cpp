// Library-level C ABI: errors, version, stand-alone decode / NMS / preprocess.
#include <algorithm>
#include <array>
#include <cmath>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>

#include "common.h"

namespace rtdm {

static thread_local std::string g_last_error;

void set_error(const std::string& msg) { g_last_error = msg; }
const char* get_error() { return g_last_error.c_str(); }

}  // namespace rtdm

using namespace rtdm;

namespace rtdm {

Tuning& default_tuning() {
  static Tuning t = [] {
    Tuning d;
    if (const char* e = getenv("RTDM_CONV_PIPE")) d.conv_pipe = atoi(e);  // A/B runs
    return d;
  }();
  return t;
}
static thread_local const Tuning* t_tuning = nullptr;
const Tuning& tune() { return t_tuning ? *t_tuning : default_tuning(); }
TuningScope::TuningScope(const Tuning* t) : prev(t_tuning) { t_tuning = t; }
TuningScope::~TuningScope() { t_tuning = prev; }

void tuning_set(Tuning& t, const char* key, int v) {
  RTDM_REQUIRE(key, RTDM_E_INVALID, "set_tuning: NULL key");
  const std::string k = key;
  if (k == "conv_pipe") t.conv_pipe = v < 0 ? 0 : v;
  else if (k == "conv_pipe_korder") t.pipe_korder = v ? 1 : 0;
  else if (k == "conv_pipe_bm") t.pipe_bm = (v == 256 || v == 128 || v == 64) ? v : 0;
  else if (k == "conv_pipe_win") t.pipe_win = v ? 1 : 0;
  else if (k == "conv_pipe_pf") t.pipe_pf = v ? 1 : 0;
  else if (k == "conv_pipe_walk") t.pipe_walk = v > 0 ? v : 0;
  else if (k == "conv_pipe_cost") t.pipe_cost = v ? 1 : 0;
  else if (k == "conv_pipe_wloop") t.pipe_wloop = v ? 1 : 0;
  else if (k == "head1x1") t.head1x1 = v ? 1 : 0;
  else if (k == "dw3_tile") t.dw3_tile = v ? 1 : 0;
  else if (k == "fuse_head") t.fuse_head = v ? 1 : 0;
  else if (k == "two_streams") t.two_streams = v ? 1 : 0;
  else if (k == "conv_c32") t.conv_c32 = v ? 1 : 0;
  else if (k == "res_fuse") t.res_fuse = v < 0 ? 0 : v > 3 ? 3 : v;
  else if (k == "stem_k16") t.stem_k16 = v ? 1 : 0;
  else if (k == "pool_sep") t.pool_sep = v ? 1 : 0;
  else if (k == "pool_small64") t.pool_small64 = v ? 1 : 0;
  else if (k == "pool_small_pf") t.pool_small_pf = v <= 0 ? 0 : v >= 2 ? 2 : 1;
  else if (k == "acff_persist") t.acff_persist = v < 0 ? 0 : v;
  else if (k == "acff_chain") t.acff_chain = v;
  else if (k == "acff_band") t.acff_band = v < 0 ? 0 : v > 2 ? 2 : v;
  else if (k == "acff_band_rows") t.acff_band_rows = v < 1 ? 1 : v > 16 ? 16 : v;
  else if (k == "stem_abl") t.stem_abl = v;
  else if (k == "nms_variant") t.nms_variant = v;
  else if (k == "resize_stream") t.resize_stream = v;
  else if (k == "cls_front") t.cls_front = v ? 1 : 0;
  else if (k == "nms_split") t.nms_split = v ? 1 : 0;
  else throw Error{RTDM_E_INVALID, "set_tuning: unknown key " + k};
}

bool tuning_is_plan_time(const char* key) {
  const std::string k = key ? key : "";
  return k == "fuse_head" || k == "two_streams";
}

}  // namespace rtdm

extern "C" {

int rtdm_abi_version(void) { return RTDM_ABI_VERSION; }

const char* rtdm_last_error(void) { return get_error(); }

const char* rtdm_build_arch(void) { return "gfx950"; }

rtdm_status rtdm_set_tuning(const char* key, int value) {
  return guard([&] { tuning_set(default_tuning(), key, value); });
}

rtdm_status rtdm_yolo_decode(const float* p, int n, int na, int no, int ny, int nx, const float* anchors, int img_h,
                             int img_w, float* io, int io_rows, int row_offset, void* stream) {
  return guard([&] {
    RTDM_REQUIRE(p && io && anchors, RTDM_E_INVALID, "yolo_decode: NULL pointer");
    RTDM_REQUIRE(na > 0 && na <= 8 && no >= 6 && ny > 0 && nx > 0, RTDM_E_INVALID, "yolo_decode: bad shape");
    RTDM_REQUIRE(row_offset >= 0 && row_offset + na * ny * nx <= io_rows, RTDM_E_INVALID,
                 "yolo_decode: rows out of range");
    // create_grids (models.py:422-436): stride = max(img) / max(ng); anchor_vec = anchors / stride
    const double ystride = (double)std::max(img_h, img_w) / (double)std::max(ny, nx);
    // anchor_vec (<= 16 floats) rides in the kernel arguments: asynchronous, no staging buffer
    AnchorVec av{};
    for (int i = 0; i < 2 * na; ++i) av.v[i] = anchors[i] / (float)ystride;
    launch_yolo_decode(p, n, na, no, ny, nx, av, (float)ystride, io, io_rows, row_offset, (hipStream_t)stream);
  });
}

rtdm_status rtdm_yolo_layer_trt(const float* input, int batch, int yolo_width, int yolo_height, int num_anchors,
                                const float* anchors, int num_classes, int input_multiplier, float scale_x_y,
                                int new_coords, float* output, void* stream) {
  return guard([&] {
    if (batch == 0) return;
    // YoloPluginCreator::createPlugin checks (yolo_layer.cu:409-413), as status codes
    RTDM_REQUIRE(input && output && anchors, RTDM_E_INVALID, "yolo_layer_trt: NULL pointer");
    RTDM_REQUIRE(batch > 0 && yolo_width > 0 && yolo_height > 0, RTDM_E_INVALID, "yolo_layer_trt: bad shape");
    RTDM_REQUIRE(num_anchors > 0 && num_anchors <= kTrtMaxAnchors, RTDM_E_INVALID,
                 "yolo_layer_trt: num_anchors must be in [1, 6]");
    RTDM_REQUIRE(anchors[0] > 0.f && anchors[1] > 0.f, RTDM_E_INVALID, "yolo_layer_trt: anchors must be positive");
    RTDM_REQUIRE(num_classes > 0, RTDM_E_INVALID, "yolo_layer_trt: num_classes must be positive");
    RTDM_REQUIRE(input_multiplier == 8 || input_multiplier == 16 || input_multiplier == 32, RTDM_E_INVALID,
                 "yolo_layer_trt: input_multiplier must be 8, 16 or 32");
    RTDM_REQUIRE(scale_x_y >= 1.0f, RTDM_E_INVALID, "yolo_layer_trt: scale_x_y must be >= 1");
    TrtYoloArgs t;
    t.n_heads = 1;
    t.rows = num_anchors * yolo_width * yolo_height;
    t.no = 5 + num_classes;
    t.nc = num_classes;
    TrtYoloHead& d = t.h[0];
    d.na = num_anchors;
    d.ny = yolo_height;
    d.nx = yolo_width;
    d.in_w = yolo_width * input_multiplier;
    d.in_h = yolo_height * input_multiplier;
    d.scale_xy = scale_x_y;
    d.new_coords = new_coords ? 1 : 0;
    for (int j = 0; j < 2 * num_anchors; ++j) d.anchors[j] = anchors[j];
    launch_yolo_trt(input, batch, t, 1, output, (hipStream_t)stream);
  });
}

size_t rtdm_nms_workspace_size(int n, int n_anchors, int nc) {
  if (n <= 0 || n_anchors <= 0 || nc <= 0) return 0;
  return nms_workspace_size(n, n_anchors, nc);
}

rtdm_status rtdm_nms(const float* io, int n, int n_anchors, int no, float conf_thres, double iou_thres,
                     int multi_label, int agnostic, uint64_t class_mask, int max_det, void* workspace,
                     size_t workspace_bytes, float* det, int32_t* idx, int32_t* count, void* stream) {
  return guard([&] {
    if (n == 0) return;
    RTDM_REQUIRE(io && det && count && workspace, RTDM_E_INVALID, "nms: NULL pointer");
    RTDM_REQUIRE(n > 0 && n_anchors > 0 && no >= 6, RTDM_E_INVALID, "nms: bad shape");
    RTDM_REQUIRE(class_mask == ~0ull || no - 5 <= 64, RTDM_E_UNSUPPORTED,
                 "nms: a classes filter needs nc <= 64 (class_mask is one 64-bit word)");
    RTDM_REQUIRE(workspace_bytes >= nms_workspace_size(n, n_anchors, no - 5), RTDM_E_CAPACITY,
                 "nms: workspace too small");
    launch_nms(io, n, n_anchors, no, conf_thres, iou_thres, multi_label, agnostic, class_mask, max_det, workspace, det,
               idx, count, (hipStream_t)stream);
  });
}

rtdm_status rtdm_preprocess_frames(const uint8_t* frames, int n, int in_h, int in_w, int out_size, float* out,
                                   void* stream) {
  return guard([&] {
    if (n == 0) return;
    RTDM_REQUIRE(frames && out, RTDM_E_INVALID, "preprocess: NULL pointer");
    RTDM_REQUIRE(n > 0 && in_h > 0 && in_w > 0 && out_size > 0, RTDM_E_INVALID, "preprocess: bad shape");
    // resize tables: built (and uploaded) once per device and geometry, kept for the process
    int dev = 0;
    RTDM_HIP(hipGetDevice(&dev));
    const ResizePlan* p;
    {
      static std::mutex mu;
      static std::map<std::array<int, 4>, std::unique_ptr<ResizePlan>> plans;
      std::lock_guard<std::mutex> lock(mu);
      auto& slot = plans[{dev, in_h, in_w, out_size}];
      if (!slot) {
        auto np = std::make_unique<ResizePlan>();
        build_resize_plan(*np, in_h, in_w, out_size, true);
        slot = std::move(np);
      }
      p = slot.get();
    }
    // the horizontal-pass scratch is stream-ordered: allocated and freed on the caller's
    // stream, so the call returns without waiting for the work
    const hipStream_t s = (hipStream_t)stream;
    void* tmp = nullptr;
    RTDM_HIP(hipMallocAsync(&tmp, (size_t)n * p->rows * p->out * 3, s));
    try {
      launch_preprocess(*p, frames, n, (uint8_t*)tmp, out, 1, RTDM_F32, s);
    } catch (...) {
      (void)hipFreeAsync(tmp, s);
      throw;
    }
    RTDM_HIP(hipFreeAsync(tmp, s));
  });
}

rtdm_status rtdm_letterbox_geometry(int in_h, int in_w, int shape_h, int shape_w, int auto_, int scale_fill,
                                    int scaleup, int* geom) {
  return guard([&] {
    RTDM_REQUIRE(geom, RTDM_E_INVALID, "letterbox_geometry: NULL geom");
    RTDM_REQUIRE(in_h > 0 && in_w > 0 && shape_h > 0 && shape_w > 0, RTDM_E_INVALID, "letterbox_geometry: bad shape");
    // datasets.py:603-627, with Python's round() (ties to even) as std::nearbyint
    double r = (double)std::max(shape_h, shape_w) / (double)std::max(in_h, in_w);
    if (!scaleup) r = std::min(r, 1.0);
    int new_w = (int)std::nearbyint(in_w * r), new_h = (int)std::nearbyint(in_h * r);
    double dw = shape_w - new_w, dh = shape_h - new_h;
    if (auto_) {
      dw = (double)(((int)dw % 32 + 32) % 32);
      dh = (double)(((int)dh % 32 + 32) % 32);
    } else if (scale_fill) {
      dw = dh = 0.0;
      new_w = shape_h;  // new_unpad = new_shape (h, w) handed to cv2.resize as (w, h)
      new_h = shape_w;
    }
    dw /= 2;
    dh /= 2;
    const int top = (int)std::nearbyint(dh - 0.1), bottom = (int)std::nearbyint(dh + 0.1);
    const int left = (int)std::nearbyint(dw - 0.1), right = (int)std::nearbyint(dw + 0.1);
    geom[0] = new_h;
    geom[1] = new_w;
    geom[2] = new_h + top + bottom;
    geom[3] = new_w + left + right;
    geom[4] = top;
    geom[5] = left;
  });
}

rtdm_status rtdm_letterbox(const uint8_t* frames, int n, int in_h, int in_w, int pitch, int new_h, int new_w,
                           int out_h, int out_w, int top, int left, uint32_t pad_rgb, int swap_rb, uint8_t* out,
                           void* stream) {
  return guard([&] {
    if (n == 0) return;
    RTDM_REQUIRE(frames && out, RTDM_E_INVALID, "letterbox: NULL pointer");
    launch_letterbox(frames, n, in_h, in_w, pitch, new_h, new_w, out_h, out_w, top, left, pad_rgb, swap_rb, out,
                     (hipStream_t)stream);
  });
}

rtdm_status rtdm_resize_linear(const uint8_t* frames, int n, int in_h, int in_w, int pitch, int out_h, int out_w,
                               int swap_rb, uint8_t* out, void* stream) {
  return guard([&] {
    if (n == 0) return;
    RTDM_REQUIRE(frames && out, RTDM_E_INVALID, "resize_linear: NULL pointer");
    RTDM_REQUIRE(out_h > 0 && out_w > 0, RTDM_E_INVALID, "resize_linear: bad output size");
    launch_letterbox(frames, n, in_h, in_w, pitch, out_h, out_w, out_h, out_w, 0, 0, 0u, swap_rb, out,
                     (hipStream_t)stream, 1);
  });
}

}  // extern "C"
