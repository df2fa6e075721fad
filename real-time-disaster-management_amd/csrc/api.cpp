// Library-level C ABI: errors, version, stand-alone decode / NMS / preprocess.
#include <cstring>

#include "common.h"

namespace rtdm {

static thread_local std::string g_last_error;

void set_error(const std::string& msg) { g_last_error = msg; }
const char* get_error() { return g_last_error.c_str(); }

}  // namespace rtdm

using namespace rtdm;

extern "C" {

int rtdm_abi_version(void) { return RTDM_ABI_VERSION; }

const char* rtdm_last_error(void) { return get_error(); }

const char* rtdm_build_arch(void) { return "gfx950"; }

rtdm_status rtdm_set_tuning(const char* key, int value) {
  return guard([&] {
    RTDM_REQUIRE(key, RTDM_E_INVALID, "set_tuning: NULL key");
    if (!strcmp(key, "conv_pipe"))
      set_conv_pipe_mode(value);
    else if (!strcmp(key, "fuse_head"))
      set_fuse_head(value);
    else if (!strcmp(key, "two_streams"))
      set_two_streams_mode(value);
    else if (!strcmp(key, "acff_persist"))
      set_acff_persist_mode(value);
    else
      throw Error{RTDM_E_INVALID, std::string("set_tuning: unknown key ") + key};
  });
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
    // anchor_vec is tiny: stage it through a device buffer owned by the stream's lifetime
    static thread_local DevBuf av;
    float host[16];
    for (int i = 0; i < 2 * na; ++i) host[i] = anchors[i] / (float)ystride;
    if (!av.p) av.alloc(sizeof(host));
    RTDM_HIP(hipMemcpyAsync(av.p, host, sizeof(float) * 2 * na, hipMemcpyHostToDevice, (hipStream_t)stream));
    launch_yolo_decode(p, n, na, no, ny, nx, av.as<float>(), (float)ystride, io, io_rows, row_offset,
                       (hipStream_t)stream);
    // the host staging array must outlive the async copy
    RTDM_HIP(hipStreamSynchronize((hipStream_t)stream));
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
    ResizePlan p;
    build_resize_plan(p, in_h, in_w, out_size, true);
    DevBuf tmp;
    tmp.alloc((size_t)n * p.rows * p.out * 3);
    launch_preprocess(p, frames, n, tmp.as<uint8_t>(), out, 1, RTDM_F32, (hipStream_t)stream);
    // plan + tmp are released on return: finish the work first
    RTDM_HIP(hipStreamSynchronize((hipStream_t)stream));
  });
}

}  // extern "C"
