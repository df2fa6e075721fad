/*
 * rtdm.h — C ABI of the MI355X-native two-stage aerial-frame inference path
 * (ACFF classifier -> Darknet YOLO detector -> YOLO decode -> NMS).
 *
 * This is the drop-in boundary.  Every entry point replaces one call site of
 * the reference (qazi0/real-time-disaster-management, paths relative to
 * /root/reference/code):
 *
 *   rtdm_classifier_create   <- load_model()            disaster_detection/aider-predict.py:22-45
 *                               (model ctor + load_state_dict; weights are the
 *                                reference state-dict tensors, passed by name)
 *   rtdm_classify            <- model(data)             disaster_detection/aider-predict.py:76
 *                               Squeeze_ErNET.forward   disaster_detection/model/squeeze_ernet.py:24-45
 *                               Squeeze_RedConv.forward disaster_detection/model/squeeze_ernet_redconv.py:27-52
 *                               ErNET.forward           disaster_detection/model/ernet.py:25-49
 *                               + (RTDM_INPUT_FRAME_U8) the CLI transform
 *                               disaster_detection/dataloaders/aider.py:412-431
 *   rtdm_detector_create     <- Darknet(cfg, img_size) + load_darknet_weights()
 *                               victim_localization/yolov3/models.py:320-330, 439-486
 *   rtdm_detect              <- model(img)[0]           victim_localization/yolov3/detect.py:87
 *                               Darknet.forward         victim_localization/yolov3/models.py:332-395
 *                               YOLOLayer.forward       victim_localization/yolov3/models.py:204-258
 *   rtdm_yolo_decode         <- YOLOLayer inference branch (models.py:252-258) on raw
 *                               head maps; also the TensorRT plugin enqueue
 *                               victim_localization/tensorrt_inference/plugins/yolo_layer.cu:308-327
 *   rtdm_detect_trt          <- context.execute_async() of a YOLO engine with YoloLayer_TRT
 *                               victim_localization/tensorrt_inference/utils/yolo_with_plugins.py:268-282
 *   rtdm_yolo_layer_trt      <- YoloLayerPlugin::enqueue   tensorrt_inference/plugins/yolo_layer.cu:323-327
 *   rtdm_nms                 <- non_max_suppression()   victim_localization/yolov3/utils/utils.py:488-557
 *                               (+ torchvision.ops.boxes.nms, utils.py:552)
 *   rtdm_letterbox           <- letterbox()             victim_localization/yolov3/utils/datasets.py:599-631
 *   rtdm_resize_linear       <- cv2.resize(frame, (w, h)) disaster_detection/real-time-inference.py:185
 *   rtdm_preprocess_frames   <- squeeze_transforms / aider_transforms  disaster_detection/dataloaders/aider.py:412-431
 *   rtdm_jpeg_*              <- cv2.imread(path)        victim_localization/yolov3/utils/datasets.py:97,
 *                                                       disaster_detection/aider-predict.py:57
 *
 * Conventions
 *   - Plain C types only.  Device pointers are HIP device pointers owned by the
 *     caller (e.g. torch.empty(..., device='cuda').data_ptr()).
 *   - Every launch is asynchronous on the given stream (hipStream_t passed as
 *     void*; NULL = legacy default stream).  No host synchronisation inside.
 *   - Errors are returned as rtdm_status; rtdm_last_error() gives a message
 *     (thread-local).  Nothing aborts the process (the reference plugin's
 *     CHECK()/abort(), yolo_layer.h:13-22, becomes a status code).
 *   - A handle is bound to the device that was current at create time and must
 *     not be used from two streams concurrently (one handle per rank/stream).
 */
#ifndef RTDM_H_
#define RTDM_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RTDM_ABI_VERSION 1

typedef enum rtdm_status {
  RTDM_OK = 0,
  RTDM_E_INVALID = 1,      /* bad argument / unknown parameter / shape mismatch   */
  RTDM_E_HIP = 2,          /* a HIP runtime call failed                            */
  RTDM_E_CAPACITY = 3,     /* batch larger than max_batch, workspace too small     */
  RTDM_E_UNSUPPORTED = 4,  /* cfg layer / input size not supported                 */
  RTDM_E_OOM = 5           /* device allocation failed                             */
} rtdm_status;

typedef enum rtdm_dtype {
  RTDM_F32 = 0, /* fp32 activations/weights, fp32 FMA (parity mode)            */
  RTDM_F16 = 1, /* fp16 activations/weights, fp32 accumulation on MFMA          */
  RTDM_I8 = 2   /* fp16 activations in HBM, int8 MFMA in the hot GEMMs, per-channel
                   activation scales folded into per-output-channel int8 weights.
                   detector: every conv with Cin % 128 == 0 runs on conv_pipe_i8
                   (v_mfma_i32_16x16x64_i8) over an int8 copy of its input
                   (rtdm_detector_calibrate); the reference's README --quant int8
                   (config 5).  classifier: the ACFF 1x1 fusion GEMMs of the persistent
                   and chained stages (rtdm_classifier_calibrate).                     */
} rtdm_dtype;

typedef enum rtdm_model_kind {
  RTDM_SQUEEZE_ERNET = 0,  /* Squeeze_ErNET,   input 140x140 (squeeze_ernet.py:7)          */
  RTDM_SQUEEZE_REDCONV = 1,/* Squeeze_RedConv, input 140x140 (squeeze_ernet_redconv.py:7)  */
  RTDM_ERNET = 2           /* ErNET,           input 240x240 (ernet.py:6)                  */
} rtdm_model_kind;

typedef enum rtdm_input_kind {
  RTDM_INPUT_NCHW_F32 = 0, /* model input tensor [n,3,H,W] fp32 (already transformed)        */
  RTDM_INPUT_NCHW_F16 = 1, /* same, fp16 (the reference's --trt --quant fp16 .half() input)   */
  RTDM_INPUT_FRAME_U8 = 2  /* raw RGB frames [n,H,W,3] uint8; transform fused on device:
                              classifier: PIL-bilinear resize(int(1.14*S)) -> center crop S ->
                              /255 -> ImageNet Normalize (aider.py:412-426);
                              detector:   /255 (detect.py:80-82; frames must be img_size^2) */
} rtdm_input_kind;

/* One named parameter tensor: the reference state_dict key and its fp32 data
 * (host memory, contiguous, the reference's own layout — OIHW for convs). */
typedef struct rtdm_param {
  const char* name;
  const float* data;
  int64_t numel;
} rtdm_param;

typedef struct rtdm_classifier_s* rtdm_classifier;
typedef struct rtdm_detector_s* rtdm_detector;

typedef struct rtdm_detector_info {
  int img_h, img_w;     /* network input size                                     */
  int n_layers;         /* number of cfg layers (module_defs minus [net])         */
  int n_yolo;           /* number of [yolo] heads                                  */
  int n_anchors_total;  /* rows of io per image (sum A*ny*nx, models.py:393-395)  */
  int no;               /* 5 + nc                                                  */
  int nc;               /* classes                                                 */
  int64_t weight_floats;/* floats expected in the darknet weight stream            */
  int64_t device_bytes; /* device memory held by the handle                        */
  double flop_per_image;/* 2*MAC over conv layers (roofline numerator)             */
} rtdm_detector_info;

/* ---- library --------------------------------------------------------------- */
int rtdm_abi_version(void);
const char* rtdm_last_error(void);
/* gfx arch string the code objects were built for ("gfx950"). */
const char* rtdm_build_arch(void);
/* Kernel-selection knobs for A/B measurement (no reference counterpart; the
 * defaults are the tuned choice).  rtdm_set_tuning sets the PROCESS DEFAULTS: a
 * detector / classifier handle copies them when it is created, and each handle's
 * copy can be changed afterwards with rtdm_detector_set_tuning /
 * rtdm_classifier_set_tuning (every call on a handle runs with its own copy, so two
 * handles in one process can differ, e.g. a latency and a throughput pipeline).
 * Plan-time keys ("fuse_head", "two_streams") only act at handle creation:
 * rtdm_detector_set_tuning refuses them on a created handle (RTDM_E_INVALID).
 * key "conv_pipe": 1 = pipelined 256x128 implicit GEMM for Cin%64==0 convs
 * (default), 0 = conv_glds_f16 128x128; key "fuse_head": 1 = conv -> 1x1 head conv
 * -> [yolo] planned as one launch, 0 = separate head conv (default: the conv then runs
 * the tap-unrolled window loop and head1x1_f16 the head, measured faster); key
 * "acff_persist": 1 = persistent ACFF kernel for the large classifier maps
 * (default), 0 = 8x8-tile fused ACFF kernel; key "two_streams": 1 = detector head
 * branches on a side stream (default), 0 = one stream.  conv_pipe variants, all
 * bit-identical to each other: "conv_pipe_bm" 0 = tile rows by the cost model
 * (default) | 256 | 128 | 64; "conv_pipe_cost" 0 = the cost model minimises one
 * launch's rounds of tiles (latency, default) | 1 = CU-time (throughput, for several
 * batches in flight); "conv_pipe_win" 1 = window mode for 3x3/s1 layers (default);
 * "conv_pipe_korder" 1 = channel-block-outer K order (default; 0 changes the fp32
 * summation order); "conv_pipe_pf" 1 = cross-tile prologue prefetch (default);
 * "conv_pipe_wloop" 1 = tap-unrolled 3x3 K-loop for the register-epilogue layers
 * (default), 0 = the cursor loop; "conv_pipe_walk" g = tile walk in N-groups of g
 * panels (default 2, 0 = M-major); "conv_c32" 1 = the Cin-32 3x3 convs on conv3_c32
 * (default; bit-identical to 0 = conv_mfma / conv3_direct); "res_fuse" 1 =
 * Darknet-53's first residual block (1x1 64 -> 32, 3x3 32 -> 64, shortcut) as one
 * conv3_c32r launch, 8 waves, and each 104x104 (at 416) block (1x1 128 -> 64, 3x3
 * 64 -> 128, shortcut) as one conv3_c64r launch (default; 2 = conv3_c32r on 4 waves
 * only; 3 = conv3_c32r on 8 waves only; 0 = two launches per block; bit-identical; a
 * fused reduce map is not materialised: layer_output refuses it); "stem_k16" 1 = the
 * Cin-3 MFMA stems with the kh = 2 third of K on a 16-deep MFMA (default; bit-identical
 * to 0 = a 32-deep one); "cls_front" 1 = a classifier's uint8-frame transform and its
 * 16-channel conv1 as one launch (default; bit-identical to 0 = two launches); "nms_split"
 * 1 = NMS images of <= 512 candidates take their IoU bitmask over many blocks and the greedy
 * scan in a third launch (default; identical survivors to 0 = one launch per image); "pool_small_pf" 0 = halo tiles in flight per conv3_pool_small
 * block by Cin (default: 2 for Cin 16, 1 for Cin 32) | 1 | 2 (bit-identical);
 * "pool_small64" 1 = 3x3 Cin 64 -> Cout 128 + 2x2 pool (+ full map) on conv3_pool_small
 * (default; bit-identical to 0 = conv_pipe); "pool_sep" 1 = stride-1 5 / 9 / 13 max pools
 * (SPP) and the zero-padded 2 x 2 stride-1 pool as separable band kernels (default;
 * bit-identical to 0).  Variants measured slower in earlier rounds (256 x 256 conv tiles,
 * the ping-pong K-loop, the fused stem pair, the persistent stem, register-epilogue pools)
 * were removed (DESIGN.md §3.4 keeps their numbers).
 * Unknown keys: RTDM_E_INVALID. */
rtdm_status rtdm_set_tuning(const char* key, int value);
/* The same keys on one handle's own copy (see above). */
rtdm_status rtdm_detector_set_tuning(rtdm_detector h, const char* key, int value);
rtdm_status rtdm_classifier_set_tuning(rtdm_classifier h, const char* key, int value);

/* ---- classifier ------------------------------------------------------------ */
/* params: the reference state_dict (e.g. weights/squeeze-ernet-state_dict.pt),
 * every key required by the model kind; num_batches_tracked may be omitted.     */
rtdm_status rtdm_classifier_create(int kind, int dtype, const rtdm_param* params, int n_params,
                                   int max_batch, rtdm_classifier* out);
rtdm_status rtdm_classifier_destroy(rtdm_classifier h);
/* Input side length the model expects (140 or 240). */
/* Per-launch timing of rtdm_classify (bench / roofline): hipEvents recorded on the call's
 * stream around each kernel launch of the next max_calls calls (0 turns it off).  read:
 * summed ms per launch over the timed calls, the launch's algorithmic HBM bytes (model
 * input / activation maps read + written, for the batch of the first timed call), its
 * name (preprocess, stem, acff<k>, acff_chain, tail) at names + i * name_stride, the
 * launch count and the timed call count.  Arrays hold >= 24 entries.  Replaces the
 * reference's per-batch wall-clock timing (evaluate-classification-metrics.py:75-79). */
rtdm_status rtdm_classifier_enable_timing(rtdm_classifier h, int max_calls);
rtdm_status rtdm_classifier_read_timing(rtdm_classifier h, double* ms_per_launch, double* bytes_per_launch,
                                        char* names, int name_stride, int* n_launches, int* calls);
int rtdm_classifier_input_size(rtdm_classifier h);
/* Human-readable plan: one line per ACFF block (geometry, kernel, pool, reducer,
 * int8); returns bytes needed including the NUL when buf is too small.            */
int64_t rtdm_classifier_describe(rtdm_classifier h, char* buf, int64_t buf_len);
/* x: see rtdm_input_kind.  For FRAME_U8, in_h/in_w are the frame size; for the
 * NCHW kinds they must equal the model input size.
 * logits: [n,5] fc output (pre-softmax) or NULL; probs: [n,5] softmax (the value
 * the reference nn.Module returns) or NULL.                                      */
rtdm_status rtdm_classify(rtdm_classifier h, const void* x, int x_kind, int n, int in_h, int in_w,
                          float* logits, float* probs, void* stream);
/* int8 calibration of an RTDM_I8 classifier (activations stay fp16; the ACFF 1x1
 * fusion GEMMs of the persistent and chained stages run on int8 MFMA): runs the
 * network in fp16 on x (kinds as rtdm_classify) recording every int8 stage's
 * per-concat-channel |x|max (max over all calls since the last reset != 0), then
 * folds s_k = |x|max_k / 127 into the fusion weights and quantises them per output
 * channel, as rtdm_detector_calibrate.  Synchronises the stream.  rtdm_classify on an
 * uncalibrated RTDM_I8 handle returns RTDM_E_INVALID.  The reference has no int8
 * classifier; this is the §8 int8 row for ErNET.                */
rtdm_status rtdm_classifier_calibrate(rtdm_classifier h, const void* x, int x_kind, int n, int in_h, int in_w,
                                      int reset, void* stream);

/* ---- detector -------------------------------------------------------------- */
/* cfg_text: contents of a Darknet .cfg (victim_localization/yolov3/cfg/NAME.cfg),
 * parsed like parse_model_cfg (utils/parse_config.py:6-52).
 * weights: the float32 stream of a darknet .weights file after its 20-byte
 * header (load_darknet_weights order, models.py:449-486); n_floats must equal
 * rtdm_detector_info.weight_floats (query with weights=NULL first).
 * If weights == NULL the handle is created for planning/introspection only
 * (no device memory).                                                           */
rtdm_status rtdm_detector_create(const char* cfg_text, int img_h, int img_w, int dtype,
                                 const float* weights, int64_t n_floats, int max_batch,
                                 rtdm_detector* out);
rtdm_status rtdm_detector_destroy(rtdm_detector h);
rtdm_status rtdm_detector_get_info(rtdm_detector h, rtdm_detector_info* info);
/* Human-readable execution plan (kernels, fusions, buffers); returns bytes
 * needed including the NUL when buf is too small.                               */
int64_t rtdm_detector_describe(rtdm_detector h, char* buf, int64_t buf_len);
/* Execution steps (kernel launches) of the plan, with the kernel symbol, the
 * algorithmic FLOPs (2*MAC) and compulsory HBM bytes per image of each step. */
int rtdm_detector_num_steps(rtdm_detector h);
rtdm_status rtdm_detector_step_info(rtdm_detector h, int step, char* name, int name_len, int* layer,
                                    double* flop_per_image, double* bytes_per_image);
/* Per-step device timing (roofline measurement): hipEvents are recorded on the
 * launch stream between steps of the next max_calls rtdm_detect calls (0 = off).
 * read_timing synchronises those events and returns the summed ms per step.    */
rtdm_status rtdm_detector_enable_timing(rtdm_detector h, int max_calls);
rtdm_status rtdm_detector_read_timing(rtdm_detector h, double* ms_per_step, int* calls);
/* io: [n, n_anchors_total, no] fp32, exactly the reference's torch.cat(io, 1).
 * Inputs must be finite: the conv kernels are built with -fno-honor-nans (their max-pool
 * and LeakyReLU epilogues skip NaN canonicalisation), so a NaN / Inf in an NCHW float
 * input yields unspecified io rows where the reference would carry NaN to its NMS finite
 * filter (utils.py:535-536).  uint8 frames (RTDM_INPUT_FRAME_U8) are always finite.   */
rtdm_status rtdm_detect(rtdm_detector h, const void* x, int x_kind, int n, float* io, void* stream);
/* int8 calibration (RTDM_I8 handles): runs the network in fp16 on x (n images, kinds
 * as rtdm_detect) recording every int8 conv's per-input-channel |x|max (max over all
 * calls since the last reset != 0), then sets the activation scales s_c = |x|max_c / 127,
 * folds them into the conv's BN-folded weights and quantises those per output channel
 * (symmetric int8, deq[o] = max|W'[o]| / 127).  Synchronises the stream (a setup step).
 * n = 0 with reset = 0 only recomputes the weights from the recorded maxima.
 * rtdm_detect on an uncalibrated RTDM_I8 handle returns RTDM_E_INVALID.  This replaces
 * the TensorRT entropy-calibration caches (calib_cache/ *.bin), which the reference
 * builds with its own engines (calibrator.py:87-153; build_tensorrt_model.py:256-259 is a
 * stub).                                                                          */
rtdm_status rtdm_detector_calibrate(rtdm_detector h, const void* x, int x_kind, int n, int reset, void* stream);
/* Raw head predictions: p [n, n_anchors_total, no] fp32 in io's row order, i.e. the
 * YOLOLayer training-branch output p.view(bs,na,no,ny,nx).permute(0,1,3,4,2)
 * (models.py:240-250) of every head, concatenated like io.                      */
rtdm_status rtdm_detect_raw(rtdm_detector h, const void* x, int x_kind, int n, float* p, void* stream);
/* TensorRT-layout detections: dets [n, n_anchors_total, 7] Detection records
 * {x, y, w, h, det_confidence, class_id, class_confidence} (yolo_layer.h:26-31),
 * per head exactly the YoloLayer_TRT plugin output (CalDetection, or
 * CalDetection_NewCoords when the [yolo] block sets new_coords=1; scale_x_y from
 * the cfg, default 1), heads in cfg order = the engine's output bindings
 * concatenated (yolo_with_plugins.py:115-119).  Replaces context.execute_async
 * (yolo_with_plugins.py:268-282) for trt_yolo.py.  Allocates a raw-head scratch
 * buffer on the first call.                                                      */
rtdm_status rtdm_detect_trt(rtdm_detector h, const void* x, int x_kind, int n, float* dets, void* stream);
/* Debug/parity: copy cfg layer `layer`'s output of the LAST rtdm_detect call as
 * NCHW fp32 [n,C,H,W] into out (only for layers whose full-resolution output is
 * materialised; returns RTDM_E_UNSUPPORTED otherwise).                          */
rtdm_status rtdm_detector_layer_output(rtdm_detector h, int layer, int n, float* out, int64_t out_numel,
                                       int* c, int* hgt, int* wid, void* stream);

/* ---- stand-alone YOLO decode (YOLOLayer inference branch) --------------------
 * p: raw head map NCHW [n, na*no, ny, nx] fp32.  anchors: [na*2] pixels (host).
 * Writes io rows [row_offset, row_offset + na*ny*nx) of io [n, io_rows, no].     */
rtdm_status rtdm_yolo_decode(const float* p, int n, int na, int no, int ny, int nx, const float* anchors,
                             int img_h, int img_w, float* io, int io_rows, int row_offset, void* stream);

/* ---- TensorRT YoloLayer_TRT plugin (yolo_layer.cu:308-327 enqueue) --------------
 * input: one head's raw map NCHW [batch, num_anchors*(5+num_classes), yolo_height,
 * yolo_width] fp32.  anchors: [num_anchors*2] pixels (host; copied into the launch).
 * output: [batch, num_anchors*yolo_height*yolo_width, 7] Detection records.  The
 * engine input size is yolo_{width,height} * input_multiplier (createPlugin,
 * yolo_layer.cu:416); its asserts (:409-413) become RTDM_E_INVALID.               */
rtdm_status rtdm_yolo_layer_trt(const float* input, int batch, int yolo_width, int yolo_height, int num_anchors,
                                const float* anchors, int num_classes, int input_multiplier, float scale_x_y,
                                int new_coords, float* output, void* stream);

/* ---- NMS (non_max_suppression, utils.py:488-557, method 'vision_batch') -------
 * io: [n, n_anchors, no] fp32 (no = 5 + nc).
 * Semantics: obj > conf, 2 < w,h < 4096, cls *= obj, xywh->xyxy, multi-label
 * ((cls > conf) pairs, in (anchor, class) order) if multi_label && nc > 1 else
 * best class, optional class filter (class_mask bit c; ~0 = all), finite filter,
 * boxes offset by class*4096 unless agnostic, greedy NMS in descending score
 * (IoU > iou_thres suppresses, torchvision.ops.boxes.nms), ties -> lower
 * candidate index first.
 * det: [n, max_det, 6] rows (x1,y1,x2,y2,conf,cls) in descending score.
 * idx: [n, max_det, 2] (anchor row, class) of each kept row, or NULL.
 * count: [n] number of survivors (may exceed max_det; rows beyond are dropped).
 * workspace: device scratch of rtdm_nms_workspace_size(n, n_anchors, nc) bytes. */
size_t rtdm_nms_workspace_size(int n, int n_anchors, int nc);
rtdm_status rtdm_nms(const float* io, int n, int n_anchors, int no, float conf_thres, double iou_thres,
                     int multi_label, int agnostic, uint64_t class_mask, int max_det, void* workspace,
                     size_t workspace_bytes, float* det, int32_t* idx, int32_t* count, void* stream);

/* ---- pre-processing (CLI transform, aider.py:412-426) --------------------------
 * frames: [n, in_h, in_w, 3] uint8 RGB.  out: [n, 3, S, S] fp32 (the tensor the
 * reference feeds to model(), NCHW).  Resize shorter side to int(S*1.14) with
 * Pillow's 8-bit antialiased BILINEAR, center crop S, ToTensor, Normalize.      */
rtdm_status rtdm_preprocess_frames(const uint8_t* frames, int n, int in_h, int in_w, int out_size,
                                   float* out, void* stream);

/* ---- detector ingest: letterbox (yolov3/utils/datasets.py:599-631, :508-522) ----
 * rtdm_letterbox_geometry: the shape arithmetic of letterbox(img, (shape_h, shape_w),
 * auto, scaleFill, scaleup) for an in_h x in_w image: geom = {new_h, new_w, out_h,
 * out_w, top, left} (resize target, canvas, placement; Python round() semantics).
 * rtdm_letterbox: frames [n, in_h, pitch] uint8, 3 channels per pixel (pitch >= 3*in_w)
 * -> out [n, out_h, out_w, 3] uint8: each frame resized to new_w x new_h with
 * cv2.INTER_AREA semantics (area averaging when shrinking, INTER_AREA's linear
 * coefficients when growing) at (left, top), the rest pad_rgb (0x00BBGGRR, output
 * order).  swap_rb = 1 reads BGR (cv2 frames) and writes RGB.  The output feeds
 * rtdm_detect with RTDM_INPUT_FRAME_U8.  Replaces cv2.resize + cv2.copyMakeBorder
 * (datasets.py:626-630) and load_image's shrink (:517-520, new = int(side * r)).  */
rtdm_status rtdm_letterbox_geometry(int in_h, int in_w, int shape_h, int shape_w, int auto_, int scale_fill,
                                    int scaleup, int* geom);
rtdm_status rtdm_letterbox(const uint8_t* frames, int n, int in_h, int in_w, int pitch, int new_h, int new_w,
                           int out_h, int out_w, int top, int left, uint32_t pad_rgb, int swap_rb, uint8_t* out,
                           void* stream);

/* ---- frame resize (real-time-inference.py:185, cv2.resize(frame, (width, height))) --
 * cv2.INTER_LINEAR (the default interpolation) of uint8 3-channel frames [n, in_h, pitch]
 * to [n, out_h, out_w, 3]: half-pixel source coordinates, 11-bit fixed-point weights
 * (OpenCV resize.cpp restated; cv2 is not in this stack, so pixel parity with cv2 itself
 * is unpinned, the kernel is bit-exact with oracle/letterbox.py resize_linear).  The
 * vertical pass models OpenCV's SCALAR rounding, (b0*h0 + b1*h1 + 2^21) >> 22; cv2's
 * SIMD 8-bit path (>> 4, mulhi, then (x + 2) >> 2) may round differently, by up to 1 LSB
 * on a pixel.  swap_rb = 1 also turns BGR into RGB (the cv2.cvtColor of :70).       */
rtdm_status rtdm_resize_linear(const uint8_t* frames, int n, int in_h, int in_w, int pitch, int out_h, int out_w,
                               int swap_rb, uint8_t* out, void* stream);

/* ---- JPEG frame decode (cv2.imread: yolov3/utils/datasets.py:97, aider-predict.py:57) ----
 * Baseline / extended sequential 8-bit Huffman JPEGs (SOF0 / SOF1), 1 or 3 components,
 * 4:4:4, 4:2:2 (h2v1) or 4:2:0 (h2v2) sampling, restart intervals, interleaved or
 * per-component scans.  Split as the data dictates: the bit-serial entropy decode on the
 * host (rtdm_jpeg_entropy_decode, into int16 coefficient blocks, natural order), the
 * per-block / per-pixel rest on the device (rtdm_jpeg_reconstruct: dequantisation, islow
 * IDCT, fancy upsampling, YCbCr -> RGB), bit-exact with libjpeg-turbo's default
 * decompression (JDCT_ISLOW, do_fancy_upsampling), i.e. with what cv2.imread and Pillow
 * return.  Progressive / arithmetic / 12-bit streams: supported = 0 and RTDM_E_UNSUPPORTED.
 *
 * rtdm_jpeg_info_get: geometry from the headers (no entropy decode).
 * rtdm_jpeg_entropy_decode: coef [nblocks][64] int16 (host memory, component c's block
 *   (by, bx) at coef_off[c] + by * bw[c] + bx), qt [ncomp][64] uint16 natural order.
 * rtdm_jpeg_reconstruct: coef / qt device copies -> rgb [height][pitch] uint8 (3 bytes per
 *   pixel, RGB, or BGR as cv2 with bgr = 1); planes: device workspace of
 *   rtdm_jpeg_workspace_bytes(info) bytes (the component sample planes).              */
typedef struct rtdm_jpeg_info {
  int width, height, ncomp;
  int h[3], v[3];        /* sampling factors */
  int bw[3], bh[3];      /* coefficient block grid of each component (MCU-padded) */
  int64_t coef_off[3];   /* first block of each component */
  int64_t nblocks;       /* coefficient buffer: nblocks * 64 int16 */
  int supported;         /* 1: decodable by rtdm_jpeg_entropy_decode + rtdm_jpeg_reconstruct */
} rtdm_jpeg_info;
rtdm_status rtdm_jpeg_info_get(const uint8_t* data, int64_t len, rtdm_jpeg_info* info);
rtdm_status rtdm_jpeg_entropy_decode(const uint8_t* data, int64_t len, int16_t* coef, int64_t nblocks, uint16_t* qt,
                                     rtdm_jpeg_info* info);
int64_t rtdm_jpeg_workspace_bytes(const rtdm_jpeg_info* info);
rtdm_status rtdm_jpeg_reconstruct(const int16_t* coef, const uint16_t* qt, const rtdm_jpeg_info* info, uint8_t* planes,
                                  int64_t planes_bytes, uint8_t* rgb, int64_t pitch, int bgr, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* RTDM_H_ */
