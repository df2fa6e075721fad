"""ctypes binding of the gfx950 HIP runtime ``librtdm.so`` (C ABI: include/rtdm.h).

This is the only way the Python side reaches the hot path: there is no eager
PyTorch or CPU fallback.  If the shared library is missing the import of any
compute entry point raises immediately (build it with ``make -C
real-time-disaster-management_amd`` or ``__graft_entry__.build()``).
"""
from __future__ import annotations

import ctypes
import os
from ctypes import (POINTER, c_char_p, c_double, c_float, c_int, c_int32, c_int64, c_size_t, c_uint32, c_uint64,
                    c_uint8, c_void_p)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("RTDM_LIB", os.path.join(_HERE, "librtdm.so"))

# rtdm_status
RTDM_OK = 0
RTDM_E_INVALID = 1
RTDM_E_HIP = 2
RTDM_E_CAPACITY = 3
RTDM_E_UNSUPPORTED = 4
RTDM_E_OOM = 5
STATUS_NAMES = {0: "OK", 1: "INVALID", 2: "HIP", 3: "CAPACITY", 4: "UNSUPPORTED", 5: "OOM"}
# rtdm_dtype
RTDM_F32 = 0
RTDM_F16 = 1
RTDM_I8 = 2
# rtdm_model_kind
RTDM_SQUEEZE_ERNET = 0
RTDM_SQUEEZE_REDCONV = 1
RTDM_ERNET = 2
# rtdm_input_kind
RTDM_INPUT_NCHW_F32 = 0
RTDM_INPUT_NCHW_F16 = 1
RTDM_INPUT_FRAME_U8 = 2


class RtdmError(RuntimeError):
    """A non-OK rtdm_status, with the library's thread-local message."""

    def __init__(self, status: int, msg: str):
        super().__init__(f"rtdm {STATUS_NAMES.get(status, status)}: {msg}")
        self.status = status


class rtdm_param(ctypes.Structure):
    _fields_ = [("name", c_char_p), ("data", POINTER(c_float)), ("numel", c_int64)]


class rtdm_detector_info(ctypes.Structure):
    _fields_ = [("img_h", c_int), ("img_w", c_int), ("n_layers", c_int), ("n_yolo", c_int),
                ("n_anchors_total", c_int), ("no", c_int), ("nc", c_int), ("weight_floats", c_int64),
                ("device_bytes", c_int64), ("flop_per_image", c_double)]


class rtdm_jpeg_info(ctypes.Structure):
    _fields_ = [("width", c_int), ("height", c_int), ("ncomp", c_int), ("h", c_int * 3), ("v", c_int * 3),
                ("bw", c_int * 3), ("bh", c_int * 3), ("coef_off", c_int64 * 3), ("nblocks", c_int64),
                ("supported", c_int)]


# name -> (restype, argtypes); must match include/rtdm.h exactly
SIGNATURES = {
    "rtdm_abi_version": (c_int, []),
    "rtdm_last_error": (c_char_p, []),
    "rtdm_build_arch": (c_char_p, []),
    "rtdm_set_tuning": (c_int, [c_char_p, c_int]),
    "rtdm_detector_set_tuning": (c_int, [c_void_p, c_char_p, c_int]),
    "rtdm_classifier_set_tuning": (c_int, [c_void_p, c_char_p, c_int]),
    "rtdm_classifier_create": (c_int, [c_int, c_int, POINTER(rtdm_param), c_int, c_int, POINTER(c_void_p)]),
    "rtdm_classifier_destroy": (c_int, [c_void_p]),
    "rtdm_classifier_input_size": (c_int, [c_void_p]),
    "rtdm_classify": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p]),
    "rtdm_classifier_calibrate": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p]),
    "rtdm_detector_create": (c_int, [c_char_p, c_int, c_int, c_int, POINTER(c_float), c_int64, c_int,
                                     POINTER(c_void_p)]),
    "rtdm_detector_destroy": (c_int, [c_void_p]),
    "rtdm_detector_get_info": (c_int, [c_void_p, POINTER(rtdm_detector_info)]),
    "rtdm_detector_describe": (c_int64, [c_void_p, c_char_p, c_int64]),
    "rtdm_classifier_describe": (c_int64, [c_void_p, c_char_p, c_int64]),
    "rtdm_detector_num_steps": (c_int, [c_void_p]),
    "rtdm_detector_step_info": (c_int, [c_void_p, c_int, c_char_p, c_int, POINTER(c_int), POINTER(c_double),
                                        POINTER(c_double)]),
    "rtdm_detector_enable_timing": (c_int, [c_void_p, c_int]),
    "rtdm_classifier_enable_timing": (c_int, [c_void_p, c_int]),
    "rtdm_classifier_read_timing": (c_int, [c_void_p, POINTER(c_double), POINTER(c_double), c_char_p, c_int,
                                            POINTER(c_int), POINTER(c_int)]),
    "rtdm_detector_read_timing": (c_int, [c_void_p, POINTER(c_double), POINTER(c_int)]),
    "rtdm_detect": (c_int, [c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p]),
    "rtdm_detect_raw": (c_int, [c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p]),
    "rtdm_detector_calibrate": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_void_p]),
    "rtdm_detect_trt": (c_int, [c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p]),
    "rtdm_yolo_layer_trt": (c_int, [c_void_p, c_int, c_int, c_int, c_int, POINTER(c_float), c_int, c_int, c_float,
                                    c_int, c_void_p, c_void_p]),
    "rtdm_detector_layer_output": (c_int, [c_void_p, c_int, c_int, c_void_p, c_int64, POINTER(c_int),
                                           POINTER(c_int), POINTER(c_int), c_void_p]),
    "rtdm_yolo_decode": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_int, POINTER(c_float), c_int, c_int,
                                 c_void_p, c_int, c_int, c_void_p]),
    "rtdm_nms_workspace_size": (c_size_t, [c_int, c_int, c_int]),
    "rtdm_nms": (c_int, [c_void_p, c_int, c_int, c_int, c_float, c_double, c_int, c_int, c_uint64, c_int, c_void_p,
                         c_size_t, c_void_p, c_void_p, c_void_p, c_void_p]),
    "rtdm_preprocess_frames": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p]),
    "rtdm_letterbox_geometry": (c_int, [c_int, c_int, c_int, c_int, c_int, c_int, c_int, POINTER(c_int)]),
    "rtdm_letterbox": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int,
                               c_uint32, c_int, c_void_p, c_void_p]),
    "rtdm_resize_linear": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p]),
    "rtdm_jpeg_info_get": (c_int, [c_void_p, c_int64, POINTER(rtdm_jpeg_info)]),
    "rtdm_jpeg_entropy_decode": (c_int, [c_void_p, c_int64, c_void_p, c_int64, c_void_p, POINTER(rtdm_jpeg_info)]),
    "rtdm_jpeg_workspace_bytes": (c_int64, [POINTER(rtdm_jpeg_info)]),
    "rtdm_jpeg_reconstruct": (c_int, [c_void_p, c_void_p, POINTER(rtdm_jpeg_info), c_void_p, c_int64, c_void_p, c_int64,
                                      c_int, c_void_p]),
}

_lib = None


def lib() -> ctypes.CDLL:
    """Load librtdm.so once; raise loudly if it is missing."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"librtdm.so not found at {LIB_PATH}: build the HIP runtime first "
                              "(make -C real-time-disaster-management_amd)")
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            try:
                fn = getattr(L, name)
            except AttributeError:
                # an older build named by RTDM_LIB (same-box A/B runs) may predate an entry
                # point; the in-tree library must export every one (tests/test_abi.py)
                if "RTDM_LIB" in os.environ:
                    continue
                raise
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def check(status: int) -> None:
    if status != RTDM_OK:
        msg = lib().rtdm_last_error()
        raise RtdmError(status, msg.decode() if msg else "")


def stream_ptr(stream=None) -> int:
    """hipStream_t of a torch stream (default: the current stream of the current device)."""
    import torch
    if stream is None:
        stream = torch.cuda.current_stream()
    return int(stream.cuda_stream)


def ptr(t) -> int:
    return int(t.data_ptr()) if t is not None else 0
