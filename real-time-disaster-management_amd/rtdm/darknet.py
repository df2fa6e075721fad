"""Darknet YOLO detector on the HIP runtime.

Drop-in for victim_localization/yolov3/models.py ``Darknet`` /
``load_darknet_weights`` as used by detect.py:21-28,87: ``Darknet(cfg,
img_size)``, ``load_darknet_weights(model, path)`` or
``model.load_state_dict(torch.load(path)['model'])``, then ``model(img)[0]`` is
the decoded io [N, sum(A*ny*nx), 5+nc] fp32.  The cfg is parsed, planned
(fusions, buffers) and executed by librtdm.so (rtdm_detector_*).
"""
from __future__ import annotations

import ctypes
import os

import numpy as np
import torch

from . import _lib as L
from .synth import ACFF_KEYS, acff_layers, conv_layers, read_darknet_weights


def read_cfg(cfg: str) -> str:
    """parse_model_cfg path rules (parse_config.py:8-11): add .cfg, try cfg/ prefix."""
    path = cfg if cfg.endswith(".cfg") else cfg + ".cfg"
    if not os.path.exists(path) and os.path.exists(os.path.join("cfg", path)):
        path = os.path.join("cfg", path)
    with open(path, "r") as f:
        return f.read()


def state_dict_to_stream(cfg_text: str, sd: dict) -> np.ndarray:
    """{'module_list.{i}.Conv2d.weight', ...BatchNorm2d.*} (the reference Darknet state_dict)
    -> darknet weight stream in save_weights order (models.py:489-512)."""
    parts = []

    def g(k):
        v = sd[k]
        if isinstance(v, torch.Tensor):
            v = v.detach().cpu().float().numpy()
        return np.asarray(v, np.float32).reshape(-1)

    convs = {i: bn for (i, cin, cout, k, bn, head) in conv_layers(cfg_text)}
    acffs = {i for (i, c, f) in acff_layers(cfg_text)}
    for i in sorted(set(convs) | acffs):
        p = f"module_list.{i}."
        if i in acffs:  # ACFF block (models.py:46-55): module_list.i.acff_i.*
            parts += [g(f"{p}acff_{i}.{k}") for k in ACFF_KEYS]
        elif convs[i]:
            parts += [g(p + "BatchNorm2d.bias"), g(p + "BatchNorm2d.weight"), g(p + "BatchNorm2d.running_mean"),
                      g(p + "BatchNorm2d.running_var")]
            parts.append(g(p + "Conv2d.weight"))
        else:
            parts.append(g(p + "Conv2d.bias"))
            parts.append(g(p + "Conv2d.weight"))
    return np.concatenate(parts).astype(np.float32)


class Darknet(torch.nn.Module):
    """models.py:317 counterpart.  img_size: int or (h, w)."""

    def __init__(self, cfg: str, img_size=(416, 416)):
        super().__init__()
        self.cfg_text = cfg if "[net]" in cfg or "[network]" in cfg else read_cfg(cfg)
        if isinstance(img_size, int):
            img_size = (img_size, img_size)
        self.img_size = (int(img_size[0]), int(img_size[1]))
        self._stream = None
        self._calib = None
        self._dtype = L.RTDM_F32
        self._handle = None
        self._handle_key = None
        self.tuning = {}  # this model's own knobs (rtdm_detector_set_tuning), re-applied to every new handle
        self.info = self._plan_info()
        self.version = np.array([0, 2, 5], dtype=np.int32)
        self.seen = np.array([0], dtype=np.int64)

    def _plan_info(self):
        h = ctypes.c_void_p()
        L.check(L.lib().rtdm_detector_create(self.cfg_text.encode(), self.img_size[0], self.img_size[1], self._dtype,
                                             None, 0, 1, ctypes.byref(h)))
        try:
            info = L.rtdm_detector_info()
            L.check(L.lib().rtdm_detector_get_info(h, ctypes.byref(info)))
            n = L.lib().rtdm_detector_describe(h, None, 0)
            buf = ctypes.create_string_buffer(int(n))
            L.lib().rtdm_detector_describe(h, buf, n)
            self.plan_text = buf.value.decode()
        finally:
            L.lib().rtdm_detector_destroy(h)
        return info

    @property
    def n_anchors(self) -> int:
        return self.info.n_anchors_total

    @property
    def no(self) -> int:
        return self.info.no

    @property
    def flop_per_image(self) -> float:
        return self.info.flop_per_image

    # ---------------------------------------------------------------- weights --
    def load_weight_stream(self, stream: np.ndarray):
        stream = np.ascontiguousarray(np.asarray(stream, np.float32))
        if stream.size != self.info.weight_floats:
            raise ValueError(f"darknet weights: {stream.size} floats, cfg needs {self.info.weight_floats}")
        self._stream = stream
        self._release()

    def load_state_dict(self, state_dict, strict: bool = True):
        self.load_weight_stream(state_dict_to_stream(self.cfg_text, state_dict))

    def half(self):
        self._dtype = L.RTDM_F16
        self._release()
        return self

    def float(self):
        self._dtype = L.RTDM_F32
        self._release()
        return self

    def int8(self, calib: torch.Tensor):
        """int8-quantise the detector (README --quant int8; BASELINE config 5): the Cin % 128
        convs run on int8 MFMA (conv_pipe_i8) with per-input-channel activation scales,
        calibrated on `calib` (uint8 frames [N,H,W,3] or NCHW inputs on the GPU, kept for
        handles created later), folded into per-output-channel int8 weights."""
        if not calib.is_cuda:
            raise RuntimeError("calibration frames must be on the GPU")
        self._calib = calib.contiguous()
        self._dtype = L.RTDM_I8
        self._release()
        return self

    def _calibrate(self, h):
        x = self._calib
        kind = (L.RTDM_INPUT_FRAME_U8 if x.dtype == torch.uint8 else
                L.RTDM_INPUT_NCHW_F32 if x.dtype == torch.float32 else L.RTDM_INPUT_NCHW_F16)
        cap = self._handle_key[1]
        with torch.cuda.device(x.device):
            for i in range(0, x.shape[0], cap):
                c = x[i:i + cap]
                L.check(L.lib().rtdm_detector_calibrate(h, L.ptr(c), kind, c.shape[0], 1 if i == 0 else 0,
                                                        L.stream_ptr()))

    def fuse(self):  # models.py:397-411 (a no-op in the reference, BN is SyncBatchNorm); BN is always folded here
        return self

    def _release(self):
        if self._handle is not None:
            L.lib().rtdm_detector_destroy(self._handle)
            self._handle = None
            self._handle_key = None

    def __del__(self):
        try:
            self._release()
        except Exception:
            pass

    def handle(self, n: int):
        if self._stream is None:
            raise RuntimeError("Darknet: load weights before calling the model")
        dev = torch.cuda.current_device()
        cap = max(1, 1 << max(0, int(n - 1).bit_length()))
        key = (dev, self._dtype)
        if self._handle is not None and self._handle_key[0] == key and self._handle_key[1] >= n:
            return self._handle
        self._release()
        h = ctypes.c_void_p()
        L.check(L.lib().rtdm_detector_create(self.cfg_text.encode(), self.img_size[0], self.img_size[1], self._dtype,
                                             self._stream.ctypes.data_as(ctypes.POINTER(ctypes.c_float)),
                                             self._stream.size, cap, ctypes.byref(h)))
        self._handle = h
        self._handle_key = (key, cap)
        for k, v in self.tuning.items():
            L.check(L.lib().rtdm_detector_set_tuning(h, k.encode(), int(v)))
        # a new device handle: cached hipGraphs that captured the old one must not replay
        # (rtdm.pipeline keys its graphs on this counter, never on the handle address)
        self.handle_generation = getattr(self, "handle_generation", 0) + 1
        if self._dtype == L.RTDM_I8:
            self._calibrate(h)
        return h

    # knobs the planner reads at rtdm_detector_create only: a created handle refuses them
    PLAN_TIME_KEYS = ("fuse_head", "two_streams")

    def set_tuning(self, key: str, value: int):
        """One launch-time knob of rtdm_set_tuning for this model only (its handles; the
        process defaults and other models are unchanged): e.g. ("conv_pipe_cost", 1) plans the
        conv tiles for throughput when several batches are in flight.  Plan-time keys
        (PLAN_TIME_KEYS) raise ValueError: set them with rtdm_set_tuning before the model's
        first handle is created.  A change on a live handle bumps handle_generation, so
        rtdm.pipeline re-captures its hipGraphs instead of replaying kernels chosen under the
        old value."""
        if key in self.PLAN_TIME_KEYS:
            raise ValueError(f"{key} is a plan-time key: set it with rtdm_set_tuning before the handle is created")
        changed = self.tuning.get(key) != int(value)
        self.tuning[key] = int(value)
        if self._handle is not None:
            L.check(L.lib().rtdm_detector_set_tuning(self._handle, key.encode(), int(value)))
            if changed:
                self.handle_generation = getattr(self, "handle_generation", 0) + 1
        return self

    # ---------------------------------------------------------------- forward --
    def forward(self, x: torch.Tensor, out: torch.Tensor | None = None, stream=None):
        """x: [N,3,H,W] fp32/fp16 in [0,1] (detect.py:79-83) or [N,H,W,3] uint8 frames (the /255
        is fused).  Returns (io, None) like the reference's eval forward (models.py:393-395)."""
        if not x.is_cuda:
            raise RuntimeError("rtdm Darknet runs on the GPU: move the input to a cuda device")
        if x.dtype == torch.uint8:
            if x.dim() != 4 or x.shape[3] != 3 or tuple(x.shape[1:3]) != self.img_size:
                raise ValueError(f"uint8 frames must be [N,{self.img_size[0]},{self.img_size[1]},3]")
            kind = L.RTDM_INPUT_FRAME_U8
        else:
            if x.dim() != 4 or x.shape[1] != 3 or tuple(x.shape[2:]) != self.img_size:
                raise ValueError(f"input must be [N,3,{self.img_size[0]},{self.img_size[1]}] (planned size)")
            kind = L.RTDM_INPUT_NCHW_F32 if x.dtype == torch.float32 else L.RTDM_INPUT_NCHW_F16
        x = x.contiguous()
        n = x.shape[0]
        with torch.cuda.device(x.device):
            h = self.handle(n)
            if out is None:
                out = torch.empty((n, self.n_anchors, self.no), device=x.device, dtype=torch.float32)
            L.check(L.lib().rtdm_detect(h, L.ptr(x), kind, n, L.ptr(out), L.stream_ptr(stream)))
        return out, None

    def _run(self, fn, x: torch.Tensor, width: int, stream=None):
        if not x.is_cuda:
            raise RuntimeError("rtdm Darknet runs on the GPU: move the input to a cuda device")
        if x.dtype == torch.uint8:
            if x.dim() != 4 or x.shape[3] != 3 or tuple(x.shape[1:3]) != self.img_size:
                raise ValueError(f"uint8 frames must be [N,{self.img_size[0]},{self.img_size[1]},3]")
            kind = L.RTDM_INPUT_FRAME_U8
        else:
            if x.dim() != 4 or x.shape[1] != 3 or tuple(x.shape[2:]) != self.img_size:
                raise ValueError(f"input must be [N,3,{self.img_size[0]},{self.img_size[1]}] (planned size)")
            kind = L.RTDM_INPUT_NCHW_F32 if x.dtype == torch.float32 else L.RTDM_INPUT_NCHW_F16
        x = x.contiguous()
        n = x.shape[0]
        out = torch.empty((n, self.n_anchors, width), device=x.device, dtype=torch.float32)
        with torch.cuda.device(x.device):
            L.check(fn(self.handle(n), L.ptr(x), kind, n, L.ptr(out), L.stream_ptr(stream)))
        return out

    def forward_raw(self, x: torch.Tensor, stream=None) -> torch.Tensor:
        """Raw head predictions [N, sum(A*ny*nx), 5+nc] (YOLOLayer training-branch p of every
        head, models.py:240-250, in io's row order)."""
        return self._run(L.lib().rtdm_detect_raw, x, self.no, stream)

    def forward_trt(self, x: torch.Tensor, stream=None) -> torch.Tensor:
        """YoloLayer_TRT Detection records [N, sum(A*ny*nx), 7] (yolo_layer.cu:203-306)."""
        return self._run(L.lib().rtdm_detect_trt, x, 7, stream)

    def describe(self) -> str:
        """Text dump of the launch plan (steps, fusions, buffers) of the current handle."""
        h = self._handle if self._handle is not None else self.handle(1)
        need = L.lib().rtdm_detector_describe(h, None, 0)
        buf = ctypes.create_string_buffer(int(need) + 1)
        L.lib().rtdm_detector_describe(h, buf, len(buf))
        return buf.value.decode()

    def layer_output(self, layer: int, n: int) -> torch.Tensor:
        """NCHW fp32 copy of cfg layer `layer`'s output from the last forward (debug/parity)."""
        h = self._handle
        c, hh, ww = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        L.check(L.lib().rtdm_detector_layer_output(h, layer, n, None, 0, ctypes.byref(c), ctypes.byref(hh),
                                                   ctypes.byref(ww), None))
        out = torch.empty((n, c.value, hh.value, ww.value), device="cuda", dtype=torch.float32)
        L.check(L.lib().rtdm_detector_layer_output(h, layer, n, L.ptr(out), out.numel(), None, None, None,
                                                   L.stream_ptr()))
        return out


def load_darknet_weights(self: Darknet, weights: str, cutoff: int = -1):
    """models.py:439-486 counterpart (full files only; cutoff unsupported)."""
    if cutoff != -1:
        raise NotImplementedError("cutoff loading is a training feature")
    self.load_weight_stream(read_darknet_weights(weights))
