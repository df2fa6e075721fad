"""ACFF classifiers (Squeeze-ErNET, Squeeze-ErNET-RedConv, ErNET) on the HIP runtime.

Drop-in for disaster_detection/model/{squeeze_ernet,squeeze_ernet_redconv,ernet}.py
and the CLIs' ``load_model`` (aider-predict.py:22-45): same class names, same
state_dict keys, ``model(x)`` returns the [N, 5] softmax the reference returns.
The forward runs entirely in librtdm.so (rtdm_classify); nothing here computes.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np
import torch

from . import _lib as L
from .synth import classifier_param_shapes

CLASSES = ['collapsed building', 'fire', 'flooded areas', 'normal', 'traffic incident']  # aider-predict.py:83

_KINDS = {"squeeze-ernet": L.RTDM_SQUEEZE_ERNET, "squeeze-redconv": L.RTDM_SQUEEZE_REDCONV, "ernet": L.RTDM_ERNET}


def _to_numpy_sd(sd) -> dict:
    out = {}
    for k, v in sd.items():
        if k.endswith("num_batches_tracked"):
            continue
        if isinstance(v, torch.Tensor):
            v = v.detach().to("cpu", torch.float32).numpy()
        out[k] = np.ascontiguousarray(np.asarray(v, dtype=np.float32))
    return out


class _ACFFClassifier(torch.nn.Module):
    MODEL = ""
    INPUT = 140

    def __init__(self):
        super().__init__()
        self._params = None
        self._handle = None
        self._handle_key = None
        self._dtype = L.RTDM_F32
        self._calib = None
        self.logits = None  # fc output of the last forward (pre-softmax)

    # ---------------------------------------------------------------- weights --
    def load_state_dict(self, state_dict, strict: bool = True):
        sd = _to_numpy_sd(state_dict)
        shapes = classifier_param_shapes(self.MODEL)
        missing = [k for k in shapes if k not in sd]
        unexpected = [k for k in sd if k not in shapes]
        if strict and (missing or unexpected):
            raise RuntimeError(f"Error(s) in loading state_dict for {type(self).__name__}: "
                               f"missing {missing}, unexpected {unexpected}")
        for k, shp in shapes.items():
            if k in sd and tuple(sd[k].shape) != tuple(shp):
                raise RuntimeError(f"size mismatch for {k}: checkpoint {tuple(sd[k].shape)}, model {tuple(shp)}")
        self._params = {k: sd[k] for k in shapes if k in sd}
        self._release()
        return torch.nn.modules.module._IncompatibleKeys(missing, unexpected)

    def state_dict(self, *args, **kwargs):
        return {k: torch.from_numpy(v.copy()) for k, v in (self._params or {}).items()}

    # ------------------------------------------------------------- precision --
    def half(self):
        self._dtype = L.RTDM_F16
        self._release()
        return self

    def float(self):
        self._dtype = L.RTDM_F32
        self._release()
        return self

    def int8(self, calib: torch.Tensor):
        """int8 ACFF fusion GEMMs (the §8 int8 row for ErNET; the reference classifier has no
        int8 mode): activations stay fp16, the 1x1 fusion convs of the persistent and chained
        ACFF stages run on int8 MFMA with per-concat-channel activation scales calibrated on
        `calib` (uint8 frames [N,H,W,3] or [N,3,S,S] inputs on the GPU, or a list of such
        batches, e.g. frames of different sizes; kept for handles created later) folded into
        per-output-channel int8 weights.  The activation maxima are taken over all of them."""
        batches = list(calib) if isinstance(calib, (list, tuple)) else [calib]
        if not batches:
            raise ValueError("int8: no calibration frames")
        for x in batches:
            if not x.is_cuda:
                raise RuntimeError("calibration frames must be on the GPU")
        self._calib = [x.contiguous() for x in batches]
        self._dtype = L.RTDM_I8
        self._release()
        return self

    def _calibrate(self, h):
        cap = self._handle_key[1]
        first = True
        for x in self._calib:
            if x.dtype == torch.uint8:
                kind, hh, ww = L.RTDM_INPUT_FRAME_U8, x.shape[1], x.shape[2]
            else:
                kind = L.RTDM_INPUT_NCHW_F32 if x.dtype == torch.float32 else L.RTDM_INPUT_NCHW_F16
                hh, ww = x.shape[2], x.shape[3]
            with torch.cuda.device(x.device):
                for i in range(0, x.shape[0], cap):
                    c = x[i:i + cap]
                    L.check(L.lib().rtdm_classifier_calibrate(h, L.ptr(c), kind, c.shape[0], hh, ww,
                                                              1 if first else 0, L.stream_ptr()))
                    first = False

    def _release(self):
        if self._handle is not None:
            L.lib().rtdm_classifier_destroy(self._handle)
            self._handle = None
            self._handle_key = None

    def __del__(self):
        try:
            self._release()
        except Exception:
            pass

    def _get_handle(self, n: int):
        if self._params is None:
            raise RuntimeError(f"{type(self).__name__}: load_state_dict() before calling the model")
        dev = torch.cuda.current_device()
        cap = max(64, 1 << max(0, int(n - 1).bit_length()))
        key = (dev, self._dtype)
        if self._handle is not None and self._handle_key[0] == key and self._handle_key[1] >= n:
            return self._handle
        self._release()
        names = list(self._params.keys())
        arr = (L.rtdm_param * len(names))()
        keep = []
        for i, k in enumerate(names):
            a = self._params[k]
            keep.append(a)
            arr[i].name = k.encode()
            arr[i].data = a.ctypes.data_as(ctypes.POINTER(ctypes.c_float))
            arr[i].numel = a.size
        h = ctypes.c_void_p()
        L.check(L.lib().rtdm_classifier_create(_KINDS[self.MODEL], self._dtype, arr, len(names), cap,
                                               ctypes.byref(h)))
        self._handle = h
        self._handle_key = (key, cap)
        for k, v in getattr(self, "tuning", {}).items():
            L.check(L.lib().rtdm_classifier_set_tuning(h, k.encode(), int(v)))
        # a new device handle: cached hipGraphs that captured the old one must not replay
        # (rtdm.pipeline keys its graphs on this counter, never on the handle address)
        self.handle_generation = getattr(self, "handle_generation", 0) + 1
        if self._dtype == L.RTDM_I8:
            self._calibrate(h)
        return h

    def set_tuning(self, key: str, value: int):
        """One knob of rtdm_set_tuning for this model's handles only.  A change on a live handle
        bumps handle_generation (rtdm.pipeline then re-captures its hipGraphs)."""
        if not hasattr(self, "tuning"):
            self.tuning = {}
        changed = self.tuning.get(key) != int(value)
        self.tuning[key] = int(value)
        if self._handle is not None:
            L.check(L.lib().rtdm_classifier_set_tuning(self._handle, key.encode(), int(value)))
            if changed:
                self.handle_generation = getattr(self, "handle_generation", 0) + 1
        return self

    def describe(self, n: int = 1) -> str:
        """Text dump of the launch plan (one line per ACFF block: kernel, int8) of a handle for n."""
        h = self._get_handle(n)
        need = L.lib().rtdm_classifier_describe(h, None, 0)
        buf = ctypes.create_string_buffer(int(need) + 1)
        L.lib().rtdm_classifier_describe(h, buf, len(buf))
        return buf.value.decode()

    # ---------------------------------------------------------------- forward --
    def forward(self, x: torch.Tensor) -> torch.Tensor:
        """x: [N,3,S,S] fp32/fp16 CUDA tensor (the transformed image batch) -> softmax [N,5]."""
        if not x.is_cuda:
            raise RuntimeError("rtdm classifier runs on the GPU: move the input to a cuda device")
        if x.dim() != 4 or x.shape[1] != 3 or x.shape[2] != self.INPUT or x.shape[3] != self.INPUT:
            raise ValueError(f"{type(self).__name__} expects [N,3,{self.INPUT},{self.INPUT}] input, got "
                             f"{list(x.shape)} (the reference silently regroups rows for other sizes; "
                             f"not reproduced)")
        if x.dtype == torch.float32:
            kind = L.RTDM_INPUT_NCHW_F32
        elif x.dtype == torch.float16:
            kind = L.RTDM_INPUT_NCHW_F16
        else:
            raise TypeError("input must be float32 or float16")
        x = x.contiguous()
        return self._run(x, kind, x.shape[0], self.INPUT, self.INPUT)

    def classify_frames(self, frames: torch.Tensor) -> torch.Tensor:
        """frames: [N,H,W,3] uint8 RGB CUDA tensor; runs the CLI transform (aider.py:421-426) on
        device, then the model.  Returns softmax [N,5]; logits in self.logits."""
        if frames.dtype != torch.uint8 or frames.dim() != 4 or frames.shape[3] != 3:
            raise ValueError("frames must be uint8 [N,H,W,3]")
        frames = frames.contiguous()
        return self._run(frames, L.RTDM_INPUT_FRAME_U8, frames.shape[0], frames.shape[1], frames.shape[2])

    def _run(self, x, kind, n, h, w, stream=None):
        with torch.cuda.device(x.device):
            handle = self._get_handle(n)
            logits = torch.empty((n, 5), device=x.device, dtype=torch.float32)
            probs = torch.empty((n, 5), device=x.device, dtype=torch.float32)
            L.check(L.lib().rtdm_classify(handle, L.ptr(x), kind, n, h, w, L.ptr(logits), L.ptr(probs),
                                          L.stream_ptr(stream)))
        self.logits = logits
        return probs


class Squeeze_ErNET(_ACFFClassifier):
    """disaster_detection/model/squeeze_ernet.py:7 — 140x140 input."""
    MODEL = "squeeze-ernet"
    INPUT = 140


class Squeeze_RedConv(_ACFFClassifier):
    """disaster_detection/model/squeeze_ernet_redconv.py:7 — 140x140 input."""
    MODEL = "squeeze-redconv"
    INPUT = 140


class ErNET(_ACFFClassifier):
    """disaster_detection/model/ernet.py:6 — 240x240 input."""
    MODEL = "ernet"
    INPUT = 240


def build_model(model_name: str) -> _ACFFClassifier:
    if model_name == "ernet":
        return ErNET()
    if model_name == "squeeze-ernet":
        return Squeeze_ErNET()
    if model_name == "squeeze-redconv":
        return Squeeze_RedConv()
    raise ValueError(f"Unsupported model: {model_name}")


# Full-module pickles (disaster_detection/weights/Squeeze-ernet-92f1score.pt, ernet.pt, ...:
# torch.save(model) of the reference classes; their ACFF blocks pickle under the legacy
# path model.ernet.ACFF).  They load with torch.load(weights_only=True): the restricted
# unpickler only builds the allowlisted globals below -- these empty nn.Module stand-ins
# for the reference classes plus plain torch.nn layers -- and runs no code from the file.
class _PickledACFF(torch.nn.Module):
    """Stand-in for the pickled model.ernet.ACFF / model.acff.ACFF (acff.py:8)."""


class _PickledSqueezeErNET(torch.nn.Module):
    """Stand-in for model.squeeze_ernet.Squeeze_ErNET (squeeze_ernet.py:7)."""


class _PickledSqueezeRedConv(torch.nn.Module):
    """Stand-in for model.squeeze_ernet_redconv.Squeeze_RedConv (squeeze_ernet_redconv.py:7)."""


class _PickledErNET(torch.nn.Module):
    """Stand-in for model.ernet.ErNET (ernet.py:6)."""


def _pickle_allowlist():
    import collections
    nn = torch.nn
    return [(_PickledACFF, "model.ernet.ACFF"), (_PickledACFF, "model.acff.ACFF"),
            (_PickledSqueezeErNET, "model.squeeze_ernet.Squeeze_ErNET"),
            (_PickledSqueezeRedConv, "model.squeeze_ernet_redconv.Squeeze_RedConv"),
            (_PickledErNET, "model.ernet.ErNET"),
            nn.Conv2d, nn.BatchNorm2d, nn.LeakyReLU, nn.Dropout, nn.MaxPool2d, nn.AvgPool2d, nn.Linear, nn.Softmax,
            set, collections.OrderedDict]


def read_weights(weights_path: str) -> dict:
    """State dict from a reference checkpoint (SURVEY.md §8b "weight inputs"): a plain state
    dict (weights/*-state_dict.pt), a {'model_state_dict': ...} training checkpoint
    (train.py:310-321), a full-module pickle (weights/Squeeze-ernet-92f1score.pt etc.,
    through the allowlist above), or an .npz of arrays.  Every .pt goes through
    torch.load(weights_only=True)."""
    if not os.path.exists(weights_path):
        raise FileNotFoundError(f"No weights found at {weights_path}")
    if weights_path.endswith(".npz"):
        z = np.load(weights_path, allow_pickle=False)
        return {k: z[k] for k in z.files}
    with torch.serialization.safe_globals(_pickle_allowlist()):
        ckpt = torch.load(weights_path, map_location="cpu", weights_only=True)
    if isinstance(ckpt, torch.nn.Module):
        return {k: v for k, v in ckpt.state_dict().items() if not k.endswith("num_batches_tracked")}
    if isinstance(ckpt, dict) and "model_state_dict" in ckpt:
        return ckpt["model_state_dict"]
    return ckpt


QUANTS = ("fp32", "fp16", "int8")


def load_model(model_name: str, weights_path: str, device: torch.device, half: bool = False,
               quant: str | None = None, calib=None) -> _ACFFClassifier:
    """aider-predict.py:22-45 / evaluate-classification-metrics.py:24-47 counterpart.
    `quant` (the README's --quant {fp32,fp16,int8}, README.md:32-40) overrides `half`; int8
    needs `calib`: uint8 frames [N,H,W,3] on the device, or a list of such batches."""
    model = build_model(model_name)
    model.load_state_dict(read_weights(weights_path))
    if quant is None:
        quant = "fp16" if half else "fp32"
    if quant not in QUANTS:
        raise ValueError(f"quant must be one of {QUANTS}, got {quant!r}")
    if quant == "fp16":
        model.half()
    elif quant == "int8":
        if calib is None:
            raise ValueError("int8 needs calibration frames (--calib)")
        model.int8(calib)
    model.eval()
    return model
