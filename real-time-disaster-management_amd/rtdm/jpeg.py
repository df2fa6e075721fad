"""Device JPEG decode: the decode inside cv2.imread (victim_localization/yolov3/utils/
datasets.py:97 load_image, disaster_detection/aider-predict.py:57) on the HIP runtime.

The bit-serial Huffman entropy decode runs on the host (``rtdm_jpeg_entropy_decode``, C++,
into int16 coefficient blocks in pinned memory); the blocks go to the device, where
dequantisation + islow IDCT (one thread per 8x8 block) and fancy upsampling + YCbCr -> RGB
(one thread per pixel) produce the uint8 [H, W, 3] frame in HBM, bit-exact with
libjpeg-turbo's default decompression, i.e. with cv2.imread / Pillow
(tests/test_gpu_jpeg.py).  Baseline and extended sequential 8-bit Huffman JPEGs (SOF0 /
SOF1; 4:4:4, 4:2:2, 4:2:0, grayscale; restart markers): every JPEG in the reference's
datasets.  ``supported(data)`` is False for progressive / arithmetic / 12-bit streams, which
``decode`` refuses with NotImplementedError (there is no silent host fallback).
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _lib as L


def info(data: bytes) -> L.rtdm_jpeg_info:
    """Header geometry (no entropy decode)."""
    buf = np.frombuffer(data, np.uint8)
    inf = L.rtdm_jpeg_info()
    L.check(L.lib().rtdm_jpeg_info_get(buf.ctypes.data, buf.size, ctypes.byref(inf)))
    return inf


def supported(data: bytes) -> bool:
    try:
        return bool(info(data).supported)
    except L.RtdmError:
        return False


def entropy_decode(data: bytes, pin: bool = False):
    """Host stage: (coef int16 [nblocks, 64], qt int16-viewed uint16 [ncomp, 64], info)."""
    buf = np.frombuffer(data, np.uint8)
    inf = info(data)
    if not inf.supported:
        raise NotImplementedError("rtdm.jpeg: only sequential 8-bit Huffman JPEGs (SOF0 / SOF1) decode on the device")
    coef = torch.empty((inf.nblocks, 64), dtype=torch.int16, pin_memory=pin)
    qt = torch.empty((max(1, inf.ncomp), 64), dtype=torch.int16, pin_memory=pin)
    L.check(L.lib().rtdm_jpeg_entropy_decode(buf.ctypes.data, buf.size, coef.data_ptr(), inf.nblocks, qt.data_ptr(),
                                            ctypes.byref(inf)))
    return coef, qt, inf


def decode(data: bytes, device=None, bgr: bool = False, out: torch.Tensor | None = None, stream=None) -> torch.Tensor:
    """JPEG bytes -> uint8 [H, W, 3] on the device (RGB; BGR with bgr=True, as cv2.imread
    returns it).  Asynchronous on the current (or given) stream."""
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    if dev.type != "cuda":
        raise ValueError("rtdm.jpeg.decode: the decoder runs on the HIP device (no CPU path)")
    coef, qt, inf = entropy_decode(data, pin=True)
    s = stream if stream is not None else torch.cuda.current_stream(dev)
    with torch.cuda.stream(s):
        coef_d = coef.to(dev, non_blocking=True)
        qt_d = qt.to(dev, non_blocking=True)
        ws = torch.empty(int(L.lib().rtdm_jpeg_workspace_bytes(ctypes.byref(inf))), dtype=torch.uint8, device=dev)
        if out is None:
            out = torch.empty((inf.height, inf.width, 3), dtype=torch.uint8, device=dev)
        if out.dtype != torch.uint8 or out.shape != (inf.height, inf.width, 3) or not out.is_contiguous():
            raise ValueError(f"rtdm.jpeg.decode: out must be a contiguous uint8 [{inf.height}, {inf.width}, 3] tensor")
        L.check(L.lib().rtdm_jpeg_reconstruct(coef_d.data_ptr(), qt_d.data_ptr(), ctypes.byref(inf), ws.data_ptr(),
                                             ws.numel(), out.data_ptr(), 3 * inf.width, int(bool(bgr)),
                                             L.stream_ptr(s)))
    return out


def imread(path: str, device=None, bgr: bool = True) -> torch.Tensor:
    """cv2.imread(path) for a JPEG file, decoded on the device (BGR by default, as cv2)."""
    with open(path, "rb") as f:
        return decode(f.read(), device=device, bgr=bgr)
