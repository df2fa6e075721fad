#!/usr/bin/env python3
"""Detector-only timing, fp16 vs int8 (RTDM_I8), with per-step event times.

  python tools/det_int8_timing.py [--cfg yolov4-tiny-aider-416] [--img 608] [--batch 64]"""
import argparse
import ctypes
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "real-time-disaster-management_amd"))

from rtdm import _lib as L  # noqa: E402
from rtdm.darknet import Darknet  # noqa: E402
from rtdm.synth import BASE_SEED, load_calibration, synth_darknet_weights, synth_frames  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--cfg", default="yolov4-tiny-aider-416")
ap.add_argument("--img", type=int, default=608)
ap.add_argument("--batch", type=int, default=64)
ap.add_argument("--iters", type=int, default=20)
args = ap.parse_args()
text = open(os.path.join(ROOT, "real-time-disaster-management_amd", "rtdm", "cfg", args.cfg + ".cfg")).read()
stream = synth_darknet_weights(text, calib=load_calibration(args.cfg))
frames = torch.from_numpy(synth_frames(args.batch, args.img, args.img)).cuda()
calib = torch.from_numpy(synth_frames(16, args.img, args.img, seed=BASE_SEED + 4321)).cuda()
res = {}
for mode in ("f16", "i8"):
    d = Darknet(text, (args.img, args.img))
    d.load_weight_stream(stream)
    if mode == "f16":
        d.half()
    else:
        d.int8(calib)
    h = d.handle(args.batch)
    for _ in range(3):
        d(frames)
    torch.cuda.synchronize()
    walls = []
    for _ in range(5):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(args.iters):
            d(frames)
        e.record()
        torch.cuda.synchronize()
        walls.append(s.elapsed_time(e) / args.iters)
    ns = L.lib().rtdm_detector_num_steps(h)
    L.check(L.lib().rtdm_detector_enable_timing(h, args.iters))
    for _ in range(args.iters):
        d(frames)
    torch.cuda.synchronize()
    ms = (ctypes.c_double * ns)()
    calls = ctypes.c_int()
    L.check(L.lib().rtdm_detector_read_timing(h, ms, ctypes.byref(calls)))
    L.check(L.lib().rtdm_detector_enable_timing(h, 0))
    steps = []
    for i in range(ns):
        nm = ctypes.create_string_buffer(128)
        layer, flop, byt = ctypes.c_int(), ctypes.c_double(), ctypes.c_double()
        L.check(L.lib().rtdm_detector_step_info(h, i, nm, 128, ctypes.byref(layer), ctypes.byref(flop),
                                                ctypes.byref(byt)))
        steps.append((layer.value, nm.value.decode(), flop.value * args.batch, ms[i] / max(1, calls.value)))
    res[mode] = (statistics.median(walls), steps)
    print(f"{mode}: forward {statistics.median(walls):.4f} ms  ({args.batch / statistics.median(walls) * 1e3:.0f} frames/s)")
for mode in ("f16", "i8"):
    print(f"-- {mode}")
    for (l, nm, f, t) in res[mode][1]:
        print(f"{l:5d} {nm[:34]:34s} {t:7.4f} ms {f / t / 1e9 if t else 0:8.1f} T(FL)OP/s")
