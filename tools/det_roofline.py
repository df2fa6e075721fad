#!/usr/bin/env python3
"""Per-step roofline of the fp16 detector forward: event time per launch step, algorithmic
FLOP and bytes (rtdm_detector_step_info), achieved PFLOP/s and TB/s, and the step's
roofline floor max(FLOP / 2.5 PF, bytes / 6.3 TB/s) with the fraction reached.

  python tools/det_roofline.py [--cfg yolov4-tiny-aider-416] [--img 608] [--batch 64]"""
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
from rtdm.synth import inline_acff, load_calibration, synth_acff_params, synth_darknet_weights, synth_frames  # noqa: E402

PEAK_F, PEAK_B = 2.5e15, 6.3e12
ap = argparse.ArgumentParser()
ap.add_argument("--cfg", default="yolov4-tiny-aider-416")
ap.add_argument("--img", type=int, default=608)
ap.add_argument("--batch", type=int, default=64)
ap.add_argument("--iters", type=int, default=20)
ap.add_argument("--bm", type=int, default=0, help="force conv_pipe tile rows (256/128/64); 0 = cost model")
args = ap.parse_args()
L.check(L.lib().rtdm_set_tuning(b"conv_pipe_bm", args.bm))
L.check(L.lib().rtdm_set_tuning(b"conv_pipe_korder", int(os.environ.get("KORDER", "1"))))
for kv in filter(None, os.environ.get("TUNE", "").split(",")):  # TUNE="key=v,key=v" (diagnostics)
    k, v = kv.split("=")
    L.check(L.lib().rtdm_set_tuning(k.encode(), int(v)))
text = open(os.path.join(ROOT, "real-time-disaster-management_amd", "rtdm", "cfg", args.cfg + ".cfg")).read()
d = Darknet(text, (args.img, args.img))
cal = load_calibration(args.cfg)
d.load_weight_stream(inline_acff(text, synth_darknet_weights(text, calib=cal), synth_acff_params(text, calib=cal)))
d.half()
frames = torch.from_numpy(synth_frames(args.batch, args.img, args.img)).cuda()
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
wall = statistics.median(walls)
print(f"forward {wall:.4f} ms  ({args.batch / wall * 1e3:.0f} frames/s)")
print(f"{'layer':>5} {'step':34s} {'ms':>7} {'GFLOP':>8} {'MB':>7} {'PF/s':>6} {'TB/s':>6} {'floor':>7} {'frac':>5}")
tot = tfl = 0.0
for i in range(ns):
    nm = ctypes.create_string_buffer(128)
    layer, flop, byt = ctypes.c_int(), ctypes.c_double(), ctypes.c_double()
    L.check(L.lib().rtdm_detector_step_info(h, i, nm, 128, ctypes.byref(layer), ctypes.byref(flop), ctypes.byref(byt)))
    t = ms[i] / max(1, calls.value) * 1e-3
    f, b = flop.value * args.batch, byt.value * args.batch
    floor = max(f / PEAK_F, b / PEAK_B)
    tot += t
    tfl += floor
    print(f"{layer.value:5d} {nm.value.decode()[:34]:34s} {t * 1e3:7.4f} {f / 1e9:8.1f} {b / 1e6:7.1f} "
          f"{f / t / 1e15 if t else 0:6.3f} {b / t / 1e12 if t else 0:6.2f} {floor * 1e3:7.4f} {floor / t if t else 0:5.2f}")
print(f"sum of steps {tot * 1e3:.4f} ms, sum of floors {tfl * 1e3:.4f} ms ({tfl / tot:.2f})")
