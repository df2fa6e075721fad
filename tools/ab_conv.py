#!/usr/bin/env python3
"""Interleaved in-process A/B of conv kernel selections on the detector of record.

  python tools/ab_conv.py [--key conv_pipe] [--values 0,1] [--rounds 6] [--iters 10]

For each round and each value v: rtdm_set_tuning(key, v), then `iters` timed
detector forwards (b64 yolov4-tiny@608 fp16) with per-step hipEvent timing.
Prints the per-layer median ms per value and the io max-abs difference between
values (same weights, same frames)."""
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
from rtdm.synth import load_calibration, synth_darknet_weights, synth_frames  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--cfg", default="yolov4-tiny-aider-416")
ap.add_argument("--img", type=int, default=608)
ap.add_argument("--batch", type=int, default=64)
ap.add_argument("--key", default="conv_pipe")
ap.add_argument("--values", default="0,1")
ap.add_argument("--rounds", type=int, default=6)
ap.add_argument("--iters", type=int, default=10)
args = ap.parse_args()
vals = [int(v) for v in args.values.split(",")]
lib = L.lib()

text = open(os.path.join(ROOT, "real-time-disaster-management_amd", "rtdm", "cfg", args.cfg + ".cfg")).read()
det = Darknet(text, (args.img, args.img))
det.load_weight_stream(synth_darknet_weights(text, calib=load_calibration(args.cfg)))
det.half()
frames = torch.from_numpy(synth_frames(args.batch, args.img, args.img)).cuda()
h = det.handle(args.batch)
ns = lib.rtdm_detector_num_steps(h)
names = []
for i in range(ns):
    nm = ctypes.create_string_buffer(128)
    layer, flop, byt = ctypes.c_int(), ctypes.c_double(), ctypes.c_double()
    L.check(lib.rtdm_detector_step_info(h, i, nm, 128, ctypes.byref(layer), ctypes.byref(flop), ctypes.byref(byt)))
    names.append((layer.value, flop.value * args.batch))

ios = {}
for v in vals:
    L.check(lib.rtdm_set_tuning(args.key.encode(), v))
    for _ in range(3):
        io, _ = det(frames)
    torch.cuda.synchronize()
    ios[v] = io.clone()
res = {v: [[] for _ in range(ns)] for v in vals}
tot = {v: [] for v in vals}
for r in range(args.rounds):
    for v in vals:
        L.check(lib.rtdm_set_tuning(args.key.encode(), v))
        det(frames)
        torch.cuda.synchronize()
        L.check(lib.rtdm_detector_enable_timing(h, args.iters))
        for _ in range(args.iters):
            det(frames)
        torch.cuda.synchronize()
        ms = (ctypes.c_double * ns)()
        calls = ctypes.c_int()
        L.check(lib.rtdm_detector_read_timing(h, ms, ctypes.byref(calls)))
        L.check(lib.rtdm_detector_enable_timing(h, 0))
        c = max(1, calls.value)
        for i in range(ns):
            res[v][i].append(ms[i] / c)
        tot[v].append(sum(ms) / c)
print(f"{'layer':>6s} {'GFLOP':>8s} " + " ".join(f"{args.key}={v:<3d} ms  TF/s " for v in vals))
for i in range(ns):
    layer, flop = names[i]
    cells = []
    for v in vals:
        m = statistics.median(res[v][i])
        cells.append(f"{m:9.4f} {flop / m / 1e9 if m > 0 else 0:7.1f}")
    print(f"{layer:6d} {flop / 1e9:8.2f} " + "  ".join(cells))
print("total  " + "  ".join(f"{args.key}={v}: {statistics.median(tot[v]):.4f} ms (min {min(tot[v]):.4f})" for v in vals))
base = ios[vals[0]]
for v in vals[1:]:
    d = (ios[v] - base).abs()
    print(f"io diff {args.key}={v} vs {vals[0]}: max {float(d.max()):.3e}, mean {float(d.mean()):.3e}, "
          f"bit-identical {bool(torch.equal(ios[v], base))}")
