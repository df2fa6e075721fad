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
ap.add_argument("--set", default="", help="fixed tunings applied first: key=v,key=v")
args = ap.parse_args()
vals = [int(v) for v in args.values.split(",")]
lib = L.lib()
for kv in filter(None, args.set.split(",")):
    k, v = kv.split("=")
    L.check(lib.rtdm_set_tuning(k.encode(), int(v)))

text = open(os.path.join(ROOT, "real-time-disaster-management_amd", "rtdm", "cfg", args.cfg + ".cfg")).read()
stream = synth_darknet_weights(text, calib=load_calibration(args.cfg))
frames = torch.from_numpy(synth_frames(args.batch, args.img, args.img)).cuda()
# one model (handle) per value: plan-time knobs (fuse_head, two_streams) apply at handle creation
dets, hs = {}, {}
for v in vals:
    L.check(lib.rtdm_set_tuning(args.key.encode(), v))
    d = Darknet(text, (args.img, args.img))
    d.load_weight_stream(stream)
    d.half()
    dets[v], hs[v] = d, d.handle(args.batch)
names = {}
for v in vals:
    h = hs[v]
    rows = []
    for i in range(lib.rtdm_detector_num_steps(h)):
        nm = ctypes.create_string_buffer(128)
        layer, flop, byt = ctypes.c_int(), ctypes.c_double(), ctypes.c_double()
        L.check(lib.rtdm_detector_step_info(h, i, nm, 128, ctypes.byref(layer), ctypes.byref(flop), ctypes.byref(byt)))
        rows.append((layer.value, flop.value * args.batch))
    names[v] = rows

ios = {}
for v in vals:
    L.check(lib.rtdm_set_tuning(args.key.encode(), v))
    for _ in range(3):
        io, _ = dets[v](frames)
    torch.cuda.synchronize()
    ios[v] = io.clone()
res = {v: {} for v in vals}
wall = {v: [] for v in vals}
tot = {v: [] for v in vals}
for r in range(args.rounds):
    for v in vals:
        L.check(lib.rtdm_set_tuning(args.key.encode(), v))
        det, h = dets[v], hs[v]
        ns = len(names[v])
        det(frames)
        torch.cuda.synchronize()
        # wall clock of the forwards alone (no per-step events)
        s0, e0 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s0.record()
        for _ in range(args.iters):
            det(frames)
        e0.record()
        torch.cuda.synchronize()
        wall[v].append(s0.elapsed_time(e0) / args.iters)
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
            res[v].setdefault(names[v][i][0], []).append(ms[i] / c)
        tot[v].append(sum(ms) / c)
layers = sorted({l for v in vals for l, _ in names[v]})
flops = {l: f for v in vals for l, f in names[v]}
print(f"{'layer':>6s} {'GFLOP':>8s} " + " ".join(f"{args.key}={v:<3d} ms  TF/s " for v in vals))
for layer in layers:
    cells = []
    for v in vals:
        if layer in res[v]:
            m = statistics.median(res[v][layer])
            cells.append(f"{m:9.4f} {flops[layer] / m / 1e9 if m > 0 else 0:7.1f}")
        else:
            cells.append(f"{'-':>9s} {'':7s}")
    print(f"{layer:6d} {flops[layer] / 1e9:8.2f} " + "  ".join(cells))
print("sum of step times  " + "  ".join(f"{args.key}={v}: {statistics.median(tot[v]):.4f} ms" for v in vals))
print("forward wall       " + "  ".join(f"{args.key}={v}: {statistics.median(wall[v]):.4f} ms (min {min(wall[v]):.4f})"
                                        for v in vals))
base = ios[vals[0]]
for v in vals[1:]:
    d = (ios[v] - base).abs()
    print(f"io diff {args.key}={v} vs {vals[0]}: max {float(d.max()):.3e}, mean {float(d.mean()):.3e}, "
          f"bit-identical {bool(torch.equal(ios[v], base))}")
