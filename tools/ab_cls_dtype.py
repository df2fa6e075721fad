#!/usr/bin/env python3
"""Interleaved in-process A/B of the classifier's fp16 and int8 (RTDM_I8) handles.

  python tools/ab_cls_dtype.py [--model ernet] [--batches 8,64] [--rounds 6] [--iters 20]

Times rtdm_classify on synthetic 608x608 uint8 frames (CLI transform + model) with
hipEvents per dtype, interleaved; prints median/min ms and the int8-vs-fp16 top-1
agreement (int8 calibrated on 64 disjoint frames)."""
import argparse
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "real-time-disaster-management_amd"))

from rtdm.classifier import build_model  # noqa: E402
from rtdm.synth import BASE_SEED, synth_classifier_state_dict, synth_frames  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--model", default="ernet")
ap.add_argument("--batches", default="8,64")
ap.add_argument("--rounds", type=int, default=6)
ap.add_argument("--iters", type=int, default=20)
args = ap.parse_args()
sd = synth_classifier_state_dict(args.model)
cal = torch.from_numpy(synth_frames(64, 608, 608, seed=BASE_SEED + 5000)).cuda()
models = {}
for dt in ("f16", "i8"):
    m = build_model(args.model)
    m.load_state_dict(sd)
    m.half() if dt == "f16" else m.int8(cal)
    models[dt] = m
for b in [int(v) for v in args.batches.split(",")]:
    frames = torch.from_numpy(synth_frames(b, 608, 608)).cuda()
    times, outs = {k: [] for k in models}, {}
    for m in models.values():
        for _ in range(3):
            m.classify_frames(frames)
    torch.cuda.synchronize()
    for _ in range(args.rounds):
        for k, m in models.items():
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(args.iters):
                out = m.classify_frames(frames)
            e.record()
            torch.cuda.synchronize()
            times[k].append(s.elapsed_time(e) / args.iters)
            outs[k] = out.clone()
    for k in models:
        print(f"{args.model} b{b} {k}: median {statistics.median(times[k]):.4f} ms  min {min(times[k]):.4f} ms")
    agree = float((outs["f16"].argmax(1) == outs["i8"].argmax(1)).float().mean())
    print(f"{args.model} b{b} i8 vs f16 top-1 agreement {agree:.4f}")
