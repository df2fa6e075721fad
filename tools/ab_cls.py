#!/usr/bin/env python3
"""Interleaved in-process A/B of a classifier tuning knob (default: acff_persist).

  python tools/ab_cls.py [--model ernet] [--key acff_persist] [--values 0,1] [--rounds 6] [--iters 20]

Times rtdm_classify on b64 synthetic 608x608 uint8 frames (CLI transform + model,
fp16) with hipEvents, per value, interleaved; prints median/min ms and the
max-abs logit difference between values."""
import argparse
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "real-time-disaster-management_amd"))

from rtdm import _lib as L  # noqa: E402
from rtdm.classifier import build_model  # noqa: E402
from rtdm.synth import synth_classifier_state_dict, synth_frames  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--model", default="ernet")
ap.add_argument("--key", default="acff_persist")
ap.add_argument("--values", default="0,1")
ap.add_argument("--rounds", type=int, default=6)
ap.add_argument("--iters", type=int, default=20)
ap.add_argument("--batch", type=int, default=64)
args = ap.parse_args()
vals = [int(v) for v in args.values.split(",")]
m = build_model(args.model)
m.load_state_dict(synth_classifier_state_dict(args.model))
m.half()
frames = torch.from_numpy(synth_frames(args.batch, 608, 608)).cuda()
outs, times = {}, {v: [] for v in vals}
for v in vals:
    m.set_tuning(args.key, v)  # the handle's own knob (tuning is copied per handle)
    for _ in range(3):
        p = m.classify_frames(frames) if hasattr(m, "classify_frames") else None
    torch.cuda.synchronize()
for r in range(args.rounds):
    for v in vals:
        m.set_tuning(args.key, v)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(args.iters):
            out = m.classify_frames(frames)
        e.record()
        torch.cuda.synchronize()
        times[v].append(s.elapsed_time(e) / args.iters)
        outs[v] = [t.clone() for t in out] if isinstance(out, (tuple, list)) else out.clone()
for v in vals:
    print(f"{args.key}={v}: median {statistics.median(times[v]):.4f} ms  min {min(times[v]):.4f} ms per b{args.batch}")
base = outs[vals[0]]
for v in vals[1:]:
    a = base[0] if isinstance(base, list) else base
    b = outs[v][0] if isinstance(outs[v], list) else outs[v]
    print(f"{args.key}={v} vs {vals[0]}: max |diff| {float((a - b).abs().max()):.3e}, "
          f"argmax agree {float((a.argmax(1) == b.argmax(1)).float().mean()):.4f}")
