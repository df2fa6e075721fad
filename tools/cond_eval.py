#!/usr/bin/env python3
"""Evaluate a synthetic detector weight set against SURVEY §8d's fp16 / int8 bars on the
CPU oracle (build container: calibrates through the reference Darknet, tests/golden/
make_synth.py).  Reports, for the fp16-storage model and the int8 scheme model against
fp32: max |dxy|, |dwh| (px), |dp| over all io rows, NMS survivors equal outside the 1e-3
band (oracle.nms.survivors_equal_outside_band), and the int8 detection match rate.

  python tools/cond_eval.py --cfg yolov3-aider-416 --size 416 --frames 4 [--preset cond]
       [--rank 16 --iso 0.05 --lp 0.85 --gamma-res 0.5 --wh 0.25 --obj 2 --cls 2]
"""
import argparse
import copy
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "real-time-disaster-management_amd"), os.path.join(ROOT, "tests", "golden")]

from oracle import int8 as OI  # noqa: E402
from oracle import nms as ON  # noqa: E402
from oracle.darknet import DarknetRef  # noqa: E402
from rtdm import synth  # noqa: E402


def iou(a, b):
    x1 = np.maximum(a[0], b[:, 0]); y1 = np.maximum(a[1], b[:, 1])
    x2 = np.minimum(a[2], b[:, 2]); y2 = np.minimum(a[3], b[:, 3])
    inter = np.clip(x2 - x1, 0, None) * np.clip(y2 - y1, 0, None)
    return inter / ((a[2] - a[0]) * (a[3] - a[1]) + (b[:, 2] - b[:, 0]) * (b[:, 3] - b[:, 1]) - inter)


def match(ref_io, io, conf=0.3, iou_thr=0.4, band=0.01):
    ref = ON.non_max_suppression(ref_io, conf, iou_thr)
    got = ON.non_max_suppression(io, conf, iou_thr)
    m = t = 0
    for b in range(len(ref)):
        r = np.zeros((0, 6), np.float32) if ref[b] is None else ref[b]
        g = np.zeros((0, 6), np.float32) if got[b] is None else got[b]
        r = r[r[:, 4] > conf + band]
        t += len(r)
        for row in r:
            same = g[g[:, 5] == row[5]]
            if len(same) and iou(row[:4], same[:, :4]).max() >= 0.9:
                m += 1
    return m, t


def stats(io32, io):
    d = np.abs(io - io32)
    return d[..., :2].max(), d[..., 2:4].max(), d[..., 4:].max()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cfg", default="yolov3-aider-416")
    ap.add_argument("--size", type=int, default=416)
    ap.add_argument("--frames", type=int, default=4)
    ap.add_argument("--preset", default="cond")
    ap.add_argument("--rank", type=int)
    ap.add_argument("--iso", type=float)
    ap.add_argument("--lp", type=float)
    ap.add_argument("--gamma-res", type=float)
    ap.add_argument("--xy", type=float)
    ap.add_argument("--wh", type=float)
    ap.add_argument("--obj", type=float)
    ap.add_argument("--cls", type=float)
    ap.add_argument("--no-int8", action="store_true")
    ap.add_argument("--stem-hp", type=float)
    ap.add_argument("--ncal", type=int, default=16)
    ap.add_argument("--headroom", type=float, default=2.0)
    args = ap.parse_args()
    torch.set_num_threads(8)
    import make_synth
    cond = make_synth.cond_for(args.cfg)
    for k in ("rank", "iso", "lp", "gamma_res"):
        if getattr(args, k) is not None:
            cond[k] = getattr(args, k)
    if args.stem_hp is not None:
        cond["stem_hp"] = args.stem_hp
    for k in ("xy", "wh", "obj", "cls"):
        if getattr(args, k) is not None:
            cond["head_std"][k] = getattr(args, k)
    t0 = time.time()
    calib = make_synth.calibrate(args.cfg, preset=args.preset, cond=cond, write=False)
    text = open(os.path.join(ROOT, "real-time-disaster-management_amd", "rtdm", "cfg", args.cfg + ".cfg")).read()
    stream = synth.synth_darknet_weights(text, calib=calib, preset=args.preset, cond=cond)
    acff = synth.synth_acff_params(text, calib=calib, preset=args.preset, cond=cond)
    ref = DarknetRef(text, stream, acff)
    x = torch.from_numpy(synth.synth_frames(args.frames, args.size, args.size, seed=synth.BASE_SEED + 700)
                         ).permute(0, 3, 1, 2).float() / 255
    io32 = ref.forward(x).numpy()
    io16 = ref.forward(x, f16_storage=True).numpy()
    t1 = time.time()
    print(f"{args.cfg}@{args.size} {args.preset} {cond}  ({t1 - t0:.0f}s)")
    nsurv = [0 if d is None else len(d) for d in ON.non_max_suppression(io32, 0.3, 0.4)]
    print("  survivors/frame", nsurv, " candidates obj>0.3/frame", (io32[..., 4] > 0.3).sum(1).tolist())
    print("  fp16-storage  dxy %.4f  dwh %.4f  dp %.2e" % stats(io32, io16))
    nr, ng, ne, bad = ON.survivors_equal_outside_band(io32, io16, 0.3, 0.4)
    print(f"  fp16 survivors ref {nr} got {ng} excluded-diff {ne} unexplained {len(bad)} {bad[:5]}")
    if not args.no_int8:
        xc = torch.from_numpy(synth.synth_frames(args.ncal, args.size, args.size, seed=synth.BASE_SEED + 4321)
                              ).permute(0, 3, 1, 2).float() / 255
        amax = OI.calibrate(ref, xc)
        io8 = ref.forward(x, f16_storage=True, conv_hook=OI.int8_hook(amax, args.headroom)).numpy()
        m, t = match(io32, io8)
        print("  int8 model    dxy %.4f  dwh %.4f  dp %.2e" % stats(io32, io8), f" match {m}/{t} = {m / max(t, 1):.3f}")


if __name__ == "__main__":
    main()
