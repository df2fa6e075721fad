#!/usr/bin/env python3
"""NMS one launch per image (nms_split 0) against the split form (nms_split 1: prep, bitmask
over (word, row block, image) blocks, scan), on the b64 (or --batch) detector io of
yolov4-tiny-aider-416@608 (synthetic calibrated weights): hipEvent time per rtdm_nms call,
interleaved, median over --iters, and the survivors of both forms compared.

  python tools/nms_split_ab.py [--batch 64] [--iters 50]"""
import argparse
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "real-time-disaster-management_amd"))

from rtdm import _lib as L  # noqa: E402
from rtdm import nms as N  # noqa: E402
from rtdm.darknet import Darknet  # noqa: E402
from rtdm.synth import load_calibration, synth_darknet_weights, synth_frames  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=64)
ap.add_argument("--iters", type=int, default=50)
ap.add_argument("--conf", type=float, default=0.3)
ap.add_argument("--iou", type=float, default=0.4)
args = ap.parse_args()
cfg = "yolov4-tiny-aider-416"
text = open(os.path.join(ROOT, "real-time-disaster-management_amd", "rtdm", "cfg", cfg + ".cfg")).read()
det = Darknet(text, (608, 608))
det.load_weight_stream(synth_darknet_weights(text, calib=load_calibration(cfg)))
det.half()
frames = torch.from_numpy(synth_frames(args.batch, 608, 608)).cuda()
io, _ = det(frames)
torch.cuda.synchronize()
times = {0: [], 1: []}
outs = {}
for it in range(args.iters + 3):
    for v in (0, 1):
        L.check(L.lib().rtdm_set_tuning(b"nms_split", v))
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        d, i, c = N.nms_batched(io, args.conf, args.iou)
        e1.record()
        torch.cuda.synchronize()
        if it >= 3:
            times[v].append(e0.elapsed_time(e1) * 1000.0)
        outs[v] = (d.cpu(), i.cpu(), c.cpu())
L.check(L.lib().rtdm_set_tuning(b"nms_split", 1))
c0, c1 = outs[0][2], outs[1][2]
same = torch.equal(c0, c1)
for b in range(args.batch):
    k = min(int(c0[b]), 300)
    same = same and torch.equal(outs[0][0][b, :k], outs[1][0][b, :k]) and torch.equal(outs[0][1][b, :k], outs[1][1][b, :k])
print(f"b{args.batch}: nms_split 0 {np.median(times[0]):.2f} us, nms_split 1 {np.median(times[1]):.2f} us "
      f"(median of {args.iters}, event-timed rtdm_nms calls incl. nms_cand_kernel); survivors identical: {same}")
assert same
