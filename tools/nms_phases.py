#!/usr/bin/env python3
"""Per-phase timing of nms_kernel from the s_memrealtime stamps it leaves in each
image's workspace slice (100 MHz clock).

  python tools/nms_phases.py [--batch 64]

Phases: 0->1 gather candidate segments, 1->2 pad + bitonic sort, 2->3 boxes/areas,
3->4 IoU bitmask, 4->5 greedy scan, 5->6 output rows."""
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
L.check(L.lib().rtdm_set_tuning(b"nms_variant", 4))  # diagnostic build path: phase stamps on
for _ in range(3):
    d, i, c = N.nms_batched(io, args.conf, args.iou)
torch.cuda.synchronize()
n, a, no = io.shape
nc = no - 5
per = int(L.lib().rtdm_nms_workspace_size(1, a, nc))
cap = 64
while cap < a * max(1, nc):
    cap <<= 1
off = cap * 32 + (cap // 32 + 1) * 4
ws = N._ws_cache[(str(io.device),)].cpu().numpy()
st = np.stack([ws[b * per + off: b * per + off + 56].view(np.uint64) for b in range(n)]).astype(np.int64)
dt = np.diff(st, axis=1) * 10 / 1000.0  # us
names = ["gather", "sort", "boxes", "mask", "scan", "output"]
cnt = c.cpu().numpy()
x = io.cpu().numpy()
ok = (x[..., 4] > args.conf) & (x[..., 2] > 2) & (x[..., 3] > 2) & (x[..., 2] < 4096) & (x[..., 3] < 4096)
ncand = ((x[..., 5:] * x[..., 4:5] > args.conf) & ok[..., None]).sum((1, 2))
print(f"candidates per image: mean {ncand.mean():.1f} max {ncand.max()}; kept: mean {cnt.mean():.1f} max {cnt.max()}")
print("phase      mean_us   max_us")
for k, nm in enumerate(names):
    print(f"{nm:8s} {dt[:, k].mean():9.2f} {dt[:, k].max():8.2f}")
tot = (st[:, 6] - st[:, 0]) * 10 / 1000.0
print(f"{'total':8s} {tot.mean():9.2f} {tot.max():8.2f}   (block span; kernel = max over images + launch)")
