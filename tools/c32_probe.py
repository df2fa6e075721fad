#!/usr/bin/env python3
"""Per-layer comparison of yolov3-aider-416 outputs with a knob on / off (layer_output):
mismatch counts, max |d| and where the first mismatches sit (image, channel, y, x)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "real-time-disaster-management_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from rtdm import _lib as L  # noqa: E402
from rtdm.synth import BASE_SEED, synth_frames  # noqa: E402
from test_gpu_config3 import _model  # noqa: E402

key = sys.argv[1] if len(sys.argv) > 1 else "conv_c32"
b, img = 2, 416
x = torch.from_numpy(synth_frames(b, img, img, seed=BASE_SEED + 811)).cuda()
outs = {}
for v in (0, 1):
    L.check(L.lib().rtdm_set_tuning(key.encode(), v))
    m, _ = _model(img=img)
    m(x)
    torch.cuda.synchronize()
    outs[v] = {l: m.layer_output(l, b).cpu() for l in (0, 1, 2, 4)}
L.check(L.lib().rtdm_set_tuning(key.encode(), 1))
for l in (0, 1, 2, 4):
    a, c = outs[0][l], outs[1][l]
    d = (a - c).abs()
    bad = (d > 0).nonzero()
    print(f"L{l} shape {tuple(a.shape)} mismatches {bad.shape[0]} of {a.numel()} max {float(d.max()):.3e}")
    for row in bad[:12].tolist():
        n, ch, yy, xx = row
        print("   ", row, float(a[n, ch, yy, xx]), float(c[n, ch, yy, xx]))
    if bad.shape[0]:
        print("    channels hit:", sorted(set(bad[:, 1].tolist()))[:40])
        print("    x mod 16 hist:", torch.bincount(bad[:, 3] % 16, minlength=16).tolist())
        print("    y mod 16 hist:", torch.bincount(bad[:, 2] % 16, minlength=16).tolist())
