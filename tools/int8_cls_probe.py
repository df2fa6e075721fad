#!/usr/bin/env python3
"""CPU: top-1 agreement of the classifier int8 scheme model (oracle/int8.py, the quantisation
RTDM_I8 handles apply) with fp32, per subset of int8 ACFF blocks and per activation headroom,
on test_gpu_int8.py's frames (160 synthetic + the reference's golden crops).
  python tools/int8_cls_probe.py [model]"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "real-time-disaster-management_amd")]
from conftest import load_npz  # noqa: E402
from oracle import classifier as OC, int8 as OQ, preprocess as P  # noqa: E402
from rtdm.synth import BASE_SEED, synth_frames  # noqa: E402

torch.set_num_threads(8)
name = sys.argv[1] if len(sys.argv) > 1 else "squeeze-ernet"
s = 240 if name == "ernet" else 140
z = np.load(os.path.join(ROOT, "tests", "golden", "classifier_weights.npz"), allow_pickle=False)
sd = {k.split("/", 1)[1]: torch.from_numpy(z[k]) for k in z.files if k.split("/", 1)[0] == name}
g = load_npz("cls_golden.npz")
frames = synth_frames(160, 300, 300, seed=BASE_SEED + 900)
cal = synth_frames(64, 300, 300, seed=BASE_SEED + 5000)
xg = torch.from_numpy(np.stack([P.to_tensor_normalize(c) for c in g[f"{name}/crops"]]))
x = torch.cat([torch.from_numpy(np.stack([P.cli_transform(f, s) for f in frames])), xg])
xc = torch.from_numpy(np.stack([P.cli_transform(f, s) for f in cal]))
ref = OC.forward(name, sd, x)[0].numpy()
blocks_all = {"squeeze-ernet": ("acff1", "acff2", "acff4"), "squeeze-redconv": ("acff4",),
              "ernet": ("acff1", "acff2", "acff3", "acff4", "acff5", "acff6")}[name]
subsets = [blocks_all] + [(b,) for b in blocks_all]
for blocks in subsets:
    amax = OQ.cls_calibrate(name, sd, xc, set(blocks))
    emu = OC.forward(name, sd, x, OQ.cls_int8_hook(amax))[0].numpy()
    print(name, blocks, "top-1 agreement", round(float((emu.argmax(1) == ref.argmax(1)).mean()), 4))
amax = OQ.cls_calibrate(name, sd, xc, set(blocks_all))
for hr in (0.75, 1.0, 1.5, 2.0):
    emu = OC.forward(name, sd, x, OQ.int8_hook(amax, hr))[0].numpy()
    print(name, "all blocks, headroom", hr, "top-1 agreement", round(float((emu.argmax(1) == ref.argmax(1)).mean()), 4))
