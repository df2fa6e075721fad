#!/usr/bin/env python3
"""Per-layer error of the YOLO-ACFF detector (yolov3-acffx) against the oracle: relative
max error of every materialised layer output, fp32 and fp16 (diagnostic for the deep,
chaotic synthetic-weight network)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "tests"), os.path.join(ROOT, "real-time-disaster-management_amd"), ROOT):
    sys.path.insert(0, p)
from test_gpu_parity import _darknet  # noqa: E402
from oracle.darknet import DarknetRef  # noqa: E402
from rtdm.synth import load_calibration, synth_acff_params, synth_darknet_weights, synth_frames  # noqa: E402

size = int(sys.argv[1]) if len(sys.argv) > 1 else 160
for half in (False, True):
    m, text, stream = _darknet("yolov3-acffx", size, half)
    frames = synth_frames(2, size, size, seed=3)
    m(torch.from_numpy(frames).cuda())
    cal = load_calibration("yolov3-acffx")
    ref = DarknetRef(text, synth_darknet_weights(text, calib=cal), synth_acff_params(text, calib=cal))
    _, outs = ref.forward(torch.from_numpy(frames).permute(0, 3, 1, 2).float() / 255.0, keep_layers=True)
    row = []
    for i, o in enumerate(outs):
        if not isinstance(o, torch.Tensor):
            continue
        try:
            got = m.layer_output(i, 2).cpu()
        except RuntimeError:
            continue
        rel = (got - o).abs().max().item() / (o.abs().max().item() + 1e-6)
        row.append(f"L{i}:{ref.mdefs[i]['type'][:4]}:{rel:.1e}")
    print("half" if half else "fp32", " ".join(row), flush=True)
