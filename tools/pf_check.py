#!/usr/bin/env python3
"""Diagnostic: detector io under conv_pipe tuning combinations (mode / window / prefetch /
tile rows) for one cfg, saved to gpurun_out/pf_<tag>.npz and compared in-process.
  python tools/pf_check.py CFG SIZE BATCH TAG"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "real-time-disaster-management_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from rtdm import _lib as L  # noqa: E402
from rtdm.synth import synth_frames  # noqa: E402
from test_gpu_pipeline import _detector  # noqa: E402

cfg, size, b, tag = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
x = torch.from_numpy(synth_frames(b, size, size, seed=23)).cuda()
combos = {"generic": dict(conv_pipe=11, conv_pipe_bm=256), "prod": dict(conv_pipe_bm=256),
          "nopf": dict(conv_pipe_bm=256, conv_pipe_pf=0), "nowin": dict(conv_pipe_bm=256, conv_pipe_win=0),
          "nowin_nopf": dict(conv_pipe_bm=256, conv_pipe_win=0, conv_pipe_pf=0)}
defaults = dict(conv_pipe=1, conv_pipe_bm=0, conv_pipe_pf=1, conv_pipe_win=1)
outs = {}
for name, kv in combos.items():
    try:
        for k, v in kv.items():
            L.check(L.lib().rtdm_set_tuning(k.encode(), v))
        m, _, _, _ = _detector(cfg, size)
        outs[name] = m(x)[0].cpu().numpy()
    except Exception as e:  # noqa: BLE001  (older libraries lack a knob)
        print(name, "skipped:", e)
    finally:
        for k, v in defaults.items():
            try:
                L.check(L.lib().rtdm_set_tuning(k.encode(), v))
            except Exception:  # noqa: BLE001
                pass
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
np.savez(os.path.join(ROOT, "gpurun_out", f"pf_{tag}.npz"), **outs)
for name, v in outs.items():
    print(tag, name, "max|d| vs generic:", float(np.abs(v - outs["generic"]).max()))

# first differing layer between prefetch on / off (production tiles)
if len(sys.argv) > 5:
    import ctypes
    lays = {}
    for v in (0, 1):
        L.check(L.lib().rtdm_set_tuning(b"conv_pipe_pf", v))
        m, _, _, _ = _detector(cfg, size)
        m(x)
        d = {}
        for li in range(200):
            try:
                d[li] = m.layer_output(li, b).cpu().numpy()
            except Exception:  # noqa: BLE001
                pass
        lays[v] = (m, d)
    L.check(L.lib().rtdm_set_tuning(b"conv_pipe_pf", 1))
    m, d1 = lays[1]
    h = m.handle(b)
    names = {}
    for i in range(L.lib().rtdm_detector_num_steps(h)):
        nm = ctypes.create_string_buffer(64)
        lay = ctypes.c_int()
        L.check(L.lib().rtdm_detector_step_info(h, i, nm, 64, ctypes.byref(lay), None, None))
        names.setdefault(lay.value, []).append(nm.value.decode())
    d0 = lays[0][1]
    for li in sorted(d1):
        if li in d0:
            dd = np.abs(d1[li] - d0[li])
            if dd.max() > 0:
                bad = np.argwhere(dd > 0)
                print("layer", li, names.get(li), "shape", d1[li].shape, "max|d|", float(dd.max()),
                      "n diff", len(bad), "first", bad[:4].tolist())
