"""Run the detector of record alone (for rocprofv3 kernel traces / PMC passes).
python tools/run_detector.py [--cfg yolov4-tiny-aider-416] [--img 608] [--batch 64] [--iters 5]"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "real-time-disaster-management_amd"))

from rtdm.darknet import Darknet  # noqa: E402
from rtdm.synth import inline_acff, load_calibration, synth_acff_params, synth_darknet_weights, synth_frames  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--cfg", default="yolov4-tiny-aider-416")
ap.add_argument("--img", type=int, default=608)
ap.add_argument("--batch", type=int, default=64)
ap.add_argument("--iters", type=int, default=5)
ap.add_argument("--dtype", default="f16")
args = ap.parse_args()
from rtdm import _lib as L  # noqa: E402
L.check(L.lib().rtdm_set_tuning(b"conv_pipe_korder", int(os.environ.get("KORDER", "1"))))
for kv in filter(None, os.environ.get("RTDM_TUNE", "").split(",")):  # "key=v,key=v"
    k, v = kv.split("=")
    L.check(L.lib().rtdm_set_tuning(k.encode(), int(v)))
text = open(os.path.join(ROOT, "real-time-disaster-management_amd", "rtdm", "cfg", args.cfg + ".cfg")).read()
det = Darknet(text, (args.img, args.img))
cal = load_calibration(args.cfg, "cond")
det.load_weight_stream(inline_acff(text, synth_darknet_weights(text, calib=cal, preset="cond"),
                                   synth_acff_params(text, calib=cal, preset="cond")))
if args.dtype == "f16":
    det.half()
frames = torch.from_numpy(synth_frames(args.batch, args.img, args.img)).cuda()
for _ in range(args.iters):
    io, _ = det(frames)
torch.cuda.synchronize()
print("ok", io.shape, float(io[..., 4].mean()))
