import os, sys, torch, numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "real-time-disaster-management_amd"))
from rtdm.darknet import Darknet
from rtdm.synth import BASE_SEED, load_calibration, synth_darknet_weights, synth_frames
cfg = "yolov4-tiny-aider-416"
text = open(os.path.join(ROOT, "real-time-disaster-management_amd", "rtdm", "cfg", cfg + ".cfg")).read()
stream = synth_darknet_weights(text, calib=load_calibration(cfg))
fr = torch.from_numpy(synth_frames(4, 608, 608, seed=BASE_SEED + 700)).cuda()
a = Darknet(text, (608, 608)); a.load_weight_stream(stream); a.half()
b = Darknet(text, (608, 608)); b.load_weight_stream(stream); b.int8(fr)
ioa, _ = a(fr); iob, _ = b(fr)
print(b.describe())
for layer in (6, 8, 10, 12, 13, 14, 21):
    try:
        la = a.layer_output(layer, 4); lb = b.layer_output(layer, 4)
        d = (la - lb).abs()
        print(layer, tuple(la.shape), "maxabs", float(la.abs().max()), "maxdiff", float(d.max()), "meandiff", float(d.mean()),
              "rel", float(d.mean() / la.abs().mean()))
    except Exception as e:
        print(layer, "n/a", str(e)[:80])
print("io obj maxdiff", float((ioa[..., 4] - iob[..., 4]).abs().max()))
