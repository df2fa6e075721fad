"""Golden vectors from the REFERENCE code (build container only; commits small .npz files).

  classifier_weights.npz  the reference's trained state dicts (weights/*-state_dict.pt,
                          loaded with weights_only=True), keys "<model>/<param>"
  cls_golden.npz          per model: uint8 crops (after Pillow resize + center crop)
                          of bundled AIDER images and synthetic frames, the
                          reference nn.Module's fc logits (forward hook), softmax
                          probs and argmax
  det_golden.npz          per (cfg, size): synthetic frames' checksums, reference
                          Darknet io (full at small sizes, strided rows + column sums
                          at full sizes) on rtdm.synth weights loaded through the
                          reference load_darknet_weights, and the reference
                          non_max_suppression survivors (torchvision nms stubbed by
                          the oracle restatement — parity unpinned at that boundary)
  shapes.json             model_summary/*.txt totals (params, mult-adds)
Run: python tests/golden/make_golden.py
"""
from __future__ import annotations

import hashlib
import json
import os
import re
import sys
import tempfile

import numpy as np
import torch
from PIL import Image

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "real-time-disaster-management_amd"))
sys.path.insert(0, ROOT)
sys.path.insert(0, HERE)

from oracle import nms as onms  # noqa: E402
from oracle import preprocess as opre  # noqa: E402
from rtdm import synth  # noqa: E402
from refimport import CLS_DIR, DET_DIR, import_classifiers, import_darknet  # noqa: E402

WEIGHTS = {"squeeze-ernet": "squeeze-ernet-state_dict.pt", "squeeze-redconv": "squeeze-redconv-state_dict.pt",
           "ernet": "ernet-state_dict.pt"}
IMAGES = ["yolov3/data/custom/test/images/fire_image0232.jpg",
          "yolov3/data/custom/test/images/flood_image0205.jpg",
          "yolov3/data/custom/test/images/collapsed_building_image0078.jpg",
          "yolov3/data/custom/test/images/traffic_incident_image0393.jpg"]
SIZES = {"squeeze-ernet": 140, "squeeze-redconv": 140, "ernet": 240}
DET_CASES = [  # (cfg, size, n_frames, full_io)
    ("yolov4-tiny-aider-416", 256, 2, True),
    ("yolov4-tiny-aider-416", 608, 1, False),
    ("yolov3-aider-416", 416, 1, False),
    ("yolov3-spp-aider", 608, 1, False),
    ("yolov3-tiny-aider-416", 416, 1, False),
    ("yolov4-tiny-swish", 416, 1, False),
    ("yolov4-tiny-3l-512x512", 512, 1, False),
    ("yolov3-acffx", 416, 1, False),
]
NMS_SETTINGS = [(0.3, 0.4), (0.01, 0.6)]
IO_STRIDE = 53


def sha(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def classifier_goldens():
    classes = import_classifiers()
    wz, gz = {}, {}
    srcs = []
    for rel in IMAGES:
        img = np.asarray(Image.open(os.path.join(REF_VL, rel)).convert("RGB"))
        srcs.append(img)
    srcs += list(synth.synth_frames(2, 224, 224, seed=synth.BASE_SEED + 500))
    gz["n_real"] = np.array(len(IMAGES))
    for name, cls in classes.items():
        sd = torch.load(os.path.join(CLS_DIR, "weights", WEIGHTS[name]), map_location="cpu", weights_only=True)
        for k, v in sd.items():
            if not k.endswith("num_batches_tracked"):
                wz[f"{name}/{k}"] = v.float().numpy()
        model = cls()
        model.load_state_dict(sd)
        model.eval()
        s = SIZES[name]
        crops = []
        for img in srcs:
            rs = opre.pil_resize_shorter(img, int(s * 1.14))
            crops.append(opre.center_crop(rs, s))
        crops = np.stack(crops).astype(np.uint8)
        x = torch.from_numpy(np.stack([opre.to_tensor_normalize(c) for c in crops]))
        feats = {}
        model.fc.register_forward_hook(lambda m, i, o: feats.__setitem__("logits", o.detach()))
        with torch.no_grad():
            probs = model(x)
        logits = feats["logits"].numpy()
        srt = np.sort(logits, 1)
        gz[f"{name}/crops"] = crops
        gz[f"{name}/logits"] = logits
        gz[f"{name}/probs"] = probs.numpy()
        gz[f"{name}/argmax"] = logits.argmax(1)
        gz[f"{name}/top2gap"] = srt[:, -1] - srt[:, -2]
        # random tensor inputs (no transform): exercises arbitrary activations
        g = torch.Generator().manual_seed(1234)
        xr = torch.randn(3, 3, s, s, generator=g)
        with torch.no_grad():
            pr = model(xr)
        gz[f"{name}/rand_x_sha"] = np.array(sha(xr.numpy()))
        gz[f"{name}/rand_logits"] = feats["logits"].numpy()
        gz[f"{name}/rand_probs"] = pr.numpy()
        print(name, "argmax", gz[f"{name}/argmax"], "gap min", float(gz[f"{name}/top2gap"].min()))
    # one raw source image pair for the on-device resize check (small real photo)
    gz["src0"] = np.ascontiguousarray(srcs[0][:200, :260])
    np.savez_compressed(os.path.join(HERE, "classifier_weights.npz"), **wz)
    np.savez_compressed(os.path.join(HERE, "cls_golden.npz"), **gz)


def det_goldens(preset: str = "he"):
    """preset "he" -> det_golden.npz (the mean-field weights, kept as the stress case);
    "cond" -> det_golden_cond.npz (the well-conditioned set the SURVEY §8d fp16 / int8 bars
    are asserted on; 2 frames per case)."""
    def nms_stub(boxes, scores, iou):
        keep = onms.nms_kernel(boxes.numpy(), scores.numpy(), float(iou))
        return torch.from_numpy(keep)

    models, utils = import_darknet(nms_stub)
    out = {}
    for (cfg, size, nf, full) in DET_CASES:
        if preset == "cond":
            nf = max(nf, 2)
        key = f"{cfg}@{size}"
        text = open(os.path.join(DET_DIR, "cfg", cfg + ".cfg")).read()
        cal = synth.load_calibration(cfg, preset)
        stream = synth.synth_darknet_weights(text, calib=cal, preset=preset)
        model = models.Darknet(os.path.join(DET_DIR, "cfg", cfg + ".cfg"), (size, size))
        with tempfile.NamedTemporaryFile(suffix=".weights") as f:
            synth.write_darknet_weights(f.name, stream)
            models.load_darknet_weights(model, f.name)
        acff = synth.synth_acff_params(text, calib=cal, preset=preset)
        for i, p in acff.items():  # [acff] blocks: state-dict parameters (not in .weights)
            sd = {k: torch.from_numpy(v) for k, v in p.items()}
            sd["batch_norm.num_batches_tracked"] = torch.tensor(0)
            model.module_list[i][0].load_state_dict(sd)
        model.eval()
        frames = synth.synth_frames(nf, size, size, seed=synth.BASE_SEED + 700)
        x = torch.from_numpy(frames).permute(0, 3, 1, 2).float() / 255.0
        with torch.no_grad():
            io, _ = model(x)
        io = io.numpy()
        out[f"{key}/frames_sha"] = np.array(sha(frames))
        out[f"{key}/stream_sha"] = np.array(sha(stream))
        out[f"{key}/stream_n"] = np.array(stream.size)
        if full:
            out[f"{key}/frames"] = frames
            out[f"{key}/io"] = io
        out[f"{key}/io_rows"] = io[:, ::IO_STRIDE]
        out[f"{key}/io_colsum"] = io.astype(np.float64).sum(1)
        out[f"{key}/io_shape"] = np.array(io.shape)
        for (conf, iou) in NMS_SETTINGS:
            if conf < 0.1 and not full:
                continue
            ties, harmful = onms.score_ties(io, conf, iou)
            assert harmful == 0, f"{key}: {harmful} overlapping tied scores at conf {conf}"
            out[f"{key}/nms{conf}_{iou}/ties"] = np.array(ties)
            dets = utils.non_max_suppression(torch.from_numpy(io.copy()), conf, iou)
            _, idx = onms.non_max_suppression(io, conf, iou, return_index=True)
            for b, d in enumerate(dets):
                d = np.zeros((0, 6), np.float32) if d is None else d.numpy()
                out[f"{key}/nms{conf}_{iou}/{b}"] = d
                out[f"{key}/nms{conf}_{iou}/{b}/idx"] = np.zeros((0, 2), np.int64) if idx[b] is None else idx[b]
            print(key, "nms", conf, iou, [0 if d is None else len(d) for d in dets])
    np.savez_compressed(os.path.join(HERE, "det_golden.npz" if preset == "he" else "det_golden_cond.npz"), **out)


def shapes_golden():
    res = {}
    for name, fn in (("squeeze-ernet", "squeeze_ernet.txt"), ("squeeze-redconv", "squeeze_redconv.txt"),
                     ("ernet", "ernet.txt")):
        txt = open(os.path.join(CLS_DIR, "model_summary", fn)).read()
        params = int(re.search(r"Total params: ([\d,]+)", txt).group(1).replace(",", ""))
        madds = float(re.search(r"Total mult-adds \(M\): ([\d.]+)", txt).group(1))
        inp = [int(v) for v in re.search(r"\[-1, 3, (\d+), (\d+)\]", txt).groups()]
        res[name] = {"params": params, "mult_adds_M": madds, "input": inp}
    with open(os.path.join(HERE, "shapes.json"), "w") as f:
        json.dump(res, f, indent=1)


REF_VL = os.path.join(os.path.dirname(CLS_DIR), "victim_localization")

if __name__ == "__main__":
    torch.set_num_threads(8)
    only = sys.argv[1:]  # e.g. "det" to regenerate only det_golden.npz
    if not only or "shapes" in only:
        shapes_golden()
    if not only or "cls" in only:
        classifier_goldens()
    if not only or "det" in only:
        det_goldens()
    if not only or "detcond" in only:
        det_goldens("cond")
