"""Golden vectors for the mAP harness, from the REFERENCE code (build container only).

  map_golden.npz
    eval/<setting>/...   the reference yolov3 ``test.test`` (test.py:11-197) driven with
                         a stand-in model that returns seeded synthetic detector output
                         ``io`` and a dataloader of the 10 ODDER test-split label files
                         (data/custom/test/labels, real annotations) plus two synthetic
                         images (one unlabelled, one whose predictions all fall under
                         conf_thres).  Stored: io, targets, the reference NMS survivors per
                         image (captured at test.py:109), and the returned
                         (mp, mr, map, mf1) + maps.
    ap/<case>/...        utils.ap_per_class (utils.py:145-205) on seeded tp/conf/class
                         arrays, including a 10-column IoU case, a class with targets but
                         no predictions, predicted classes without targets, and an
                         empty prediction set.
    cap/<case>/...       utils.compute_ap (utils.py:208-234) on seeded curves.
The reference NMS calls torchvision.ops.boxes.nms, stubbed (as in make_golden.py) by the
oracle restatement: the harness is pinned downstream of NMS, NMS itself as before.
Run: python tests/golden/make_map_golden.py
"""
from __future__ import annotations

import glob
import os
import sys
import tempfile

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, HERE)

from oracle import nms as onms  # noqa: E402
from refimport import DET_DIR, _cwd, import_yolov3_test  # noqa: E402

IMG = 416
NC = 2
BATCH = 4
ROWS = 320
SETTINGS = {"default": (0.001, 0.6), "strict": (0.1, 0.45)}


def nms_stub(boxes, scores, iou):
    return torch.from_numpy(onms.nms_kernel(boxes.numpy(), scores.numpy(), float(iou)))


def odder_labels():
    files = sorted(glob.glob(os.path.join(DET_DIR, "data", "custom", "test", "labels", "*.txt")))
    out = []
    for f in files:
        rows = [ln.split() for ln in open(f).read().splitlines() if ln.strip()]
        out.append(np.array(rows, np.float32).reshape(-1, 5))
    return out


def synth_io(rng, labels, mode):
    """[ROWS, 5+NC] rows (x, y, w, h px, obj, cls probs): jittered copies of each
    target at several IoU levels, some with the wrong class, then clutter."""
    io = np.zeros((ROWS, 5 + NC), np.float32)
    k = 0
    for (c, x, y, w, h) in labels:
        for sig in (0.02, 0.06, 0.12, 0.25, 0.5):
            if k >= ROWS // 2:
                break
            jx, jy = rng.normal(0, sig, 2) * (w, h)
            sw, sh = np.exp(rng.normal(0, sig, 2))
            io[k, :4] = ((x + jx) * IMG, (y + jy) * IMG, w * sw * IMG, h * sh * IMG)
            io[k, 4] = rng.uniform(0.05, 1.0)
            cls = int(c) if rng.uniform() < 0.85 else 1 - int(c)
            io[k, 5:] = rng.uniform(0.0, 0.3, NC)
            io[k, 5 + cls] = rng.uniform(0.5, 1.0)
            k += 1
    n = ROWS - k
    io[k:, 0:2] = rng.uniform(0, IMG, (n, 2))
    io[k:, 2:4] = rng.uniform(8, IMG / 3, (n, 2))
    io[k:, 4] = 0.6 * rng.uniform(0, 1, n) ** 6
    io[k:, 5:] = rng.uniform(0, 1, (n, NC))
    if mode == "empty":
        io[:, 4] = rng.uniform(0, 1e-4, ROWS)
    return io


def eval_goldens(test_mod, out):
    labels = odder_labels()
    assert len(labels) == 10, len(labels)
    rng = np.random.default_rng(20240611)
    labels.insert(3, np.zeros((0, 5), np.float32))                      # unlabelled image
    labels.append(np.array([[0, 0.5, 0.5, 0.2, 0.3]], np.float32))      # all predictions below conf
    modes = ["normal"] * len(labels)
    modes[-1] = "empty"
    ios = np.stack([synth_io(rng, lab, m) for lab, m in zip(labels, modes)])
    targets = []
    for i, lab in enumerate(labels):
        t = np.zeros((len(lab), 6), np.float32)
        t[:, 0] = i % BATCH
        t[:, 1:] = lab
        targets.append(t)
    for name, (conf, iou) in SETTINGS.items():
        batches = []
        for b0 in range(0, len(labels), BATCH):
            idx = list(range(b0, min(b0 + BATCH, len(labels))))
            imgs = torch.zeros((len(idx), 3, IMG, IMG), dtype=torch.uint8)
            batches.append((imgs, torch.from_numpy(np.concatenate([targets[i] for i in idx])),
                            [f"img{i}.jpg" for i in idx], None))
        queue = [torch.from_numpy(ios[b0:b0 + BATCH]) for b0 in range(0, len(labels), BATCH)]

        class StandIn(torch.nn.Module):
            def __init__(self):
                super().__init__()
                self.p = torch.nn.Parameter(torch.zeros(1))

            def forward(self, x):
                return queue.pop(0), None

        captured = []
        real_nms = test_mod.non_max_suppression

        def nms_capture(*a, **kw):
            r = real_nms(*a, **kw)
            captured.extend(r)
            return r

        test_mod.non_max_suppression = nms_capture
        with tempfile.TemporaryDirectory() as td, _cwd(td):
            open("odder.names", "w").write("person\nvehicle\n")
            open("odder.data", "w").write(f"classes={NC}\nvalid=none.txt\nnames=odder.names\n")
            open("test_batch0.png", "w").close()   # skip plot_images (test.py:81-82)
            res, maps = test_mod.test(None, "odder.data", batch_size=BATCH, img_size=IMG, conf_thres=conf,
                                      iou_thres=iou, model=StandIn(), dataloader=batches)
        test_mod.non_max_suppression = real_nms
        cnt = np.array([0 if d is None else len(d) for d in captured], np.int32)
        dets = np.concatenate([d.numpy() for d in captured if d is not None]).astype(np.float32)
        key = f"eval/{name}"
        out[f"{key}/conf_iou"] = np.array([conf, iou])
        out[f"{key}/result"] = np.array(res[:4], np.float64)
        out[f"{key}/maps"] = np.asarray(maps, np.float64)
        out[f"{key}/nms_count"] = cnt
        out[f"{key}/nms_det"] = dets
        print(name, "P R mAP F1", np.round(res[:4], 4), "maps", np.round(maps, 4), "survivors", cnt.sum())
    out["eval/io"] = ios
    out["eval/targets"] = np.concatenate(targets)
    out["eval/n_labels"] = np.array([len(lab) for lab in labels], np.int32)
    out["eval/batch"] = np.array(BATCH)
    out["eval/img"] = np.array(IMG)


def ap_goldens(utils, out):
    rng = np.random.default_rng(777)
    cases = {
        "basic": (300, 1, 3, 3, 80),
        "extra_pred_cls": (250, 1, 4, 3, 60),     # predicted class 3 has no targets
        "iou10": (200, 10, 3, 3, 50),
        "missing_cls": (120, 1, 2, 4, 40),        # target classes 2,3 have no predictions
        "empty_pred": (0, 1, 2, 3, 30),
    }
    for name, (n, niou, npc, ntc, nt) in cases.items():
        tp = rng.uniform(size=(n, niou)) < np.linspace(0.7, 0.2, niou)
        conf = rng.uniform(size=n).astype(np.float32)
        pred_cls = rng.integers(0, npc, n).astype(np.float32)
        target_cls = rng.integers(0, ntc, nt).astype(np.float64)
        p, r, ap, f1, cls = utils.ap_per_class(tp, conf, pred_cls, target_cls)
        for k, v in dict(tp=tp, conf=conf, pred_cls=pred_cls, target_cls=target_cls, p=p, r=r, ap=ap, f1=f1,
                         cls=cls).items():
            out[f"ap/{name}/{k}"] = v
    for i, n in enumerate((1, 7, 50, 400)):
        recall = np.sort(rng.uniform(size=n)) * rng.uniform(0.5, 1.0)
        precision = rng.uniform(size=n)
        if i == 2:
            recall[-1] = 1.0
        out[f"cap/{i}/recall"] = recall
        out[f"cap/{i}/precision"] = precision
        out[f"cap/{i}/ap"] = np.array(utils.compute_ap(recall, precision))


def main():
    test_mod = import_yolov3_test(nms_stub)
    out = {}
    eval_goldens(test_mod, out)
    ap_goldens(test_mod, out)
    np.savez_compressed(os.path.join(HERE, "map_golden.npz"), **out)


if __name__ == "__main__":
    main()
