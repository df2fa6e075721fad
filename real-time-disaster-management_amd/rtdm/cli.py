"""Shared pieces of the drop-in CLIs (aider-predict.py, real-time-inference.py,
evaluate-classification-metrics.py, detect.py next to this package).

The reference CLIs decode images with cv2 (BGR) and convert to RGB
(aider-predict.py:59-62); cv2 is not part of this stack, so images are decoded
with Pillow straight to RGB.  The classifier transform then runs on the GPU
(rtdm_classify with RTDM_INPUT_FRAME_U8: Pillow-exact bilinear resize, center
crop, Normalize — dataloaders/aider.py:412-431).  Everything runs on the HIP
runtime; there is no CPU inference path (``--no-cuda`` is refused loudly).
"""
from __future__ import annotations

import logging
import os

import numpy as np
import torch

from .classifier import CLASSES

logging.basicConfig(level=logging.INFO, format='%(asctime)s - %(name)s - %(levelname)s - %(message)s')

IMG_EXTS = ('.jpg', '.jpeg', '.png', '.bmp', '.tif', '.tiff', '.webp')


def select_device(no_cuda: bool = False) -> torch.device:
    """aider-predict.py:143 counterpart; the rtdm kernels exist only for the GPU."""
    if no_cuda:
        raise SystemExit("rtdm runs on the MI355X HIP runtime only: --no-cuda has no CPU path here")
    if not torch.cuda.is_available():
        raise SystemExit("rtdm needs a HIP device (torch.cuda.is_available() is False)")
    return torch.device("cuda", torch.cuda.current_device())


def read_image_rgb(path: str) -> np.ndarray:
    """uint8 [H, W, 3] RGB (cv2.imread + COLOR_BGR2RGB in the reference)."""
    from PIL import Image
    if not os.path.exists(path):
        raise ValueError(f"Could not load image at {path}")
    with Image.open(path) as im:
        return np.array(im.convert("RGB"), dtype=np.uint8)


def load_image(path: str, device) -> torch.Tensor:
    """cv2.imread + COLOR_BGR2RGB (aider-predict.py:57-58, yolov3/utils/datasets.py:97) as a
    device frame uint8 [H, W, 3] RGB: baseline JPEGs are decoded on the device (rtdm.jpeg:
    host entropy decode, then IDCT / upsampling / colour conversion in HIP, bit-exact with
    libjpeg-turbo); other formats (PNG, progressive JPEG, ...) decode through Pillow and
    are uploaded."""
    from . import jpeg
    if not os.path.exists(path):
        raise ValueError(f"Could not load image at {path}")
    with open(path, "rb") as f:
        data = f.read()
    if data[:2] == b"\xff\xd8" and jpeg.supported(data):
        return jpeg.decode(data, device)
    return torch.from_numpy(read_image_rgb(path)).to(device)


def list_images(source: str):
    if os.path.isdir(source):
        return sorted(os.path.join(source, f) for f in os.listdir(source) if f.lower().endswith(IMG_EXTS))
    return [source]


def predict_frames(model, frames: torch.Tensor):
    """frames [N,H,W,3] uint8 on the device -> (class ids, class names, confidence %).
    confidence = softmax(model output)[cls] * 100, i.e. softmax of the probabilities the
    model already returns — the reference's double softmax (aider-predict.py:77-80)."""
    probs = model.classify_frames(frames)
    cls = probs.argmax(dim=1)
    conf = torch.softmax(probs, dim=1).gather(1, cls[:, None])[:, 0] * 100.0
    ids = cls.cpu().tolist()
    return ids, [CLASSES[i] for i in ids], conf.cpu().tolist()


def confusion_matrix(preds, targets, nc: int = 5) -> np.ndarray:
    cm = np.zeros((nc, nc), np.int64)
    for p, t in zip(preds, targets):
        cm[int(t), int(p)] += 1
    return cm


def classification_metrics(preds, targets, nc: int = 5) -> dict:
    """evaluate-classification-metrics.py:57-101 counterpart.  torchmetrics'
    task="multiclass" Accuracy/F1Score/Precision/Recall default to micro averaging,
    under which all four equal the fraction of correct predictions; per-class
    precision/recall/F1 from the confusion matrix as compute_per_class_metrics (:106-130)."""
    cm = confusion_matrix(preds, targets, nc)
    total = int(cm.sum())
    acc = float(np.trace(cm)) / total if total else 0.0
    m = {"accuracy": acc, "f1_score": acc, "precision": acc, "recall": acc, "confusion_matrix": cm}
    for i, name in enumerate(CLASSES[:nc]):
        tp = int(cm[i, i])
        fp = int(cm[:, i].sum()) - tp
        fn = int(cm[i, :].sum()) - tp
        p = tp / (tp + fp) if tp + fp > 0 else 0
        r = tp / (tp + fn) if tp + fn > 0 else 0
        f = 2 * p * r / (p + r) if p + r > 0 else 0
        m.update({f"{name}_precision": p, f"{name}_recall": r, f"{name}_f1": f})
    return m


def read_split_csv(path: str):
    """dataloaders/aider_*.csv rows: relative image path, label."""
    rows = []
    with open(path) as f:
        for line in f:
            line = line.strip()
            if not line:
                continue
            p, lab = line.rsplit(",", 1)
            try:
                rows.append((p, int(lab)))
            except ValueError:  # header
                continue
    return rows


def calibration_frames(calib: str | None, fallback, device: torch.device, limit: int = 64):
    """int8 calibration set of the CLIs (--quant int8): the images of `calib` (a directory or
    one image; at most `limit`), uploaded as uint8 [1,H,W,3] device frames; without --calib,
    the host RGB frames in `fallback` (the inputs themselves).  The reference's int8 TRT
    engines were calibrated on a separate image set (tensorrt_inference/yolo/calibrator.py:
    87-153); pass one with --calib for a calibration disjoint from the evaluated frames."""
    if calib is not None:
        imgs = [read_image_rgb(p) for p in list_images(calib)[:limit]]
        if not imgs:
            raise SystemExit(f"--calib {calib}: no images")
    else:
        logging.getLogger(__name__).warning("--quant int8 without --calib: calibrating on the input frames")
        imgs = list(fallback)[:limit]
    return [torch.from_numpy(np.ascontiguousarray(im)[None]).to(device) for im in imgs]
