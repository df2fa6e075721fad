"""Labelled test-set loader for the mAP harness: LoadImagesAndLabels counterpart
(victim_localization/yolov3/utils/datasets.py:258-505) for the evaluation case only
(augment=False, rect=False, image_weights=False): list file of image paths, YOLO label
files found by replacing 'images' with 'labels', load_image shrink + letterbox to a
square img_size (auto=False, scaleup=False, pad 128), labels re-normalised to the
letterboxed frame.  Frames come out NHWC uint8 RGB — the detector's native input
(the /255 and the NCHW view are fused into its first kernel) — instead of the
reference's NCHW copy.
"""
from __future__ import annotations

import os

import numpy as np
import torch

from .letterbox import labels_to_letterbox, letterbox, load_image

IMG_FORMATS = ('.bmp', '.jpg', '.jpeg', '.png', '.tif', '.tiff', '.dng')   # datasets.py:19


def read_rgb(path: str) -> np.ndarray:
    from PIL import Image
    with Image.open(path) as im:
        return np.asarray(im.convert('RGB'), np.uint8)


def label_path(img_path: str) -> str:
    """datasets.py:286-287."""
    return img_path.replace('images', 'labels').replace(os.path.splitext(img_path)[-1], '.txt')


def read_labels(path: str) -> np.ndarray:
    if not os.path.isfile(path):
        return np.zeros((0, 5), np.float32)
    with open(path) as f:
        rows = [ln.split() for ln in f.read().splitlines() if ln.strip()]
    return np.array(rows, np.float32).reshape(-1, 5)


class LoadImagesAndLabels(torch.utils.data.Dataset):
    def __init__(self, path: str, img_size: int = 416, batch_size: int = 16, root: str | None = None):
        path = str(path)
        if not os.path.isfile(path):
            raise FileNotFoundError(f"File not found {path}")
        base = root if root is not None else os.getcwd()
        with open(path) as f:
            files = [x for x in f.read().splitlines() if os.path.splitext(x)[-1].lower() in IMG_FORMATS]
        if not files:
            raise ValueError(f"No images found in {path}")
        # list files hold paths relative to the directory test.py runs from (the cwd)
        self.img_files = [x if os.path.isabs(x) else os.path.join(base, x) for x in files]
        self.label_files = [label_path(x) for x in self.img_files]
        self.img_size = img_size
        self.batch_size = batch_size

    def __len__(self):
        return len(self.img_files)

    def __getitem__(self, index):
        img0 = read_rgb(self.img_files[index])
        img, (h0, w0), (h, w) = load_image(img0, self.img_size)
        img, ratio, pad = letterbox(img, self.img_size, auto=False, scaleup=False)
        labels = labels_to_letterbox(read_labels(self.label_files[index]), ratio, pad, h, w, img.shape[0],
                                     img.shape[1])
        out = torch.zeros((len(labels), 6))
        if len(labels):
            out[:, 1:] = torch.from_numpy(labels)
        shapes = (h0, w0), ((h / h0, w / w0), pad)
        return torch.from_numpy(np.ascontiguousarray(img)), out, self.img_files[index], shapes

    @staticmethod
    def collate_fn(batch):
        """datasets.py:501-505: stack frames, concatenate labels with their image index."""
        img, label, path, shapes = zip(*batch)
        for i, lab in enumerate(label):
            lab[:, 0] = i
        return torch.stack(img, 0), torch.cat(label, 0), path, shapes
