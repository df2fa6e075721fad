"""Labelled test-set loader for the mAP harness: LoadImagesAndLabels counterpart
(victim_localization/yolov3/utils/datasets.py:258-505) for the evaluation case only
(augment=False, rect=False, image_weights=False): list file of image paths, YOLO label
files found by replacing 'images' with 'labels', labels re-normalised to the letterboxed
frame (load_image shrink + letterbox(auto=False, scaleup=False) to img_size², pad 128).

Workers only decode (Pillow, RGB) and do the label arithmetic; the resize + pad runs on
the GPU when the batch is moved there (``RawFrames.to_device`` → rtdm_letterbox, one
launch per distinct source size), so frames cross PCIe at their source size and come
out as the detector's NHWC uint8 input.
"""
from __future__ import annotations

import os

import numpy as np
import torch

from .letterbox import dataset_geometry, labels_to_letterbox, letterbox_frames

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


class RawFrames:
    """A collated batch of decoded source images (host uint8 [h0, w0, 3], any sizes) and
    their letterbox geometries; ``to_device`` letterboxes them into one [N, S, S, 3] tensor."""

    def __init__(self, imgs, geoms, img_size: int, color=(128, 128, 128)):
        self.imgs = list(imgs)
        self.geoms = list(geoms)
        self.img_size = img_size
        self.color = color

    def __len__(self):
        return len(self.imgs)

    @property
    def shape(self):
        return (len(self.imgs), self.img_size, self.img_size, 3)

    def to_device(self, device) -> torch.Tensor:
        out = torch.empty(self.shape, dtype=torch.uint8, device=device)
        for i, (img, g) in enumerate(zip(self.imgs, self.geoms)):
            x = torch.from_numpy(img).pin_memory().to(device, non_blocking=True)[None]
            letterbox_frames(x, g, self.color, out=out[i:i + 1])
        return out


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
        h0, w0 = img0.shape[:2]
        g, (h, w), ratio, pad = dataset_geometry(h0, w0, self.img_size)
        labels = labels_to_letterbox(read_labels(self.label_files[index]), ratio, pad, h, w, g[2], g[3])
        out = torch.zeros((len(labels), 6))
        if len(labels):
            out[:, 1:] = torch.from_numpy(labels)
        shapes = (h0, w0), ((h / h0, w / w0), pad)
        return (img0, g), out, self.img_files[index], shapes

    def collate_fn(self, batch):
        """datasets.py:501-505: labels concatenated with their image index; frames stay
        raw (RawFrames) until they reach the GPU."""
        img, label, path, shapes = zip(*batch)
        for i, lab in enumerate(label):
            lab[:, 0] = i
        return (RawFrames([x for x, _ in img], [g for _, g in img], self.img_size), torch.cat(label, 0), path,
                shapes)
