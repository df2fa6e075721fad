#!/usr/bin/env python3
"""Drop-in for disaster_detection/real-time-inference.py on the HIP runtime.

Same flags (:134-152) and statistics (average / min / max FPS, :218-221).  Per frame, on
the device: cv2.resize(frame, (--width, --height)) with its default INTER_LINEAR (:185;
rtdm_resize_linear, OpenCV's algorithm restated), then the CLI transform + classifier
(rtdm_classify on the uint8 frame, :62-107).  Video decoding
(imutils/cv2) is not part of this stack: --video takes a directory of image frames or an
.npy array [T,H,W,3] uint8; webcam capture is not available.  ``--trt --quant int8`` runs the int8 path
(calibrated on ``--calib`` images).  ``--batch`` > 1 classifies
that many frames per call (throughput mode); the default 1 is the reference's per-frame loop.
"""
import argparse
import logging
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from rtdm.classifier import load_model  # noqa: E402
from rtdm.cli import calibration_frames, list_images, predict_frames, read_image_rgb, select_device  # noqa: E402
from rtdm.letterbox import resize_linear  # noqa: E402

logger = logging.getLogger(__name__)


def frame_source(video: str):
    """Host RGB frames, in order (decoding stays on the host)."""
    if video is None:
        raise SystemExit("webcam capture needs cv2/imutils, which this stack does not ship: pass --video")
    if video.endswith(".npy"):
        frames = np.load(video, allow_pickle=False)
        it = (frames[i] for i in range(frames.shape[0]))
    else:
        it = (read_image_rgb(p) for p in list_images(video))
    yield from it


def main(argv=None):
    parser = argparse.ArgumentParser(description='Real-time disaster detection inference')
    parser.add_argument('--model', type=str, default='ernet', choices=['ernet', 'squeeze-ernet', 'squeeze-redconv'])
    parser.add_argument('--weights', type=str, required=True)
    parser.add_argument('--video', type=str, default=None, help='directory of frames or .npy [T,H,W,3] uint8')
    parser.add_argument('--width', type=int, default=640)
    parser.add_argument('--height', type=int, default=480)
    parser.add_argument('--no-cuda', action='store_true')
    parser.add_argument('--trt', action='store_true', help='fp16 path stand-in for TensorRT')
    parser.add_argument('--quant', type=str, default='fp16', choices=['fp16', 'fp32', 'int8'])
    parser.add_argument('--calib', type=str, default=None,
                        help='int8: directory of calibration images; default: the first 16 stream frames')
    parser.add_argument('--batch', type=int, default=1, help='frames per classifier call')
    args = parser.parse_args(argv)

    device = select_device(args.no_cuda)
    logger.info(f"Using device: {device}")
    quant = args.quant if args.trt else 'fp32'
    calib = None
    if quant == 'int8':
        import itertools
        calib = calibration_frames(args.calib, itertools.islice(frame_source(args.video), 16), device)
    model = load_model(args.model, args.weights, device, quant=quant, calib=calib)
    fps_list, results = [], []
    prev = time.time()
    pending = []
    logger.info("Starting inference...")

    def flush():
        nonlocal prev
        frames = torch.stack(pending)
        _, names, conf = predict_frames(model, frames)
        now = time.time()
        fps_list.append(len(pending) / (now - prev))
        prev = now
        results.extend(zip(names, conf))
        pending.clear()

    for f in frame_source(args.video):
        # upload the decoded frame, cv2.resize(frame, (width, height)) on the device (:185)
        pending.append(resize_linear(torch.from_numpy(np.ascontiguousarray(f)).to(device), args.height, args.width))
        if len(pending) == args.batch:
            flush()
    if pending:
        flush()
    if fps_list:
        logger.info(f"Average FPS: {sum(fps_list) / len(fps_list):.2f}")
        logger.info(f"Min FPS: {min(fps_list):.2f}")
        logger.info(f"Max FPS: {max(fps_list):.2f}")
    return results, fps_list


if __name__ == '__main__':
    main()
