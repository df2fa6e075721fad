#!/usr/bin/env python3
"""Drop-in for disaster_detection/evaluate-classification-metrics.py on the HIP runtime.

Same flags (:133-153) and the same report: accuracy / F1 / precision / recall
(torchmetrics multiclass defaults = micro averaging), average batch inference time and
"FPS" = 1 / mean batch time (batches/s, :96 — kept for drop-in output), per-class
precision / recall / F1 from the confusion matrix (:106-130).  Also reports frames/s.
Images are decoded on the host (Pillow; the reference's DataLoader workers), each one
resized/cropped/normalised on the GPU (rtdm_preprocess_frames, Pillow-exact) and the
batch classified in one rtdm_classify call.  ``--trt --quant fp16`` selects the fp16 path,
``--trt --quant int8`` the int8 one (calibrated on ``--calib`` images).
"""
import argparse
import logging
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from rtdm.classifier import CLASSES, load_model  # noqa: E402
from rtdm.cli import (calibration_frames, classification_metrics, read_image_rgb, read_split_csv,  # noqa: E402
                      select_device)
from rtdm.preprocess import preprocess_frames  # noqa: E402

logger = logging.getLogger(__name__)


def evaluate_model(model, rows, root_dir, batch_size, device, num_workers=4, half=False):
    """evaluate_model (:49-104): returns the metrics dict."""
    size = model.INPUT
    preds, targets, times = [], [], []
    pool = ThreadPoolExecutor(max(1, num_workers))
    for b0 in range(0, len(rows), batch_size):
        batch = rows[b0:b0 + batch_size]
        imgs = list(pool.map(lambda r: read_image_rgb(os.path.join(root_dir, r[0])), batch))
        x = torch.empty((len(batch), 3, size, size), device=device, dtype=torch.float32)
        for i, img in enumerate(imgs):
            x[i:i + 1] = preprocess_frames(torch.from_numpy(img[None]).to(device), size)
        if half:
            x = x.half()
        torch.cuda.synchronize()
        t0 = time.time()
        out = model(x)
        torch.cuda.synchronize()
        times.append(time.time() - t0)
        preds += out.argmax(dim=1).cpu().tolist()
        targets += [r[1] for r in batch]
    pool.shutdown()
    m = classification_metrics(preds, targets)
    m["avg_inference_time"] = float(np.mean(times)) if times else 0.0
    m["fps"] = 1.0 / m["avg_inference_time"] if times else 0.0
    m["frames_per_s"] = len(preds) / float(np.sum(times)) if times else 0.0
    return m


def main(argv=None):
    parser = argparse.ArgumentParser(description='Evaluate model on test set')
    parser.add_argument('--model', type=str, default='ernet', choices=['ernet', 'squeeze-ernet', 'squeeze-redconv'])
    parser.add_argument('--weights', type=str, required=True)
    parser.add_argument('--test-split', type=str, default='dataloaders/aider_test.csv')
    parser.add_argument('--root-dir', type=str, default='data/AIDER')
    parser.add_argument('--batch-size', type=int, default=64)
    parser.add_argument('--num-workers', type=int, default=4)
    parser.add_argument('--no-cuda', action='store_true')
    parser.add_argument('--trt', action='store_true', help='fp16 path stand-in for TensorRT')
    parser.add_argument('--quant', type=str, default='fp16', choices=['fp16', 'fp32', 'int8'])
    parser.add_argument('--calib', type=str, default=None,
                        help='int8: directory of calibration images; default: the first 64 test images')
    args = parser.parse_args(argv)

    device = select_device(args.no_cuda)
    logger.info(f"Using device: {device}")
    rows = read_split_csv(args.test_split)
    half = args.trt and args.quant == 'fp16'
    quant = args.quant if args.trt else 'fp32'
    calib = None
    if quant == 'int8':
        calib = calibration_frames(args.calib, (read_image_rgb(os.path.join(args.root_dir, r[0])) for r in rows[:64]),
                                   device)
    model = load_model(args.model, args.weights, device, quant=quant, calib=calib)
    metrics = evaluate_model(model, rows, args.root_dir, args.batch_size, device, args.num_workers, half)

    logger.info("\nEvaluation Results:")
    logger.info(f"Accuracy: {metrics['accuracy']:.4f}")
    logger.info(f"F1 Score: {metrics['f1_score']:.4f}")
    logger.info(f"Precision: {metrics['precision']:.4f}")
    logger.info(f"Recall: {metrics['recall']:.4f}")
    logger.info(f"Average Inference Time: {metrics['avg_inference_time']:.4f} seconds")
    logger.info(f"FPS: {metrics['fps']:.2f}")
    logger.info(f"Frames/s: {metrics['frames_per_s']:.2f}")
    logger.info("\nPer-class Metrics:")
    for class_name in CLASSES:
        logger.info(f"\n{class_name}:")
        logger.info(f"  Precision: {metrics[f'{class_name}_precision']:.4f}")
        logger.info(f"  Recall: {metrics[f'{class_name}_recall']:.4f}")
        logger.info(f"  F1 Score: {metrics[f'{class_name}_f1']:.4f}")
    return metrics


if __name__ == '__main__':
    main()
