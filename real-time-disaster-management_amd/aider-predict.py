#!/usr/bin/env python3
"""Drop-in for disaster_detection/aider-predict.py on the MI355X HIP runtime.

Same flags (--model --image --weights --no-cuda --trt --quant, aider-predict.py:124-138)
and the same printed result: class name + confidence = softmax(model output)[cls]·100
(the reference's double softmax, :77-80).  The image transform
(Resize(int(1.14·S)) → CenterCrop(S) → ToTensor → Normalize, dataloaders/aider.py:412-431)
runs on the GPU, Pillow-exact.  ``--trt`` has no TensorRT behind it: it adds a second
prediction on the fp16 path (``--quant fp16``), the fp32 path, or the int8 path (``--quant
int8``: int8 MFMA ACFF fusion GEMMs, calibrated on ``--calib`` frames), which is what the
reference's TRT engines were for (README.md:32-40 promises the three schemes).  Plotting (cv2/matplotlib) is replaced by ``--save``.
"""
import argparse
import logging
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import torch  # noqa: E402

from rtdm.classifier import load_model  # noqa: E402
from rtdm.cli import calibration_frames, load_image, predict_frames, read_image_rgb, select_device  # noqa: E402

logger = logging.getLogger(__name__)


def predict(model, image_path, device):
    """aider-predict.py:47-86 counterpart -> (class name, confidence %)."""
    frames = load_image(image_path, device)[None]  # JPEGs decoded on the device
    _, names, conf = predict_frames(model, frames)
    return names[0], conf[0]


def main(argv=None):
    parser = argparse.ArgumentParser(description='Predict disaster types from aerial images')
    parser.add_argument('--model', type=str, default='ernet', choices=['ernet', 'squeeze-ernet', 'squeeze-redconv'],
                        help='model architecture')
    parser.add_argument('--image', type=str, required=True, help='path to input image')
    parser.add_argument('--weights', type=str, default=None, help='path to model weights')
    parser.add_argument('--no-cuda', action='store_true', help='disable CUDA (not supported: GPU-only runtime)')
    parser.add_argument('--trt', action='store_true', help='also run the reduced-precision path (TensorRT stand-in)')
    parser.add_argument('--quant', type=str, default='fp16', choices=['fp16', 'fp32', 'int8'],
                        help='precision of the --trt path')
    parser.add_argument('--calib', type=str, default=None,
                        help='int8: directory (or image) of calibration frames; default: the input image')
    parser.add_argument('--save', type=str, default=None, help='write the annotated image here (replaces plt.show)')
    args = parser.parse_args(argv)

    device = select_device(args.no_cuda)
    logger.info(f"Using device: {device}")
    if args.weights is None:
        args.weights = f'weights/{args.model}.pt'
        if not os.path.exists(args.weights):
            raise FileNotFoundError(f"No weights found at {args.weights}")

    model = load_model(args.model, args.weights, device)
    prediction, confidence = predict(model, args.image, device)
    logger.info(f"Prediction: {prediction} ({confidence:.1f}%)")
    result = {"prediction": prediction, "confidence": confidence}
    if args.trt:
        calib = calibration_frames(args.calib, [read_image_rgb(args.image)], device) \
            if args.quant == 'int8' else None
        trt_model = load_model(args.model, args.weights, device, quant=args.quant, calib=calib)
        trt_prediction, trt_confidence = predict(trt_model, args.image, device)
        logger.info(f"TensorRT Prediction: {trt_prediction} ({trt_confidence:.1f}%)")
        result.update({"trt_prediction": trt_prediction, "trt_confidence": trt_confidence})
    if args.save:
        from PIL import Image, ImageDraw
        im = Image.open(args.image).convert("RGB")
        d = ImageDraw.Draw(im)
        d.text((10, 10), f"{prediction} ({confidence:.1f}%)", fill=(255, 255, 255))
        if args.trt:
            d.text((10, 30), f"TRT: {result['trt_prediction']} ({result['trt_confidence']:.1f}%)", fill=(255, 255, 255))
        im.save(args.save)
    return result


if __name__ == '__main__':
    main()
