#!/usr/bin/env python3
"""Drop-in for victim_localization/yolov3/test.py (mAP@0.5 harness) on the HIP runtime.

Same flags (:201-211) and the same table: P, R, mAP@0.5 and F1 per class at
conf_thres 0.001 / iou_thres from the command line.  Tasks: 'test' (default) and
'benchmark' (img-size 320..608 x iou 0.5/0.7, :225-233); 'study' needs matplotlib
plotting and is not carried over.  Evaluation logic: rtdm.evaluation.test.

Several GPUs (the reference's nn.DataParallel, :42-43): one process per GPU,
  python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 test.py ...
each rank evaluates a contiguous shard of the list file and every rank prints / returns
the single-process result.
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import numpy as np  # noqa: E402

from rtdm.evaluation import test  # noqa: E402


def main(argv=None):
    parser = argparse.ArgumentParser(prog='test.py')
    parser.add_argument('--cfg', type=str, default='cfg/yolov3-tiny-aider-416.cfg', help='*.cfg path')
    parser.add_argument('--data', type=str, default='data/aider.data', help='*.data path')
    parser.add_argument('--weights', type=str, default='weights/yolov3-tiny-aider-416.weights', help='weights path')
    parser.add_argument('--batch-size', type=int, default=32, help='size of each image batch')
    parser.add_argument('--img-size', type=int, default=416, help='inference size (pixels)')
    parser.add_argument('--conf-thres', type=float, default=0.001, help='object confidence threshold')
    parser.add_argument('--iou-thres', type=float, default=0.4, help='IOU threshold for NMS')
    parser.add_argument('--task', default='test', help="'test', 'benchmark'")
    parser.add_argument('--device', default='', help='device id (cpu is refused: GPU-only runtime)')
    parser.add_argument('--half', action='store_true', help='fp16 detector')
    opt = parser.parse_args(argv)
    print(opt)
    if opt.device == 'cpu':
        raise SystemExit("rtdm runs on the MI355X HIP runtime only: --device cpu has no CPU path here")
    if opt.task == 'test':
        return test(opt.cfg, opt.data, opt.weights, opt.batch_size, opt.img_size, opt.conf_thres, opt.iou_thres,
                    half=opt.half)
    if opt.task == 'benchmark':
        y = []
        for i in [320, 416, 512, 608]:
            for j in [0.5, 0.7]:
                t = time.time()
                r = test(opt.cfg, opt.data, opt.weights, opt.batch_size, i, opt.conf_thres, j, half=opt.half)[0]
                y.append(r + (time.time() - t,))
        np.savetxt('benchmark.txt', y, fmt='%10.4g')
        return y
    raise SystemExit(f"unsupported --task {opt.task}")


if __name__ == '__main__':
    main()
