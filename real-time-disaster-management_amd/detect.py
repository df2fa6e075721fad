#!/usr/bin/env python3
"""Drop-in for victim_localization/yolov3/detect.py on the HIP runtime.

Same flags (:159-174) and outputs: per image "%gx%g <counts per class> Done. (time)",
``--save-txt`` rows "x1 y1 x2 y2 cls conf" (:118-121), annotated images in --output.
Darknet(cfg, img_size) + load_darknet_weights / torch.load(...)['model'] (:21-28) →
model(img)[0] (:87) → non_max_suppression(conf, iou, classes, agnostic) (:91) →
scale_coords back to the source image (:108).  Frames are letterboxed on the GPU like
LoadImages → letterbox (utils/datasets.py:599-631, auto=True: longer side → img_size,
the shorter padded to a multiple of 32 with (128,128,128)) by rtdm_letterbox, whose
resize restates cv2.INTER_AREA (rtdm.letterbox).  Each distinct letterboxed
shape gets its own planned detector handle (the reference rebuilds grids per shape,
models.py:228-230).
"""
import argparse
import os
import shutil
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from rtdm.cli import list_images, load_image, select_device  # noqa: E402
from rtdm.darknet import Darknet, load_darknet_weights  # noqa: E402
from rtdm.letterbox import geometry, letterbox, letterbox_frames, scale_coords  # noqa: E402,F401
from rtdm.nms import non_max_suppression  # noqa: E402


def load_names(path):
    if path and os.path.exists(path):
        with open(path) as f:
            return [x.strip() for x in f if x.strip()]
    return None


def detect(opt):
    device = select_device(opt.device == 'cpu')
    out = opt.output
    if os.path.exists(out):
        shutil.rmtree(out)
    os.makedirs(out)
    model = Darknet(opt.cfg, opt.img_size)
    if opt.weights.endswith('.pt'):
        model.load_state_dict(torch.load(opt.weights, map_location='cpu', weights_only=True)['model'])
    else:
        load_darknet_weights(model, opt.weights)
    if opt.half:
        model.half()
    models = {model.img_size: model}

    def model_for(shape):
        if shape not in models:
            m = Darknet(model.cfg_text, shape)
            m.load_weight_stream(model._stream)
            if opt.half:
                m.half()
            models[shape] = m
        return models[shape]

    names = load_names(opt.names) or [str(i) for i in range(model.no - 5)]
    t0 = time.time()
    results = {}
    for path in list_images(opt.source):
        x0 = load_image(path, device)  # JPEGs decoded on the device (rtdm.jpeg), others via Pillow
        # letterbox (INTER_AREA resize + pad) on the device
        g = geometry(x0.shape[0], x0.shape[1], opt.img_size, auto=True)
        x = letterbox_frames(x0[None], g)  # uint8 NHWC; /255 fused in the stem
        img_shape = (g[2], g[3])
        torch.cuda.synchronize()
        t1 = time.time()
        pred, _ = model_for(img_shape)(x)
        det = non_max_suppression(pred, opt.conf_thres, opt.iou_thres, classes=opt.classes,
                                  agnostic=opt.agnostic_nms)[0]
        torch.cuda.synchronize()
        t2 = time.time()
        s = '%gx%g ' % img_shape
        save_path = os.path.join(out, os.path.basename(path))
        rows = []
        if det is not None and len(det):
            det = det.cpu()
            det[:, :4] = scale_coords(img_shape, det[:, :4], tuple(x0.shape)).round()
            for c in det[:, -1].unique():
                n = int((det[:, -1] == c).sum())
                s += '%g %ss, ' % (n, names[int(c)])
            for *xyxy, conf, cls in det.tolist():
                rows.append((*xyxy, cls, conf))
                if opt.save_txt:
                    with open(save_path + '.txt', 'a') as f:
                        f.write(('%g ' * 6 + '\n') % (*xyxy, cls, conf))
            if not opt.no_save_img:
                from PIL import Image, ImageDraw
                im = Image.fromarray(x0.cpu().numpy())
                d = ImageDraw.Draw(im)
                for x1, y1, x2, y2, cls, conf in rows:
                    d.rectangle([x1, y1, x2, y2], outline=(255, 0, 0), width=2)
                    d.text((x1, max(0, y1 - 12)), '%s %.2f' % (names[int(cls)], conf), fill=(255, 0, 0))
                im.save(save_path)
        results[path] = rows
        print('%sDone. (%.3fs)' % (s, t2 - t1))
    print('Done. (%.3fs)' % (time.time() - t0))
    return results


def main(argv=None):
    parser = argparse.ArgumentParser()
    parser.add_argument('--cfg', type=str, default='cfg/yolov3-spp.cfg', help='*.cfg path')
    parser.add_argument('--names', type=str, default='data/aider.names', help='*.names path')
    parser.add_argument('--weights', type=str, default='weights/best.pt', help='weights path')
    parser.add_argument('--source', type=str, default='data/custom/test/images', help='image file or folder')
    parser.add_argument('--output', type=str, default='output', help='output folder')
    parser.add_argument('--img-size', type=int, default=416, help='inference size (pixels)')
    parser.add_argument('--conf-thres', type=float, default=0.3, help='object confidence threshold')
    parser.add_argument('--iou-thres', type=float, default=0.4, help='IOU threshold for NMS')
    parser.add_argument('--half', action='store_true', help='half precision FP16 inference')
    parser.add_argument('--device', default='', help='device id (cpu is refused: GPU-only runtime)')
    parser.add_argument('--save-txt', action='store_true', help='save results to *.txt')
    parser.add_argument('--no-save-img', action='store_true', help='do not write annotated images')
    parser.add_argument('--classes', nargs='+', type=int, help='filter by class')
    parser.add_argument('--agnostic-nms', action='store_true', help='class-agnostic NMS')
    opt = parser.parse_args(argv)
    print(opt)
    with torch.no_grad():
        return detect(opt)


if __name__ == '__main__':
    main()
