"""Import helpers for the reference code (used ONLY by the golden/calibration
generators in this directory, run in the build container where /root/reference
exists; nothing on the GPU box imports this)."""
from __future__ import annotations

import contextlib
import os
import sys
import types

REF = "/root/reference/code"
CLS_DIR = os.path.join(REF, "disaster_detection")
DET_DIR = os.path.join(REF, "victim_localization", "yolov3")


def import_classifiers():
    if CLS_DIR not in sys.path:
        sys.path.insert(0, CLS_DIR)
    from model.ernet import ErNET
    from model.squeeze_ernet import Squeeze_ErNET
    from model.squeeze_ernet_redconv import Squeeze_RedConv
    return {"squeeze-ernet": Squeeze_ErNET, "squeeze-redconv": Squeeze_RedConv, "ernet": ErNET}


@contextlib.contextmanager
def _cwd(path):
    old = os.getcwd()
    os.chdir(path)
    try:
        yield
    finally:
        os.chdir(old)


def import_darknet(nms_impl=None):
    """yolov3 models/utils with cv2 stubbed (import-time only) and torchvision stubbed
    by a module whose ops.boxes.nms is `nms_impl` (the oracle restatement)."""
    cv2 = types.ModuleType("cv2")
    cv2.setNumThreads = lambda n: None
    sys.modules.setdefault("cv2", cv2)
    tv = types.ModuleType("torchvision")
    ops = types.ModuleType("torchvision.ops")
    boxes = types.ModuleType("torchvision.ops.boxes")
    boxes.nms = nms_impl
    ops.boxes = boxes
    tv.ops = ops
    sys.modules["torchvision"] = tv
    sys.modules["torchvision.ops"] = ops
    sys.modules["torchvision.ops.boxes"] = boxes
    if DET_DIR not in sys.path:
        sys.path.insert(0, DET_DIR)
    with _cwd(DET_DIR):
        import models
        from utils import utils
    return models, utils


def import_yolov3_test(nms_impl=None):
    """yolov3/test.py as a module (named ref_yolov3_test: the bare name `test` is the
    stdlib's regression-test package).  Same stubs as import_darknet."""
    import importlib.util
    import_darknet(nms_impl)
    # utils/datasets.py reads cv2 constants as default arguments at import time only
    # (letterbox/load_image are never called here): plain sentinels suffice
    cv2 = sys.modules["cv2"]
    for k in ("INTER_AREA", "INTER_LINEAR", "BORDER_CONSTANT"):
        if not hasattr(cv2, k):
            setattr(cv2, k, -1)
    spec = importlib.util.spec_from_file_location("ref_yolov3_test", os.path.join(DET_DIR, "test.py"))
    mod = importlib.util.module_from_spec(spec)
    with _cwd(DET_DIR):
        spec.loader.exec_module(mod)
    return mod
