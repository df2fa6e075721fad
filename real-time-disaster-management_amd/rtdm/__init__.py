"""rtdm — MI355X-native two-stage aerial-frame inference (ACFF classifier -> Darknet YOLO
-> decode -> NMS) over a gfx950 HIP runtime (librtdm.so, C ABI in include/rtdm.h)."""
from ._lib import RtdmError, lib  # noqa: F401
from .classifier import CLASSES, ErNET, Squeeze_ErNET, Squeeze_RedConv, build_model, load_model  # noqa: F401
from .darknet import Darknet, load_darknet_weights  # noqa: F401
from .nms import nms_batched, non_max_suppression  # noqa: F401
from .pipeline import TwoStagePipeline  # noqa: F401
from .preprocess import preprocess_frames  # noqa: F401
