"""CPU: the C-ABI library loads, exports every symbol include/rtdm.h declares, and
the host-side planner (cfg parse, shape inference, fusion plan, weight-stream
size, FLOP count) matches the reference — no kernel launches, no GPU."""
import ctypes
import os
import re

import numpy as np
import pytest

from conftest import ROOT, cfg_text

CFGS = {  # cfg -> (img, anchors, weight floats, FLOP/img from BASELINE.md §2)
    "yolov4-tiny-aider-416": (608, 30324, None, 15178403840),
    "yolov3-aider-416": (416, 10647, None, 65297143808),
    "yolov3-spp-aider": (608, 22743, None, 140237953024),
    "yolov3-tiny-aider-416": (416, 2535, None, None),
}


def header_symbols():
    with open(os.path.join(ROOT, "include", "rtdm.h")) as f:
        txt = f.read()
    return sorted(set(re.findall(r"\b(rtdm_[a-z0-9_]+)\s*\(", txt)))


def test_library_exports_every_header_symbol():
    from rtdm import _lib as L
    lib = L.lib()
    syms = header_symbols()
    assert len(syms) >= 20
    for s in syms:
        assert hasattr(lib, s), s
        assert s in L.SIGNATURES, f"{s} missing from the ctypes binding"
    assert lib.rtdm_abi_version() == 1
    assert lib.rtdm_build_arch() == b"gfx950"


def test_library_is_gfx950_code_object():
    from rtdm import _lib as L
    data = open(L.LIB_PATH, "rb").read()
    assert b"gfx950" in data
    assert b"amdgcn-amd-amdhsa" in data


def _plan(cfg, img, dtype=1):
    from rtdm import _lib as L
    h = ctypes.c_void_p()
    L.check(L.lib().rtdm_detector_create(cfg_text(cfg).encode(), img, img, dtype, None, 0, 64, ctypes.byref(h)))
    info = L.rtdm_detector_info()
    L.check(L.lib().rtdm_detector_get_info(h, ctypes.byref(info)))
    n = L.lib().rtdm_detector_describe(h, None, 0)
    buf = ctypes.create_string_buffer(int(n))
    L.lib().rtdm_detector_describe(h, buf, n)
    return h, info, buf.value.decode()


@pytest.mark.parametrize("cfg", list(CFGS))
def test_planner_matches_reference(cfg):
    from rtdm import _lib as L
    from rtdm.synth import conv_layers, synth_darknet_weights
    img, anchors, _, flop = CFGS[cfg]
    h, info, plan = _plan(cfg, img)
    try:
        assert info.n_anchors_total == anchors
        assert info.no == 7 and info.nc == 2
        if flop:
            assert info.flop_per_image == flop
        assert info.weight_floats == synth_darknet_weights(cfg_text(cfg)).size
        assert info.n_yolo == sum(1 for c in conv_layers(cfg_text(cfg)) if c[5])
        assert info.device_bytes == 0  # planning only: nothing allocated
    finally:
        L.lib().rtdm_detector_destroy(h)


def test_planner_fusions_yolov4_tiny():
    from rtdm import _lib as L
    h, info, plan = _plan("yolov4-tiny-aider-416", 608)
    L.lib().rtdm_detector_destroy(h)
    # conv+maxpool(2,2) fused for the 5 stride-2 pools; upsample fused into the 1x1 convs;
    # the route concats are written in place; three yolo decodes fused into head convs
    assert plan.count(" quad ") == 5
    assert plan.count("up=up") == 2
    assert plan.count(" yolo") == 3
    assert "copy" not in plan
    assert "@route20+128" in plan and "@route27+128" in plan
    assert "maxpool k2 s1 zeropad" in plan
    assert plan.count("valu") == 1  # only the Cin=3 stem


def test_planner_fusions_yolov3_shortcuts():
    from rtdm import _lib as L
    h, info, plan = _plan("yolov3-aider-416", 416)
    L.lib().rtdm_detector_destroy(h)
    assert len(re.findall(r"res=conv|res=\w+\d+\[", plan)) == 23  # every shortcut fused as a residual epilogue


_SHORTCUT_MISMATCH = """[net]
width=32
height=32
channels=3

[convolutional]
batch_normalize=1
filters=8
size=3
stride=1
pad=1
activation=leaky

[convolutional]
batch_normalize=1
filters=16
size=1
stride=1
pad=1
activation=leaky

[shortcut]
from=-2
activation=linear

[convolutional]
batch_normalize=1
filters=8
size=3
stride=1
pad=1
activation=leaky

[shortcut]
from=-2
activation=linear

[convolutional]
size=1
stride=1
pad=1
filters=14
activation=linear

[yolo]
mask=0,1
anchors=10,14, 23,27
classes=2
num=2
"""


def test_planner_shortcut_channel_mismatch():
    """weightedFeatureFusion with dc > 0 (16-channel map + 8-channel residual) and dc < 0
    (8-channel map + 16-channel residual), models.py:146-154: planned as unfused adds whose
    output keeps the current map's channels (the GPU parity test runs it vs the oracle)."""
    from rtdm import _lib as L
    h = ctypes.c_void_p()
    L.check(L.lib().rtdm_detector_create(_SHORTCUT_MISMATCH.encode(), 32, 32, 1, None, 0, 2, ctypes.byref(h)))
    try:
        n = L.lib().rtdm_detector_describe(h, None, 0)
        buf = ctypes.create_string_buffer(int(n))
        L.lib().rtdm_detector_describe(h, buf, n)
        plan = buf.value.decode()
    finally:
        L.lib().rtdm_detector_destroy(h)
    assert plan.count("shortcut add") == 2, plan
    assert "res=-" in plan and not re.search(r"res=[^-]", plan), plan


def test_error_paths_return_status_not_abort():
    from rtdm import _lib as L
    lib = L.lib()
    h = ctypes.c_void_p()
    st = lib.rtdm_detector_create(b"[net]\n[convolutional]\nfilters=8\nsize=3\nstride=1\npad=1\n"
                                  b"activation=leaky\n[reorg3d]\n", 64, 64, 1, None, 0, 1, ctypes.byref(h))
    assert st == 4 and b"unsupported" in lib.rtdm_last_error()
    st = lib.rtdm_detector_create(b"garbage", 64, 64, 1, None, 0, 1, ctypes.byref(h))
    assert st == 1
    st = lib.rtdm_detector_create(cfg_text("yolov4-tiny-aider-416").encode(), 608, 608, 7, None, 0, 1,
                                  ctypes.byref(h))
    assert st == 1
    w = np.zeros(10, np.float32)
    st = lib.rtdm_detector_create(cfg_text("yolov4-tiny-aider-416").encode(), 608, 608, 1,
                                  w.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), 10, 1, ctypes.byref(h))
    assert st == 1 and b"weights" in lib.rtdm_last_error()
    assert lib.rtdm_nms(None, 1, 10, 7, 0.3, 0.4, 1, 0, 0, 10, None, 0, None, None, None, None) == 1
    assert lib.rtdm_classifier_create(9, 0, None, 0, 1, ctypes.byref(h)) == 1
    assert lib.rtdm_nms_workspace_size(2, 30324, 2) > 0


def test_nms_workspace_size_scales():
    from rtdm import _lib as L
    a = L.lib().rtdm_nms_workspace_size(1, 30324, 2)
    b = L.lib().rtdm_nms_workspace_size(64, 30324, 2)
    assert b == 64 * a


def _step_names(h):
    from rtdm import _lib as L
    out = []
    for i in range(L.lib().rtdm_detector_num_steps(h)):
        nm = ctypes.create_string_buffer(64)
        L.check(L.lib().rtdm_detector_step_info(h, i, nm, 64, None, None, None))
        out.append(nm.value.decode())
    return out


def test_tuning_is_per_handle():
    """the knobs a plan reads are per handle.  rtdm_set_tuning sets the process
    defaults a handle copies at creation; rtdm_detector_set_tuning changes one handle only.
    Checked through the kernel each step would launch (step_info names, host-side planning):
    the pooled stem of yolov4-tiny@608 is conv_stem3<true,1,k16> by default (the kh = 2 third of
    K on a 16-deep MFMA) and conv_stem3<true,1> with stem_k16 0."""
    from rtdm import _lib as L
    lib = L.lib()
    h1, _, _ = _plan("yolov4-tiny-aider-416", 608)
    h2, _, _ = _plan("yolov4-tiny-aider-416", 608)
    try:
        n1 = _step_names(h1)
        assert n1[0] == "conv_stem3<true,1,k16>" and "conv_pipew_f16<640,256>" in n1, n1
        L.check(lib.rtdm_detector_set_tuning(h2, b"stem_k16", 0))
        n2 = _step_names(h2)
        assert n2[0] == "conv_stem3<true,1>" and n2[1:] == n1[1:], n2
        assert _step_names(h1) == n1  # the other handle is unchanged
        assert lib.rtdm_detector_set_tuning(h2, b"no_such_key", 1) != 0
        # process defaults: a handle created after rtdm_set_tuning copies them; older ones keep theirs
        L.check(lib.rtdm_set_tuning(b"stem_k16", 0))
        try:
            h3, _, _ = _plan("yolov4-tiny-aider-416", 608)
            try:
                assert _step_names(h3)[0] == "conv_stem3<true,1>"
            finally:
                lib.rtdm_detector_destroy(h3)
            assert _step_names(h1) == n1
        finally:
            L.check(lib.rtdm_set_tuning(b"stem_k16", 1))
    finally:
        lib.rtdm_detector_destroy(h1)
        lib.rtdm_detector_destroy(h2)


def test_plan_time_keys_refused_on_live_handle():
    """fuse_head / two_streams are read when a handle is planned: rtdm_detector_set_tuning
    refuses them on a created handle (RTDM_E_INVALID) instead of accepting a silent no-op, and
    Darknet.set_tuning raises for them; rtdm_set_tuning (process defaults) still takes them."""
    from rtdm import _lib as L
    from rtdm.darknet import Darknet
    lib = L.lib()
    h, _, _ = _plan("yolov4-tiny-aider-416", 608)
    try:
        for key in (b"fuse_head", b"two_streams"):
            assert lib.rtdm_detector_set_tuning(h, key, 1) == 1
            assert b"plan-time" in lib.rtdm_last_error()
        L.check(lib.rtdm_detector_set_tuning(h, b"conv_pipe_cost", 1))  # launch-time keys still apply
    finally:
        lib.rtdm_detector_destroy(h)
    L.check(lib.rtdm_set_tuning(b"fuse_head", 0))
    m = Darknet(cfg_text("yolov4-tiny-aider-416"), (608, 608))
    with pytest.raises(ValueError, match="plan-time"):
        m.set_tuning("two_streams", 0)
