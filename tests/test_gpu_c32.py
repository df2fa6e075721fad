"""GPU: the Cin-32 3x3 convs of Darknet-53 (yolov3 / yolov3-spp L1: 32 -> 64 stride 2; L3:
32 -> 64 + shortcut) on conv3_c32 (csrc/conv_c32.hip, rtdm_set_tuning("conv_c32"), default
on) against the kernels they ran on before (conv_mfma for L1, conv3_direct for L3), and the
first residual block (L2 1x1 64 -> 32, L3, the shortcut) as one conv3_c32r launch
("res_fuse", default on) against conv_mfma + conv3_c32, and the two 104 x 104 residual blocks
(1x1 128 -> 64, 3x3 64 -> 128, shortcut) as conv3_c64r launches against conv_mfma + conv_pipe.  Every path takes each tap's 32
channels as one 32-deep MFMA (the 1x1's 64 channels as two), in order, then bias ->
LeakyReLU (rounded to fp32) -> (+ residual) -> fp16, so the io must be BIT-IDENTICAL;
batches of several images (halo tiles at every image border), 416 and 608 frames, and a
frame alone equal to its row in the batch."""
import ctypes

import pytest
import torch

from test_gpu_config3 import _model

pytestmark = pytest.mark.gpu

DEFAULTS = {"conv_c32": 1, "res_fuse": 1}


def _names(m, n):
    from rtdm import _lib as L
    h = m.handle(n)
    out = []
    for i in range(L.lib().rtdm_detector_num_steps(h)):
        nm = ctypes.create_string_buffer(64)
        L.check(L.lib().rtdm_detector_step_info(h, i, nm, 64, None, None, None))
        out.append(nm.value.decode())
    return out


def _run(settings, img, b, seed):
    """io and step names per tuning dict (process defaults set before each model's handle is
    created, restored after)."""
    from rtdm import _lib as L
    from rtdm.synth import BASE_SEED, synth_frames
    x = torch.from_numpy(synth_frames(b, img, img, seed=BASE_SEED + seed)).cuda()
    outs, names = [], []
    try:
        for st in settings:
            for k, v in st.items():
                L.check(L.lib().rtdm_set_tuning(k.encode(), v))
            m, _ = _model(img=img)
            outs.append(m(x)[0].float().cpu())
            names.append(_names(m, b))
    finally:
        for k, v in DEFAULTS.items():
            L.check(L.lib().rtdm_set_tuning(k.encode(), v))
    return x, outs, names


@pytest.mark.parametrize("img,b", [(416, 3), (608, 2)])
def test_c32_bit_identical(img, b):
    x, outs, names = _run([{"conv_c32": 0, "res_fuse": 0}, {"conv_c32": 1, "res_fuse": 0},
                           {"conv_c32": 1, "res_fuse": 1}, {"conv_c32": 1, "res_fuse": 3}], img, b, 811)
    assert not any(nm.startswith("conv3_c32") for nm in names[0])
    c32 = [nm for nm in names[1] if nm.startswith("conv3_c32")]
    assert c32 == ["conv3_c32<2,false>", "conv3_c32<1,true>"], names[1][:6]
    c32r = [nm for nm in names[2] if nm.startswith("conv3_c32")]
    assert c32r == ["conv3_c32<2,false>", "conv3_c32r", "conv3_c32r:fused"], names[2][:6]
    # the two 104 x 104 (416) / 152 x 152 (608) blocks on conv3_c64r; res_fuse 3 keeps them apart
    assert [nm for nm in names[2] if nm.startswith("conv3_c64r")] == ["conv3_c64r", "conv3_c64r:fused"] * 2
    assert not any(nm.startswith("conv3_c64r") for nm in names[3])
    assert [nm for nm in names[3] if nm.startswith("conv3_c32")] == c32r
    for k in (1, 2, 3):
        d = (outs[0] - outs[k]).abs()
        assert torch.equal(outs[0], outs[k]), (k, float(d[..., :4].max()), float(d[..., 4:].max()))
    # a frame alone (defaults): the same rows
    m, _ = _model(img=img)
    io1 = m(x[b - 1:b].contiguous())[0].float().cpu()
    assert torch.equal(io1[0], outs[2][b - 1])


def test_c32r_layer_output_refused():
    """The reduce map fused away by conv3_c32r is refused by layer_output (not stale)."""
    from rtdm import _lib as L
    from rtdm.synth import BASE_SEED, synth_frames
    x = torch.from_numpy(synth_frames(2, 416, 416, seed=BASE_SEED + 812)).cuda()
    m, _ = _model(img=416)
    m(x)
    with pytest.raises(L.RtdmError, match="fused away"):
        m.layer_output(2, 2)
    m.layer_output(1, 2)
