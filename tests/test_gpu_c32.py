"""GPU: the Cin-32 3x3 convs of Darknet-53 (yolov3 / yolov3-spp L1: 32 -> 64 stride 2; L3:
32 -> 64 + shortcut) on conv3_c32 (csrc/conv_c32.hip, rtdm_set_tuning("conv_c32"), default
on) against the kernels they ran on before (conv_mfma for L1, conv3_direct for L3).  Every
path takes each tap's 32 channels as one 32-deep MFMA, taps in order, then bias ->
LeakyReLU (rounded to fp32) -> (+ residual) -> fp16, so the io must be BIT-IDENTICAL;
batches of several images (halo tiles at every image border), 416 and 608 frames, and a
frame alone equal to its row in the batch."""
import ctypes

import pytest
import torch

from test_gpu_config3 import _model

pytestmark = pytest.mark.gpu


def _names(m, n):
    from rtdm import _lib as L
    h = m.handle(n)
    out = []
    for i in range(L.lib().rtdm_detector_num_steps(h)):
        nm = ctypes.create_string_buffer(64)
        L.check(L.lib().rtdm_detector_step_info(h, i, nm, 64, None, None, None))
        out.append(nm.value.decode())
    return out


def _run(key, vals, img, b, seed):
    """io and step names per value of a plan-time knob (process default set before the
    model's handle is created, restored after)."""
    from rtdm import _lib as L
    from rtdm.synth import BASE_SEED, synth_frames
    x = torch.from_numpy(synth_frames(b, img, img, seed=BASE_SEED + seed)).cuda()
    outs, names = {}, {}
    default = {"conv_c32": 1}[key]
    try:
        for v in vals:
            L.check(L.lib().rtdm_set_tuning(key.encode(), v))
            m, _ = _model(img=img)
            outs[v] = m(x)[0].float().cpu()
            names[v] = _names(m, b)
    finally:
        L.check(L.lib().rtdm_set_tuning(key.encode(), default))
    return x, outs, names


@pytest.mark.parametrize("img,b", [(416, 3), (608, 2)])
def test_c32_bit_identical(img, b):
    x, outs, names = _run("conv_c32", (0, 1), img, b, 811)
    c32 = [i for i, nm in enumerate(names[1]) if nm.startswith("conv3_c32")]
    assert [names[1][i] for i in c32] == ["conv3_c32<2,false>", "conv3_c32<1,true>"], names[1][:6]
    assert not any(nm.startswith("conv3_c32") for nm in names[0])
    d = (outs[0] - outs[1]).abs()
    assert torch.equal(outs[0], outs[1]), (float(d[..., :4].max()), float(d[..., 4:].max()))
    # a frame alone: the same rows
    m, _ = _model(img=img)
    io1 = m(x[b - 1:b].contiguous())[0].float().cpu()
    assert torch.equal(io1[0], outs[1][b - 1])

