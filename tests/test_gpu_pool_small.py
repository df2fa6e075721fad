"""GPU: 3x3 Cin 64 -> Cout 128 + 2x2 max-pool (yolov4-tiny / yolov3-tiny L6) on
conv3_pool_small<64,128,...,8 waves> (rtdm_set_tuning("pool_small64"), default on) against
conv_pipe's LDS-epilogue tile (0).  Both take each tap's 64 channels as two 32-deep MFMAs,
taps in order; bias -> LeakyReLU -> fp16 for the full map (yolov4-tiny's L6, read by a
route), the pool on the same values: the io must be BIT-IDENTICAL.  Also the halo prefetch
depth of the Cin-16 layer (pool_small_pf 1 vs the default 2)."""
import ctypes

import pytest
import torch

from test_gpu_pipeline import _detector

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


@pytest.mark.parametrize("knob", [("pool_small64", 0, 1), ("pool_small_pf", 1, 0)])
@pytest.mark.parametrize("case", ["yolov4-tiny-aider-416@608:3", "yolov4-tiny-aider-416@416:5",
                                  "yolov3-tiny-aider-416@416:2", "yolov4-tiny-aider-416@256:7"])
def test_pool_small_variants_bit_identical(case, knob):
    from rtdm import _lib as L
    from rtdm.synth import synth_frames
    key, v0, v1 = knob
    default = {"pool_small64": 1, "pool_small_pf": 0}[key]
    cfg, rest = case.split("@")
    size, b = (int(v) for v in rest.split(":"))
    x = torch.from_numpy(synth_frames(b, size, size, seed=83)).cuda()
    outs, names = {}, {}
    try:
        for v in (v0, v1):
            L.check(L.lib().rtdm_set_tuning(key.encode(), v))
            m, _, _, _ = _detector(cfg, size, preset="cond")
            outs[v] = m(x)[0].cpu()
            names[v] = _names(m, b)
    finally:
        L.check(L.lib().rtdm_set_tuning(key.encode(), default))
    if key == "pool_small64":
        assert "conv3_pool_small<64,128,8,4,2,1,8>" in names[1], names[1][:8]
        assert "conv3_pool_small<64,128,8,4,2,1,8>" not in names[0]
    assert torch.equal(outs[v0], outs[v1]), float((outs[v0] - outs[v1]).abs().max())


@pytest.mark.parametrize("case", ["yolov3-spp-aider@320:3", "yolov3-spp-aider@608:1", "yolov4-tiny-aider-416@608:3",
                                  "yolov3-tiny-aider-416@416:2"])
def test_spp_separable_maxpool_bit_identical(case):
    """Stride-1 max pools as separable band kernels (pool_sep 1, default: horizontal K-maxima
    per row once, then K of them per output) against the direct K x K kernel (0): the SPP
    block's 5 / 9 / 13 (-inf padding) and the tiny nets' 2 x 2 with Darknet's zero pad on the
    right / bottom.  max is exact over the same window, so the io is BIT-IDENTICAL."""
    from rtdm import _lib as L
    from rtdm.synth import synth_frames
    cfg, rest = case.split("@")
    size, b = (int(v) for v in rest.split(":"))
    x = torch.from_numpy(synth_frames(b, size, size, seed=89)).cuda()
    outs = {}
    try:
        for v in (0, 1):
            L.check(L.lib().rtdm_set_tuning(b"pool_sep", v))
            m, _, _, _ = _detector(cfg, size, preset="cond")
            outs[v] = m(x)[0].cpu()
    finally:
        L.check(L.lib().rtdm_set_tuning(b"pool_sep", 1))
    assert torch.equal(outs[0], outs[1]), float((outs[0] - outs[1]).abs().max())
