"""GPU: conv_wide (csrc/conv_wide.hip), the 256 x 256-tile window-mode twin of conv_pipew for
the big 3x3 / s1 layers.  Every output is the same K-ordered fp32 dot product as conv_pipe's,
so the detector's io must be bit-identical with the wide tiles on or off:
  * rtdm_set_tuning("conv_wide", 2): every eligible layer on 256 x 256 tiles;
  * ("conv_wide", 3): whole rounds of wide tiles + the remaining wide units as 256 x 128
    conv_pipew tiles in a second launch (the split the latency cost model picks at b64);
  * ("conv_wide", 0): conv_pipe alone (the reference of the comparison).
Batches cover partial last tiles, tiles spanning image boundaries, workgroups walking several
tiles, the Darknet-53 residual 3x3s (fused shortcut, ABL 896) and 13 / 19 / 26 / 38-wide maps."""
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


@pytest.mark.parametrize("case", ["yolov4-tiny-aider-416@608:3", "yolov4-tiny-aider-416@608:24",
                                  "yolov3-aider-416@416:5", "yolov3-spp-aider@608:2"])
def test_wide_tiles_bit_identical(case):
    from rtdm import _lib as L
    from rtdm.synth import synth_frames
    cfg, rest = case.split("@")
    size, b = (int(v) for v in rest.split(":"))
    x = torch.from_numpy(synth_frames(b, size, size, seed=61)).cuda()
    outs, names = {}, {}
    try:
        for v in (0, 2, 3):
            L.check(L.lib().rtdm_set_tuning(b"conv_wide", v))
            m, _, _, _ = _detector(cfg, size)
            outs[v] = m(x)[0].cpu()
            names[v] = _names(m, b)
    finally:
        L.check(L.lib().rtdm_set_tuning(b"conv_wide", 0))
    assert not any(n.startswith("conv_wide") for n in names[0]), names[0]
    assert any(n.startswith("conv_wide") for n in names[2]), names[2]
    if cfg.startswith("yolov3-aider"):
        assert any(n.startswith("conv_wide_f16<896>") for n in names[2]), names[2]
    for v in (2, 3):
        assert torch.equal(outs[0], outs[v]), (v, float((outs[0] - outs[v]).abs().max()))


def test_wide_plan_at_bench_batch():
    """The cost model at the bench's b64 (latency objective): L10 / L14 (182 wide tiles) all
    wide, L12 / L21 (364 / 361 wide units over 256 CUs) split; and the b64 forward with the
    model's plan equals conv_pipe's bits."""
    from rtdm import _lib as L
    from rtdm.synth import synth_frames
    x = torch.from_numpy(synth_frames(64, 608, 608, seed=67)).cuda()
    outs = {}
    try:
        for v in (0, 1):
            L.check(L.lib().rtdm_set_tuning(b"conv_wide", v))
            m, _, _, _ = _detector("yolov4-tiny-aider-416", 608, preset="cond")
            outs[v] = m(x)[0].cpu()
            if v == 1:
                names = _names(m, 64)
    finally:
        L.check(L.lib().rtdm_set_tuning(b"conv_wide", 0))
    print("b64 plan:", [n for n in names if "conv" in n])
    assert sum(n.startswith("conv_wide") for n in names) >= 2, names
    assert torch.equal(outs[0], outs[1])
