"""GPU: the fused stem pair (csrc/stem_fused.hip conv_stem_pool2: pooled stem 3 -> 16 + the
16 -> 32 pooled 3x3 conv that reads its map, one launch) against the two unfused kernels
(conv_stem3<true> + conv3_pool_small<16,32>, rtdm_set_tuning("stem_fuse", 0)).  The fused
kernel recomputes each tile's stem halo but every value takes the unfused kernels' operations
in their order, so the io must be BIT-IDENTICAL: batches with several images (tiles at image
borders on every side), 608 / 416 / 256 frames, both tiny cfgs with the pattern.  The swish
cfg (non-lean stem epilogue) and NCHW float inputs keep the unfused pair."""
import ctypes

import numpy as np
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


@pytest.mark.parametrize("case", ["yolov4-tiny-aider-416@608:3", "yolov4-tiny-aider-416@608:64",
                                  "yolov4-tiny-aider-416@416:5", "yolov3-tiny-aider-416@416:2",
                                  "yolov4-tiny-aider-416@256:7", "yolov4-tiny-swish@416:2"])
def test_stem_pair_fused_bit_identical(case):
    from rtdm import _lib as L
    from rtdm.synth import synth_frames
    cfg, rest = case.split("@")
    size, b = (int(v) for v in rest.split(":"))
    x = torch.from_numpy(synth_frames(b, size, size, seed=71)).cuda()
    outs, names = {}, {}
    try:
        for v in (0, 1):
            L.check(L.lib().rtdm_set_tuning(b"stem_fuse", v))
            m, _, _, _ = _detector(cfg, size, preset="cond" if "swish" not in cfg else "he")
            outs[v] = m(x)[0].cpu()
            names[v] = _names(m, b)
    finally:
        L.check(L.lib().rtdm_set_tuning(b"stem_fuse", 0))
    assert "conv_stem_pool2" not in names[0], names[0]
    fused = "conv_stem_pool2" in names[1]
    assert fused == ("swish" not in cfg), names[1]
    if fused:
        i = names[1].index("conv_stem_pool2")
        assert names[1][i + 1] == "conv_stem_pool2:fused", names[1]
        assert names[0][i].startswith("conv_stem3") and names[0][i + 1].startswith("conv3_pool_small<16,32"), names[0]
    assert torch.equal(outs[0], outs[1]), float((outs[0] - outs[1]).abs().max())


def test_stem_pair_fused_layer_output_and_nchw():
    """The fused-away pooled stem map is refused by layer_output (not silently stale); NCHW
    float input runs the unfused pair, whose io equals the frame path's (x / 255 exact)."""
    from rtdm import _lib as L
    from rtdm.synth import synth_frames
    frames = synth_frames(2, 608, 608, seed=73)
    x = torch.from_numpy(frames).cuda()
    m, _, _, _ = _detector("yolov4-tiny-aider-416", 608, preset="cond")
    m.set_tuning("stem_fuse", 1)  # this model's handles only
    io_u8 = m(x)[0].clone()
    with pytest.raises(L.RtdmError, match="fused away"):
        m.layer_output(1, 2)
    m.layer_output(3, 2)  # the second conv's pooled map (layer 3) is written
    h = m.handle(2)
    ctypes_io = torch.empty_like(io_u8)
    xf = (torch.from_numpy(frames).permute(0, 3, 1, 2).float() / 255.0).contiguous().cuda()
    L.check(L.lib().rtdm_detect(h, L.ptr(xf), L.RTDM_INPUT_NCHW_F32, 2, L.ptr(ctypes_io), L.stream_ptr()))
    torch.cuda.synchronize()
    m.layer_output(1, 2)  # unfused this time: the map exists
    d = (ctypes_io - io_u8).abs()  # the float frames round to fp16 in the stem: the fp16 bar
    assert float(d[..., :4].max()) <= 0.5 and float(d[..., 4:].max()) <= 2e-2, float(d.max())



@pytest.mark.parametrize("knob", [("stem_persist", 0, 1, "conv_stem3p<1>"), ("stem_k16", 0, 1, None)])
@pytest.mark.parametrize("case", ["yolov4-tiny-aider-416@608:3", "yolov4-tiny-aider-416@416:5",
                                  "yolov3-tiny-aider-416@416:2", "yolov4-tiny-aider-416@256:7"])
def test_stem_variants_bit_identical(case, knob):
    """Pooled uint8 stem variants against conv_stem3<true> with its defaults: conv_stem3p
    (persistent: the next band's frame bytes in flight while the current band computes;
    rtdm_set_tuning("stem_persist", 1); measured slower, off by default), and the kh = 2 third
    of K as a 32-deep MFMA (stem_k16 0) instead of the default 16-deep one (the same nonzero
    products).  BIT-IDENTICAL io."""
    from rtdm import _lib as L
    from rtdm.synth import synth_frames
    key, base, alt, name = knob
    cfg, rest = case.split("@")
    size, b = (int(v) for v in rest.split(":"))
    x = torch.from_numpy(synth_frames(b, size, size, seed=79)).cuda()
    outs, names = {}, {}
    try:
        for v in (base, alt):
            L.check(L.lib().rtdm_set_tuning(key.encode(), v))
            m, _, _, _ = _detector(cfg, size, preset="cond")
            outs[v] = m(x)[0].cpu()
            names[v] = _names(m, b)
    finally:
        L.check(L.lib().rtdm_set_tuning(key.encode(), {"stem_persist": 0, "stem_k16": 1}[key]))
    assert names[base][0].startswith("conv_stem3<true"), names[base][:2]
    if name:
        assert names[alt][0] == name, names[alt][:2]
    assert torch.equal(outs[base], outs[alt]), float((outs[base] - outs[alt]).abs().max())
