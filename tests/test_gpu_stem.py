"""GPU: the Cin-3 MFMA stems (csrc/conv.hip conv_stem3) with the kh = 2 third of K on one
16-deep MFMA (stem_k16 1, the default) against the 32-deep form (stem_k16 0) whose lane groups
2, 3 re-read kh = 2 pixels against zero weights.  The two compute the same nonzero products in
the same order, so every output must be BIT-IDENTICAL -- for every instantiation: the pooled
stem with the lean epilogue (yolov4-tiny / yolov3-tiny), the pooled stem with the swish
epilogue (yolov4-tiny-swish), the channel-major plain stem with two 16-channel tiles
(Darknet-53's 3 -> 32 conv) and the classifiers' stride-2 conv1.

Round 4 found NaN / wrong values with the 16-deep link (swish stem all-NaN io, classifier stem
83 % argmax): the link read the 32-deep MFMA's accumulator as SrcC back to back, across
opcodes, with no wait states (the compiler's hazard model inserts none for a full-register
SrcC overlap), so it read a stale accumulator.  conv.hip now keeps every chain's 32-deep link
before mfma_opcode_switch() and every 16-deep link after it.  Each case also asserts that the
K16 kernel is the one that ran (its step / describe name) and that the output is finite."""
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


# case -> the K16 stem kernel that must run (the stem is step 0)
DET_CASES = {
    "yolov4-tiny-aider-416@608:3": "conv_stem3<true,1,k16>",
    "yolov4-tiny-aider-416@608:64": "conv_stem3<true,1,k16>",
    "yolov4-tiny-aider-416@416:5": "conv_stem3<true,1,k16>",
    "yolov3-tiny-aider-416@416:2": "conv_stem3<true,1,k16>",
    "yolov4-tiny-aider-416@256:7": "conv_stem3<true,1,k16>",
    "yolov4-tiny-swish@416:2": "conv_stem3<true,1,k16>",  # swish epilogue (round 4: all-NaN io)
    "yolov3-aider-416@416:2": "conv_stem3<false,2,k16>",  # channel-major, two channel tiles
}


@pytest.mark.parametrize("case", list(DET_CASES))
def test_stem_k16_bit_identical(case):
    from rtdm import _lib as L
    from rtdm.synth import synth_frames
    cfg, rest = case.split("@")
    size, b = (int(v) for v in rest.split(":"))
    x = torch.from_numpy(synth_frames(b, size, size, seed=79)).cuda()
    preset = "he" if "swish" in cfg else "cond"
    outs, names = {}, {}
    for v in (0, 1):
        m, _, _, _ = _detector(cfg, size, preset=preset)
        m.set_tuning("stem_k16", v)  # this model's handles only
        outs[v] = m(x)[0].cpu()
        names[v] = _names(m, b)
    assert names[1][0] == DET_CASES[case], names[1][:2]
    assert names[0][0] == DET_CASES[case].replace(",k16", ""), names[0][:2]
    assert bool(torch.isfinite(outs[1]).all()), "non-finite io"
    assert torch.equal(outs[0], outs[1]), float((outs[0] - outs[1]).abs().max())


@pytest.mark.parametrize("name", ["squeeze-ernet", "squeeze-redconv", "ernet"])
@pytest.mark.parametrize("half", [True, False])
def test_classifier_stem_k16_bit_identical(name, half, cls_weights):
    """The classifiers' conv1 (3 -> 16, stride 2, channel-major) on frames through the CLI
    transform: logits bit-identical with stem_k16 0 / 1, the K16 kernel named in describe().
    (fp32 handles run the VALU stem: the knob must not change them either.)"""
    from rtdm.classifier import build_model
    from rtdm.synth import synth_frames
    frames = torch.from_numpy(synth_frames(16, 608, 608, seed=81)).cuda()
    logits = {}
    for v in (0, 1):
        m = build_model(name)
        m.load_state_dict(cls_weights[name])
        if half:
            m.half()
        m.set_tuning("stem_k16", v)
        logits[v] = m.classify_frames(frames).cpu()
        desc = m.describe(16)
        if half:
            want = "conv1 kernel conv_stem3<false,1" + (",k16>" if v else ">")
            assert want in desc, desc
    assert bool(torch.isfinite(logits[1]).all())
    assert torch.equal(logits[0], logits[1]), float((logits[0] - logits[1]).abs().max())
    assert np.array_equal(logits[0].argmax(1).numpy(), logits[1].argmax(1).numpy())


@pytest.mark.parametrize("name", ["squeeze-ernet", "squeeze-redconv", "ernet"])
@pytest.mark.parametrize("geom", [(16, 608, 608), (5, 720, 1280), (3, 100, 160), (2, 97, 131)])
def test_classifier_front_fused_bit_identical(name, geom, cls_weights):
    """The CLI transform + conv1 as one launch (resize_stream_kernel<.., STEM>, cls_front 1,
    the default) against two launches (resize_stream_kernel -> model input -> conv_stem3,
    cls_front 0): the fused kernel stages the same fp16 pixels in LDS and runs conv_stem3's
    K16 MFMA links and epilogue on them, so logits must be BIT-IDENTICAL -- downscale
    (608, 1280 wide), upscale (100 x 160) and a width whose rows are not 16-byte multiples
    (131: the fused path declines, both runs take two launches).  The 8-channel squeeze
    stem never fuses."""
    from rtdm.classifier import build_model
    from rtdm.synth import synth_frames
    b, hh, ww = geom
    frames = torch.from_numpy(synth_frames(b, hh, ww, seed=83)).cuda()
    logits = {}
    for v in (0, 1):
        m = build_model(name)
        m.load_state_dict(cls_weights[name])
        m.half()
        m.set_tuning("cls_front", v)
        logits[v] = m.classify_frames(frames).cpu()
        if v:
            desc = m.describe(b)
            assert ("conv1 on frames: fused with the transform" in desc) == (name != "squeeze-redconv"), desc
    assert bool(torch.isfinite(logits[1]).all())
    assert torch.equal(logits[0], logits[1]), float((logits[0] - logits[1]).abs().max())
