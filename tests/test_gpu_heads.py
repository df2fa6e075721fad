"""GPU: the YOLO head paths at the bench's batch.  yolov4-tiny@608 L28 -> L29 (3x3 conv 256 ->
128, then the 1x1 head 128 -> 28 + [yolo] decode) runs either as one fused launch
(conv_pipew0_f16<8,...>: the activated conv tile goes through LDS into the head GEMM) or as the
window conv (register epilogue, fp16 map) followed by head1x1_f16 (which at b64 takes 64 rows
per wave, head1x1_f16<4>).  Both take the same fp16 activations and the same K order, so io
must be BIT-IDENTICAL, at b64 (where the unfused head picks its 4-fragment waves) and b8."""
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


@pytest.mark.parametrize("b", [64, 8])
def test_fused_and_split_head_bit_identical(b):
    from rtdm import _lib as L
    from rtdm.synth import synth_frames
    x = torch.from_numpy(synth_frames(b, 608, 608, seed=79)).cuda()
    outs, names = {}, {}
    try:
        for v in (1, 0):  # plan-time knob: the process default a new handle is planned with
            L.check(L.lib().rtdm_set_tuning(b"fuse_head", v))
            m, _, _, _ = _detector("yolov4-tiny-aider-416", 608, preset="cond")
            outs[v] = m(x)[0].cpu()
            names[v] = _names(m, b)
    finally:
        L.check(L.lib().rtdm_set_tuning(b"fuse_head", 0))
    assert any(n.startswith("conv_pipew0_f16<8,") for n in names[1]), names[1]
    heads0 = [n for n in names[0] if n.startswith("head1x1_f16")]
    assert len(heads0) == 3, names[0]
    if b == 64:
        assert "head1x1_f16<4>" in heads0, heads0
    assert torch.equal(outs[0], outs[1]), float((outs[0] - outs[1]).abs().max())
