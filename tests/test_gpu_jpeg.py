"""GPU: device JPEG decode (rtdm_jpeg_reconstruct after the host entropy decode) against
the reference decode — cv2.imread's libjpeg-turbo defaults, which Pillow runs here
(victim_localization/yolov3/utils/datasets.py:97, disaster_detection/aider-predict.py:57):
bit-exact on the reference's 15 bundled JPEGs and on Pillow-encoded 4:4:4 / 4:2:2 /
4:2:0, restart-marker, optimised-table, grayscale and 1..33-pixel streams; BGR output as
cv2 returns it; progressive streams refused."""
import numpy as np
import pytest
import torch

from jpeg_cases import FIXTURES, pillow_rgb, progressive, variants

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "gpu tests need a HIP device"
    return torch.device("cuda:0")


def test_device_decode_bit_exact(dev):
    from rtdm import jpeg as J
    cases = [(f.rsplit("/", 1)[1], open(f, "rb").read()) for f in FIXTURES] + variants()
    assert len(cases) > 25
    outs = [(name, d, J.decode(d, dev)) for name, d in cases]  # all queued, then checked
    torch.cuda.synchronize()
    for name, d, out in outs:
        want = pillow_rgb(d)
        got = out.cpu().numpy()
        assert got.shape == want.shape, name
        assert np.array_equal(got, want), (name, int((got != want).sum()), int(np.abs(got.astype(int) - want).max()))


def test_device_decode_bgr_and_out_buffer(dev):
    from rtdm import jpeg as J
    d = open(FIXTURES[0], "rb").read()
    want = pillow_rgb(d)
    bgr = J.decode(d, dev, bgr=True).cpu().numpy()
    assert np.array_equal(bgr, want[..., ::-1])
    out = torch.full(want.shape, 7, dtype=torch.uint8, device=dev)
    assert J.decode(d, dev, out=out) is out
    assert np.array_equal(out.cpu().numpy(), want)
    with pytest.raises(ValueError):
        J.decode(d, dev, out=torch.empty((1, 1, 3), dtype=torch.uint8, device=dev))
    with pytest.raises(NotImplementedError):
        J.decode(progressive(), dev)
    with pytest.raises(ValueError):
        J.decode(d, "cpu")
