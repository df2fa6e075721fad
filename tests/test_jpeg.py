"""CPU: the JPEG decode oracle (oracle/jpeg.py) pinned against Pillow — the reference's
cv2.imread decode (victim_localization/yolov3/utils/datasets.py:97) is libjpeg-turbo with
its defaults, which Pillow links too — and the C-ABI host stage (header parse + Huffman
entropy decode, rtdm_jpeg_info_get / rtdm_jpeg_entropy_decode) bit-exact against the
oracle's coefficients.  The device stage is tests/test_gpu_jpeg.py."""
import numpy as np
import pytest

from jpeg_cases import FIXTURES, pillow_rgb, progressive, variants


def _cases():
    return [(f.rsplit("/", 1)[1], open(f, "rb").read()) for f in FIXTURES] + variants()


def test_fixtures_present():
    assert len(FIXTURES) == 15


def test_oracle_matches_pillow():
    from oracle import jpeg as OJ
    for name, d in _cases():
        got, want = OJ.decode(d), pillow_rgb(d)
        assert got.shape == want.shape and np.array_equal(got, want), (name, int((got != want).sum()))


def test_host_entropy_decode_matches_oracle():
    from oracle import jpeg as OJ
    from rtdm import jpeg as J
    for name, d in _cases():
        coef, qt, inf = J.entropy_decode(d)
        oc, oq = OJ.coefficients(d)
        assert np.array_equal(coef.numpy(), oc), name
        assert np.array_equal(qt.numpy().view(np.uint16)[:inf.ncomp], oq), name
        want = pillow_rgb(d)
        assert (inf.height, inf.width) == want.shape[:2] and inf.supported == 1, name


def test_unsupported_and_corrupt_streams_refused():
    from rtdm import _lib as L
    from rtdm import jpeg as J
    p = progressive()
    assert J.supported(p) is False and J.info(p).supported == 0
    with pytest.raises(NotImplementedError):
        J.entropy_decode(p)
    with pytest.raises(L.RtdmError):
        J.info(b"\x00\x01not a jpeg")
    with pytest.raises(L.RtdmError):
        J.info(b"\xff\xd8\xff\xd9")  # SOI EOI: no frame
    # truncated entropy data decodes (zeros past the end, as libjpeg) without error
    d = open(FIXTURES[0], "rb").read()
    coef, _, _ = J.entropy_decode(d[:len(d) // 2])
    assert coef.shape[1] == 64
