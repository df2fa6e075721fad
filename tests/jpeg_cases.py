"""JPEG decode cases shared by the CPU and GPU tests: the reference's bundled JPEGs
(tests/golden/jpeg, copied by tests/golden/copy_jpeg_fixtures.py) and Pillow-encoded
variants of one of them covering the other stream features the decoder handles."""
import glob
import io
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
FIXTURES = sorted(glob.glob(os.path.join(HERE, "golden", "jpeg", "*.jpg")))


def pillow_rgb(data: bytes) -> np.ndarray:
    """The reference decode: libjpeg-turbo with its defaults (cv2.imread's, as BGR)."""
    from PIL import Image
    with Image.open(io.BytesIO(data)) as im:
        return np.asarray(im.convert("RGB"))


def variants():
    """(name, bytes) of Pillow-encoded streams: 4:4:4 / 4:2:2 / 4:2:0, restart markers,
    optimised Huffman tables, low / high quality, grayscale, odd and tiny sizes."""
    from PIL import Image
    src = pillow_rgb(open(os.path.join(HERE, "golden", "jpeg", "normal_image2085.jpg"), "rb").read())
    out = []

    def enc(name, arr, **kw):
        b = io.BytesIO()
        Image.fromarray(arr).save(b, "JPEG", **kw)
        out.append((name, b.getvalue()))

    crop = src[:117, :203]
    enc("444", crop, subsampling=0)
    enc("422", crop, subsampling=1)
    enc("420_restart3", crop, subsampling=2, restart_marker_blocks=3)
    enc("420_restart_rows", src[:75, :91], subsampling=2, restart_marker_rows=1)
    enc("420_optimize_q95", crop, subsampling=2, optimize=True, quality=95)
    enc("420_q20", crop, subsampling=2, quality=20)
    enc("422_q100", crop, subsampling=1, quality=100)
    enc("gray", np.ascontiguousarray(crop[..., 1]))
    for w, h in ((1, 1), (2, 3), (3, 2), (5, 4), (17, 9), (33, 31)):
        enc(f"420_{w}x{h}", np.ascontiguousarray(src[:h, :w]), subsampling=2)
        enc(f"422_{w}x{h}", np.ascontiguousarray(src[:h, :w]), subsampling=1)
    return out


def progressive():
    from PIL import Image
    b = io.BytesIO()
    Image.fromarray(np.zeros((16, 16, 3), np.uint8)).save(b, "JPEG", progressive=True)
    return b.getvalue()
