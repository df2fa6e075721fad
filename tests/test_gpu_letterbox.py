"""GPU: rtdm_letterbox (device INTER_AREA resize + pad, datasets.py:599-631) bit-exact
against the numpy restatement (oracle/letterbox.py) in all three resize modes (area,
integral area-fast, growing linear), with pitched rows, BGR input, pad colours and
batches; and the LoadImagesAndLabels → RawFrames → device path of the mAP harness.
Pixel parity with cv2 itself is unpinned (cv2 absent; see oracle/letterbox.py)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "gpu tests need a HIP device"
    return torch.device("cuda:0")


CASES = [  # (in_h, in_w, new_shape, auto, scale_fill, scaleup)
    (480, 640, 416, True, False, True),      # video frame -> area, auto pad to /32
    (480, 640, 608, False, False, True),     # area, square canvas
    (832, 832, 416, False, False, True),     # integral 2x -> area-fast
    (1248, 1664, 416, True, False, True),    # integral 4x
    (1080, 1920, 608, True, False, True),    # 3.16x area
    (200, 300, 416, True, False, True),      # grow -> linear
    (300, 500, 416, False, True, True),      # scaleFill: x shrinks, y grows -> linear
    (417, 415, 416, False, False, False),    # near-identity area
    (416, 416, 416, False, False, True),     # identity
    (7, 5, 64, False, False, True),          # tiny grow
]


@pytest.mark.parametrize("case", CASES)
def test_letterbox_matches_oracle(dev, case):
    from oracle import letterbox as OL
    from rtdm.letterbox import geometry, letterbox_frames
    h, w, new, auto, fill, up = case
    g = geometry(h, w, new, auto, fill, up)
    assert g == OL.geometry(h, w, new, auto, fill, up)
    rng = np.random.default_rng(h * 7 + w)
    frames = rng.integers(0, 256, (3, h, w, 3), dtype=np.uint8)
    frames[1] = (np.arange(w)[None, :, None] * 255 // max(1, w - 1)).astype(np.uint8)   # smooth ramp
    got = letterbox_frames(torch.from_numpy(frames).to(dev), g, color=(128, 128, 128)).cpu().numpy()
    for i in range(3):
        ref = OL.letterbox(frames[i], g)
        assert np.array_equal(got[i], ref), (case, i, int(np.abs(got[i].astype(int) - ref).max()))


def test_letterbox_pitch_bgr_pad(dev):
    """Rows with padding (a view into a wider buffer), BGR input, non-grey pad."""
    from oracle import letterbox as OL
    from rtdm.letterbox import geometry, letterbox_frames
    rng = np.random.default_rng(1)
    wide = torch.from_numpy(rng.integers(0, 256, (2, 360, 700, 3), dtype=np.uint8)).to(dev)
    frames = wide[:, :, :640]                              # pitch 2100 bytes, width 640
    g = geometry(360, 640, 416, auto=False)
    got = letterbox_frames(frames, g, color=(10, 20, 30), bgr=True).cpu().numpy()
    host = frames.cpu().numpy()
    for i in range(2):
        ref = OL.letterbox(host[i][..., ::-1].copy(), g, color=(10, 20, 30))
        assert np.array_equal(got[i], ref)
    assert (got[:, 0, 0] == [10, 20, 30]).all()


def test_letterbox_rejects_bad_geometry(dev):
    from rtdm import _lib as L
    from rtdm.letterbox import letterbox_frames
    x = torch.zeros((1, 10, 10, 3), dtype=torch.uint8, device=dev)
    with pytest.raises(L.RtdmError):
        letterbox_frames(x, (20, 20, 16, 16, 0, 0))       # resized frame larger than the canvas
    with pytest.raises(L.RtdmError):
        letterbox_frames(torch.zeros((1, 400, 400, 3), dtype=torch.uint8, device=dev), (21, 21, 21, 21, 0, 0))  # 19x: > 16 taps


def test_dataset_raw_frames_on_device(dev, tmp_path):
    """LoadImagesAndLabels counterpart: decoded frames letterboxed on the GPU equal the
    oracle's load_image shrink + square pad; labels re-normalised to the padded frame."""
    from PIL import Image

    from oracle import letterbox as OL
    from rtdm.datasets import LoadImagesAndLabels
    rng = np.random.default_rng(2)
    (tmp_path / "images").mkdir()
    (tmp_path / "labels").mkdir()
    sizes = [(300, 500), (480, 640), (416, 200)]
    names = []
    for i, (h, w) in enumerate(sizes):
        Image.fromarray(rng.integers(0, 256, (h, w, 3), dtype=np.uint8)).save(tmp_path / "images" / f"f{i}.png")
        (tmp_path / "labels" / f"f{i}.txt").write_text("1 0.5 0.5 0.2 0.4\n0 0.25 0.3 0.1 0.1\n")
        names.append(f"images/f{i}.png")
    lst = tmp_path / "list.txt"
    lst.write_text("\n".join(names) + "\n")
    ds = LoadImagesAndLabels(str(lst), 416, 4, root=str(tmp_path))
    imgs, targets, paths, shapes = ds.collate_fn([ds[i] for i in range(len(ds))])
    x = imgs.to_device(dev).cpu().numpy()
    for i, (h0, w0) in enumerate(sizes):
        src = np.asarray(Image.open(tmp_path / names[i]).convert("RGB"))
        r = 416 / max(h0, w0)
        h, w = (int(h0 * r), int(w0 * r)) if r < 1 else (h0, w0)
        ref = OL.letterbox(src, (h, w) + OL.geometry(h, w, 416, auto=False, scaleup=False)[2:])
        assert np.array_equal(x[i], ref), i
    assert targets.shape == (6, 6) and targets[:, 0].tolist() == [0, 0, 1, 1, 2, 2]
    # the padded axis shrinks the normalised height of a label (300x500 -> 249x416 in 416x416)
    assert abs(float(targets[0, 5]) - 0.4 * int(300 * 416 / 500) / 416) < 1e-6
