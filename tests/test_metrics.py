"""CPU: the mAP harness (rtdm.metrics / rtdm.evaluation) against golden vectors the
reference produced (tests/golden/make_map_golden.py): utils.ap_per_class / compute_ap on
seeded arrays, and the reference test.test driven end to end with seeded detector
output over the ODDER test-split labels.  float64 host reductions over identical
inputs: the bar is equality to 1e-12."""
import numpy as np
import pytest
import torch

from conftest import load_npz


@pytest.fixture(scope="module")
def g():
    return load_npz("map_golden.npz")


def _cases(g, prefix):
    return sorted({k.split("/")[1] for k in g if k.startswith(prefix + "/")})


def test_compute_ap_golden(g):
    from rtdm.metrics import compute_ap
    for c in _cases(g, "cap"):
        got = compute_ap(g[f"cap/{c}/recall"], g[f"cap/{c}/precision"])
        assert abs(got - float(g[f"cap/{c}/ap"])) <= 1e-12, c


def test_ap_per_class_golden(g):
    from rtdm.metrics import ap_per_class
    cases = _cases(g, "ap")
    assert {"basic", "extra_pred_cls", "iou10", "missing_cls", "empty_pred"} <= set(cases)
    for c in cases:
        p, r, ap, f1, cls = ap_per_class(g[f"ap/{c}/tp"], g[f"ap/{c}/conf"], g[f"ap/{c}/pred_cls"],
                                         g[f"ap/{c}/target_cls"])
        assert np.array_equal(cls, g[f"ap/{c}/cls"]), c
        for k, v in (("p", p), ("r", r), ("ap", ap), ("f1", f1)):
            ref = g[f"ap/{c}/{k}"]
            assert v.shape == ref.shape, (c, k)
            assert np.allclose(v, ref, rtol=0, atol=1e-12), (c, k)


def _batches(g):
    io = g["eval/io"]
    t = g["eval/targets"]
    nl = g["eval/n_labels"]
    bs = int(g["eval/batch"])
    starts = np.concatenate([[0], np.cumsum(nl)])
    for b0 in range(0, io.shape[0], bs):
        idx = range(b0, min(b0 + bs, io.shape[0]))
        yield b0, io[b0:b0 + bs], np.concatenate([t[starts[i]:starts[i + 1]] for i in idx])


def _ref_survivors(g, name):
    cnt = g[f"eval/{name}/nms_count"]
    det = g[f"eval/{name}/nms_det"]
    off = np.concatenate([[0], np.cumsum(cnt)])
    return [None if c == 0 else det[off[i]:off[i + 1]] for i, c in enumerate(cnt)]


@pytest.mark.parametrize("name", ["default", "strict"])
def test_detection_stats_match_reference_test_py(g, name):
    """DetectionStats on the reference's own NMS survivors reproduces test.test's
    (P, R, mAP@0.5, F1) and per-class maps."""
    from rtdm.metrics import DetectionStats
    surv = _ref_survivors(g, name)
    img = int(g["eval/img"])
    st = DetectionStats(nc=len(g[f"eval/{name}/maps"]))
    for b0, io, t in _batches(g):
        st.update(surv[b0:b0 + io.shape[0]], torch.from_numpy(t), img, img)
    r = st.compute()
    got = np.array([r["mp"], r["mr"], r["map"], r["mf1"]])
    assert np.allclose(got, g[f"eval/{name}/result"], rtol=0, atol=1e-12), (got, g[f"eval/{name}/result"])
    assert np.allclose(r["maps"], g[f"eval/{name}/maps"], rtol=0, atol=1e-12)
    assert r["seen"] == g["eval/io"].shape[0]


@pytest.mark.parametrize("name", ["default", "strict"])
def test_oracle_nms_reproduces_captured_survivors(g, name):
    """The survivors captured inside the reference test.py equal the oracle NMS on the
    stored io (so the GPU test can start from io and rtdm_nms)."""
    from oracle import nms as ON
    conf, iou = g[f"eval/{name}/conf_iou"]
    ref = _ref_survivors(g, name)
    got = ON.non_max_suppression(g["eval/io"], float(conf), float(iou))
    for a, b in zip(got, ref):
        assert (a is None) == (b is None)
        if a is not None:
            assert np.array_equal(a, b)


def test_match_image_edge_cases():
    """test.py:133-160 rules: a target is taken once; a prediction whose best target is
    taken is not re-assigned; IoU must exceed 0.5 strictly; classes never cross."""
    from rtdm.metrics import match_image
    lab = np.array([[0, 0.5, 0.5, 0.2, 0.2], [1, 0.2, 0.2, 0.1, 0.1]], np.float32)
    box = [40, 40, 60, 60]   # target 0 in a 100x100 frame
    pred = np.array([box + [0.9, 0], box + [0.8, 0], [45, 45, 65, 65, 0.7, 0], box + [0.6, 1]], np.float32)
    c = match_image(pred, lab, 100, 100)
    assert c[:, 0].tolist() == [True, False, False, False]
    # exactly IoU 0.5 is not a match: a box of half the target's area inside it
    half = np.array([[40, 40, 60, 50, 0.9, 0]], np.float32)
    assert not match_image(half, lab, 100, 100)[0, 0]
    assert match_image(np.zeros((0, 6), np.float32), lab, 100, 100).shape == (0, 1)
    assert not match_image(pred, np.zeros((0, 5), np.float32), 100, 100).any()


def test_detection_stats_empty():
    from rtdm.metrics import DetectionStats
    st = DetectionStats(nc=2)
    st.update([None, None], torch.zeros((0, 6)), 64, 64)
    r = st.compute()
    assert r["seen"] == 2 and r["map"] == 0.0 and np.array_equal(r["maps"], [0.0, 0.0])


def test_letterbox_geometry():
    """datasets.py:599-631 geometry (ratio, unpadded size, padding split; rtdm_letterbox_geometry
    against the oracle restatement over many shapes and flags), the LoadImagesAndLabels
    composition (load_image shrink + square pad), and utils.py:123-136 scale_coords
    inverting it; labels re-normalised like datasets.py:441-482."""
    from oracle import letterbox as OL
    from rtdm.letterbox import dataset_geometry, geometry, labels_to_letterbox, scale_coords
    rng = np.random.default_rng(5)
    shapes = [(300, 500), (480, 640), (416, 416), (1080, 1920), (200, 100), (833, 411), (5, 7)]
    shapes += [tuple(int(v) for v in rng.integers(1, 2000, 2)) for _ in range(40)]
    for (h, w) in shapes:
        for new in (416, 608, (320, 416)):
            for auto in (True, False):
                for up in (True, False):
                    assert geometry(h, w, new, auto, False, up) == OL.geometry(h, w, new, auto, False, up), \
                        (h, w, new, auto, up)
    g, (h, w), ratio, pad = dataset_geometry(300, 500, 416)
    assert (h, w) == (int(300 * 416 / 500), 416) and ratio == (1.0, 1.0)
    assert g == (h, w, 416, 416, int(round(pad[1] - 0.1)), 0) and pad == (0.0, (416 - h) / 2)
    assert dataset_geometry(200, 300, 416)[0][:2] == (200, 300)     # never grows
    lab = np.array([[1, 0.5, 0.5, 0.2, 0.4]], np.float32)
    ll = labels_to_letterbox(lab, ratio, pad, h, w, 416, 416)
    assert np.allclose(ll[0], [1, 0.5, 0.5, 0.2, 0.4 * h / 416], atol=1e-6)
    gn = 416 / 500
    py = (416 - 300 * gn) / 2    # scale_coords' own padding (from the source shape, not load_image's int())
    box = torch.tensor([[100.0, 50.0 + py, 200.0, 150.0 + py]])
    back = scale_coords((416, 416), box.clone(), (300, 500))
    assert torch.allclose(back, torch.tensor([[100 / gn, 50 / gn, 200 / gn, 150 / gn]]), atol=1e-3)
    far = scale_coords((416, 416), torch.tensor([[-50.0, -50.0, 900.0, 900.0]]), (300, 500))
    assert far[0, 0] < 0 and far[0, 2] > 500    # reference clip_coords is a no-op


def test_oracle_letterbox_resize_properties():
    """Known answers for the INTER_AREA restatement: integral shrink = rounded box mean;
    constant frames stay constant in all three modes; pad colour outside the frame."""
    from oracle import letterbox as OL
    rng = np.random.default_rng(3)
    img = rng.integers(0, 256, (64, 96, 3), dtype=np.uint8)
    fast = OL.resize_area(img, 48, 32)
    mean = img.reshape(32, 2, 48, 2, 3).astype(np.float64).mean(axis=(1, 3))
    assert np.abs(fast.astype(np.float64) - mean).max() <= 0.5
    for (nw, nh) in ((48, 32), (37, 29), (150, 100), (80, 100)):
        c = np.full((64, 96, 3), 77, np.uint8)
        assert (OL.resize_area(c, nw, nh) == 77).all(), (nw, nh)
    out = OL.letterbox(img, OL.geometry(64, 96, 128, auto=False), color=(1, 2, 3))
    assert out.shape == (128, 128, 3) and (out[0, 0] == [1, 2, 3]).all()


def test_classification_metrics_known_answer():
    """evaluate-classification-metrics.py:106-130 definitions on a hand-checked matrix
    (per-class P = tp/(tp+fp), R = tp/(tp+fn), 0 when undefined); the torchmetrics
    summary (micro average) is the fraction correct (torchmetrics absent: unpinned)."""
    from rtdm.cli import classification_metrics
    preds = [0, 0, 1, 2, 2, 2, 4, 4]
    targs = [0, 1, 1, 2, 3, 2, 4, 0]
    m = classification_metrics(preds, targs)
    assert m["accuracy"] == 5 / 8 and m["f1_score"] == 5 / 8
    assert m["collapsed building_precision"] == 0.5 and m["collapsed building_recall"] == 0.5
    assert m["fire_precision"] == 1.0 and m["fire_recall"] == 0.5
    assert m["flooded areas_precision"] == 2 / 3 and m["flooded areas_recall"] == 1.0
    assert m["normal_precision"] == 0 and m["normal_recall"] == 0 and m["normal_f1"] == 0
    assert abs(m["flooded areas_f1"] - 0.8) < 1e-12
