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
    """datasets.py:599-631 geometry (ratio, unpadded size, padding split) and
    utils.py:123-136 scale_coords inverting it; labels re-normalised like
    datasets.py:441-482."""
    from rtdm.letterbox import labels_to_letterbox, letterbox, load_image, scale_coords
    img0 = np.random.default_rng(0).integers(0, 255, (300, 500, 3), dtype=np.uint8)
    img, (h0, w0), (h, w) = load_image(img0, 416)
    assert (h0, w0) == (300, 500) and (h, w) == (int(300 * 416 / 500), 416)
    out, ratio, pad = letterbox(img, 416, auto=False, scaleup=False)
    assert out.shape == (416, 416, 3) and ratio == (1.0, 1.0)
    assert pad == (0.0, (416 - h) / 2)
    assert (out[0] == 128).all() and (out[-1] == 128).all()
    out_auto, _, pad_a = letterbox(img0, 416)           # LoadImages (detect.py) form
    assert out_auto.shape[1] == 416 and out_auto.shape[0] % 32 == 0
    lab = np.array([[1, 0.5, 0.5, 0.2, 0.4]], np.float32)
    ll = labels_to_letterbox(lab, ratio, pad, h, w, 416, 416)
    assert np.allclose(ll[0], [1, 0.5, 0.5, 0.2, 0.4 * h / 416], atol=1e-6)
    g = 416 / 500
    py = (416 - 300 * g) / 2     # scale_coords' own padding (from the source shape, not load_image's int())
    box = torch.tensor([[100.0, 50.0 + py, 200.0, 150.0 + py]])
    back = scale_coords((416, 416), box.clone(), (300, 500))
    assert torch.allclose(back, torch.tensor([[100 / g, 50 / g, 200 / g, 150 / g]]), atol=1e-3)
    far = scale_coords((416, 416), torch.tensor([[-50.0, -50.0, 900.0, 900.0]]), (300, 500))
    assert far[0, 0] < 0 and far[0, 2] > 500    # reference clip_coords is a no-op


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
