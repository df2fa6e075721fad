"""GPU: the mAP harness on the HIP runtime — rtdm.evaluation.test (test.py:11-197
counterpart) with rtdm_nms on the device, against the (P, R, mAP@0.5, F1) and maps the
reference test.test returned for the same detector output and labels
(tests/golden/map_golden.npz).  A stand-in model returns the stored io, so the check
covers NMS on the GPU + matching + ap_per_class end to end."""
import os

import numpy as np
import pytest
import torch

from conftest import load_npz

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", ["default", "strict"])
def test_rtdm_test_harness_matches_reference(name, tmp_path):
    from rtdm.evaluation import test
    g = load_npz("map_golden.npz")
    assert torch.cuda.is_available(), "gpu tests need a HIP device"
    io = g["eval/io"]
    t = g["eval/targets"]
    nl = g["eval/n_labels"]
    bs = int(g["eval/batch"])
    img = int(g["eval/img"])
    starts = np.concatenate([[0], np.cumsum(nl)])
    loader, queue = [], []
    for b0 in range(0, io.shape[0], bs):
        idx = range(b0, min(b0 + bs, io.shape[0]))
        frames = torch.zeros((len(idx), img, img, 3), dtype=torch.uint8)
        loader.append((frames, torch.from_numpy(np.concatenate([t[starts[i]:starts[i + 1]] for i in idx])),
                       None, None))
        queue.append(torch.from_numpy(io[b0:b0 + bs]).cuda())

    class StandIn:
        def __call__(self, x):
            assert x.is_cuda and x.dtype == torch.uint8 and x.shape[1:] == (img, img, 3)
            return queue.pop(0), None

    (tmp_path / "odder.names").write_text("person\nvehicle\n")
    data = tmp_path / "odder.data"
    data.write_text(f"classes=2\nvalid=none.txt\nnames={tmp_path / 'odder.names'}\n")
    conf, iou = g[f"eval/{name}/conf_iou"]
    res, maps = test(None, str(data), batch_size=bs, img_size=img, conf_thres=float(conf), iou_thres=float(iou),
                     model=StandIn(), dataloader=loader)
    assert not queue
    ref = g[f"eval/{name}/result"]
    assert np.allclose(np.array(res[:4]), ref, rtol=0, atol=1e-12), (res[:4], ref)
    assert np.allclose(maps, g[f"eval/{name}/maps"], rtol=0, atol=1e-12)
    assert os.path.exists(data)
