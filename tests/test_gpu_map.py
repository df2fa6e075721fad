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


def _rank_worker(rank, world, port, tmp, q):
    """One rank of rtdm.evaluation.test's multi-GPU path (the process group is created by the
    harness from the torch.distributed.run environment; both ranks share the box's one GPU,
    so the group is gloo)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world), RANK=str(rank),
                      LOCAL_RANK=str(rank))
    import torch.distributed as dist
    try:
        from rtdm.evaluation import image_shard, test
        g = load_npz("map_golden.npz")
        io, t, nl = g["eval/io"], g["eval/targets"], g["eval/n_labels"]
        bs, img = int(g["eval/batch"]), int(g["eval/img"])
        starts = np.concatenate([[0], np.cumsum(nl)])
        lo, hi = image_shard(io.shape[0], world, rank)
        out = {}
        for name in ("default", "strict"):
            loader, queue = [], []
            for b0 in range(lo, hi, bs):
                idx = range(b0, min(b0 + bs, hi))
                tb = np.concatenate([t[starts[i]:starts[i + 1]] for i in idx]).copy()
                k = 0
                for j, i in enumerate(idx):  # batch-relative image column (datasets.py collate)
                    tb[k:k + nl[i], 0] = j
                    k += nl[i]
                loader.append((torch.zeros((len(idx), img, img, 3), dtype=torch.uint8), torch.from_numpy(tb), None,
                               None))
                queue.append(torch.from_numpy(io[b0:b0 + len(idx)]).cuda())

            class StandIn:
                def __call__(self, x):
                    return queue.pop(0), None

            conf, iou = g[f"eval/{name}/conf_iou"]
            res, maps = test(None, os.path.join(tmp, "odder.data"), batch_size=bs, img_size=img,
                             conf_thres=float(conf), iou_thres=float(iou), model=StandIn(), dataloader=loader)
            out[name] = (list(res[:4]), np.asarray(maps).tolist(), not queue, dist.get_backend())
        q.put((rank, out))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def test_rtdm_test_harness_two_ranks(tmp_path):
    """The multi-GPU harness (rank r evaluates its contiguous image shard, the per-image stats
    are merged in rank order): two ranks on this box's GPU reproduce the reference test.test
    result for the stored detector output on every rank, NMS on the device."""
    import torch.multiprocessing as mp
    (tmp_path / "odder.names").write_text("person\nvehicle\n")
    (tmp_path / "odder.data").write_text(f"classes=2\nvalid=none.txt\nnames={tmp_path / 'odder.names'}\n")
    g = load_npz("map_golden.npz")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 31500 + os.getpid() % 1000
    procs = [ctx.Process(target=_rank_worker, args=(r, 2, port, str(tmp_path), q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(2)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for _, out in res:
        for name in ("default", "strict"):
            vals, maps, drained, backend = out[name]
            assert drained and backend == "gloo"
            assert np.allclose(vals, g[f"eval/{name}/result"], rtol=0, atol=1e-12), (name, vals)
            assert np.allclose(maps, g[f"eval/{name}/maps"], rtol=0, atol=1e-12)
