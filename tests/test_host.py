"""CPU: host-side logic — weight formats, synthetic data determinism, frame
sharding and the multi-process (gloo, world_size 2) weight broadcast / result gather."""
import os
import sys

import numpy as np
import pytest
import torch

from conftest import ROOT, cfg_text


def test_synth_frames_deterministic_and_shardable():
    from rtdm.synth import synth_frames
    a = synth_frames(4, 64, 80)
    b = np.concatenate([synth_frames(2, 64, 80, first=0), synth_frames(2, 64, 80, first=2)])
    assert a.dtype == np.uint8 and a.shape == (4, 64, 80, 3)
    assert np.array_equal(a, b)
    assert a.std() > 10


def test_darknet_weight_file_roundtrip(tmp_path):
    from rtdm.synth import read_darknet_weights, synth_darknet_weights, write_darknet_weights
    s = synth_darknet_weights(cfg_text("yolov3-tiny-aider-416"))
    p = tmp_path / "x.weights"
    write_darknet_weights(str(p), s)
    assert os.path.getsize(p) == 20 + 4 * s.size
    assert np.array_equal(read_darknet_weights(str(p)), s)


def test_state_dict_to_stream_order():
    """{'model': state_dict} checkpoints map onto the darknet stream order (save_weights)."""
    from oracle.darknet import DarknetRef
    from rtdm.darknet import state_dict_to_stream
    from rtdm.synth import synth_darknet_weights
    text = cfg_text("yolov4-tiny-aider-416")
    s = synth_darknet_weights(text)
    ref = DarknetRef(text, s)
    sd = {}
    for i, p in ref.params.items():
        if "gamma" in p:
            sd[f"module_list.{i}.BatchNorm2d.bias"] = p["beta"]
            sd[f"module_list.{i}.BatchNorm2d.weight"] = p["gamma"]
            sd[f"module_list.{i}.BatchNorm2d.running_mean"] = p["mean"]
            sd[f"module_list.{i}.BatchNorm2d.running_var"] = p["var"]
        else:
            sd[f"module_list.{i}.Conv2d.bias"] = p["bias"]
        sd[f"module_list.{i}.Conv2d.weight"] = p["w"]
    assert np.array_equal(state_dict_to_stream(text, sd), s)


def test_classifier_state_dict_validation(cls_weights):
    from rtdm.classifier import build_model, load_model
    m = build_model("squeeze-ernet")
    m.load_state_dict(cls_weights["squeeze-ernet"])
    bad = dict(cls_weights["squeeze-ernet"])
    bad.pop("fc.bias")
    with pytest.raises(RuntimeError):
        build_model("squeeze-ernet").load_state_dict(bad)
    with pytest.raises(RuntimeError):
        build_model("ernet").load_state_dict(cls_weights["squeeze-ernet"])
    with pytest.raises(ValueError):
        build_model("resnet")
    with pytest.raises(FileNotFoundError):
        load_model("ernet", "/nonexistent.pt", "cpu")


def test_cpu_tensor_input_fails_loudly(cls_weights):
    from rtdm.classifier import build_model
    m = build_model("squeeze-ernet")
    m.load_state_dict(cls_weights["squeeze-ernet"])
    with pytest.raises(RuntimeError):
        m(torch.zeros(1, 3, 140, 140))


def test_shard_range_partitions():
    from rtdm.distributed import shard_range
    for gb in (1, 7, 64, 128):
        for world in (1, 2, 3, 8):
            covered = []
            for r in range(world):
                s, c = shard_range(gb, world, r)
                covered += list(range(s, s + c))
            assert covered == list(range(gb))


def _dist_worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from rtdm.distributed import broadcast_state_dict, gather_results, shard_range
        from rtdm.synth import classifier_param_shapes, synth_classifier_state_dict, synth_frames
        shapes = classifier_param_shapes("ernet")
        sd = synth_classifier_state_dict("ernet") if rank == 0 else None
        got = broadcast_state_dict(sd, shapes, device="cpu")
        ref = synth_classifier_state_dict("ernet")
        ok = all(np.array_equal(got[k], ref[k]) for k in shapes)
        s, c = shard_range(8, world, rank)
        frames = synth_frames(c, 32, 32, first=s)
        rec = {"sum": torch.tensor([float(frames.sum())]), "rank": torch.tensor([rank])}
        out = gather_results(rec)
        # bench.py's per-step gather: one flat record per rank (float fields + int32 bit
        # patterns), unpacked on rank 0
        from rtdm.distributed import gather_records
        from rtdm.pipeline import TwoStagePipeline, unpack_record
        # (a detector placeholder: the layout has det / idx / count fields only with one;
        # record_layout reads nothing else from it)
        pipe = TwoStagePipeline(None, object(), max_det=7)
        lay, total_len = pipe.record_layout(c)
        mine = unpack_record(torch.zeros(total_len), pipe, c)
        mine["logits"][:] = torch.arange(c * 5, dtype=torch.float32).view(c, 5) + 100 * rank
        mine["det"][:] = float(rank) + 0.5
        mine["idx"][:] = torch.arange(c * 7 * 2, dtype=torch.int32).view(c, 7, 2) - rank
        mine["count"][:] = torch.arange(s, s + c, dtype=torch.int32)
        allrec = gather_records(mine["record"])
        if rank == 0:
            for r in range(world):
                u = unpack_record(allrec[r], pipe, c)
                ok = ok and torch.equal(u["logits"], torch.arange(c * 5, dtype=torch.float32).view(c, 5) + 100 * r)
                ok = ok and bool((u["det"] == float(r) + 0.5).all())
                ok = ok and torch.equal(u["idx"], torch.arange(c * 14, dtype=torch.int32).view(c, 7, 2) - r)
                ok = ok and torch.equal(u["count"], torch.arange(r * c, r * c + c, dtype=torch.int32))
            total = sum(float(t.item()) for t in out["sum"])
            q.put((ok, total, [int(t.item()) for t in out["rank"]]))
        else:
            q.put((ok, None, None))
    finally:
        dist.destroy_process_group()


def test_two_rank_gloo_broadcast_and_gather():
    import torch.multiprocessing as mp
    from rtdm.synth import synth_frames
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + os.getpid() % 1000
    procs = [ctx.Process(target=_dist_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(2)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(r[0] for r in res)
    total = [r for r in res if r[1] is not None][0]
    assert total[1] == float(synth_frames(8, 32, 32).sum())
    assert total[2] == [0, 1]


def test_yolo_acff_stream_from_reference_state_dict():
    """The reference Darknet state_dict of a YOLO-ACFF cfg (module_list.i.Conv2d/BatchNorm2d
    and module_list.i.acff_i.* keys) maps to the same inline stream as the synthetic path,
    and the C++ planner asks for exactly that many floats."""
    from rtdm.darknet import Darknet, state_dict_to_stream
    from rtdm.synth import (ACFF_KEYS, conv_layers, inline_acff, synth_acff_params,
                            synth_darknet_weights)
    text = cfg_text("yolov3-acffx")
    conv = synth_darknet_weights(text)
    acff = synth_acff_params(text)
    sd, ptr = {}, 0
    for (i, cin, cout, k, bn, head) in conv_layers(text):
        p = f"module_list.{i}."
        if bn:
            for name in ("bias", "weight", "running_mean", "running_var"):
                sd[p + "BatchNorm2d." + name] = conv[ptr:ptr + cout]
                ptr += cout
        else:
            sd[p + "Conv2d.bias"] = conv[ptr:ptr + cout]
            ptr += cout
        sd[p + "Conv2d.weight"] = conv[ptr:ptr + cout * cin * k * k].reshape(cout, cin, k, k)
        ptr += cout * cin * k * k
    for i, prm in acff.items():
        for key in ACFF_KEYS:
            sd[f"module_list.{i}.acff_{i}.{key}"] = prm[key]
    stream = inline_acff(text, conv, acff)
    assert np.array_equal(state_dict_to_stream(text, sd), stream)
    assert Darknet(text, (416, 416)).info.weight_floats == stream.size



REF_WEIGHTS = "/root/reference/code/disaster_detection/weights"


@pytest.mark.skipif(not os.path.isdir(REF_WEIGHTS), reason="reference checkpoints not present")
@pytest.mark.parametrize("model,pickle_name", [("squeeze-ernet", "Squeeze-ernet-92f1score.pt"),
                                               ("squeeze-redconv", "Squeeze-ernet-redconv92acc.pt"),
                                               ("ernet", "ernet-96f1scor.pt")])
def test_full_module_pickle_loads_allowlisted(model, pickle_name, cls_weights):
    """The reference's full-module pickles load through torch.load(weights_only=True) with
    the allowlist (no code from the file runs) and give the same tensors as the state-dict
    checkpoints (*-state_dict.pt are bit-identical to these)."""
    from rtdm.classifier import build_model, read_weights
    sd = read_weights(os.path.join(REF_WEIGHTS, pickle_name))
    ref = cls_weights[model]
    assert set(sd) == set(ref)
    for k in ref:
        assert np.array_equal(sd[k].numpy(), ref[k]), k
    build_model(model).load_state_dict(sd)  # strict key / shape check


def test_read_weights_checkpoint_formats(tmp_path, cls_weights):
    """Plain state dict, {'model_state_dict': ...} and .npz all give the same tensors."""
    from rtdm.classifier import read_weights
    sd = {k: torch.from_numpy(v) for k, v in cls_weights["ernet"].items()}
    torch.save(sd, tmp_path / "a.pt")
    torch.save({"model_state_dict": sd, "epoch": 3}, tmp_path / "b.pt")
    np.savez(tmp_path / "c.npz", **cls_weights["ernet"])
    for f in ("a.pt", "b.pt", "c.npz"):
        got = read_weights(str(tmp_path / f))
        assert all(np.array_equal(np.asarray(got[k]), cls_weights["ernet"][k]) for k in cls_weights["ernet"]), f


def _map_worker(rank, world, port, q):
    """One rank of the sharded mAP harness (rtdm.evaluation): its contiguous image shard of the
    reference's stored detector output, NMS by the CPU oracle, DetectionStats merged over the
    gloo group."""
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from conftest import load_npz
        from oracle import nms as ON
        from rtdm.evaluation import image_shard, merge_stats
        from rtdm.metrics import DetectionStats
        g = load_npz("map_golden.npz")
        io, t, nl = g["eval/io"], g["eval/targets"], g["eval/n_labels"]
        img = int(g["eval/img"])
        starts = np.concatenate([[0], np.cumsum(nl)])
        lo, hi = image_shard(io.shape[0], world, rank)
        res = {}
        for name in ("default", "strict"):
            conf, iou = g[f"eval/{name}/conf_iou"]
            st = DetectionStats(2)
            for b0 in range(lo, hi, 3):  # batches of 3 inside the shard
                idx = range(b0, min(b0 + 3, hi))
                tb = np.concatenate([t[starts[i]:starts[i + 1]] for i in idx]).copy()
                # the image column is batch-relative (datasets.py collate)
                k = 0
                for j, i in enumerate(idx):
                    tb[k:k + nl[i], 0] = j
                    k += nl[i]
                out = ON.non_max_suppression(io[b0:b0 + len(idx)], float(conf), float(iou))
                st.update(out, tb, img, img)
            merged = merge_stats(st, dist)
            r = merged.compute()
            res[name] = (merged.seen, [r["mp"], r["mr"], r["map"], r["mf1"]], np.asarray(r["maps"]).tolist())
        q.put((rank, res))
    finally:
        dist.destroy_process_group()


def test_two_rank_gloo_map_harness_shards():
    """rtdm.evaluation's multi-GPU path (one process per GPU instead of the reference's
    nn.DataParallel, yolov3/test.py:42-43): each rank's contiguous image shard, stats merged in
    rank order, gives the reference test.test's (P, R, mAP@0.5, F1) and maps for the stored
    detector output (tests/golden/map_golden.npz) on every rank."""
    import torch.multiprocessing as mp
    from conftest import load_npz
    from rtdm.evaluation import image_shard
    g = load_npz("map_golden.npz")
    n = g["eval/io"].shape[0]
    for world in (1, 2, 3, 5):
        cover = []
        for r in range(world):
            lo, hi = image_shard(n, world, r)
            cover += list(range(lo, hi))
        assert cover == list(range(n))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 30500 + os.getpid() % 1000
    procs = [ctx.Process(target=_map_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in range(2)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for _, rr in res:
        for name in ("default", "strict"):
            seen, vals, maps = rr[name]
            assert seen == n
            assert np.allclose(vals, g[f"eval/{name}/result"], rtol=0, atol=1e-12), (name, vals)
            assert np.allclose(maps, g[f"eval/{name}/maps"], rtol=0, atol=1e-12)


def _bench(args, env_extra=None, timeout=180):
    import subprocess
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env, capture_output=True,
                          text=True, timeout=timeout)


def test_bench_gpus_n_starts_n_ranks():
    """`bench.py --gpus 2` starts two ranks itself (no torch.distributed.run), each with its
    own RANK / LOCAL_RANK and the shared WORLD_SIZE / MASTER_*, and the parent prints exactly
    one JSON line, rank 0's, with n_gpus 2 (yolov3/test.py:42-43)."""
    import json
    r = _bench(["--gpus", "2", "--dry-run"])
    assert r.returncode == 0, r.stderr
    lines = [l for l in r.stdout.splitlines() if l.strip()]
    assert len(lines) == 1, r.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["dry_run"] is True
    envs = rec["ranks"]
    assert [e["RANK"] for e in envs] == ["0", "1"] and [e["LOCAL_RANK"] for e in envs] == ["0", "1"]
    assert all(e["WORLD_SIZE"] == "2" and e["MASTER_ADDR"] == "127.0.0.1" for e in envs)
    assert envs[0]["MASTER_PORT"] == envs[1]["MASTER_PORT"]


def test_bench_rank_failure_propagates():
    r = _bench(["--gpus", "2", "--dry-run", "--dry-fail-rank", "1"])
    assert r.returncode != 0
    assert "rank 1 exited with status 3" in r.stderr
    assert r.stdout.strip() == ""


def test_bench_world_size_must_match_gpus():
    r = _bench(["--gpus", "4", "--dry-run"], {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0 and "WORLD_SIZE=2 but --gpus 4" in r.stderr
    r = _bench(["--dry-run"])  # no --gpus, no launcher: one rank
    assert r.returncode == 0 and '"n_gpus": 1' in r.stdout
