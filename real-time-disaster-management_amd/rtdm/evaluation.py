"""mAP@0.5 harness on the HIP runtime: counterpart of victim_localization/yolov3/test.py:11-197.

``test(cfg, data, weights, batch_size, img_size, conf_thres, iou_thres, model, dataloader)``
keeps the reference signature and return value ``((mp, mr, map, mf1, *loss), maps)``:
frames → rtdm Darknet → rtdm_nms → per-image matching + ap_per_class (rtdm.metrics).
The loss terms are 0: the rtdm detector is inference-only (test.py:103-104 only adds them
when the model carries training hyper-parameters).

Multi-GPU: where the reference wraps the model in nn.DataParallel when more than one GPU is
present (test.py:42-43: every batch split over the GPUs, outputs gathered to GPU 0), this
harness runs one process per GPU (``python -m torch.distributed.run --nproc-per-node N
test.py ...``): with a process group of world size > 1, rank r evaluates the contiguous
image shard [r·n/N, (r+1)·n/N) of the list file on its own GPU (cuda:LOCAL_RANK), and the
ranks' per-image stats are gathered and concatenated in rank order — the single-process
order — before ap_per_class, so every rank returns the single-process result.  A caller
passing its own ``dataloader`` under a process group passes that rank's shard.
"""
from __future__ import annotations

import os
import time

import numpy as np
import torch

from .metrics import DetectionStats
from .nms import non_max_suppression


def parse_data_cfg(path: str) -> dict:
    """utils/parse_config.py:55-71: key=value lines, '#' comments."""
    if not os.path.exists(path) and os.path.exists(os.path.join('data', path)):
        path = os.path.join('data', path)
    options = {}
    with open(path) as f:
        for line in f:
            line = line.strip()
            if not line or line.startswith('#'):
                continue
            key, val = line.split('=')
            options[key.strip()] = val.strip()
    return options


def load_classes(path: str):
    """utils.py:37-41."""
    with open(path) as f:
        return [x for x in f.read().split('\n') if x]


def _process_group():
    """(torch.distributed, world, rank) of an initialised group of more than one rank;
    (None, 1, 0) otherwise.  Under torch.distributed.run (WORLD_SIZE > 1 in the environment)
    the group is created here and owned by the process for its lifetime (test() may be called
    again): 'nccl' (RCCL) when every rank on this node has its own GPU (LOCAL_WORLD_SIZE <=
    the node's device count, so a multi-node launch keeps RCCL), else 'gloo'.  Only the gloo
    path is exercised by the tests (2 ranks sharing one GPU box); the RCCL path is unverified."""
    import torch.distributed as dist
    if not dist.is_available():
        return None, 1, 0
    if not dist.is_initialized() and int(os.environ.get("WORLD_SIZE", "1")) > 1:
        local = int(os.environ.get("LOCAL_RANK", "0"))
        own_gpu = torch.cuda.is_available() and torch.cuda.device_count() > local
        if own_gpu:
            torch.cuda.set_device(local)
        local_world = int(os.environ.get("LOCAL_WORLD_SIZE", os.environ["WORLD_SIZE"]))
        dist.init_process_group("nccl" if own_gpu and torch.cuda.device_count() >= local_world else "gloo")
    if dist.is_initialized() and dist.get_world_size() > 1:
        return dist, dist.get_world_size(), dist.get_rank()
    return None, 1, 0


def image_shard(n: int, world: int, rank: int):
    """Contiguous image range [lo, hi) of `rank` (the shards concatenate in rank order)."""
    return n * rank // world, n * (rank + 1) // world


def merge_stats(stats: DetectionStats, dist) -> DetectionStats:
    """Every rank's DetectionStats, concatenated in rank order (all ranks get the merge)."""
    parts = [None] * dist.get_world_size()
    dist.all_gather_object(parts, (stats.seen, stats.stats))
    out = DetectionStats(stats.nc, stats.clip)
    for seen, st in parts:
        out.seen += seen
        out.stats.extend(st)
    return out


def _frames_nhwc(imgs, device) -> torch.Tensor:
    """uint8 frames to the detector's NHWC input: RawFrames batches are letterboxed on the
    device; NCHW batches (the reference loader's layout) are viewed back to NHWC there."""
    if hasattr(imgs, "to_device"):
        return imgs.to_device(device)
    imgs = imgs.to(device, non_blocking=True)
    if imgs.dtype == torch.uint8 and imgs.dim() == 4 and imgs.shape[1] == 3 and imgs.shape[3] != 3:
        imgs = imgs.permute(0, 2, 3, 1).contiguous()
    return imgs


def test(cfg, data, weights=None, batch_size=16, img_size=416, conf_thres=0.001, iou_thres=0.6, model=None,
         dataloader=None, half=False, verbose=None, num_workers=4):
    from .darknet import Darknet, load_darknet_weights
    dist, world, rank = _process_group()
    if model is None:
        if not torch.cuda.is_available():
            raise RuntimeError("rtdm test.py runs on the HIP runtime: no GPU visible")
        device = torch.device('cuda', torch.cuda.current_device() if world > 1 else 0)
        verbose = (rank == 0) if verbose is None else verbose
        model = Darknet(cfg, img_size)
        if weights.endswith('.pt'):
            model.load_state_dict(torch.load(weights, map_location='cpu', weights_only=True)['model'])
        else:
            load_darknet_weights(model, weights)
        if half:
            model.half()
    else:
        device = torch.device('cuda', torch.cuda.current_device())
        verbose = False if verbose is None else verbose

    data = parse_data_cfg(data)
    nc = int(data['classes'])
    names = load_classes(data['names']) if os.path.exists(data.get('names', '')) else [str(i) for i in range(nc)]

    if dataloader is None:
        from .datasets import LoadImagesAndLabels
        dataset = LoadImagesAndLabels(data['valid'], img_size, batch_size)
        if world > 1:  # this rank's contiguous shard of the list file
            lo, hi = image_shard(len(dataset), world, rank)
            collate = dataset.collate_fn
            dataset = torch.utils.data.Subset(dataset, range(lo, hi))
            dataset.collate_fn = collate
        batch_size = max(1, min(batch_size, len(dataset)))
        dataloader = torch.utils.data.DataLoader(dataset, batch_size=batch_size, num_workers=num_workers,
                                                 pin_memory=False, collate_fn=dataset.collate_fn)

    stats = DetectionStats(nc)
    t0 = t1 = 0.0
    for imgs, targets, paths, shapes in dataloader:
        x = _frames_nhwc(imgs, device)
        height, width = x.shape[1:3] if x.dtype == torch.uint8 else x.shape[2:4]
        torch.cuda.synchronize()
        t = time.time()
        with torch.no_grad():
            inf_out, _ = model(x)
        torch.cuda.synchronize()
        t0 += time.time() - t
        t = time.time()
        output = non_max_suppression(inf_out, conf_thres=conf_thres, iou_thres=iou_thres)
        t1 += time.time() - t
        stats.update(output, targets, int(height), int(width))

    local_seen = stats.seen  # (the speed line: this rank's images and time)
    if world > 1:
        stats = merge_stats(stats, dist)
    r = stats.compute()
    pf = '%20s' + '%10.3g' * 6
    if rank != 0:
        verbose = False
    if rank == 0:
        print(('%20s' + '%10s' * 6) % ('Class', 'Images', 'Targets', 'P', 'R', 'mAP@0.5', 'F1'))
        print(pf % ('all', r['seen'], r['nt'].sum(), r['mp'], r['mr'], r['map'], r['mf1']))
    if verbose and nc > 1 and len(r['ap_class']):
        for i, c in enumerate(r['ap_class']):
            print(pf % (names[c], r['seen'], r['nt'][c], r['p'][i], r['r'][i], r['ap'][i], r['f1'][i]))
    if verbose and local_seen:
        ms = tuple(v / local_seen * 1e3 for v in (t0, t1, t0 + t1)) + (img_size, img_size, batch_size)
        print('Speed: %.1f/%.1f/%.1f ms inference/NMS/total per %gx%g image at batch-size %g' % ms)
    return (r['mp'], r['mr'], r['map'], r['mf1'], 0.0, 0.0, 0.0), np.asarray(r['maps'])
