#!/usr/bin/env python3
"""Two-stage aerial-frame inference benchmark (BASELINE.json metric).

One step = one batch of synthetic 608x608 uint8 frames through the whole hot
path on the GPU: classifier CLI transform + ACFF classifier (ErNET by default),
Darknet detector of record (yolov4-tiny-aider-416.cfg run at 608x608; /255
fused), YOLO decode (fused into the head convs) and per-image NMS (conf 0.3,
IoU 0.4, detect.py defaults).  Frames are resident in HBM before timing.

  python bench.py [--gpus N] [--steps K] [--warmup W]
  N>1: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N
       (one rank per GPU; each rank processes its own shard of frames —
       batch 64 per GPU, weak scaling; weights broadcast once over RCCL).

Prints ONE JSON line on rank 0 (value = frames/s over all ranks), with
  roofline:     the dominant kernel (largest summed device time in the timed
                region, measured with hipEvents on the launch stream) against
                the dense fp16 MFMA peak
  cpu_baseline: the CPU oracle (torch-CPU restatement of the reference path,
                incl. NMS) timed on a bounded sample on this host, rank 0 only.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "real-time-disaster-management_amd"))

MFMA_F16_DENSE_PEAK_TFLOPS = 2500.0  # MI355X_MICROARCH.md: ~2.5 PF dense bf16/fp16
HBM_PEAK_GBS = 8000.0
CLASSIFIER_FLOP = {"squeeze-ernet": 90953544.0, "squeeze-redconv": 77593080.0, "ernet": 319307650.0}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=64, help="frames per GPU per step")
    ap.add_argument("--img", type=int, default=608)
    ap.add_argument("--cfg", default="yolov4-tiny-aider-416")
    ap.add_argument("--classifier", default="ernet", choices=["ernet", "squeeze-ernet", "squeeze-redconv"])
    ap.add_argument("--dtype", default="f16", choices=["f16", "f32"])
    ap.add_argument("--conf", type=float, default=0.3)
    ap.add_argument("--iou", type=float, default=0.4)
    ap.add_argument("--max-det", type=int, default=300)
    ap.add_argument("--overlap", type=int, default=1,
                    help="1: classifier on a side stream beside the detector; 0: both stages serial")
    ap.add_argument("--priority", type=int, default=0,
                    help="1: detector + NMS on a high-priority stream, classifier on a low-priority one")
    ap.add_argument("--step-events", type=int, default=1,
                    help="0: no per-step hipEvents in the timed region (roofline fields then null)")
    ap.add_argument("--cpu-baseline", type=int, default=1, help="0 disables the CPU oracle leg")
    ap.add_argument("--cpu-seconds", type=float, default=15.0,
                    help="CPU oracle leg: time chunks of 16 frames until this much CPU time has passed")
    return ap.parse_args()


def dist_setup(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    return world, rank, local


def build(args, world, rank):
    from rtdm.classifier import build_model
    from rtdm.darknet import Darknet
    from rtdm.pipeline import TwoStagePipeline
    from rtdm.synth import (inline_acff, load_calibration, synth_acff_params, synth_classifier_state_dict,
                            synth_darknet_weights)

    cfg_path = os.path.join(ROOT, "real-time-disaster-management_amd", "rtdm", "cfg", args.cfg + ".cfg")
    text = open(cfg_path).read()
    det = Darknet(text, (args.img, args.img))
    cls = build_model(args.classifier)
    # rank 0 makes the weights; RCCL broadcast to the other ranks (once, untimed)
    if rank == 0:
        calib = load_calibration(args.cfg)
        conv, acff = synth_darknet_weights(text, calib=calib), synth_acff_params(text, calib=calib)
        stream = inline_acff(text, conv, acff)  # YOLO-ACFF cfgs: [acff] params inline
        args.ref_weights = (conv, acff)         # the CPU oracle takes them apart
        sd = synth_classifier_state_dict(args.classifier)
    else:
        stream, sd = None, None
    if world > 1:
        import torch.distributed as dist
        n = torch.tensor([det.info.weight_floats], device="cuda")
        t = torch.from_numpy(stream).cuda() if rank == 0 else torch.empty(int(n.item()), device="cuda")
        dist.broadcast(t, 0)
        stream = t.cpu().numpy()
        keys = sorted(synth_classifier_state_dict(args.classifier).keys())
        flat = torch.cat([torch.from_numpy(sd[k]).reshape(-1) for k in keys]).cuda() if rank == 0 else None
        shapes = {k: v.shape for k, v in synth_classifier_state_dict(args.classifier).items()}
        total = sum(int(np.prod(shapes[k])) for k in keys)
        if rank != 0:
            flat = torch.empty(total, device="cuda")
        dist.broadcast(flat, 0)
        flat = flat.cpu().numpy()
        sd, o = {}, 0
        for k in keys:
            c = int(np.prod(shapes[k]))
            sd[k] = flat[o:o + c].reshape(shapes[k])
            o += c
    det.load_weight_stream(stream)
    cls.load_state_dict(sd)
    if args.dtype == "f16":
        det.half()
        cls.half()
    pipe = TwoStagePipeline(cls, det, args.conf, args.iou, args.max_det, overlap=bool(args.overlap),
                            priority=bool(args.priority))
    return pipe, det, cls, text, stream, sd


def step_table(det, n):
    from rtdm import _lib as L
    h = det.handle(n)
    ns = L.lib().rtdm_detector_num_steps(h)
    rows = []
    for i in range(ns):
        name = ctypes.create_string_buffer(128)
        layer, flop, byt = ctypes.c_int(), ctypes.c_double(), ctypes.c_double()
        L.check(L.lib().rtdm_detector_step_info(h, i, name, 128, ctypes.byref(layer), ctypes.byref(flop),
                                                ctypes.byref(byt)))
        rows.append((name.value.decode(), layer.value, flop.value * n, byt.value * n))
    return h, rows


def pmc_traffic(kernel):
    """HBM bytes per launch of `kernel` from the newest committed PMC summary
    (profiles/*_traffic.json, written by tools/prof_summary.py from separate
    rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over this same bench command;
    FETCH_SIZE doubled per the gfx950 correction).  None when no pass covers it."""
    import glob
    base = kernel.split("<")[0]
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*_traffic.json")))  # tags sort by round
    for path in reversed(files):
        try:
            d = json.load(open(path))
        except (OSError, ValueError):
            continue
        for k, t in d.items():
            if k.split("<")[0] == base and "fetch_size_bytes_avg" in t and "write_size_bytes_avg" in t:
                return {"bytes_per_launch": t["hbm_bytes_avg"], "source": os.path.relpath(path, ROOT)}
    return None


def cpu_baseline(args, text, stream, sd):
    """Oracle leg: the torch-CPU restatement of the reference path (preprocess + classifier +
    Darknet + decode + NMS) on a bounded sample of the same workload."""
    sys.path.insert(0, ROOT)
    from oracle import classifier as OC
    from oracle import nms as ON
    from oracle import preprocess as OP
    from oracle.darknet import DarknetRef
    from rtdm.synth import synth_frames
    cores = int(os.environ.get("OMP_NUM_THREADS") or len(os.sched_getaffinity(0)))
    torch.set_num_threads(cores)
    conv, acff = getattr(args, "ref_weights", (stream, {}))
    ref = DarknetRef(text, conv, acff)
    s = 240 if args.classifier == "ernet" else 140
    sdt = {k: torch.from_numpy(np.asarray(v, np.float32)) for k, v in sd.items()}

    def run(frames):
        x = torch.from_numpy(np.stack([OP.cli_transform(f, s) for f in frames]))
        with torch.no_grad():
            OC.forward(args.classifier, sdt, x)
            io = ref.forward(torch.from_numpy(frames).permute(0, 3, 1, 2).float() / 255.0)
        ON.non_max_suppression(io.numpy(), args.conf, args.iou)

    warm = synth_frames(2, args.img, args.img, seed=1)
    run(warm)
    chunk, done, dt = 16, 0, 0.0
    while dt < args.cpu_seconds and done < 64 * 16:
        frames = synth_frames(chunk, args.img, args.img, first=done)
        t0 = time.perf_counter()
        run(frames)
        dt += time.perf_counter() - t0
        done += chunk
    return {"value": round(done / dt, 3), "unit": "frames/s", "cores": cores, "kind": "port",
            "sample": f"first {done} frames of the same synthetic {args.img}x{args.img} workload in chunks of {chunk}, "
                      f"fp32 torch-CPU oracle ({args.classifier} + {args.cfg} + decode + NMS), {dt:.1f} s"}


def main():
    args = parse()
    world, rank, local = dist_setup(args)
    from rtdm.synth import synth_frames
    dev = torch.device("cuda", torch.cuda.current_device())
    pipe, det, cls, text, stream, sd = build(args, world, rank)
    b = args.batch
    frames = torch.from_numpy(synth_frames(b, args.img, args.img, first=rank * b)).to(dev)
    torch.cuda.synchronize()
    for _ in range(args.warmup):
        pipe(frames)
    torch.cuda.synchronize()
    h, steps = step_table(det, b)
    from rtdm import _lib as L
    if args.step_events:
        L.check(L.lib().rtdm_detector_enable_timing(h, args.steps))
    if world > 1:
        import torch.distributed as dist
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        pipe(frames)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    ms = (ctypes.c_double * len(steps))()
    calls = ctypes.c_int()
    if args.step_events:
        L.check(L.lib().rtdm_detector_read_timing(h, ms, ctypes.byref(calls)))
        L.check(L.lib().rtdm_detector_enable_timing(h, 0))
    # roofline: kernel symbol with the largest summed device time
    agg = {}
    for (name, layer, flop, byt), t in zip(steps, ms):
        a = agg.setdefault(name, [0.0, 0.0, 0.0, 0])
        a[0] += t
        a[1] += flop * calls.value
        a[2] += byt * calls.value
        a[3] += calls.value
    dom = max(agg, key=lambda k: agg[k][0])
    t_ms, flop, byt, launches = agg[dom]
    det_ms = sum(ms) / max(1, calls.value)
    avg_ms = t_ms / launches if launches else 0.0
    achieved_tflops = (flop / launches) / (avg_ms * 1e-3) / 1e12 if avg_ms > 0 else 0.0
    tr = pmc_traffic(dom)
    traffic = round(tr["bytes_per_launch"]) if tr else None
    frames_total = world * b * args.steps
    value = frames_total / elapsed
    pipe_flop = det.flop_per_image + CLASSIFIER_FLOP[args.classifier]
    counts = pipe._bufs[(b, str(dev))]["count"].cpu()
    rec = {
        "metric": "frames/sec two-stage (ErNET→YOLOv4) 608×608 b64 @1/2/4/8 GPU; top-1/mAP parity",
        "value": round(value, 2), "unit": "frames/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(elapsed * 1e3 / args.steps, 4), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f16" if args.dtype == "f16" else "f32",
        "data": "synthetic 608x608 uint8 frames (seeded), synthetic calibrated detector weights, "
                "random-init classifier weights",
        "config": {"workload": f"two-stage {args.classifier} -> {args.cfg}@{args.img} + decode + NMS "
                               f"(conf {args.conf}, iou {args.iou})",
                   "global_batch": b * world, "per_gpu_batch": b, "img": args.img,
                   "parallelism": f"dp{world} (frame shards, no data-path collective)"},
        "roofline": {"bound": "mfma", "kernel": dom, "achieved": round(achieved_tflops, 2),
                     "peak": MFMA_F16_DENSE_PEAK_TFLOPS, "unit": "TFLOP/s",
                     "frac": round(achieved_tflops / MFMA_F16_DENSE_PEAK_TFLOPS, 4), "traffic": traffic,
                     "avg_launch_ms": round(avg_ms, 4), "launches": launches,
                     "traffic_unit": "bytes/launch (HBM, PMC)", "traffic_source": tr["source"] if tr else None,
                     "algorithmic_bytes_per_launch": round(byt / launches) if launches else None},
        "pipeline": {"flop_per_frame": pipe_flop,
                     "pipeline_tflops": round(pipe_flop * value / world / 1e12, 2),
                     "pipeline_frac": round(pipe_flop * value / world / 1e12 / MFMA_F16_DENSE_PEAK_TFLOPS, 4),
                     "detector_kernel_ms_per_step": round(det_ms, 4),
                     "detections_per_frame": round(float(counts.float().mean()), 2)},
    }
    if rank == 0 and world == 1 and args.cpu_baseline:
        rec["cpu_baseline"] = cpu_baseline(args, text, stream, sd)
    if rank == 0:
        step_ms = {}
        for (name, layer, flop, byt), t in zip(steps, ms):
            step_ms[f"L{layer}:{name}"] = round(t / max(1, calls.value), 4)
        with open(os.path.join(ROOT, "gpurun_out" if os.path.isdir(os.path.join(ROOT, "gpurun_out")) else ".",
                               "bench_steps.json"), "w") as f:
            json.dump(step_ms, f, indent=1)
        print(json.dumps(rec), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
