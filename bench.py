#!/usr/bin/env python3
"""Two-stage aerial-frame inference benchmark (BASELINE.json metric).

One step = one GLOBAL batch of synthetic 608x608 uint8 frames (default 64) through
the whole hot path on the GPU(s): classifier CLI transform + ACFF classifier (ErNET,
the reference's trained weights), Darknet detector of record (yolov4-tiny-aider-416.cfg
run at 608x608; /255 fused), YOLO decode (fused into the head convs) and per-image NMS
(conf 0.3, IoU 0.4, detect.py defaults).  Frames are resident in HBM before timing.

  python bench.py [--gpus N] [--steps K] [--warmup W]
  N>1: `python bench.py --gpus N` starts N ranks itself (fresh child processes of this
       script, one per GPU, RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set, before any GPU
       call; rank 0's JSON line is the output, a failing rank fails the run), or
       python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N
       (then WORLD_SIZE must equal N);
       one rank per GPU; the global batch is frame-sharded (rank r processes frames
       [r*B/N, (r+1)*B/N), SURVEY.md §8e: 8 frames per GPU at N=8), weights are
       broadcast once over RCCL and every step ends with a gather of all ranks'
       results (logits, probs, detections, indices, counts) to rank 0 over RCCL.
       --per-gpu-batch b instead fixes the frames per GPU (weak scaling).

Each rank replays the step as one hipGraph per input buffer (TwoStagePipeline
graphs=True); the steps cycle over --rotate distinct frame batches so no step
re-reads the previous step's frames from the 256 MB Infinity Cache.

Prints ONE JSON line on rank 0 (value = frames/s over all ranks), with
  roofline:     the dominant kernel (largest summed device time), its algorithmic FLOP
                per launch / its average launch time from hipEvents recorded on its
                launch stream around every detector launch, over --roofline-steps eager
                steps run right after the timed region (events cannot sit inside the
                replayed graphs), against the dense fp16 MFMA peak; traffic from the
                committed rocprofv3 PMC passes (profiles/*_traffic.json)
  cpu_baseline: the CPU oracle (torch-CPU restatement of the reference path, incl. NMS)
                timed on a bounded sample on this host, rank 0 at N=1 only
  h2d:          the same step with the frames uploaded from pinned host memory inside
                the timed step (PCIe-inclusive rate; never `value`)
"""
from __future__ import annotations

import argparse
import ctypes
import json
import re
import os
import statistics
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "real-time-disaster-management_amd"))

MFMA_F16_DENSE_PEAK_TFLOPS = 2500.0  # MI355X_MICROARCH.md: ~2.5 PF dense bf16/fp16
MFMA_I8_DENSE_PEAK_TOPS = 5000.0     # int8 MFMA: 2x the bf16 rate per clock (same table)
CLASSIFIER_FLOP = {"squeeze-ernet": 90953544.0, "squeeze-redconv": 77593080.0, "ernet": 319307650.0, "none": 0.0}
METRIC = "frames/sec two-stage (ErNET→YOLOv4) 608×608 b64 @1/2/4/8 GPU; top-1/mAP parity"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks (one per GPU); default WORLD_SIZE or 1.  > 1 without WORLD_SIZE: this script "
                         "starts the N ranks itself")
    ap.add_argument("--dry-run", action="store_true",
                    help="launcher self-test (no GPU): the ranks join a gloo group and rank 0 prints one JSON "
                         "line with every rank's launch environment")
    ap.add_argument("--dry-fail-rank", type=int, default=-1, help="(--dry-run) this rank exits with status 3")
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch", type=int, default=64, help="global frames per step (sharded over the ranks)")
    ap.add_argument("--per-gpu-batch", type=int, default=0,
                    help="> 0: frames per GPU per step instead (weak scaling; global = this * N)")
    ap.add_argument("--img", type=int, default=608)
    ap.add_argument("--cfg", default="yolov4-tiny-aider-416",
                    help="detector cfg; none: classification only (BASELINE config 2: --classifier squeeze-redconv "
                         "--cfg none --img 224 --batch 32)")
    ap.add_argument("--weights", default="cond", choices=["cond", "he"],
                    help="synthetic detector weight set (rtdm.synth): cond = the well-conditioned set the "
                         "SURVEY §8d bars are asserted on; he = the mean-field stress set")
    ap.add_argument("--classifier", default="ernet", choices=["ernet", "squeeze-ernet", "squeeze-redconv", "none"],
                    help="none: detection only (BASELINE config 3)")
    ap.add_argument("--dtype", default="f16", choices=["f16", "f32", "i8"],
                    help="i8: int8-quantised detector (BASELINE config 5) and classifier ACFF fusion GEMMs")
    ap.add_argument("--conf", type=float, default=0.3)
    ap.add_argument("--iou", type=float, default=0.4)
    ap.add_argument("--max-det", type=int, default=300)
    ap.add_argument("--overlap", type=int, default=0,
                    help="1: classifier on a side stream beside the detector; 0: both stages on the batch's stream")
    ap.add_argument("--priority", type=int, default=0,
                    help="1: detector + NMS on a high-priority stream, classifier on a low-priority one")
    ap.add_argument("--det-streams", type=int, default=1, help="detector head branches on a side stream (2) or not (1)")
    ap.add_argument("--graphs", type=int, default=-1,
                    help="1: replay each step as a hipGraph; 0: eager launches; -1: by per-GPU batch (graphs from 64 "
                         "frames up, eager below)")
    ap.add_argument("--rotate", type=int, default=4, help="distinct frame batches the steps cycle over")
    ap.add_argument("--inflight", type=int, default=0,
                    help="batches in flight per GPU (0: 3 for <= 16 frames per GPU, else 2): step k runs on "
                         "pipeline k %% inflight (own handles, buffers and ONE stream), so consecutive batches "
                         "run concurrently and fill the CUs one batch's low-occupancy kernels leave idle")
    ap.add_argument("--roofline-steps", type=int, default=20,
                    help="eager steps with per-launch hipEvents after the timed region (0: no roofline)")
    ap.add_argument("--h2d-steps", type=int, default=20, help="PCIe-inclusive steps (0: skip)")
    ap.add_argument("--cpu-baseline", type=int, default=1, help="0 disables the CPU oracle leg")
    ap.add_argument("--cpu-seconds", type=float, default=15.0,
                    help="CPU oracle leg: time chunks of 16 frames until this much CPU time has passed")
    return ap.parse_args()


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(n):
    """`--gpus N` (N > 1) without a launcher: start N fresh processes of this script, one per
    GPU (the reference's multi-GPU inference takes every visible GPU,
    yolov3/test.py:42-43).  Runs before anything touches the GPU, and never replaces this
    process (children via subprocess, no exec).  Rank 0's JSON lines are relayed to our
    stdout (the run's one line); everything else the ranks print (library banners such as
    gloo's) goes to stderr.  Waits for all; if one fails, the others are stopped and the
    run exits non-zero."""
    import subprocess
    import threading
    port = free_port()
    cmd = [sys.executable, os.path.abspath(__file__)] + sys.argv[1:]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE if r == 0 else sys.stderr, text=r == 0))

    def relay(f):
        for line in f:
            (sys.stdout if line.startswith("{") else sys.stderr).write(line)
            (sys.stdout if line.startswith("{") else sys.stderr).flush()
    reader = threading.Thread(target=relay, args=(procs[0].stdout,), daemon=True)
    reader.start()
    rc, alive = 0, list(procs)
    while alive:
        for p in list(alive):
            c = p.poll()
            if c is None:
                continue
            alive.remove(p)
            if c != 0 and rc == 0:
                rc = c if c > 0 else 1
                print(f"bench.py: rank {procs.index(p)} exited with status {c}; stopping the other ranks",
                      file=sys.stderr, flush=True)
                for q in alive:
                    q.terminate()
                deadline = time.time() + 15
                for q in alive:
                    try:
                        q.wait(timeout=max(0.1, deadline - time.time()))
                    except subprocess.TimeoutExpired:
                        q.kill()
        time.sleep(0.05)
    reader.join(timeout=10)
    return rc


def dry_run(args, world, rank):
    """Launcher self-test: the ranks meet in a gloo group (CPU), rank 0 prints one line."""
    import torch.distributed as dist
    env = {k: os.environ.get(k) for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")}
    if rank == args.dry_fail_rank:
        raise SystemExit(3)
    envs = [env]
    if world > 1:
        dist.init_process_group("gloo")
        envs = [None] * world
        dist.all_gather_object(envs, env)
        dist.destroy_process_group()
    if rank == 0:
        print(json.dumps({"metric": METRIC, "dry_run": True, "n_gpus": world, "ranks": envs}), flush=True)


def dist_setup():
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


def trained_classifier(name):
    """The reference's trained state dict (weights/<name>-state_dict.pt, copied into
    tests/golden/classifier_weights.npz by tests/golden/make_golden.py)."""
    z = np.load(os.path.join(ROOT, "tests", "golden", "classifier_weights.npz"), allow_pickle=False)
    return {k.split("/", 1)[1]: z[k] for k in z.files if k.split("/", 1)[0] == name}


def build(args, world, rank):
    from rtdm.classifier import build_model
    from rtdm.darknet import Darknet
    from rtdm.pipeline import TwoStagePipeline
    from rtdm.synth import classifier_param_shapes, inline_acff, load_calibration, synth_acff_params, \
        synth_darknet_weights

    from rtdm import _lib as L
    L.check(L.lib().rtdm_set_tuning(b"two_streams", 1 if args.det_streams > 1 else 0))
    for kv in filter(None, os.environ.get("RTDM_TUNE", "").split(",")):  # diagnostics: "key=v,key=v"
        k, v = kv.split("=")
        L.check(L.lib().rtdm_set_tuning(k.encode(), int(v)))
    use_det = args.cfg != "none"
    text = open(os.path.join(ROOT, "real-time-disaster-management_amd", "rtdm", "cfg", args.cfg + ".cfg")).read() \
        if use_det else None
    det = Darknet(text, (args.img, args.img)) if use_det else None
    use_cls = args.classifier != "none"
    if not (use_det or use_cls):
        raise SystemExit("--cfg none needs a classifier")
    cls = build_model(args.classifier) if use_cls else None
    # rank 0 makes / loads the weights; RCCL broadcast to the other ranks (once, untimed)
    if rank == 0:
        stream = None
        if use_det:
            calib = load_calibration(args.cfg, args.weights)
            conv = synth_darknet_weights(text, calib=calib, preset=args.weights)
            acff = synth_acff_params(text, calib=calib, preset=args.weights)
            stream = inline_acff(text, conv, acff)  # YOLO-ACFF cfgs: [acff] params inline
            args.ref_weights = (conv, acff)         # the CPU oracle takes them apart
        sd = trained_classifier(args.classifier) if use_cls else {}
    else:
        stream, sd = None, None
    if world > 1:
        from rtdm.distributed import broadcast_array, broadcast_state_dict
        stream = broadcast_array(stream) if use_det else None
        sd = broadcast_state_dict(sd, classifier_param_shapes(args.classifier)) if use_cls else {}
    if use_det:
        det.load_weight_stream(stream)
    if use_cls:
        cls.load_state_dict(sd)
    calib = None
    if args.dtype == "i8":  # calibration frames disjoint from the timed ones
        from rtdm.synth import BASE_SEED, synth_frames
        calib = torch.from_numpy(synth_frames(16, args.img, args.img, seed=BASE_SEED + 4321)).cuda()
    if args.dtype in ("f16", "i8"):
        if use_det:
            det.half() if args.dtype == "f16" else det.int8(calib)
        if use_cls:
            cls.half() if args.dtype == "f16" else cls.int8(calib)
    pipes = []
    for j in range(args.inflight):
        if j:  # another instance: own device weights, arenas, buffers and streams
            det = Darknet(text, (args.img, args.img)) if use_det else None
            cls = build_model(args.classifier) if use_cls else None
            if use_det:
                det.load_weight_stream(stream)
            if use_cls:
                cls.load_state_dict(sd)
            if args.dtype in ("f16", "i8"):
                if use_det:
                    det.half() if args.dtype == "f16" else det.int8(calib)
                if use_cls:
                    cls.half() if args.dtype == "f16" else cls.int8(calib)
        if use_det:
            # several batches in flight fill each other's idle CUs: plan conv tiles for CU-time, not
            # for one launch's rounds (larger tiles; bit-identical either way), on these detectors'
            # own handles only (rtdm_detector_set_tuning).  Measured with 4 in flight (r03an): b8
            # 31.8k -> 33.0k, b16 36.9k -> 39.3k frames/s
            det.set_tuning("conv_pipe_cost", 1 if args.inflight > 1 else 0)
        pipes.append(TwoStagePipeline(cls, det, args.conf, args.iou, args.max_det, overlap=bool(args.overlap),
                                      priority=bool(args.priority), graphs=bool(args.graphs)))
    return pipes, text, stream, sd


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


def pmc_traffic(kernel, workload):
    """HBM bytes per launch of `kernel` from the newest committed PMC summary of the same
    workload (profiles/*_traffic.json "_workload": config.workload, dtype, per-GPU batch;
    written by tools/prof_summary.py from separate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE
    passes over this bench command; FETCH_SIZE doubled per the gfx950 correction).  None
    when no pass covers it."""
    import glob
    def tag_key(path):  # rNN + a letter tag that runs a..z, aa..az, ... (+ a repeat number: fin, fin2, ...):
        # by round, then tag length, then tag, then repeat
        m = re.match(r"r(\d+)([a-z]*)(\d*)", os.path.basename(path))
        return (int(m.group(1)), len(m.group(2)), m.group(2), int(m.group(3) or 0)) if m else (-1, 0, "", 0)
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*_traffic.json")), key=tag_key)
    for path in reversed(files):
        try:
            d = json.load(open(path))
        except (OSError, ValueError):
            continue
        if d.get("_workload") != workload:
            continue
        t = d.get(kernel)
        if isinstance(t, dict) and "fetch_size_bytes_avg" in t and "write_size_bytes_avg" in t:
            return {"bytes_per_launch": t["hbm_bytes_avg"], "source": os.path.relpath(path, ROOT)}
    return None


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


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
    ref = DarknetRef(text, conv, acff) if text is not None else None
    s = 240 if args.classifier == "ernet" else 140
    sdt = {k: torch.from_numpy(np.asarray(v, np.float32)) for k, v in sd.items()}

    def run(frames):
        with torch.no_grad():
            if args.classifier != "none":
                x = torch.from_numpy(np.stack([OP.cli_transform(f, s) for f in frames]))
                OC.forward(args.classifier, sdt, x)
            if ref is None:
                return
            io = ref.forward(torch.from_numpy(frames).permute(0, 3, 1, 2).float() / 255.0)
        ON.non_max_suppression(io.numpy(), args.conf, args.iou)

    warm = synth_frames(2, args.img, args.img, seed=1)
    run(warm)
    # the median over >= 3 batches of the bench's own batch size (64 frames), each
    # timed alone; more batches while the time budget (--cpu-seconds) lasts, at most 8
    batch = 64
    rates, dt = [], 0.0
    while len(rates) < 3 or (dt < args.cpu_seconds and len(rates) < 8):
        frames = synth_frames(batch, args.img, args.img, first=batch * len(rates))
        t0 = time.perf_counter()
        run(frames)
        t = time.perf_counter() - t0
        dt += t
        rates.append(batch / t)
    med = float(np.median(rates))
    return {"value": round(med, 3), "unit": "frames/s", "cores": cores, "kind": "port",
            "cpu_model": cpu_model(), "batches": len(rates), "batch_rates": [round(r, 3) for r in rates],
            "sample": f"median over {len(rates)} batches of {batch} frames of the same synthetic {args.img}x{args.img} "
                      f"workload (frames 0..{batch * len(rates) - 1}), each timed alone, fp32 torch-CPU oracle ("
                      + (f"{args.classifier} + {args.cfg} + decode + NMS" if ref is not None else
                         f"CLI transform + {args.classifier}") + f"), {dt:.1f} s in total"}


HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec; 6.29 TB/s measured float4 copy)


def classifier_roofline(args, pipe, frames, b, workload):
    """Classification only (BASELINE config 2): the classifier is HBM- / latency-bound, so the
    roofline is bytes: per launch of the step (preprocess, stem, ACFF stages, chain + tail)
    its algorithmic HBM bytes (maps read + written, rtdm_classifier_read_timing) over its
    average hipEvent time on the launch stream, eager calls after the timed region; the
    dominant launch (largest summed time) is reported, with the whole step beside it."""
    from rtdm import _lib as L
    cls = pipe.classifier
    h = cls._get_handle(b)
    L.check(L.lib().rtdm_classifier_enable_timing(h, args.roofline_steps))
    for k in range(args.roofline_steps):
        pipe._launch(frames[k % len(frames)])
    torch.cuda.synchronize()
    ms = (ctypes.c_double * 24)()
    byt = (ctypes.c_double * 24)()
    names = ctypes.create_string_buffer(24 * 32)
    nl, calls = ctypes.c_int(), ctypes.c_int()
    L.check(L.lib().rtdm_classifier_read_timing(h, ms, byt, names, 32, ctypes.byref(nl), ctypes.byref(calls)))
    L.check(L.lib().rtdm_classifier_enable_timing(h, 0))
    rows = [(names.raw[32 * i:32 * i + 32].split(b"\0")[0].decode(), ms[i] / calls.value, byt[i]) for i in range(nl.value)]
    dom = max(rows, key=lambda r: r[1])
    ach = dom[2] / (dom[1] * 1e-3) / 1e9
    tot_ms, tot_b = sum(r[1] for r in rows), sum(r[2] for r in rows)
    tr = pmc_traffic(dom[0], {"workload": workload, "dtype": args.dtype, "per_gpu_batch": b})
    return {"bound": "hbm", "kernel": dom[0], "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": round(tr["bytes_per_launch"]) if tr else None,
            "avg_launch_ms": round(dom[1], 4), "algorithmic_bytes_per_launch": round(dom[2]),
            "traffic_unit": "bytes/launch (HBM, PMC)", "traffic_source": tr["source"] if tr else None,
            "launches": {r[0]: {"ms": round(r[1], 4), "GB/s": round(r[2] / (r[1] * 1e-3) / 1e9, 1)} for r in rows},
            "step": {"ms": round(tot_ms, 4), "bytes": round(tot_b), "GB/s": round(tot_b / (tot_ms * 1e-3) / 1e9, 1)},
            "timing": f"hipEvents around each classifier launch on its stream, {calls.value} eager calls after the "
                      f"timed region"}


def make_frames(args, first, count, dev):
    """`--rotate` distinct frame batches of this rank's shard: the seeded synthetic frames
    (frame i depends only on the seed and its global index) and, for
    rotation j > 0, the same frames cyclically shifted by (37j, 53j) pixels on the device."""
    from rtdm.synth import synth_frames
    base = torch.from_numpy(synth_frames(count, args.img, args.img, first=first)).to(dev)
    out = [base]
    for j in range(1, max(1, args.rotate)):
        out.append(torch.roll(base, shifts=(37 * j, 53 * j), dims=(1, 2)).contiguous())
    return out


def main():
    args = parse()
    env_world = os.environ.get("WORLD_SIZE")
    if args.gpus is None:
        args.gpus = int(env_world or 1)
    if args.gpus < 1:
        raise SystemExit(f"--gpus {args.gpus}: need at least one rank")
    if env_world is None and args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus))  # parent: starts the ranks, relays rank 0's line
    if env_world is not None and int(env_world) != args.gpus:
        raise SystemExit(f"WORLD_SIZE={env_world} but --gpus {args.gpus}: launch one rank per GPU "
                         f"(--nproc-per-node {args.gpus}) or drop the launcher and let bench.py start them")
    if args.dry_run:
        return dry_run(args, args.gpus, int(os.environ.get("RANK", "0")))
    world, rank, local = dist_setup()
    dist = None
    if world > 1:
        import torch.distributed as dist
    from rtdm.distributed import gather_records, shard_range
    dev = torch.device("cuda", torch.cuda.current_device())
    if args.per_gpu_batch > 0:
        global_batch, scaling = args.per_gpu_batch * world, "weak"
    else:
        global_batch, scaling = args.batch, "strong"
    if global_batch % world:
        raise SystemExit(f"global batch {global_batch} does not shard evenly over {world} ranks")
    first, b = shard_range(global_batch, world, rank)
    if args.graphs < 0 or args.inflight <= 0:
        # measured on MI355X (profiles/r03_operating_points.md): below 64 frames per GPU, eager
        # launches with 4 batches in flight beat graph replay with 3 (b8 33.5k vs 30.4k frames/s,
        # b16 39.1k vs 36.7k, b32 41.8k vs 39.4k, int8 b16 43.7k vs 40.5k); replayed graphs on a 4th
        # in-flight stream serialise (b8 graphs 4 in flight: 21-25k).  At b64 graphs with 2 in flight
        # stay best (45.3k; eager 2 / 3 / 4: 43.8k / 44.4k / 44.8k).
        small = b < 64
        if args.graphs < 0:
            args.graphs = 0 if small else 1
        if args.inflight <= 0:
            args.inflight = (4 if not args.graphs else 3) if small else 2
    pipes, text, stream, sd = build(args, world, rank)
    pipe, det = pipes[0], pipes[0].detector
    streams = [torch.cuda.current_stream()] + [torch.cuda.Stream() for _ in pipes[1:]]
    frames = make_frames(args, first, b, dev)
    rec_len = pipe.record_layout(b)[1]
    # one gather buffer per in-flight pipeline: each pipeline's gather runs on its own stream, so a
    # shared buffer would be a cross-stream write-after-write between steps in flight
    gathered = [torch.empty((world, rec_len), device=dev, dtype=torch.float32) for _ in pipes] \
        if world > 1 and rank == 0 else None
    torch.cuda.synchronize()

    def step(k, ev=None):
        j = k % len(pipes)
        with torch.cuda.stream(streams[j]):
            if ev is not None:
                ev[0].record()
            out = pipes[j](frames[k % len(frames)])
            if world > 1:
                gather_records(out["record"], gathered[j] if rank == 0 else None)
            if ev is not None:
                ev[1].record()
        return out

    for k in range(args.warmup):
        step(k)
    torch.cuda.synchronize()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        out = step(k, evs[k])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    step_ms = [s.elapsed_time(e) for s, e in evs]
    counts = out["count"].cpu() if det is not None else None
    if det is not None and world > 1 and rank == 0:  # every rank's shard arrived: the global batch's counts
        from rtdm.pipeline import unpack_record
        last = gathered[(args.steps - 1) % len(pipes)]  # the buffer of the last timed step's pipeline
        counts = torch.cat([unpack_record(last[r], pipe, b)["count"].cpu() for r in range(world)])

    # ---- roofline: per-launch hipEvents on the detector's launch streams, eager steps ----
    if det is None:
        workload = (f"classification only: {args.classifier} on {args.img}x{args.img} uint8 frames "
                    f"(CLI transform on device)")
    else:
        workload = ((f"two-stage {args.classifier} -> " if args.classifier != "none" else "detection only: ")
                    + f"{args.cfg}@{args.img} + decode + NMS (conf {args.conf}, iou {args.iou})")
    from rtdm import _lib as L
    rl = None
    if det is None and args.roofline_steps > 0:
        rl = classifier_roofline(args, pipe, frames, b, workload)
    if det is not None:
        h, steps = step_table(det, b)
    if det is not None and args.roofline_steps > 0:
        L.check(L.lib().rtdm_detector_enable_timing(h, args.roofline_steps))
        for k in range(args.roofline_steps):
            pipe._launch(frames[k % len(frames)])
        torch.cuda.synchronize()
        ms = (ctypes.c_double * len(steps))()
        calls = ctypes.c_int()
        L.check(L.lib().rtdm_detector_read_timing(h, ms, ctypes.byref(calls)))
        L.check(L.lib().rtdm_detector_enable_timing(h, 0))
        agg = {}
        for (name, layer, flop, byt), t in zip(steps, ms):
            a = agg.setdefault(name, [0.0, 0.0, 0.0, 0])
            a[0] += t
            a[1] += flop * calls.value
            a[2] += byt * calls.value
            a[3] += calls.value
        dom = max(agg, key=lambda k: agg[k][0])
        t_ms, flop, byt, launches = agg[dom]
        avg_ms = t_ms / launches
        achieved = (flop / launches) / (avg_ms * 1e-3) / 1e12
        tr = pmc_traffic(dom, {"workload": workload, "dtype": args.dtype, "per_gpu_batch": b})
        i8k = "_i8" in dom
        peak = MFMA_I8_DENSE_PEAK_TOPS if i8k else MFMA_F16_DENSE_PEAK_TFLOPS
        rl = {"bound": "mfma", "kernel": dom, "achieved": round(achieved, 2), "peak": peak,
              "unit": "TOP/s" if i8k else "TFLOP/s", "frac": round(achieved / peak, 4),
              "traffic": round(tr["bytes_per_launch"]) if tr else None,
              "avg_launch_ms": round(avg_ms, 4), "launches": launches,
              "algorithmic_flop_per_launch": round(flop / launches),
              "algorithmic_bytes_per_launch": round(byt / launches),
              "traffic_unit": "bytes/launch (HBM, PMC)", "traffic_source": tr["source"] if tr else None,
              "timing": f"hipEvents around each detector launch on its launch stream, {calls.value} eager steps "
                        f"after the timed region"}
        # the whole implicit-GEMM family: every conv_pipe* instantiation (conv_pipe_, conv_pipew_,
        # conv_pipew0_ (the cursor-loop window kernels, e.g. the fused head), conv_pipewpp_, ...,
        # int8 twins priced at the int8 peak); the dominant symbol above is one variant of it
        fam = [k for k in agg if k.startswith("conv_pipe")]
        if fam:
            f_ms = sum(agg[k][0] for k in fam)
            f_flop = sum(agg[k][1] for k in fam)
            f_peak_ms = sum(agg[k][1] / ((MFMA_I8_DENSE_PEAK_TOPS if "_i8" in k else MFMA_F16_DENSE_PEAK_TFLOPS) * 1e12)
                            * 1e3 for k in fam)
            rl["family"] = {"kernels": "conv_pipe* (all MFMA implicit-GEMM convs, every variant)",
                            "symbols": sorted(fam),
                            "achieved": round(f_flop / (f_ms * 1e-3) / 1e12, 2),
                            "frac": round(f_peak_ms / f_ms, 4),
                            "ms_per_step": round(f_ms / max(1, calls.value), 4)}
        # per-layer fractions of the big convs (>= 5 % of the step's conv FLOP), so a change in the
        # dominant symbol's composition (which layers share one instantiation) cannot move them
        tot_flop = sum(f for (_, _, f, _) in steps)
        lay = {}
        for (name, layer, flop, byt), t in zip(steps, ms):
            if not name.startswith("conv_pipe") or flop < 0.05 * tot_flop or t <= 0:
                continue
            lms = t / max(1, calls.value)
            lpk = MFMA_I8_DENSE_PEAK_TOPS if "_i8" in name else MFMA_F16_DENSE_PEAK_TFLOPS
            ach = flop / (lms * 1e-3) / 1e12
            lay[f"L{layer}"] = {"kernel": name, "gflop": round(flop / 1e9, 2), "ms": round(lms, 4),
                                "achieved": round(ach, 1), "frac": round(ach / lpk, 4)}
        rl["layers"] = lay
        if rank == 0:
            per_step = {f"L{layer}:{name}": round(t / max(1, calls.value), 4)
                        for (name, layer, flop, byt), t in zip(steps, ms)}
            outdir = os.path.join(ROOT, "gpurun_out") if os.path.isdir(os.path.join(ROOT, "gpurun_out")) else ROOT
            with open(os.path.join(outdir, "bench_steps.json"), "w") as f:
                json.dump(per_step, f, indent=1)

    # ---- PCIe-inclusive variant: frames uploaded from pinned host memory each step, on a copy
    #      stream into double-buffered device inputs (rtdm.pipeline.FrameUploader), so batch
    #      k+1's upload overlaps batch k's compute ----
    h2d = None
    if args.h2d_steps > 0:
        from rtdm.pipeline import FrameUploader
        host = [f.cpu().pin_memory() for f in frames]
        up = FrameUploader(pipes, streams, dev)
        for k in range(2 * len(pipes)):  # each pipeline's two buffers: capture their graphs
            up.submit(k, host[k % len(host)])
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for k in range(args.h2d_steps):
            o2 = up.submit(k, host[k % len(host)])
            if world > 1:
                with torch.cuda.stream(streams[k % len(pipes)]):
                    gather_records(o2["record"], gathered[k % len(pipes)] if rank == 0 else None)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        e2 = time.perf_counter() - t1
        if world > 1:
            t = torch.tensor([e2], device=dev, dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            e2 = float(t.item())
        h2d = {"value": round(global_batch * args.h2d_steps / e2, 2), "unit": "frames/s",
               "bytes_per_frame": args.img * args.img * 3, "steps": args.h2d_steps,
               "pcie_GBps": round(global_batch * args.h2d_steps * args.img * args.img * 3 / e2 / 1e9, 2),
               "note": "uint8 frames copied host(pinned)->HBM on a copy stream, double-buffered per in-flight "
                       "pipeline (rtdm.pipeline.FrameUploader): uploads overlap compute"}

    value = global_batch * args.steps / elapsed
    pipe_flop = (det.flop_per_image if det is not None else 0.0) + CLASSIFIER_FLOP[args.classifier]
    rec = {
        "metric": METRIC,
        "value": round(value, 2), "unit": "frames/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(elapsed * 1e3 / args.steps, 4), "higher_is_better": True,
        "scaling": scaling, "vs_baseline": None, "dtype": args.dtype,
        "data": f"synthetic {args.img}x{args.img} uint8 frames (seeded, {len(frames)} rotations), synthetic "
                f"calibrated detector weights ({args.weights} set)"
                + (f", the reference's trained {args.classifier} weights" if args.classifier != "none" else ""),
        "config": {"workload": workload,
                   "global_batch": global_batch, "per_gpu_batch": b, "img": args.img,
                   "parallelism": f"dp{world}: frame-sharded global batch"
                                  + (", per-step RCCL gather of every rank's results to rank 0" if world > 1 else ""),
                   "graphs": bool(args.graphs), "inflight": len(pipes)},
        "step_latency_ms_median": round(statistics.median(step_ms), 4),
        "step_latency_ms_p90": round(sorted(step_ms)[int(0.9 * (len(step_ms) - 1))], 4),
        "roofline": rl,
        "pipeline": {"flop_per_frame": pipe_flop,
                     "pipeline_tflops": round(pipe_flop * value / world / 1e12, 2),
                     "pipeline_frac": round(pipe_flop * value / world / 1e12 / MFMA_F16_DENSE_PEAK_TFLOPS, 4),
                     "detections_per_frame": round(float(counts.float().mean()), 2) if counts is not None else None},
        "h2d": h2d,
    }
    if rank == 0 and world == 1 and args.cpu_baseline:
        rec["cpu_baseline"] = cpu_baseline(args, text, stream, sd)
    if rank == 0:
        print(json.dumps(rec), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
