#!/usr/bin/env python3
"""Host-side enqueue time of one eager two-stage pipeline call (no synchronisation inside the
timed loop): if it approaches the per-step GPU time, small per-rank batches are launch-bound.
Prints the mean host microseconds per call, and cProfile's top entries.

  python tools/host_launch.py [--batch 8] [--calls 200]"""
import argparse
import cProfile
import os
import pstats
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "real-time-disaster-management_amd"))

import bench  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=8)
ap.add_argument("--calls", type=int, default=200)
ap.add_argument("--inflight", type=int, default=4)
a = ap.parse_args()
sys.argv = ["bench.py", "--batch", str(a.batch), "--inflight", str(a.inflight), "--graphs", "0"]
args = bench.parse()
pipes, text, stream, sd = bench.build(args, 1, 0)
dev = torch.device("cuda", 0)
frames = bench.make_frames(args, 0, a.batch, dev)
streams = [torch.cuda.current_stream()] + [torch.cuda.Stream() for _ in pipes[1:]]


def call(k):
    j = k % len(pipes)
    with torch.cuda.stream(streams[j]):
        pipes[j](frames[k % len(frames)])


for k in range(20):
    call(k)
torch.cuda.synchronize()
t0 = time.perf_counter()
for k in range(a.calls):
    call(k)
t1 = time.perf_counter()
torch.cuda.synchronize()
t2 = time.perf_counter()
print(f"b{a.batch}: host enqueue {1e6 * (t1 - t0) / a.calls:.1f} us/call, wall {1e6 * (t2 - t0) / a.calls:.1f} us/call",
      flush=True)
pr = cProfile.Profile()
pr.enable()
for k in range(a.calls):
    call(k)
pr.disable()
torch.cuda.synchronize()
pstats.Stats(pr).sort_stats("tottime").print_stats(12)
