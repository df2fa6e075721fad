#!/usr/bin/env python3
"""Wall time attributed to each kernel in an overlapped (several batches in flight) run:
every interval between two kernel start / end events is split equally among the kernels
running in it, so the attributed times sum to the GPU's busy wall time.  A kernel that only
runs beside others costs little here even if its own duration is long; one that runs alone
costs its whole duration.   python tools/overlap.py gpurun_out/prof_TAG/.../run_results.db
[--skip FRACTION of the trace to drop at the start (warm-up), default 0.3]"""
import argparse
import re
import sqlite3
from collections import defaultdict

ap = argparse.ArgumentParser()
ap.add_argument("db")
ap.add_argument("--skip", type=float, default=0.3)
ap.add_argument("--top", type=int, default=30)
args = ap.parse_args()
con = sqlite3.connect(args.db)
rows = con.execute("select name, start, end from kernels order by start").fetchall()
rows = rows[int(len(rows) * args.skip):]


def short(n):
    n = re.sub(r"\(.*", "", n.replace("void ", "").replace("rtdm::", ""))
    return n[:48]


ev = []
for i, (n, s, e) in enumerate(rows):
    ev.append((s, 1, i))
    ev.append((e, 0, i))
ev.sort()
running = set()
attr = defaultdict(float)
dur = defaultdict(float)
calls = defaultdict(int)
alone = defaultdict(float)
busy = 0.0
last = ev[0][0]
for t, kind, i in ev:
    if running and t > last:
        dt = (t - last) / 1000.0
        busy += dt
        for j in running:
            attr[short(rows[j][0])] += dt / len(running)
        if len(running) == 1:
            alone[short(rows[next(iter(running))][0])] += dt
    last = t
    if kind == 1:
        running.add(i)
    else:
        running.discard(i)
for n, s, e in rows:
    dur[short(n)] += (e - s) / 1000.0
    calls[short(n)] += 1
span = (rows[-1][2] - rows[0][1]) / 1000.0
print(f"span {span:.1f} us, busy {busy:.1f} us ({busy / span:.3f}), kernels {len(rows)}")
print(f"{'kernel':48s} {'calls':>6s} {'dur us':>9s} {'attr us':>9s} {'alone us':>9s} {'attr/dur':>8s}")
for k in sorted(attr, key=lambda k: -attr[k])[: args.top]:
    print(f"{k:48s} {calls[k]:6d} {dur[k]:9.1f} {attr[k]:9.1f} {alone[k]:9.1f} {attr[k] / max(dur[k], 1e-9):8.3f}")
