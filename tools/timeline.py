#!/usr/bin/env python3
"""Kernel timeline of a rocprofv3 --kernel-trace database: the last N dispatches with
start/end (µs, relative), duration, queue/stream, and the idle gap before each kernel on
its own stream.   python tools/timeline.py gpurun_out/trace_TAG_i/run_results.db [N]"""
import re
import sqlite3
import sys

db = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 60
con = sqlite3.connect(db)
rows = con.execute("select name, start, end, stream_id, queue_id from kernels order by start").fetchall()
rows = rows[-n:]
t0 = rows[0][1]
last_end = {}
gaps = []
for name, s, e, st, q in rows:
    nm = re.sub(r"\(.*", "", name.replace("void ", "").replace("rtdm::", ""))[:44]
    g = (s - last_end[st]) / 1000 if st in last_end else float("nan")
    last_end[st] = e
    gaps.append(g)
    print(f"{(s - t0) / 1000:9.1f} {(e - s) / 1000:7.1f}  gap {g:6.1f}  st{st} q{q} {nm}")
