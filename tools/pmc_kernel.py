#!/usr/bin/env python3
"""Per-counter totals of one kernel from tools/pmc_detector.sh passes (last dispatch), normalised
per wave: python tools/pmc_kernel.py TAG NPASS SUBSTRING"""
import sqlite3
import sys

tag, npass, sub = sys.argv[1], int(sys.argv[2]), sys.argv[3]
vals = {}
for p in range(1, npass + 1):
    con = sqlite3.connect(f"gpurun_out/pmcdet_{tag}_{p}/run_results.db")
    q = con.execute("select dispatch_id, counter_name, sum(value), duration from counters_collection "
                    "where kernel_name like ? group by dispatch_id, counter_name order by dispatch_id",
                    (f"%{sub}%",)).fetchall()
    last = max(r[0] for r in q)
    for did, c, v, dur in q:
        if did == last:
            vals[c] = v
            vals["dur_us"] = dur / 1e3
w = vals.get("SQ_WAVES", 1)
for k, v in sorted(vals.items()):
    print(f"{k:28s} {v:16.0f} {v / w:12.1f}/wave")
