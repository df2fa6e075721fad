#!/usr/bin/env python3
"""Summarise rocprofv3 rocpd databases (gpurun_out/…/run_results.db) into the
markdown/JSON files committed under profiles/.

  python tools/prof_summary.py TAG [--out profiles] [--gpurun gpurun_out]

Reads   gpurun_out/prof_TAG/run_results.db            (--kernel-trace --stats)
        gpurun_out/pmc_FETCH_SIZE_TAG/run_results.db  (--pmc FETCH_SIZE)
        gpurun_out/pmc_WRITE_SIZE_TAG/run_results.db  (--pmc WRITE_SIZE)
Writes  profiles/TAG_kernel_stats.md   per-kernel calls / total / avg / min / max / %
        profiles/TAG_traffic.json      per-kernel HBM bytes per launch from the PMC passes,
                                       FETCH_SIZE doubled (gfx950: FETCH_SIZE counts 64 B per
                                       128-B request, MI355X_MICROARCH.md "HBM"), WRITE_SIZE as is;
                                       both counters are reported by rocprofv3 in KB.
"""
from __future__ import annotations

import argparse
import json
import os
import re
import sqlite3
import statistics


def short(name: str) -> str:
    name = re.sub(r"^void ", "", name)
    name = re.sub(r"\(.*\)$", "", name)
    return name.replace("rtdm::", "").replace(" ", "")


def kernel_rows(db):
    con = sqlite3.connect(db)
    rows = con.execute("select name, duration from kernels order by start").fetchall()
    con.close()
    return rows


def pmc_rows(db):
    con = sqlite3.connect(db)
    rows = con.execute("select kernel_name, counter_name, value from counters_collection order by dispatch_id").fetchall()
    con.close()
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("tag")
    ap.add_argument("--out", default="profiles")
    ap.add_argument("--gpurun", default="gpurun_out")
    ap.add_argument("--note", default="")
    a = ap.parse_args()
    os.makedirs(a.out, exist_ok=True)
    db = os.path.join(a.gpurun, f"prof_{a.tag}", "run_results.db")
    if not os.path.exists(db):  # PMC passes only: their own kernel trace gives the launch times
        db = os.path.join(a.gpurun, f"pmc_FETCH_SIZE_{a.tag}", "run_results.db")
    rows = kernel_rows(db)
    agg = {}
    for name, dur in rows:
        agg.setdefault(short(name), []).append(dur / 1000.0)
    total = sum(sum(v) for v in agg.values())
    lines = [f"# rocprofv3 --kernel-trace --stats — {a.tag}", ""]
    if a.note:
        lines += [a.note, ""]
    lines += ["| kernel | calls | total µs | avg µs | median µs | min µs | max µs | % |", "|---|---|---|---|---|---|---|---|"]
    for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
        lines.append(f"| `{k}` | {len(v)} | {sum(v):.1f} | {sum(v)/len(v):.2f} | {statistics.median(v):.2f} | "
                     f"{min(v):.2f} | {max(v):.2f} | {100*sum(v)/total:.2f} |")
    traffic = {}
    for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
        pdb = os.path.join(a.gpurun, f"pmc_{ctr}_{a.tag}", "run_results.db")
        if not os.path.exists(pdb):
            continue
        per = {}
        for name, cname, val in pmc_rows(pdb):
            if cname != ctr:
                continue
            per.setdefault(short(name), []).append(val * 1024.0 * (2.0 if ctr == "FETCH_SIZE" else 1.0))
        for k, v in per.items():
            traffic.setdefault(k, {})[ctr.lower() + "_bytes_avg"] = sum(v) / len(v)
            traffic[k]["launches"] = len(v)
    if traffic:
        for k, t in traffic.items():
            if k.startswith("_"):
                continue
            t["hbm_bytes_avg"] = t.get("fetch_size_bytes_avg", 0.0) + t.get("write_size_bytes_avg", 0.0)
        lines += ["", "## HBM traffic per launch (PMC passes, FETCH_SIZE ×2 gfx950 correction)", "",
                  "| kernel | launches | read MB | write MB | total MB |", "|---|---|---|---|---|"]
        for k, t in sorted(((k, t) for k, t in traffic.items() if not k.startswith("_")),
                           key=lambda kv: -kv[1]["hbm_bytes_avg"]):
            lines.append(f"| `{k}` | {t['launches']} | {t.get('fetch_size_bytes_avg', 0)/1e6:.2f} | "
                         f"{t.get('write_size_bytes_avg', 0)/1e6:.2f} | {t['hbm_bytes_avg']/1e6:.2f} |")
        # the workload the PMC passes ran (bench.py's JSON line in their logs): bench.py only
        # takes traffic from a summary of the same workload, dtype and per-GPU batch
        for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
            log = os.path.join(a.gpurun, f"pmc_{ctr}_{a.tag}.log")
            if os.path.exists(log):
                for line in open(log):
                    if line.startswith("{"):
                        d = json.loads(line)
                        traffic["_workload"] = {"workload": d["config"]["workload"], "dtype": d["dtype"],
                                                "per_gpu_batch": d["config"]["per_gpu_batch"]}
                break
        with open(os.path.join(a.out, f"{a.tag}_traffic.json"), "w") as f:
            json.dump(traffic, f, indent=1, sort_keys=True)
    with open(os.path.join(a.out, f"{a.tag}_kernel_stats.md"), "w") as f:
        f.write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main()
