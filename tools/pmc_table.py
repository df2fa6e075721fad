#!/usr/bin/env python3
"""Per-dispatch PMC table from tools/pmc_detector.sh output (last iteration of run_detector.py).
python tools/pmc_table.py TAG [npasses]"""
import sqlite3
import sys

tag = sys.argv[1]
npass = int(sys.argv[2]) if len(sys.argv) > 2 else 2
passes = []
for p in range(1, npass + 1):
    con = sqlite3.connect(f"gpurun_out/pmcdet_{tag}_{p}/run_results.db")
    q = con.execute("select dispatch_id, kernel_name, counter_name, value, duration from counters_collection "
                    "order by dispatch_id").fetchall()
    d = {}
    for did, k, c, v, dur in q:
        r = d.setdefault(did, {"k": k, "dur": dur})
        r[c] = r.get(c, 0) + v
    ids = sorted(d)
    passes.append([d[i] for i in ids[len(ids) // 2:]])
merged = []
for rows in zip(*passes):
    m = {}
    for r in rows:
        m.update(r)
    merged.append(m)
print(f"{'kernel':34s} {'us':>7s} {'waves':>7s} {'valu/w':>8s} {'salu/w':>7s} {'lds/w':>6s} {'vmrd/w':>6s} {'mfma/w':>7s} "
      f"{'valu/mfma':>9s} {'mfma%':>6s} {'waitI/cyc':>9s} {'wait/cyc':>8s} {'ldsconf':>7s}")
for m in merged:
    w = max(1, m.get("SQ_WAVES", 1))
    mf = m.get("SQ_INSTS_MFMA", 0)
    busy = m.get("SQ_BUSY_CYCLES", 0)
    cyc = max(1, m.get("SQ_WAVE_CYCLES", 1))
    name = m["k"].replace("void ", "").replace("rtdm::", "")[:34]
    print(f"{name:34s} {m.get('dur', 0)/1000:7.1f} {w:7.0f} {m.get('SQ_INSTS_VALU', 0)/w:8.1f} "
          f"{m.get('SQ_INSTS_SALU', 0)/w:7.1f} {m.get('SQ_INSTS_LDS', 0)/w:6.1f} {m.get('SQ_INSTS_VMEM_RD', 0)/w:6.1f} "
          f"{mf/w:7.1f} {m.get('SQ_INSTS_VALU', 0)/max(1, mf):9.2f} "
          f"{100*m.get('SQ_VALU_MFMA_BUSY_CYCLES', 0)/max(1, busy)/4:6.1f} "
          f"{m.get('SQ_WAIT_INST_ANY', 0)/cyc:9.3f} {m.get('SQ_WAIT_ANY', 0)/cyc:8.3f} "
          f"{m.get('SQ_LDS_BANK_CONFLICT', 0)/max(1, m.get('SQ_ACTIVE_INST_LDS', 1)):7.2f}")
