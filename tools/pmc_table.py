#!/usr/bin/env python3
"""Per-dispatch PMC table from tools/pmc_detector.sh output (last iteration of run_detector.py).
python tools/pmc_table.py TAG [npasses]

Columns: us = dispatch time; GHz = GRBM_GUI_ACTIVE / 8 XCDs / wall (effective clock);
mfma% = SQ_VALU_MFMA_BUSY_CYCLES over all SIMD-cycles (GRBM_GUI_ACTIVE x 128);
wait/inst/act = SQ_WAIT_ANY / SQ_WAIT_INST_ANY / SQ_ACTIVE_INST_ANY shares of SQ_WAVE_CYCLES;
ldsconf = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE; lds% = SQ_LDS_IDX_ACTIVE over all CU-cycles
(GRBM_GUI_ACTIVE x 256 CUs / 8 XCDs: the LDS-array busy share); l2hit = TCC_HIT / (TCC_HIT + TCC_MISS)."""
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


def g(m, k, default=0.0):
    return float(m.get(k, default))


print(f"{'kernel':34s} {'us':>7s} {'GHz':>5s} {'waves':>6s} {'mfma/w':>7s} {'mfma%':>6s} {'wait':>5s} {'inst':>5s} "
      f"{'act':>5s} {'ldsI/w':>6s} {'ldsconf':>7s} {'lds%':>5s} {'vmrd/w':>6s} {'valu/w':>7s} {'l2hit':>6s}")
for m in merged:
    w = max(1.0, g(m, "SQ_WAVES", 1))
    cyc = max(1.0, g(m, "SQ_WAVE_CYCLES", 1))
    dur = g(m, "dur") / 1e9
    ghz = g(m, "GRBM_GUI_ACTIVE") / 8 / dur / 1e9 if dur > 0 and "GRBM_GUI_ACTIVE" in m else 0.0
    gui = g(m, "GRBM_GUI_ACTIVE")  # summed over the 8 XCDs: x 1024 SIMDs / 8 = SIMD-cycles / 128
    mf = 100 * g(m, "SQ_VALU_MFMA_BUSY_CYCLES") / max(1.0, gui * 128) if gui else 0.0
    hit, miss = g(m, "TCC_HIT_sum"), g(m, "TCC_MISS_sum")
    name = m["k"].replace("void ", "").replace("rtdm::", "")[:34]
    print(f"{name:34s} {g(m, 'dur') / 1000:7.1f} {ghz:5.2f} {w:6.0f} {g(m, 'SQ_INSTS_MFMA') / w:7.1f} {mf:6.1f} "
          f"{g(m, 'SQ_WAIT_ANY') / cyc:5.2f} {g(m, 'SQ_WAIT_INST_ANY') / cyc:5.2f} {g(m, 'SQ_ACTIVE_INST_ANY') / cyc:5.2f} "
          f"{g(m, 'SQ_INSTS_LDS') / w:6.1f} {g(m, 'SQ_LDS_BANK_CONFLICT') / max(1.0, g(m, 'SQ_LDS_IDX_ACTIVE', 1)):7.3f} "
          f"{100 * g(m, 'SQ_LDS_IDX_ACTIVE') / max(1.0, gui * 32):5.1f} "
          f"{g(m, 'SQ_INSTS_VMEM_RD') / w:6.1f} {g(m, 'SQ_INSTS_VALU') / w:7.1f} {hit / max(1.0, hit + miss):6.3f}")
