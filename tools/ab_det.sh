#!/bin/bash
# Per-layer A/B of two librtdm.so builds: tools/det_roofline.py alternating RTDM_LIB between
# the in-tree library and abtmp/$1.  Usage (gpurun): bash tools/ab_det.sh OLD_SO TAG ["det_roofline args"]
set -u
OLD=$1; TAG=$2; EXTRA=${3:-}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
for I in 1 2; do
  for L in new old; do
    if [ $L = old ]; then export RTDM_LIB=$R/abtmp/$OLD; else export RTDM_LIB=$R/real-time-disaster-management_amd/rtdm/librtdm.so; fi
    timeout -k 10 200 python tools/det_roofline.py $EXTRA > $OUT/${TAG}_${L}$I.log 2>&1 || { tail -5 $OUT/${TAG}_${L}$I.log; exit 1; }
  done
done
python3 - "$OUT" "$TAG" <<'PY'
import sys, re
out, tag = sys.argv[1], sys.argv[2]
rows = {}
for L in ("new", "old"):
    for I in (1, 2):
        for line in open(f"{out}/{tag}_{L}{I}.log"):
            m = re.match(r"\s+(\d+) (\S+)\s+([\d.]+)", line)
            if m:
                rows.setdefault((int(m.group(1)), m.group(2)), {}).setdefault(L, []).append(float(m.group(3)))
            if line.startswith("forward"):
                rows.setdefault((999, "forward"), {}).setdefault(L, []).append(float(line.split()[1]))
for (l, n), d in sorted(rows.items()):
    nw, od = min(d.get("new", [0])), min(d.get("old", [0]))
    print(f"{l:4d} {n:34s} new {nw:.4f}  old {od:.4f}  {100 * (nw - od) / max(od, 1e-9):+.1f}%")
PY
