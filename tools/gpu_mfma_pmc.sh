#!/bin/bash
# MFMA kernel perf study: ablation timings + PMC passes on the product build of the probe.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/${TAG:-mfmapmc}
mkdir -p "$OUT"
export TMPDIR=/tmp
cd tools/probes
for A in 0 1 2 3; do timeout -k 5 60 ./mfma_probe_$A; done
cd /tmp
i=0
while read -r GROUP; do
  [ -z "$GROUP" ] && continue
  i=$((i+1))
  timeout -s KILL 60 rocprofv3 --pmc $GROUP --kernel-include-regex mfma_window --output-format csv -d "$OUT/pmc$i" -o run -- "$ROOT/tools/probes/mfma_probe_0" > "$OUT/pmc$i.log" 2>&1 || { tail -5 "$OUT/pmc$i.log"; exit 1; }
done <<'GROUPS'
SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE
SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INST_LEVEL_VMEM
FETCH_SIZE
GROUPS
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
tot = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "/pmc*/**/*counter_collection.csv", recursive=True):
    per = collections.defaultdict(float)
    for r in csv.DictReader(open(f)):
        per[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
    for (d, c), v in per.items():
        tot[c].append(v)
for c, v in sorted(tot.items()):
    print(f"{c:28s} {sorted(v)[len(v)//2]:.4g}")
PY
