#!/bin/bash
# A/B of baseline_kernel variants: the baseline pass alone and the whole step
# (PROBE_BASELINE / PROBE_STEP of window_probe), interleaved over two repetitions, then one
# FETCH_SIZE pass per binary on baseline_kernel.
#   VARIANTS="baseline32 baseline128" TAG=r04l bash tools/baseline_ab.sh
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/${TAG:-baseline_ab}
mkdir -p "$OUT"
export TMPDIR=/tmp
P=$ROOT/tools/probes
for rep in 1 2; do
  for v in "" ${VARIANTS:-}; do
    b=$P/window_probe${v:+_$v}
    echo -n "baseline ${v:-product} rep$rep: "; PROBE_BASELINE=1 PROBE_ITERS=3000 timeout -k 5 120 $b
    echo -n "step ${v:-product} rep$rep: "; PROBE_STEP=1 PROBE_ITERS=1500 timeout -k 5 120 $b
  done
done
cd /tmp
for v in "" ${VARIANTS:-}; do
  b=$P/window_probe${v:+_$v}
  d=$OUT/pmc_fetch_${v:-product}
  PROBE_BASELINE=1 PROBE_ITERS=20 timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex baseline_kernel --output-format csv -d $d -o run -- $b > $d.log 2>&1 || { tail -5 $d.log; exit 1; }
  python3 - "$d" "${v:-product}" <<'PY'
import csv, glob, statistics, sys
rows = [r for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)
        for r in csv.DictReader(open(f))]
vals = [float(r["Counter_Value"]) for r in rows if r.get("Counter_Name") == "FETCH_SIZE"]
kib = statistics.median(vals) if vals else float("nan")
print("%s: FETCH_SIZE median %.1f KiB per dispatch -> x2 (gfx950) %.1f B per epoch (algorithmic 608)"
      % (sys.argv[2], kib, kib * 1024 * 2 / 1e6))
PY
done
