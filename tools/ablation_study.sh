#!/bin/bash
# Energy split of the window kernel: the product probe and the ablation
# builds of tools/probes/ablations/ under sustained load, each with socket power and shader clock
# (amd-smi, sampled mid-run) and one SQ counter pass (instruction mix per wave).
#   TAG=r03d_ablate ABL="cascade nodma l2src regdirect nofp64" bash tools/ablation_study.sh
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/${TAG:-ablate}
mkdir -p "$OUT"
export TMPDIR=/tmp
ABL=${ABL:-"cascade nodma l2src regdirect nofp64"}
ABL="$ABL" bash tools/probes/build_probes.sh || { echo "probe build failed"; exit 1; }
PROBES="window_probe"
for a in $ABL; do PROBES="$PROBES window_probe_$a"; done
TAG=${TAG:-ablate} PROBES="$PROBES" WLS="${WLS:-c3}" PMC=0 bash tools/power_study.sh || exit 1
cd /tmp
for p in $PROBES; do
  for wl in ${WLS:-c3}; do
    if [ "$wl" = c32 ]; then export PROBE_WIDE=1; RX=window_; else unset PROBE_WIDE; RX=window_kernel; fi
    d=$OUT/pmc_${p}_$wl
    PROBE_ITERS=200 timeout -s KILL 60 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_CVT SQ_WAVE_CYCLES --kernel-include-regex $RX --output-format csv -d $d -o run -- "$ROOT/tools/probes/$p" > $d.log 2>&1 || { echo "pmc $p failed"; tail -5 $d.log; exit 1; }
    echo "== $p $wl"; python3 "$ROOT/tools/pmc_summary.py" $d
  done
done
