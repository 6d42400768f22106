#!/bin/bash
# A/B timing of window-kernel variants on one GPU box (tools/probes/window_probe*), interleaved
# A B A B so that slow clock drift hits both, then one SQ counter pass per binary.
#   VARIANTS="v1" WIDE_VARIANTS="w1" TAG=ab1 bash tools/probe_ab.sh
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/${TAG:-ab}
mkdir -p "$OUT"
export TMPDIR=/tmp
P=$ROOT/tools/probes
ITERS=${ITERS:-2000}
for rep in 1 2; do
  for v in "" ${VARIANTS:-}; do
    b=$P/window_probe${v:+_$v}
    for num in fma ${EXACT:+exact}; do
      echo -n "c3 ${v:-product} rep$rep: "
      if [ "$num" = exact ]; then PROBE_EXACT=1 PROBE_ITERS=$ITERS timeout -k 5 120 $b; else PROBE_ITERS=$ITERS timeout -k 5 120 $b; fi
    done
  done
  for v in "" ${WIDE_VARIANTS:-}; do
    b=$P/window_probe${v:+_$v}
    echo -n "c32 ${v:-product} rep$rep: "; PROBE_WIDE=1 PROBE_ITERS=$((ITERS/3)) timeout -k 5 120 $b
  done
done
if [ "${PMC:-1}" = "1" ]; then
  cd /tmp
  for v in "" ${VARIANTS:-} ${WIDE_VARIANTS:-}; do
    b=$P/window_probe${v:+_$v}
    for wl in c3 c32; do
      if [ "$wl" = c32 ]; then export PROBE_WIDE=1; RX=window_; else unset PROBE_WIDE; RX=window_kernel; fi
      d=$OUT/pmc_${v:-product}_$wl
      PROBE_ITERS=20 timeout -s KILL 60 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_MUL_F64 SQ_WAVE_CYCLES --kernel-include-regex $RX --output-format csv -d $d -o run -- $b > $d.log 2>&1 || { tail -5 $d.log; exit 1; }
      echo "== $wl ${v:-product}"; python3 $ROOT/tools/pmc_summary.py $d
    done
  done
fi
