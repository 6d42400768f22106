#!/bin/bash
# Socket power and shader clock of window-kernel builds under sustained load (one GPU box):
# each probe runs PROBE_ITERS back-to-back launches; amd-smi samples power and clocks mid-run.
# Then one SQ/GRBM counter pass on the product (VALU issue share, effective clock).
#   TAG=power1 PROBES="window_probe window_probe_nodma window_probe_nocompute" bash tools/power_study.sh
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/${TAG:-power}
mkdir -p "$OUT"
export TMPDIR=/tmp
for p in ${PROBES:-window_probe}; do
  for wl in ${WLS:-c3}; do
    if [ "$wl" = c32 ]; then export PROBE_WIDE=1; IT=1200; else unset PROBE_WIDE; IT=4000; fi
    PROBE_ITERS=$IT timeout -k 10 60 "$ROOT/tools/probes/$p" > "$OUT/${p}_$wl.txt" 2>&1 &
    pid=$!
    sleep 2.0
    timeout 20 amd-smi metric -p -c -g 0 > "$OUT/${p}_${wl}_smi.txt" 2>&1
    wait $pid || { echo "$p failed"; cat "$OUT/${p}_$wl.txt"; exit 1; }
    echo "$p $wl: $(tail -1 "$OUT/${p}_$wl.txt" | cut -c1-60) | $(grep -E 'SOCKET_POWER' "$OUT/${p}_${wl}_smi.txt" | head -1 | xargs) | $(grep -A2 'GFX_0:' "$OUT/${p}_${wl}_smi.txt" | grep -E 'CLK:' | head -1 | xargs)"
  done
done
if [ "${PMC:-1}" = "1" ]; then
  cd /tmp
  for wl in ${WLS:-c3}; do
    if [ "$wl" = c32 ]; then export PROBE_WIDE=1; RX=window_; else unset PROBE_WIDE; RX=window_kernel; fi
    i=0
    for G in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE" \
             "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_MUL_F64 SQ_ACTIVE_INST_LDS GRBM_COUNT"; do
      i=$((i+1))
      d=$OUT/pmc_${wl}_$i
      PROBE_ITERS=400 timeout -s KILL 90 rocprofv3 --pmc $G --kernel-include-regex $RX --output-format csv -d $d -o run -- "$ROOT/tools/probes/window_probe" > $d.log 2>&1 || { tail -5 $d.log; exit 1; }
      tail -1 $d.log
      python3 "$ROOT/tools/pmc_summary.py" $d
    done
  done
fi
