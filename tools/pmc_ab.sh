#!/bin/bash
# SQ counter passes (one group per pass) on window_kernel* of several probe builds.
#   PROBES="window_probe window_probe_p1" TAG=pmcab bash tools/pmc_ab.sh
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/${TAG:-pmcab}
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
for p in ${PROBES:-window_probe}; do
  i=0
  for G in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS GRBM_COUNT" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_LDS SQ_INSTS_VALU_FMA_F64 SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_FLAT"; do
    i=$((i+1))
    d=$OUT/${p}_$i
    PROBE_ITERS=300 timeout -s KILL 90 rocprofv3 --pmc $G --kernel-include-regex window_ --output-format csv -d $d -o run -- "$ROOT/tools/probes/$p" > $d.log 2>&1 || { echo "pass $i of $p failed"; tail -5 $d.log; exit 1; }
    echo "== $p pass $i: $(tail -1 $d.log | cut -c1-60)"
    python3 "$ROOT/tools/pmc_summary.py" $d
  done
done
