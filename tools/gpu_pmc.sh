#!/bin/bash
# PMC passes (one group per pass, kernel trace only) on one kernel of `bench.py --numerics $NUM`.
#   NUM=fma REGEX=window_kernel TAG=x [LIB=tools/ab/<variant>/libeegfx.so] bash tools/gpu_pmc.sh
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/${TAG:-pmc}
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
i=0
while read -r GROUP; do
  [ -z "$GROUP" ] && continue
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $GROUP --kernel-include-regex "${REGEX:-window_kernel}" --output-format csv -d "$OUT/pmc$i" -o run -- python3 "$ROOT/bench.py" ${LIB:+--lib "$ROOT/$LIB"} --numerics "${NUM:-fma}" --steps 3 --warmup 1 --cpu-sample 0 --alt-steps 0 > "$OUT/pmc$i.log" 2>&1 || { tail -5 "$OUT/pmc$i.log"; exit 1; }
done <<GROUPS
${GROUPS_OVERRIDE:-SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE
SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VALU_FMA_F64 SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INST_LEVEL_VMEM
SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU_CVT SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_THREAD_CYCLES_VALU SQ_LEVEL_WAVES SQ_INSTS_VMEM
FETCH_SIZE}
GROUPS
python3 "$ROOT/tools/pmc_summary.py" "$OUT"
