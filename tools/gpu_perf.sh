#!/bin/bash
# Perf probes for the fused kernel: ablation timings + rocprofv3 PMC passes (one counter group
# per pass, --kernel-trace style only; never combined with sys/runtime traces).
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/${TAG:-perf}
mkdir -p "$OUT"
export TMPDIR=/tmp
BENCH="$ROOT/bench.py --steps ${STEPS:-20} --warmup 3 --cpu-sample 0"
for ABL in ${ABLS:-0 1 2 3 4}; do
  for NUM in exact fma; do
    echo "== ablation $ABL $NUM"
    EEGFX_PERF_ABLATION=$ABL timeout -k 10 200 python $BENCH --numerics $NUM > "$OUT/abl${ABL}_${NUM}.json" 2>"$OUT/abl${ABL}_${NUM}.err" || { tail "$OUT/abl${ABL}_${NUM}.err"; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['roofline'])" "$OUT/abl${ABL}_${NUM}.json"
  done
done
[ "${PMC:-1}" = "1" ] || exit 0
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 $ROOT/bench.py --steps 10 --warmup 2 --cpu-sample 0 > "$OUT/trace.log" 2>&1 || { tail -20 "$OUT/trace.log"; exit 1; }
grep -E "window|baseline" "$OUT"/trace/run_kernel_stats.csv | cut -c1-160
timeout -k 10 120 rocprofv3 -L > "$OUT/counters.txt" 2>&1 || true
i=0
while read -r GROUP; do
  [ -z "$GROUP" ] && continue
  i=$((i+1))
  echo "== pmc pass $i: $GROUP"
  timeout -k 10 300 rocprofv3 --pmc $GROUP --kernel-include-regex "${PMC_REGEX:-window}" --output-format csv -d "$OUT/pmc$i" -o run -- python3 $ROOT/bench.py --steps 5 --warmup 1 --cpu-sample 0 > "$OUT/pmc$i.log" 2>&1 || { tail -20 "$OUT/pmc$i.log"; exit 1; }
done <<'GROUPS'
SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE
SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS
SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_THREAD_CYCLES_VALU
SQ_ACTIVE_INST_VALU2 SQ_INST_LEVEL_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_UNALIGNED_STALL SQ_LDS_ADDR_CONFLICT SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_INSTS_SMEM
FETCH_SIZE
WRITE_SIZE
GROUPS
echo "== done"
