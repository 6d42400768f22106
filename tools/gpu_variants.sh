#!/bin/bash
# Times every fused-kernel implementation variant (EEGFX_FUSED_IMPL) after a parity check.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/${TAG:-variants}
mkdir -p "$OUT"
for IMPL in ${IMPLS:-s20 s21 s30 s40 s41 p20 p21}; do
  export EEGFX_FUSED_IMPL=$IMPL
  timeout -k 10 120 python tools/variant_check.py > "$OUT/check_$IMPL.log" 2>&1 || { cat "$OUT/check_$IMPL.log"; exit 1; }
  for NUM in exact fma; do
    timeout -k 10 120 python bench.py --numerics $NUM --cpu-sample 0 > "$OUT/${IMPL}_${NUM}.json" 2>"$OUT/${IMPL}_$NUM.err" || { tail "$OUT/${IMPL}_$NUM.err"; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], sys.argv[3], round(d['value']/1e6,1), 'Mep/s  kernel_ms', d['roofline']['kernel_ms'], 'frac', d['roofline']['frac'])" "$OUT/${IMPL}_${NUM}.json" $IMPL $NUM
  done
done
