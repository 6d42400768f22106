#!/bin/bash
# MFMA path bring-up on one GPU box: its parity tests, then bench + kernel trace.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/${TAG:-mfma}
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "== pytest mfma"; date
timeout -k 10 300 python -u -m pytest tests/test_gpu_mfma.py -x -v --timeout 120 --timeout-method thread > "$OUT/pytest_mfma.log" 2>&1 || { tail -60 "$OUT/pytest_mfma.log"; exit 1; }
tail -3 "$OUT/pytest_mfma.log"
for NUM in ${NUMS:-mfma fma}; do
  echo "== bench $NUM"; date
  timeout -k 10 200 python bench.py --numerics $NUM --cpu-sample 0 --alt-steps 0 > "$OUT/bench_$NUM.json" 2> "$OUT/bench_$NUM.err" || { tail -30 "$OUT/bench_$NUM.err"; exit 1; }
  cat "$OUT/bench_$NUM.json"
done
cd /tmp
echo "== rocprofv3 kernel trace mfma"; date
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_mfma" -o run -- python3 "$ROOT/bench.py" --numerics mfma --steps 20 --warmup 3 --cpu-sample 0 --alt-steps 0 > "$OUT/trace_mfma.log" 2>&1 || { tail -30 "$OUT/trace_mfma.log"; exit 1; }
grep -E "window|baseline" "$OUT/trace_mfma/run_kernel_stats.csv" | cut -c1-220
echo "== done"; date
