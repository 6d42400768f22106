#!/bin/bash
# Round evidence on one GPU box: parity tests -> smoke -> bench (fma headline, exact alt) ->
# rocprofv3 kernel trace + stats of the bench -> PMC FETCH_SIZE / WRITE_SIZE passes on
# window_kernel (one counter per pass, kernel trace only) -> traffic summaries -> extra workloads.
# Every GPU step has its own time limit; the chain stops at the first failure.
#   TAG=r02a TESTS=1 NUMS="fma exact" EXTRA="c32 stream dropin big" bash tools/gpu_round.sh
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
TAG=${TAG:-round}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ "${TESTS:-1}" = "1" ]; then
  echo "== pytest -m gpu"; date
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { tail -60 "$OUT/pytest_gpu.log"; exit 1; }
  tail -3 "$OUT/pytest_gpu.log"
  echo "== smoke"; date
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { cat "$OUT/smoke.log"; exit 1; }
  cat "$OUT/smoke.log"
fi
if [ "${BENCH:-1}" = "1" ]; then
  echo "== bench"; date
  timeout -k 10 400 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -30 "$OUT/bench.err"; exit 1; }
  cat "$OUT/bench.json"
fi
cd /tmp
for NUM in ${NUMS:-fma}; do
  echo "== rocprofv3 kernel trace $NUM"; date
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_$NUM" -o run -- python3 "$ROOT/bench.py" --numerics $NUM --cpu-sample 0 --alt-steps 0 > "$OUT/trace_$NUM.log" 2>&1 || { tail -30 "$OUT/trace_$NUM.log"; exit 1; }
  tail -1 "$OUT/trace_$NUM.log"
  find "$OUT/trace_$NUM" -name "*kernel_stats.csv" -exec cut -c1-200 {} \;
  for C in FETCH_SIZE WRITE_SIZE; do
    echo "== pmc $C $NUM"; date
    timeout -k 10 300 rocprofv3 --pmc $C --kernel-include-regex window_kernel --output-format csv -d "$OUT/pmc_${C}_$NUM" -o run -- python3 "$ROOT/bench.py" --numerics $NUM --steps 5 --warmup 1 --cpu-sample 0 --alt-steps 0 > "$OUT/pmc_${C}_$NUM.log" 2>&1 || { tail -30 "$OUT/pmc_${C}_$NUM.log"; exit 1; }
  done
  python3 "$ROOT/tools/traffic_summary.py" --fetch "$OUT/pmc_FETCH_SIZE_$NUM" --write "$OUT/pmc_WRITE_SIZE_$NUM" \
    --kernel window_kernel --workload-key "fused_dwt8_c3_int16_1000000_$NUM" \
    --algorithmic-bytes 3476000000 --out "$OUT/traffic_$NUM.json"
done
if [ "${C32TRAFFIC:-1}" = "1" ]; then  # configs[3]'s dominant kernel: trace + traffic passes
  echo "== rocprofv3 kernel trace c32"; date
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_c32" -o run -- python3 "$ROOT/bench.py" --workload c32 --cpu-sample 0 --alt-steps 0 > "$OUT/trace_c32.log" 2>&1 || { tail -30 "$OUT/trace_c32.log"; exit 1; }
  for C in FETCH_SIZE WRITE_SIZE; do
    echo "== pmc $C c32"; date
    timeout -k 10 300 rocprofv3 --pmc $C --kernel-include-regex window_c32 --output-format csv -d "$OUT/pmc_${C}_c32" -o run -- python3 "$ROOT/bench.py" --workload c32 --steps 5 --warmup 1 --cpu-sample 0 --alt-steps 0 > "$OUT/pmc_${C}_c32.log" 2>&1 || { tail -30 "$OUT/pmc_${C}_c32.log"; exit 1; }
  done
  python3 "$ROOT/tools/traffic_summary.py" --fetch "$OUT/pmc_FETCH_SIZE_c32" --write "$OUT/pmc_WRITE_SIZE_c32" \
    --kernel window_c32 --workload-key "fused_dwt8_c32_int16_250000_fma" \
    --algorithmic-bytes 9250000000 --out "$OUT/traffic_c32_fma.json"
fi
cd "$ROOT"
for WL in ${EXTRA:-c32 stream dropin big}; do
  echo "== bench $WL"; date
  if [ "$WL" = "big" ]; then  # configs[2]: one rank's 8M-epoch shard (48 GB recording)
    timeout -k 10 400 python bench.py --epochs 8000000 --steps 20 --warmup 10 --cpu-sample 0 --alt-steps 3 > "$OUT/bench_$WL.json" 2> "$OUT/bench_$WL.err" || { tail -30 "$OUT/bench_$WL.err"; exit 1; }
  else
    timeout -k 10 400 python bench.py --workload $WL > "$OUT/bench_$WL.json" 2> "$OUT/bench_$WL.err" || { tail -30 "$OUT/bench_$WL.err"; exit 1; }
  fi
  cat "$OUT/bench_$WL.json"
done
echo "== done"; date
