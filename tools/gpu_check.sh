#!/bin/bash
# One GPU session: parity tests -> smoke -> bench -> rocprofv3 kernel trace.  Every GPU step has
# its own time limit and the chain stops at the first failure.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/${TAG:-check}
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "== pytest -m gpu"; date
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { tail -40 "$OUT/pytest_gpu.log"; exit 1; }
tail -3 "$OUT/pytest_gpu.log"
echo "== smoke"; date
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { cat "$OUT/smoke.log"; exit 1; }
cat "$OUT/smoke.log"
echo "== bench exact"; date
timeout -k 10 300 python bench.py > "$OUT/bench_exact.json" 2> "$OUT/bench_exact.err" || { tail -30 "$OUT/bench_exact.err"; exit 1; }
cat "$OUT/bench_exact.json"
echo "== bench fma"; date
timeout -k 10 300 python bench.py --numerics fma --cpu-sample 0 > "$OUT/bench_fma.json" 2> "$OUT/bench_fma.err" || { tail -30 "$OUT/bench_fma.err"; exit 1; }
cat "$OUT/bench_fma.json"
echo "== rocprofv3 kernel trace"; date
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python3 "$ROOT/bench.py" --steps 10 --warmup 2 --cpu-sample 0 > "$OUT/prof.log" 2>&1 || { tail -30 "$OUT/prof.log"; exit 1; }
find "$OUT/prof" -name "*kernel_stats.csv" -exec cat {} \;
echo "== done"; date
