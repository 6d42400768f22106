#!/bin/bash
# GPU classifier tests (logistic + SVM) and the logreg / svm bench legs.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${TAG:-svm}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_logreg.py -x -v --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -3 "$OUT/pytest.log"
for WL in logreg svm; do
  timeout -k 10 300 python bench.py --workload $WL > "$OUT/bench_$WL.json" 2> "$OUT/bench_$WL.err" || { tail -20 "$OUT/bench_$WL.err"; exit 1; }
  cat "$OUT/bench_$WL.json"
done
