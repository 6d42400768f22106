#!/bin/bash
# The final round-5 tree: GPU suite, smoke, the default bench line and the drop-in line.
set -o pipefail
OUT=gpurun_out/r05an
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > $OUT/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" \
    > $OUT/smoke.log 2>&1 &&
timeout -k 10 300 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err &&
timeout -k 10 300 python -u bench.py --workload dropin > $OUT/bench_dropin.json 2> $OUT/bench_dropin.err
