#!/bin/bash
# Round-5 final tree after the timing-event change: GPU suite, smoke, default bench.
set -o pipefail
mkdir -p gpurun_out/r05af
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/r05af/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" \
    > gpurun_out/r05af/smoke.log 2>&1 &&
timeout -k 10 300 python -u bench.py > gpurun_out/r05af/bench.json 2> gpurun_out/r05af/bench.err
