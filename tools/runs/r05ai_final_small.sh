#!/bin/bash
# Final tree after the per-epoch change: GPU suite, smoke, parity sweeps that now include the
# per-epoch kernel and the resident server, and the drop-in bench line (second run: after the
# streamed staging became grow-only; the first sweep stalled on hipHostFree behind the server).
set -o pipefail
OUT=gpurun_out/r05ai
mkdir -p $OUT
timeout -k 10 120 python -u -m pytest tests/test_gpu_mailbox.py -x -q -s --timeout 120 --timeout-method thread > $OUT/pytest_mailbox.log 2>&1 &&
timeout -k 10 60 python -u tools/probes/sweep_timing.py > $OUT/sweep_timing.log 2>&1 &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > $OUT/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" \
    > $OUT/smoke.log 2>&1 &&
timeout -k 10 600 python -u tools/parity_sweep.py --cases 15000 --seed0 400000 --max-seconds 240 \
    --out $OUT/parity_sweep_15000.json > $OUT/sweep.log 2>&1 &&
timeout -k 10 600 python -u tools/parity_sweep.py --cases 15000 --seed0 500000 --flat --max-seconds 240 \
    --out $OUT/parity_sweep_flat_15000.json > $OUT/sweep_flat.log 2>&1 &&
timeout -k 10 300 python -u bench.py --workload dropin > $OUT/bench_dropin.json 2> $OUT/bench_dropin.err
