#!/bin/bash
# round 6: full GPU suite on the register-rows window kernel + streamed-rows change, then the
# flag-rate A/B (product vs EEGFX_REG_ROWS=0) and the stream line.
set -uo pipefail
OUT=gpurun_out/r06g; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log
TAG=r06g LIBS="new: regoff:tools/ab/regoff/libeegfx.so" SPECS="none flat:0.32" REPS=3 bash tools/runs/bench_ab.sh || exit 1
timeout -k 10 300 python bench.py --workload stream --steps 10 --warmup 3 > $OUT/bench_stream.json 2> $OUT/bench_stream.err || { tail -20 $OUT/bench_stream.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench_stream.json')); print('stream', d['ms_per_step'], d['host_link'], (d.get('cpu_baseline') or {}).get('value'))"
