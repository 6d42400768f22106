#!/bin/bash
# The other bench workloads on the final tree (the streamed path now keeps its pinned staging).
set -o pipefail
OUT=gpurun_out/r05ar
mkdir -p $OUT
timeout -k 10 400 python -u bench.py --workload stream > $OUT/bench_stream.json 2> $OUT/bench_stream.err &&
timeout -k 10 300 python -u bench.py --workload c32 > $OUT/bench_c32.json 2> $OUT/bench_c32.err &&
timeout -k 10 400 python -u bench.py --epochs 8000000 > $OUT/bench_big.json 2> $OUT/bench_big.err &&
timeout -k 10 300 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err
