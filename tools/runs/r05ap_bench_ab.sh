#!/bin/bash
# Default bench line: the final library against the d5efc75 build (r05af's code,
# tools/ab_r05af/libeegfx.so, not in git), interleaved on one box, three repetitions.
set -o pipefail
OUT=gpurun_out/r05ap
mkdir -p $OUT
for rep in 1 2 3; do
  timeout -k 10 300 python -u bench.py --lib tools/ab_r05af/libeegfx.so > $OUT/old_r${rep}.json 2> $OUT/old_r${rep}.err || exit 1
  timeout -k 10 300 python -u bench.py > $OUT/new_r${rep}.json 2> $OUT/new_r${rep}.err || exit 1
done
