#!/bin/bash
# The resident server's stream: highest priority (product) against a normal-priority stream
# (tools/ab_noprio/libeegfx.so), tools/dropin_bench interleaved, three repetitions.
set -o pipefail
OUT=gpurun_out/r05ak
mkdir -p $OUT
for rep in 1 2 3; do
  LD_LIBRARY_PATH=$PWD/tools/ab_noprio timeout -k 10 180 tools/dropin_bench . 2000 1 \
      > $OUT/noprio_r${rep}.json 2> $OUT/noprio_r${rep}.err || exit 1
  timeout -k 10 180 tools/dropin_bench . 2000 1 > $OUT/prio_r${rep}.json 2> $OUT/prio_r${rep}.err || exit 1
done
