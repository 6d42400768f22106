#!/bin/bash
# The per-epoch drop-in at Spark local[*] thread counts: the bench line (tools/dropin_bench:
# single-epoch latency launched and resident, 2-32 threads with a server each) and the native
# harness tests/c_abi/mailbox_threads.c (built as tools/mailbox_threads) at 4, 5, 8, 16, 32 threads.
set -uo pipefail
OUT=gpurun_out/${TAG:?}; mkdir -p $OUT
timeout -k 10 600 python bench.py --workload dropin > $OUT/bench_dropin.json 2> $OUT/bench_dropin.err || { tail -20 $OUT/bench_dropin.err; exit 1; }
cat $OUT/bench_dropin.json
for T in 4 5 8 16 32; do
  timeout -k 10 120 tools/mailbox_threads tests/golden/test-data/DoD/DoD2015_01.vhdr $T 500 2>&1 | tee -a $OUT/mailbox_threads.log || exit 1
done
