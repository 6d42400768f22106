#!/bin/bash
set -euo pipefail
R=$(pwd); OUT=$R/gpurun_out/c32pmc; mkdir -p $OUT; export TMPDIR=/tmp; cd /tmp
for C in FETCH_SIZE WRITE_SIZE; do
timeout -s KILL 120 rocprofv3 --pmc $C --kernel-include-regex window_wide_kernel --output-format csv -d $OUT/$C -o run -- python3 $R/bench.py --workload c32 --steps 5 --warmup 1 --cpu-sample 0 --alt-steps 0 > $OUT/$C.log 2>&1
done
python3 $R/tools/traffic_summary.py --fetch $OUT/FETCH_SIZE --write $OUT/WRITE_SIZE --kernel window_wide_kernel --workload-key fused_dwt8_c32_int16_250000_fma --algorithmic-bytes 9250000000 --out $OUT/traffic_c32_fma.json
