#!/bin/bash
set -euo pipefail
OUT=$(pwd)/gpurun_out/nospill; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_mfma.py -m gpu -x -q --timeout 120 --timeout-method thread 2>&1 | tail -1
for NUM in fma exact; do echo -n "$NUM: "; timeout -k 10 200 python bench.py --numerics $NUM --cpu-sample 0 --alt-steps 0 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["kernel_ms"], d["roofline"]["frac"])'; done
R=$(pwd)
cd /tmp
for NUM in fma exact; do for C in WRITE_SIZE FETCH_SIZE; do
timeout -s KILL 90 rocprofv3 --pmc $C --kernel-include-regex window_kernel --output-format csv -d $OUT/${NUM}_$C -o run -- python3 $R/bench.py --numerics $NUM --steps 5 --warmup 1 --cpu-sample 0 --alt-steps 0 > $OUT/${NUM}_$C.log 2>&1
done; python3 $R/tools/traffic_summary.py --fetch $OUT/${NUM}_FETCH_SIZE --write $OUT/${NUM}_WRITE_SIZE --kernel window_kernel --workload-key "fused_dwt8_c3_int16_1000000_$NUM" --algorithmic-bytes 3476000000 --out $OUT/traffic_$NUM.json | cut -c1-400; done
