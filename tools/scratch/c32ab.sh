#!/bin/bash
# Wide-kernel change: GPU parity suite, c32 bench, SQ counters on window_wide_kernel.
set -euo pipefail
R=$(pwd); OUT=$R/gpurun_out/${TAG:-c32ab}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 300 python bench.py --workload c32 > $OUT/bench_c32.json 2> $OUT/bench_c32.err || { tail -20 $OUT/bench_c32.err; exit 1; }
cat $OUT/bench_c32.json
export TMPDIR=/tmp; cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_CVT SQ_INSTS_VALU_FMA_F64 SQ_INSTS_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE --kernel-include-regex window_wide_kernel --output-format csv -d $OUT/sq -o run -- python3 $R/bench.py --workload c32 --steps 5 --warmup 1 --cpu-sample 0 --alt-steps 0 > $OUT/sq.log 2>&1
