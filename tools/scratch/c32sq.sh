#!/bin/bash
# SQ instruction / clock counters on window_wide_kernel (configs[3], 32 channels), one pass.
set -euo pipefail
R=$(pwd); OUT=$R/gpurun_out/c32sq; mkdir -p $OUT; export TMPDIR=/tmp; cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_CVT SQ_INSTS_VALU_FMA_F64 SQ_INSTS_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE --kernel-include-regex window_wide_kernel --output-format csv -d $OUT/sq -o run -- python3 $R/bench.py --workload c32 --steps 5 --warmup 1 --cpu-sample 0 --alt-steps 0 > $OUT/sq.log 2>&1
