#!/bin/bash
# window_kernel ablation times + one SQ counter pass on the product probe.
set -euo pipefail
OUT=$(pwd)/gpurun_out/abl; mkdir -p $OUT; export TMPDIR=/tmp
for A in 0 1 2 3 4 5 6 7; do timeout -k 10 60 tools/probes/window_probe_$A; done
P=$(pwd)/tools/probes/window_probe_0
cd /tmp
timeout -s KILL 60 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE --kernel-include-regex window_kernel --output-format csv -d $OUT/p1 -o run -- $P > $OUT/p1.log 2>&1
timeout -s KILL 60 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INST_LEVEL_VMEM SQ_LDS_BANK_CONFLICT --kernel-include-regex window_kernel --output-format csv -d $OUT/p2 -o run -- $P > $OUT/p2.log 2>&1
