#!/bin/bash
# Store-mode study: time + WRITE_SIZE / FETCH_SIZE of window_kernel per EEGFX_STORE_MODE probe.
set -euo pipefail
ROOT=$(pwd); OUT=$ROOT/gpurun_out/store; mkdir -p $OUT; export TMPDIR=/tmp
for M in s0 s1 s2; do
  timeout -k 10 60 $ROOT/tools/probes/window_probe_$M
  timeout -k 10 60 $ROOT/tools/probes/window_probe_$M
done
cd /tmp
for M in s0 s1 s2; do
  for C in WRITE_SIZE FETCH_SIZE; do
    timeout -s KILL 60 rocprofv3 --pmc $C --kernel-include-regex window_kernel --output-format csv -d $OUT/${M}_$C -o run -- $ROOT/tools/probes/window_probe_$M > $OUT/${M}_$C.log 2>&1
    python3 - $OUT/${M}_$C <<'PY'
import csv,glob,sys,statistics
f=glob.glob(sys.argv[1]+'/**/*counter_collection.csv',recursive=True)[0]
v=[float(r['Counter_Value']) for r in csv.DictReader(open(f))]
print(sys.argv[1].split('/')[-1], 'KiB/launch median', statistics.median(v), 'bytes/epoch', statistics.median(v)*1024/1e6)
PY
  done
done
