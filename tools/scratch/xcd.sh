#!/bin/bash
set -euo pipefail
R=$(pwd); OUT=$R/gpurun_out/xcd; mkdir -p $OUT; export TMPDIR=/tmp
for SP in 1000 100; do for V in 0 nox; do
  echo -n "spacing $SP $V: "; PROBE_SPACING=$SP PROBE_RANDOM=1 PROBE_ITERS=1000 timeout -k 10 60 tools/probes/window_probe_$V
done; done
cd /tmp
for V in 0 nox; do
  PROBE_SPACING=100 PROBE_RANDOM=1 timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex window_kernel --output-format csv -d $OUT/f_$V -o run -- $R/tools/probes/window_probe_$V > $OUT/f_$V.log 2>&1
  python3 - $OUT/f_$V <<'PY'
import csv,glob,sys,statistics
f=glob.glob(sys.argv[1]+'/**/*counter_collection.csv',recursive=True)[0]
v=[float(r['Counter_Value']) for r in csv.DictReader(open(f))]
print(sys.argv[1].split('/')[-1], 'FETCH bytes/launch (x2 corrected)', statistics.median(v)*1024*2/1e9, 'GB')
PY
done
