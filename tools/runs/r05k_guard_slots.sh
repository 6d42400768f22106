# The guard's running counters spread over 256 slots (one shared word serialised every flagged
# workgroup's atomic): the guard / small-path GPU tests, then the flag-rate study again.
set -uo pipefail
OUT=gpurun_out/r05k
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_guard.py tests/test_gpu_epochs_features.py tests/test_gpu_c_abi.py tests/test_gpu_mailbox.py -x -q --timeout 150 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
B="--cpu-sample 0 --alt-steps 0 --steps 50 --warmup 20"
for spec in none flat:0.01 flat:0.1 flat:0.32 flat:1.0 null:0.01 null:0.1; do
  if [ $spec = none ]; then PL=""; else PL="--plant $spec"; fi
  f=$OUT/plant_${spec/:/_}
  timeout -k 10 300 python bench.py $B $PL > $f.json 2> $f.err || { tail -20 $f.err; exit 1; }
  python3 -c "
import json
d = json.load(open('$f.json'))
g = d['config']['guard']
print('$spec', 'step ms', d['ms_per_step'], 'window ms', d['roofline']['kernel_ms'], 'checked', g['rows_checked'], 'rechecked', g['rows_rechecked'], 'recomputed', g['rows_recomputed'])
"
done
