# (1) GPU tests of this round's changes: the guard's second stage (every int16 fma kernel), the
#     mini-batch logistic regression, the Java shim's call sequence from C, the resident
#     per-epoch server, the unaligned-features route; then the per-epoch drop-in latency with
#     and without the resident server (tools/dropin_bench);
# (2) the guard's flag-rate study on the fast second stage (--plant flat / null);
# (3) window kernel with 1, 2, 3 sub-tiles per workgroup (EEGFX_WIN_SUBS, probes wp_s1..3) and
#     the 32-channel kernel one-epoch-per-workgroup vs persistent ping-pong (wp_c32base /
#     wp_c32pp), interleaved, three repetitions.
set -uo pipefail
OUT=gpurun_out/r05h
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_gpu_guard.py tests/test_gpu_logreg.py tests/test_gpu_c_abi.py tests/test_gpu_epochs_features.py tests/test_gpu_mailbox.py -x -q --timeout 150 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
timeout -k 10 120 ./tools/dropin_bench . 2000 1 > $OUT/dropin_fma.json 2> $OUT/dropin_fma.err || { tail -20 $OUT/dropin_fma.err; exit 1; }
timeout -k 10 120 ./tools/dropin_bench . 2000 0 > $OUT/dropin_exact.json 2> $OUT/dropin_exact.err || { tail -20 $OUT/dropin_exact.err; exit 1; }
cat $OUT/dropin_fma.json

B="--cpu-sample 0 --alt-steps 0 --steps 50 --warmup 20"
for spec in none flat:0.01 flat:0.1 flat:0.32 flat:1.0 null:0.01 null:0.1 null:0.32; do
  if [ $spec = none ]; then PL=""; else PL="--plant $spec"; fi
  timeout -k 10 300 python bench.py $B $PL > $OUT/plant_${spec/:/_}.json 2> $OUT/plant_${spec/:/_}.err || { tail -20 $OUT/plant_${spec/:/_}.err; exit 1; }
  python3 -c "
import json
d = json.load(open('$OUT/plant_${spec/:/_}.json'))
g = d['config']['guard']
print('$spec', 'step ms', d['ms_per_step'], 'window ms', d['roofline']['kernel_ms'], 'checked', g['rows_checked'], 'rechecked', g['rows_rechecked'], 'recomputed', g['rows_recomputed'])
"
done
P=tools/probes/r05
for rep in 1 2 3; do
  for v in wp_s1 wp_s2 wp_s3; do
    timeout -k 10 60 $P/$v >> $OUT/subs_window.log 2>&1 || { echo "$v failed"; tail -3 $OUT/subs_window.log; exit 1; }
    PROBE_STEP=1 timeout -k 10 60 $P/$v >> $OUT/subs_step.log 2>&1 || { echo "$v step failed"; exit 1; }
  done
  for v in wp_c32base2 wp_c32pp2; do
    PROBE_WIDE=1 PROBE_ITERS=1000 timeout -k 10 60 $P/$v >> $OUT/c32_window.log 2>&1 || { echo "$v failed"; tail -3 $OUT/c32_window.log; exit 1; }
  done
done
echo "== window (s1 s2 s3 x3)"; cat $OUT/subs_window.log; echo "== step"; cat $OUT/subs_step.log
echo "== c32 (base pp x3)"; cat $OUT/c32_window.log
