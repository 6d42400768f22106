# Round 5 bench study on one box:
#  (1) the guard's second stage costs nothing on the headline: window kernel and step of HEAD's
#      sources (wp_head) against the tree's (wp_new), interleaved, three repetitions;
#  (2) bench.py at configs[1] (1M) and configs[2]'s rank shard (8M), interleaved, twice; the
#      8M shard in one call against 8 slices (tools/chunk_probe.py);
#  (3) the guard's flag-rate study: --plant flat / null at 0, 1, 10, 32, 100 % of the markers;
#  (4) FETCH_SIZE / WRITE_SIZE passes on the 8M shard's window_kernel (traffic for its key);
#  (5) the complete 8M line (cpu_baseline included).
set -uo pipefail
OUT=gpurun_out/r05b
mkdir -p $OUT
export TMPDIR=/tmp
P=tools/probes/r05
B="--cpu-sample 0 --alt-steps 0"
for rep in 1 2 3; do
  for v in wp_head wp_new; do
    timeout -k 10 60 $P/$v >> $OUT/ab_window.log 2>&1 || { echo "$v failed"; exit 1; }
    PROBE_STEP=1 timeout -k 10 60 $P/$v >> $OUT/ab_step.log 2>&1 || { echo "$v step failed"; exit 1; }
  done
done
echo "== (1) window"; cat $OUT/ab_window.log; echo "== (1) step"; cat $OUT/ab_step.log
for rep in 1 2; do
  timeout -k 10 300 python bench.py --steps 100 --warmup 50 $B > $OUT/bench_1M_$rep.json 2> $OUT/bench_1M_$rep.err || { tail -20 $OUT/bench_1M_$rep.err; exit 1; }
  timeout -k 10 300 python bench.py --epochs 8000000 --steps 20 --warmup 10 $B > $OUT/bench_8M_$rep.json 2> $OUT/bench_8M_$rep.err || { tail -20 $OUT/bench_8M_$rep.err; exit 1; }
  python3 -c "
import json
for k in ('1M', '8M'):
    d = json.load(open('$OUT/bench_%s_$rep.json' % k))
    n = d['config']['epochs_per_gpu'] / 1e6
    print(k, 'value', d['value'], 'step/1M', round(d['ms_per_step'] / n, 4), 'window/1M', round(d['roofline']['kernel_ms'] / n, 4), 'frac', d['roofline']['frac'], 'whole', d['roofline']['whole_path']['frac'])
"
done
timeout -k 10 300 python tools/chunk_probe.py --slices 1,8 --rounds 3 --reps 10 > $OUT/chunk.log 2>&1 || { tail -20 $OUT/chunk.log; exit 1; }
tail -7 $OUT/chunk.log
echo "== (3) flag rates"
for spec in none flat:0.01 flat:0.1 flat:0.32 flat:1.0 null:0.01 null:0.1 null:0.32 null:1.0; do
  if [ $spec = none ]; then PL=""; else PL="--plant $spec"; fi
  timeout -k 10 300 python bench.py --steps 50 --warmup 20 $B $PL > $OUT/plant_${spec/:/_}.json 2> $OUT/plant_${spec/:/_}.err || { tail -20 $OUT/plant_${spec/:/_}.err; exit 1; }
  python3 -c "
import json
d = json.load(open('$OUT/plant_${spec/:/_}.json'))
g = d['config']['guard']
print('$spec', 'step ms', d['ms_per_step'], 'window ms', d['roofline']['kernel_ms'], 'checked', g['rows_checked'], 'rechecked', g['rows_rechecked'], 'recomputed', g['rows_recomputed'], 'ref', g['reference_recordings'])
"
done
echo "== (4) 8M traffic"
cd /tmp
R=$GRAFT_REPO_ROOT
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $C --kernel-include-regex window_kernel --output-format csv -d $R/$OUT/pmc_${C}_8M -o run -- python3 $R/bench.py --epochs 8000000 --steps 3 --warmup 1 $B > $R/$OUT/pmc_${C}_8M.log 2>&1 || { tail -20 $R/$OUT/pmc_${C}_8M.log; exit 1; }
done
python3 $R/tools/traffic_summary.py --fetch $R/$OUT/pmc_FETCH_SIZE_8M --write $R/$OUT/pmc_WRITE_SIZE_8M \
  --kernel window_kernel --workload-key fused_dwt8_c3_int16_8000000_fma \
  --algorithmic-bytes 27808000000 --out $R/$OUT/traffic_8M_fma.json || exit 1
cat $R/$OUT/traffic_8M_fma.json
cd $R
cp $OUT/traffic_8M_fma.json profiles/r05b_traffic_8M_fma.json  # what bench.py reads for the key
echo "== (5) the 8M line"
timeout -k 10 400 python bench.py --epochs 8000000 --steps 20 --warmup 10 --alt-steps 3 > $OUT/bench_big.json 2> $OUT/bench_big.err || { tail -20 $OUT/bench_big.err; exit 1; }
cat $OUT/bench_big.json
