# Where the guard's second stage costs: SQ counters of window_kernel with no planted windows and
# with 32 % flat windows (bench.py --plant), one counter pass each.
set -uo pipefail
OUT=$PWD/gpurun_out/r05q
mkdir -p $OUT
ROOT=$PWD
cd /tmp
export TMPDIR=/tmp
CTR="SQ_INSTS_VALU SQ_WAVES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU"
for spec in none flat:0.32 flat:1.0; do
  if [ $spec = none ]; then PL=""; else PL="--plant $spec"; fi
  tag=${spec/:/_}
  timeout -k 10 300 rocprofv3 --pmc $CTR --kernel-include-regex window_kernel --output-format csv -d $OUT/pmc_$tag -o run -- python3 $ROOT/bench.py --steps 5 --warmup 1 --cpu-sample 0 --alt-steps 0 $PL > $OUT/pmc_$tag.log 2>&1 || { tail -20 $OUT/pmc_$tag.log; exit 1; }
  python3 $ROOT/tools/pmc_summary.py $OUT/pmc_$tag > $OUT/pmc_$tag.summary 2>&1 || true
  echo "== $spec"; cat $OUT/pmc_$tag.summary | head -20
done
