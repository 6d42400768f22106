# configs[2]'s 8M-epoch rank shard against the 1M-epoch configs[1] batch (VERDICT r04 Next #1):
# window_kernel per launch for the product tile order, no XCD remap, and 1M-epoch XCD super-tiles
# (tools/probes/r05/wp_{prod,remap0,super}), interleaved, two repetitions, with socket power and
# clocks sampled mid-run; then counter passes on the product at both sizes.
set -uo pipefail
OUT=gpurun_out/r05a
mkdir -p $OUT
export TMPDIR=/tmp
P=tools/probes/r05
run() {  # name n iters
  PROBE_N=$2 PROBE_ITERS=$3 PROBE_WARMUP=$4 timeout -k 10 120 $P/$1 > $OUT/t_$1_$2_$5.txt 2>&1 &
  pid=$!
  sleep ${6:-2.5}
  timeout 20 amd-smi metric -p -c -g 0 > $OUT/smi_$1_$2_$5.txt 2>&1
  wait $pid || { echo "$1 $2 failed"; cat $OUT/t_$1_$2_$5.txt; exit 1; }
  echo "$1 $2 rep$5: $(tail -1 $OUT/t_$1_$2_$5.txt | cut -c1-70) | $(grep -E 'SOCKET_POWER' $OUT/smi_$1_$2_$5.txt | head -1 | xargs) | $(grep -A2 'GFX_0:' $OUT/smi_$1_$2_$5.txt | grep -E 'CLK:' | head -1 | xargs)"
}
for rep in 1 2; do
  for v in wp_prod wp_remap0 wp_super; do
    run $v 1000000 6000 300 $rep 3.0
    run $v 8000000 900 40 $rep 4.5
  done
done
# the step (baseline + window) at both sizes, product
PROBE_STEP=1 PROBE_N=1000000 PROBE_ITERS=3000 timeout -k 10 120 $P/wp_prod > $OUT/step_1M.txt 2>&1 || exit 1
PROBE_STEP=1 PROBE_N=8000000 PROBE_ITERS=400 PROBE_WARMUP=40 timeout -k 10 120 $P/wp_prod > $OUT/step_8M.txt 2>&1 || exit 1
tail -1 $OUT/step_1M.txt; tail -1 $OUT/step_8M.txt
cd /tmp
R=$GRAFT_REPO_ROOT
i=0
for G in "FETCH_SIZE SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_VALU GRBM_GUI_ACTIVE GRBM_COUNT" \
         "TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_REQUEST_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_TCC_READ_REQ_LATENCY_sum TCC_EA0_RDREQ_DRAM_sum TCC_HIT_sum TCC_MISS_sum" \
         "TCP_UTCL1_TRANSLATION_MISS_UNDER_MISS_sum TCP_UTCL1_STALL_MULTI_MISS_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum SQ_ACTIVE_INST_VALU SQ_WAIT_ANY"; do
  i=$((i+1))
  for v in wp_prod wp_super; do
    for n in 1000000 8000000; do
      [ $v = wp_super ] && [ $n = 1000000 ] && continue
      d=$R/$OUT/pmc_${v}_${n}_$i
      PROBE_N=$n PROBE_ITERS=20 PROBE_WARMUP=20 timeout -s KILL 120 rocprofv3 --pmc $G --kernel-include-regex window_kernel --output-format csv -d $d -o run -- $R/$P/$v > $d.log 2>&1 || { echo "pmc $i $v $n failed"; tail -5 $d.log; exit 1; }
      echo "== pass $i $v $n"
      python3 $R/tools/pmc_summary.py $d | tee $d.summary
    done
  done
done
