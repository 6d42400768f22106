# The step in one launch (window_fb_kernel, baselines folded into the window workgroup) against
# the two-launch step (baseline_kernel + window_kernel), same build, interleaved, three
# repetitions; fma then EXACT.  The checksums must agree between the two forms.
set -uo pipefail
OUT=gpurun_out/r05aa
mkdir -p $OUT
P=tools/probes/r05/wp_fb
for rep in 1 2 3; do
  echo -n "two-launch rep$rep: " >> $OUT/ab.log
  PROBE_STEP=1 timeout -k 10 60 $P >> $OUT/ab.log 2>&1 || { echo "two-launch failed"; tail -3 $OUT/ab.log; exit 1; }
  echo -n "one-launch rep$rep: " >> $OUT/ab.log
  PROBE_FB=1 timeout -k 10 60 $P >> $OUT/ab.log 2>&1 || { echo "one-launch failed"; tail -3 $OUT/ab.log; exit 1; }
done
for m in "PROBE_STEP=1" "PROBE_FB=1"; do
  echo -n "exact $m: " >> $OUT/ab.log
  env $m PROBE_EXACT=1 PROBE_ITERS=600 timeout -k 10 60 $P >> $OUT/ab.log 2>&1 || { echo "exact failed"; tail -3 $OUT/ab.log; exit 1; }
done
cat $OUT/ab.log
