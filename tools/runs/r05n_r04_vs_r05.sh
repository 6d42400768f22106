# The round-4 window kernels (built from commit 9664984's sources) against this round's, on one
# box, interleaved: window launches alone and whole steps (baseline + window), three repetitions.
set -uo pipefail
OUT=gpurun_out/r05n
mkdir -p $OUT
P=tools/probes/r05
for rep in 1 2 3; do
  for v in wp_r04 wp_r05; do
    echo -n "$v rep$rep window: " >> $OUT/ab.log
    timeout -k 10 60 $P/$v >> $OUT/ab.log 2>&1 || { echo "$v failed"; exit 1; }
    echo -n "$v rep$rep step: " >> $OUT/ab.log
    PROBE_STEP=1 timeout -k 10 60 $P/$v >> $OUT/ab.log 2>&1 || { echo "$v step failed"; exit 1; }
  done
done
cat $OUT/ab.log
