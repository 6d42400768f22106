# Host-pushed request rows (tools/probes/push_probe.hip): pool listing, then the three protocols,
# safest first; stops at the first failure.
set -uo pipefail
OUT=gpurun_out/r05j
mkdir -p $OUT
P=tools/probes/r05/push_probe
timeout -k 10 60 $P > $OUT/pools.log 2>&1; rc=$?; cat $OUT/pools.log; [ $rc -eq 0 ] || exit 1
for m in "A" "A sys" "B" "B sys" "C" "C sys"; do
  f=$OUT/mode_${m/ /_}.log
  timeout -k 10 60 $P $m > $f 2>&1; rc=$?; cat $f; [ $rc -eq 0 ] || { echo "mode $m rc=$rc"; exit 1; }
done
