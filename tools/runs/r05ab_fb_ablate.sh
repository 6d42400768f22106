# Where the one-launch step's extra time goes: the fold skipped (FB_NOFOLD) and the pre-stimulus
# DMAs skipped (FB_NOBASEDMA), against the full one-launch kernel and the two-launch step.
set -uo pipefail
OUT=gpurun_out/r05ab
mkdir -p $OUT
P=tools/probes/r05
for rep in 1 2; do
  for v in "wp_fb PROBE_STEP=1" "wp_fb PROBE_FB=1" "wp_fb_NOFOLD PROBE_FB=1" "wp_fb_NOBASEDMA PROBE_FB=1"; do
    set -- $v
    echo -n "$1 $2 rep$rep: " >> $OUT/ab.log
    env $2 timeout -k 10 60 $P/$1 >> $OUT/ab.log 2>&1 || { echo "$v failed"; tail -3 $OUT/ab.log; exit 1; }
  done
done
cat $OUT/ab.log
