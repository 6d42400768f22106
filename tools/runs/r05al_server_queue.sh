#!/bin/bash
# The resident server's stream priority: other contexts' streamed calls and 11-epoch batches beside
# it (tools/probes/server_stall.py), for the product (highest priority), a normal-priority stream
# and the lowest priority (tools/ab_noprio/, tools/ab_low/); then tools/dropin_bench on the low build.
set -o pipefail
OUT=gpurun_out/r05al
mkdir -p $OUT
for rep in 1 2; do
  for v in prio noprio low; do
    lib=eeg_dataanalysispackage_amd/libeegfx.so
    [ $v = noprio ] && lib=tools/ab_noprio/libeegfx.so
    [ $v = low ] && lib=tools/ab_low/libeegfx.so
    timeout -k 10 120 python -u tools/probes/server_stall.py $lib > $OUT/${v}_r${rep}.json 2> $OUT/${v}_r${rep}.err || exit 1
  done
done
LD_LIBRARY_PATH=$PWD/tools/ab_low timeout -k 10 180 tools/dropin_bench . 2000 1 > $OUT/dropin_low.json 2> $OUT/dropin_low.err
