#!/bin/bash
# Interleaved A/B of window_probe builds (tools/probes/window_probe.hip) on one box.
#   TAG=r06b VARIANTS="base:;b64:-DEEGFX_LDS_B64=1" MODES="PROBE_STEP=1;" REPS=3 bash tools/runs/probe_ab.sh
# VARIANTS: name:defines pairs separated by ';' (each built against the product sources with the
# defines); MODES: probe environments separated by ';' (empty = the window kernel alone).
# Output: gpurun_out/$TAG/ab.log (one line per run).
set -euo pipefail
cd "$(dirname "$0")/../probes"
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:?}; mkdir -p $O
IFS=';' read -ra VS <<< "${VARIANTS:?}"
IFS=';' read -ra MS <<< "${MODES:-PROBE_STEP=1;}"
pids=()
for v in "${VS[@]}"; do
  name=${v%%:*}; defs=${v#*:}
  /opt/rocm/bin/hipcc -O3 -std=c++17 -ffp-contract=off --offload-arch=gfx950 -w -I../../include \
    -I../../eeg_dataanalysispackage_amd/csrc $defs window_probe.hip -o wp_$name & pids+=($!)
done
for p in "${pids[@]}"; do wait $p; done
for rep in $(seq ${REPS:-2}); do
  for m in "${MS[@]}"; do
    for v in "${VS[@]}"; do
      name=${v%%:*}
      line=$(env $m PROBE_ITERS=${ITERS:-1000} timeout -k 10 120 ./wp_$name 2>/dev/null | tail -1)
      echo "rep=$rep mode=[$m] $name: $line" | tee -a $O/ab.log
    done
  done
done
