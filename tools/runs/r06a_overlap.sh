#!/bin/bash
# Round 6: the step with the baseline pass under the window kernel (two streams, K chunks)
# against the serial step (tools/probes/window_probe PROBE_OVERLAP / PROBE_STRICT).
set -euo pipefail
cd "$(dirname "$0")/../probes"
O=$GRAFT_REPO_ROOT/gpurun_out/r06a; mkdir -p $O
/opt/rocm/bin/hipcc -O3 -std=c++17 -ffp-contract=off --offload-arch=gfx950 -w -I../../include \
  -I../../eeg_dataanalysispackage_amd/csrc window_probe.hip -o window_probe
run() { echo "== $*" | tee -a $O/overlap.log; env "$@" PROBE_ITERS=1000 timeout -k 10 120 ./window_probe 2>&1 | tee -a $O/overlap.log; }
for rep in 1 2; do
  run PROBE_STEP=1
  run PROBE_OVERLAP=1 PROBE_STRICT=1
  run PROBE_OVERLAP=4 PROBE_STRICT=1
  run PROBE_OVERLAP=8 PROBE_STRICT=1
  run PROBE_OVERLAP=4 PROBE_RAMP=4 PROBE_STRICT=1
  run PROBE_OVERLAP=8 PROBE_RAMP=4 PROBE_STRICT=1
  run PROBE_OVERLAP=2
  run PROBE_OVERLAP=4
  run PROBE_WINDOW_ONLY=1
done
