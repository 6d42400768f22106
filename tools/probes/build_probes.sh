#!/bin/bash
# Builds the perf probes in-tree (they travel to the GPU box with the snapshot).
set -euo pipefail
cd "$(dirname "$0")"
HIPCC=${HIPCC:-/opt/rocm/bin/hipcc}
FL="-O3 -std=c++17 -ffp-contract=off --offload-arch=gfx950 -w -I../../include -I../../eeg_dataanalysispackage_amd/csrc"
for A in 0 1 2 3; do
  $HIPCC $FL -DEEGFX_MFMA_ABLATION=$A mfma_probe.hip ../../eeg_dataanalysispackage_amd/csrc/dwt8_operator.cpp -o mfma_probe_$A &
done
for A in 0 1 2 3 4 5 6 7 8 16 24; do
  $HIPCC $FL -DEEGFX_FUSED_ABLATION=$A window_probe.hip -o window_probe_$A &
done
for p in fp64_probe cascade_probe mem_probe; do $HIPCC $FL $p.hip -o $p & done
for M in 1 2; do
  $HIPCC $FL -DEEGFX_STORE_MODE=$M window_probe.hip -o window_probe_s$M &
done
wait
