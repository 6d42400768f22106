#!/bin/bash
# Builds the perf probes in-tree (they travel to the GPU box with the snapshot):
#   window_probe          the product window / wide kernels under sustained load
#   window_probe_<v>      the same against tools/probes/variants/<v>/{fused,wide}.hip (A/B studies)
#   fp64_probe, cascade_probe, mem_probe, dma_probe   micro-benchmarks
set -euo pipefail
cd "$(dirname "$0")"
HIPCC=${HIPCC:-/opt/rocm/bin/hipcc}
FL="-O3 -std=c++17 -ffp-contract=off --offload-arch=gfx950 -w -I../../include -I../../eeg_dataanalysispackage_amd/csrc"
$HIPCC $FL window_probe.hip -o window_probe &
for d in variants/*/; do
  [ -d "$d" ] || continue
  v=$(basename "$d")
  defs=()
  [ -f "$d/fused.hip" ] && defs+=("-DFUSED_SRC=\"variants/$v/fused.hip\"")
  [ -f "$d/wide.hip" ] && defs+=("-DWIDE_SRC=\"variants/$v/wide.hip\"")
  $HIPCC $FL "${defs[@]}" window_probe.hip -o window_probe_$v &
done
if [ "${ALL:-0}" = "1" ]; then
  for p in fp64_probe cascade_probe mem_probe dma_probe; do $HIPCC $FL $p.hip -o $p & done
fi
wait
