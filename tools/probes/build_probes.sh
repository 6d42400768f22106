#!/bin/bash
# Builds the perf probes in-tree (here, or on the GPU box, which has the same toolchain):
#   window_probe          the product window / wide kernels under sustained load
#   window_probe_<a>      the same against the product sources with tools/probes/ablations/<a>.patch
#                         applied (A/B and ablation studies; a patch may touch fused.hip, wide.hip
#                         and dwt8.h, and is applied to copies under tools/probes/build/<a>/)
#   fp64_probe, cascade_probe, mem_probe, dma_probe   micro-benchmarks (ALL=1)
#   ABL="a b" limits the ablations built; DEFS="-DX=1" is passed to every build.
set -euo pipefail
cd "$(dirname "$0")"
HIPCC=${HIPCC:-/opt/rocm/bin/hipcc}
CSRC=../../eeg_dataanalysispackage_amd/csrc
FL="-O3 -std=c++17 -ffp-contract=off --offload-arch=gfx950 -w -I../../include -I$CSRC ${DEFS:-}"
pids=()
$HIPCC $FL window_probe.hip -o window_probe & pids+=($!)
for p in ablations/*.patch; do
  [ -f "$p" ] || continue
  a=$(basename "$p" .patch)
  if [ -n "${ABL:-}" ] && [[ " $ABL " != *" $a "* ]]; then continue; fi
  d=build/$a
  rm -rf "$d" && mkdir -p "$d"
  cp $CSRC/fused.hip $CSRC/wide.hip $CSRC/dwt8.h "$d/"
  patch -s -d "$d" -p1 < "$p"
  # the copies include each other by quoted name, so the patched dwt8.h shadows the product's
  $HIPCC $FL -I"$d" -DFUSED_SRC="\"$d/fused.hip\"" -DWIDE_SRC="\"$d/wide.hip\"" window_probe.hip \
    -o window_probe_$a & pids+=($!)
done
if [ "${ALL:-0}" = "1" ]; then
  for p in fp64_probe cascade_probe mem_probe dma_probe; do $HIPCC $FL $p.hip -o $p & pids+=($!); done
fi
fail=0
for pid in "${pids[@]}"; do wait "$pid" || fail=1; done
exit $fail
