#!/bin/bash
# Builds a study variant of libeegfx.so (compile-time macros of the product sources) for library
# A/Bs (bench.py --lib, tools/epochs_bench.py --lib):
#   tools/build_ab_lib.sh <out_dir> "-DEEGFX_RECHECK_ROWS=0"
set -euo pipefail
OUT=${1:?out dir}; DEFS=${2:-}
cd "$(dirname "$0")/.."
CSRC=eeg_dataanalysispackage_amd/csrc
B=$OUT/build; mkdir -p $B
F="-O3 -fPIC -std=c++17 -ffp-contract=off -Iinclude -I$CSRC -w --offload-arch=gfx950 $DEFS"
pids=()
for s in kernels fused wide guard logreg plan; do
  /opt/rocm/bin/hipcc $F -x hip -munsafe-fp-atomics -c $CSRC/$s.hip -o $B/$s.o & pids+=($!)
done
for s in api brainvision comm; do
  /opt/rocm/bin/hipcc $F -D__HIP_PLATFORM_AMD__ -c $CSRC/$s.cpp -o $B/$s.o & pids+=($!)
done
for p in "${pids[@]}"; do wait $p; done
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o $OUT/libeegfx.so $B/*.o \
  -L/opt/rocm/lib -lamdhip64 -lrccl -lpthread -Wl,-rpath,/opt/rocm/lib
rm -rf $B
