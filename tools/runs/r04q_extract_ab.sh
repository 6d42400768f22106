# features_from_epochs_kernel: rows in LDS vs through `out` (both with non-temporal epoch loads)
# against the HEAD library, interleaved, two repetitions per channel count.
mkdir -p gpurun_out/r04q
for C in 32 24 16 12; do
  n=$((3200000 / C))
  for rep in 1 2; do
    for lib in head ldsrows rowsout; do
      timeout -k 10 120 python -u tools/epochs_bench.py --lib tools/probes/libeegfx_$lib.so --epochs $n --channels $C --steps 20 --warmup 5 --tag $lib >> gpurun_out/r04q/ab.log 2>&1 || exit 1
    done
  done
done
