# configs[4] streamed path: chunk size sweep (bench.py --workload stream --chunk-frames), two repetitions
mkdir -p gpurun_out/r04t
for rep in 1 2; do
  for cf in 4194304 8388608 16777216 33554432; do
    echo -n "$cf " >> gpurun_out/r04t/sweep.log
    timeout -k 10 180 python -u bench.py --workload stream --steps 30 --warmup 5 --chunk-frames $cf >> gpurun_out/r04t/sweep.log 2>/dev/null || exit 1
  done
done
