# configs[4] streamed path: the chunk ramp of HEAD (c/4 ...) against the library in the tree,
# interleaved, three repetitions (bench.py --workload stream with the library path swapped).
mkdir -p gpurun_out/r04s
for rep in 1 2 3; do
  for lib in tools/probes/libeegfx_head.so eeg_dataanalysispackage_amd/libeegfx.so; do
    echo -n "$lib " >> gpurun_out/r04s/ab.log
    timeout -k 10 180 python -u -c "
import sys, runpy
import eeg_dataanalysispackage_amd._lib as L
L.LIB_PATH = '$lib'
sys.argv = ['bench.py', '--workload', 'stream', '--steps', '30', '--warmup', '5']
runpy.run_path('bench.py', run_name='__main__')
" >> gpurun_out/r04s/ab.log 2>/dev/null || exit 1
  done
done
cat gpurun_out/r04s/ab.log
