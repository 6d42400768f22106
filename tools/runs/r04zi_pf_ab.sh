# window_kernel with an L2 prefetch of the sub-tile D workgroups ahead (EEGFX_PREFETCH_TILES = D)
# against HEAD: bench.py c3, interleaved, three repetitions.
mkdir -p gpurun_out/r04zi
for rep in 1 2 3; do
  for lib in head pf48 pf96 pf192; do
    echo -n "$lib " >> gpurun_out/r04zi/ab.log
    timeout -k 10 180 python -u -c "
import sys, runpy
import eeg_dataanalysispackage_amd._lib as L
L.LIB_PATH = 'tools/probes/libeegfx_$lib.so'
sys.argv = ['bench.py', '--steps', '200', '--warmup', '20', '--alt-steps', '0', '--cpu-sample', '0']
runpy.run_path('bench.py', run_name='__main__')
" >> gpurun_out/r04zi/ab.log 2>/dev/null || exit 1
  done
done
python3 - <<'PY'
import json
for l in open("gpurun_out/r04zi/ab.log"):
    lib, _, js = l.partition(" ")
    d = json.loads(js)
    print(lib, d["value"], d["ms_per_step"], d["roofline"]["kernel_ms"], d["roofline"]["frac"])
PY
