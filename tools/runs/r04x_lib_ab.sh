# bench.py (c3 headline workload, and c32 with WL=c32) with the HEAD library against the tree's,
# interleaved, REPS repetitions: window kernel (HIP events) and whole step.
mkdir -p gpurun_out/${TAG:-r04x}
for rep in $(seq 1 ${REPS:-3}); do
  for lib in tools/probes/libeegfx_head.so eeg_dataanalysispackage_amd/libeegfx.so; do
    echo -n "$lib " >> gpurun_out/${TAG:-r04x}/ab.log
    timeout -k 10 180 python -u -c "
import sys, runpy
import eeg_dataanalysispackage_amd._lib as L
L.LIB_PATH = '$lib'
sys.argv = ['bench.py', '--workload', '${WL:-c3}', '--steps', '${STEPS:-200}', '--warmup', '20', '--alt-steps', '0', '--cpu-sample', '0'] + '${ARGS:-}'.split()
runpy.run_path('bench.py', run_name='__main__')
" >> gpurun_out/${TAG:-r04x}/ab.log 2>/dev/null || exit 1
  done
done
python3 - <<'PY'
import json, os
tag = os.environ.get("TAG", "r04x")
for l in open(f"gpurun_out/{tag}/ab.log"):
    lib, _, js = l.partition(" ")
    d = json.loads(js)
    print(lib.split("/")[-1], d["value"], d["ms_per_step"], d["roofline"]["kernel_ms"], d["roofline"]["frac"])
PY
