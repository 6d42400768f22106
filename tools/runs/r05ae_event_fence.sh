# bench.py with the window-kernel timing events created without the system-scope fence (the tree)
# against the same library with default events (tools/probes/r05/baselib), interleaved, three
# repetitions each.
set -uo pipefail
OUT=gpurun_out/r05ae
mkdir -p $OUT
B="--cpu-sample 0 --alt-steps 0 --steps 100 --warmup 20"
for rep in 1 2 3; do
  for v in base tree; do
    if [ $v = base ]; then L="--lib tools/probes/r05/baselib/libeegfx.so"; else L=""; fi
    f=$OUT/${v}_$rep
    timeout -k 10 300 python bench.py $B $L > $f.json 2> $f.err || { tail -20 $f.err; exit 1; }
    python3 -c "
import json
d = json.load(open('$f.json'))
r = d['roofline']
print('$v rep$rep', 'step ms', d['ms_per_step'], 'window ms', r['kernel_ms'], 'value', d['value'])
"
  done
done
