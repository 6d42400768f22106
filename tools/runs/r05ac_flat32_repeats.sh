# The 32 % flat-window case against no planted windows, interleaved, three repetitions (the
# box-to-box spread of single runs is about the size of the effect being judged).
set -uo pipefail
OUT=gpurun_out/r05ac
mkdir -p $OUT
B="--cpu-sample 0 --alt-steps 0 --steps 50 --warmup 20"
for rep in 1 2 3; do
  for spec in none flat:0.32; do
    if [ $spec = none ]; then PL=""; else PL="--plant $spec"; fi
    f=$OUT/${spec/:/_}_$rep
    timeout -k 10 300 python bench.py $B $PL > $f.json 2> $f.err || { tail -20 $f.err; exit 1; }
    python3 -c "
import json
d = json.load(open('$f.json'))
print('$spec rep$rep', 'step ms', d['ms_per_step'], 'window ms', d['roofline']['kernel_ms'])
"
  done
done
