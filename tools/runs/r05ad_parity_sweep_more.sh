# 30,000 more randomised parity cases on the final tree, with planted flat / silent spans.
set -uo pipefail
OUT=gpurun_out/r05ad
mkdir -p $OUT
timeout -k 10 900 python -u tools/parity_sweep.py --cases 30000 --seed0 300000 --flat --out $OUT/parity_sweep_flat_30000.json > $OUT/flat.log 2>&1 || { tail -20 $OUT/flat.log; exit 1; }
tail -1 $OUT/flat.log | cut -c1-300
