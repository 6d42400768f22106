# The randomised parity sweep on the final round-5 tree: 20,000 cases with flat / silent spans
# planted at a third of the markers (the guard's second stage in every kernel family), then
# 20,000 plain cases on fresh seeds.
set -uo pipefail
OUT=gpurun_out/r05v
mkdir -p $OUT
timeout -k 10 500 python -u tools/parity_sweep.py --cases 20000 --seed0 100000 --flat --out $OUT/parity_sweep_flat_20000.json > $OUT/flat.log 2>&1 || { tail -20 $OUT/flat.log; exit 1; }
tail -1 $OUT/flat.log
timeout -k 10 500 python -u tools/parity_sweep.py --cases 20000 --seed0 200000 --out $OUT/parity_sweep_20000.json > $OUT/plain.log 2>&1 || { tail -20 $OUT/plain.log; exit 1; }
tail -1 $OUT/plain.log
