# Host staging of the per-epoch path with plain memcpy (tools/probes/r05/baselib: the library
# before the change) against non-temporal stores (the tree), interleaved, two repetitions each.
set -uo pipefail
OUT=gpurun_out/r05p
mkdir -p $OUT
for rep in 1 2; do
  LD_LIBRARY_PATH=$PWD/tools/probes/r05/baselib timeout -k 10 120 ./tools/dropin_bench . 2000 1 > $OUT/base_$rep.json 2> $OUT/base_$rep.err || { tail -5 $OUT/base_$rep.err; exit 1; }
  timeout -k 10 120 ./tools/dropin_bench . 2000 1 > $OUT/nt_$rep.json 2> $OUT/nt_$rep.err || { tail -5 $OUT/nt_$rep.err; exit 1; }
done
python3 - <<'PY'
import json, re
for v in ("base", "nt"):
    for rep in (1, 2):
        t = open(f"gpurun_out/r05p/{v}_{rep}.json").read()
        d = json.loads(t)
        print(v, rep, "launch", d["single_epoch"]["median_us"], d["single_epoch"]["p99_us"],
              "mailbox", d["mailbox"]["single_epoch"]["median_us"], d["mailbox"]["single_epoch"]["p99_us"],
              "batch11", d["batch_11"]["median_us"], d["mailbox"]["batch_11"]["median_us"])
PY
