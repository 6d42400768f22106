#!/bin/bash
# Where does the driver's bench number (--steps 20 --warmup 5) differ from the builder's
# (--steps 100 --warmup 50)?  Runs both commands back to back on one box, alternating, each in a
# fresh process with the per-step device trace (bench.py --trace-steps), while amd-smi samples
# socket power and shader clock in the background.
#   TAG=r04a bash tools/driver_gap.sh
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/${TAG:-gap}
mkdir -p "$OUT"
export TMPDIR=/tmp
( for i in $(seq 1 400); do
    echo "t=$(date +%s.%N)"
    timeout 10 amd-smi metric -p -c -g 0 2>&1 | grep -E "SOCKET_POWER|GFX_0|CLK:" | head -4
    sleep 0.1
  done ) > "$OUT/smi_samples.txt" 2>&1 &
SMI=$!
run() {  # name, bench args
  local name=$1; shift
  echo "t=$(date +%s.%N) start $name" >> "$OUT/marks.txt"
  timeout -k 10 240 python bench.py --cpu-sample 0 --alt-steps 0 --trace-steps "$@" \
    > "$OUT/$name.json" 2> "$OUT/$name.err" || { echo "$name failed"; tail -20 "$OUT/$name.err"; kill $SMI; exit 1; }
  echo "t=$(date +%s.%N) end $name" >> "$OUT/marks.txt"
  python3 - "$OUT/$name.json" <<'EOF'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
t = d["step_trace"]
w, s = t["warmup"], t["timed"]
print("%-14s value %.4g  ms/step(wall) %.4f  kernel %.4f  warmup[0:5] %s  timed first5 %s  timed mean %.4f  last5 %s" % (
    sys.argv[1].split("/")[-1], d["value"], d["ms_per_step"], d["roofline"]["kernel_ms"],
    w[:5], s[:5], sum(s) / len(s), s[-5:]))
EOF
}
run driverA1 --steps 20 --warmup 5
run builderB1 --steps 100 --warmup 50
run driverA2 --steps 20 --warmup 5
run builderB2 --steps 100 --warmup 50
run driverA3 --steps 20 --warmup 5
run long_warm --steps 100 --warmup 400
kill $SMI 2>/dev/null
wait 2>/dev/null
exit 0
