set -euo pipefail
cd "${GRAFT_REPO_ROOT}"
ROOT=$(pwd)
export TMPDIR=/tmp
cd /tmp
for A in 0 1 6; do
  timeout -s KILL 60 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES --kernel-include-regex window_kernel --kernel-trace --output-format csv -d $ROOT/gpurun_out/clk$A -o run -- $ROOT/tools/probes/window_probe_$A > $ROOT/gpurun_out/clk$A.log 2>&1
  echo "== ablation $A"; python3 $ROOT/tools/pmc_summary.py $ROOT/gpurun_out/clk$A 2>/dev/null || true
  python3 - $ROOT/gpurun_out/clk$A <<'PY'
import csv,glob,sys,statistics
for f in glob.glob(sys.argv[1]+"/**/*kernel_trace.csv",recursive=True):
    d=[int(r["End_Timestamp"])-int(r["Start_Timestamp"]) for r in csv.DictReader(open(f)) if "window_kernel" in r["Kernel_Name"]]
    print("kernel ms median", statistics.median(d)/1e6)
PY
done
