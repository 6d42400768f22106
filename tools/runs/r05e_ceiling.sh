# Round-5 power-capped ceiling of the final kernels and the per-step energy budget:
# the product window_probe, power study for c3 and c32 with the SQ passes, the baseline pass
# alone, the step (baseline + window) back to back, then the summary -> r05_ceiling.json.
set -euo pipefail
cd "${GRAFT_REPO_ROOT}"
(cd tools/probes && ABL=none timeout -k 10 300 bash build_probes.sh)
TAG=r05e/power PROBES=window_probe WLS="c3 c32" timeout -k 10 400 bash tools/power_study.sh
TAG=r05e/power timeout -k 10 120 bash tools/baseline_power.sh
OUT=gpurun_out/r05e/power
PROBE_STEP=1 PROBE_ITERS=6000 timeout -k 10 60 tools/probes/window_probe > $OUT/step.txt 2>&1 &
pid=$!
sleep 3.0
timeout 20 amd-smi metric -p -c -g 0 > $OUT/step_smi.txt 2>&1
wait $pid
echo "step: $(tail -1 $OUT/step.txt | cut -c1-70) | $(grep -E 'SOCKET_POWER' $OUT/step_smi.txt | head -1 | xargs)"
python3 tools/ceiling_summary.py $OUT gpurun_out/r05e/r05_ceiling.json
