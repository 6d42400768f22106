# The power-capped VALU ceiling of the final kernels: product window_probe only,
# power study for c3 and c32 with the SQ passes, the baseline pass alone, then the summary.
set -euo pipefail
cd "${GRAFT_REPO_ROOT}"
(cd tools/probes && ABL=none timeout -k 10 300 bash build_probes.sh)
TAG=r04zg/power PROBES=window_probe WLS="c3 c32" timeout -k 10 400 bash tools/power_study.sh
TAG=r04zg/power timeout -k 10 120 bash tools/baseline_power.sh
python3 tools/ceiling_summary.py gpurun_out/r04zg/power gpurun_out/r04zg/r04_ceiling.json
cat gpurun_out/r04zg/r04_ceiling.json
