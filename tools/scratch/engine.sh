set -euo pipefail
cd "${GRAFT_REPO_ROOT}"
echo "== parity (engine default)"
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread 2>&1 | tail -4
cd tools/probes
for G in 3 2 4; do echo "G=$G"; EEGFX_ENGINE_G=$G timeout -k 5 60 ./window_probe_0; EEGFX_ENGINE_G=$G timeout -k 5 60 ./window_probe_1; done
echo "old"; EEGFX_ENGINE=0 timeout -k 5 60 ./window_probe_0
