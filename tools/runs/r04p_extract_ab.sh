mkdir -p gpurun_out/r04p
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_epochs_kernels.py tests/test_gpu_guard.py > gpurun_out/r04p/pytest.log 2>&1 || { tail -30 gpurun_out/r04p/pytest.log; exit 1; }
tail -3 gpurun_out/r04p/pytest.log
for C in 32 8 3; do
  n=$((3200000 / C))
  for lib in tools/probes/libeegfx_head.so eeg_dataanalysispackage_amd/libeegfx.so tools/probes/libeegfx_head.so eeg_dataanalysispackage_amd/libeegfx.so; do
    timeout -k 10 120 python -u tools/epochs_bench.py --lib $lib --epochs $n --channels $C --steps 20 --warmup 5 --tag $(basename $lib) >> gpurun_out/r04p/ab.log 2>&1 || exit 1
  done
done
cat gpurun_out/r04p/ab.log
