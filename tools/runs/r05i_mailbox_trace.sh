# The small-path GPU tests, then where the resident server's per-epoch time goes: the step-by-step probe, then EEGFX_MB_TRACE
# medians (host post -> answer; kernel poll exit -> windows staged -> filter bank ->
# normalisation -> rows written; the rest = the link both ways) over the drop-in bench's mailbox legs.
set -uo pipefail
OUT=gpurun_out/r05i
mkdir -p $OUT
# timeout -k 10 400 python -u -m pytest tests/test_gpu_mailbox.py tests/test_gpu_epochs_features.py tests/test_gpu_c_abi.py tests/test_gpu_guard.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
# tail -2 $OUT/pytest.log
timeout -k 10 90 ./tools/mailbox_probe . > $OUT/probe.log 2>&1; rc=$?; cat $OUT/probe.log; [ $rc -eq 0 ] || exit 1
EEGFX_MB_TRACE=1 timeout -k 10 120 ./tools/dropin_bench . 2000 1 > $OUT/dropin_fma.json 2> $OUT/dropin_fma.err || { tail -20 $OUT/dropin_fma.err; exit 1; }
cat $OUT/dropin_fma.json; grep EEGFX_MB_TRACE $OUT/dropin_fma.err | head -4
