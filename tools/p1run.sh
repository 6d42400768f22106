set -e
cd $GRAFT_REPO_ROOT
VARIANTS="p1" WIDE_VARIANTS="" PMC=0 TAG=ab3 bash tools/probe_ab.sh
cd /tmp
for v in "" _p1; do
  for C in FETCH_SIZE WRITE_SIZE; do
    PROBE_ITERS=20 timeout -s KILL 60 rocprofv3 --pmc $C --kernel-include-regex window_ --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/ab3/pmc${v}_$C -o run -- $GRAFT_REPO_ROOT/tools/probes/window_probe$v > /dev/null 2>&1
    echo "$v $C"; python3 $GRAFT_REPO_ROOT/tools/pmc_summary.py $GRAFT_REPO_ROOT/gpurun_out/ab3/pmc${v}_$C
  done
done
