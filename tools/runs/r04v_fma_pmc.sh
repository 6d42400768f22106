# SQ counters of the fma window kernel (instruction mix, waits) -- one pass per counter group
set -e
mkdir -p gpurun_out/r04v
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA" \
           "SQ_WAVES SQ_INSTS_VALU_CVT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES"; do
  tag=$(echo $grp | md5sum | cut -c1-6)
  timeout -s KILL 90 rocprofv3 --pmc $grp --kernel-include-regex window_kernel --output-format csv -d $R/gpurun_out/r04v/pmc_$tag -o run -- python3 $R/bench.py --numerics fma --steps 5 --warmup 1 --settle-ms 0 --alt-steps 0 --cpu-sample 0 > $R/gpurun_out/r04v/pmc_$tag.log 2>&1
done
python3 - <<'PY'
import csv, glob, collections, os
R = os.environ["GRAFT_REPO_ROOT"]
tot = collections.defaultdict(list)
for f in glob.glob(R + "/gpurun_out/r04v/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        tot[r["Counter_Name"]].append(float(r["Counter_Value"]))
import statistics
for k, v in sorted(tot.items()):
    print(k, statistics.median(v), len(v))
PY
