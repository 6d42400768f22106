#!/bin/bash
# configs[4] streamed ingest: bench line, then a kernel + memory-copy trace of a few steps
# (where the host link sits idle: the unoverlapped first upload, the last chunk's kernels and row
# download, gaps between chunks).
set -uo pipefail
OUT=gpurun_out/${TAG:-r06d}; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 python bench.py --workload stream --steps 10 --warmup 3 --cpu-sample 0 ${ARGS:-} > $OUT/bench_stream.json 2> $OUT/bench_stream.err || { tail -20 $OUT/bench_stream.err; exit 1; }
cat $OUT/bench_stream.json
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $OUT/trace -o stream -- python bench.py --workload stream --steps 3 --warmup 1 --cpu-sample 0 ${ARGS:-} > $OUT/trace.log 2>&1 || { tail -20 $OUT/trace.log; exit 1; }
find $OUT/trace -name "*.csv" | head
