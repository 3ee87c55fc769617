#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4g
mkdir -p $O
cd $R
timeout -k 10 300 python tools/png_device_bench.py > $O/png_bench.json 2> $O/png_bench.err || { tail -20 $O/png_bench.err; exit 1; }
cat $O/png_bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o trace --output-format csv -- python $R/tools/png_device_bench.py > $O/png_bench_trace.json 2> $O/trace.err || { tail -20 $O/trace.err; exit 2; }
cat $O/trace/trace_kernel_stats.csv | head -20
