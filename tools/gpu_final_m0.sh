#!/bin/bash
# The default bench line (committed tuning replayed) and rocprofv3 kernel stats of the same
# command without the CPU baseline: bash tools/gpu_final_m0.sh <tag>
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-final}
cd $R
mkdir -p gpurun_out
source tools/gpu_steps.sh
O=$R/gpurun_out
step bench_default_$TAG 400 python bench.py
step stats_default_$TAG 300 bash -c "cd /tmp && export TMPDIR=/tmp && rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_default_$TAG -o p -- python3 $R/bench.py --no-cpu-baseline"
rm -f $O/prof_default_$TAG/p_kernel_trace.csv
