R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r02j}
cd $R
mkdir -p gpurun_out
source tools/gpu_steps.sh
step bench_$TAG 300 python bench.py --tune-cache gpurun_out/tune_$TAG.json --no-cpu-baseline
cd /tmp && export TMPDIR=/tmp
step trace_$TAG 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/trace_$TAG -o p -- python3 $R/bench.py --no-cpu-baseline --steps 10 --warmup 3 --trace-only --tune-cache $R/gpurun_out/tune_$TAG.json
cd $R
N=$(grep -h launches_per_lane gpurun_out/trace_$TAG.log | python3 -c "import sys,json; print(2*json.loads(sys.stdin.read().strip().splitlines()[-1])['launches_per_lane'])")
python3 tools/step_trace.py $(find gpurun_out/trace_$TAG -name "*kernel_trace.csv" | head -1) $N 8 > gpurun_out/timeline_$TAG.txt 2>&1
find gpurun_out/trace_$TAG -name "*kernel_trace.csv" -delete
