R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r02y}
cd $R
mkdir -p gpurun_out
source tools/gpu_steps.sh
O=$R/gpurun_out
step bench_$TAG 400 python bench.py
step stats_m0_$TAG 300 bash -c "cd /tmp && export TMPDIR=/tmp && rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_m0_$TAG -o p -- python3 $R/bench.py --no-cpu-baseline --steps 50 --warmup 5"
step bench3_$TAG 400 python bench.py --model 3 --batch 256 --no-cpu-baseline
