R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r02ac}
cd $R
mkdir -p gpurun_out
source tools/gpu_steps.sh
T=$R/gpurun_out/tune_$TAG.json
step b0_$TAG 300 python bench.py --tune-cache $T --no-cpu-baseline
step b1_$TAG 300 env TIC_LANE_PRIO=1 python bench.py --tune-cache $T --no-cpu-baseline
step b2_$TAG 300 python bench.py --tune-cache $T --no-cpu-baseline
step b3_$TAG 300 env TIC_LANE_PRIO=1 python bench.py --tune-cache $T --no-cpu-baseline
step b4_$TAG 300 env TIC_LANE_PRIO=1 python bench.py --tune-cache none --no-cpu-baseline
