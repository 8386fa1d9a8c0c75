R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r02p}
cd $R
mkdir -p gpurun_out
source tools/gpu_steps.sh
T=gpurun_out/tune_$TAG.json
step b20a_$TAG 300 python bench.py --tune-cache $T --no-cpu-baseline
step b20b_$TAG 300 python bench.py --tune-cache $T --no-cpu-baseline
step b200_$TAG 300 python bench.py --tune-cache $T --no-cpu-baseline --steps 200 --warmup 20
step b200g_$TAG 300 python bench.py --tune-cache $T --no-cpu-baseline --steps 200 --warmup 20 --graph
step b1000_$TAG 300 python bench.py --tune-cache $T --no-cpu-baseline --steps 1000 --warmup 20
