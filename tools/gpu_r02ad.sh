R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r02ad}
cd $R
mkdir -p gpurun_out
source tools/gpu_steps.sh
step s1_$TAG 300 env TIC_TUNE_LOG=1 python bench.py --streams 1 --tune-cache none --no-cpu-baseline
step s1c_$TAG 300 env TIC_CHAIN=1 python bench.py --streams 1 --tune-cache none --no-cpu-baseline
step s2_$TAG 300 python bench.py --tune-cache none --no-cpu-baseline
