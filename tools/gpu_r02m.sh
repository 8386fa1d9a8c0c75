R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r02m}
cd $R
mkdir -p gpurun_out
source tools/gpu_steps.sh
step bench_auto1_$TAG 300 env TIC_TUNE_LOG=1 python bench.py --tune-cache none --no-cpu-baseline
step bench_c1_$TAG 300 env TIC_CHAIN=1 python bench.py --tune-cache none --no-cpu-baseline
step bench_auto2_$TAG 300 env TIC_TUNE_LOG=1 python bench.py --tune-cache none --no-cpu-baseline
step bench_m3_$TAG 300 env TIC_TUNE_LOG=1 python bench.py --model 3 --tune-cache none --no-cpu-baseline
