R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r02w}
cd $R
mkdir -p gpurun_out
source tools/gpu_steps.sh
step bench_$TAG 300 python bench.py --tune-cache gpurun_out/tune_$TAG.json --no-cpu-baseline
export TIC_DEC10_VARIANT=16
step kc_$TAG 600 bash tools/kcounters.sh $TAG gpurun_out/tune_$TAG.json
