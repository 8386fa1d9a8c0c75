R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r02h}
cd $R
mkdir -p gpurun_out
source tools/gpu_steps.sh
step bench_$TAG 300 env TIC_FUSE_TAIL=1 python bench.py --tune-cache gpurun_out/tune_$TAG.json --no-cpu-baseline --layers-out gpurun_out/bench_layers_$TAG.json
step kc_$TAG 900 env TIC_FUSE_TAIL=1 bash tools/kcounters.sh $TAG $R/gpurun_out/tune_$TAG.json
