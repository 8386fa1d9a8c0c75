R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r02i}
cd $R
mkdir -p gpurun_out
source tools/gpu_steps.sh
step img_$TAG 400 python bench.py --workload image4k --no-cpu-baseline
step bench3_$TAG 300 python bench.py --model 3 --batch 256 --tune-cache gpurun_out/tune3_$TAG.json --no-cpu-baseline --layers-out gpurun_out/bench_layers3_$TAG.json
step kc3_$TAG 900 bash tools/kcounters.sh m3_$TAG $R/gpurun_out/tune3_$TAG.json --model 3 --batch 256
