# Quick: configs[1] and configs[2] bench lines only.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-quick}
cd $R
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --no-cpu-baseline --layers-out gpurun_out/bench_layers_$TAG.json > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
timeout -k 10 300 python bench.py --model 3 --batch 256 --no-cpu-baseline --layers-out gpurun_out/bench_layers_${TAG}_model3.json > gpurun_out/bench_${TAG}_model3.json 2> gpurun_out/bench_${TAG}_model3.err
