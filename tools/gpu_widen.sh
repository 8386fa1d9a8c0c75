# GPU check of the widened rows: all -m gpu tests, default bench, configs[2] and configs[4] benches.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-w}
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1
timeout -k 10 300 python bench.py --layers-out gpurun_out/bench_layers_$TAG.json > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
timeout -k 10 400 python bench.py --model 3 --batch 256 --steps 10 --warmup 3 --layers-out gpurun_out/bench_layers_m3_$TAG.json > gpurun_out/bench_m3_$TAG.json 2> gpurun_out/bench_m3_$TAG.err
timeout -k 10 400 python bench.py --workload image4k --steps 5 --warmup 2 > gpurun_out/bench_4k_$TAG.json 2> gpurun_out/bench_4k_$TAG.err
