# Round-2 pass c: the chain kernel's tests first (bit identity, oversubscribed grid), then
# the whole suite, then bench A/B with the chain forced off / on.
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r02c}
cd $R
mkdir -p gpurun_out
source tools/gpu_steps.sh
step chain_$TAG 300 python -u -m pytest tests/test_gpu_chain.py -x -v --timeout 120 --timeout-method thread
step pytest_gpu_$TAG 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread
step bench_off_$TAG 300 env TIC_CHAIN=0 python bench.py --tune-cache none --no-cpu-baseline --layers-out gpurun_out/bench_layers_off_$TAG.json
step bench_on_$TAG 300 env TIC_CHAIN=1 python bench.py --tune-cache none --no-cpu-baseline --layers-out gpurun_out/bench_layers_on_$TAG.json
step bench_auto_$TAG 300 python bench.py --tune-cache gpurun_out/tune_m0_$TAG.json --no-cpu-baseline --layers-out gpurun_out/bench_layers_$TAG.json
step bench3_$TAG 300 python bench.py --model 3 --batch 256 --tune-cache none --no-cpu-baseline --layers-out gpurun_out/bench_layers3_$TAG.json
