R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r02d}
cd $R
mkdir -p gpurun_out
source tools/gpu_steps.sh
step chain_$TAG 300 python -u -m pytest tests/test_gpu_chain.py tests/test_gpu_parity.py tests/test_gpu_image.py -x -q --timeout 120 --timeout-method thread
step probe_$TAG 400 python tools/chain_probe.py
step bench_off_$TAG 300 env TIC_CHAIN=0 python bench.py --tune-cache none --no-cpu-baseline --layers-out gpurun_out/bench_layers_off_$TAG.json
step bench_on_$TAG 300 env TIC_CHAIN=1 python bench.py --tune-cache none --no-cpu-baseline --layers-out gpurun_out/bench_layers_on_$TAG.json
step bench3_$TAG 300 python bench.py --model 3 --batch 256 --tune-cache none --no-cpu-baseline --layers-out gpurun_out/bench_layers3_$TAG.json
