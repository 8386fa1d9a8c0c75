R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r02e}
cd $R
mkdir -p gpurun_out
source tools/gpu_steps.sh
step par_$TAG 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_image.py -x -q --timeout 120 --timeout-method thread
step d10probe_$TAG 400 python tools/dec10_probe.py
step bench_$TAG 300 python bench.py --tune-cache none --no-cpu-baseline --layers-out gpurun_out/bench_layers_$TAG.json
