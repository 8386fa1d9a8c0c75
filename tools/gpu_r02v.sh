R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r02v}
cd $R
mkdir -p gpurun_out
source tools/gpu_steps.sh
step par_$TAG 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_image.py
step probe_$TAG 400 python tools/dec10_probe.py
step bench_$TAG 300 env TIC_TUNE_LOG=1 python bench.py --tune-cache none --no-cpu-baseline
