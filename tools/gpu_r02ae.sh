R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r02ae}
cd $R
mkdir -p gpurun_out
source tools/gpu_steps.sh
step par_$TAG 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "winograd or chain"
step b_$TAG 300 env TIC_TUNE_LOG=1 python bench.py --tune-cache none --no-cpu-baseline
step b1_$TAG 300 env TIC_TUNE_LOG=1 python bench.py --streams 1 --tune-cache none --no-cpu-baseline
