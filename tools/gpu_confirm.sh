# quick checks: bash tools/gpu_confirm.sh <tag> [bench args...]  (parity subset + bench)
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1
shift
cd $R
mkdir -p gpurun_out
source tools/gpu_steps.sh
step par_$TAG 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_chain.py
step q_$TAG 400 python bench.py --no-cpu-baseline --tune-cache none "$@"
step q3_$TAG 400 python bench.py --no-cpu-baseline --tune-cache none --model 3 --batch 256 "$@"
