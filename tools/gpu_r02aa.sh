R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r02aa}
cd $R
mkdir -p gpurun_out
source tools/gpu_steps.sh
step ch128_$TAG 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_configs.py -k "ch128" tests/test_abi.py
bash tools/gpu_r02z.sh $TAG
