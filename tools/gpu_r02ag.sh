R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r02ag}
cd $R
mkdir -p gpurun_out
source tools/gpu_steps.sh
step par_$TAG 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "fused_tail"
step probe_$TAG 400 python tools/dec10_probe.py
