R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r02af}
cd $R
mkdir -p gpurun_out
source tools/gpu_steps.sh
step probe_$TAG 400 python tools/dec10_probe.py
