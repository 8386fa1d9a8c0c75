# quick bench probes: bash tools/gpu_confirm.sh <tag> [bench args...]
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1
shift
cd $R
mkdir -p gpurun_out
source tools/gpu_steps.sh
step q_$TAG 400 python bench.py --no-cpu-baseline "$@"
