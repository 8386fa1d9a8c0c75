# the whole GPU suite against the shipped tuning:   bash tools/gpu_suite.sh <tag>
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-s}
cd $R
source tools/gpu_steps.sh
step gputest_$TAG 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread
tail -3 gpurun_out/gputest_$TAG.log
