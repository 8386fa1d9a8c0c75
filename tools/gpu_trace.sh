# kernel trace of a short bench run: bash tools/gpu_trace.sh <tag> [bench args...]
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1
shift
cd $R
mkdir -p gpurun_out
source tools/gpu_steps.sh
O=$R/gpurun_out
step tr_$TAG 300 bash -c "cd /tmp && export TMPDIR=/tmp && rocprofv3 --kernel-trace --output-format csv -d $O/tr_$TAG -o p -- python3 $R/bench.py --no-cpu-baseline --steps 30 --warmup 5 $*"
