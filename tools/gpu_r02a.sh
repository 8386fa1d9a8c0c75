# Round-2 first GPU pass: full -m gpu suite (incl. the configs[2]/[3]/[4], RCCL and plugin
# tests), the default bench, PMC passes of the default bench, rocprofv3 kernel stats.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r02a}
cd $R
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1
timeout -k 10 300 python bench.py --layers-out gpurun_out/bench_layers_$TAG.json > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
bash tools/pmc_box.sh m0_$TAG
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$TAG -o p -- python3 $R/bench.py --no-cpu-baseline --steps 20 > $R/gpurun_out/prof_$TAG.log 2>&1
rm -f $R/gpurun_out/prof_$TAG/p_kernel_trace.csv
