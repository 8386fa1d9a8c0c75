# Round validation on the GPU box: parity tests, default bench, rocprofv3 kernel stats.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r01}
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
timeout -k 10 300 python bench.py --layers-out gpurun_out/bench_layers_$TAG.json > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$TAG -o p -- python3 $R/bench.py --no-cpu-baseline --steps 20 > $R/gpurun_out/prof_$TAG.log 2>&1
