# Round-2 pass b: GPU suite, default bench (tuning saved), PMC passes replaying that
# tuning, rocprofv3 kernel stats of the bench replaying it too.
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r02b}
cd $R
mkdir -p gpurun_out
source tools/gpu_steps.sh
step pytest_gpu_$TAG 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread
step bench_$TAG 300 python bench.py --tune-cache gpurun_out/tune_m0_$TAG.json --layers-out gpurun_out/bench_layers_$TAG.json
step pmc_$TAG 1000 bash tools/pmc_box.sh m0_$TAG $R/gpurun_out/tune_m0_$TAG.json
cd /tmp && export TMPDIR=/tmp
step prof_$TAG 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$TAG -o p -- python3 $R/bench.py --no-cpu-baseline --steps 20 --tune-cache $R/gpurun_out/tune_m0_$TAG.json
rm -f $R/gpurun_out/prof_$TAG/p_kernel_trace.csv
