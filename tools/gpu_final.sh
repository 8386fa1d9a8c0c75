# Round-end evidence: full GPU suite, the three bench configurations, rocprofv3 kernel
# stats of the default bench, PMC traffic (summarised on the box) for configs[1]/[2].
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r01}
cd $R
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1
bash tools/pmc_round.sh $TAG
timeout -k 10 300 python bench.py --layers-out gpurun_out/bench_layers_$TAG.json > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
timeout -k 10 300 python bench.py --model 3 --batch 256 --no-cpu-baseline --traffic profiles/traffic_${TAG}_model3.json --layers-out gpurun_out/bench_layers_${TAG}_model3.json > gpurun_out/bench_${TAG}_model3.json 2> gpurun_out/bench_${TAG}_model3.err
timeout -k 10 400 python bench.py --workload image4k > gpurun_out/bench_${TAG}_image4k.json 2> gpurun_out/bench_${TAG}_image4k.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$TAG -o p -- python3 $R/bench.py --no-cpu-baseline --steps 20 > $R/gpurun_out/prof_$TAG.log 2>&1
rm -f $R/gpurun_out/prof_$TAG/p_kernel_trace.csv
