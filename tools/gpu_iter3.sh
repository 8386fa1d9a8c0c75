# Round-3 iteration: chain bit-identity after the hand-off rework, one-lane launch timings,
# fresh step-tuned benches for model_0 (configs[1]) and model_3 (configs[2]), states saved.
#   bash tools/gpu_iter3.sh <tag>
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-it}
cd $R
mkdir -p gpurun_out/tune_$TAG
source tools/gpu_steps.sh
O=$R/gpurun_out
step chaintest_$TAG 600 python -u -m pytest tests/test_gpu_chain.py tests/test_gpu_parity.py -k "chain or fused" -v --timeout 300 --timeout-method thread
step probe_$TAG 400 python tools/layer_probe.py 0 32 opt:chain_wh=2 opt:chain_wh=2,opt:chain_order=1 opt:chain_wh=4
TIC_TUNE_LOG=1 step bench_$TAG 600 python bench.py --tune-cache none --tune-save $O/tune_$TAG --no-cpu-baseline
TIC_TUNE_LOG=1 step bench_m3_$TAG 900 python bench.py --model 3 --batch 256 --tune-cache none --tune-save $O/tune_$TAG --no-cpu-baseline
