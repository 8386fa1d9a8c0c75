# Round-3 iteration: chain bit-identity, one-lane launch timings, a fresh step-tuned bench
# (state saved), then the investigative SQ counter passes (LDS conflicts, instruction mix)
# replaying that state.   bash tools/gpu_iter2.sh <tag>
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-it}
cd $R
mkdir -p gpurun_out/tune_$TAG
source tools/gpu_steps.sh
O=$R/gpurun_out
step chaintest_$TAG 600 python -u -m pytest tests/test_gpu_chain.py tests/test_gpu_parity.py -k "chain or fused" -v --timeout 300 --timeout-method thread
step probe_$TAG 400 python tools/layer_probe.py 0 32 opt:chain_wh=2 opt:chain_wh=4
TIC_TUNE_LOG=1 step bench_$TAG 600 python bench.py --tune-cache none --tune-save $O/tune_$TAG --no-cpu-baseline
step kc_$TAG 900 bash tools/kcounters.sh $TAG $O/tune_$TAG/model0_p256_b64_s2.json
