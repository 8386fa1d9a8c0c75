# Round-3 iteration: XCD-aware Winograd tile order — parity, model_3 configs[2] fresh-tuned
# bench (state saved) and its PMC traffic passes replaying that state.
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-it}
cd $R
mkdir -p gpurun_out/tune_$TAG
source tools/gpu_steps.sh
O=$R/gpurun_out
step wtest_$TAG 600 python -u -m pytest tests/test_gpu_parity.py -k "winograd or s1_forms or model3 or small_patches" -v --timeout 300 --timeout-method thread
TIC_TUNE_LOG=1 step bench_m3_$TAG 900 python bench.py --model 3 --batch 256 --tune-cache none --tune-save $O/tune_$TAG --no-cpu-baseline
step pmc_m3_$TAG 900 bash tools/pmc_box.sh m3_$TAG $O/tune_$TAG/model3_p256_b256_s2.json --model 3 --batch 256
