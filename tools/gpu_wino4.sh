#!/bin/bash
# Winograd F(4x4,3x3) (s1_form 2, model_3's default): parity tests, model_3 configs[2] tuned in
# the run (state saved to gpurun_out/), then SQ counters replaying that state.
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -v --timeout 200 \
  --timeout-method thread -k "winograd4 or s1_form or model3" > gpurun_out/wino4_tests.log 2>&1 || exit 1
TIC_TUNE_LOG=1 timeout -k 10 500 python -u bench.py --no-cpu-baseline --model 3 --batch 256 \
  --steps 30 --warmup 5 --tune-cache gpurun_out/tune_model3_b256_f2.json \
  --layers-out gpurun_out/bench_layers_m3_f2.json > gpurun_out/bench_m3_f2.json 2> gpurun_out/bench_m3_f2.err || exit 1
timeout -k 10 900 bash tools/kcounters.sh m3f2 gpurun_out/tune_model3_b256_f2.json --model 3 --batch 256; rc=$?
rm -rf gpurun_out/kc_m3f2/pmc_a gpurun_out/kc_m3f2/pmc_b gpurun_out/kc_m3f2/pmc_c
exit $rc
