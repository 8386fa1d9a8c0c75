#!/bin/bash
# Chain kernel iteration on the GPU box: bit-identity tests, phase timing in the two-lane
# step, then the bench tuned in the run (state saved to gpurun_out/ for tf_image_compression_amd/tune/).
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_chain.py -x -q --timeout 120 --timeout-method thread > gpurun_out/chain_tests.log 2>&1
timeout -k 10 120 python -u tools/chain_timing.py --tune-file tf_image_compression_amd/tune/model0_p256_b64_s2.json > gpurun_out/chain_timing.jsonl 2> gpurun_out/chain_timing.err
TIC_TUNE_LOG=1 timeout -k 10 400 python -u bench.py --no-cpu-baseline --streams 2 \
  --tune-cache gpurun_out/tune_model0_s2.json --layers-out gpurun_out/bench_layers_s2.json \
  > gpurun_out/bench_s2.json 2> gpurun_out/bench_s2.err
