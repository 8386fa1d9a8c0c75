#!/bin/bash
# Tune + bench model_0 (configs[1]) at 2 lanes with the step tuner's log (the tuned state
# lands in gpurun_out/ for tf_image_compression_amd/tune/), then an alternating A/B replaying that state with
# the chain off / on.
set -e
mkdir -p gpurun_out
TIC_TUNE_LOG=1 timeout -k 10 400 python -u bench.py --no-cpu-baseline --streams 2 \
  --tune-cache gpurun_out/tune_model0_s2.json --layers-out gpurun_out/bench_layers_s2.json \
  > gpurun_out/bench_s2.json 2> gpurun_out/bench_s2.err
timeout -k 10 400 python -u tools/ab.py --model 0 --batch 64 --rounds 9 --steps 40 \
  --tune-file gpurun_out/tune_model0_s2.json --refork \
  --cfg streams=2,chain=0 --cfg streams=2,chain=1,chain_wh=2 --cfg streams=2,chain=1,chain_wh=1 \
  > gpurun_out/ab_chain.json 2> gpurun_out/ab_chain.err
