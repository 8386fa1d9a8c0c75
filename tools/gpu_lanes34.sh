#!/bin/bash
# Lanes 3 and 4 with the chain kernel in the step tuner: tune + bench model_0 configs[1].
set -e
mkdir -p gpurun_out
for s in 3 4; do
  TIC_TUNE_LOG=1 timeout -k 10 400 python -u bench.py --no-cpu-baseline --streams $s \
    --tune-cache gpurun_out/tune_model0_s$s.json --layers-out gpurun_out/bench_layers_s$s.json \
    > gpurun_out/bench_s$s.json 2> gpurun_out/bench_s$s.err
done
