#!/bin/bash
# model_3 configs[2] at 1, 2, 3 and 4 lanes, each tuned in the run (F(4x4,3x3) form)
mkdir -p gpurun_out
for s in 1 3 4 2; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --model 3 --batch 256 --streams $s --steps 60 --warmup 10 \
    --tune-cache none > gpurun_out/lanes_m3_s$s.json 2> gpurun_out/lanes_m3_s$s.err || exit 1
done
