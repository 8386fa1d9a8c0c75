#!/bin/bash
# Two-lane steady state after fresh forks: per-round step times (is it bimodal?) with the
# chain off / on (512- and 256-thread workgroups) and one lane with the chain.
set -e
mkdir -p gpurun_out
T=tf_image_compression_amd/tune/model0_p256_b64_s2.json
timeout -k 10 400 python -u tools/ab.py --model 0 --batch 64 --rounds 12 --steps 40 --tune-file $T --refork \
  --cfg streams=2,chain=0 \
  --cfg streams=2,chain=1,chain_wh=2 \
  --cfg streams=2,chain=1,chain_wh=1 \
  --cfg streams=1,chain=1,chain_wh=1 \
  > gpurun_out/probe_modes.json 2> gpurun_out/probe_modes.err
