#!/bin/bash
# debugging: model_3 bench with the runtime's default stride-1 form (no env), normal and --pmc-plan
mkdir -p gpurun_out
TIC_TUNE_LOG=1 timeout -k 10 400 python -u bench.py --no-cpu-baseline --model 3 --batch 256 --steps 10 --warmup 2 \
  --tune-cache gpurun_out/tune_m3_dbg.json > gpurun_out/dbg_bench.json 2> gpurun_out/dbg_bench.err; echo "bench rc=$?"
TIC_TUNE_LOG=1 timeout -k 10 400 python -u bench.py --no-cpu-baseline --model 3 --batch 256 --steps 3 --warmup 1 \
  --tune-cache gpurun_out/tune_m3_dbg.json --pmc-plan gpurun_out/dbg_plan.json > gpurun_out/dbg_plan.out 2> gpurun_out/dbg_plan.err; echo "plan rc=$?"
tail -5 gpurun_out/dbg_bench.err gpurun_out/dbg_plan.err
