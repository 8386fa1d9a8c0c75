#!/bin/bash
# SQ counters and HBM traffic of model_3 configs[2] in its default stride-1 form, replaying a
# state tuned by an unprofiled bench run first.  On failure the raw counter CSVs are removed
# so gpurun_out/ stays small enough to return.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
TUNE=gpurun_out/tune_m3_kc.json
timeout -k 10 400 python -u bench.py --no-cpu-baseline --model 3 --batch 256 --steps 10 --warmup 2 \
  --tune-cache $TUNE > gpurun_out/kc_bench.json 2> gpurun_out/kc_bench.err || exit 1
timeout -k 10 900 bash tools/kcounters.sh m3f2 $TUNE --model 3 --batch 256; rc=$?
rm -rf gpurun_out/kc_m3f2/pmc_a gpurun_out/kc_m3f2/pmc_b gpurun_out/kc_m3f2/pmc_c
[ $rc -ne 0 ] && { tail -n 30 gpurun_out/kc_m3f2/*.log; exit $rc; }
timeout -k 10 900 bash tools/pmc_box.sh m3f2 $TUNE --model 3 --batch 256; rc=$?
rm -rf gpurun_out/pmc_m3f2/pmc_fetch gpurun_out/pmc_m3f2/pmc_write gpurun_out/pmc_m3f2/pmc_sq
[ $rc -ne 0 ] && { tail -n 30 gpurun_out/pmc_m3f2/*.log; exit $rc; }
exit 0
