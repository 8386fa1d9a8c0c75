#!/bin/bash
# Run on the GPU box (via gpurun): three separate PMC passes (FETCH_SIZE; WRITE_SIZE; SQ
# timing + MFMA counters) over `bench.py --pmc-plan` — the bench's tuning replayed from
# TUNE (tic_tuning_export of an unprofiled bench run, so every pass launches the same
# kernels), then steady steps on one lane at the per-lane batch — kernel-trace only
# besides --pmc; then the per-launch-unit summary stamped with the kernel-source digest.
#   bash tools/pmc_box.sh <tag> <tune.json> [bench args...]  -> gpurun_out/pmc_<tag>/traffic.json
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1
TUNE=$(realpath $2)
shift 2
O=$R/gpurun_out/pmc_$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for pass in fetch write sq; do
  case $pass in
    fetch) CTR="FETCH_SIZE" ;;
    write) CTR="WRITE_SIZE" ;;
    sq) CTR="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" ;;
  esac
  timeout -k 10 300 rocprofv3 --pmc $CTR --kernel-trace --output-format csv -d $O/pmc_$pass -o p -- \
    python3 $R/bench.py --no-cpu-baseline --steps 4 --warmup 1 --tune-cache $TUNE --pmc-plan $O/plan_$pass.json "$@" \
    > $O/$pass.log 2>&1
  rm -f $O/pmc_$pass/p_kernel_trace.csv
done
cd $R
python3 tools/pmc_summary.py $O $O/traffic.json > $O/summary.txt 2>&1 || true
# keep the summary, drop the raw per-dispatch CSVs (tens of MB)
rm -rf $O/pmc_fetch $O/pmc_write $O/pmc_sq
