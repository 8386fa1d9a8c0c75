#!/bin/bash
# Run on the GPU box (via gpurun): three separate PMC passes (FETCH_SIZE; WRITE_SIZE; SQ
# timing + MFMA counters) over `bench.py --pmc-plan` (the bench's tuning, then steady
# steps on one lane at the per-lane batch), kernel-trace only besides --pmc, then the
# per-launch-unit summary stamped with the kernel-source digest.
#   bash tools/pmc_box.sh <tag> [bench args...]   -> gpurun_out/pmc_<tag>/traffic.json
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-m0}
shift || true
O=$R/gpurun_out/pmc_$TAG
mkdir -p $O
ARGS="--no-cpu-baseline --steps 4 --warmup 1 --pmc-plan $O/plan.json $*"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/pmc_fetch -o p -- python3 $R/bench.py $ARGS > $O/fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/pmc_write -o p -- python3 $R/bench.py $ARGS > $O/write.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $O/pmc_sq -o p -- python3 $R/bench.py $ARGS > $O/sq.log 2>&1
cd $R
python3 tools/pmc_summary.py $O $O/plan.json $O/traffic.json > $O/summary.txt
rm -f $O/pmc_*/p_kernel_trace.csv
