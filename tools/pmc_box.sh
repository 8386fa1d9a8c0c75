#!/bin/bash
# Run on the GPU box (via gpurun): three separate PMC passes over the default bench
# (FETCH_SIZE, WRITE_SIZE, SQ timing counters), kernel-trace only besides --pmc.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
ARGS="--no-cpu-baseline --steps 5 --warmup 2 --profile-iters 1 $*"
P=${PMC_PREFIX:-pmc}
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/${P}_fetch -o p -- python3 $R/bench.py $ARGS > $R/gpurun_out/${P}_fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/${P}_write -o p -- python3 $R/bench.py $ARGS > $R/gpurun_out/${P}_write.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $R/gpurun_out/${P}_sq -o p -- python3 $R/bench.py $ARGS > $R/gpurun_out/${P}_sq.log 2>&1
