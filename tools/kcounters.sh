#!/bin/bash
# Investigative SQ counter passes (separate rocprofv3 --pmc runs, <= 8 SQ counters each)
# over `bench.py --pmc-plan` with a replayed tuning state; per launch unit medians are
# printed by tools/kcounters.py.   bash tools/kcounters.sh <tag> <tune.json> [bench args]
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1
TUNE=$(realpath $2)
shift 2
O=$R/gpurun_out/kc_$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
A="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"
B="SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_SMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_VALU"
C="SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_INST_LEVEL_VMEM"
for pass in a b c; do
  case $pass in a) CTR=$A ;; b) CTR=$B ;; c) CTR=$C ;; esac
  timeout -k 10 300 rocprofv3 --pmc $CTR --kernel-trace --output-format csv -d $O/pmc_$pass -o p -- \
    python3 $R/bench.py --no-cpu-baseline --steps 3 --warmup 1 --tune-cache $TUNE --tune-any-stamp --pmc-plan $O/plan_$pass.json "$@" \
    > $O/$pass.log 2>&1
  rm -f $O/pmc_$pass/p_kernel_trace.csv
done
cd $R
python3 tools/kcounters.py $O > $O/counters.txt 2>&1 || true
rm -rf $O/pmc_a $O/pmc_b $O/pmc_c
