# round 4: F(2x2,3x3) chain phase by phase in the two-lane step (shipped tuning)
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 120 python tools/chain_timing.py > gpurun_out/r04n_chain_timing.txt 2>&1 || { cat gpurun_out/r04n_chain_timing.txt; exit 1; }
cat gpurun_out/r04n_chain_timing.txt
