# Iteration experiments (round 3): chain shapes x region order (ticket / dispatch order), enc01
# with the table loads first, phase stamps at the one-lane 32-patch launch, two-lane benches.
#   bash tools/gpu_iter.sh <tag>
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-it}
cd $R
source tools/gpu_steps.sh
O=$R/gpurun_out
step probe_$TAG 400 python tools/layer_probe.py 0 32 opt:chain_wh=2 opt:chain_wh=2,opt:chain_order=1 opt:chain_wh=3,opt:chain_order=1 opt:chain_wh=4 opt:chain_wh=4,opt:chain_order=1
TIC_CHAIN_ORDER=1 step ctime_$TAG 200 python tools/chain_timing.py --streams 1 --batch 32 --chain-wh 4
TIC_CHAIN_ORDER=1 step ctime2_$TAG 200 python tools/chain_timing.py --streams 1 --batch 32 --chain-wh 2
step etime_$TAG 200 python tools/chain_timing.py --streams 1 --batch 32 --enc01
TIC_CHAIN_ORDER=1 step chaintest_$TAG 600 python -u -m pytest tests/test_gpu_chain.py -v --timeout 300 --timeout-method thread
TIC_TUNE_LOG=1 TIC_CHAIN_ORDER=1 step bench_ord1_$TAG 600 python bench.py --tune-cache none --no-cpu-baseline
TIC_TUNE_LOG=1 step bench_ord0_$TAG 600 python bench.py --tune-cache none --no-cpu-baseline
