# Channel-split chain shapes (chain_wh 3 / 4) against the 512-thread one: bit-identity tests,
# one-lane launch timings, phase stamps (one lane and two lanes), and the two-lane bench with
# each shape pinned (step-tuned in the run, tuner log kept).
#   bash tools/gpu_chain_cs.sh <tag>
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-cs}
cd $R
mkdir -p gpurun_out/tune_$TAG
source tools/gpu_steps.sh
O=$R/gpurun_out
step chaintest_$TAG 600 python -u -m pytest tests/test_gpu_chain.py tests/test_gpu_product.py tests/test_gpu_parity.py -k "chain or product or fused_first or splits or golden" -v --timeout 300 --timeout-method thread
step probe_e01_$TAG 300 python tools/layer_probe.py 0 32 TIC_ENC01_VARIANT=3 TIC_ENC01_VARIANT=5 TIC_ENC01_VARIANT=4
step probe_$TAG 300 python tools/layer_probe.py 0 32 opt:chain_wh=2 opt:chain_wh=3 opt:chain_wh=4
step ctime1_$TAG 200 python tools/chain_timing.py --streams 1 --chain-wh 3
step ctime1b_$TAG 200 python tools/chain_timing.py --streams 1 --chain-wh 4
step ctime2_$TAG 200 python tools/chain_timing.py --streams 2 --chain-wh 3
for wh in 2 3 4; do
  TIC_TUNE_LOG=1 TIC_CHAIN_WH=$wh step bench_wh${wh}_$TAG 600 python bench.py --tune-cache none --no-cpu-baseline
done
step etime1_$TAG 200 python tools/chain_timing.py --streams 1 --enc01
step etime2_$TAG 200 python tools/chain_timing.py --streams 2 --enc01
