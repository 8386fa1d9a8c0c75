# One GPU call of round-3 iteration work: the GPU suite, one-lane launch timings of the
# chain shapes, the default bench (shipped tuning), a fresh step-tuned bench (state saved for
# tf_image_compression_amd/tune/), configs[3] sharded and configs[4] image4k lines.
#   bash tools/gpu_round.sh <tag> [skip-tests]
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r}
cd $R
mkdir -p gpurun_out/tune_$TAG
source tools/gpu_steps.sh
O=$R/gpurun_out
if [ "$2" != "skip-tests" ]; then
  step gputest_$TAG 1100 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread
fi
step probe_chain_$TAG 300 python tools/layer_probe.py 0 32 opt:chain_wh=2 opt:chain_wh=3 opt:chain_wh=1 opt:chain=0
step bench_m0_$TAG 400 python bench.py
step bench_m0_fresh_$TAG 600 python bench.py --tune-cache none --tune-save $O/tune_$TAG --no-cpu-baseline
step bench_shard_$TAG 400 python bench.py --workload sharded --steps 5 --warmup 1
step bench_img_$TAG 600 python bench.py --workload image4k --no-cpu-baseline --steps 10 --warmup 2 --tune-save $O/tune_$TAG
