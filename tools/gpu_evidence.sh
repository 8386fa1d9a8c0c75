# Round-end evidence on the GPU box, one tuning state per model shared by every pass:
#   bash tools/gpu_evidence.sh <tag>
# -> gpurun_out/{gputest,bench_m0,bench_m3,bench_img}_<tag>.log, tune_m{0,3}_<tag>.json,
#    pmc_m{0,3}_<tag>/traffic.json + summary.txt, prof_m0_<tag>/ (rocprofv3 kernel stats)
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-ev}
cd $R
mkdir -p gpurun_out
source tools/gpu_steps.sh
O=$R/gpurun_out
step gputest_$TAG 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step bench_m0_$TAG 400 python bench.py --tune-cache $O/tune_m0_$TAG.json
step pmc_m0_$TAG 900 bash tools/pmc_box.sh m0_$TAG $O/tune_m0_$TAG.json
step stats_m0_$TAG 300 bash -c "cd /tmp && export TMPDIR=/tmp && rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_m0_$TAG -o p -- python3 $R/bench.py --tune-cache $O/tune_m0_$TAG.json --no-cpu-baseline --steps 50 --warmup 5"
step bench_m3_$TAG 400 python bench.py --model 3 --batch 256 --tune-cache $O/tune_m3_$TAG.json --no-cpu-baseline
step pmc_m3_$TAG 900 bash tools/pmc_box.sh m3_$TAG $O/tune_m3_$TAG.json --model 3 --batch 256
step bench_img_$TAG 400 python bench.py --workload image4k --no-cpu-baseline
