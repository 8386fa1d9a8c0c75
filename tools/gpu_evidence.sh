# evidence on the current sources (shipped tuning): PMC traffic per lane batch, the
# driver-protocol bench line and the 200-step one for configs[1], configs[2], configs[4],
# configs[3] (world 1), rocprofv3 kernel stats of the default bench.
#   bash tools/gpu_evidence.sh <tag> [pmc|bench|all]   (one gpurun call each for pmc / bench)
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r04}
PART=${2:-all}
cd $R
source tools/gpu_steps.sh
O=$R/gpurun_out
T=$R/tf_image_compression_amd/tune
if [ $PART != bench ]; then
step pmc_m0_$TAG 400 bash tools/pmc_box.sh m0_$TAG $T/model0_p256_b64_s2.json
cp $O/pmc_m0_$TAG/traffic.json tools/pmc/traffic_model0_lb32.json
step pmc_m3_$TAG 600 bash tools/pmc_box.sh m3_$TAG $T/model3_p256_b256_s2.json --model 3 --batch 256
cp $O/pmc_m3_$TAG/traffic.json tools/pmc/traffic_model3_lb128.json
step pmc_m3i_$TAG 400 bash tools/pmc_box.sh m3i_$TAG $T/model3_p256_b135_s2.json --model 3 --batch 135
cp $O/pmc_m3i_$TAG/traffic.json tools/pmc/traffic_model3_lb68.json
step pmc_c128_$TAG 400 bash tools/pmc_box.sh c128_$TAG $T/model128_p256_b64_s2.json --model 128 --batch 64
cp $O/pmc_c128_$TAG/traffic.json tools/pmc/traffic_model128_lb32.json
mkdir -p $O/pmc_traffic_$TAG && cp tools/pmc/traffic_*.json $O/pmc_traffic_$TAG/
fi
[ $PART = pmc ] && exit 0
step bench_m0_drv_$TAG 300 python bench.py --gpus 1 --steps 20 --warmup 5
step bench_m0_$TAG 300 python bench.py --no-cpu-baseline
step bench_m3_$TAG 400 python bench.py --model 3 --batch 256
step bench_img_$TAG 400 python bench.py --workload image4k --steps 10 --warmup 2
step bench_shard_$TAG 400 python bench.py --workload sharded --steps 5 --warmup 1
step bench_c128_$TAG 300 python bench.py --model 128 --batch 64 --steps 20 --warmup 5 --no-cpu-baseline
cd /tmp && export TMPDIR=/tmp
step prof_m0_$TAG 300 rocprofv3 --kernel-trace --stats -d $O/prof_m0_$TAG -o p -- python3 $R/bench.py --no-cpu-baseline --steps 20 --warmup 5
step prof_m3_$TAG 300 rocprofv3 --kernel-trace --stats -d $O/prof_m3_$TAG -o p -- python3 $R/bench.py --no-cpu-baseline --model 3 --batch 256 --steps 20 --warmup 5
rm -f $O/prof_m0_$TAG/p_kernel_trace.csv $O/prof_m3_$TAG/p_kernel_trace.csv
