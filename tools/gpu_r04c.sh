# round 4: (1) why the driver's 20-step protocol reads ~7 % under 200 steps: kernel trace of the
# timed region (--trace-only), warm-up lengths; (2) the F(4x4,3x3) patch chain phase by phase
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=tf_image_compression_amd/tune/model0_p256_b64_s2.json
for w in 5 100; do
  timeout -k 10 200 python bench.py --steps 20 --warmup $w --no-cpu-baseline --tune-cache $T > gpurun_out/r04c_s20_w$w.json 2>> gpurun_out/r04c.err || exit $?
  echo "s20 w$w: $(python -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['ms_per_step'])" gpurun_out/r04c_s20_w$w.json)"
done
timeout -k 10 200 python bench.py --steps 200 --warmup 5 --no-cpu-baseline --tune-cache $T > gpurun_out/r04c_s200_w5.json 2>> gpurun_out/r04c.err || exit $?
echo "s200 w5: $(python -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['ms_per_step'])" gpurun_out/r04c_s200_w5.json)"
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r04c_tr -o tr -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline --tune-cache $T --trace-only > gpurun_out/r04c_trace.json 2>> gpurun_out/r04c.err || exit $?
cat gpurun_out/r04c_trace.json
timeout -k 10 120 python tools/chain_timing.py --tune-file tools/tune_r04/model0_p256_b64_s2_wino4.json > gpurun_out/r04c_pchain_timing.txt 2>&1 || exit $?
timeout -k 10 120 python tools/chain_timing.py --tune-file tools/tune_r04/model0_p256_b64_s2_wino4.json --streams 1 --batch 32 > gpurun_out/r04c_pchain_timing_1lane.txt 2>&1 || exit $?
cat gpurun_out/r04c_pchain_timing*.txt
