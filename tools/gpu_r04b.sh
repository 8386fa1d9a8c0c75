# round 4: patch-chain bit identity, F(4x4) margin / split / tuner tests, form-1 vs form-2 model_0
# bench (tuned in the run, saved), then the driver's protocol (20 steps, 5 warm-up) on both
# tunings, alternating, beside the 200-step figure
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests/test_gpu_pchain.py tests/test_gpu_wino4.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r04b_pytest.log 2>&1 || { tail -40 gpurun_out/r04b_pytest.log; exit 1; }
tail -3 gpurun_out/r04b_pytest.log
cat gpurun_out/wino4_margin.json
for f in wino wino4; do
  TIC_TUNE_LOG=1 TIC_S1_FORM=$f timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --tune-save gpurun_out/tune_$f > gpurun_out/r04b_$f.json 2> gpurun_out/r04b_$f.err || exit $?
  python tools/show_bench.py r04b_$f.json || true
done
for i in 1 2 3; do
  for f in wino wino4; do
    TIC_S1_FORM=$f timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --tune-cache gpurun_out/tune_$f/model0_p256_b64_s2.json > gpurun_out/r04b_${f}_s20_$i.json 2>> gpurun_out/r04b_s20.err || exit $?
    echo "$f s20 run $i: $(python -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['ms_per_step'], d['tuning'])" gpurun_out/r04b_${f}_s20_$i.json)"
  done
done
