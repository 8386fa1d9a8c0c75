# round 4: patch-chain bit identity, F(4x4) margin / split / tuner tests, form-1 vs form-2 model_0 bench
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests/test_gpu_pchain.py tests/test_gpu_wino4.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r04b_pytest.log 2>&1 || { tail -40 gpurun_out/r04b_pytest.log; exit 1; }
tail -3 gpurun_out/r04b_pytest.log
for f in wino wino4; do
  TIC_TUNE_LOG=1 TIC_S1_FORM=$f timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --tune-save gpurun_out/tune_$f > gpurun_out/r04b_$f.json 2> gpurun_out/r04b_$f.err || exit $?
  tail -c 300 gpurun_out/r04b_$f.json
done
