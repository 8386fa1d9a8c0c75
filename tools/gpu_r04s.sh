# round 4: region chain VALU trims (weights by buffer loads, sign-pattern transform) — tests,
# then old / new library alternating on the shipped tuning, and chain phases
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_chain.py tests/test_gpu_parity.py > gpurun_out/r04s_pytest.log 2>&1 || { tail -30 gpurun_out/r04s_pytest.log; exit 1; }
tail -1 gpurun_out/r04s_pytest.log
T=tf_image_compression_amd/tune/model0_p256_b64_s2.json
for i in 1 2 3; do
  for v in old new; do
    if [ $v = new ]; then L=tf_image_compression_amd/libtic.so; else L=tf_image_compression_amd/libtic_old.so; fi
    TIC_LIB=$L timeout -k 10 200 python tools/ab.py --model 0 --batch 64 --rounds 3 --steps 100 --tune-file $T --cfg streams=2 > gpurun_out/r04s_ab_${v}_$i.json 2>> gpurun_out/r04s.err || exit 1
    echo "$v $i $(python -c "import json,sys; d=json.load(open(sys.argv[1])); v=list(d.values())[0]; print(v['median_ms'], v['mpix_s'])" gpurun_out/r04s_ab_${v}_$i.json)"
  done
done
timeout -k 10 120 python tools/chain_timing.py --tune-file $T > gpurun_out/r04s_chain_timing.txt 2>&1 || { cat gpurun_out/r04s_chain_timing.txt; exit 1; }
head -c 700 gpurun_out/r04s_chain_timing.txt
