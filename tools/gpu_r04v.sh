# round 4: staged B^T d in conv3x3_wino4_kernel and the patch chain — form-2 / chain tests,
# phase timing, model_3 old / new alternating
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_wino4.py tests/test_gpu_pchain.py tests/test_gpu_chain.py tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_image.py > gpurun_out/r04v_pytest.log 2>&1 || { tail -30 gpurun_out/r04v_pytest.log; exit 1; }
tail -1 gpurun_out/r04v_pytest.log
TIC_LIB=tf_image_compression_amd/libtic.so timeout -k 10 120 python tools/wino4_timing.py > gpurun_out/r04v_timing_new.txt 2>&1 || { cat gpurun_out/r04v_timing_new.txt; exit 1; }
head -c 700 gpurun_out/r04v_timing_new.txt
T=tf_image_compression_amd/tune/model3_p256_b256_s2.json
for i in 1 2 3; do
  for v in old new; do
    if [ $v = new ]; then L=tf_image_compression_amd/libtic.so; else L=tf_image_compression_amd/libtic_old.so; fi
    TIC_LIB=$L timeout -k 10 200 python tools/ab.py --model 3 --batch 256 --rounds 3 --steps 60 --tune-file $T --cfg streams=2 > gpurun_out/r04v_ab_m3_${v}_$i.json 2>> gpurun_out/r04v.err || exit 1
    echo "m3 $v $i $(python -c "import json,sys; d=json.load(open(sys.argv[1])); v=list(d.values())[0]; print(v['median_ms'], v['mpix_s'])" gpurun_out/r04v_ab_m3_${v}_$i.json)"
  done
done
