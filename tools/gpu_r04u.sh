# round 4: F(4x4,3x3) with B^T d staged once per (column, channel) — form-2 tests, per-launch
# phase timing, then old / new library alternating on model_3 (configs[2]) and model_0
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_wino4.py tests/test_gpu_parity.py tests/test_gpu_configs.py > gpurun_out/r04u_pytest.log 2>&1 || { tail -30 gpurun_out/r04u_pytest.log; exit 1; }
tail -1 gpurun_out/r04u_pytest.log
for v in old new; do
  if [ $v = new ]; then L=tf_image_compression_amd/libtic.so; else L=tf_image_compression_amd/libtic_old.so; fi
  TIC_LIB=$L timeout -k 10 120 python tools/wino4_timing.py > gpurun_out/r04u_timing_$v.txt 2>&1 || { cat gpurun_out/r04u_timing_$v.txt; exit 1; }
  echo "== timing $v"; head -c 900 gpurun_out/r04u_timing_$v.txt
done
for cfg in "3 256 model3_p256_b256_s2"; do
  set -- $cfg
  T=tf_image_compression_amd/tune/$3.json
  for i in 1 2 3; do
    for v in old new; do
      if [ $v = new ]; then L=tf_image_compression_amd/libtic.so; else L=tf_image_compression_amd/libtic_old.so; fi
      TIC_LIB=$L timeout -k 10 200 python tools/ab.py --model $1 --batch $2 --rounds 3 --steps 60 --tune-file $T --cfg streams=2 > gpurun_out/r04u_ab_m$1_${v}_$i.json 2>> gpurun_out/r04u.err || exit 1
      echo "m$1 $v $i $(python -c "import json,sys; d=json.load(open(sys.argv[1])); v=list(d.values())[0]; print(v['median_ms'], v['mpix_s'])" gpurun_out/r04u_ab_m$1_${v}_$i.json)"
    done
  done
done
