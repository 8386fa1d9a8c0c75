# round 4: F(4x4,3x3) K-loop schedules (W4_SCHED 0 = shipped, 1 = sched_group_barrier, 2 = explicit
# interleave): phase stamps, alternating, + a parity check of each variant
set -o pipefail
cd $GRAFT_REPO_ROOT
for rep in 1 2; do
for v in 0 s1 s2; do
  if [ $v = 0 ]; then L=tf_image_compression_amd/libtic.so; else L=tf_image_compression_amd/libtic_$v.so; fi
  TIC_LIB=$L timeout -k 10 120 python tools/wino4_timing.py --n 128 --hw 64 --res 1 --reps 2 > gpurun_out/r04j_$v.txt 2>&1 || { cat gpurun_out/r04j_$v.txt; exit 1; }
  echo "$v: $(tail -1 gpurun_out/r04j_$v.txt)"
done
done
for v in s1 s2; do
  TIC_LIB=tf_image_compression_amd/libtic_$v.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "winograd4" > gpurun_out/r04j_pt_$v.log 2>&1 || { tail -20 gpurun_out/r04j_pt_$v.log; exit 1; }
  echo "$v parity: $(tail -1 gpurun_out/r04j_pt_$v.log)"
done
