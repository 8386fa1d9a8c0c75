# round 4: conv3x3_wino4_kernel phase stamps per wave, with timing probes (bits: 1 weights from one
# step, 2 no staging loads, 4 no stores / residual loads; results invalid under a probe)
set -o pipefail
cd $GRAFT_REPO_ROOT
for p in 0 1 2 4 7; do
  timeout -k 10 120 python tools/wino4_timing.py --n 128 --hw 64 --res 1 --reps 2 --probe $p > gpurun_out/r04i_p$p.txt 2>&1 || { cat gpurun_out/r04i_p$p.txt; exit 1; }
  tail -1 gpurun_out/r04i_p$p.txt
done
