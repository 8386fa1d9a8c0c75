# round 4: conv3x3_wino4_kernel phase stamps (configs[2]'s dominant launch: 128 patches of 64x64x64, residual)
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 120 python tools/wino4_timing.py --n 128 --hw 64 --res 1 > gpurun_out/r04f_w4_64.txt 2>&1 || { cat gpurun_out/r04f_w4_64.txt; exit 1; }
timeout -k 10 120 python tools/wino4_timing.py --n 128 --hw 32 --res 0 > gpurun_out/r04f_w4_32.txt 2>&1 || { cat gpurun_out/r04f_w4_32.txt; exit 1; }
cat gpurun_out/r04f_w4_*.txt
