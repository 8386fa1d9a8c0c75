# round 4: the shader clock inside conv3x3_wino4_kernel's K loop
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 120 python tools/wino4_timing.py --n 128 --hw 64 --res 1 --reps 3 > gpurun_out/r04k.txt 2>&1 || { cat gpurun_out/r04k.txt; exit 1; }
cat gpurun_out/r04k.txt
