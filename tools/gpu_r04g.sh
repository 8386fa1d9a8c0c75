# round 4: F(4x4,3x3) weights through raw buffer loads: parity (per-layer + end to end) and phase stamps
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_wino4.py tests/test_gpu_pchain.py tests/test_gpu_chain.py > gpurun_out/r04h_pytest.log 2>&1 || { tail -30 gpurun_out/r04h_pytest.log; exit 1; }
tail -2 gpurun_out/r04h_pytest.log
timeout -k 10 120 python tools/wino4_timing.py --n 128 --hw 64 --res 1 --reps 2 > gpurun_out/r04h_w4_64.txt 2>&1 || { cat gpurun_out/r04h_w4_64.txt; exit 1; }
timeout -k 10 120 python tools/wino4_timing.py --n 128 --hw 32 --res 0 --reps 2 > gpurun_out/r04h_w4_32.txt 2>&1 || { cat gpurun_out/r04h_w4_32.txt; exit 1; }
cat gpurun_out/r04h_w4_64.txt gpurun_out/r04h_w4_32.txt
