set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "lanes or s1_forms or golden" > gpurun_out/pytest_lanes.log 2>&1
timeout -k 10 300 python tools/ab.py --model 0 --batch 64 --rounds 5 --steps 20 --cfg streams=2 --cfg streams=3 --cfg streams=4 > gpurun_out/ab_m0_lanes.json 2> gpurun_out/ab_m0_lanes.err
timeout -k 10 300 python tools/ab.py --model 3 --batch 256 --rounds 3 --steps 5 --cfg streams=2 --cfg streams=4 > gpurun_out/ab_m3_lanes.json 2> gpurun_out/ab_m3_lanes.err
