# Winograd stride-1 form + LDS-weight VALU last layer: parity, then interleaved A/B timing.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread \
  -k "winograd or s1_forms or valu or conv3x3_layer" > gpurun_out/pytest_wino.log 2>&1
timeout -k 10 240 python tools/ab.py --model 0 --batch 64 --rounds 5 --steps 20 \
  --cfg s1_form=0 --cfg s1_form=1 > gpurun_out/ab_m0_wino.json 2> gpurun_out/ab_m0_wino.err
timeout -k 10 300 python tools/ab.py --model 3 --batch 256 --rounds 3 --steps 5 \
  --cfg s1_form=0 --cfg s1_form=1 > gpurun_out/ab_m3_wino.json 2> gpurun_out/ab_m3_wino.err
