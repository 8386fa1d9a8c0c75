R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r02s}
cd $R
mkdir -p gpurun_out
source tools/gpu_steps.sh
step par_$TAG 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "fused"
step probe_$TAG 400 python tools/dec10_probe.py
step lp0_$TAG 400 python tools/layer_probe.py 0 32 "opt:fuse01=0" "opt:fuse01=1,TIC_ENC01_VARIANT=1" "opt:fuse01=1,TIC_ENC01_VARIANT=2" "opt:fuse01=1,TIC_ENC01_VARIANT=3" "opt:fuse01=1,TIC_ENC01_VARIANT=4"
step bench_$TAG 300 python bench.py --tune-cache none --no-cpu-baseline
