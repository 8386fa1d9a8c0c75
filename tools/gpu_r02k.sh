R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r02k}
cd $R
mkdir -p gpurun_out
source tools/gpu_steps.sh
step pytest_gpu_$TAG 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step bench_d0_$TAG 300 env TIC_DECOUPLE=0 python bench.py --tune-cache none --no-cpu-baseline
step bench_d1_$TAG 300 env TIC_DECOUPLE=1 python bench.py --tune-cache none --no-cpu-baseline
step bench_d0b_$TAG 300 env TIC_DECOUPLE=0 python bench.py --tune-cache none --no-cpu-baseline
step bench_d1b_$TAG 300 env TIC_DECOUPLE=1 python bench.py --tune-cache none --no-cpu-baseline
step bench3_$TAG 300 python bench.py --model 3 --batch 256 --tune-cache none --no-cpu-baseline
step img_$TAG 400 python bench.py --workload image4k --no-cpu-baseline
