R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r02l}
cd $R
mkdir -p gpurun_out
source tools/gpu_steps.sh
for cfg in "2 0" "2 1" "3 0" "3 1" "4 0" "2 0" "2 1"; do
  set -- $cfg
  step bench_s$1_c$2_$TAG 300 env TIC_CHAIN=$2 python bench.py --streams $1 --tune-cache none --no-cpu-baseline
done
