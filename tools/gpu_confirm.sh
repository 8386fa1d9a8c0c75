R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
source tools/gpu_steps.sh
step confirm_m0 400 python bench.py
step confirm_m3 400 python bench.py --model 3 --batch 256 --no-cpu-baseline
