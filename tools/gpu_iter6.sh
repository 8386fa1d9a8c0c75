# Round-3 iteration: chain hand-off stress across shapes / lanes (model_3 b256, model_0 b64),
# then the model_3 configs[2] fresh-tuned bench (tuner now rejects timed-out chain trials).
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-it}
cd $R
mkdir -p gpurun_out/tune_$TAG
source tools/gpu_steps.sh
O=$R/gpurun_out
step stress_m3_$TAG 400 python -u tools/chain_stress.py --model 3 --batch 256 --iters 20
step stress_m0_$TAG 300 python -u tools/chain_stress.py --model 0 --batch 64 --iters 40
TIC_TUNE_LOG=1 step bench_m3_$TAG 900 python bench.py --model 3 --batch 256 --tune-cache none --tune-save $O/tune_$TAG --no-cpu-baseline
