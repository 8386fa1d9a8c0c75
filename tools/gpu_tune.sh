# Tuning call: fresh step-tuned states for every benched configuration (saved, then
# installed as the shipped tuning); the GPU suite against them runs as its own call
# (python -u -m pytest tests -m gpu ...).   bash tools/gpu_tune.sh <tag>
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-fa}
cd $R
mkdir -p gpurun_out/tune_$TAG
source tools/gpu_steps.sh
O=$R/gpurun_out
step tune_m0_$TAG 600 python bench.py --tune-cache none --tune-save $O/tune_$TAG --no-cpu-baseline
step tune_m3_$TAG 900 python bench.py --model 3 --batch 256 --tune-cache none --tune-save $O/tune_$TAG --no-cpu-baseline
step tune_c128_$TAG 600 python bench.py --model 128 --batch 64 --tune-cache none --tune-save $O/tune_$TAG --no-cpu-baseline --steps 20 --warmup 5
step tune_img_$TAG 600 python bench.py --workload image4k --no-cpu-baseline --steps 10 --warmup 2 --tune-cache none --tune-save $O/tune_$TAG
cp $O/tune_$TAG/*.json tf_image_compression_amd/tune/
