set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
bash tools/gpu_tune.sh r06m || exit $?
source tools/gpu_steps.sh
step timing_r06m 300 python tools/chain_timing.py --steps 40
step kc_r06m 600 bash tools/kcounters.sh r06m tf_image_compression_amd/tune/model0_p256_b64_s2.json
