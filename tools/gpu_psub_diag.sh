# Round 6 diagnosis of tools/experiments/psub_all_transforms.patch: the polyphase layer tests
# with the packed subtraction in the polyphase transforms only, written two ways — A: the
# chain's psub (operand halves built element by element), B: halves as .xy / .zw swizzles.
#   bash tools/gpu_psub_diag.sh <tag>
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1
cd $R
source tools/gpu_steps.sh
for v in pA pB; do
  TIC_LIB=$R/tf_image_compression_amd/libtic_$v.so step diag_${v}_$TAG 300 python -u -m pytest \
    tests/test_gpu_pwino.py -v --timeout 120 --timeout-method thread -k "pwino_layer or chain_decode2"
  tail -2 gpurun_out/diag_${v}_$TAG.log
done
