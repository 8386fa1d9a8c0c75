# Round 6, packed subtractions in every Winograd transform (tic_kernels.h psub): alternating
# A/B of the previous build (libtic_base.so) against the new one on the shipped tunings, then a
# fresh tuning of the new sources and the GPU suite against it.   bash tools/gpu_psub.sh <tag>
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1
cd $R
mkdir -p gpurun_out
T=tf_image_compression_amd/tune
export ABA=tf_image_compression_amd/libtic_base.so ABB=tf_image_compression_amd/libtic.so
bash tools/gpu_ab.sh ${TAG}_m0 0 64 $T/model0_p256_b64_s2.json 3 || exit 1
bash tools/gpu_ab.sh ${TAG}_m3 3 256 $T/model3_p256_b256_s2.json 2 || exit 1
unset ABA ABB
bash tools/gpu_tune.sh $TAG || exit 1
bash tools/gpu_suite.sh $TAG
