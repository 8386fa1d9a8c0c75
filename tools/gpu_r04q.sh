# round 4: SQ instruction counters per launch unit of the configs[1] step (3 PMC passes)
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 bash tools/kcounters.sh m0_r04 tf_image_compression_amd/tune/model0_p256_b64_s2.json || exit 1
cat gpurun_out/kc_m0_r04/counters.txt
