#!/bin/bash
# Round-6 polyphase Winograd (s2_form) GPU steps:  bash tools/gpu_pwino.sh <tag> <part>...
#   tests : tests/test_gpu_pwino.py (per-layer and codec parity, fusion independence)
#   probe : one-lane per-launch times, s2_form 0 vs 1 (model_0 n=32, model_3 n=128)
#   ab    : alternating two-lane step A/B, s2_form 0 vs 1 (model_0 b64, model_3 b256)
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1
shift
cd $R
mkdir -p gpurun_out
source tools/gpu_steps.sh
T=$R/tf_image_compression_amd/tune
for part in "$@"; do
  case $part in
    tests) step pwtests_$TAG 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu \
             tests/test_gpu_pwino.py tests/test_gpu_chain.py ;;
    probe) step pwprobe0_$TAG 300 python tools/layer_probe.py 0 32 'opt:s2_form=0' 'opt:s2_form=1' \
             'opt:s1_form=0,opt:s2_form=0' 'opt:s1_form=0,opt:s2_form=1' &&
           step pwprobe3_$TAG 400 python tools/layer_probe.py 3 128 'opt:s2_form=0' 'opt:s2_form=1' ;;
    ab) step pwab0_$TAG 600 python tools/ab.py --model 0 --batch 64 --rounds 6 --steps 60 \
             --tune-file $T/model0_p256_b64_s2.json --cfg s2_form=0 --cfg s2_form=1 &&
        step pwab3_$TAG 900 python tools/ab.py --model 3 --batch 256 --rounds 5 --steps 10 \
             --tune-file $T/model3_p256_b256_s2.json --cfg s2_form=0 --cfg s2_form=1 ;;
  esac
done
