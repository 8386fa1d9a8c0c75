R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
source tools/gpu_steps.sh
T=$R/tf_image_compression_amd/tune
step pwtests_f 900 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_gpu_pwino.py tests/test_gpu_chain.py tests/test_gpu_product.py tests/test_gpu_configs.py
step pwab3_f 900 python tools/ab.py --model 3 --batch 256 --rounds 6 --steps 10 --tune-file $T/model3_p256_b256_s2.json --cfg s2_form=0 --cfg s2_form=1
step pwab0_f 600 python tools/ab.py --model 0 --batch 64 --rounds 6 --steps 60 --tune-file $T/model0_p256_b64_s2.json --cfg s2_form=0 --cfg s2_form=1
