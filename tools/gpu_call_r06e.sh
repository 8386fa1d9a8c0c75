R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
source tools/gpu_steps.sh
T=$R/tf_image_compression_amd/tune
step pwtests_e 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_gpu_pwino.py tests/test_gpu_chain.py
ABA=$R/tf_image_compression_amd/libtic_base.so ABB=$R/tf_image_compression_amd/libtic.so step abil_e 900 bash tools/gpu_ab.sh il_e 0 64 $T/model0_p256_b64_s2.json 4
step pwprobe0_e 300 python tools/layer_probe.py 0 32 'opt:s2_form=0' 'opt:s2_form=1' 'opt:s1_form=0,opt:s2_form=1'
step pwprobe3_e 400 python tools/layer_probe.py 3 128 'opt:s2_form=0' 'opt:s2_form=1'
