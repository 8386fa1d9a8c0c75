# Round-6 GPU steps (one gpurun call per invocation):  bash tools/gpu_r06.sh <tag> <part>...
#   tests   : the chain / product / parity / enc01 GPU tests on the current build
#   timing  : tools/chain_timing.py (phase stamps incl. wave 4) on the current build
#   kc      : SQ counters of the model_0 step (tools/kcounters.sh) on the current build
#   kcold   : the same on libtic_old.so
#   ab      : alternating A/B libtic_old.so vs libtic.so, model_0 b64, shipped tuning replayed
#   ab3     : the same for model_3 b256
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1
shift
cd $R
source tools/gpu_steps.sh
T=$R/tf_image_compression_amd/tune
for part in "$@"; do
  case $part in
    tests) step tests_$TAG 900 python -u -m pytest -v --timeout 240 --timeout-method thread -m gpu \
             tests/test_gpu_chain.py tests/test_gpu_product.py tests/test_gpu_parity.py ;;
    timing) step timing_$TAG 300 python tools/chain_timing.py --steps 40 ;;
    kc) step kc_$TAG 600 bash tools/kcounters.sh $TAG $T/model0_p256_b64_s2.json ;;
    kc3) step kc3_$TAG 600 bash tools/kcounters.sh m3_$TAG $T/model3_p256_b256_s2.json --model 3 --batch 256 ;;
    kcold) TIC_LIB=$R/tf_image_compression_amd/libtic_old.so step kcold_$TAG 600 bash tools/kcounters.sh old_$TAG $T/model0_p256_b64_s2.json ;;
    ab) step ab_$TAG 900 bash tools/gpu_ab.sh $TAG 0 64 $T/model0_p256_b64_s2.json 4 ;;
    ab3) step ab3_$TAG 900 bash tools/gpu_ab.sh m3_$TAG 3 256 $T/model3_p256_b256_s2.json 3 ;;
    abd2e) ABA=$R/tf_image_compression_amd/libtic.so ABB=$R/tf_image_compression_amd/libtic_d2e.so \
             step abd2e_$TAG 900 bash tools/gpu_ab.sh d2e_$TAG 0 64 $T/model0_p256_b64_s2.json 3 ;;
    abd2e4) ABA=$R/tf_image_compression_amd/libtic.so ABB=$R/tf_image_compression_amd/libtic_d2e4.so \
             step abd2e4_$TAG 900 bash tools/gpu_ab.sh d2e4_$TAG 0 64 $T/model0_p256_b64_s2.json 3 ;;
    abst) ABA=$R/tf_image_compression_amd/libtic_nostage.so step abst_$TAG 900 bash tools/gpu_ab.sh st_$TAG 0 64 \
             $T/model0_p256_b64_s2.json 4 ;;
    abst3) ABA=$R/tf_image_compression_amd/libtic_nostage.so step abst3_$TAG 900 bash tools/gpu_ab.sh st3_$TAG 3 256 \
             $T/model3_p256_b256_s2.json 3 ;;
    abpre) ABA=$R/tf_image_compression_amd/libtic_pre.so step abpre_$TAG 900 bash tools/gpu_ab.sh pre_$TAG 0 64 \
             $T/model0_p256_b64_s2.json 4 ;;
    abpre3) ABA=$R/tf_image_compression_amd/libtic_pre.so step abpre3_$TAG 900 bash tools/gpu_ab.sh pre3_$TAG 3 256 \
             $T/model3_p256_b256_s2.json 3 ;;
    abpfl) ABA=$R/tf_image_compression_amd/libtic.so ABB=$R/tf_image_compression_amd/libtic_pflate.so \
             step abpfl_$TAG 900 bash tools/gpu_ab.sh pfl_$TAG 0 64 $T/model0_p256_b64_s2.json 4 ;;
    timingv) TIC_LIB=$R/tf_image_compression_amd/libtic_$VAR.so step timing_${VAR}_$TAG 300 python tools/chain_timing.py --steps 40 ;;
    abtune) step abtune_$TAG 900 bash tools/gpu_ab_tune.sh m0_$TAG 0 64 $R/tools/tune_ab/model0_r05.json \
             $T/model0_p256_b64_s2.json 5 ;;
    abtune3) step abtune3_$TAG 900 bash tools/gpu_ab_tune.sh m3_$TAG 3 256 $R/tools/tune_ab/model3_r05.json \
             $T/model3_p256_b256_s2.json 3 ;;
    cumask) step cumask_$TAG 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
             tests/test_gpu_chain.py -k exact_fill ;;
    forms) step forms_layers_$TAG 300 python tools/layer_probe.py 0 32 'TIC_FUSE_TAIL=1' 'TIC_FUSE_TAIL=0' \
             'TIC_FUSE_TAIL=0,TIC_RGB_OUT_FORM=scatter' 'TIC_FUSE_TAIL=0,TIC_RGB_OUT_FORM=dense' &&
           step forms_ab_$TAG 600 python tools/ab.py --model 0 --batch 64 --rounds 5 --steps 60 \
             --tune-file $T/model0_p256_b64_s2.json --cfg streams=2,fuse_tail=1,env:TIC_RGB_OUT_FORM=valu \
             --cfg streams=2,fuse_tail=0,env:TIC_RGB_OUT_FORM=valu --cfg streams=2,env:TIC_RGB_OUT_FORM=scatter \
             --cfg streams=2,env:TIC_RGB_OUT_FORM=dense ;;
    split) step split_$TAG 900 bash tools/gpu_ab_env.sh $TAG 0 64 $T/model0_p256_b64_s2.json 3 - \
             TIC_LANE_CU_SPLIT=half TIC_LANE_CU_SPLIT=alt ;;
    split3) step split3_$TAG 900 bash tools/gpu_ab_env.sh m3_$TAG 3 256 $T/model3_p256_b256_s2.json 3 - \
             TIC_LANE_CU_SPLIT=half TIC_LANE_CU_SPLIT=alt ;;
    tune) step tune_m0_$TAG 600 env TIC_TUNE_LOG=1 python bench.py --tune-cache none --tune-save $R/gpurun_out/tune_$TAG \
             --no-cpu-baseline --steps 50 --warmup 10 ;;
    tune3) step tune_m3_$TAG 1000 env TIC_TUNE_LOG=1 python bench.py --model 3 --batch 256 --tune-cache none \
             --tune-save $R/gpurun_out/tune_$TAG --no-cpu-baseline --steps 20 --warmup 5 ;;
    tunec) step tune_c128_$TAG 600 env TIC_TUNE_LOG=1 python bench.py --model 128 --batch 64 --tune-cache none \
             --tune-save $R/gpurun_out/tune_$TAG --no-cpu-baseline --steps 20 --warmup 5 ;;
    tunei) step tune_img_$TAG 600 env TIC_TUNE_LOG=1 python bench.py --workload image4k --no-cpu-baseline --steps 10 \
             --warmup 2 --tune-cache none --tune-save $R/gpurun_out/tune_$TAG ;;
  esac
done
