#!/bin/bash
# Round-6 final evidence on the current sources (one gpurun call per part):
#   bash tools/gpu_r06_final.sh <tag> pmc    PMC traffic summaries (tools/pmc_box.sh per config),
#                                            SQ counters (tools/kcounters.sh), chain phase stamps
#   bash tools/gpu_r06_final.sh <tag> bench  the bench lines (driver command x3, 200 steps, the
#                                            other configs) and rocprofv3 kernel stats
#   bash tools/gpu_r06_final.sh <tag> abdrv [pairs]  the driver's command alternating between the
#                                            round-5 library + its shipped tuning (libtic_r05.so,
#                                            tools/tune_ab/model{0,3}_r05.json) and the current
#                                            ones, separate processes, model_0 then model_3
#   bash tools/gpu_r06_final.sh <tag> retune  a second fresh model_0 / model_3 tuning (compared
#                                            with the shipped files: the tuner's reproducibility)
#   bash tools/gpu_r06_final.sh <tag> extra   the driver's command twice more, SQ counters of the
#                                            model_3 step, rocprofv3 stats of configs[4]
#   bash tools/gpu_r06_final.sh <tag> exp     one-lane layer times of model_3 with the polyphase
#                                            form in libtic_exp.so (tools/experiments/pwino_nnb2.patch)
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1
PART=$2
cd $R
source tools/gpu_steps.sh
O=$R/gpurun_out
T=$R/tf_image_compression_amd/tune
if [ "$PART" = pmc ]; then
  bash tools/gpu_evidence.sh $TAG pmc || exit $?
  step kc_$TAG 600 bash tools/kcounters.sh $TAG $T/model0_p256_b64_s2.json
  step timing_$TAG 300 python tools/chain_timing.py --steps 40
fi
if [ "$PART" = bench ]; then
  step bench_m0_drv2_$TAG 300 python bench.py --gpus 1 --steps 20 --warmup 5
  step bench_m0_drv3_$TAG 300 python bench.py --gpus 1 --steps 20 --warmup 5
  bash tools/gpu_evidence.sh $TAG bench
fi
if [ "$PART" = abdrv ]; then
  PAIRS=${3:-4}
  for i in $(seq 1 $PAIRS); do
    for v in r05 r06; do
      if [ $v = r05 ]; then
        TIC_LIB=$R/tf_image_compression_amd/libtic_r05.so step abdrv_${TAG}_m0_${v}_$i 300 python bench.py --gpus 1 \
          --steps 20 --warmup 5 --no-cpu-baseline --tune-cache $R/tools/tune_ab/model0_r05.json --tune-any-stamp
      else
        step abdrv_${TAG}_m0_${v}_$i 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline
      fi
      echo "m0 $v $i $(grep -o '"value": [0-9.]*' $O/abdrv_${TAG}_m0_${v}_$i.log | head -1)"
    done
  done
  for i in $(seq 1 2); do
    for v in r05 r06; do
      if [ $v = r05 ]; then
        TIC_LIB=$R/tf_image_compression_amd/libtic_r05.so step abdrv_${TAG}_m3_${v}_$i 400 python bench.py --gpus 1 \
          --model 3 --batch 256 --steps 20 --warmup 5 --no-cpu-baseline --tune-cache $R/tools/tune_ab/model3_r05.json \
          --tune-any-stamp
      else
        step abdrv_${TAG}_m3_${v}_$i 400 python bench.py --gpus 1 --model 3 --batch 256 --steps 20 --warmup 5 --no-cpu-baseline
      fi
      echo "m3 $v $i $(grep -o '"value": [0-9.]*' $O/abdrv_${TAG}_m3_${v}_$i.log | head -1)"
    done
  done
fi
if [ "$PART" = retune ]; then
  mkdir -p $O/tune_$TAG
  step retune_m0_$TAG 600 python bench.py --tune-cache none --tune-save $O/tune_$TAG --no-cpu-baseline
  step retune_m3_$TAG 900 python bench.py --model 3 --batch 256 --tune-cache none --tune-save $O/tune_$TAG \
    --no-cpu-baseline --steps 20 --warmup 5
fi
if [ "$PART" = exp ]; then
  TIC_LIB=$R/tf_image_compression_amd/libtic_exp.so step exp3_$TAG 400 python tools/layer_probe.py 3 128 \
    'opt:s2_form=0' 'opt:s2_form=1'
fi
if [ "$PART" = extra ]; then
  step xdrv1_$TAG 300 python bench.py --gpus 1 --steps 20 --warmup 5
  step xdrv2_$TAG 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline
  step kc3_$TAG 900 bash tools/kcounters.sh m3_$TAG $T/model3_p256_b256_s2.json --model 3 --batch 256
  cd /tmp && export TMPDIR=/tmp
  step prof_img_$TAG 400 rocprofv3 --kernel-trace --stats -d $O/prof_img_$TAG -o p -- python3 $R/bench.py \
    --no-cpu-baseline --workload image4k --steps 10 --warmup 2
  cd $R
fi
