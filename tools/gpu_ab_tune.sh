# Alternating A/B of two tuning states on one library (one tools/ab.py process per sample):
#   bash tools/gpu_ab_tune.sh <tag> <model> <batch> <tune A json> <tune B json> [pairs]
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; M=$2; B=$3; TA=$4; TB=$5; PAIRS=${6:-3}
for i in $(seq 1 $PAIRS); do
  for v in A B; do
    if [ $v = A ]; then T=$TA; else T=$TB; fi
    timeout -k 10 200 python tools/ab.py --model $M --batch $B --rounds 3 --steps 60 --tune-file $T --cfg streams=2 \
      > gpurun_out/abtune_${TAG}_${v}_$i.json 2>> gpurun_out/abtune_$TAG.err || exit 1
    echo "m$M $v $i $(python -c "import json,sys; d=json.load(open(sys.argv[1])); v=list(d.values())[0]; print(v['median_ms'], v['mpix_s'])" gpurun_out/abtune_${TAG}_${v}_$i.json)"
  done
done
