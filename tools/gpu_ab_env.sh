# Alternating A/B of environment settings read at handle creation (one ab.py process per
# sample, same library and replayed tuning, settings in rotating order):
#   bash tools/gpu_ab_env.sh <tag> <model> <batch> <tune json> <pairs> 'ENV=..[ ENV2=..]' 'ENV=..' ...
# ('-' = no extra environment); results in gpurun_out/abenv_<tag>_<k>_<i>.json, one line per run.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; M=$2; B=$3; T=$4; PAIRS=$5
shift 5
for i in $(seq 1 $PAIRS); do
  k=0
  for setting in "$@"; do
    k=$((k + 1))
    if [ "$setting" = "-" ]; then E=""; else E="$setting"; fi
    env $E timeout -k 10 200 python tools/ab.py --model $M --batch $B --rounds 3 --steps 60 --tune-file $T \
      --cfg streams=2 > gpurun_out/abenv_${TAG}_${k}_$i.json 2>> gpurun_out/abenv_$TAG.err || exit 1
    echo "m$M [$setting] $i $(python -c "import json,sys; d=json.load(open(sys.argv[1])); v=list(d.values())[0]; print(v['median_ms'], v['mpix_s'])" gpurun_out/abenv_${TAG}_${k}_$i.json)"
  done
done
