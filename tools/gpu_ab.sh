# Alternating A/B of two builds of libtic.so on one box (methodology: the variants in
# alternating rounds, same device, same replayed tuning):
#   bash tools/gpu_ab.sh <tag> <model> <batch> <tune json> [pairs]
# compares tf_image_compression_amd/libtic_old.so (A) with tf_image_compression_amd/libtic.so (B)
# (or $ABA / $ABB: other library paths),
# each pair = one ab.py run of each (3 rounds x 60 steps, two lanes); results in
# gpurun_out/ab_<tag>_{old,new}_<i>.json and one line per run on stdout.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; M=$2; B=$3; T=$4; PAIRS=${5:-3}
for i in $(seq 1 $PAIRS); do
  for v in old new; do
    if [ $v = new ]; then L=${ABB:-tf_image_compression_amd/libtic.so}; else L=${ABA:-tf_image_compression_amd/libtic_old.so}; fi
    TIC_LIB=$L timeout -k 10 200 python tools/ab.py --model $M --batch $B --rounds 3 --steps 60 --tune-file $T \
      --cfg streams=2 > gpurun_out/ab_${TAG}_${v}_$i.json 2>> gpurun_out/ab_$TAG.err || exit 1
    echo "m$M $v $i $(python -c "import json,sys; d=json.load(open(sys.argv[1])); v=list(d.values())[0]; print(v['median_ms'], v['mpix_s'])" gpurun_out/ab_${TAG}_${v}_$i.json)"
  done
done
