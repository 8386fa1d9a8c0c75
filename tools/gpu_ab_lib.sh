# A/B of two builds of libtic (TIC_LIB: exp_libs/libtic_base.so vs the tree's) on the default
# bench and configs[2], alternating on one box, both replaying ONE tuning state (tuned with
# the tree's build first) so that only the kernels differ:  bash tools/gpu_ab_lib.sh <tag>
# With AB_SEPARATE=1 each build is tuned with itself (for a build that adds candidates).
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-ab}
cd $R
mkdir -p gpurun_out
source tools/gpu_steps.sh
O=$R/gpurun_out
step abt0_$TAG 400 python bench.py --no-cpu-baseline --tune-cache $O/abtune0_$TAG.json --steps 20
step abt3_$TAG 400 python bench.py --no-cpu-baseline --model 3 --batch 256 --tune-cache $O/abtune3_$TAG.json --steps 5
B0=$O/abtune0_$TAG.json; B3=$O/abtune3_$TAG.json
if [ "${AB_SEPARATE:-0}" = 1 ]; then
  B0=$O/abtune0b_$TAG.json; B3=$O/abtune3b_$TAG.json
  step abt0b_$TAG 400 env TIC_LIB=$R/exp_libs/libtic_base.so python bench.py --no-cpu-baseline --tune-cache $B0 --steps 20
  step abt3b_$TAG 400 env TIC_LIB=$R/exp_libs/libtic_base.so python bench.py --no-cpu-baseline --model 3 --batch 256 --tune-cache $B3 --steps 5
fi
for round in 1 2 3; do
  for v in base new; do
    if [ $v = new ]; then L=$R/tf_image_compression_amd/libtic.so; T=$O/abtune0_$TAG.json; else L=$R/exp_libs/libtic_base.so; T=$B0; fi
    step ab0_${v}_${round}_$TAG 300 env TIC_LIB=$L python bench.py --no-cpu-baseline --tune-cache $T
  done
done
for round in 1 2; do
  for v in base new; do
    if [ $v = new ]; then L=$R/tf_image_compression_amd/libtic.so; T=$O/abtune3_$TAG.json; else L=$R/exp_libs/libtic_base.so; T=$B3; fi
    step ab3_${v}_${round}_$TAG 400 env TIC_LIB=$L python bench.py --no-cpu-baseline --model 3 --batch 256 --tune-cache $T
  done
done
