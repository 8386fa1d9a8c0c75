# A/B of two builds of libtic (TIC_LIB) on the default bench and configs[2], alternating.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
for round in 1 2; do
for v in base new; do
  if [ $v = new ]; then L=$R/tf_image_compression_amd/libtic.so; else L=$R/exp_libs/libtic_base.so; fi
  TIC_LIB=$L timeout -k 10 300 python bench.py --no-cpu-baseline --layers-out gpurun_out/abl_${v}_$round.json > gpurun_out/ab_${v}_$round.json 2> gpurun_out/ab_${v}_$round.err
done
done
for v in base new; do
  if [ $v = new ]; then L=$R/tf_image_compression_amd/libtic.so; else L=$R/exp_libs/libtic_base.so; fi
  TIC_LIB=$L timeout -k 10 300 python bench.py --model 3 --batch 256 --no-cpu-baseline --layers-out gpurun_out/abl3_${v}.json > gpurun_out/ab3_${v}.json 2> gpurun_out/ab3_${v}.err
done
