# PMC traffic passes for configs[1] (model_0) and configs[2] (model_3 b256), summarised on
# the box (the raw counter CSVs exceed gpurun's copy-back limit).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r01}
cd $R
bash tools/pmc_box.sh
PMC_PREFIX=pmc python3 tools/pmc_summary.py $TAG > gpurun_out/pmc_summary_$TAG.txt
cp profiles/traffic_$TAG.json gpurun_out/
rm -rf gpurun_out/pmc_fetch gpurun_out/pmc_write gpurun_out/pmc_sq
PMC_PREFIX=pmc3 bash tools/pmc_box.sh --model 3 --batch 256
PMC_PREFIX=pmc3 python3 tools/pmc_summary.py ${TAG}_model3 > gpurun_out/pmc_summary_${TAG}_model3.txt
cp profiles/traffic_${TAG}_model3.json gpurun_out/
rm -rf gpurun_out/pmc3_fetch gpurun_out/pmc3_write gpurun_out/pmc3_sq
