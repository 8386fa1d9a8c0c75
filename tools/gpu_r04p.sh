# round 4: (1) f32 MFMA vs VALU on one SIMD (tools/probes/mfma_valu.hip); (2) chain workgroup
# shapes in the lockstep two-lane step; (3) the chain's hand-off cost: phase stamps with the
# hand-off left out (TIC_CHAIN_PROBE=1: no publish / wait / halo; 2: publish, no wait / halo;
# results invalid) and the step time beside
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 60 ./tools/probes/mfma_valu > gpurun_out/r04p_mfma_valu.txt 2>&1 || { cat gpurun_out/r04p_mfma_valu.txt; exit 1; }
cat gpurun_out/r04p_mfma_valu.txt
bash tools/gpu_r04o.sh || exit 1
for p in 1 2; do
  TIC_CHAIN_PROBE=$p timeout -k 10 120 python tools/chain_timing.py > gpurun_out/r04p_chain_probe$p.txt 2>&1 || { cat gpurun_out/r04p_chain_probe$p.txt; exit 1; }
  echo "probe $p: $(head -c 700 gpurun_out/r04p_chain_probe$p.txt)"
done
timeout -k 10 300 python tools/ab.py --model 0 --batch 64 --rounds 5 --steps 50 --tune-file tf_image_compression_amd/tune/model0_p256_b64_s2.json --cfg streams=2 --cfg streams=2,env:TIC_CHAIN_PROBE=1 --cfg streams=2,env:TIC_CHAIN_PROBE=0 > gpurun_out/r04p_ab_probe.json 2>> gpurun_out/r04p.err || exit 1
python -c "import json; d=json.load(open('gpurun_out/r04p_ab_probe.json')); [print(k, v['median_ms'], v['mpix_s']) for k, v in d.items()]"
