# round 4: chain workgroup shapes in the lockstep two-lane step (interleaved A/B, one process)
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python tools/ab.py --model 0 --batch 64 --rounds 7 --steps 50 --tune-file tf_image_compression_amd/tune/model0_p256_b64_s2.json --cfg chain_wh=2 --cfg chain_wh=4 --cfg chain_wh=3 --cfg chain_wh=1 > gpurun_out/r04o_ab.json 2> gpurun_out/r04o_ab.err || { tail -20 gpurun_out/r04o_ab.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/r04o_ab.json')); [print(k, v['median_ms'], v['mpix_s']) for k, v in d.items()]"
