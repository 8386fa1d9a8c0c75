set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 300 python tools/ab.py --model 0 --batch 64 --rounds 5 --steps 20 --cfg streams=2,fuse01=0,fuse_tail=1 --cfg streams=2,fuse01=1,fuse_tail=1 > gpurun_out/ab_m0_fuse01.json 2> gpurun_out/ab_m0_fuse01.err
timeout -k 10 300 python tools/ab.py --model 3 --batch 256 --rounds 3 --steps 5 --cfg streams=2,fuse01=0 --cfg streams=2,fuse01=1 > gpurun_out/ab_m3_fuse01.json 2> gpurun_out/ab_m3_fuse01.err
timeout -k 10 400 python bench.py --workload image4k > gpurun_out/bench_image4k_v6.json 2> gpurun_out/bench_image4k_v6.err
