set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -k "fused_tail" > gpurun_out/pytest_tail.log 2>&1
timeout -k 10 300 python tools/ab.py --model 0 --batch 64 --rounds 5 --steps 20 --cfg streams=2,fuse_tail=0 --cfg streams=2,fuse_tail=1 > gpurun_out/ab_m0_tail.json 2> gpurun_out/ab_m0_tail.err
timeout -k 10 300 python tools/ab.py --model 3 --batch 256 --rounds 3 --steps 5 --cfg streams=2,fuse_tail=0 --cfg streams=2,fuse_tail=1 > gpurun_out/ab_m3_tail.json 2> gpurun_out/ab_m3_tail.err
timeout -k 10 300 python tools/ab.py --model 0 --batch 64 --rounds 5 --steps 20 --cfg streams=2,fuse_tail=0 --cfg streams=2,fuse_tail=1,env:TIC_DEC10_VARIANT=0 --cfg streams=2,fuse_tail=1,env:TIC_DEC10_VARIANT=1 > gpurun_out/ab_m0_tail2.json 2> gpurun_out/ab_m0_tail2.err
