R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r02z}
cd $R
mkdir -p gpurun_out
source tools/gpu_steps.sh
step lp_$TAG 600 python tools/layer_probe.py 0 32 "opt:fuse01=1,opt:fuse_tail=1,TIC_ENC01_VARIANT=3,TIC_DEC10_VARIANT=8" "opt:fuse01=1,opt:fuse_tail=1,TIC_ENC01_VARIANT=3,TIC_DEC10_VARIANT=8,TIC_STAGGER=1" "opt:fuse01=1,opt:fuse_tail=1,TIC_ENC01_VARIANT=3,TIC_DEC10_VARIANT=8,TIC_STAGGER=2" "opt:fuse01=1,opt:fuse_tail=1,TIC_ENC01_VARIANT=3,TIC_DEC10_VARIANT=8,TIC_STAGGER=4" "opt:fuse01=1,opt:fuse_tail=1,TIC_ENC01_VARIANT=3,TIC_DEC10_VARIANT=8"
step lp64_$TAG 600 python tools/layer_probe.py 0 64 "opt:fuse01=1,opt:fuse_tail=1,TIC_ENC01_VARIANT=3,TIC_DEC10_VARIANT=8" "opt:fuse01=1,opt:fuse_tail=1,TIC_ENC01_VARIANT=3,TIC_DEC10_VARIANT=8,TIC_STAGGER=2"
