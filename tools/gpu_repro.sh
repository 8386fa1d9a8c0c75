# reproducibility of the driver's protocol: the exact driver command twice (separate
# processes) for configs[1], once for configs[2]   bash tools/gpu_repro.sh <tag>
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-rp}
cd $R
source tools/gpu_steps.sh
step drv1_m0_$TAG 300 python3 bench.py --gpus 1 --steps 20 --warmup 5
step drv2_m0_$TAG 300 python3 bench.py --gpus 1 --steps 20 --warmup 5
step drv_m3_$TAG 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 --model 3 --batch 256
for f in drv1_m0 drv2_m0 drv_m3; do python3 -c "
import json,sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        d=json.loads(l); r=d['roofline']; print(sys.argv[2], d['value'], d['ms_per_step'], r['kernel_instance'], r['frac'])
" gpurun_out/${f}_$TAG.log $f; done
