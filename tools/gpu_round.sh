set -e
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
timeout -k 10 240 python tools/ab.py --rounds 5 --cfg streams=2,graph=0 --cfg streams=2,graph=1 > gpurun_out/ab_graph.log 2>&1
timeout -k 10 300 python bench.py > gpurun_out/bench_v3.json 2> gpurun_out/bench_v3.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_v3 -o p -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --steps 20 > $GRAFT_REPO_ROOT/gpurun_out/prof_v3.log 2>&1
cd $GRAFT_REPO_ROOT
bash tools/pmc_box.sh
