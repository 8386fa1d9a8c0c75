# quick GPU iteration: parity tests, then one bench with the tuner log
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
TIC_TUNE_LOG=1 timeout -k 10 300 python bench.py --no-cpu-baseline --layers-out gpurun_out/bench_layers_q.json > gpurun_out/bench_q.json 2> gpurun_out/bench_q.err
