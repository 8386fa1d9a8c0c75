# Round-3 iteration: enc01 variants (bit-identity incl. the persistent / producer-consumer
# ones), one-lane timings, and the two-lane bench with variant 6 pinned.
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-it}
cd $R
source tools/gpu_steps.sh
O=$R/gpurun_out
step e01test_$TAG 600 python -u -m pytest tests/test_gpu_parity.py -k "fused_first or fused_rmbe_first" -v --timeout 300 --timeout-method thread
step probe_$TAG 400 python tools/layer_probe.py 0 32 TIC_ENC01_VARIANT=3 TIC_ENC01_VARIANT=6 TIC_ENC01_VARIANT=5
TIC_ENC01_VARIANT=6 step bench_e6_$TAG 600 python bench.py --tune-cache none --no-cpu-baseline
