# round 4: region chain with data-tagged granule hand-off — bit identity, phases, step time
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_chain.py tests/test_gpu_pchain.py tests/test_gpu_parity.py > gpurun_out/r04r_pytest.log 2>&1 || { tail -30 gpurun_out/r04r_pytest.log; exit 1; }
tail -1 gpurun_out/r04r_pytest.log
timeout -k 10 120 python tools/chain_timing.py --tune-file tf_image_compression_amd/tune/model0_p256_b64_s2.json > gpurun_out/r04r_chain_timing.txt 2>&1 || { cat gpurun_out/r04r_chain_timing.txt; exit 1; }
head -c 1500 gpurun_out/r04r_chain_timing.txt
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r04r_bench.json 2> gpurun_out/r04r_bench.err || exit 1
python -c "import json; d=json.load(open('gpurun_out/r04r_bench.json')); r=d['roofline']; print(d['value'], d['ms_per_step'], d['tuning'], r['ms_per_launch'], r['frac'], r.get('ms_per_launch_in_step'))"
timeout -k 10 200 python tools/chain_stress.py > gpurun_out/r04r_stress.txt 2>&1 || { tail -20 gpurun_out/r04r_stress.txt; exit 1; }
tail -3 gpurun_out/r04r_stress.txt
