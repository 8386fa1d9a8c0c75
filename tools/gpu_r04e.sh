# round 4: first process on a fresh box with the 3 s preheat (the driver's command), then
# without preheat, then with it again
set -o pipefail
cd $GRAFT_REPO_ROOT
show() { python -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['ms_per_step'], d['preheat'])" $1; }
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r04e_1.json 2>> gpurun_out/r04e.err || exit $?
show gpurun_out/r04e_1.json
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --preheat-s 0 > gpurun_out/r04e_2.json 2>> gpurun_out/r04e.err || exit $?
show gpurun_out/r04e_2.json
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r04e_3.json 2>> gpurun_out/r04e.err || exit $?
show gpurun_out/r04e_3.json
