# round 4: the driver's exact command, three times, on the shipped tuning
set -o pipefail
cd $GRAFT_REPO_ROOT
for i in 1 2 3; do
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r04d_drv_$i.json 2>> gpurun_out/r04d.err || exit $?
  python -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(d['value'], d['ms_per_step'], d['tuning'], r['kernel_instance'], r['frac'], r.get('frac_in_step'), r.get('most_in_step_time',{}).get('kernel'), d.get('cpu_baseline',{}).get('value'))" gpurun_out/r04d_drv_$i.json
done
