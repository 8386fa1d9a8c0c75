# round 4: steady-state timeline of the configs[1] step (kernel trace of --trace-only: the trace
# ends with the timed steps)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r04m_tr -o tr -- python bench.py --steps 30 --warmup 5 --no-cpu-baseline --trace-only > gpurun_out/r04m_trace.json 2> gpurun_out/r04m.err || exit $?
cat gpurun_out/r04m_trace.json
python tools/step_trace.py gpurun_out/r04m_tr/tr_kernel_trace.csv 16 5
