# Final-tree check, as the driver runs it at round end: the GPU suite, smoke(), the default bench.
#   bash tools/gpu_final_check.sh <tag>
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1
cd $R
source tools/gpu_steps.sh
bash tools/gpu_suite.sh $TAG || exit 1
step smoke_$TAG 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
step bench_$TAG 300 python bench.py
