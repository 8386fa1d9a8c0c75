# round 4: persistent F(4x4,3x3) (next tile's input prefetched behind the epilogue) vs one tile
# per workgroup, per tiling; + parity of the persistent forms
set -o pipefail
cd $GRAFT_REPO_ROOT
for th in 4 8 16; do
  for wr in 1 2; do
    TIC_FORCE_TILE=$th,1,5,$wr timeout -k 10 120 python tools/wino4_timing.py --n 128 --hw 64 --res 1 --reps 2 > gpurun_out/r04l_${th}_$wr.txt 2>&1 || { cat gpurun_out/r04l_${th}_$wr.txt; exit 1; }
    echo "th $th wr $wr: $(tail -1 gpurun_out/r04l_${th}_$wr.txt | cut -c1-330)"
  done
done
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_wino4.py > gpurun_out/r04l_pt.log 2>&1 || { tail -30 gpurun_out/r04l_pt.log; exit 1; }
tail -1 gpurun_out/r04l_pt.log
