set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03p
O=gpurun_out/r03p
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_conv_t2d.py > $O/t.log 2>&1 &&
PC_T2D_128=8 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_conv_t2d.py -k "128" > $O/t8.log 2>&1 &&
PC_T2D_128=8 timeout -k 10 200 python -u tools/probe_layers.py arc 256 > $O/arc_t8.txt 2>&1 &&
PC_T2D_128=4 timeout -k 10 200 python -u tools/probe_layers.py arc 256 > $O/arc_t4.txt 2>&1 &&
timeout -k 10 200 python -u tools/probe_layers.py arc 256 > $O/arc_def.txt 2>&1
rc=$?
tail -2 $O/t.log; tail -2 $O/t8.log; for f in arc_t8 arc_t4 arc_def; do echo "== $f"; head -4 $O/$f.txt; done
exit $rc
