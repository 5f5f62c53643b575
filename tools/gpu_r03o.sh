set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03o
O=gpurun_out/r03o
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_conv_t2d.py > $O/t.log 2>&1 &&
timeout -k 10 200 python -u tools/probe_layers.py arc 256 > $O/arc_wide.txt 2>&1 &&
PC_T2D_NARROW=1 timeout -k 10 200 python -u tools/probe_layers.py arc 256 > $O/arc_narrow.txt 2>&1 &&
timeout -k 10 200 python -u tools/probe_layers.py scrfd 64 > $O/scrfd_wide.txt 2>&1 &&
PC_T2D_NARROW=1 timeout -k 10 200 python -u tools/probe_layers.py scrfd 64 > $O/scrfd_narrow.txt 2>&1
rc=$?
tail -3 $O/t.log; for f in arc_wide arc_narrow scrfd_wide scrfd_narrow; do echo "== $f"; head -8 $O/$f.txt; done
exit $rc
