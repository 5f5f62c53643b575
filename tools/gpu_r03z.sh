set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03z
O=gpurun_out/r03z
PC_T2D_NBUF3=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_conv_t2d.py > $O/t.log 2>&1 &&
timeout -k 10 200 python -u tools/probe_layers.py scrfd 64 > $O/scrfd_b2.txt 2>&1 &&
PC_T2D_NBUF3=1 timeout -k 10 200 python -u tools/probe_layers.py scrfd 64 > $O/scrfd_b3.txt 2>&1 &&
timeout -k 10 200 python -u tools/probe_layers.py arc 256 > $O/arc_b2.txt 2>&1 &&
PC_T2D_NBUF3=1 timeout -k 10 200 python -u tools/probe_layers.py arc 256 > $O/arc_b3.txt 2>&1
rc=$?
tail -2 $O/t.log; for f in scrfd_b2 scrfd_b3 arc_b2 arc_b3; do echo "== $f"; grep -E "batch|t0 " $O/$f.txt | head -8; done
exit $rc
