# t2d Cin 64: 8 waves x 4 rows (2 waves per SIMD, PC_T2D_W8) vs 4 waves x 8 rows
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/s2k; mkdir -p $O
PC_T2D_W8=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_conv_t2d.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 &&
PROBE_SHAPES=sc_160_64,s1_3x3_64,s0_3x3_64_112 timeout -k 10 200 python -u tools/probe_conv.py auto > $O/probe4.log 2>&1 &&
PC_T2D_W8=1 PROBE_SHAPES=sc_160_64,s1_3x3_64,s0_3x3_64_112 timeout -k 10 200 python -u tools/probe_conv.py auto > $O/probe8.log 2>&1
rc=$?
tail -1 $O/tests.log; grep -v amdgpu.ids $O/probe4.log; grep -v amdgpu.ids $O/probe8.log
exit $rc
