# t2d epilogue with uniform row / 24-bit lane addressing: t2d + conv suites, probes, SCRFD layers, C3
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/s2l; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_conv_t2d.py tests/test_gpu_conv.py tests/test_gpu_scrfd.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 &&
PROBE_SHAPES=sc_160_64,sc_80_96,sc_320_32,s1_3x3_64,s0_3x3_64_112 timeout -k 10 200 python -u tools/probe_conv.py auto > $O/probe.log 2>&1 &&
timeout -k 10 200 python -u tools/probe_layers.py scrfd 32 > $O/scrfd32.txt 2>&1 &&
timeout -k 10 400 python -u bench.py --no-cpu --no-parity > $O/c3.log 2>&1
rc=$?
tail -1 $O/tests.log; grep -v amdgpu.ids $O/probe.log; grep -v amdgpu.ids $O/scrfd32.txt | head -5; tail -1 $O/c3.log | cut -c1-160
exit $rc
