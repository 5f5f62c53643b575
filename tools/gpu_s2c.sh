# conv_fast with MUBUF LDS-DMA + pinned two-substep schedule: probe, conv tests, C3/C2 bench
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/s2c; mkdir -p $O
PROBE_SHAPES=s3_3x3_256,s2_3x3_128,s4_3x3_512,gemm_1x1_2304,sc_80_96,sc_20_224,sc_40_96 timeout -k 10 200 python -u tools/probe_conv.py auto f13 > $O/probe.log 2>&1 &&
timeout -k 10 400 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_chain.py tests/test_gpu_conv_t2d.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 &&
timeout -k 10 400 python -u bench.py > $O/c3.log 2>&1 &&
timeout -k 10 200 python -u bench.py --workload c2 > $O/c2.log 2>&1
rc=$?
grep -v amdgpu.ids $O/probe.log; tail -2 $O/tests.log; for f in c3 c2; do tail -1 $O/$f.log | cut -c1-250; done
exit $rc
