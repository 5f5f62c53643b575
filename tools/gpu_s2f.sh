# cfg 14 (128x224, 2 per CU, ROWB 64) + pinned KSTEPS-1 schedule: conv tests, probes, layers, C3/C2
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/s2f; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_chain.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 &&
PROBE_SHAPES=s3_3x3_256,s2_3x3_128,gemm_1x1_2304,s4_3x3_512 timeout -k 10 200 python -u tools/probe_conv.py auto f13 f14 f10 > $O/probe.log 2>&1 &&
timeout -k 10 200 python -u tools/probe_layers.py arc 256 > $O/arc256.txt 2>&1 &&
timeout -k 10 400 python -u bench.py > $O/c3.log 2>&1 &&
PC_CONV_FAST=15 timeout -k 10 400 python -u bench.py > $O/c3_f14.log 2>&1
rc=$?
tail -2 $O/tests.log; grep -v amdgpu.ids $O/probe.log; grep -v amdgpu.ids $O/arc256.txt | head -6; for f in c3 c3_f14; do tail -1 $O/$f.log | cut -c1-200; done
exit $rc
