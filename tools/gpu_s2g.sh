# EARLY slot refill (tile 13) vs tile 15 (same tile, refill one tile later): conv tests, probes, layers, C3/C2
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/s2g; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_chain.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 &&
PROBE_SHAPES=s3_3x3_256,gemm_1x1_2304 timeout -k 10 200 python -u tools/probe_conv.py f13 f15 f13 f15 > $O/probe.log 2>&1 &&
timeout -k 10 200 python -u tools/probe_layers.py arc 256 > $O/arc256.txt 2>&1 &&
timeout -k 10 400 python -u bench.py > $O/c3.log 2>&1 &&
timeout -k 10 200 python -u bench.py --workload c2 > $O/c2.log 2>&1
rc=$?
tail -2 $O/tests.log; grep -v amdgpu.ids $O/probe.log; grep -v amdgpu.ids $O/arc256.txt | head -4; for f in c3 c2; do tail -1 $O/$f.log | cut -c1-200; done
exit $rc
