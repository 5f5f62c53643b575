# MUBUF LDS-DMA in conv_fast / conv_t2d / conv_igemm: conv tests, per-layer profiles, C3/C2 bench
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/s2d; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_chain.py tests/test_gpu_conv_t2d.py tests/test_gpu_stem.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 &&
timeout -k 10 200 python -u tools/probe_layers.py scrfd 64 > $O/scrfd64.txt 2>&1 &&
timeout -k 10 200 python -u tools/probe_layers.py scrfd 32 > $O/scrfd32.txt 2>&1 &&
timeout -k 10 200 python -u tools/probe_layers.py arc 256 > $O/arc256.txt 2>&1 &&
timeout -k 10 400 python -u bench.py > $O/c3.log 2>&1 &&
timeout -k 10 200 python -u bench.py --workload c2 > $O/c2.log 2>&1
rc=$?
tail -2 $O/tests.log; for f in scrfd64 scrfd32 arc256; do grep -v amdgpu.ids $O/$f.txt | head -8; done; for f in c3 c2; do tail -1 $O/$f.log | cut -c1-200; done
exit $rc
