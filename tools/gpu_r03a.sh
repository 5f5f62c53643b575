set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 240 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_chain.py > gpurun_out/chain_test.log 2>&1 &&
timeout -k 10 240 python -u tools/probe_chain_cross.py 8,16,32,48,64,128,256,512 3 > gpurun_out/cross.log 2>&1 &&
timeout -k 10 400 python -u bench.py > gpurun_out/bench_c3.log 2>&1
rc=$?
tail -3 gpurun_out/chain_test.log; cat gpurun_out/cross.log; tail -2 gpurun_out/bench_c3.log
exit $rc
