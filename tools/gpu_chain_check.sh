set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_chain.py > gpurun_out/chain_test.log 2>&1
rc=$?
tail -5 gpurun_out/chain_test.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 200 python -u tools/probe_chain.py 256 292 128 > gpurun_out/probe_chain.log 2>&1
cat gpurun_out/probe_chain.log
