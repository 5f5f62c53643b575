set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_staging.py tests/test_gpu_chain.py > gpurun_out/t_staging.log 2>&1 &&
timeout -k 10 800 python -u -m pytest -x -v -s --timeout 700 --timeout-method thread tests/test_gpu_c5_composed.py tests/test_gpu_c4_composed.py > gpurun_out/t_c45.log 2>&1
rc=$?
tail -5 gpurun_out/t_staging.log; grep -E "spans|C4 composed|passed|failed|Error|assert" gpurun_out/t_c45.log | tail -15
exit $rc
