set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -x -v -s --timeout 700 --timeout-method thread tests/test_gpu_c5_composed.py tests/test_gpu_c4_composed.py > gpurun_out/t_c45.log 2>&1
rc=$?
grep -E "spans|C4 composed|passed|failed|Error|assert|crop " gpurun_out/t_c45.log | tail -25
exit $rc
