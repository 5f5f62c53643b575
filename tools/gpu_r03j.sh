set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03j
O=gpurun_out/r03j
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_yolo_face.py tests/test_gpu_staging.py > $O/t.log 2>&1
rc=$?
grep -E "PASS|FAIL|Error|assert" $O/t.log | tail -20
exit $rc
