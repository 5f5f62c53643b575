set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03r
O=gpurun_out/r03r
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gpu_fallbacks.py tests/test_gpu_face_embedder.py tests/test_gpu_prescan.py > $O/t.log 2>&1
rc=$?
grep -E "PASS|FAIL|prefetched|Error" $O/t.log | tail -30
exit $rc
