set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03m
O=gpurun_out/r03m
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_reid.py tests/test_gpu_yolo.py > $O/t.log 2>&1 &&
timeout -k 10 400 python -u bench.py --workload c4 --steps 2 --warmup 1 > $O/c4.log 2>&1
rc=$?
tail -3 $O/t.log; tail -1 $O/c4.log | cut -c1-1200
exit $rc
