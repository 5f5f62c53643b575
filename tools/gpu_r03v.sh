set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03v
O=gpurun_out/r03v
timeout -k 10 200 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_scrfd_scratch.py > $O/t.log 2>&1 &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/kt_c4 -o c4 -- python3 $GRAFT_REPO_ROOT/bench.py --workload c4 --steps 1 --warmup 1 > $GRAFT_REPO_ROOT/$O/kt_c4.log 2>&1
rc=$?
cd $GRAFT_REPO_ROOT
tail -2 $O/t.log
find $O/kt_c4 -name "*kernel_stats.csv" -exec head -12 {} \; | cut -c1-150
exit $rc
