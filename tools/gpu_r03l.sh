set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03l
O=gpurun_out/r03l
timeout -k 10 400 python -u bench.py --workload c4 --steps 2 --warmup 1 > $O/c4.log 2>&1 &&
timeout -k 10 300 python -u bench.py --workload c5 > $O/c5.log 2>&1 &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/kt_c4 -o c4 -- python3 $GRAFT_REPO_ROOT/bench.py --workload c4 --steps 1 --warmup 1 > $GRAFT_REPO_ROOT/$O/kt_c4.log 2>&1
rc=$?
cd $GRAFT_REPO_ROOT
for f in c4 c5; do echo "== $f"; tail -1 $O/$f.log | cut -c1-1500; done
find $O/kt_c4 -name "*kernel_stats.csv" -exec head -14 {} \; | cut -c1-160
exit $rc
