set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03s
O=gpurun_out/r03s
timeout -k 10 500 python -u bench.py > $O/c3.log 2>&1 &&
timeout -k 10 200 python -u bench.py --workload c2 > $O/c2.log 2>&1 &&
timeout -k 10 200 python -u bench.py --workload c5 > $O/c5.log 2>&1 &&
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
rc=$?
for f in c3 c2 c5; do tail -1 $O/$f.log | cut -c1-400; done; tail -1 $O/smoke.log
exit $rc
