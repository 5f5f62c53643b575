# final tree check: full GPU suite, smoke, C3 and C2 bench lines
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/s2z; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/gpu_full.log 2>&1 &&
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 &&
timeout -k 10 400 python -u bench.py > $O/c3.log 2>&1 &&
timeout -k 10 200 python -u bench.py --workload c2 > $O/c2.log 2>&1
rc=$?
tail -1 $O/gpu_full.log; tail -1 $O/smoke.log; for f in c3 c2; do tail -1 $O/$f.log | cut -c1-200; done
exit $rc
