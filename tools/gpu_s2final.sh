# round 3 session 2 close: full GPU suite, smoke, round profile (kernel trace, FETCH/WRITE, MFMA busy), bench lines
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/s2final; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/gpu_full.log 2>&1 &&
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 &&
timeout -k 10 1500 bash tools/profile_round.sh r03s2 > $O/prof.log 2>&1 &&
timeout -k 10 400 python -u bench.py > $O/c3.log 2>&1 &&
timeout -k 10 200 python -u bench.py --workload c2 > $O/c2.log 2>&1 &&
timeout -k 10 300 python -u bench.py --workload c5 > $O/c5.log 2>&1 &&
timeout -k 10 300 python -u bench.py --workload c4 > $O/c4.log 2>&1
rc=$?
tail -2 $O/gpu_full.log; tail -1 $O/smoke.log; tail -3 $O/prof.log; for f in c3 c2 c5 c4; do tail -1 $O/$f.log | cut -c1-220; done
exit $rc
