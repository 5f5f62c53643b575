# round 3, session 2: restored tree check (suite + smoke + C3 bench) and a 14x14x256 ROWB probe
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/s2a; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/gpu_full.log 2>&1 &&
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 &&
timeout -k 10 400 python -u bench.py > $O/c3.log 2>&1 &&
PROBE_SHAPES=s3_3x3_256 timeout -k 10 120 python -u tools/probe_conv.py f13 f13:64 f0 f2 > $O/probe_s3.log 2>&1
rc=$?
tail -2 $O/gpu_full.log; tail -1 $O/smoke.log; tail -1 $O/c3.log | cut -c1-300; cat $O/probe_s3.log
exit $rc
