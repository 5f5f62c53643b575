set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03g
O=gpurun_out/r03g
timeout -k 10 900 python -u -m pytest -x -q --timeout 700 --timeout-method thread -m gpu tests > $O/suite.log 2>&1 &&
timeout -k 10 150 python -u bench.py --no-cpu --frames per-frame --steps 2 --warmup 1 > $O/c3_pf640.log 2>&1 &&
timeout -k 10 150 python -u bench.py --no-cpu --frames per-frame --det-size 1408 --face-conf 0.75 --steps 2 --warmup 1 > $O/c3_pf1408.log 2>&1
rc=$?
tail -3 $O/suite.log
for f in c3_pf640 c3_pf1408; do echo "== $f"; tail -1 $O/$f.log | cut -c1-300; done
exit $rc
