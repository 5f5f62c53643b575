set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03f
O=gpurun_out/r03f
timeout -k 10 400 python -u bench.py > $O/c3.log 2>&1 &&
timeout -k 10 200 python -u bench.py --no-cpu --frames host > $O/c3_host.log 2>&1 &&
timeout -k 10 200 python -u bench.py --no-cpu --frames per-frame --steps 2 --warmup 1 > $O/c3_pf640.log 2>&1 &&
timeout -k 10 200 python -u bench.py --no-cpu --frames per-frame --det-size 1408 --steps 2 --warmup 1 > $O/c3_pf1408.log 2>&1 &&
timeout -k 10 200 python -u bench.py --workload c2 > $O/c2.log 2>&1
rc=$?
for f in c3 c3_host c3_pf640 c3_pf1408 c2; do echo "== $f"; tail -1 $O/$f.log | cut -c1-600; done
exit $rc
