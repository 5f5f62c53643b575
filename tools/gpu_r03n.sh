set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03n
O=gpurun_out/r03n
timeout -k 10 1100 python -u -m pytest -x -q --timeout 700 --timeout-method thread -m gpu tests > $O/suite.log 2>&1
rc=$?
tail -5 $O/suite.log; ls gpurun_out/parity 2>/dev/null && cat gpurun_out/parity/*.json
exit $rc
