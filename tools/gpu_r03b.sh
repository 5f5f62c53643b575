set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py --no-cpu > gpurun_out/bench_c3_chain.log 2>&1 &&
PC_CHAIN=0 timeout -k 10 300 python -u bench.py --no-cpu --no-parity > gpurun_out/bench_c3_nochain.log 2>&1
rc=$?
tail -2 gpurun_out/bench_c3_chain.log; tail -1 gpurun_out/bench_c3_nochain.log
exit $rc
