set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05u
timeout -k 10 300 python -u bench.py --frames per-frame --no-cpu --no-parity > gpurun_out/r05u/pf.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r05u/kt -o pf -- python3 $GRAFT_REPO_ROOT/bench.py --frames per-frame --no-cpu --no-parity --steps 2 --warmup 1 > $GRAFT_REPO_ROOT/gpurun_out/r05u/kt.log 2>&1
