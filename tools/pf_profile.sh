# per-frame extract() kernel trace: usage bash tools/pf_profile.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-pf}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o pf -- python3 $GRAFT_REPO_ROOT/bench.py --frames per-frame --no-cpu --no-parity --steps 2 --warmup 1 > $O/kt.log 2>&1
