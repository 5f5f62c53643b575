# kernel trace of the C5 bench (1 step): usage bash tools/c5_prof.sh <tag>
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-c5prof}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o c5 -- python3 $GRAFT_REPO_ROOT/bench.py --workload c5 --steps 1 --warmup 1 --no-cpu --no-parity > $O/kt.log 2>&1
