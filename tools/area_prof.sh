# kernel trace of the INTER_AREA batch probe: usage bash tools/area_prof.sh <tag>
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-area}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o area -- python3 $GRAFT_REPO_ROOT/tools/probe_area.py 32 20 > $O/kt.log 2>&1
